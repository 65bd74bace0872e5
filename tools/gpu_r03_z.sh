#!/bin/bash
# Round-3 pass z: seed loop keeping the valid later seeds of a round
# (ORBPL_SPEC_KEEP): LSD parity tests, A/B against the build without it at
# batch 1 / 3072 (two rounds), then the lines tracker parity tests.
set -o pipefail
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/tests.log | head; exit $rc; }
for r in 1 2; do
  for v in cur nokeep; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    for b in 1 3072; do
      ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py $b > $O/t_${v}_$b.log 2>&1 || { echo "fail $v $b"; tail -3 $O/t_${v}_$b.log; exit 1; }
      echo "$r $v $(head -2 $O/t_${v}_$b.log | tr '\n' ' ' | cut -c1-330)"
    done
  done
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_track.py -k "lines" -x -q --timeout 300 --timeout-method thread > $O/track.log 2>&1
rc=$?; echo "track tests exit $rc: $(tail -1 $O/track.log)"
exit $rc
