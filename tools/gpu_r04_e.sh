#!/bin/bash
# Round-4 pass e: the sparse small-batch seed loop (k_lsd_spec_sparse, 64
# seeds per round over 4 waves x 16 lanes): LSD parity tests, then LSD batch
# 1 / 16 / 64 / 96 against the one-wave loop (ORBPL_SPEC_SPARSE=0), two rounds.
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error|FAIL" $O/tests.log | head -20; exit $rc; }
for r in 1 2; do
  for v in sparse onewave; do
    E=""; [ "$v" = onewave ] && E="ORBPL_SPEC_SPARSE=0"
    for b in 1 16 64 96; do
      env $E timeout -k 10 120 python tools/time_lsd.py $b > $O/t_${v}_$b.log 2>&1 || { echo "fail $v $b"; tail -3 $O/t_${v}_$b.log; exit 1; }
      echo "$r $v $(head -2 $O/t_${v}_$b.log | tr '\n' ' ' | cut -c1-300)"
    done
  done
done
exit 0
