#!/bin/bash
# Round-3 pass h: fit-pass batch size of the small-batch seed loop
# (ORBPL_FIT_B_SMALL): LSD parity tests on the in-tree build (32) and the 16
# variant, then LSD probe at batch 1 / 16 / 64 for 32 / 8 / 16 / 24, 2 rounds.
set -o pipefail
O=gpurun_out/r03h
mkdir -p $O
for v in cur kb16; do
  L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
  ORBPL_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v tests exit $rc: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
  for v in cur kb8 kb16 kb24; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    for b in 1 16 64; do
      ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py $b > $O/t_${v}_$b.log 2>&1 || { echo "fail $v $b"; tail -3 $O/t_${v}_$b.log; exit 1; }
      echo "$r $v $(head -2 $O/t_${v}_$b.log | tr '\n' ' ' | cut -c1-330)"
    done
  done
done
