#!/bin/bash
# Small-batch LSD A/B over library variants ($1): LSD parity tests, then the
# LSD probe at batch 1 / 16 / 64, $2 rounds alternating.
set -o pipefail
mkdir -p gpurun_out/abs
VS=${1:-cur}
for v in $VS; do
  L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
  ORBPL_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/abs/tests_$v.log 2>&1
  rc=$?; echo "$v tests exit $rc: $(tail -1 gpurun_out/abs/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for r in $(seq 1 ${2:-2}); do
  for v in $VS; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    for b in 1 16 64; do
      ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py $b > gpurun_out/abs/t_${v}_$b.log 2>&1 || { echo "fail $v $b"; exit 1; }
      echo "$r $v $(head -1 gpurun_out/abs/t_${v}_$b.log | cut -c1-60)"
    done
  done
done
