#!/bin/bash
# Seed-loop A/B: for each library variant in $1 ("cur" = in-tree, else
# variants/<name>/liborbpl.so): the bit-exact LSD parity tests, then the LSD
# batch probe at batch 1 and 3072. Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out/ablsd
for v in ${1:-cur}; do
  L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
  ORBPL_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ablsd/tests_$v.log 2>&1
  rc=$?; echo "$v tests exit $rc: $(tail -1 gpurun_out/ablsd/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
  for b in 1 3072; do
    ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py $b > gpurun_out/ablsd/time_${v}_$b.log 2>&1 || { echo "time_lsd $v $b failed"; tail -5 gpurun_out/ablsd/time_${v}_$b.log; exit 1; }
    echo "$v $(head -2 gpurun_out/ablsd/time_${v}_$b.log | tr '\n' ' ' | cut -c1-400)"
  done
done
