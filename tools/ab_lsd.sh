#!/bin/bash
# LSD A/B on the GPU box: LSD parity tests with each variant library, then
# tools/time_lsd.py at the batch sizes in $1 for the in-tree library and each
# variants/<name>/liborbpl.so in $2.
set -o pipefail
mkdir -p gpurun_out/ab
BS=${1:-"3072 4096"}
VS="default ${2:-}"
for v in $VS; do
  if [ $v = default ]; then L=""; else L=variants/$v/liborbpl.so; fi
  ORBPL_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/lsd_tests_$v.log 2>&1 || { echo "tests fail $v"; tail -20 gpurun_out/ab/lsd_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/ab/lsd_tests_$v.log)"
  for b in $BS; do
    ORBPL_LIB=$L timeout -k 10 200 python tools/time_lsd.py $b > gpurun_out/ab/lsd_${v}_$b.log 2>&1 || { echo "time fail $v $b"; tail -5 gpurun_out/ab/lsd_${v}_$b.log; exit 1; }
    echo "$v $(head -1 gpurun_out/ab/lsd_${v}_$b.log)"
  done
done
