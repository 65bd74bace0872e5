#!/bin/bash
# A/B timing on the GPU box: parity tests matching $1 (-k), then the
# headline bench at each stream count in $2 (default "256 1024") for the
# in-tree library and every variants/<name>/liborbpl.so named in $3.
set -o pipefail
mkdir -p gpurun_out/ab
K=${1:-"pose or tracker"}
SS=${2:-"256 1024"}
VS="default ${3:-}"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { tail -20 gpurun_out/ab/tests.log; exit 1; }
tail -2 gpurun_out/ab/tests.log
for v in $VS; do
  for s in $SS; do
    if [ $v = default ]; then L=""; else L=variants/$v/liborbpl.so; fi
    ORBPL_LIB=$L timeout -k 10 200 python bench.py --streams $s --steps 10 --warmup 3 --no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --isolated-steps 3 > gpurun_out/ab/${v}_$s.log 2>&1 || { echo fail $v $s; tail -5 gpurun_out/ab/${v}_$s.log; exit 1; }
  done
done
