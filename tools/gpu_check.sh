#!/bin/bash
# GPU validation used during development: parity tests, then a short bench.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -2 gpurun_out/bench.log
exit $rc
