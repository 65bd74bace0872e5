#!/bin/bash
# Quick GPU iteration: selected parity tests (-k expression in $1, "" = all
# GPU tests), then a kernel trace of a short headline bench run (extra
# arguments go to bench.py). Every GPU step has its own time limit; the
# script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
shift
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -k "$K" --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
else
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
fi
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/quick_tests.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_quick
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_quick -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --isolated-steps 0 --ingress-steps 0 "$@" > $R/gpurun_out/quick_bench.log 2>&1
rc=$?; echo "trace exit $rc"; tail -c 300 $R/gpurun_out/quick_bench.log
[ $rc -ne 0 ] && exit $rc
cut -d, -f1-4 $R/gpurun_out/prof_quick/run_kernel_stats.csv | cut -c1-160 | head -16
