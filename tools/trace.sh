#!/bin/bash
# Kernel trace + stats of a short points bench (no PMC): per-dispatch
# durations under gpurun_out/trace_<tag>/.
set -o pipefail
tag=${1:-run}; shift
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/trace_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --no-cpu-baseline "$@" > $out/trace.log 2>&1 || { echo "trace failed"; tail -5 $out/trace.log; exit 1; }
find $out -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
find $out -name '*kernel_trace.csv' -exec cp {} $out/kernel_trace.csv \;
echo trace ok
