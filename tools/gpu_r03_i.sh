#!/bin/bash
# Round-3 pass i: kernel trace of the lines workload (3072 streams, 4 timed
# steps, pipelined) for the per-stream timeline (tools/timeline.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/trace_lines
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python3 $R/bench.py --workload lines --streams 3072 --steps 4 --warmup 2 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --sweep 0 --isolated-steps 0 --no-cpu-baseline --no-parity > $out/trace.log 2>&1 || { echo "trace failed"; tail -5 $out/trace.log; exit 1; }
find $out -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
find $out -name '*kernel_trace.csv' -exec cp {} $out/kernel_trace.csv \;
tail -c 400 $out/trace.log
echo trace ok
