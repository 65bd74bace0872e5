#!/bin/bash
# Kernel trace of the headline leg, non-pipelined (every kernel's own time).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/iso
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/iso/trace -o run --output-format csv -- python3 $R/bench.py --pipelined 0 --steps 10 --warmup 5 --no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --isolated-steps 0 --ingress-steps 0 $ISO_ARGS > $R/gpurun_out/iso/trace.log 2>&1 || { echo "trace failed"; tail -5 $R/gpurun_out/iso/trace.log; exit 1; }
python3 $R/tools/trace_summary.py $R/gpurun_out/iso/trace/run_kernel_trace.csv > $R/gpurun_out/iso/summary.txt
head -32 $R/gpurun_out/iso/summary.txt
