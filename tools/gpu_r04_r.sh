#!/bin/bash
# Round-4 pass r: kernel stats of the LSD detector at 1 and 16 frames (current
# build), for the per-kernel split of the single-stream lines latency.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
for B in 1 16; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/b$B -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $O/b$B.log 2>&1 || { echo "b$B failed"; tail -5 $O/b$B.log; exit 1; }
  head -1 $O/b$B.log
done
exit 0
