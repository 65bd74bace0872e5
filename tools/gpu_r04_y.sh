#!/bin/bash
# Round-4 pass y: the cooperative fit's phase split (profiling build
# -DORBPL_FIT_PROF, frame 0, wave cycles summed over rounds) at 1 / 16 frames.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04y
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
for B in 1 16; do
  ORBPL_LIB=$R/variants/fitprof/liborbpl.so timeout -k 10 200 python3 tools/time_lsd.py $B > $O/fitprof_$B.log 2>&1 || { echo "fitprof $B failed"; tail -5 $O/fitprof_$B.log; exit 1; }
  grep -m1 "^batch" $O/fitprof_$B.log; grep fitprof $O/fitprof_$B.log | tail -1
done
