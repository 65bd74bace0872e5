#!/bin/bash
# Round-3 GPU pass d: map parity after the k_map_finish rework, then the
# headline (points, map model) trace + PMC, the FETCH calibration, the stereo
# and rig trace + PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py -q --timeout 300 --timeout-method thread > gpurun_out/gpu_map_d.log 2>&1
rc=$?
echo "map tests rc=$rc"; tail -3 gpurun_out/gpu_map_d.log
if [ $rc -ne 0 ]; then grep -E "assert|Error" gpurun_out/gpu_map_d.log | head -20; exit 1; fi
MODE=points bash tools/prof.sh points_r03 || exit 1
python3 tools/trace_summary.py gpurun_out/prof_points_r03/trace/run_kernel_trace.csv > gpurun_out/prof_points_r03/trace_summary.txt 2>&1 || true
head -30 gpurun_out/prof_points_r03/trace_summary.txt
mkdir -p gpurun_out/calib
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/calib/fetch -o run --output-format csv -- $R/tools/calib/fetch_calib > $R/gpurun_out/calib/run.log 2>&1) || { echo "calib failed"; tail -5 gpurun_out/calib/run.log; exit 1; }
echo calib ok
MODE=kitti bash tools/prof.sh kitti_r03 || exit 1
MODE=rig bash tools/prof.sh rig_r03 || exit 1
echo all ok
