#!/bin/bash
# Round-3 first GPU pass: the -m gpu suite, the FETCH_SIZE calibration, the
# stereo (configs[3]) and rig (configs[4]) trace + PMC passes, one bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
mkdir -p gpurun_out/calib
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/calib/fetch -o run --output-format csv -- $R/tools/calib/fetch_calib > $R/gpurun_out/calib/run.log 2>&1) || { echo "calib failed"; tail -5 gpurun_out/calib/run.log; exit 1; }
echo calib ok
MODE=kitti bash tools/prof.sh kitti_r03 || exit 1
MODE=rig bash tools/prof.sh rig_r03 || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r03_a.json 2> gpurun_out/bench_r03_a.err || { echo "bench failed"; tail -20 gpurun_out/bench_r03_a.err; exit 1; }
echo bench ok
