#!/bin/bash
# LSD development check: the bit-exact LSD / LineExtractor parity tests, the
# seed-loop profile at batch 1 / 64 / 3072, then a kernel trace of a short
# points run (per-kernel times of the tracker, local map included).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lsd_tests.log 2>&1
rc=$?; echo "lsd tests exit $rc"; tail -3 gpurun_out/lsd_tests.log; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/time_lsd.log
for b in 1 64 3072; do
  timeout -k 10 120 python tools/time_lsd.py $b >> gpurun_out/time_lsd.log 2>&1 || { echo "time_lsd $b failed"; tail -5 gpurun_out/time_lsd.log; exit 1; }
done
cat gpurun_out/time_lsd.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_lm -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --isolated-steps 0 > $R/gpurun_out/prof_lm.log 2>&1 || { echo "trace failed"; tail -5 $R/gpurun_out/prof_lm.log; exit 1; }
head -25 $R/gpurun_out/prof_lm/run_kernel_stats.csv | cut -c1-150
