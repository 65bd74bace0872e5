#!/bin/bash
# LSD iteration: the bit-exact LSD parity tests, the seed-loop profile at
# batch 1 and 3072, then a short lines-headline bench (sampled timed streams
# replayed through the oracle). Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lsd_tests.log 2>&1
rc=$?; echo "lsd tests exit $rc"; tail -3 gpurun_out/lsd_tests.log; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/time_lsd.log
for b in 1 3072; do
  timeout -k 10 120 python tools/time_lsd.py $b >> gpurun_out/time_lsd.log 2>&1 || { echo "time_lsd $b failed"; tail -5 gpurun_out/time_lsd.log; exit 1; }
done
cat gpurun_out/time_lsd.log
timeout -k 10 400 python bench.py --workload lines --streams 3072 --steps 5 --warmup 2 --no-cpu-baseline --sweep 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 "$@" > gpurun_out/lines_bench.log 2>&1
rc=$?; echo "lines bench exit $rc"; tail -c 400 gpurun_out/lines_bench.log
exit $rc
