#!/bin/bash
# Multi-wave seed loop check: every GPU parity test, then the LSD batch probe
# at batch 1 / 64 / 1024 / 3072 (4 / 4 / 2 / 1 waves per frame).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/time_lsd.log
for b in 1 64 1024 3072; do
  timeout -k 10 120 python tools/time_lsd.py $b >> gpurun_out/time_lsd.log 2>&1 || { echo "time_lsd $b failed"; tail -5 gpurun_out/time_lsd.log; exit 1; }
done
cut -c1-330 gpurun_out/time_lsd.log
