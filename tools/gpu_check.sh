#!/bin/bash
# GPU validation used during development: host facts, parity tests, then the
# default bench. Every GPU step has its own time limit; the script stops at
# the first failure. Extra arguments go to bench.py.
set -o pipefail
mkdir -p gpurun_out
{ nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket|NUMA node\(s\)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; \
  echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; grep -o -w -E "avx512f|avx512bw|avx512vl|avx2" /proc/cpuinfo | sort | uniq -c; } > gpurun_out/host.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -c 600 gpurun_out/bench.log
exit $rc
