#!/bin/bash
# k_match_local iteration: local-search parity tests, the phase timing variant
# (variants/lprof, built with -DORBPL_LOCAL_PROF) at 1024 streams, then the
# headline bench at 1024 and 256 streams.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "${1:-local}" --timeout 200 --timeout-method thread > gpurun_out/lt.log 2>&1
rc=$?; tail -3 gpurun_out/lt.log; [ $rc -ne 0 ] && exit $rc
B="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0"
ORBPL_LIB=variants/lprof/liborbpl.so timeout -k 10 300 python bench.py --streams 1024 --steps 3 --warmup 2 --isolated-steps 0 $B > gpurun_out/lprof.log 2>&1 || exit 1
grep "local blk" gpurun_out/lprof.log | tail -8
timeout -k 10 200 python bench.py --streams 1024 --steps 10 --warmup 3 --isolated-steps 3 $B > gpurun_out/b1024.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --isolated-steps 3 $B > gpurun_out/b256.log 2>&1 || exit 1
for f in b256 b1024; do grep '^{' gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']), d['ms_per_step'], d['stage_ms'])"; done
