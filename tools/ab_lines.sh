#!/bin/bash
# LSD A/B: the LSD and line-tracker parity tests against a library variant
# ($1: variants/<name>/liborbpl.so), then the lines workload (3072 streams)
# with the in-tree library and the variant.
set -o pipefail
mkdir -p gpurun_out/ab
V=$1
ORBPL_LIB=variants/$V/liborbpl.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "lsd or lines or line" --timeout 300 --timeout-method thread > gpurun_out/ab/lines_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab/lines_tests.log; [ $rc -ne 0 ] && exit $rc
B="--workload lines --streams 3072 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for r in 1 2; do
  for v in cur $V; do
    L=""; [ $v != cur ] && L=variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 300 python bench.py $B > gpurun_out/ab/lines_$v.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/ab/lines_$v.log; exit 1; }
    grep '^{' gpurun_out/ab/lines_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']), d['ms_per_step'], {k: round(d['stage_ms'][k],1) for k in ('lsd','lsd_seed','lsd_sort','lsd_validate') if k in d['stage_ms']})"
  done
done
