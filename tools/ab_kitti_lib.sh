#!/bin/bash
# Stereo (KITTI) leg A/B over library variants ($1, "cur" = in-tree) at 1024
# pairs, $2 rounds alternating.
set -o pipefail
mkdir -p gpurun_out/abk
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for r in $(seq 1 ${2:-2}); do
  for v in ${1:-cur}; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 300 python bench.py --workload kitti --streams 1024 --steps 4 --warmup 1 $C > gpurun_out/abk/b_$v.log 2>&1 || { echo "fail bench $v"; tail -5 gpurun_out/abk/b_$v.log; exit 1; }
    grep '^{' gpurun_out/abk/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $v kitti', round(d['value']), d['ms_per_step'], round(d['stage_ms'].get('right_lines', 0),1))"
  done
done
