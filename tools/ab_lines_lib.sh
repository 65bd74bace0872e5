#!/bin/bash
# Lines A/B over library variants ($1, "cur" = in-tree): LSD probe at 3072
# and the lines workload at 3072 streams, $2 rounds alternating.
set -o pipefail
mkdir -p gpurun_out/abl
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for r in $(seq 1 ${2:-2}); do
  for v in ${1:-cur}; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py 3072 > gpurun_out/abl/t_$v.log 2>&1 || { echo "fail probe $v"; exit 1; }
    echo "$r $v probe $(head -1 gpurun_out/abl/t_$v.log)"
    ORBPL_LIB=$L timeout -k 10 300 python bench.py --workload lines --streams 3072 --steps 4 --warmup 1 $C > gpurun_out/abl/b_$v.log 2>&1 || { echo "fail bench $v"; exit 1; }
    grep '^{' gpurun_out/abl/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $v lines', round(d['value']), d['ms_per_step'], round(d['stage_ms']['lsd_seed'],1))"
  done
done
