#!/bin/bash
# A/B of settings across workloads: items as in tools/ab_lib.sh
# ("<variant>[:NAME=VALUE[+NAME=VALUE]]"), $2 = workloads (points lines kitti
# rig), $3 rounds. Default stream counts of bench.py; frames/s, ms per step
# and the batch-1 latency of the leg's sweep when present.
set -o pipefail
mkdir -p gpurun_out/abw
C="--no-cpu-baseline --no-parity --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for r in $(seq 1 ${3:-1}); do
  for w in ${2:-points lines}; do
    for it in ${1:-cur}; do
      v=${it%%:*}; e=""; [ "$it" != "$v" ] && e=${it#*:}
      L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
      tag=$(echo "$it" | tr ':=,/' '____')_$w
      S="--sweep 0"; [ "$w" = points ] && S="--sweep 1"
      env ORBPL_LIB=$L ${e//+/ } timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 $S $C > gpurun_out/abw/$tag.log 2>&1 || { echo "fail $it $w"; tail -5 gpurun_out/abw/$tag.log; exit 1; }
      grep '^{' gpurun_out/abw/$tag.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); b=d.get('summary',{}).get('batch1_ms',{})
print('$r $w $it', round(d['value']), d['ms_per_step'], 'batch1', b)"
    done
  done
done
