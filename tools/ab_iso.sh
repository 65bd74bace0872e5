#!/bin/bash
# Headline A/B with the isolated extraction time: items as in tools/ab_lib.sh
# ("<variant>[:NAME=VALUE[+NAME=VALUE]]"), $2 streams (1024), $3 rounds (2).
# Prints frames/s, ms per step and the isolated (non-pipelined) step's
# pyramid + FAST span + octree + orientation/descriptor milliseconds.
set -o pipefail
mkdir -p gpurun_out/ab
B="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 3"
for r in $(seq 1 ${3:-2}); do
  for it in ${1:-cur}; do
    v=${it%%:*}; e=""; [ "$it" != "$v" ] && e=${it#*:}
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    tag=$(echo "$it" | tr ':=,/' '____')
    env ORBPL_LIB=$L ${e//+/ } timeout -k 10 200 python bench.py --streams ${2:-1024} --steps 10 --warmup 3 $B > gpurun_out/ab/iso_${tag}.log 2>&1 || { echo "fail $it"; tail -5 gpurun_out/ab/iso_${tag}.log; exit 1; }
    grep '^{' gpurun_out/ab/iso_${tag}.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); i=d['roofline']['isolated']['stage_ms']
ext=sum(i[k] for k in ('pyramid','fast','octree','orient_desc'))
print('$it', round(d['value']), d['ms_per_step'], 'iso pyr %.2f fast %.2f oct %.2f od %.2f' % (i['pyramid'], i['fast'], i['octree'], i['orient_desc']))"
  done
done
