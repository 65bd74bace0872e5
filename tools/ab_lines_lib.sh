#!/bin/bash
# Lines A/B over library variants and settings: each item of $1 is
# "<variant>[:NAME=VALUE[+NAME=VALUE]]" ("cur" = the in-tree library, else
# variants/<variant>/liborbpl.so): LSD probe at 3072 and the lines workload
# at 3072 streams, $2 rounds alternating.
set -o pipefail
mkdir -p gpurun_out/abl
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
IT=${1:-cur}
for r in $(seq 1 ${2:-2}); do
  # rotate the order every round (the first run of a round is slow)
  set -- $IT
  k=$(( (r - 1) % $# )); ORD="${@:k+1} ${@:1:k}"
  for it in $ORD; do
    v=${it%%:*}; e=""; [ "$it" != "$v" ] && e=${it#*:}
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    tag=$(echo "$it" | tr ':=,/' '____')
    env ORBPL_LIB=$L ${e//+/ } timeout -k 10 120 python tools/time_lsd.py 3072 > gpurun_out/abl/t_$tag.log 2>&1 || { echo "fail probe $it"; exit 1; }
    echo "$r $it probe $(head -1 gpurun_out/abl/t_$tag.log)"
    D=gpurun_out/abl/b_$tag.detail.json
    env ORBPL_LIB=$L ${e//+/ } timeout -k 10 300 python bench.py --workload lines --streams 3072 --steps 4 --warmup 1 $C --detail $D > gpurun_out/abl/b_$tag.log 2>&1 || { echo "fail bench $it"; exit 1; }
    python -c "import json; d=json.load(open('$D')); st=d['stage_ms']; print('$r $it lines', round(d['value']), d['ms_per_step'], {k: round(st[k], 1) for k in ('lsd_sort', 'lsd_seed', 'lsd_validate', 'lsd') if k in st})"
  done
done
