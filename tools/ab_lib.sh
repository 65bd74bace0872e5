#!/bin/bash
# Headline bench A/B over libraries and settings: each item of $1 is
# "<variant>[:NAME=VALUE]" (variant "cur" = the in-tree library, else
# variants/<variant>/liborbpl.so); stream counts in $2 (default 256); $3 rounds.
set -o pipefail
mkdir -p gpurun_out/ab
IT=${1:-cur}
SS=${2:-256}
RN=${3:-2}
B="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for r in $(seq 1 $RN); do
  # rotate the order every round: the first run of a round is ~0.6 % slow
  # (profiles/r06/ab/trk_prio_ab.txt)
  set -- $IT
  k=$(( (r - 1) % $# )); ORD="${@:k+1} ${@:1:k}"
  for s in $SS; do
    for it in $ORD; do
      v=${it%%:*}; e=""; [ "$it" != "$v" ] && e=${it#*:}
      L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
      tag=$(echo "$it" | tr ':=,/' '____')
      D=gpurun_out/ab/lib_${tag}_$s.detail.json
      env ORBPL_LIB=$L ${e//+/ } timeout -k 10 200 python bench.py --streams $s --steps 10 --warmup 3 $B --detail $D > gpurun_out/ab/lib_${tag}_$s.log 2>&1 || { echo "fail $it $s"; tail -5 gpurun_out/ab/lib_${tag}_$s.log; exit 1; }
      python -c "import json; d=json.load(open('$D')); st=d['stage_ms']; print('$it', $s, round(d['value']), d['ms_per_step'], {k: st.get(k) for k in ('pyramid', 'fast', 'octree', 'orient_desc', 'match', 'pose', 'local_map')})"
    done
  done
done
