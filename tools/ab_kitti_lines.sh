#!/bin/bash
# Stereo (configs[3], 1024 pairs) and lines (configs[2], 3072 streams) legs
# over library variants ($1, "cur" = in-tree), $2 rounds alternating.
set -o pipefail
mkdir -p gpurun_out/abk
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
VS=${1:-cur}
for r in $(seq 1 ${2:-2}); do
  for v in $VS; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    for w in "kitti 1024" "lines 3072"; do
      wl=${w% *}; ns=${w#* }
      ORBPL_LIB=$L timeout -k 10 300 python bench.py --workload $wl --streams $ns --steps 4 --warmup 1 $C > gpurun_out/abk/b_${v}_$wl.log 2>&1 || { echo "fail $v $wl"; exit 1; }
      grep '^{' gpurun_out/abk/b_${v}_$wl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $v $wl', round(d['value']), d['ms_per_step'], round(d['stage_ms']['lsd_seed'],1))"
    done
  done
done
