#!/bin/bash
# Round-4 pass ah: lines leg at 3072 streams with k_lsd_validate at 4
# workgroups per frame (val4) and k_lsd_sort at 1024 threads for every batch
# (widesort: ORBPL_SORT_WIDE_BATCH=4096) against the defaults, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/abl
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for r in 1 2; do
  for v in cur val4 widesort; do
    L=""; [ "$v" = val4 ] && L=variants/$v/liborbpl.so
    W=256; [ "$v" = widesort ] && W=4096
    ORBPL_SORT_WIDE_BATCH=$W ORBPL_LIB=$L timeout -k 10 300 python bench.py --workload lines --streams 3072 --steps 4 --warmup 1 $C > gpurun_out/abl/b_$v.log 2>&1 || { echo "fail bench $v"; exit 1; }
    grep '^{' gpurun_out/abl/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $v lines', round(d['value']), d['ms_per_step'])"
  done
done
