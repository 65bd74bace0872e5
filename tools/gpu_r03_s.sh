#!/bin/bash
# Round-3 pass s: streams-per-GPU sweep of every leg at 16 hardware queues
# (split LSD on), parity on.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03s
mkdir -p $O
cd $R
C="--no-cpu-baseline --sweep 0 --isolated-steps 0 --ingress-steps 0"
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python bench.py "$@" $C > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], 'parity', d['parity']['pass'])"
}
for s in 1024 1536 2048; do run p_$s --streams $s --steps 20 --warmup 5 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 || exit 1; done
for s in 2048 3072 4096; do run l_$s --workload lines --streams $s --steps 5 --warmup 2 || exit 1; done
for s in 1024 1536 2048; do run k_$s --workload kitti --streams $s --steps 5 --warmup 2 || exit 1; done
for s in 256 512 1024; do run r_$s --workload rig --streams $s --steps 10 --warmup 3 || exit 1; done
