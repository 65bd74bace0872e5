#!/bin/bash
# Lines workload (configs[2], full Track, pipelined) at several stream counts
# ($1, default "1024 1536 3072"): frames/s and ms per step of each.
set -o pipefail
mkdir -p gpurun_out/lines_sweep
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for s in ${1:-1024 1536 3072}; do
  timeout -k 10 300 python bench.py --workload lines --streams $s --steps 4 --warmup 1 $C > gpurun_out/lines_sweep/l_$s.log 2>&1 || { echo "fail $s"; tail -3 gpurun_out/lines_sweep/l_$s.log; exit 1; }
  grep '^{' gpurun_out/lines_sweep/l_$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($s, round(d['value']), d['ms_per_step'], round(d['stage_ms']['lsd_seed'],1))"
done
