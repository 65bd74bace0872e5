set -o pipefail
B="--workload lines --steps 3 --warmup 1 --no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for s in 1536 2048 3072 4096; do
  timeout -k 10 300 python bench.py --streams $s $B > gpurun_out/lines_$s.log 2>&1 || { echo fail $s; tail -3 gpurun_out/lines_$s.log; exit 1; }
  grep '^{' gpurun_out/lines_$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($s, round(d['value']), d['ms_per_step'], {k: round(d['stage_ms'][k],1) for k in ('lsd','lsd_seed','lsd_sort','lsd_validate','lsd_prep') if k in d['stage_ms']})"
done
