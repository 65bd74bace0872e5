#!/bin/bash
# Round-4 pass b: small-batch seed-loop A/B (prefetching grow vs without vs
# the first-aligned-loop grow) at batch 1 / 16 / 64, two rounds; then the
# headline bench with trk_load and its kernel trace.
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
for r in 1 2; do
  for v in cur nopf pf2 growloop; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    for b in 1 16 64; do
      ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py $b > $O/t_${v}_$b.log 2>&1 || { echo "fail $v $b"; tail -3 $O/t_${v}_$b.log; exit 1; }
      echo "$r $v $(head -2 $O/t_${v}_$b.log | tr '\n' ' ' | cut -c1-250)"
    done
  done
done
COMMON="--no-cpu-baseline --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 $COMMON > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['parity']['pass']); print(json.dumps(d.get('trk_load'))); print(json.dumps(d['summary']))"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && export GPU_MAX_HW_QUEUES=16
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-parity $COMMON > $R/$O/trace.log 2>&1
rc=$?; echo "trace exit $rc"; [ $rc -ne 0 ] && { tail -5 $R/$O/trace.log; exit $rc; }
f=$(find $R/$O/trace -name "*kernel_stats.csv" | head -1)
grep -E "Name|k_trk_bow|k_fast|k_pose" $f | cut -c1-200
exit 0
