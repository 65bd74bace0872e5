#!/bin/bash
# Round-4 pass a: parallel SearchByBoW (k_trk_bow / k_match_bow) and
# TrackReferenceKeyFrame under load (BoW + map parity tests, the headline
# bench with trk_load and a 6-level vocabulary, its kernel trace); the
# prefetching small-batch region grow (LSD parity tests, batch 1 / 16 / 64
# A/B against the build without it and the first-aligned-loop grow).
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_bow.py tests/test_gpu_map.py tests/test_gpu_lsd.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error|FAIL" $O/tests.log | head -20; exit $rc; }
for r in 1 2; do
  for v in cur nopf growloop; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    for b in 1 16 64; do
      ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py $b > $O/t_${v}_$b.log 2>&1 || { echo "fail $v $b"; tail -3 $O/t_${v}_$b.log; exit 1; }
      echo "$r $v $(head -2 $O/t_${v}_$b.log | tr '\n' ' ' | cut -c1-300)"
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
