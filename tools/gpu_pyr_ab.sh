#!/bin/bash
# k_pyramid A/B: ORB parity tests on the in-tree build, then per-level phase
# stamps (ORBPL_PYR_PROFILE) and the headline leg for the in-tree library and
# variants/<name>/liborbpl.so ($1, default pyr_old), two rounds each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
V=${1:-pyr_old}
O=$R/gpurun_out/pyr_ab
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > $O/orb_tests.log 2>&1
rc=$?; echo "orb tests exit $rc: $(tail -1 $O/orb_tests.log)"; [ $rc -ne 0 ] && exit $rc
B="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --steps 20 --warmup 5"
for r in 1 2; do
  for lib in cur $V; do
    L=""; [ $lib != cur ] && L=variants/$lib/liborbpl.so
    ORBPL_LIB=$L ORBPL_PYR_PROFILE=1 timeout -k 10 120 python tools/probe_extract.py 1024 > $O/probe_${lib}_$r.log 2>&1 || { echo "probe $lib failed"; tail -5 $O/probe_${lib}_$r.log; exit 1; }
    ORBPL_LIB=$L timeout -k 10 300 python bench.py $B > $O/bench_${lib}_$r.json 2> $O/bench_${lib}_$r.err || { echo "bench $lib failed"; tail -5 $O/bench_${lib}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/bench_${lib}_$r.json').read().strip().splitlines()[-1])
iso=d['roofline'].get('isolated',{}).get('stage_ms',{})
print('$lib', $r, round(d['value']), d['ms_per_step'], 'iso pyr', iso.get('pyramid'), 'fast', iso.get('fast'))"
    grep -E "^B=|total" $O/probe_${lib}_$r.log
  done
done
