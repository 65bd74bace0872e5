#!/bin/bash
# Round-3 pass f2 (final build, seed loop keeping valid seeds): full -m gpu suite, profiles of the headline
# (points, 1024 streams) and lines (3072, split LSD) legs, the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03f2
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" $O/gpu_tests.log | head -20; exit $rc; }
MODE=points bash tools/prof.sh r03f2_points || exit 1
MODE=lines bash tools/prof.sh r03f2_lines || exit 1
timeout -k 10 480 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('points', d['value'], 'lines', d['secondary']['value'], 'stereo', d['stereo']['value'], 'rig', d['rig']['value'], 'ingress', d['ingress']['value'], 'parity', d['parity']['pass'])"
