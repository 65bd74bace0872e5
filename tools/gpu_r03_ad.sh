#!/bin/bash
# Round-3 pass ad (final): full -m gpu suite and the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03ad
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 480 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('points', d['value'], 'lines', d['secondary']['value'], 'stereo', d['stereo']['value'], 'rig', d['rig']['value'], 'ingress', d['ingress']['value'], 'parity', d['parity']['pass'])"
