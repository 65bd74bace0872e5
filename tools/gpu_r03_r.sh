#!/bin/bash
# Round-3 pass r: the box's GPU_MAX_HW_QUEUES, then profiles of the split
# build at 16 queues (points headline + lines), then the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}"
MODE=points bash tools/prof.sh r03r_points || exit 1
MODE=lines bash tools/prof.sh r03r_lines || exit 1
timeout -k 10 480 python bench.py > gpurun_out/r03r_bench.json 2> gpurun_out/r03r_bench.err
rc=$?; echo "bench exit $rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03r_bench.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r03r_bench.json').read().strip().splitlines()[-1])
print('points', d['value'], 'lines', d['secondary']['value'], 'stereo', d['stereo']['value'], 'rig', d['rig']['value'], 'ingress', d['ingress']['value'], 'parity', d['parity']['pass'])"
