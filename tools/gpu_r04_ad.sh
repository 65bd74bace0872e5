#!/bin/bash
# Round-4 pass ad (final build of session 2, after the paired descriptor kernel): the whole -m gpu suite at HEAD, smoke(),
# then the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ad
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(json.dumps(d.get('summary'))[:1500])"

cd /tmp && export TMPDIR=/tmp && export GPU_MAX_HW_QUEUES=16
for B in 1 1536; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/lsd_b$B -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $O/lsd_b$B.log 2>&1 || { echo "lsd b$B failed"; tail -5 $O/lsd_b$B.log; exit 1; }
  grep "^batch" $O/lsd_b$B.log
done

cd $R && MODE=points bash tools/prof.sh s2points || exit 1
exit 0
