#!/bin/bash
# Round-4 pass aj: the whole -m gpu suite and smoke() at the session's HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04aj
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
