#!/bin/bash
# Round-3 pass f: full -m gpu suite at HEAD's library, then the seed-loop A/B
# (in-tree library vs variants given in $1) with the LSD parity tests per
# variant and the LSD probe at batch 1 / 3072.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" $O/gpu_tests.log | head -20; exit $rc; }
bash tools/ab_lsd_variants.sh "$1"
