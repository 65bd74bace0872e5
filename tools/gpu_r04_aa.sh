#!/bin/bash
# Round-4 pass aa: the seed scan with two list windows per iteration (cur)
# against one (scan1): LSD parity, then 1 / 16 / 1536 frames, two rounds;
# "sel" = the seed loop's cycles outside grow / fit / commit (the scans).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04aa
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1 || { echo "parity FAILED"; tail -30 $O/lsd_tests.log; exit 1; }
echo "cur $(tail -1 $O/lsd_tests.log)"
for r in 1 2; do
for B in 1 16 1536; do
  for v in cur scan1; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 200 python3 tools/time_lsd.py $B > $O/t_${v}_${B}_$r.log 2>&1 || { echo "time $v $B failed"; tail -5 $O/t_${v}_${B}_$r.log; exit 1; }
    python3 -c "
import ast
L=open('$O/t_${v}_${B}_$r.log').read().splitlines()
p=ast.literal_eval(L[1].split(': ',1)[1])
print('$v', L[0].split(',')[0], 'sel %.1fM' % ((p['total_cyc']-p['grow_cyc']-p['fit_cyc']-p['validate_commit_cyc'])/1e6), 'total %.1fM' % (p['total_cyc']/1e6))"
  done
done
done
