#!/bin/bash
# Round-4 pass s: k_lsd_sort with an LDS segment table and larger partition
# chunks (cur: 1024 elements; c1024w8 / c512w8: register budget of 8 waves;
# c256: table only) against the previous sort (base): LSD parity of cur and
# c512w8, k_lsd_sort kernel time at 1 / 1536 frames, then the lines leg.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04s
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
for v in cur c512w8; do
  L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
  ORBPL_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests_$v.log 2>&1 || { echo "$v parity FAILED"; tail -30 $O/lsd_tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/lsd_tests_$v.log)"
done
cd /tmp && export TMPDIR=/tmp
for B in 1 1536; do
  for v in base cur c1024w8 c512w8 c256; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${v}_$B -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $O/${v}_$B.log 2>&1 || { echo "$v $B failed"; tail -5 $O/${v}_$B.log; exit 1; }
    python3 -c "
import csv
r={x['Name'].split('(')[0]:float(x['AverageNs'])/1e3 for x in csv.DictReader(open('$O/${v}_$B/run_kernel_stats.csv'))}
print('$v', $B, 'sort %.1f us' % r['orbpl::k_lsd_sort'], 'local %.1f us' % r['orbpl::k_lsd_sort_local'])"
  done
done
cd $R
bash tools/ab_lines_lib.sh "base cur c512w8" 2
