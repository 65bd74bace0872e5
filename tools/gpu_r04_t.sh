#!/bin/bash
# Round-4 pass t: k_lsd_sort with 1024-thread workgroups for batches <= 256
# and the key fill's loads in flight together (cur) against 512 threads at
# every batch (ORBPL_SORT_WIDE_BATCH=0) and the previous sort (base): LSD
# parity, kernel time at 1 / 16 / 1536 frames.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04t
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1 || { echo "parity FAILED"; tail -30 $O/lsd_tests.log; exit 1; }
echo "cur $(tail -1 $O/lsd_tests.log)"
ORBPL_SORT_WIDE_BATCH=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests_nw.log 2>&1 || { echo "narrow parity FAILED"; tail -30 $O/lsd_tests_nw.log; exit 1; }
echo "narrow $(tail -1 $O/lsd_tests_nw.log)"
cd /tmp && export TMPDIR=/tmp
for B in 1 16 1536; do
  for v in base cur narrow; do
    L=""; [ "$v" = base ] && L=$R/variants/$v/liborbpl.so
    W=256; [ "$v" = narrow ] && W=0
    ORBPL_SORT_WIDE_BATCH=$W ORBPL_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${v}_$B -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $O/${v}_$B.log 2>&1 || { echo "$v $B failed"; tail -5 $O/${v}_$B.log; exit 1; }
    python3 -c "
import csv
r={x['Name'].split('(')[0].split('<')[0]:float(x['AverageNs'])/1e3 for x in csv.DictReader(open('$O/${v}_$B/run_kernel_stats.csv'))}
print('$v', $B, ' '.join('%s %.1f' % (k.replace('orbpl::k_lsd_',''), v) for k, v in sorted(r.items()) if 'lsd' in k))"
  done
done
