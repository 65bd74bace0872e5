#!/bin/bash
# Round-4 pass w: the introsort replay's chunk -> segment map in LDS (cur)
# against the binary search (nomap): LSD parity, kernel time at 1 / 1536
# frames, then the lines leg.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04w
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1 || { echo "parity FAILED"; tail -30 $O/lsd_tests.log; exit 1; }
echo "cur $(tail -1 $O/lsd_tests.log)"
cd /tmp && export TMPDIR=/tmp
for B in 1 1536; do
  for v in cur nomap; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${v}_$B -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $O/${v}_$B.log 2>&1 || { echo "$v $B failed"; tail -5 $O/${v}_$B.log; exit 1; }
    python3 -c "
import csv
r={x['Name'].split('(')[0].split('<')[0]:float(x['AverageNs'])/1e3 for x in csv.DictReader(open('$O/${v}_$B/run_kernel_stats.csv'))}
print('$v', $B, ' '.join('%s %.1f' % (k.replace('orbpl::k_lsd_','').replace('void ',''), v) for k, v in sorted(r.items()) if 'lsd' in k))"
  done
done
cd $R
bash tools/ab_lines_lib.sh "cur nomap" 2
