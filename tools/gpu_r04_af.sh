#!/bin/bash
# Round-4 pass af: k_lbd kernel time on the lines leg (3072 streams), batched
# gradient loads (cur) vs the per-sample loop (lbd1).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04af
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && export GPU_MAX_HW_QUEUES=16
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --isolated-steps 0 --ingress-steps 0"
for v in cur lbd1; do
  L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
  ORBPL_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 $R/bench.py --workload lines --streams 3072 --steps 3 --warmup 1 $C > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  python3 -c "
import csv
r={x['Name'].split('(')[0].replace('void ','').replace('orbpl::',''):float(x['AverageNs'])/1e3 for x in csv.DictReader(open('$O/$v/run_kernel_stats.csv'))}
print('$v', ' '.join('%s %.0f' % (k, r[k]) for k in ['k_lbd', 'k_blur_sobel', 'k_keylines'] if k in r))"
done
