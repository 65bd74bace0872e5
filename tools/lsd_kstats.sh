#!/bin/bash
# Kernel stats of the LSD probe (tools/time_lsd.py <batch>) under rocprofv3,
# per env setting: gpurun_out/lsdk/<tag>.csv. usage: tools/lsd_kstats.sh <batch> "<env|-> ..."
set -o pipefail
B=${1:-1536}; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/lsdk
cd /tmp && export TMPDIR=/tmp
for e in "$@"; do
  tag=$(echo "$e" | tr '=/,:' '____')
  E=""; [ "$e" != "-" ] && E="$e"
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/lsdk_$tag -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $R/gpurun_out/lsdk/$tag.log 2>&1 || { echo "fail $e"; tail -5 $R/gpurun_out/lsdk/$tag.log; exit 1; }
  f=$(find /tmp/lsdk_$tag -name '*kernel_stats.csv' | head -1)
  cp "$f" $R/gpurun_out/lsdk/$tag.csv
  echo "== $e: $(head -1 $R/gpurun_out/lsdk/$tag.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'lsd' in r['Name']: print('  %-40s calls %4s avg %8.3f ms' % (r['Name'].split('(')[0][-40:], r['Calls'], float(r['AverageNs'])/1e6))
"
done
