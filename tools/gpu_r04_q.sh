#!/bin/bash
# Round-4 pass q: the grow's 32-bit neighbour offsets (cur) against the 64-bit
# address form (u0) at 1 / 16 frames, then k_lsd_sort's register budget /
# (chain0: the cooperative fit's three sums on one lane instead of three)
# workgroup (sortw10, sortw12, sort256) and u0 on the lines leg at 3072 streams.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04q
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1 || { echo "parity FAILED"; tail -30 $O/lsd_tests.log; exit 1; }
echo "cur $(tail -1 $O/lsd_tests.log)"
for r in 1 2; do
for B in 1 16; do
  for v in cur u0 chain0; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 200 python3 tools/time_lsd.py $B > $O/t_${v}_${B}_$r.log 2>&1 || { echo "time $v $B failed"; tail -5 $O/t_${v}_${B}_$r.log; exit 1; }
    echo "$v $(head -2 $O/t_${v}_${B}_$r.log | tr '\n' ' ' | cut -c1-200)"
  done
done
done
bash tools/ab_lines_lib.sh "cur chain0 sortw10 sortw12 sort256" 2
