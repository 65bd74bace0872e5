#!/bin/bash
# Round-4 pass m: the LSD seed loop's wave-wide fit passes (coop2) and, with
# them, refine's second grow on the whole wave (coopg) against the per-lane
# default (cur): LSD parity of each build (test_gpu_lsd.py through
# ORBPL_LIB), then the detector at 1 / 16 / 1536 frames.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04m
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
for v in coopg coop2; do
  ORBPL_LIB=$R/variants/$v/liborbpl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests_$v.log 2>&1 || { echo "$v parity FAILED"; tail -30 $O/lsd_tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/lsd_tests_$v.log)"
done
for B in 1 16 1536; do
  for v in cur coop2 coopg; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 200 python3 tools/time_lsd.py $B > $O/t_${v}_$B.log 2>&1 || { echo "time $v $B failed"; tail -5 $O/t_${v}_$B.log; exit 1; }
    echo "$v $(head -2 $O/t_${v}_$B.log | tr '\n' ' ' | cut -c1-330)"
  done
done
exit 0
