#!/bin/bash
# Round-4 pass m: the wave-cooperative fit of the LSD seed loop: parity (LSD
# tests), then the detector at 1 / 16 / 1536 frames with it (cur) and
# without (nocoop).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04m
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1 || { tail -40 $O/lsd_tests.log; exit 1; }
tail -1 $O/lsd_tests.log
for B in 1 16 1536; do
  for v in cur nogrow2 nocoop; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 200 python3 tools/time_lsd.py $B > $O/t_${v}_$B.log 2>&1 || { echo "time $v $B failed"; tail -5 $O/t_${v}_$B.log; exit 1; }
    echo "$v $(head -2 $O/t_${v}_$B.log | tr '\n' ' ' | cut -c1-400)"
  done
done
exit 0
