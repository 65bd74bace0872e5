#!/bin/bash
# Round-4 pass p: two waves per frame with the cooperative fit (w2c): LSD
# parity of the build, then 1 / 16 frames against cur / coop2 / w2, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04p
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
ORBPL_LIB=$R/variants/w2c/liborbpl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests_w2c.log 2>&1 || { echo "w2c parity FAILED"; tail -30 $O/lsd_tests_w2c.log; exit 1; }
echo "w2c $(tail -1 $O/lsd_tests_w2c.log)"
for r in 1 2; do
for B in 1 16; do
  for v in cur coop2 w2 w2c; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 200 python3 tools/time_lsd.py $B > $O/t_${v}_${B}_$r.log 2>&1 || { echo "time $v $B failed"; tail -5 $O/t_${v}_${B}_$r.log; exit 1; }
    echo "$v $(head -2 $O/t_${v}_${B}_$r.log | tr '\n' ' ' | cut -c1-250)"
  done
done
done
exit 0
