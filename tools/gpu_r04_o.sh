#!/bin/bash
# Round-4 pass o: the seed loop at 2 / 4 waves per frame (128 / 256 seeds per
# round, no seed carry) against the one-wave default at 1 / 16 frames, two
# rounds; plus the cooperative fit (coop2) again.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04o
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
for B in 1 16; do
  for v in cur w2 w4 coop2; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 200 python3 tools/time_lsd.py $B > $O/t_${v}_${B}_$r.log 2>&1 || { echo "time $v $B failed"; tail -5 $O/t_${v}_${B}_$r.log; exit 1; }
    echo "$v $(head -2 $O/t_${v}_${B}_$r.log | tr '\n' ' ' | cut -c1-300)"
  done
done
done
exit 0
