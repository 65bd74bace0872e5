#!/bin/bash
# Round-4 pass d: seeds per round of the one-wave seed loop (64 / 32 / 16,
# ORBPL_SPEC_WIN build override): per-round grow / fit cycles at batch 1 and
# 16, two rounds. Fewer lanes per wave shrink the union of divergent add
# bodies a grow step executes; the rounds grow in number.
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
for r in 1 2; do
  for v in cur win32 win16; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    for b in 1 16; do
      ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py $b > $O/t_${v}_$b.log 2>&1 || { echo "fail $v $b"; tail -3 $O/t_${v}_$b.log; exit 1; }
      echo "$r $v $(head -2 $O/t_${v}_$b.log | tr '\n' ' ' | cut -c1-330)"
    done
  done
done
exit 0
