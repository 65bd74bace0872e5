#!/bin/bash
# Round-3 pass k: lazy region angle in the grow + reduce_region_radius changes (integer distance test, no
# re-fit when nothing is removed, centroid sums in the merge): LSD parity
# tests, A/B against HEAD's build (variants/base) at batch 1 / 3072, and the
# fit anatomy of the new build.
set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/tests.log | head; exit $rc; }
for r in 1 2; do
  for v in cur nolazy base; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    for b in 1 3072; do
      ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py $b > $O/t_${v}_$b.log 2>&1 || { echo "fail $v $b"; tail -3 $O/t_${v}_$b.log; exit 1; }
      echo "$r $v $(head -1 $O/t_${v}_$b.log | cut -c1-60)"
    done
  done
done
for b in 1 3072; do
  ORBPL_LIB=variants/fitprof/liborbpl.so timeout -k 10 120 python tools/time_lsd.py $b > $O/fitprof_$b.log 2>&1 || { echo "fitprof $b failed"; exit 1; }
  grep fitprof $O/fitprof_$b.log | tail -1
done
