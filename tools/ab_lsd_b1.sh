set -o pipefail
for r in 1 2; do
for v in cur c725bf30 c12afd9d; do
  L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
  ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py 1 > gpurun_out/b1_$v.log 2>&1 || { echo fail $v; tail -3 gpurun_out/b1_$v.log; exit 1; }
  echo "$r $v $(head -2 gpurun_out/b1_$v.log | tr '\n' ' ')"
done
done
