set -o pipefail
mkdir -p gpurun_out/abw
for v in cur w1; do
  L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
  for b in 1 64 256 1024; do
    ORBPL_LIB=$L timeout -k 10 120 python tools/time_lsd.py $b > gpurun_out/abw/${v}_$b.log 2>&1 || { echo "fail $v $b"; exit 1; }
    echo "$v $(head -1 gpurun_out/abw/${v}_$b.log)"
  done
done
