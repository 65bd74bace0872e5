#!/bin/bash
# Build an A/B variant of liborbpl.so with extra -D flags for one source file.
#   tools/build_variant.sh <name> <source.hip> -DFOO=1 ...
# -> variants/<name>/liborbpl.so ; run with ORBPL_LIB=variants/<name>/liborbpl.so
set -euo pipefail
name=$1; src=$2; shift 2
here=$(cd "$(dirname "$0")/.." && pwd)
csrc=$here/orb_slam2_modification_with-point-and-line-feature_amd/csrc
obj=$here/orb_slam2_modification_with-point-and-line-feature_amd/build_obj
out=$here/variants/$name
mkdir -p "$out"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -Wno-unused-result"
# several sources: comma-separated (a layout shared by two kernels' files)
objs=$(ls $obj/*.o)
mine=""
for s in ${src//,/ }; do
  /opt/rocm/bin/hipcc $F "$@" -x hip -c "$csrc/$s" -o "$out/$s.o"
  objs=$(echo "$objs" | grep -v "/$s.o\$")
  mine="$mine $out/$s.o"
done
/opt/rocm/bin/hipcc $F -shared -o "$out/liborbpl.so" $objs $mine
echo "$out/liborbpl.so"
