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
/opt/rocm/bin/hipcc $F "$@" -x hip -c "$csrc/$src" -o "$out/$src.o"
objs=$(ls $obj/*.o | grep -v "/$src.o\$")
/opt/rocm/bin/hipcc $F -shared -o "$out/liborbpl.so" $objs "$out/$src.o"
echo "$out/liborbpl.so"
