#!/bin/bash
# Per-kernel resources (VGPRs, spills, static LDS, scratch) of the gfx950 code
# objects: device-only assembly of every .hip source, metadata summary.
cd "$(dirname "$0")/../orb_slam2_modification_with-point-and-line-feature_amd/csrc"
for f in ${@:-*.hip}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
    -fhip-fp32-correctly-rounded-divide-sqrt --cuda-device-only -S -o /tmp/kres_$f.s -x hip $f 2>/dev/null
  awk '/\.name:/{n=$2} /\.vgpr_count:/{v=$2} /\.vgpr_spill_count:/{sp=$2} /\.group_segment_fixed_size:/{l=$2} /\.private_segment_fixed_size:/{p=$2} /\.max_flat_workgroup_size:/{w=$2} /\.wavefront_size:/{printf "%-60s vgpr %3d spill %3d lds %6d scratch %5d wg %4d\n", substr(n,1,60), v, sp, l, p, w}' /tmp/kres_$f.s
done
