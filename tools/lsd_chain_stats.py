"""Critical-path model of the speculative LSD seed loop (CPU, development).

Builds an instrumented copy of the oracle's LSD restatement under /tmp (the
oracle itself is untouched) that records, per grown seed, the dependent load
round trips a lane of k_lsd_spec spends in region_grow (one per region
point), in the fit (region2rect / weight passes in batches of 8, refine's
second grow) and in reduce_region_radius's removal scan (one per point and
pass when the scan loads a point at a time). Seeds are then grouped in rounds
of 64 as the wave runs them (conflicts ignored) and the per-round maximum of
each part is summed: the round's time is its slowest lane.

usage: python tools/lsd_chain_stats.py [frames]
"""
import ctypes
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
OUT = Path("/tmp/lsd_chain_stats")


def build():
    OUT.mkdir(exist_ok=True)
    s = (ROOT / "oracle" / "lsd_oracle.cpp").read_text()
    s = s.replace('#include "pinned_math.h"', f'#include "{ROOT}/oracle/pinned_math.h"')
    s = s.replace('#include "oracle_api.h"',
                  f'#include "{ROOT}/oracle/oracle_api.h"\n'
                  'static double C_grow = 0, C_fit = 0, C_red = 0;\n'
                  'extern "C" double st_costs[1 << 20][3]; double st_costs[1 << 20][3];\n'
                  'extern "C" int st_n; int st_n = 0;\n'
                  'static inline double b8(size_t n) { return (double)((n + 7) / 8); }')
    subs = [
        ("      radSq *= 0.75 * 0.75;\n      for (size_t i = 0; i < reg.size(); ++i) {",
         "      radSq *= 0.75 * 0.75;\n      C_red += reg.size();\n      for (size_t i = 0; i < reg.size(); ++i) {"),
        ("      if (reg.size() < 2) return false;\n      region2rect(reg, reg_angle, prec, p, rec);",
         "      if (reg.size() < 2) return false;\n      C_red += 3 * b8(reg.size());\n"
         "      region2rect(reg, reg_angle, prec, p, rec);"),
        ("    region_grow(reg[0].x, reg[0].y, reg, reg_angle, tau);\n    if (reg.size() < 2) return false;",
         "    C_fit += b8(reg.size());\n    region_grow(reg[0].x, reg[0].y, reg, reg_angle, tau);\n"
         "    C_fit += reg.size();\n    if (reg.size() < 2) return false;\n    C_fit += 5 * b8(reg.size());"),
        ("      region_grow(px, py, reg, reg_angle, prec);\n      if (reg.size() < min_reg_size) continue;",
         "      region_grow(px, py, reg, reg_angle, prec);\n      C_grow = reg.size(); C_fit = 0; C_red = 0;\n"
         "      struct Rec_ { double* c; ~Rec_() { c[0] = C_grow; c[1] = C_fit; c[2] = C_red;"
         " if (st_n < (1 << 20) - 1) st_n++; } } rr{st_costs[st_n]};\n"
         "      if (reg.size() < min_reg_size) continue;\n      C_fit += 5 * b8(reg.size());"),
    ]
    for a, b in subs:
        assert a in s, a
        s = s.replace(a, b)
    (OUT / "lsd_stats.cpp").write_text(s)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-shared",
                           "-o", str(OUT / "libstats.so"), str(OUT / "lsd_stats.cpp"),
                           str(ROOT / "oracle" / "orb_oracle.cpp"), f"-I{ROOT}/oracle", "-lm"])
    return ctypes.CDLL(str(OUT / "libstats.so"))


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    L = build()
    sys.path.insert(0, str(ROOT))
    import bench
    g, _ = bench.render_loop(nf, 7, 4, cam_name="TUM3")
    costs = np.ctypeslib.as_array((ctypes.c_double * (3 << 20)).in_dll(L, "st_costs")).reshape(-1, 3)
    n = ctypes.c_int.in_dll(L, "st_n")
    out = np.zeros(4 * 5000, np.float32)
    no = ctypes.c_int()
    for f in range(nf):
        img = np.ascontiguousarray(g[f])
        n.value = 0
        L.oracle_lsd_detect(img.ctypes.data_as(ctypes.c_void_p), img.shape[1], img.shape[0],
                            out.ctypes.data_as(ctypes.c_void_p), 5000, ctypes.byref(no))
        c = costs[:n.value].copy()
        R = (len(c) + 63) // 64
        pad = np.zeros((R * 64, 3))
        pad[:len(c)] = c
        r = pad.reshape(R, 64, 3)
        print(f"frame {f}: seeds {len(c)}, lines {no.value}, rounds {R}; per-round max "
              f"(load round trips): grow {r[:, :, 0].max(1).sum():.0f}, fit {r[:, :, 1].max(1).sum():.0f}, "
              f"reduce scan {r[:, :, 2].max(1).sum():.0f}, whole lane {r.sum(2).max(1).sum():.0f}; "
              f"balanced (sum / 64): grow {c[:, 0].sum() / 64:.0f}, whole lane {c.sum() / 64:.0f}; "
              f"seeds >= min size {int((c[:, 1] > 0).sum())}, fit+reduce sum {c[:, 1:].sum():.0f}")


if __name__ == "__main__":
    main()
