"""Model of the seed loop's fit phase (CPU, development): per grown seed the
fit's point-passes (region2rect 3 passes, refine's statistics pass, the
second rect, reduce_region_radius' count + merge + rect passes per iteration)
and the second grow's steps, from an instrumented copy of the oracle's LSD
under /tmp. Rounds of 64 seeds as the wave runs them (conflicts ignored).
Compares, per frame, the fit as the lanes run it now (the round's cost = the
largest lane's point-passes, SIMT) with a wave-cooperative fit (the fitting
regions one after another, each pass over 64 points per step: the round's
cost = the sum of its lanes' point-passes at a cheaper per-point cost), the
second grows staying per lane in both.

usage: python tools/lsd_fit_model.py [frames]
"""
import ctypes
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
OUT = Path("/tmp/lsd_fit_model")


def build():
    OUT.mkdir(exist_ok=True)
    s = (ROOT / "oracle" / "lsd_oracle.cpp").read_text()
    s = s.replace('#include "pinned_math.h"', f'#include "{ROOT}/oracle/pinned_math.h"')
    s = s.replace('#include "oracle_api.h"',
                  f'#include "{ROOT}/oracle/oracle_api.h"\n'
                  'static double C_g1 = 0, C_pp = 0, C_g2 = 0;\n'
                  'extern "C" double fm_costs[1 << 20][3]; double fm_costs[1 << 20][3];\n'
                  'extern "C" int fm_n; int fm_n = 0;')
    subs = [
        ("      radSq *= 0.75 * 0.75;\n      for (size_t i = 0; i < reg.size(); ++i) {",
         "      radSq *= 0.75 * 0.75;\n      C_pp += reg.size();\n      for (size_t i = 0; i < reg.size(); ++i) {"),
        ("      if (reg.size() < 2) return false;\n      region2rect(reg, reg_angle, prec, p, rec);",
         "      if (reg.size() < 2) return false;\n      C_pp += 3 * (double)reg.size();\n"
         "      region2rect(reg, reg_angle, prec, p, rec);"),
        ("    region_grow(reg[0].x, reg[0].y, reg, reg_angle, tau);\n    if (reg.size() < 2) return false;",
         "    C_pp += reg.size();\n    region_grow(reg[0].x, reg[0].y, reg, reg_angle, tau);\n"
         "    C_g2 += reg.size();\n    if (reg.size() < 2) return false;\n    C_pp += 3 * (double)reg.size();"),
        ("      region_grow(px, py, reg, reg_angle, prec);\n      if (reg.size() < min_reg_size) continue;",
         "      region_grow(px, py, reg, reg_angle, prec);\n      C_g1 = reg.size(); C_pp = 0; C_g2 = 0;\n"
         "      struct Rec_ { double* c; ~Rec_() { c[0] = C_g1; c[1] = C_pp; c[2] = C_g2;"
         " if (fm_n < (1 << 20) - 1) fm_n++; } } rr{fm_costs[fm_n]};\n"
         "      if (reg.size() < min_reg_size) continue;\n      C_pp += 3 * (double)reg.size();"),
    ]
    for a, b in subs:
        assert a in s, a
        s = s.replace(a, b)
    (OUT / "lsd_fm.cpp").write_text(s)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-shared",
                           "-o", str(OUT / "libfm.so"), str(OUT / "lsd_fm.cpp"),
                           str(ROOT / "oracle" / "orb_oracle.cpp"), f"-I{ROOT}/oracle", "-lm"])
    return ctypes.CDLL(str(OUT / "libfm.so"))


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    L = build()
    sys.path.insert(0, str(ROOT))
    import bench
    g, _ = bench.render_loop(nf, 1, 4, cam_name="TUM1")
    costs = np.ctypeslib.as_array((ctypes.c_double * (3 << 20)).in_dll(L, "fm_costs")).reshape(-1, 3)
    n = ctypes.c_int.in_dll(L, "fm_n")
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
        g1max = r[:, :, 0].max(1).sum()
        pp_max = r[:, :, 1].max(1).sum()
        pp_sum = r[:, :, 1].sum(1).sum()
        g2max = r[:, :, 2].max(1).sum()
        fitters = (r[:, :, 1] > 0).sum(1)
        print(f"frame {f}: seeds {len(c)} rounds {R}: first-grow steps (round max) {g1max:.0f}; "
              f"fit point-passes: round max {pp_max:.0f}, round sum {pp_sum:.0f} "
              f"(sum / max {pp_sum / max(pp_max, 1):.2f}); second-grow steps (round max) {g2max:.0f}; "
              f"fitting seeds per round {fitters.mean():.2f}")


if __name__ == "__main__":
    main()
