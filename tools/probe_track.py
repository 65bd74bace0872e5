"""Tracker probe (dev tool): per-stage device times of the points tracker on
the bench's synthetic loop, plus stream 0's PoseOptimization phase profile
when ORBPL_POSE_PROFILE is set (the stream's last pose launch: TrackLocalMap's
with local_map=1). Usage: probe_track.py [streams] [pipelined] [local_map]."""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import bench  # noqa: E402
from _pkg import load_pkg  # noqa: E402

pkg = load_pkg()
import orbpl.synth as synth  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
pipelined = int(sys.argv[2]) if len(sys.argv) > 2 else 0
local_map = int(sys.argv[3]) if len(sys.argv) > 3 else 0
F = 32
gray, depth = bench.render_loop(F, seed=1, workers=min(16, os.cpu_count() or 4))
L = bench.Layout(synth.loop_trajectory(F, seed=1))
rep = L.replicated(S)
d_gray = pkg.DeviceBuffer.from_array(gray[rep])
d_depth = pkg.DeviceBuffer.from_array(depth[rep])
tr = pkg.Tracker(pkg.OrbParams(*bench.ORB), pkg.make_camera(synth.TUM1), S, local_map=bool(local_map))
tr.set_pipelined(bool(pipelined))
tr.reset(np.stack([np.linalg.inv(L.Twc(s, 0)).astype(np.float32) for s in range(S)]).reshape(S, 16))
fb, db = 640 * 480, 640 * 480 * 4
for k in range(12):
    o = k % F
    tr.step_device(d_gray.ptr + o * fb, d_depth.ptr + o * db)
tr.synchronize()
tim = tr.timings(8).mean(0)
print("stage ms:", dict(zip(tr.STAGES, np.round(tim, 3).tolist())))
if os.environ.get("ORBPL_POSE_PROFILE"):
    lib = pkg.lib()
    lib.orbpl_tracker_debug_pose_profile.argtypes = [C.c_void_p, C.c_void_p]
    out = np.zeros(8, np.int64)
    pkg.check(lib.orbpl_tracker_debug_pose_profile(tr._h, out.ctypes.data_as(C.c_void_p)),
              "pose profile")
    names = ("edges", "linearize", "solve_exp", "trial", "classify")
    print("pose stream 0 (us):", {n: round(v / 1000, 1) for n, v in zip(names, out[:5])},
          "iterations", int(out[5]), "trials", int(out[6]),
          "of which linearize edge loop", round(out[7] / 1000, 1))
if os.environ.get("ORBPL_MATCH_PROFILE"):
    lib = pkg.lib()
    lib.orbpl_tracker_debug_match_profile.argtypes = [C.c_void_p, C.c_void_p]
    out = np.zeros(5, np.int64)
    pkg.check(lib.orbpl_tracker_debug_match_profile(tr._h, out.ctypes.data_as(C.c_void_p)),
              "match profile")
    names = ("grid", "candidates", "ordered_claims", "rotation", "output")
    print("match stream 0 (us):", {n: round(v / 1000, 1) for n, v in zip(names, out)})
