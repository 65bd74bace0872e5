"""Quick throughput probe of batched ORB extraction (dev tool)."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from _pkg import load_pkg  # noqa: E402

pkg = load_pkg()
import orbpl.synth as synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
base = [synth.textured_image(640, 480, seed=100 + i) for i in range(8)]
imgs = np.stack([base[i % 8] for i in range(B)])
ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, width=640, height=480, max_batch=B)
cap = ex.max_keypoints
d_img = pkg.DeviceBuffer.from_array(imgs)
d_kps = pkg.DeviceBuffer(B * cap * 28)
d_desc = pkg.DeviceBuffer(B * cap * 32)
d_n = pkg.DeviceBuffer(B * 4)
for it in range(3):
    ex.extract_batch_device(d_img.ptr, B, 640, 640 * 480, d_kps.ptr, d_desc.ptr, cap, d_n.ptr)
    ex.synchronize()
ms = ex.stage_ms()
t = time.time()
R = 10
for it in range(R):
    ex.extract_batch_device(d_img.ptr, B, 640, 640 * 480, d_kps.ptr, d_desc.ptr, cap, d_n.ptr)
ex.synchronize()
dt = (time.time() - t) / R
n = d_n.download(np.int32, B)
print(f"B={B} wall {dt*1e3:.2f} ms/batch -> {B/dt:.0f} fps; stages ms (pyr, blur, fast, octree, desc) = {np.round(ms, 3).tolist()} ; n[0:4]={n[:4].tolist()}")
if getattr(pkg.lib(), "orbx_debug_pyr_profile", None) is not None and __import__("os").environ.get(
        "ORBPL_PYR_PROFILE"):
    import ctypes as C
    out = np.zeros(64, np.int64)
    n = C.c_int(0)
    L = pkg.lib()
    L.orbx_debug_pyr_profile.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_int)]
    pkg.check(L.orbx_debug_pyr_profile(ex._h, out.ctypes.data_as(C.c_void_p), 64, C.byref(n)),
              "orbx_debug_pyr_profile")
    ph = out[:n.value].reshape(-1, 4) / 1000.0
    print("k_pyramid block(0,0) phases us [content, side, mirror, blur] per level:")
    for l, r in enumerate(ph):
        print(f"  L{l}: " + " ".join(f"{x:7.1f}" for x in r))
    print(f"  total {ph.sum():.1f} us")
if __import__("os").environ.get("ORBPL_OCT_PROFILE"):
    import ctypes as C
    L = pkg.lib()
    L.orbx_debug_octree_profile.argtypes = [C.c_void_p, C.c_void_p]
    out = np.zeros(128, np.int64)
    pkg.check(L.orbx_debug_octree_profile(ex._h, out.ctypes.data_as(C.c_void_p)), "octree profile")
    o = out.reshape(16, 8)
    print("k_octree frame 0 per level: setup_us pass_us retain_us passes cands size")
    for l in range(8):
        print(f"  L{l}: {o[l,0]/1000:7.1f} {o[l,1]/1000:7.1f} {o[l,3]/1000:7.1f} {o[l,4]:4d} {o[l,5]:6d} {o[l,6]:5d}")
    print("k_orient_desc first keypoint phases ns [setup, kp load, IC, trig, BRIEF, store]:",
          out[120:126].tolist())
