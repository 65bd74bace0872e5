"""The -O3 -march=x86-64-v3 / -v4 builds of the oracle (oracle/Makefile,
used by bench.py's CPU baseline) compute the same bits as the -O2 checker:
ORB keypoints + descriptors, LSD/LBD key lines, and three frames of the
points+lines VO loop (poses and counts), each build in its own process."""
import hashlib
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

SCRIPT = r"""
import hashlib, sys
sys.path.insert(0, %(tests)r)
import numpy as np
from _pkg import load_oracle, load_pkg
load_pkg()
O = load_oracle()
O.use_variant(%(variant)r)
from _scenes import sequence
cfg, traj, frames = sequence(3, 61, cam_name="TUM3")
h = hashlib.sha256()
kps, desc, _ = O.extract(O.params(), frames[0][0])
h.update(kps.tobytes()); h.update(desc.tobytes())
kl, ld, coef, _ = O.line_extract(frames[0][0])
h.update(kl.tobytes()); h.update(ld.tobytes()); h.update(coef.tobytes())
lvo = O.LVO(O.params(), O.camera(cfg), 1, use_lines=True)
lvo.reset(np.linalg.inv(traj[0]).astype(np.float32).reshape(1, 16))
for g, d in frames:
    T, st = lvo.step(0, g, d)
    h.update(T.tobytes()); h.update(repr(sorted(st.items())).encode())
print(h.hexdigest())
"""


def _digest(variant):
    out = subprocess.run([sys.executable, "-c", SCRIPT % dict(tests=str(ROOT / "tests"),
                                                              variant=variant)],
                         capture_output=True, text=True, timeout=300, check=True)
    return out.stdout.strip().splitlines()[-1]


def test_fast_builds_bit_identical():
    sys.path.insert(0, str(ROOT))
    from oracle import oracle as O
    level = O.host_isa_level()
    if level == "O2":
        pytest.skip("host runs neither x86-64-v3 nor v4")
    ref = _digest("O2")
    assert _digest("v3") == ref
    if level == "v4":
        assert _digest("v4") == ref
