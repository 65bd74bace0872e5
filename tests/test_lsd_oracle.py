"""CPU tests of the line-feature oracle (oracle/lsd_oracle.cpp) and of the
pinned math it shares with the kernels (csrc/lsd_math.h)."""
import hashlib
import math
from pathlib import Path

import numpy as np
import pytest


def _ulp(a, b):
    return 0 if a == b else abs(a - b) / math.ulp(max(abs(a), abs(b)))


@pytest.mark.parametrize("fn,f,lo,hi,bound", [
    (0, math.exp, -40, 40, 1), (1, math.log, 1e-6, 1e6, 1), (2, math.log10, 1e-6, 1e6, 2),
    (3, math.sin, -10, 10, 1), (4, math.cos, -10, 10, 1), (6, math.sinh, -0.6, 0.6, 8)])
def test_pinned_math_within_ulps_of_libm(oracle, fn, f, lo, hi, bound):
    xs = np.random.default_rng(fn).uniform(lo, hi, 4000)
    assert max(_ulp(oracle.lsdm(fn, x), f(x)) for x in xs) <= bound


def test_pinned_atan2_within_one_ulp(oracle):
    rng = np.random.default_rng(5)
    for x, y in zip(rng.uniform(-50, 50, 4000), rng.uniform(-50, 50, 4000)):
        assert _ulp(oracle.lsdm(5, x, y), math.atan2(y, x)) <= 1
    for x, y in [(0.0, 1.0), (0.0, -1.0), (-1.0, 0.0), (1.0, 0.0), (-3.0, -0.0)]:
        assert oracle.lsdm(5, x, y) == math.atan2(y, x)


def test_line_iterator_count(oracle):
    assert oracle.line_iterator_count(640, 480, 0, 0, 10, 3) == 11
    assert oracle.line_iterator_count(640, 480, 5.4, 5.6, 5.4, 5.6) == 1
    assert oracle.line_iterator_count(640, 480, 2.5, 0, 3.5, 0) == 3  # cvRound: 2, 4
    assert oracle.line_iterator_count(640, 480, -10, 10, 10, 10) == 11  # clipped at x = 0
    assert oracle.line_iterator_count(640, 480, -10, -10, -5, -5) == 0  # fully outside


def test_introsort_oracle_is_a_descending_permutation(oracle):
    keys = np.random.default_rng(1).integers(0, 16, 3000)
    perm = oracle.introsort_perm(keys)
    assert np.array_equal(np.sort(perm), np.arange(3000))
    assert np.all(np.diff(keys[perm]) <= 0)


def _tilted_rect(deg=12.0):
    """Bright square rotated by `deg` on a dark background (4x supersampled)."""
    ss = 4
    ys, xs = np.mgrid[0:480 * ss, 0:640 * ss].astype(np.float64) / ss
    a = np.deg2rad(deg)
    u = (xs - 320) * np.cos(a) + (ys - 240) * np.sin(a)
    v = -(xs - 320) * np.sin(a) + (ys - 240) * np.cos(a)
    inside = (np.abs(u) < 120) & (np.abs(v) < 120)
    img = 40 + 160 * inside.reshape(480, ss, 640, ss).mean(axis=(1, 3))
    return img.round().astype(np.uint8), a


@pytest.mark.parametrize("deg", [3.0, 12.0, 30.0, 45.0, 80.0])
def test_lsd_finds_tilted_square_edges(oracle, deg):
    img, a = _tilted_rect(deg)
    L = oracle.lsd_detect(img)
    lens = np.hypot(L[:, 0] - L[:, 2], L[:, 1] - L[:, 3])
    long_ = L[lens > 150]
    assert len(long_) >= 4
    # every long segment lies on one of the square's sides |u| = 120 or |v| = 120
    for x1, y1, x2, y2 in long_:
        for x, y in ((x1, y1), (x2, y2)):
            u = (x - 320) * np.cos(a) + (y - 240) * np.sin(a)
            v = -(x - 320) * np.sin(a) + (y - 240) * np.cos(a)
            assert min(abs(abs(u) - 120), abs(abs(v) - 120)) < 2.5


def test_line_extract_keeps_80_longest(oracle):
    from _scenes import sequence
    cfg, traj, fr = sequence(1, 1)
    kl, desc, coef, nd = oracle.line_extract(fr[0][0])
    assert nd > 80 and len(kl) == 80 and desc.shape == (80, 32)
    assert np.all(np.diff(kl["response"]) <= 0)
    assert np.allclose(np.linalg.norm(coef, axis=1), 1.0)
    # coefficients are the normalised cross product of the homogeneous end points
    s = np.stack([kl["startPointX"], kl["startPointY"], np.ones(80)], 1).astype(np.float64)
    e = np.stack([kl["endPointX"], kl["endPointY"], np.ones(80)], 1).astype(np.float64)
    c = np.cross(s, e)
    assert np.allclose(coef, c / np.linalg.norm(c, axis=1, keepdims=True))
    assert np.all(kl["octave"] == 0) and len(set(kl["class_id"])) == 80


LINE_GOLDEN = sorted((Path(__file__).resolve().parent / "golden").glob("lines_*.npz"))


@pytest.mark.parametrize("path", LINE_GOLDEN, ids=[p.stem for p in LINE_GOLDEN])
def test_line_oracle_matches_golden(path, oracle, synth):
    z = np.load(path)
    img = synth.textured_image(int(z["width"]), int(z["height"]), seed=int(z["seed"]))
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(z["sha256"])
    assert np.array_equal(oracle.lsd_detect(img), z["lsd_lines"])
    kl, desc, coef, nd = oracle.line_extract(img)
    assert kl.view(np.uint8).tobytes() == z["keylines"].tobytes()
    assert np.array_equal(desc, z["desc"]) and np.array_equal(coef, z["coef"])
    assert nd == int(z["n_detected"])


def test_lsd_traffic_counts(oracle):
    """The instrumented detection (oracle.lsd_traffic: the touch floors of the
    LSD kernels in bench.py) finds the same segments and its counts hold the
    algorithm's invariants: every added region point is expanded once, every
    expansion reads at most 8 neighbours, the sort makes ~log2(n) compares
    per element, every refined rectangle is NFA-evaluated at least once."""
    from _scenes import sequence
    cfg, traj, fr = sequence(1, 1)
    img = fr[0][0]
    t = oracle.lsd_traffic(img)
    assert t["segments"] == len(oracle.lsd_detect(img)) > 100
    assert t["grow_add"] == t["grow_expand"]
    assert t["grow_expand"] < t["grow_nb"] <= 8 * t["grow_expand"]
    sw, sh = 512, 384
    n = (sw - 1) * (sh - 1)
    assert t["seeds"] == n
    assert 10 * n < t["sort_cmp"] < 30 * n and t["sort_moves"] > n
    assert t["nfa_evals"] >= t["segments"] and t["nfa_px"] > t["nfa_evals"]
    assert t["grows"] >= t["nfa_evals"] / 16
    # distinct addresses: bounded by the image and by the access counts
    assert t["sort_n"] == n
    assert t["u_used_px"] <= t["u_seed_px"] <= sw * sh
    assert t["u_seed_px"] <= t["seeds"] + t["grow_nb"]
    assert t["u_q_px"] <= t["u_used_px"] and t["u_nfa_px"] <= min(t["nfa_px"], sw * sh)
    assert 0 < t["max_reg"] < sw * sh and t["segments"] <= t["rects"] <= t["nfa_evals"]
