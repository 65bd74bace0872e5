"""CPU tests of the oracle (test infrastructure) against its committed golden
fixtures and against properties of the reference algorithm
(src/ORBextractor.cc). No GPU."""
import hashlib
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"
CASES = sorted(GOLDEN.glob("orb_*.npz"))


def _img(synth, z):
    img = synth.textured_image(int(z["width"]), int(z["height"]), seed=int(z["seed"]))
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(z["sha256"]), \
        "synthetic generator drifted; regenerate tests/golden with make_golden.py"
    return img


@pytest.mark.parametrize("path", CASES, ids=[p.stem for p in CASES])
def test_oracle_matches_golden(path, oracle, synth):
    z = np.load(path)
    img = _img(synth, z)
    p = oracle.params(*[t(v) for t, v in zip((int, float, int, int, int), z["params"])])
    kps, desc, cnt = oracle.extract(p, img)
    assert np.array_equal(cnt, z["level_counts"])
    assert np.array_equal(kps, z["kps"])
    assert np.array_equal(desc, z["desc"])


def test_level_geometry_matches_survey(oracle):
    # SURVEY.md §8 pyramid table for 640x480, 1.2, 8 levels, 1000 features
    lw, lh, nf, sc, isc = oracle.level_sizes(oracle.params(), 640, 480)
    assert lw.tolist() == [640, 533, 444, 370, 309, 257, 214, 179]
    assert lh.tolist() == [480, 400, 333, 278, 231, 193, 161, 134]
    assert nf.tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    assert sum(int(a) * int(b) for a, b in zip(lw, lh)) == 950532
    lw, lh, nf, _, _ = oracle.level_sizes(oracle.params(2000), 1241, 376)
    assert nf.tolist() == [434, 362, 302, 251, 209, 175, 145, 122]


def test_keypoint_invariants(oracle, synth):
    img = synth.textured_image(640, 480, seed=5)
    p = oracle.params()
    kps, desc, cnt = oracle.extract(p, img)
    lw, lh, nf, sc, _ = oracle.level_sizes(p, 640, 480)
    assert desc.shape == (len(kps), 32)
    # level-major order, octave tags, sizes (ORBextractor.cc:837-847, 1075-1104)
    assert np.all(np.diff(kps["octave"]) >= 0)
    for l in range(8):
        k = kps[kps["octave"] == l]
        assert len(k) == cnt[l]
        assert len(k) <= nf[l] + 3
        assert np.all(k["size"] == np.float32(int(31 * sc[l])))
        # level coords stay >= 19 px inside the level content
        x = k["x"] / sc[l] if l else k["x"]
        assert np.all(x >= 18.5) and np.all(x <= lw[l] - 19.5)
    assert np.all((kps["angle"] >= 0) & (kps["angle"] < 360.0))
    assert np.all(kps["class_id"] == -1)


def test_empty_and_flat_images(oracle):
    p = oracle.params()
    flat = np.full((480, 640), 128, np.uint8)
    kps, desc, cnt = oracle.extract(p, flat)
    assert len(kps) == 0 and cnt.sum() == 0


def test_pyramid_border_is_reflect101(oracle, synth):
    img = synth.textured_image(320, 240, seed=7)
    p = oracle.params(500, 1.2, 4, 20, 7)
    levels = oracle.pyramid(p, img)
    L0 = levels[0]
    assert np.array_equal(L0[19:-19, 19:-19], img)
    # BORDER_REFLECT_101: padded(19 - k) == content(k)
    for k in range(1, 20):
        assert np.array_equal(L0[19:-19, 19 - k], img[:, k])
        assert np.array_equal(L0[19 - k, 19:-19], img[k, :])


def test_fast_atan2_properties(oracle):
    # cv::fastAtan2 accuracy is ~0.3 degrees; range [0, 360)
    rng = np.random.default_rng(0)
    for y, x in rng.normal(size=(200, 2)) * 100:
        a = oracle.lib().oracle_fast_atan2(float(y), float(x))
        ref = np.degrees(np.arctan2(y, x)) % 360.0
        d = abs(a - ref)
        assert min(d, 360 - d) < 0.3
