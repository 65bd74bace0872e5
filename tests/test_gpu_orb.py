"""GPU parity of the HIP ORB extractor against the CPU oracle: bit-exact
keypoints (all cv::KeyPoint fields) and descriptors, stage by stage."""
import hashlib
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).resolve().parent / "golden"
CASES = sorted(GOLDEN.glob("orb_*.npz"))


def _params(z):
    nf, sf, nl, ini, mn = z["params"]
    return int(nf), float(sf), int(nl), int(ini), int(mn)


def _extractor(orbpl, pp, w, h, batch=1):
    nf, sf, nl, ini, mn = pp
    return orbpl.ORBextractor(nf, sf, nl, ini, mn, width=w, height=h, max_batch=batch)


def _kp_equal(a, b):
    if len(a) != len(b):
        return False
    return all(np.array_equal(a[f].view(np.uint32), b[f].view(np.uint32))
               for f in ("x", "y", "size", "angle", "response")) and \
        np.array_equal(a["octave"], b["octave"]) and np.array_equal(a["class_id"], b["class_id"])


@pytest.mark.parametrize("path", CASES, ids=[p.stem for p in CASES])
def test_gpu_matches_golden(path, orbpl, synth):
    z = np.load(path)
    w, h = int(z["width"]), int(z["height"])
    img = synth.textured_image(w, h, seed=int(z["seed"]))
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(z["sha256"])
    ex = _extractor(orbpl, _params(z), w, h)
    kps, desc = ex(img)
    gk, gd = z["kps"], z["desc"]
    if not _kp_equal(kps, gk):
        cnt = np.bincount(kps["octave"], minlength=len(z["level_counts"]))
        pytest.fail(f"keypoints differ: gpu n={len(kps)} levels={cnt.tolist()} "
                    f"golden n={len(gk)} levels={z['level_counts'].tolist()}")
    ndiff = int((desc != gd).any(axis=1).sum())
    assert ndiff == 0, f"{ndiff} descriptor rows differ"


def test_stage_parity_vga(orbpl, oracle, synth):
    img = synth.textured_image(640, 480, seed=11)
    pp = (1000, 1.2, 8, 20, 7)
    ex = _extractor(orbpl, pp, 640, 480)
    kps, desc = ex(img)
    p = oracle.params(*pp)
    opyr = oracle.pyramid(p, img)
    oblur = oracle.pyramid(p, img, blurred=True)
    for l in range(8):
        g = ex.pyramid_level(l, padded=True)
        assert np.array_equal(g, opyr[l]), f"pyramid level {l} differs"
        gb = ex.pyramid_level(l, blurred=True)
        assert np.array_equal(gb, oblur[l][19:-19, 19:-19]), f"blur level {l} differs"
    gc = ex.candidates()
    oc = oracle.candidates(p, img)
    for l in range(8):
        assert np.array_equal(gc[l], oc[l]), f"FAST candidates level {l} differ"
    okps, odesc, _ = oracle.extract(p, img)
    assert _kp_equal(kps, okps)
    assert np.array_equal(desc, odesc)


@pytest.mark.parametrize("seed", [21, 22, 23])
def test_random_images_match_oracle(seed, orbpl, oracle, synth):
    rng = np.random.default_rng(seed)
    w, h = [(640, 480), (752, 480), (1280, 720)][seed % 3]
    img = synth.textured_image(w, h, seed=seed)
    if seed == 22:   # add saturated blobs and pure-noise stripes (edge-heavy)
        img = img.copy()
        img[100:140, :] = rng.integers(0, 256, (40, w), dtype=np.uint8)
        img[:, 300:310] = 255
    pp = (2000 if w > 1000 else 1000, 1.2, 8, 20, 7)
    ex = _extractor(orbpl, pp, w, h)
    kps, desc = ex(img)
    okps, odesc, _ = oracle.extract(oracle.params(*pp), img)
    assert _kp_equal(kps, okps)
    assert np.array_equal(desc, odesc)


def test_flat_and_empty(orbpl):
    ex = _extractor(orbpl, (1000, 1.2, 8, 20, 7), 640, 480)
    kps, desc = ex(np.full((480, 640), 77, np.uint8))
    assert len(kps) == 0 and desc is None
    kps, desc = ex(np.zeros((0, 0), np.uint8))
    assert len(kps) == 0


def test_batch_device_matches_single(orbpl, synth):
    B = 4
    imgs = np.stack([synth.textured_image(640, 480, seed=30 + i) for i in range(B)])
    ex1 = _extractor(orbpl, (1000, 1.2, 8, 20, 7), 640, 480)
    singles = [ex1(imgs[i]) for i in range(B)]
    exb = _extractor(orbpl, (1000, 1.2, 8, 20, 7), 640, 480, batch=B)
    cap = exb.max_keypoints
    d_img = orbpl.DeviceBuffer.from_array(imgs)
    d_kps = orbpl.DeviceBuffer(B * cap * 28)
    d_desc = orbpl.DeviceBuffer(B * cap * 32)
    d_n = orbpl.DeviceBuffer(B * 4)
    exb.extract_batch_device(d_img.ptr, B, 640, 640 * 480, d_kps.ptr, d_desc.ptr, cap, d_n.ptr)
    exb.synchronize()
    n = d_n.download(np.int32, B)
    kraw = d_kps.download(orbpl.KP_DTYPE, (B, cap))
    dd = d_desc.download(np.uint8, (B, cap, 32))
    for i in range(B):
        assert _kp_equal(kraw[i, :n[i]], singles[i][0])
        assert np.array_equal(dd[i, :n[i]], singles[i][1])


@pytest.mark.parametrize("pipe,groups", [("1", "1/2/3"), ("1", "1/3/5"), ("1", "2/4/6"),
                                         ("0", "")])
def test_level_pipeline_batch_bit_exact(orbpl, synth, monkeypatch, pipe, groups):
    """A 64-frame batch (the level pipeline's minimum, kLevelPipeMinBatch)
    with the pipeline forced on (ORBPL_LEVEL_PIPE=1; several ORBPL_LEVEL_GROUPS
    splits) or off: keypoints, descriptors and counts byte for byte equal to
    single-frame extraction (itself bit-exact against the oracle above)."""
    monkeypatch.setenv("ORBPL_LEVEL_PIPE", pipe)
    if groups:
        monkeypatch.setenv("ORBPL_LEVEL_GROUPS", groups)
    B, U = 64, 8
    uniq = [synth.textured_image(640, 480, seed=60 + i) for i in range(U)]
    imgs = np.stack([uniq[i % U] if i % 3 else np.ascontiguousarray(uniq[i % U][::-1])
                     for i in range(B)])
    ex1 = _extractor(orbpl, (1000, 1.2, 8, 20, 7), 640, 480)
    singles = {}
    exb = _extractor(orbpl, (1000, 1.2, 8, 20, 7), 640, 480, batch=B)
    cap = exb.max_keypoints
    d_img = orbpl.DeviceBuffer.from_array(imgs)
    d_kps = orbpl.DeviceBuffer(B * cap * 28)
    d_desc = orbpl.DeviceBuffer(B * cap * 32)
    d_n = orbpl.DeviceBuffer(B * 4)
    for rep in range(2):   # twice: the second batch reuses the group events and streams
        exb.extract_batch_device(d_img.ptr, B, 640, 640 * 480, d_kps.ptr, d_desc.ptr, cap,
                                 d_n.ptr)
        exb.synchronize()
        n = d_n.download(np.int32, B)
        kraw = d_kps.download(orbpl.KP_DTYPE, (B, cap))
        dd = d_desc.download(np.uint8, (B, cap, 32))
        for i in range(B):
            key = (i % U, bool(i % 3))
            if key not in singles:
                singles[key] = ex1(imgs[i])
            kp, de = singles[key]
            assert n[i] == len(kp) > 0, (rep, i)
            assert _kp_equal(kraw[i, :n[i]], kp), (rep, i)
            assert np.array_equal(dd[i, :n[i]], de), (rep, i)

