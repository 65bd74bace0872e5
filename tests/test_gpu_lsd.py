"""GPU parity of the LSD line detector (LineExtractor.cpp:20-21) against the
CPU oracle (oracle/lsd_oracle.cpp): every stage bit-exact."""
from pathlib import Path

import numpy as np
import pytest

from _scenes import sequence

pytestmark = pytest.mark.gpu


def _keysets():
    rng = np.random.default_rng(7)
    yield "tiny", rng.integers(0, 4, 5)
    yield "seventeen", rng.integers(0, 3, 17)
    yield "uniform", rng.integers(0, 1024, 5000)
    yield "dups", rng.integers(0, 8, 20000)
    yield "skewed", np.minimum(1023, rng.exponential(30, 100000).astype(int))
    yield "sorted", np.arange(3000) % 1024
    yield "reversed", (np.arange(3000)[::-1]) % 1024
    yield "constant", np.full(4000, 5)
    yield "organ", np.concatenate([np.arange(2000), np.arange(2000)[::-1]]) % 1024


@pytest.mark.parametrize("name,keys", list(_keysets()), ids=[k for k, _ in _keysets()])
def test_introsort_replica_matches_std_sort(orbpl, oracle, name, keys):
    keys = np.asarray(keys, np.int32)
    assert np.array_equal(orbpl.test_introsort(keys), oracle.introsort_perm(keys))


@pytest.fixture(scope="module")
def frames():
    out = []
    for seed in (1, 2, 3):
        cfg, traj, fr = sequence(1, seed)
        out.append(fr[0][0])
    return out


def test_lsd_stages_bit_exact(orbpl, oracle, frames):
    det = orbpl.LineSegmentDetector(640, 480)
    for g in frames:
        det.detect(g)
        scaled, deg, order = det.stages(0)
        s_o, ang_o, ord_o = oracle.lsd_stages(g)
        assert np.array_equal(scaled, s_o)
        notdef = ang_o == -1024.0
        assert np.array_equal(deg < 0, notdef)
        a = deg.astype(np.float64) * (np.pi / 180)
        assert np.array_equal(a[~notdef], ang_o[~notdef])
        # pseudo-ordering: the list up to its last defined (non-NOTDEF) pixel
        # is the reference's std::sort order exactly; the tail holds only
        # NOTDEF pixels, which the seed loop never takes and the device sort
        # leaves in partition order (same elements)
        defined = ~notdef[ord_o >> 16, ord_o & 0xFFFF]   # list entries: x | y << 16
        last = int(np.nonzero(defined)[0].max()) + 1 if defined.any() else 0
        assert np.array_equal(order[:last], ord_o[:last])
        assert np.array_equal(np.sort(order), np.sort(ord_o))


@pytest.mark.parametrize("fused", ["1", "0"], ids=["k_lsd_prep", "blur_resize_grad"])
def test_lsd_front_paths_bit_exact(orbpl, oracle, frames, fused, monkeypatch):
    """Both LSD fronts against the oracle's scaled image and angles: the fused
    per-tile k_lsd_prep (default) and the three-kernel path it falls back to
    where a tile's source span does not fit (ORBPL_LSD_PREP=0 at create),
    on VGA and on the KITTI geometry (1241x376: ragged last tiles)."""
    monkeypatch.setenv("ORBPL_LSD_PREP", fused)
    cfg, traj, fr = sequence(1, 4, cam_name="KITTI00", width=1241, height=376)
    for (W, H), imgs in (((640, 480), frames[:2]), ((1241, 376), [fr[0][0]])):
        det = orbpl.LineSegmentDetector(W, H)
        for g in imgs:
            L = det.detect(g)
            scaled, deg, order = det.stages(0)
            s_o, ang_o, ord_o = oracle.lsd_stages(g)
            assert np.array_equal(scaled, s_o)
            notdef = ang_o == -1024.0
            assert np.array_equal(deg < 0, notdef)
            a = deg.astype(np.float64) * (np.pi / 180)
            assert np.array_equal(a[~notdef], ang_o[~notdef])
            assert np.array_equal(L, oracle.lsd_detect(g))


@pytest.mark.parametrize("serial", [False, True], ids=["speculative", "wave_serial"])
def test_lsd_lines_bit_exact(orbpl, oracle, frames, serial):
    det = orbpl.LineSegmentDetector(640, 480)
    det.set_serial_grow(serial)
    for g in frames:
        L = det.detect(g)
        Lo = oracle.lsd_detect(g)
        assert len(L) == len(Lo) and len(L) > 50
        assert np.array_equal(L, Lo)


def test_lsd_batch_device_matches_single(orbpl, oracle, frames):
    B = len(frames)
    det = orbpl.LineSegmentDetector(640, 480, max_batch=B)
    buf = orbpl.DeviceBuffer.from_array(np.stack(frames))
    det.detect_batch_device(buf.ptr, B)
    det.synchronize()
    for f, g in enumerate(frames):
        assert np.array_equal(det.lines(f), oracle.lsd_detect(g))


@pytest.mark.parametrize("B", [128, 800], ids=["4_waves_per_frame", "1_wave_per_frame"])
def test_lsd_batch_multiwave_seed_loop(orbpl, oracle, frames, B):
    """Batches of 97-384 frames run the seed loop with 4 waves per frame,
    larger ones with one (lsd_kernels.h lsd_spec_waves): sampled frames of the
    batch equal the sequential oracle."""
    det = orbpl.LineSegmentDetector(640, 480, max_batch=B)
    buf = orbpl.DeviceBuffer.from_array(np.stack([frames[i % len(frames)] for i in range(B)]))
    det.detect_batch_device(buf.ptr, B)
    det.synchronize()
    ref = [oracle.lsd_detect(g) for g in frames]
    for f in (0, 1, 2, B // 2, B - 1):
        assert np.array_equal(det.lines(f), ref[f % len(frames)])


def test_lsd_batch_multiwave_kitti(orbpl, oracle):
    """4 waves per frame on the KITTI geometry (1241x376: ragged tiles)."""
    kit = [sequence(1, s, cam_name="KITTI00", width=1241, height=376)[2][0][0] for s in (4, 5)]
    B = 128
    det = orbpl.LineSegmentDetector(1241, 376, max_batch=B)
    buf = orbpl.DeviceBuffer.from_array(np.stack([kit[i % 2] for i in range(B)]))
    det.detect_batch_device(buf.ptr, B)
    det.synchronize()
    ref = [oracle.lsd_detect(g) for g in kit]
    for f in (0, 1, B - 2, B - 1):
        assert np.array_equal(det.lines(f), ref[f % 2])


def test_lsd_kitti_geometry(orbpl, oracle):
    cfg, traj, fr = sequence(1, 4, cam_name="KITTI00", width=1241, height=376)
    g = fr[0][0]
    det = orbpl.LineSegmentDetector(1241, 376)
    assert np.array_equal(det.detect(g), oracle.lsd_detect(g))


def _cmp_keylines(kl, desc, coef, kl_o, desc_o, coef_o):
    assert len(kl) == len(kl_o)
    for name in kl.dtype.names:
        assert np.array_equal(kl[name], kl_o[name]), name
    assert np.array_equal(desc, desc_o)
    assert np.array_equal(coef, coef_o)


@pytest.mark.parametrize("fused", ["1", "0"], ids=["blur_sobel", "blur_then_sobel"])
def test_line_extract_bit_exact(orbpl, oracle, frames, fused, monkeypatch):
    """KeyLines, LBD rows and coefficients; the LBD gradients from the fused
    5x5 blur + Sobel kernel (default) and from the separate kernels."""
    monkeypatch.setenv("ORBPL_BLUR_SOBEL", fused)
    ex = orbpl.LineExtractor(640, 480)
    for g in frames:
        kl, desc, coef = ex.ExtractLineSegment(g)
        kl_o, desc_o, coef_o, nd = oracle.line_extract(g)
        assert nd > 80 and len(kl) == 80
        _cmp_keylines(kl, desc, coef, kl_o, desc_o, coef_o)


def test_line_extract_batch_and_few_lines(orbpl, oracle, frames):
    # a frame with fewer than 80 segments keeps detection order (no sort)
    few = np.full((480, 640), 60, np.uint8)
    few[100:300, 200:400] = 180
    imgs = np.stack(frames + [few])
    ex = orbpl.LineExtractor(640, 480, max_batch=len(imgs))
    buf = orbpl.DeviceBuffer.from_array(imgs)
    ex.extract_batch_device(buf.ptr, len(imgs))
    ex.synchronize()
    for f, g in enumerate(imgs):
        kl_o, desc_o, coef_o, nd = oracle.line_extract(g)
        _cmp_keylines(*ex.keylines(f), kl_o, desc_o, coef_o)
    assert 0 < len(ex.keylines(len(imgs) - 1)[0]) < 80


def test_line_extract_kitti(orbpl, oracle):
    cfg, traj, fr = sequence(1, 5, cam_name="KITTI00", width=1241, height=376)
    g = fr[0][0]
    ex = orbpl.LineExtractor(1241, 376)
    kl_o, desc_o, coef_o, nd = oracle.line_extract(g)
    _cmp_keylines(*ex.ExtractLineSegment(g), kl_o, desc_o, coef_o)


def test_lsd_regions_longer_than_a_lane_buffer(orbpl, oracle):
    """Sawtooth images: every tooth is one aligned region of ~20k pixels,
    beyond a lane's speculative buffer, so the speculative loop hands those
    seeds to the wave-cooperative program. Lines equal the oracle's."""
    x = np.arange(640)[None, :].repeat(480, 0)
    y = np.arange(480)[:, None].repeat(640, 1)
    imgs = [((x * 8) % 256).astype(np.uint8), (((x + 2 * y) * 3) % 256).astype(np.uint8)]
    det = orbpl.LineSegmentDetector(640, 480)
    for img in imgs:
        L = det.detect(img)
        assert np.array_equal(L, oracle.lsd_detect(img))
        assert det.debug_profile()["coop_regions"] > 0
    # the same with 4 waves per frame (a batch of 128): wave 0 runs the
    # cooperative program while the others wait
    B = 128
    det = orbpl.LineSegmentDetector(640, 480, max_batch=B)
    buf = orbpl.DeviceBuffer.from_array(np.stack([imgs[i % 2] for i in range(B)]))
    det.detect_batch_device(buf.ptr, B)
    det.synchronize()
    for f in (0, 1, B - 1):
        assert np.array_equal(det.lines(f), oracle.lsd_detect(imgs[f % 2]))


LINE_GOLDEN = sorted((Path(__file__).resolve().parent / "golden").glob("lines_*.npz"))


@pytest.mark.parametrize("path", LINE_GOLDEN, ids=[p.stem for p in LINE_GOLDEN])
def test_line_extract_matches_golden(orbpl, synth, path):
    z = np.load(path)
    w, h = int(z["width"]), int(z["height"])
    img = synth.textured_image(w, h, seed=int(z["seed"]))
    det = orbpl.LineExtractor(w, h)
    assert np.array_equal(det.detect(img), z["lsd_lines"])
    kl, desc, coef = det.ExtractLineSegment(img)
    assert kl.view(np.uint8).tobytes() == z["keylines"].tobytes()
    assert np.array_equal(desc, z["desc"]) and np.array_equal(coef, z["coef"])
