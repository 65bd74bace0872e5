"""The compiled C++ drop-in classes (orb_slam2_..._amd/dropin: ORBextractor,
LineExtractor, Frame, KeyFrame, ORBVocabulary, ORBmatcher, LineMatcher,
Optimizer with the reference's signatures, g++-built, linked to liborbpl.so)
against the oracle: three RGB-D frames through extraction, frame glue, the
first frame's map and keyframe (ComputeBoW), the second frame's
TrackWithMotionModel (SearchByProjection points / lines, the pose), the third
frame's TrackReferenceKeyFrame (SearchByBoW, the reference-keyframe line
overload, the pose, the discard) and TrackLocalMap (IsInFrustum,
SearchByProjection over the local map points / lines, the second pose). The
driver binary reads / writes flat files (dropin_driver.cpp's header)."""
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

from _pkg import load_oracle, load_pkg
from _scenes import sequence

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "orb_slam2_modification_with-point-and-line-feature_amd"
DRIVER = PKG / "dropin_driver"


def _frame(buf, off, KP, KL):
    (n,) = struct.unpack_from("<i", buf, off); off += 4
    kps = np.frombuffer(buf, KP, n, off); off += n * KP.itemsize
    desc = np.frombuffer(buf, np.uint8, n * 32, off).reshape(n, 32); off += n * 32
    (nl,) = struct.unpack_from("<i", buf, off); off += 4
    kl = np.frombuffer(buf, KL, nl, off); off += nl * KL.itemsize
    ld = np.frombuffer(buf, np.uint8, nl * 32, off).reshape(nl, 32); off += nl * 32
    coef = np.frombuffer(buf, np.float64, nl * 3, off).reshape(nl, 3); off += nl * 24
    ku = np.frombuffer(buf, KP, n, off); off += n * KP.itemsize
    dep = np.frombuffer(buf, np.float32, n, off); off += n * 4
    return dict(kps=kps, desc=desc, kl=kl, ldesc=ld, coef=coef, kps_un=ku, depth=dep), off


class _Reader:
    def __init__(self, buf):
        self.buf, self.off = buf, 0

    def i32(self, n=None):
        k = 1 if n is None else n
        a = np.frombuffer(self.buf, np.int32, k, self.off)
        self.off += 4 * k
        return int(a[0]) if n is None else a

    def arr(self, dt, n, shape=None):
        a = np.frombuffer(self.buf, dt, n, self.off)
        self.off += a.nbytes
        return a.reshape(shape) if shape else a

    def frame(self, KP, KL):
        F, self.off = _frame(self.buf, self.off, KP, KL)
        return F


@pytest.mark.gpu
@pytest.mark.parametrize("cam_name,seed", [("TUM1", 5), ("TUM3", 8)])
def test_dropin_classes_match_oracle(tmp_path, cam_name, seed):
    pkg = load_pkg()
    O = load_oracle()
    assert DRIVER.exists(), "build the drop-in first (make -C .../dropin)"
    from _vocab import vocabulary
    vpath, _ = vocabulary(k=10, L=5, seed=3, n_frames=8)
    cfg, traj, frames = sequence(3, seed, cam_name=cam_name)
    (g0, d0), (g1, d1), (g2, d2) = frames
    H, W = g0.shape
    orb = (1000, 1.2, 8, 20, 7)
    T0 = np.linalg.inv(traj[0]).astype(np.float32)
    cam = O.camera(cfg)
    camv = [cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"], cfg["k1"], cfg["k2"], cfg["p1"],
            cfg["p2"], cfg["k3"], cam.bf, cam.th_depth]
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(struct.pack("<2i", W, H))
        f.write(np.asarray(camv, np.float32).tobytes())
        f.write(struct.pack("<ifiii", orb[0], orb[1], orb[2], orb[3], orb[4]))
        f.write(T0.tobytes())
        for g, d in frames:
            f.write(np.ascontiguousarray(g, np.uint8).tobytes())
            f.write(np.ascontiguousarray(d, np.float32).tobytes())
        pb = str(vpath).encode()
        f.write(struct.pack("<i", len(pb)) + pb)
    out = tmp_path / "out.bin"
    r = subprocess.run([str(DRIVER), str(inp), str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    R = _Reader(out.read_bytes())
    KP, KL = O.KP_DTYPE, O.KEYLINE_DTYPE
    F0 = R.frame(KP, KL)
    F1 = R.frame(KP, KL)
    p = O.params(*orb)

    def check_frame(F, g, d):
        okps, odesc, _ = O.extract(p, g)
        assert F["kps"].tobytes() == okps.tobytes()
        assert np.array_equal(F["desc"], odesc)
        okl, old, ocoef, _ = O.line_extract(g)
        assert F["kl"].tobytes() == okl.tobytes()
        assert np.array_equal(F["ldesc"], old) and np.array_equal(F["coef"], ocoef)
        ku, dep, ur, _, _ = O.frame_prepare(cam, okps, d)
        assert F["kps_un"].tobytes() == ku.tobytes() and np.array_equal(F["depth"], dep)
        F["uright"] = ur
        F["kl_un"] = O.line_frame_prepare(cam, okl, d)[0]

    check_frame(F0, g0, d0)
    check_frame(F1, g1, d1)
    # ORBextractor::mvImagePyramid of frame 0 = the oracle's level contents
    nlev = R.i32()
    opyr = O.pyramid(p, g0)
    for lv in range(nlev):
        w, h = R.i32(2)
        img = R.arr(np.uint8, w * h, (h, w))
        assert np.array_equal(img, opyr[lv][19:19 + h, 19:19 + w]), lv
    nm, nlm, ninl = R.i32(3)
    T1 = R.arr(np.float32, 16, (4, 4))
    R.i32(F1["kps"].size), R.arr(np.uint8, F1["kps"].size)
    R.i32(F1["kl"].size), R.arr(np.uint8, F1["kl"].size)
    # the oracle's tracking loop over the first two frames (TrackWithMotionModel,
    # no local map: the driver's sequence)
    lvo = O.LVO(p, cam, 1, use_lines=True)
    lvo.reset(T0.reshape(1, 16))
    lvo.step(0, g0, d0)
    To, so = lvo.step(0, g1, d1)
    assert (nm, nlm, ninl) == (so["nmatches"], so["line_matches"], so["ninliers"])
    assert nm > 50 and nlm >= 15
    assert np.abs(T1 - To).max() < 1e-4

    # frame 0's map and the FeatureVectors (Frame / KeyFrame::ComputeBoW)
    N0, NL0 = len(F0["kps"]), len(F0["kl"])
    mp = R.arr(np.dtype([("has", "u1"), ("v", "<f4", 8)]), N0)
    ml = R.arr(np.dtype([("has", "u1"), ("v", "<f4", 6)]), NL0)
    has_mp, has_ml = mp["has"].astype(np.uint8), ml["has"].astype(np.uint8)
    assert np.array_equal(has_mp, (F0["depth"] > 0).astype(np.uint8))
    node0 = R.i32(N0)
    F2 = R.frame(KP, KL)
    check_frame(F2, g2, d2)
    N2, NL2 = len(F2["kps"]), len(F2["kl"])
    node2 = R.i32(N2)
    voc = O.Vocabulary(vpath)
    assert np.array_equal(node0, voc.transform(F0["desc"], 4)[2])
    assert np.array_equal(node2, voc.transform(F2["desc"], 4)[2])

    # TrackReferenceKeyFrame: SearchByBoW(KF0, F2), LineMatcher(0.7)(F2, KF0)
    nb = R.i32()
    bow = R.i32(N2)
    mb_o, nb_o = O.search_by_bow(node0, has_mp, F0["desc"], F0["kps_un"]["angle"], node2,
                                 F2["desc"], F2["kps"]["angle"], 0.7, True)
    assert nb == nb_o and np.array_equal(bow, mb_o), (nb, nb_o)
    assert nb > 20
    nlb = R.i32()
    lbm = R.i32(NL2)
    xyz6 = ml["v"]
    ml_o, nl_o, _ = O.line_search_by_projection_list(cam, T1, F2["kl_un"], F2["ldesc"], None,
                                                      has_ml, xyz6, F0["ldesc"])
    assert nlb == nl_o and np.array_equal(lbm, ml_o)
    go, ninl2 = R.i32(2)
    T2 = R.arr(np.float32, 16, (4, 4))
    out2, lout2 = R.arr(np.uint8, N2), R.arr(np.uint8, NL2)
    nmap, lnmap = R.i32(2)
    assert go == int(nb >= 15 and nlb >= 10)
    lw, lh, nfl, scl, isc = O.level_sizes(p, W, H)
    isg = (1.0 / (scl * scl)).astype(np.float32)

    def pose(match, lmatch, T):
        prob = dict(kps_un=F2["kps_un"], uright=F2["uright"], has_mp=(match >= 0).astype(np.uint8),
                    mp_xyz=np.where((match >= 0)[:, None], mp["v"][np.maximum(match, 0), :3], 0),
                    inv_sigma2=isg,
                    kl_obs=np.stack([F2["kl_un"][k] for k in ("startPointX", "startPointY",
                                                              "endPointX", "endPointY")], 1),
                    kl_octave=F2["kl_un"]["octave"], has_ml=(lmatch >= 0).astype(np.uint8),
                    ml_xyz=np.where((lmatch >= 0)[:, None], xyz6[np.maximum(lmatch, 0)], 0))
        return O.pose_optimization(cam, prob, T, np.zeros(N2, np.uint8), np.zeros(NL2, np.uint8))

    m2, l2 = bow.copy(), lbm.copy()
    Tcur = T1
    if go:
        To2, oo, lo, no = pose(m2, l2, T1)
        assert np.abs(T2 - To2).max() < 1e-4 and ninl2 == no
        assert np.array_equal(out2, oo) and np.array_equal(lout2, lo)
        m2[(m2 >= 0) & (oo == 1)] = -1
        l2[(l2 >= 0) & (lo == 1)] = -1
        assert nmap == int((m2 >= 0).sum())
        Tcur = T2
    else:
        assert np.array_equal(T2, T1)
        m2[:] = -1          # the matches stay in vpMapPointMatches (Tracking.cc:968-973)

    # TrackLocalMap over KF0: SearchLocalPoints
    seen, inview = R.arr(np.uint8, N0), R.arr(np.uint8, N0)
    nloc = R.i32()
    mloc = R.i32(N2)
    want_seen = np.zeros(N0, np.uint8)
    want_seen[m2[m2 >= 0]] = 1
    if go:   # the discarded outliers are marked seen too (Tracking.cc:1006-1011)
        want_seen[bow[(bow >= 0) & (oo == 1)]] = 1
    assert np.array_equal(seen, want_seen)
    loc = np.nonzero(has_mp)[0]          # UpdateLocalPoints: KF0's map points in index order
    mps = dict(xyz=mp["v"][loc, :3], normal=mp["v"][loc, 3:6], min_dist=mp["v"][loc, 6],
               max_dist=mp["v"][loc, 7])
    tr = O.frame_is_in_frustum(cam, float(np.float32(O.lsdm(1, float(np.float32(1.2))))), 8,
                               Tcur, mps, 0.5)
    tr["in_view"] = tr["in_view"] & (seen[loc] == 0)
    assert np.array_equal(inview[loc], tr["in_view"]) and not inview[has_mp == 0].any()
    cur = dict(kps_un=F2["kps_un"], desc=F2["desc"], uright=F2["uright"])
    if tr["in_view"].any():
        mlo, nlo = O.search_by_projection_local(cam, scl, cur, tr, F0["desc"][loc],
                                                np.ones(len(loc), np.int32),
                                                (m2 >= 0).astype(np.int32), 3.0, 0.8)
    else:
        mlo, nlo = np.full(N2, -1, np.int32), 0
    want = m2.copy()
    want[mlo >= 0] = loc[mlo[mlo >= 0]]
    assert nloc == nlo and np.array_equal(mloc, want), (nloc, nlo)
    # SearchLocalLines
    lseen, linview = R.arr(np.uint8, NL0), R.arr(np.uint8, NL0)
    nlloc = R.i32()
    lloc = R.i32(NL2)
    want_ls = np.zeros(NL0, np.uint8)
    want_ls[l2[l2 >= 0]] = 1
    if go:
        want_ls[lbm[(lbm >= 0) & (lo == 1)]] = 1
    assert np.array_equal(lseen, want_ls)
    lid = np.nonzero(has_ml)[0]
    lv = O.line_is_in_frustum(Tcur, xyz6[lid]) & (lseen[lid] == 0)
    assert np.array_equal(linview[lid], lv)
    want_l = l2.copy()
    if lv.any():
        mll, nll, wiped = O.line_search_by_projection_list(
            cam, Tcur, F2["kl_un"], F2["ldesc"], (l2 >= 0).astype(np.int32), lv, xyz6[lid],
            F0["ldesc"][lid])
        if wiped:
            want_l[:] = -1
        want_l[mll >= 0] = lid[mll[mll >= 0]]
    else:
        nll = 0
    assert nlloc == nll and np.array_equal(lloc, want_l), (nlloc, nll)
    ninl3 = R.i32()
    T3 = R.arr(np.float32, 16, (4, 4))
    To3, _, _, no3 = pose(mloc, lloc, Tcur)
    assert np.abs(T3 - To3).max() < 1e-4 and ninl3 == no3
    assert R.off == len(R.buf)


def test_dropin_frame_error_reaches_caller():
    """A library error inside the drop-in Frame constructor (an 8x8 image the
    extractors reject on the GPU box; no HIP device here) reaches the caller
    as a C++ exception after the line thread is joined, instead of
    std::terminate (dropin/Frame.cc). No compute is launched."""
    if not DRIVER.exists():
        pytest.skip("dropin_driver not built (__graft_entry__.build())")
    r = subprocess.run([str(DRIVER), "--fail"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert r.stdout.startswith("caught: "), r.stdout


def _features_in_area(ku, gcell, bounds, x, y, r, min_level=-1, max_level=-1):
    """Frame::GetFeaturesInArea (Frame.cc:432-485) restated in numpy float32
    over the oracle's grid cells (gx + 64 gy per keypoint, index order within
    a cell) and image bounds."""
    f32 = np.float32
    minx, maxx, miny, maxy = (f32(v) for v in bounds)
    winv = f32(64) / f32(maxx - minx)
    hinv = f32(48) / f32(maxy - miny)
    x, y, r = f32(x), f32(y), f32(r)
    x0 = max(0, int(np.floor(f32(f32(x - minx) - r) * winv)))
    if x0 >= 64:
        return []
    x1 = min(63, int(np.ceil(f32(f32(x - minx) + r) * winv)))
    if x1 < 0:
        return []
    y0 = max(0, int(np.floor(f32(f32(y - miny) - r) * hinv)))
    if y0 >= 48:
        return []
    y1 = min(47, int(np.ceil(f32(f32(y - miny) + r) * hinv)))
    if y1 < 0:
        return []
    check = min_level > 0 or max_level >= 0
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for j in np.nonzero(gcell == ix + 64 * iy)[0]:
                oc = int(ku["octave"][j])
                if check and (oc < min_level or (max_level >= 0 and oc > max_level)):
                    continue
                if abs(f32(ku["x"][j] - x)) < r and abs(f32(ku["y"][j] - y)) < r:
                    out.append(int(j))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 4])
def test_dropin_stereo_frame_matches_oracle(tmp_path, seed):
    """The drop-in stereo Frame (Frame.cc:71-132: ORB left || right on two
    host threads, ComputeStereoMatches on the two extractors' device
    pyramids), GetFeaturesInArea, and frame 1's TrackWithMotionModel (th = 7,
    zero velocity, PoseOptimizationWithLines with NL = 0) against the oracle:
    keypoints, descriptors, right keypoints, mvKeysUn, mvuRight and mvDepth
    bit-exact, the query results equal, the pose within 1e-4 of the oracle's
    stereo VO loop (LVO.step_stereo) with identical match and inlier counts."""
    load_pkg()
    O = load_oracle()
    assert DRIVER.exists(), "build the drop-in first (make -C .../dropin)"
    from _scenes import stereo_sequence
    cfg, traj, pairs = stereo_sequence(2, seed)
    (l0, r0), (l1, r1) = pairs
    H, W = l0.shape
    orb = (2000, 1.2, 8, 20, 7)
    p = O.params(*orb)
    cam = O.camera(cfg)
    T0 = np.linalg.inv(traj[0]).astype(np.float32)
    camv = [cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"], cfg["k1"], cfg["k2"], cfg["p1"],
            cfg["p2"], cfg["k3"], cam.bf, cam.th_depth]
    queries = [(300.0, 150.0, 20.0, -1, -1), (620.5, 190.25, 7.0, -1, -1),
               (900.0, 60.0, 40.0, 1, 3), (100.0, 300.0, 15.0, 0, 0), (5.0, 5.0, 3.0, -1, -1),
               (-50.0, 100.0, 10.0, -1, -1), (1300.0, 100.0, 30.0, -1, -1),
               (700.0, 200.0, 60.0, 2, -1)]
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(struct.pack("<2i", W, H))
        f.write(np.asarray(camv, np.float32).tobytes())
        f.write(struct.pack("<ifiii", orb[0], orb[1], orb[2], orb[3], orb[4]))
        f.write(T0.tobytes())
        for left, right in pairs:
            f.write(np.ascontiguousarray(left, np.uint8).tobytes())
            f.write(np.ascontiguousarray(right, np.uint8).tobytes())
        f.write(struct.pack("<i", len(queries)))
        for q in queries:
            f.write(struct.pack("<3f2i", *q))
    out = tmp_path / "out.bin"
    r = subprocess.run([str(DRIVER), "--stereo", str(inp), str(out)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    R = _Reader(out.read_bytes())
    KP = O.KP_DTYPE
    frames = []
    for left, right in pairs:
        n = R.i32()
        kps = R.arr(KP, n)
        desc = R.arr(np.uint8, n * 32, (n, 32))
        nr = R.i32()
        kpr = R.arr(KP, nr)
        ku = R.arr(KP, n)
        ur = R.arr(np.float32, n)
        dep = R.arr(np.float32, n)
        okps, odesc, _ = O.extract(p, left)
        okr, odr, _ = O.extract(p, right)
        assert kps.tobytes() == okps.tobytes() and np.array_equal(desc, odesc)
        assert kpr.tobytes() == okr.tobytes()
        oku, _, _, ogc, ob = O.frame_prepare(cam, okps, None)
        assert ku.tobytes() == oku.tobytes()
        our, odep = O.stereo_matches(cam, p, left, right, okps, odesc, okr, odr)
        assert ur.view(np.uint32).tobytes() == our.view(np.uint32).tobytes()
        assert dep.view(np.uint32).tobytes() == odep.view(np.uint32).tobytes()
        assert (dep > 0).sum() > 0.3 * n
        frames.append((oku, ogc, ob))
    oku, ogc, ob = frames[0]
    nonempty = 0
    for q in queries:
        k = R.i32()
        got = R.arr(np.int32, k).tolist()
        assert got == _features_in_area(oku, ogc, ob, *q), q
        nonempty += k > 0
    assert nonempty >= 4
    nm, ninl = R.i32(2)
    T1 = R.arr(np.float32, 16, (4, 4))
    lvo = O.LVO(p, cam, 1, use_lines=False)
    lvo.reset(T0.reshape(1, 16))
    lvo.step_stereo(0, l0, r0)
    To, so = lvo.step_stereo(0, l1, r1)
    assert (nm, ninl) == (so["nmatches"], so["ninliers"]) and nm > 100
    assert np.abs(T1 - To).max() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("cam_name,seed", [("TUM1", 5), ("TUM3", 8)])
def test_dropin_harness_line_overloads_match_oracle(tmp_path, cam_name, seed):
    """The reference's Test/ harness calls against the drop-in LineMatcher
    (dropin_driver --harness): SearchByProjection(F1, F0, new_kls,
    match_indices) (LineMatcher.cpp:272-487, Test/LastFrameProjection.cpp:293),
    SearchByProjection(F2, local map lines, new_kls, match_indices) (:954-1170,
    Test/LocalMapProjectionTest.cpp:334) and SearchByProjection(F2, KF0,
    vpMapLineMatches) (:492-525): counts, new_kls bytes, match_indices and the
    frames' map line assignments equal the oracle's (oracle_line_search_pairs,
    oracle_line_match_bf_knn) on the same lines."""
    load_pkg()
    O = load_oracle()
    assert DRIVER.exists(), "build the drop-in first (make -C .../dropin)"
    cfg, traj, frames = sequence(3, seed, cam_name=cam_name)
    H, W = frames[0][0].shape
    orb = (1000, 1.2, 8, 20, 7)
    T0 = np.linalg.inv(traj[0]).astype(np.float32)
    cam = O.camera(cfg)
    camv = [cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"], cfg["k1"], cfg["k2"], cfg["p1"],
            cfg["p2"], cfg["k3"], cam.bf, cam.th_depth]
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(struct.pack("<2i", W, H))
        f.write(np.asarray(camv, np.float32).tobytes())
        f.write(struct.pack("<ifiii", orb[0], orb[1], orb[2], orb[3], orb[4]))
        f.write(T0.tobytes())
        for g, d in frames:
            f.write(np.ascontiguousarray(g, np.uint8).tobytes())
            f.write(np.ascontiguousarray(d, np.float32).tobytes())
    out = tmp_path / "out.bin"
    r = subprocess.run([str(DRIVER), "--harness", str(inp), str(out)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    R = _Reader(out.read_bytes())
    KL = O.KEYLINE_DTYPE
    fr = []
    for k in range(3):
        nl = R.i32()
        fr.append((R.arr(KL, nl).copy(), R.arr(np.uint8, nl * 32, (nl, 32)).copy()))
    # the frames' lines are the oracle's (extraction + UndistortKeyLines)
    for k, (g, d) in enumerate(frames):
        okl, old, _, _ = O.line_extract(g)
        oku = O.line_frame_prepare(cam, okl, d)[0]
        assert fr[k][0].tobytes() == oku.tobytes() and np.array_equal(fr[k][1], old), k
    nl0 = len(fr[0][0])
    has = np.zeros(nl0, np.uint8)
    xyz = np.zeros((nl0, 6), np.float32)
    nobs = np.zeros(nl0, np.int32)
    for j in range(nl0):
        has[j] = R.arr(np.uint8, 1)[0]
        xyz[j] = R.arr(np.float32, 6)
        nobs[j] = R.i32()
    assert has.sum() > 10 and (nobs[has == 1] > 0).any() and (nobs[has == 1] == 0).any()

    def read_search():
        n = R.i32()
        nn = R.i32()
        kls = R.arr(KL, nn).copy()
        npr = R.i32()
        pr = R.arr(np.int32, 2 * npr, (npr, 2)).copy() if npr else np.zeros((0, 2), np.int32)
        return n, kls, pr

    # A: the last-frame harness overload
    T1 = R.arr(np.float32, 16, (4, 4)).copy()
    nA, klsA, prA = read_search()
    mA = R.i32(len(fr[1][0]))
    m, n, w, pk, ps, pr = O.line_search_pairs(cam, T1, 0, fr[1][0], fr[1][1], None, has,
                                              fr[0][0], xyz, fr[0][1], nobs)
    assert nA == n and klsA.tobytes() == pk.tobytes() and np.array_equal(prA, pr)
    assert np.array_equal(mA, m), (mA, m)
    assert n > 5
    # B: the local-map harness overload over frame 0's map lines (index order)
    T2 = R.arr(np.float32, 16, (4, 4)).copy()
    seen = R.arr(np.uint8, nl0).copy()
    iv = O.line_is_in_frustum(T2, xyz)
    assert np.array_equal(seen[has == 1], iv[has == 1])
    loc = np.nonzero(has)[0]
    nB, klsB, prB = read_search()
    mB = R.i32(len(fr[2][0]))
    m, n, w, pk, ps, pr = O.line_search_pairs(cam, T2, 1, fr[2][0], fr[2][1], None, iv[loc], None,
                                              xyz[loc], fr[0][1][loc], nobs[loc])
    assert nB == n and klsB.tobytes() == pk.tobytes() and np.array_equal(prB, pr)
    assert np.array_equal(mB, np.where(m >= 0, loc[np.maximum(m, 0)], -1))
    # C: BFMatcher knnMatch + ratio against the keyframe of frame 0
    nC = R.i32()
    mC = R.i32(len(fr[2][0]))
    o, n = O.line_match_bf_knn(fr[0][1], fr[2][1])
    assert nC == n > 0
    assert np.array_equal(mC, np.where((o >= 0) & (has[np.maximum(o, 0)] == 1), o, -1))
    assert R.off == len(R.buf)
