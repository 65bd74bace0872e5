"""ctypes bindings of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline. The product package never
imports it. Parity status: see orb_oracle.cpp header ("parity unpinned").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liborbpl_oracle.so"
# -O3 -march builds of the same sources (oracle/Makefile) for the CPU baseline
VARIANTS = {"O2": "liborbpl_oracle.so", "v3": "liborbpl_oracle_v3.so",
            "v4": "liborbpl_oracle_v4.so"}


def host_isa_level():
    """Highest x86-64 micro-architecture level this host runs ("v4": AVX-512
    F/BW/CD/DQ/VL, "v3": AVX2/FMA/BMI2, else "O2"), from /proc/cpuinfo."""
    try:
        flags = set()
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                flags = set(line.split(":", 1)[1].split())
                break
    except OSError:
        return "O2"
    v3 = {"avx2", "fma", "bmi1", "bmi2", "movbe", "f16c", "lzcnt" if "lzcnt" in flags else "abm"}
    v4 = {"avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl"}
    if v3 <= flags and v4 <= flags:
        return "v4"
    if v3 <= flags:
        return "v3"
    return "O2"


def use_variant(name):
    """Select the oracle build before the first call ("O2", "v3", "v4" or
    "best" = the highest level the host runs). Returns the variant used."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("oracle library already loaded")
    if name == "best":
        name = host_isa_level()
    LIB_PATH = HERE / "_build" / VARIANTS[name]
    return name


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class KeyPoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        if not LIB_PATH.exists():
            raise FileNotFoundError(LIB_PATH)
        _lib = C.CDLL(str(LIB_PATH))
        _setup(_lib)
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _setup(L):
    vp, ip, i = C.c_void_p, C.POINTER(C.c_int), C.c_int
    L.oracle_orb_level_sizes.argtypes = [vp, i, i, vp, vp, vp, vp, vp]
    L.oracle_orb_pyramid.argtypes = [vp, vp, i, i, i, vp, i]
    L.oracle_orb_candidates.argtypes = [vp, vp, i, i, i, vp, i, vp]
    L.oracle_orb_extract.argtypes = [vp, vp, i, i, i, vp, vp, i, ip, vp]
    L.oracle_fast_atan2.argtypes = [C.c_float, C.c_float]
    L.oracle_fast_atan2.restype = C.c_float


def params(nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
    return OrbParams(nfeatures, scale_factor, nlevels, ini_th, min_th)


def level_sizes(p, w, h):
    n = p.nlevels
    lw = np.zeros(n, np.int32)
    lh = np.zeros(n, np.int32)
    nf = np.zeros(n, np.int32)
    sc = np.zeros(n, np.float32)
    isc = np.zeros(n, np.float32)
    lib().oracle_orb_level_sizes(C.byref(p), w, h, _p(lw), _p(lh), _p(nf), _p(sc), _p(isc))
    return lw, lh, nf, sc, isc


def pyramid(p, img, blurred=False):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    lw, lh, _, _, _ = level_sizes(p, w, h)
    sizes = [(int(a) + 38) * (int(b) + 38) for a, b in zip(lw, lh)]
    out = np.zeros(sum(sizes), np.uint8)
    lib().oracle_orb_pyramid(C.byref(p), _p(img), w, h, w, _p(out), int(blurred))
    levels, off = [], 0
    for a, b, s in zip(lw, lh, sizes):
        levels.append(out[off:off + s].reshape(int(b) + 38, int(a) + 38))
        off += s
    return levels


def candidates(p, img, cap=1 << 20):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((cap, 3), np.float32)
    cnt = np.zeros(p.nlevels, np.int32)
    n = lib().oracle_orb_candidates(C.byref(p), _p(img), w, h, w, _p(out), cap, _p(cnt))
    assert n >= 0
    res, off = [], 0
    for c in cnt:
        res.append(out[off:off + c].copy())
        off += c
    return res


def extract(p, img, cap=None):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    if cap is None:
        cap = p.nfeatures * 2 + 64
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(0)
    cnt = np.zeros(p.nlevels, np.int32)
    rc = lib().oracle_orb_extract(C.byref(p), _p(img), w, h, w, _p(kps), _p(desc), cap,
                                  C.byref(n), _p(cnt))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy(), cnt


# ---------------------------------------------------------------------------
# tracking half (track_oracle.cpp); argument conventions match the product's
# Python mirror (orbpl.frame_prepare / ORBmatcher / pose_optimization)
# ---------------------------------------------------------------------------
class Camera(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("k1", C.c_float), ("k2", C.c_float), ("p1", C.c_float), ("p2", C.c_float),
                ("k3", C.c_float), ("bf", C.c_float), ("th_depth", C.c_float),
                ("width", C.c_int32), ("height", C.c_int32)]


class MatchCurrent(C.Structure):
    _fields_ = [("n", C.c_int32), ("Tcw", C.c_void_p), ("kps_un", C.c_void_p),
                ("desc", C.c_void_p), ("uright", C.c_void_p)]


class MatchLast(C.Structure):
    _fields_ = [("n", C.c_int32), ("Tcw", C.c_void_p), ("kps_un", C.c_void_p),
                ("has_mp", C.c_void_p), ("outlier", C.c_void_p), ("mp_xyz", C.c_void_p),
                ("mp_desc", C.c_void_p), ("mp_nobs", C.c_void_p)]


class PoseProblem(C.Structure):
    _fields_ = [("n", C.c_int32), ("kps_un", C.c_void_p), ("uright", C.c_void_p),
                ("has_mp", C.c_void_p), ("mp_xyz", C.c_void_p), ("nl", C.c_int32),
                ("kl_obs", C.c_void_p), ("kl_octave", C.c_void_p), ("has_ml", C.c_void_p),
                ("ml_xyz", C.c_void_p), ("inv_sigma2", C.c_void_p), ("nlevels", C.c_int32)]


def camera(cfg):
    return Camera(cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"], cfg["k1"], cfg["k2"], cfg["p1"],
                  cfg["p2"], cfg["k3"], cfg["bf"],
                  float(np.float32(cfg["bf"]) * np.float32(cfg["thdepth"]) / np.float32(cfg["fx"])),
                  cfg["width"], cfg["height"])


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _setup_track(L):
    vp, i, ip = C.c_void_p, C.c_int, C.POINTER(C.c_int)
    L.oracle_frame_prepare.argtypes = [vp, vp, i, vp, vp, vp, vp, vp, vp]
    L.oracle_search_by_projection_last.argtypes = [vp, vp, i, vp, vp, C.c_float, i, i, vp, ip]
    L.oracle_pose_optimization.argtypes = [vp, vp, vp, vp, vp, ip]
    L.oracle_pose_optimization_ex.argtypes = [vp, vp, i, vp, vp, vp, ip]
    L.oracle_stereo_matches.argtypes = [vp, vp, vp, i, vp, vp, vp, vp, vp, vp, i, vp, vp, i, vp,
                                        vp]
    L.oracle_search_by_bow.argtypes = [i, vp, vp, vp, vp, i, vp, vp, vp, C.c_float, i, vp, ip]
    L.oracle_frame_is_in_frustum.argtypes = [vp, C.c_float, i, vp, i, vp, vp, vp, vp, C.c_float,
                                             vp, vp, vp, vp, vp, vp]
    L.oracle_search_by_projection_local.argtypes = [vp, vp, i, vp, i, vp, vp, vp, vp, vp, vp, vp,
                                                    vp, vp, C.c_float, C.c_float, vp, ip]
    L.oracle_vo_create.argtypes = [vp, vp, i]
    L.oracle_vo_create.restype = vp
    L.oracle_vo_destroy.argtypes = [vp]
    L.oracle_vo_reset.argtypes = [vp, vp]
    L.oracle_vo_step.argtypes = [vp, i, vp, vp, vp, vp]


_setup_orb = _setup


def _setup(L):  # noqa: F811
    _setup_orb(L)
    _setup_track(L)


def frame_prepare(cam, kps, depth=None):
    kps = _c(kps, KP_DTYPE)
    n = len(kps)
    ku = np.zeros(n, KP_DTYPE)
    d = np.zeros(n, np.float32)
    ur = np.zeros(n, np.float32)
    gc = np.zeros(n, np.int32)
    b = np.zeros(4, np.float32)
    dp = None if depth is None else _c(depth, np.float32)
    lib().oracle_frame_prepare(C.byref(cam), _p(kps), n, None if dp is None else _p(dp), _p(ku),
                               _p(d), _p(ur), _p(gc), _p(b))
    return ku, d, ur, gc, b


def search_by_projection_last(cam, scale_factors, cur, last, th, mono=False, check_ori=True):
    keep = []

    def arr(a, dt):
        a = _c(a, dt)
        keep.append(a)
        return _p(a)

    sf = _c(scale_factors, np.float32)
    mc = MatchCurrent(len(cur["kps_un"]), arr(cur["Tcw"], np.float32), arr(cur["kps_un"], KP_DTYPE),
                      arr(cur["desc"], np.uint8), arr(cur["uright"], np.float32))
    ml = MatchLast(len(last["kps_un"]), arr(last["Tcw"], np.float32), arr(last["kps_un"], KP_DTYPE),
                   arr(last["has_mp"], np.uint8), arr(last["outlier"], np.uint8),
                   arr(last["mp_xyz"], np.float32), arr(last["mp_desc"], np.uint8),
                   arr(last["mp_nobs"], np.int32))
    match = np.zeros(max(1, mc.n), np.int32)
    nm = C.c_int(0)
    lib().oracle_search_by_projection_last(C.byref(cam), _p(sf), len(sf), C.byref(mc), C.byref(ml),
                                           float(th), int(mono), int(check_ori), _p(match),
                                           C.byref(nm))
    return match[:mc.n].copy(), nm.value


def frame_is_in_frustum(cam, log_scale_factor, nlevels, Tcw, mps, view_cos_limit=0.5):
    n = len(mps["xyz"])
    keep = [_c(Tcw, np.float32), _c(mps["xyz"], np.float32), _c(mps["normal"], np.float32),
            _c(mps["min_dist"], np.float32), _c(mps["max_dist"], np.float32)]
    out = dict(in_view=np.zeros(n, np.uint8), proj_x=np.zeros(n, np.float32),
               proj_y=np.zeros(n, np.float32), proj_xr=np.zeros(n, np.float32),
               level=np.zeros(n, np.int32), view_cos=np.zeros(n, np.float32))
    lib().oracle_frame_is_in_frustum(
        C.byref(cam), C.c_float(log_scale_factor), int(nlevels), _p(keep[0]), n, _p(keep[1]),
        _p(keep[2]), _p(keep[3]), _p(keep[4]), C.c_float(view_cos_limit), _p(out["in_view"]),
        _p(out["proj_x"]), _p(out["proj_y"]), _p(out["proj_xr"]), _p(out["level"]),
        _p(out["view_cos"]))
    return out


def search_by_projection_local(cam, scale_factors, cur, track, mp_desc, mp_nobs, cur_nobs, th,
                               nnratio):
    keep = []

    def arr(a, dt):
        a = _c(a, dt)
        keep.append(a)
        return _p(a)

    sf = _c(scale_factors, np.float32)
    n = len(cur["kps_un"])
    mc = MatchCurrent(n, arr(np.eye(4), np.float32), arr(cur["kps_un"], KP_DTYPE),
                      arr(cur["desc"], np.uint8), arr(cur["uright"], np.float32))
    match = np.zeros(max(1, n), np.int32)
    nm = C.c_int(0)
    lib().oracle_search_by_projection_local(
        C.byref(cam), _p(sf), len(sf), C.byref(mc), len(track["in_view"]),
        arr(track["in_view"], np.uint8), arr(track["proj_x"], np.float32),
        arr(track["proj_y"], np.float32), arr(track["proj_xr"], np.float32),
        arr(track["level"], np.int32), arr(track["view_cos"], np.float32), arr(mp_desc, np.uint8),
        arr(mp_nobs, np.int32), None if cur_nobs is None else arr(cur_nobs, np.int32),
        C.c_float(th), C.c_float(nnratio), _p(match), C.byref(nm))
    return match[:n].copy(), nm.value


def search_by_bow(kf_node, kf_valid, kf_desc, kf_angle, f_node, f_desc, f_angle, nnratio=0.7,
                  check_ori=True):
    keep = [_c(kf_node, np.int32), _c(kf_valid, np.uint8), _c(kf_desc, np.uint8),
            _c(kf_angle, np.float32), _c(f_node, np.int32), _c(f_desc, np.uint8),
            _c(f_angle, np.float32)]
    nf = len(keep[4])
    match = np.zeros(max(1, nf), np.int32)
    nm = C.c_int(0)
    lib().oracle_search_by_bow(len(keep[0]), _p(keep[0]), _p(keep[1]), _p(keep[2]), _p(keep[3]),
                               nf, _p(keep[4]), _p(keep[5]), _p(keep[6]), C.c_float(nnratio),
                               int(check_ori), _p(match), C.byref(nm))
    return match[:nf].copy(), nm.value


def stereo_matches(cam, p, left, right, kl, dl, kr, dr):
    """Frame::ComputeStereoMatches on the oracle's own pyramids of the pair."""
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    h, w = left.shape
    lw, lh, _, sc, isc = level_sizes(p, w, h)
    pl = np.concatenate([x.reshape(-1) for x in pyramid(p, left)])
    pr = np.concatenate([x.reshape(-1) for x in pyramid(p, right)])
    kl = _c(kl, KP_DTYPE)
    kr = _c(kr, KP_DTYPE)
    dl = _c(dl, np.uint8)
    dr = _c(dr, np.uint8)
    ur = np.zeros(max(1, len(kl)), np.float32)
    dp = np.zeros(max(1, len(kl)), np.float32)
    lw = _c(lw, np.int32)
    lh = _c(lh, np.int32)
    sc = _c(sc, np.float32)
    isc = _c(isc, np.float32)
    lib().oracle_stereo_matches(C.byref(cam), _p(sc), _p(isc), len(sc), _p(lw), _p(lh), _p(pl),
                                _p(pr), _p(kl), _p(dl), len(kl), _p(kr), _p(dr), len(kr), _p(ur),
                                _p(dp))
    return ur[:len(kl)].copy(), dp[:len(kl)].copy()


def pose_optimization(cam, prob, Tcw, outlier, line_outlier=None, fixed_line_jac=False):
    keep = []

    def arr(a, dt):
        a = _c(a, dt)
        keep.append(a)
        return _p(a)

    n = len(prob["kps_un"])
    nl = len(prob.get("kl_obs", ()))
    isg = _c(prob["inv_sigma2"], np.float32)
    P = PoseProblem(n, arr(prob["kps_un"], KP_DTYPE), arr(prob["uright"], np.float32),
                    arr(prob["has_mp"], np.uint8), arr(prob["mp_xyz"], np.float32), nl,
                    arr(prob.get("kl_obs", np.zeros((0, 4))), np.float32),
                    arr(prob.get("kl_octave", np.zeros(0)), np.int32),
                    arr(prob.get("has_ml", np.zeros(0)), np.uint8),
                    arr(prob.get("ml_xyz", np.zeros((0, 6))), np.float32), _p(isg), len(isg))
    T = _c(Tcw, np.float32).copy()
    out = _c(outlier, np.uint8).copy()
    lout = _c(line_outlier if line_outlier is not None else np.zeros(nl), np.uint8).copy()
    nin = C.c_int(0)
    lib().oracle_pose_optimization_ex(C.byref(cam), C.byref(P), int(bool(fixed_line_jac)), _p(T),
                                      _p(out), _p(lout), C.byref(nin))
    return T, out, lout, nin.value


class VO:
    """CPU oracle of the batched tracker (one stream at a time)."""

    def __init__(self, orb_params, cam, n_streams):
        self.h = lib().oracle_vo_create(C.byref(orb_params), C.byref(cam), n_streams)

    def reset(self, Tcw0=None):
        T = None if Tcw0 is None else _c(Tcw0, np.float32)
        lib().oracle_vo_reset(self.h, None if T is None else _p(T))

    def step(self, stream, gray, depth):
        g = _c(gray, np.uint8)
        d = _c(depth, np.float32)
        T = np.zeros(16, np.float32)
        o = np.zeros(5, np.int32)
        rc = lib().oracle_vo_step(self.h, stream, _p(g), _p(d), _p(T), _p(o))
        assert rc == 0
        return T.reshape(4, 4), dict(nkeypoints=int(o[0]), nmatches=int(o[1]), ninliers=int(o[2]),
                                     nmatches_map=int(o[3]), ok=int(o[4]))

    def __del__(self):
        try:
            lib().oracle_vo_destroy(self.h)
        except Exception:
            pass


# ---------------------------------------------------------------------------
# line features (lsd_oracle.cpp)
# ---------------------------------------------------------------------------
KEYLINE_DTYPE = np.dtype([("angle", "<f4"), ("class_id", "<i4"), ("octave", "<i4"),
                          ("pt_x", "<f4"), ("pt_y", "<f4"), ("response", "<f4"), ("size", "<f4"),
                          ("startPointX", "<f4"), ("startPointY", "<f4"), ("endPointX", "<f4"),
                          ("endPointY", "<f4"), ("sPointInOctaveX", "<f4"),
                          ("sPointInOctaveY", "<f4"), ("ePointInOctaveX", "<f4"),
                          ("ePointInOctaveY", "<f4"), ("lineLength", "<f4"),
                          ("numOfPixels", "<i4")])
assert KEYLINE_DTYPE.itemsize == 68

_setup_track_orb = _setup


def _setup(L):  # noqa: F811
    _setup_track_orb(L)
    vp, i, f = C.c_void_p, C.c_int, C.c_float
    L.oracle_lsd_detect.argtypes = [vp, i, i, vp, i, vp]
    L.oracle_lsd_traffic.argtypes = [vp, i, i, vp]
    L.oracle_lsd_stages.argtypes = [vp, i, i, vp, vp, vp, vp, vp, vp]
    L.oracle_line_extract.argtypes = [vp, i, i, vp, vp, vp, i, vp, vp]
    L.oracle_lsdm.argtypes = [i, C.c_double, C.c_double]
    L.oracle_lsdm.restype = C.c_double
    L.oracle_line_iterator_count.argtypes = [i, i, f, f, f, f]
    L.oracle_introsort_perm.argtypes = [vp, i, vp]


def lsd_detect(img, cap=4096):
    """Raw LSD segments (x1, y1, x2, y2) in detection order."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((cap, 4), np.float32)
    n = C.c_int(0)
    rc = lib().oracle_lsd_detect(_p(img), w, h, _p(out), cap, C.byref(n))
    assert rc == 0, rc
    return out[:n.value].copy()


LSD_TRAFFIC_KEYS = ("sort_cmp", "sort_moves", "seeds", "grow_nb", "grow_add", "grow_expand",
                    "grows", "fit_reads", "fit_writes", "nfa_evals", "nfa_px",
                    # distinct addresses (touched-address bitmap): entries sorted,
                    # longest region list, rectangles validated, distinct pixels
                    # the seed loop reads / marks USED / reads q of, NFA pixels
                    "sort_n", "max_reg", "rects", "u_seed_px", "u_used_px", "u_q_px",
                    "u_nfa_px")


def lsd_traffic(img):
    """Element accesses of the sequential LSD on one image (the pseudo-order
    sort's compares / element writes, the seed loop's seeds, neighbour reads,
    adds, expansions and fit list accesses, the NFA's evaluations and
    rectangle pixels) and the distinct addresses each stage touches: the
    access-volume and unique-bytes inputs of bench.py."""
    img = _c(img, np.uint8)
    h, w = img.shape
    o = np.zeros(len(LSD_TRAFFIC_KEYS), np.int64)
    n = lib().oracle_lsd_traffic(_p(img), w, h, _p(o))
    out = dict(zip(LSD_TRAFFIC_KEYS, (int(x) for x in o)))
    out["segments"] = int(n)
    return out


def lsd_stages(img):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    sw, sh = int(round(w * 0.8)), int(round(h * 0.8))
    scaled = np.zeros((sh, sw), np.uint8)
    ang = np.zeros((sh, sw), np.float64)
    order = np.zeros((sw - 1) * (sh - 1), np.uint32)
    a, b, n = C.c_int(0), C.c_int(0), C.c_int(0)
    lib().oracle_lsd_stages(_p(img), w, h, _p(scaled), _p(ang), _p(order), C.byref(a), C.byref(b),
                            C.byref(n))
    assert (a.value, b.value) == (sw, sh)
    return scaled, ang, order[:n.value]


def line_extract(img, cap=80):
    """LineExtractor::ExtractLineSegment: keylines, 32-byte LBD rows, coefficients."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    kl = np.zeros(cap, KEYLINE_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    coef = np.zeros((cap, 3), np.float64)
    n, nd = C.c_int(0), C.c_int(0)
    rc = lib().oracle_line_extract(_p(img), w, h, _p(kl), _p(desc), _p(coef), cap, C.byref(n),
                                   C.byref(nd))
    assert rc == 0, rc
    k = n.value
    return kl[:k].copy(), desc[:k].copy(), coef[:k].copy(), nd.value


def lsdm(fn, x, y=0.0):
    return lib().oracle_lsdm(fn, float(x), float(y))


def line_iterator_count(w, h, x1, y1, x2, y2):
    return lib().oracle_line_iterator_count(w, h, x1, y1, x2, y2)


def introsort_perm(keys):
    """libstdc++ std::sort permutation of records ordered by key descending."""
    k = np.ascontiguousarray(keys, np.int32)
    perm = np.zeros(len(k), np.int32)
    lib().oracle_introsort_perm(_p(k), len(k), _p(perm))
    return perm


_setup_lines_orb = _setup


def _setup(L):  # noqa: F811
    _setup_lines_orb(L)
    vp, i, ip = C.c_void_p, C.c_int, C.POINTER(C.c_int)
    L.oracle_line_frame_prepare.argtypes = [vp, vp, i, vp, vp, vp, vp, vp, vp]
    L.oracle_line_search_by_projection_last.argtypes = [vp, vp, i, vp, vp, i, vp, vp, vp, vp, vp,
                                                        vp, ip]
    L.oracle_line_search_by_projection_list.argtypes = [vp, vp, i, vp, vp, vp, i, vp, vp, vp, vp,
                                                        ip, ip]
    L.oracle_line_is_in_frustum.argtypes = [vp, i, vp, vp]
    L.oracle_line_search_pairs.argtypes = [vp, vp, i, i, vp, vp, vp, i, vp, vp, vp, vp, vp, vp, vp,
                                           ip, vp, i, ip, vp, ip, ip]
    L.oracle_line_match_bf_knn.argtypes = [i, vp, i, vp, vp, ip]
    L.oracle_stereo_line_depths.argtypes = [vp, vp, vp, i, vp, vp, i, vp, vp]
    L.oracle_lvo_create.argtypes = [vp, vp, i, i]
    L.oracle_lvo_create.restype = vp
    L.oracle_lvo_create_ex.argtypes = [vp, vp, i, i]
    L.oracle_lvo_create_ex.restype = vp
    L.oracle_lvo_destroy.argtypes = [vp]
    L.oracle_lvo_reset.argtypes = [vp, vp]
    L.oracle_lvo_step.argtypes = [vp, i, vp, vp, vp, vp]
    L.oracle_lvo_step_stereo.argtypes = [vp, i, vp, vp, vp, vp]
    L.oracle_lvo_local_stats.argtypes = [vp, i, vp]
    L.oracle_lvo_set_vocabulary.argtypes = [vp, vp]
    L.oracle_lvo_trk.argtypes = [vp, i]


def line_frame_prepare(cam, kl, depth=None):
    kl = _c(kl, KEYLINE_DTYPE)
    n = len(kl)
    ku = np.zeros(n, KEYLINE_DTYPE)
    ds, de, us, ue = (np.zeros(n, np.float32) for _ in range(4))
    dp = None if depth is None else _c(depth, np.float32)
    lib().oracle_line_frame_prepare(C.byref(cam), _p(kl), n, None if dp is None else _p(dp),
                                    _p(ku), _p(ds), _p(de), _p(us), _p(ue))
    return ku, ds, de, us, ue


def line_is_in_frustum(Tcw, ml_xyz6):
    T = _c(Tcw, np.float32)
    X = _c(ml_xyz6, np.float32)
    out = np.zeros(len(X), np.uint8)
    lib().oracle_line_is_in_frustum(_p(T), len(X), _p(X), _p(out))
    return out


def line_search_by_projection_list(cam, Tcw, cur_kl_un, cur_desc, cur_nobs, valid, ml_xyz6,
                                   ml_desc):
    keep = [_c(Tcw, np.float32), _c(cur_kl_un, KEYLINE_DTYPE), _c(cur_desc, np.uint8),
            _c(valid, np.uint8), _c(ml_xyz6, np.float32), _c(ml_desc, np.uint8)]
    cn = None if cur_nobs is None else _c(cur_nobs, np.int32)
    ncur = len(keep[1])
    match = np.zeros(max(1, ncur), np.int32)
    nm, wiped = C.c_int(0), C.c_int(0)
    lib().oracle_line_search_by_projection_list(
        C.byref(cam), _p(keep[0]), ncur, _p(keep[1]), _p(keep[2]), None if cn is None else _p(cn),
        len(keep[3]), _p(keep[3]), _p(keep[4]), _p(keep[5]), _p(match), C.byref(nm),
        C.byref(wiped))
    return match[:ncur].copy(), nm.value, bool(wiped.value)


def line_search_by_projection_last(cam, Tcw, cur_kl_un, cur_desc, last_kl_un, has_ml, outlier,
                                   ml_xyz6, last_desc):
    keep = [_c(Tcw, np.float32), _c(cur_kl_un, KEYLINE_DTYPE), _c(cur_desc, np.uint8),
            _c(last_kl_un, KEYLINE_DTYPE), _c(has_ml, np.uint8), _c(outlier, np.uint8),
            _c(ml_xyz6, np.float32), _c(last_desc, np.uint8)]
    ncur = len(keep[1])
    match = np.zeros(max(1, ncur), np.int32)
    nm = C.c_int(0)
    lib().oracle_line_search_by_projection_last(C.byref(cam), _p(keep[0]), ncur, _p(keep[1]),
                                                _p(keep[2]), len(keep[3]), _p(keep[3]), _p(keep[4]),
                                                _p(keep[5]), _p(keep[6]), _p(keep[7]), _p(match),
                                                C.byref(nm))
    return match[:ncur].copy(), nm.value


def line_search_pairs(cam, Tcw, mode, cur_kl_un, cur_desc, cur_nobs, valid, base_kl, ml_xyz6,
                      ml_desc, ml_nobs):
    """The harness overloads of LineMatcher::SearchByProjection that also
    return new_kls and match_indices (oracle_line_search_pairs; mode 0 =
    LineMatcher.cpp:272-487 last frame, 1 = :954-1170 local map). Returns
    (match, nmatches, wiped, proj_kl, proj_src, pairs (npairs, 2))."""
    keep = [_c(Tcw, np.float32), _c(cur_kl_un, KEYLINE_DTYPE), _c(cur_desc, np.uint8),
            _c(valid, np.uint8), _c(ml_xyz6, np.float32), _c(ml_desc, np.uint8)]
    cn = None if cur_nobs is None else _c(cur_nobs, np.int32)
    mn = None if ml_nobs is None else _c(ml_nobs, np.int32)
    bk = None if base_kl is None else _c(base_kl, KEYLINE_DTYPE)
    ncur, nml = len(keep[1]), len(keep[3])
    match = np.zeros(max(1, ncur), np.int32)
    pk = np.zeros(max(1, nml), KEYLINE_DTYPE)
    ps = np.zeros(max(1, nml), np.int32)
    cap = max(1, ncur * nml)
    pairs = np.zeros((cap, 2), np.int32)
    nm, wiped, npj, npr = C.c_int(0), C.c_int(0), C.c_int(0), C.c_int(0)
    lib().oracle_line_search_pairs(
        C.byref(cam), _p(keep[0]), mode, ncur, _p(keep[1]), _p(keep[2]),
        None if cn is None else _p(cn), nml, _p(keep[3]), None if bk is None else _p(bk),
        _p(keep[4]), _p(keep[5]), None if mn is None else _p(mn), _p(pk), _p(ps), C.byref(npj),
        _p(pairs), cap, C.byref(npr), _p(match), C.byref(nm), C.byref(wiped))
    return (match[:ncur].copy(), nm.value, bool(wiped.value), pk[:npj.value].copy(),
            ps[:npj.value].copy(), pairs[:npr.value].copy())


def line_match_bf_knn(qdesc, tdesc):
    """LineMatcher::SearchByProjection(Frame&, KeyFrame*, vector<MapLine*>&)'s
    knnMatch(k = 2) + 0.75 ratio (LineMatcher.cpp:492-525): (out, n)."""
    q, t = _c(qdesc, np.uint8), _c(tdesc, np.uint8)
    out = np.zeros(max(1, len(t)), np.int32)
    n = C.c_int(0)
    lib().oracle_line_match_bf_knn(len(q), _p(q), len(t), _p(t), _p(out), C.byref(n))
    return out[:len(t)].copy(), n.value


TRACK_LINES, TRACK_STEREO, TRACK_LOCAL_MAP, TRACK_FIXED_LINE_JAC, TRACK_REFKF = 1, 2, 4, 8, 16
TWO_THREADS = 1 << 16


def stereo_line_depths(cam, kl, desc, kr, desc_r):
    """P17 stereo line end-point depths (dstart, dend) of the left lines."""
    kl = np.ascontiguousarray(kl)
    kr = np.ascontiguousarray(kr)
    d = _c(desc, np.uint8)
    dr = _c(desc_r, np.uint8)
    ds = np.zeros(max(1, len(kl)), np.float32)
    de = np.zeros(max(1, len(kl)), np.float32)
    lib().oracle_stereo_line_depths(C.byref(cam), _p(kl), _p(d), len(kl), _p(kr), _p(dr), len(kr),
                                    _p(ds), _p(de))
    return ds[:len(kl)], de[:len(kl)]


class LVO:
    """CPU oracle of the points (+ lines) tracker, one stream at a time.
    flags: extra ORBPL_TRACK_* bits (TRACK_LOCAL_MAP, ...) and TWO_THREADS
    (ORB || LineExtractor on two host threads per frame, Frame.cc:152-155)."""

    def __init__(self, orb_params, cam, n_streams, use_lines=True, flags=0):
        f = (TRACK_LINES if use_lines else 0) | flags
        self.h = lib().oracle_lvo_create_ex(C.byref(orb_params), C.byref(cam), n_streams, f)

    def reset(self, Tcw0=None):
        T = None if Tcw0 is None else _c(Tcw0, np.float32)
        lib().oracle_lvo_reset(self.h, None if T is None else _p(T))

    def step(self, stream, gray, depth):
        g = _c(gray, np.uint8)
        d = _c(depth, np.float32)
        T = np.zeros(16, np.float32)
        o = np.zeros(8, np.int32)
        rc = lib().oracle_lvo_step(self.h, stream, _p(g), _p(d), _p(T), _p(o))
        assert rc == 0
        keys = ("nkeypoints", "nmatches", "ninliers", "nmatches_map", "ok", "nlines",
                "line_matches", "line_nmatches_map")
        return T.reshape(4, 4), dict(zip(keys, (int(x) for x in o)))

    def set_vocabulary(self, voc):
        """KeyFrame::ComputeBoW / TrackReferenceKeyFrame vocabulary (Vocabulary)."""
        self._voc = voc
        lib().oracle_lvo_set_vocabulary(self.h, voc.h if voc is not None else None)

    def trk(self, stream):
        """1 when the stream's last step ran TrackReferenceKeyFrame."""
        return int(lib().oracle_lvo_trk(self.h, stream))

    def local_stats(self, stream):
        """TrackLocalMap counts of the stream's last step: local point matches,
        point inliers, local line matches, line inliers."""
        o = np.zeros(4, np.int32)
        lib().oracle_lvo_local_stats(self.h, stream, _p(o))
        return dict(zip(("local_matches", "local_inliers", "local_line_matches",
                         "local_line_inliers"), (int(x) for x in o)))

    def step_stereo(self, stream, left, right):
        """Stereo Frame + TrackWithMotionModel (th = 7); with lines the defined
        stereo line mode (LineExtractor on both images, P17 line depths)."""
        gl = _c(left, np.uint8)
        gr = _c(right, np.uint8)
        T = np.zeros(16, np.float32)
        o = np.zeros(8, np.int32)
        rc = lib().oracle_lvo_step_stereo(self.h, stream, _p(gl), _p(gr), _p(T), _p(o))
        assert rc == 0
        keys = ("nkeypoints", "nmatches", "ninliers", "nmatches_map", "ok", "nlines",
                "line_matches", "line_nmatches_map")
        return T.reshape(4, 4), dict(zip(keys, (int(x) for x in o)))

    def __del__(self):
        try:
            lib().oracle_lvo_destroy(self.h)
        except Exception:
            pass


# ---- DBoW2 vocabulary (bow_oracle.cpp) ----
def _setup_voc(L):
    vp, i = C.c_void_p, C.c_int
    L.oracle_voc_load_text.argtypes = [C.c_char_p]
    L.oracle_voc_load_text.restype = vp
    L.oracle_voc_destroy.argtypes = [vp]
    L.oracle_voc_info.argtypes = [vp, vp]
    L.oracle_voc_nodes.argtypes = [vp, vp, vp, vp, vp, vp]
    L.oracle_voc_transform.argtypes = [vp, vp, i, i, vp, vp, C.POINTER(C.c_int), vp, vp, vp]
    L.oracle_voc_create.argtypes = [i, i, i, i, i, vp, vp, vp, vp]
    L.oracle_voc_create.restype = vp


class Vocabulary:
    """ORBVocabulary::loadFromTextFile + transform (TemplatedVocabulary.h:1338,
    1127-1262)."""

    def __init__(self, path=None, arrays=None):
        L = lib()
        if not hasattr(L, "_voc_ready"):
            _setup_voc(L)
            L._voc_ready = True
        if path is not None:
            self.h = L.oracle_voc_load_text(str(path).encode())
        else:
            a = arrays
            self._keep = [_c(a["parent"], np.int32), _c(a["leaf"], np.uint8),
                          _c(a["desc"], np.uint8), _c(a["weight"], np.float64)]
            self.h = L.oracle_voc_create(int(a["k"]), int(a["L"]), int(a["scoring"]),
                                         int(a["weighting"]), len(self._keep[0]),
                                         *[_p(x) for x in self._keep])
        if not self.h:
            raise ValueError(f"vocabulary load failed: {path}")
        info = np.zeros(6, np.int32)
        L.oracle_voc_info(self.h, _p(info))
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words = map(int, info)

    def nodes(self):
        n = self.n_nodes
        parent = np.zeros(n, np.int32)
        leaf = np.zeros(n, np.uint8)
        word = np.zeros(n, np.int32)
        weight = np.zeros(n, np.float64)
        desc = np.zeros((n, 32), np.uint8)
        lib().oracle_voc_nodes(self.h, _p(parent), _p(leaf), _p(word), _p(weight), _p(desc))
        return dict(parent=parent, leaf=leaf, word=word, weight=weight, desc=desc)

    def transform(self, desc, levelsup=4):
        """-> (bow_words u32, bow_values f64, feat_node i32 (-1 = stopped),
        feat_word i32, feat_weight f64)"""
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(desc)
        words = np.zeros(max(1, n), np.uint32)
        vals = np.zeros(max(1, n), np.float64)
        node = np.zeros(max(1, n), np.int32)
        fw = np.zeros(max(1, n), np.int32)
        fwt = np.zeros(max(1, n), np.float64)
        bn = C.c_int(0)
        lib().oracle_voc_transform(self.h, _p(desc), n, levelsup, _p(words), _p(vals), C.byref(bn),
                                   _p(node), _p(fw), _p(fwt))
        k = bn.value
        return words[:k].copy(), vals[:k].copy(), node[:n].copy(), fw[:n].copy(), fwt[:n].copy()

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_voc_destroy(self.h)
            self.h = None


# ---- Tracking::Track with the map model (map_oracle.cpp) ----
_setup_before_map = _setup


def _setup(L):  # noqa: F811
    _setup_before_map(L)
    vp, i = C.c_void_p, C.c_int
    L.oracle_map_create.argtypes = [vp, vp, i, i]
    L.oracle_map_create.restype = vp
    L.oracle_map_destroy.argtypes = [vp]
    L.oracle_map_reset.argtypes = [vp, vp]
    L.oracle_map_clear_velocity.argtypes = [vp, i]
    L.oracle_map_step_stereo.argtypes = [vp, i, vp, vp, vp, vp]
    L.oracle_map_set_fps.argtypes = [vp, C.c_float]
    L.oracle_map_stage_times.argtypes = [vp, vp]
    L.oracle_map_set_vocabulary.argtypes = [vp, vp]
    L.oracle_map_step.argtypes = [vp, i, vp, vp, vp, vp]
    L.oracle_map_keyframes.argtypes = [vp, i, vp, vp, i, vp]
    L.oracle_map_points.argtypes = [vp, i, vp, vp, vp, i]
    L.oracle_map_points_geom.argtypes = [vp, i, vp, vp, i]
    L.oracle_map_lines.argtypes = [vp, i, vp, vp, vp, i]


MAP_COUNTS = ("nkeypoints", "nmatches", "ninliers", "nmatches_map", "ok", "nlines",
              "line_matches", "line_nmatches_map", "local_matches", "local_inliers",
              "local_line_matches", "local_line_inliers", "keyframe", "keyframes", "map_points",
              "map_lines", "temporal_points", "trk", "ref_kf", "state", "local_keyframes",
              "local_points", "local_lines", "temporal_lines")


class MapVO:
    """CPU oracle of Tracking::Track with the reference's map model
    (UpdateLastFrame, NeedNewKeyFrame, CreateNewKeyFrame, observation counts,
    covisibility local map; LocalMapping = ProcessNewKeyFrame, pinned P23).
    flags: ORBPL_TRACK_LINES / ORBPL_TRACK_REFKF / ORBPL_TRACK_FIXED_LINE_JAC and
    TWO_THREADS (ORB || LineExtractor on two host threads, Frame.cc:152-155)."""

    def __init__(self, orb_params, cam, n_streams, use_lines=True, flags=0):
        f = (TRACK_LINES if use_lines else 0) | flags
        self.h = lib().oracle_map_create(C.byref(orb_params), C.byref(cam), n_streams, f)
        self._voc = None

    def reset(self, Tcw0=None):
        T = None if Tcw0 is None else _c(Tcw0, np.float32)
        lib().oracle_map_reset(self.h, None if T is None else _p(T))

    def clear_velocity(self, stream):
        lib().oracle_map_clear_velocity(self.h, stream)

    def set_vocabulary(self, voc):
        self._voc = voc
        lib().oracle_map_set_vocabulary(self.h, voc.h if voc is not None else None)

    def step(self, stream, gray, depth):
        g = _c(gray, np.uint8)
        d = _c(depth, np.float32)
        T = np.zeros(16, np.float32)
        o = np.zeros(24, np.int32)
        rc = lib().oracle_map_step(self.h, stream, _p(g), _p(d), _p(T), _p(o))
        assert rc == 0
        return T.reshape(4, 4), dict(zip(MAP_COUNTS, (int(x) for x in o)))

    def step_stereo(self, stream, left, right):
        """Tracking::GrabImageStereo + Track() with the map model on a
        rectified pair (ComputeStereoMatches, P17 line depths)."""
        gl = _c(left, np.uint8)
        gr = _c(right, np.uint8)
        T = np.zeros(16, np.float32)
        o = np.zeros(24, np.int32)
        rc = lib().oracle_map_step_stereo(self.h, stream, _p(gl), _p(gr), _p(T), _p(o))
        assert rc == 0
        return T.reshape(4, 4), dict(zip(MAP_COUNTS, (int(x) for x in o)))

    def set_fps(self, fps):
        """Camera.fps: mMaxFrames (0 -> 30)."""
        lib().oracle_map_set_fps(self.h, C.c_float(fps))

    def stage_times(self):
        """The last step's stage times in ms: ORB on the calling thread, the
        LineExtractor on its own thread (TWO_THREADS) or inline, the calling
        thread's join wait, the whole step."""
        o = np.zeros(4, np.float64)
        lib().oracle_map_stage_times(self.h, _p(o))
        return dict(orb=float(o[0]), lines=float(o[1]), join_wait=float(o[2]), step=float(o[3]))

    def keyframes(self, stream, cap=64):
        par = np.zeros(256, np.int32)
        ord_ = np.zeros((256, cap), np.int32)
        nord = np.zeros(256, np.int32)
        n = lib().oracle_map_keyframes(self.h, stream, _p(par), _p(ord_), cap, _p(nord))
        return par[:n], [ord_[k, :min(nord[k], cap)].copy() for k in range(n)]

    def points(self, stream, cap=1 << 18):
        nobs = np.zeros(cap, np.int32)
        desc = np.zeros((cap, 32), np.uint8)
        xyz = np.zeros((cap, 3), np.float32)
        n = lib().oracle_map_points(self.h, stream, _p(nobs), _p(desc), _p(xyz), cap)
        n = min(n, cap)
        return nobs[:n], desc[:n], xyz[:n]

    def points_geom(self, stream, cap=1 << 18):
        """(normal (n, 3), [min, max] distance (n, 2)) per map point."""
        nrm = np.zeros((cap, 3), np.float32)
        d2 = np.zeros((cap, 2), np.float32)
        n = min(lib().oracle_map_points_geom(self.h, stream, _p(nrm), _p(d2), cap), cap)
        return nrm[:n], d2[:n]

    def lines(self, stream, cap=1 << 16):
        """(nobs, descriptors, end points (n, 6)) per map line."""
        nobs = np.zeros(cap, np.int32)
        desc = np.zeros((cap, 32), np.uint8)
        pos = np.zeros((cap, 6), np.float32)
        n = min(lib().oracle_map_lines(self.h, stream, _p(nobs), _p(desc), _p(pos), cap), cap)
        return nobs[:n], desc[:n], pos[:n]

    def __del__(self):
        try:
            lib().oracle_map_destroy(self.h)
        except Exception:
            pass
