"""MI355X-native front-end of the ORB-SLAM2 point+line fork — host-side mirror.

Python mirror of the reference's per-frame operator interfaces, each a thin
ctypes layer over the C-ABI in include/orbpl.h (liborbpl.so, built in-tree
from csrc/ for gfx950):

  ORBextractor  — ORB_SLAM2::ORBextractor (include/ORBextractor.h:44-112)

Every call goes to the HIP library; there is no CPU fallback. If liborbpl.so
is missing or no GPU is visible, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
# ORBPL_LIB: an alternative build of the same library (dev A/B runs)
LIB_PATH = Path(os.environ.get("ORBPL_LIB") or (PKG_DIR / "liborbpl.so"))

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

ORBPL_OK = 0
ORBPL_ERR_ARG = -1
ORBPL_ERR_CAPACITY = -2
ORBPL_ERR_HIP = -3
ORBPL_ERR_NODEVICE = -4
ORBPL_ERR_OVERFLOW = -5


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class OrbplError(RuntimeError):
    pass


_lib = None


def lib():
    """Load liborbpl.so (fails loudly: the product has no fallback path)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise OrbplError(f"{LIB_PATH} not built; run __graft_entry__.build() or make -C csrc")
        _lib = C.CDLL(str(LIB_PATH))
        _declare(_lib)
    return _lib


def _declare(L):
    vp, i, ip = C.c_void_p, C.c_int, C.POINTER(C.c_int)
    L.orbpl_last_error.restype = C.c_char_p
    L.orbpl_version.restype = C.c_char_p
    L.orbpl_device_count.argtypes = [ip]
    L.orbx_create.argtypes = [vp, i, i, i, i, C.POINTER(vp)]
    L.orbx_destroy.argtypes = [vp]
    L.orbx_get_scale_info.argtypes = [vp, ip, vp, vp, vp, vp]
    L.orbx_get_level_info.argtypes = [vp, vp, vp, vp]
    L.orbx_max_keypoints.argtypes = [vp]
    L.orbx_describe.argtypes = [vp, i, i, vp, vp, vp, vp, ip]
    L.orbx_extract.argtypes = [vp, vp, i, i, i, vp, vp, i, ip]
    L.orbx_extract_batch_device.argtypes = [vp, vp, i, i, C.c_int64, vp, vp, i, vp]
    L.orbx_get_pyramid.argtypes = [vp, i, i, i, i, vp, i, ip, ip]
    L.orbx_get_candidates.argtypes = [vp, vp, i, vp, ip]
    L.orbx_synchronize.argtypes = [vp]
    L.orbx_last_stage_ms.argtypes = [vp, vp]
    L.orbpl_descriptor_distance.argtypes = [vp, vp]
    L.orbpl_dev_malloc.argtypes = [i, C.c_int64, C.POINTER(vp)]
    L.orbpl_dev_free.argtypes = [i, vp]
    L.orbpl_memcpy_htod.argtypes = [i, vp, vp, C.c_int64]
    L.orbpl_host_alloc.argtypes = [C.c_int64, C.POINTER(vp)]
    L.orbpl_host_free.argtypes = [vp]
    L.orbpl_memcpy_dtoh.argtypes = [i, vp, vp, C.c_int64]
    L.orbpl_memset_d.argtypes = [i, vp, i, C.c_int64]
    L.orbpl_device_synchronize.argtypes = [i]


def check(rc, what=""):
    if rc != ORBPL_OK:
        msg = lib().orbpl_last_error().decode(errors="replace")
        raise OrbplError(f"{what} failed with {rc}: {msg}")
    return rc


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _rows_u8(image):
    """A 2-D u8 image as (array, row pitch in bytes): a view whose rows are
    contiguous (a cv::Mat ROI: step > cols) is passed as is with its pitch,
    anything else is copied contiguous."""
    a = np.asarray(image)
    if a.dtype == np.uint8 and a.ndim == 2 and a.strides[1] == 1 and a.strides[0] >= a.shape[1]:
        return a, int(a.strides[0])
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, (a.shape[1] if a.ndim == 2 else 0)


class DeviceBuffer:
    """Owned device allocation (hipMalloc via the C-ABI)."""

    def __init__(self, nbytes, device=0):
        self.nbytes, self.device = int(nbytes), device
        p = C.c_void_p()
        check(lib().orbpl_dev_malloc(device, self.nbytes, C.byref(p)), "orbpl_dev_malloc")
        self.ptr = p.value

    @classmethod
    def from_array(cls, arr, device=0):
        arr = np.ascontiguousarray(arr)
        b = cls(arr.nbytes, device)
        b.upload(arr)
        return b

    def upload(self, arr, offset=0):
        arr = np.ascontiguousarray(arr)
        assert 0 <= offset and offset + arr.nbytes <= self.nbytes
        check(lib().orbpl_memcpy_htod(self.device, C.c_void_p(self.ptr + offset), _ptr(arr),
                                      arr.nbytes), "orbpl_memcpy_htod")

    def download(self, dtype, shape):
        out = np.empty(shape, dtype)
        assert out.nbytes <= self.nbytes
        check(lib().orbpl_memcpy_dtoh(self.device, _ptr(out), C.c_void_p(self.ptr), out.nbytes),
              "orbpl_memcpy_dtoh")
        return out

    def zero(self):
        check(lib().orbpl_memset_d(self.device, C.c_void_p(self.ptr), 0, self.nbytes),
              "orbpl_memset_d")

    def free(self):
        if self.ptr:
            lib().orbpl_dev_free(self.device, C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HostBuffer:
    """Page-locked host allocation (orbpl_host_alloc) viewed as a numpy array."""

    def __init__(self, shape, dtype):
        self.dtype, self.shape = np.dtype(dtype), tuple(np.atleast_1d(shape))
        nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = C.c_void_p()
        check(lib().orbpl_host_alloc(nbytes, C.byref(p)), "orbpl_host_alloc")
        self.ptr = p.value
        buf = (C.c_uint8 * nbytes).from_address(self.ptr)
        self.array = np.frombuffer(buf, np.uint8, nbytes).view(self.dtype).reshape(self.shape)

    def free(self):
        if self.ptr:
            self.array = None
            lib().orbpl_host_free(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def device_count():
    n = C.c_int(0)
    lib().orbpl_device_count(C.byref(n))
    return n.value


def describe(nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7,
             width=640, height=480):
    """Device-free geometry of an extractor (level sizes, budgets, capacity)."""
    p = OrbParams(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
    lw = np.zeros(nlevels, np.int32)
    lh = np.zeros(nlevels, np.int32)
    nf = np.zeros(nlevels, np.int32)
    sc = np.zeros(nlevels, np.float32)
    mk = C.c_int(0)
    check(lib().orbx_describe(C.byref(p), width, height, _ptr(lw), _ptr(lh), _ptr(nf), _ptr(sc),
                              C.byref(mk)), "orbx_describe")
    return dict(width=lw, height=lh, nfeatures=nf, scale=sc, max_keypoints=mk.value)


class ORBextractor:
    """Drop-in for ORB_SLAM2::ORBextractor (ORBextractor.h:44-112).

    ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) with
    the image geometry fixed at construction (the device buffers and the
    pyramid/cell/resize tables are sized for it). ``extractor(image)`` returns
    ``(keypoints, descriptors)`` exactly like ``operator()(image, mask,
    keypoints, descriptors)``: keypoints as a KP_DTYPE structured array
    (cv::KeyPoint fields), descriptors as an (N, 32) uint8 array.
    """

    def __init__(self, nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7,
                 width=640, height=480, max_batch=1, device=0):
        self._p = OrbParams(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        self.width, self.height, self.max_batch, self.device = width, height, max_batch, device
        h = C.c_void_p()
        check(lib().orbx_create(C.byref(self._p), width, height, max_batch, device, C.byref(h)),
              "orbx_create")
        self._h = h
        self.nlevels = nlevels
        self.scaleFactor = scaleFactor
        n = C.c_int(0)
        self._scale = np.zeros(nlevels, np.float32)
        self._inv_scale = np.zeros(nlevels, np.float32)
        self._sigma2 = np.zeros(nlevels, np.float32)
        self._inv_sigma2 = np.zeros(nlevels, np.float32)
        check(lib().orbx_get_scale_info(h, C.byref(n), _ptr(self._scale), _ptr(self._inv_scale),
                                        _ptr(self._sigma2), _ptr(self._inv_sigma2)),
              "orbx_get_scale_info")
        self.max_keypoints = lib().orbx_max_keypoints(h)

    def close(self):
        if getattr(self, "_h", None):
            lib().orbx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- ORBextractor.h:60-80 getters ---
    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return float(np.float32(self.scaleFactor))

    def GetScaleFactors(self):
        return self._scale.copy()

    def GetInverseScaleFactors(self):
        return self._inv_scale.copy()

    def GetScaleSigmaSquares(self):
        return self._sigma2.copy()

    def GetInverseScaleSigmaSquares(self):
        return self._inv_sigma2.copy()

    def __call__(self, image, mask=None):
        """operator()(image, mask, keypoints, descriptors); mask is ignored as
        in the reference (ORBextractor.h:56)."""
        if image is None or image.size == 0:
            return np.zeros(0, KP_DTYPE), None
        img, stride = _rows_u8(image)
        assert img.ndim == 2, "CV_8UC1 image expected (ORBextractor.cc:1050)"
        h, w = img.shape
        cap = self.max_keypoints
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        check(lib().orbx_extract(self._h, _ptr(img), w, h, stride, _ptr(kps), _ptr(desc), cap,
                                 C.byref(n)), "orbx_extract")
        k = n.value
        return kps[:k].copy(), (desc[:k].copy() if k else None)

    def extract_batch_device(self, d_imgs, batch, stride, frame_pitch, d_kps, d_desc, kp_pitch, d_n):
        """Batched device-resident extraction (pointers are device addresses)."""
        check(lib().orbx_extract_batch_device(self._h, C.c_void_p(d_imgs), batch, stride,
                                              frame_pitch, C.c_void_p(d_kps), C.c_void_p(d_desc),
                                              kp_pitch, C.c_void_p(d_n)),
              "orbx_extract_batch_device")

    def synchronize(self):
        check(lib().orbx_synchronize(self._h), "orbx_synchronize")

    def stage_ms(self):
        ms = np.zeros(5, np.float32)
        check(lib().orbx_last_stage_ms(self._h, _ptr(ms)), "orbx_last_stage_ms")
        return ms

    def pyramid_level(self, level, padded=False, blurred=False, frame=0):
        w, h = C.c_int(0), C.c_int(0)
        check(lib().orbx_get_pyramid(self._h, frame, level, int(padded), int(blurred), None, 0,
                                     C.byref(w), C.byref(h)), "orbx_get_pyramid")
        out = np.zeros((h.value, w.value), np.uint8)
        check(lib().orbx_get_pyramid(self._h, frame, level, int(padded), int(blurred), _ptr(out),
                                     out.size, C.byref(w), C.byref(h)), "orbx_get_pyramid")
        return out

    @property
    def mvImagePyramid(self):
        """Public member of the reference (ORBextractor.h:83): content of each
        level of the last extracted image."""
        return [self.pyramid_level(l) for l in range(self.nlevels)]

    def candidates(self, cap=1 << 21):
        """Pre-octree FAST candidates per level (debug/parity)."""
        xyr = np.zeros((cap, 3), np.float32)
        cnt = np.zeros(self.nlevels, np.int32)
        tot = C.c_int(0)
        check(lib().orbx_get_candidates(self._h, _ptr(xyr), cap, _ptr(cnt), C.byref(tot)),
              "orbx_get_candidates")
        out, off = [], 0
        for c in cnt:
            out.append(xyr[off:off + c].copy())
            off += c
        return out


def DescriptorDistance(a, b):
    """ORBmatcher::DescriptorDistance (ORBmatcher.cc:2083-2103)."""
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().orbpl_descriptor_distance(_ptr(a), _ptr(b))


# ---------------------------------------------------------------------------
# Frame glue / matcher / pose optimiser / tracker (include/orbpl.h)
# ---------------------------------------------------------------------------
class Camera(C.Structure):
    """orbpl_camera: Camera.* settings (Examples/RGB-D/TUM1.yaml)."""
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("k1", C.c_float), ("k2", C.c_float), ("p1", C.c_float), ("p2", C.c_float),
                ("k3", C.c_float), ("bf", C.c_float), ("th_depth", C.c_float),
                ("width", C.c_int32), ("height", C.c_int32)]


class Settings(C.Structure):
    """orbpl_settings: Tracking::Tracking's settings (Tracking.cc:53-147)."""
    _fields_ = [("orb", OrbParams), ("cam", Camera), ("fps", C.c_float),
                ("max_frames", C.c_int32), ("depth_map_factor", C.c_float),
                ("depth_map_factor_setting", C.c_float), ("rgb", C.c_int32)]


SENSOR = {"monocular": 0, "stereo": 1, "rgbd": 2}


def load_settings(path, sensor="rgbd"):
    """The reference's OpenCV FileStorage YAML settings through the native
    reader (orbpl_settings_load, OpenCV 3.4 FileNode semantics): (OrbParams,
    Camera, dict(fps, max_frames, depth_map_factor, rgb))."""
    out = Settings()
    L = lib()
    L.orbpl_settings_load.argtypes = [C.c_char_p, C.c_int, C.c_void_p]
    check(L.orbpl_settings_load(str(path).encode(), SENSOR[sensor], C.byref(out)),
          "orbpl_settings_load")
    return out.orb, out.cam, dict(fps=out.fps, max_frames=out.max_frames,
                                  depth_map_factor=out.depth_map_factor,
                                  depth_map_factor_setting=out.depth_map_factor_setting,
                                  rgb=out.rgb)


def th_depth(cfg):
    """mThDepth = mbf * (float)ThDepth / fx in float arithmetic, as
    Tracking::Tracking computes it (Tracking.cc:136)."""
    return float(np.float32(cfg["bf"]) * np.float32(cfg["thdepth"]) / np.float32(cfg["fx"]))


def make_camera(cfg):
    """Camera from a settings dict (synth.TUM1 etc.); mThDepth = bf*ThDepth/fx
    (Tracking.cc:134-138, th_depth)."""
    return Camera(cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"], cfg["k1"], cfg["k2"], cfg["p1"],
                  cfg["p2"], cfg["k3"], cfg["bf"], th_depth(cfg),
                  cfg["width"], cfg["height"])


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


def _declare_track(L):
    vp, i, ip = C.c_void_p, C.c_int, C.POINTER(C.c_int)
    L.orbpl_frame_prepare.argtypes = [vp, vp, i, vp, vp, vp, vp, vp, vp]
    L.orbm_search_by_projection_last.argtypes = [vp, vp, i, vp, vp, C.c_float, i, i, vp, ip]
    L.orbpl_pose_optimization.argtypes = [vp, vp, vp, vp, vp, ip]
    L.orbpl_pose_optimization_ex.argtypes = [vp, vp, i, vp, vp, vp, ip]
    L.orbpl_tracker_create.argtypes = [vp, vp, i, i, C.POINTER(vp)]
    L.orbpl_tracker_destroy.argtypes = [vp]
    L.orbpl_tracker_reset.argtypes = [vp, vp]
    L.orbpl_tracker_clear_velocity.argtypes = [vp, vp]
    L.orbpl_tracker_set_fps.argtypes = [vp, C.c_float]
    L.orbpl_tracker_step.argtypes = [vp, vp, vp]
    L.orbpl_tracker_synchronize.argtypes = [vp]
    L.orbpl_tracker_set_pipelined.argtypes = [vp, C.c_int]
    L.orbpl_tracker_launch_frames.argtypes = [vp, ip, ip]
    L.orbpl_tracker_get_state.argtypes = [vp, vp, vp, vp, vp, vp]
    L.orbpl_tracker_stage_ms.argtypes = [vp, vp]
    L.orbpl_tracker_kp_capacity.argtypes = [vp]
    L.orbpl_tracker_timings.argtypes = [vp, i, vp, ip]
    L.orbpl_tracker_timings_reset.argtypes = [vp]
    L.orbpl_tracker_timing_counts.argtypes = [vp]
    L.orbpl_tracker_kernel_timings.argtypes = [vp, i, vp, ip]
    L.orbpl_tracker_get_frame.argtypes = [vp, i, vp, vp, vp, vp, ip]
    L.orbpl_tracker_create_ex.argtypes = [vp, vp, i, i, i, C.POINTER(vp)]
    L.orbpl_line_frame_prepare.argtypes = [vp, vp, i, vp, vp, vp, vp, vp, vp]
    L.orbl_frame_is_in_frustum.argtypes = [vp, i, vp, vp]
    L.orbpl_stereo_matches.argtypes = [vp, vp, vp, i, vp, vp, i, vp, vp, i, vp, vp]
    L.orbm_search_by_bow.argtypes = [i, vp, vp, vp, vp, i, vp, vp, vp, C.c_float, i, vp, ip]
    L.orbl_search_by_projection_list.argtypes = [vp, vp, i, vp, vp, vp, i, vp, vp, vp, vp, ip, ip]
    L.orbpl_frame_is_in_frustum.argtypes = [vp, C.c_float, i, vp, i, vp, vp, vp, vp, C.c_float,
                                            vp, vp, vp, vp, vp, vp]
    L.orbm_search_by_projection_local.argtypes = [vp, vp, i, vp, i, vp, vp, vp, vp, vp, vp, vp, vp,
                                                  vp, C.c_float, C.c_float, vp, ip]
    L.orbl_search_by_projection_last.argtypes = [vp, vp, i, vp, vp, i, vp, vp, vp, vp, vp, vp, ip]
    L.orbl_search_by_projection_pairs.argtypes = [vp, vp, i, i, vp, vp, vp, i, vp, vp, vp, vp, vp,
                                                  vp, vp, ip, vp, i, ip, vp, ip, ip]
    L.orbl_match_bf_knn.argtypes = [i, vp, i, vp, vp, ip]
    L.orbpl_tracker_get_status.argtypes = [vp, vp, vp, vp, vp]
    L.orbpl_tracker_get_lines.argtypes = [vp, i, vp, vp, vp, vp, ip]
    L.orbpl_tracker_line_timings.argtypes = [vp, i, vp, ip]
    L.orbpl_tracker_step_stereo.argtypes = [vp, vp, vp]
    L.orbpl_tracker_stereo_timings.argtypes = [vp, i, vp, ip]
    L.orbpl_tracker_lsd_timings.argtypes = [vp, i, vp, ip]
    L.orbpl_tracker_set_history.argtypes = [vp, i]
    L.orbpl_tracker_get_history.argtypes = [vp, i, i, vp, vp, ip]
    L.orbpl_tracker_get_local_stats.argtypes = [vp, vp, vp, vp, vp]
    L.orbpl_tracker_set_vocabulary.argtypes = [vp, vp, i]
    L.orbpl_tracker_step_host.argtypes = [vp, vp, vp, C.c_float]
    L.orbpl_tracker_get_bow.argtypes = [vp, i, vp, vp, ip, vp, ip]
    L.orbpl_tracker_get_trk.argtypes = [vp, vp]
    L.orbpl_tracker_get_map_history.argtypes = [vp, i, i, vp, ip]
    L.orbpl_tracker_get_map_errors.argtypes = [vp, vp]
    L.orbpl_tracker_get_map_keyframes.argtypes = [vp, i, vp, vp, i, vp, ip]
    L.orbpl_tracker_get_map_points.argtypes = [vp, i, i, vp, vp, vp, vp, vp, ip]
    L.orbpl_tracker_get_map_lines.argtypes = [vp, i, i, vp, vp, vp, ip]


_declare_orig = _declare


def _declare(L):  # noqa: F811
    _declare_orig(L)
    _declare_track(L)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def frame_prepare(camera, kps, depth=None):
    """Frame glue of the RGB-D Frame constructor (Frame.cc:135-205) on the GPU.
    Returns (kps_un, depth, uright, grid_cell, bounds)."""
    kps = _c(kps, KP_DTYPE)
    n = len(kps)
    ku = np.zeros(n, KP_DTYPE)
    d = np.zeros(n, np.float32)
    ur = np.zeros(n, np.float32)
    gc = np.zeros(n, np.int32)
    b = np.zeros(4, np.float32)
    dp = None if depth is None else _c(depth, np.float32)
    check(lib().orbpl_frame_prepare(C.byref(camera), _ptr(kps), n,
                                    None if dp is None else _ptr(dp), _ptr(ku), _ptr(d), _ptr(ur),
                                    _ptr(gc), _ptr(b)), "orbpl_frame_prepare")
    return ku, d, ur, gc, b


class ORBmatcher:
    """ORB_SLAM2::ORBmatcher(nnratio, checkOri) — per-frame SearchByProjection."""

    def __init__(self, nnratio=0.6, checkOri=True):
        self.nnratio, self.checkOri = nnratio, checkOri

    def SearchByProjectionLastFrame(self, camera, scale_factors, cur, last, th, bMono=False):
        """SearchByProjection(CurrentFrame, LastFrame, th, bMono)
        (ORBmatcher.cc:1710-1879). ``cur``/``last`` are dicts of arrays (see
        tests). Returns (match, nmatches): match[i] = last-frame index or -1."""
        sf = _c(scale_factors, np.float32)
        keep = []

        def arr(a, dt):
            a = _c(a, dt)
            keep.append(a)
            return _ptr(a)

        mc = MatchCurrent(len(cur["kps_un"]), arr(cur["Tcw"], np.float32),
                          arr(cur["kps_un"], KP_DTYPE), arr(cur["desc"], np.uint8),
                          arr(cur["uright"], np.float32))
        ml = MatchLast(len(last["kps_un"]), arr(last["Tcw"], np.float32),
                       arr(last["kps_un"], KP_DTYPE), arr(last["has_mp"], np.uint8),
                       arr(last["outlier"], np.uint8), arr(last["mp_xyz"], np.float32),
                       arr(last["mp_desc"], np.uint8), arr(last["mp_nobs"], np.int32))
        match = np.zeros(max(1, mc.n), np.int32)
        nm = C.c_int(0)
        check(lib().orbm_search_by_projection_last(C.byref(camera), _ptr(sf), len(sf),
                                                   C.byref(mc), C.byref(ml), float(th),
                                                   int(bMono), int(self.checkOri), _ptr(match),
                                                   C.byref(nm)), "orbm_search_by_projection_last")
        return match[:mc.n].copy(), nm.value

    def SearchByBoW(self, kf_node, kf_valid, kf_desc, kf_angle, f_node, f_desc, f_angle):
        """SearchByBoW(pKF, F) (ORBmatcher.cc:247-410) with per-feature
        vocabulary node ids. Returns (match, nmatches)."""
        keep = [_c(kf_node, np.int32), _c(kf_valid, np.uint8), _c(kf_desc, np.uint8),
                _c(kf_angle, np.float32), _c(f_node, np.int32), _c(f_desc, np.uint8),
                _c(f_angle, np.float32)]
        nf = len(keep[4])
        match = np.zeros(max(1, nf), np.int32)
        nm = C.c_int(0)
        check(lib().orbm_search_by_bow(len(keep[0]), _ptr(keep[0]), _ptr(keep[1]), _ptr(keep[2]),
                                       _ptr(keep[3]), nf, _ptr(keep[4]), _ptr(keep[5]),
                                       _ptr(keep[6]), float(self.nnratio), int(self.checkOri),
                                       _ptr(match), C.byref(nm)), "orbm_search_by_bow")
        return match[:nf].copy(), nm.value

    def SearchByProjectionLocalMap(self, camera, scale_factors, cur, track, mp_desc, mp_nobs,
                                   cur_nobs, th):
        """SearchByProjection(F, vpLocalMapPoints, th) (ORBmatcher.cc:72-183);
        ``track`` = frame_is_in_frustum output. Returns (match, nmatches)."""
        sf = _c(scale_factors, np.float32)
        keep = []

        def arr(a, dt):
            a = _c(a, dt)
            keep.append(a)
            return _ptr(a)

        n = len(cur["kps_un"])
        mc = MatchCurrent(n, arr(np.eye(4), np.float32), arr(cur["kps_un"], KP_DTYPE),
                          arr(cur["desc"], np.uint8), arr(cur["uright"], np.float32))
        nmp = len(track["in_view"])
        match = np.zeros(max(1, n), np.int32)
        nm = C.c_int(0)
        check(lib().orbm_search_by_projection_local(
            C.byref(camera), _ptr(sf), len(sf), C.byref(mc), nmp, arr(track["in_view"], np.uint8),
            arr(track["proj_x"], np.float32), arr(track["proj_y"], np.float32),
            arr(track["proj_xr"], np.float32), arr(track["level"], np.int32),
            arr(track["view_cos"], np.float32), arr(mp_desc, np.uint8), arr(mp_nobs, np.int32),
            None if cur_nobs is None else arr(cur_nobs, np.int32), float(th), float(self.nnratio),
            _ptr(match), C.byref(nm)), "orbm_search_by_projection_local")
        return match[:n].copy(), nm.value


def stereo_matches(camera, left, right, kl, dl, kr, dr, frame=0):
    """Frame::ComputeStereoMatches with the pyramids of two ORBextractor
    objects (left / right) that extracted the pair: (uright, depth)."""
    kl = _c(kl, KP_DTYPE)
    kr = _c(kr, KP_DTYPE)
    dl = _c(dl, np.uint8)
    dr = _c(dr, np.uint8)
    ur = np.zeros(max(1, len(kl)), np.float32)
    dp = np.zeros(max(1, len(kl)), np.float32)
    check(lib().orbpl_stereo_matches(C.byref(camera), left._h, right._h, frame, _ptr(kl), _ptr(dl),
                                     len(kl), _ptr(kr), _ptr(dr), len(kr), _ptr(ur), _ptr(dp)),
          "orbpl_stereo_matches")
    return ur[:len(kl)].copy(), dp[:len(kl)].copy()


def frame_is_in_frustum(camera, scale_factor, nlevels, Tcw, mps, view_cos_limit=0.5):
    """Frame::IsInFrustum(MapPoint*, limit) for the map points in ``mps`` (dict:
    xyz, normal, min_dist, max_dist = the raw mfMinDistance / mfMaxDistance; the
    library applies GetMin/MaxDistanceInvariance's 0.8f / 1.2f to the range test
    and PredictScale's mfMaxDistance / dist, MapPoint.cc:387-431). Returns the
    mTrack* fields as a dict."""
    n = len(mps["xyz"])
    keep = [_c(Tcw, np.float32), _c(mps["xyz"], np.float32), _c(mps["normal"], np.float32),
            _c(mps["min_dist"], np.float32), _c(mps["max_dist"], np.float32)]
    out = dict(in_view=np.zeros(n, np.uint8), proj_x=np.zeros(n, np.float32),
               proj_y=np.zeros(n, np.float32), proj_xr=np.zeros(n, np.float32),
               level=np.zeros(n, np.int32), view_cos=np.zeros(n, np.float32))
    check(lib().orbpl_frame_is_in_frustum(
        C.byref(camera), float(scale_factor), int(nlevels), _ptr(keep[0]), n, _ptr(keep[1]),
        _ptr(keep[2]), _ptr(keep[3]), _ptr(keep[4]), float(view_cos_limit), _ptr(out["in_view"]),
        _ptr(out["proj_x"]), _ptr(out["proj_y"]), _ptr(out["proj_xr"]), _ptr(out["level"]),
        _ptr(out["view_cos"])), "orbpl_frame_is_in_frustum")
    return out


def pose_optimization(camera, prob, Tcw, outlier, line_outlier=None, fixed_line_jac=False):
    """Optimizer::PoseOptimization[WithLines] (Optimizer.cc:375-619, 2132-2486).
    ``prob``: dict of arrays. Returns (Tcw, outlier, line_outlier, n_inliers).
    fixed_line_jac: the analytic line Jacobian (ORBPL_POSE_FIXED_LINE_JAC)
    instead of the reference's as-written one (pinned P7)."""
    keep = []

    def arr(a, dt):
        a = _c(a, dt)
        keep.append(a)
        return _ptr(a)

    n = len(prob["kps_un"])
    nl = len(prob.get("kl_obs", ()))
    isg = _c(prob["inv_sigma2"], np.float32)
    P = PoseProblem(n, arr(prob["kps_un"], KP_DTYPE), arr(prob["uright"], np.float32),
                    arr(prob["has_mp"], np.uint8), arr(prob["mp_xyz"], np.float32), nl,
                    arr(prob.get("kl_obs", np.zeros((0, 4))), np.float32),
                    arr(prob.get("kl_octave", np.zeros(0)), np.int32),
                    arr(prob.get("has_ml", np.zeros(0)), np.uint8),
                    arr(prob.get("ml_xyz", np.zeros((0, 6))), np.float32), _ptr(isg), len(isg))
    T = _c(Tcw, np.float32).copy()
    out = _c(outlier, np.uint8).copy()
    lout = _c(line_outlier if line_outlier is not None else np.zeros(nl), np.uint8).copy()
    nin = C.c_int(0)
    check(lib().orbpl_pose_optimization_ex(C.byref(camera), C.byref(P), int(bool(fixed_line_jac)),
                                           _ptr(T), _ptr(out), _ptr(lout), C.byref(nin)),
          "orbpl_pose_optimization_ex")
    return T, out, lout, nin.value


def line_frame_prepare(camera, kl, depth=None):
    """Frame::UndistortKeyLines + line depths (orbpl_line_frame_prepare):
    (kl_un, depth_start, depth_end, uright_start, uright_end)."""
    kl = np.ascontiguousarray(kl, KEYLINE_DTYPE)
    n = len(kl)
    ku = np.zeros(n, KEYLINE_DTYPE)
    ds, de, us, ue = (np.zeros(n, np.float32) for _ in range(4))
    dp = None if depth is None else np.ascontiguousarray(depth, np.float32)
    check(lib().orbpl_line_frame_prepare(C.byref(camera), _ptr(kl), n,
                                         None if dp is None else _ptr(dp), _ptr(ku), _ptr(ds),
                                         _ptr(de), _ptr(us), _ptr(ue)), "orbpl_line_frame_prepare")
    return ku, ds, de, us, ue


class LineMatcher:
    """LineMatcher(0.9, true) tracking overloads on the GPU."""

    @staticmethod
    def SearchByProjectionLocalMap(camera, Tcw, cur_kl_un, cur_desc, cur_nobs, in_view, ml_xyz6,
                                   ml_desc):
        """SearchByProjection(F, vpLocalMapLines): (match, nmatches, wiped)."""
        return _line_search_list(camera, Tcw, cur_kl_un, cur_desc, cur_nobs, in_view, ml_xyz6,
                                 ml_desc)

    @staticmethod
    def SearchByProjectionRefKF(camera, Tcw, cur_kl_un, cur_desc, cur_nobs, has_ml, ml_xyz6,
                                ml_desc):
        """SearchByProjection(F, RefKF): (match, nmatches, wiped)."""
        return _line_search_list(camera, Tcw, cur_kl_un, cur_desc, cur_nobs, has_ml, ml_xyz6,
                                 ml_desc)

    @staticmethod
    def SearchByProjectionLastFrame(camera, Tcw, cur_kl_un, cur_desc, last_kl_un, has_ml, outlier,
                                    ml_xyz6, last_desc):
        keep = [np.ascontiguousarray(Tcw, np.float32), np.ascontiguousarray(cur_kl_un, KEYLINE_DTYPE),
                np.ascontiguousarray(cur_desc, np.uint8),
                np.ascontiguousarray(last_kl_un, KEYLINE_DTYPE), np.ascontiguousarray(has_ml, np.uint8),
                np.ascontiguousarray(outlier, np.uint8), np.ascontiguousarray(ml_xyz6, np.float32),
                np.ascontiguousarray(last_desc, np.uint8)]
        ncur = len(keep[1])
        match = np.zeros(max(1, ncur), np.int32)
        nm = C.c_int(0)
        check(lib().orbl_search_by_projection_last(
            C.byref(camera), _ptr(keep[0]), ncur, _ptr(keep[1]), _ptr(keep[2]), len(keep[3]),
            _ptr(keep[3]), _ptr(keep[4]), _ptr(keep[5]), _ptr(keep[6]), _ptr(keep[7]), _ptr(match),
            C.byref(nm)), "orbl_search_by_projection_last")
        return match[:ncur].copy(), nm.value


    @staticmethod
    def SearchByProjectionPairs(camera, Tcw, mode, cur_kl_un, cur_desc, cur_nobs, valid, base_kl,
                                ml_xyz6, ml_desc, ml_nobs):
        """The reference's harness overloads (orbl_search_by_projection_pairs;
        mode 0 = (Frame&, const Frame&, new_kls, match_indices), 1 = (Frame&,
        const vector<MapLine*>&, new_kls, match_indices)): (match, nmatches,
        wiped, new_kls, their map-line index, match_indices (n, 2))."""
        keep = [np.ascontiguousarray(Tcw, np.float32), np.ascontiguousarray(cur_kl_un, KEYLINE_DTYPE),
                np.ascontiguousarray(cur_desc, np.uint8), np.ascontiguousarray(valid, np.uint8),
                np.ascontiguousarray(ml_xyz6, np.float32), np.ascontiguousarray(ml_desc, np.uint8)]
        cn = None if cur_nobs is None else np.ascontiguousarray(cur_nobs, np.int32)
        mn = None if ml_nobs is None else np.ascontiguousarray(ml_nobs, np.int32)
        bk = None if base_kl is None else np.ascontiguousarray(base_kl, KEYLINE_DTYPE)
        ncur, nml = len(keep[1]), len(keep[3])
        match = np.zeros(max(1, ncur), np.int32)
        pk = np.zeros(max(1, nml), KEYLINE_DTYPE)
        ps = np.zeros(max(1, nml), np.int32)
        cap = max(1, ncur * nml)
        pairs = np.zeros((cap, 2), np.int32)
        nm, wiped, npj, npr = C.c_int(0), C.c_int(0), C.c_int(0), C.c_int(0)
        check(lib().orbl_search_by_projection_pairs(
            C.byref(camera), _ptr(keep[0]), mode, ncur, _ptr(keep[1]), _ptr(keep[2]),
            None if cn is None else _ptr(cn), nml, _ptr(keep[3]), None if bk is None else _ptr(bk),
            _ptr(keep[4]), _ptr(keep[5]), None if mn is None else _ptr(mn), _ptr(pk), _ptr(ps),
            C.byref(npj), _ptr(pairs), cap, C.byref(npr), _ptr(match), C.byref(nm),
            C.byref(wiped)), "orbl_search_by_projection_pairs")
        return (match[:ncur].copy(), nm.value, bool(wiped.value), pk[:npj.value].copy(),
                ps[:npj.value].copy(), pairs[:npr.value].copy())

    @staticmethod
    def MatchBFKnn(qdesc, tdesc):
        """SearchByProjection(Frame&, KeyFrame*, vector<MapLine*>&)'s knnMatch
        + 0.75 ratio (orbl_match_bf_knn): (out, nmatches)."""
        q = np.ascontiguousarray(qdesc, np.uint8)
        t = np.ascontiguousarray(tdesc, np.uint8)
        out = np.zeros(max(1, len(t)), np.int32)
        n = C.c_int(0)
        check(lib().orbl_match_bf_knn(len(q), _ptr(q), len(t), _ptr(t), _ptr(out), C.byref(n)),
              "orbl_match_bf_knn")
        return out[:len(t)].copy(), n.value


def line_is_in_frustum(Tcw, ml_xyz6):
    """Frame::IsInFrustum(MapLine*) for n map lines (n x 6 world end points)."""
    T = np.ascontiguousarray(Tcw, np.float32)
    X = np.ascontiguousarray(ml_xyz6, np.float32)
    out = np.zeros(len(X), np.uint8)
    check(lib().orbl_frame_is_in_frustum(_ptr(T), len(X), _ptr(X), _ptr(out)),
          "orbl_frame_is_in_frustum")
    return out


def _line_search_list(camera, Tcw, cur_kl_un, cur_desc, cur_nobs, valid, ml_xyz6, ml_desc):
    keep = [np.ascontiguousarray(Tcw, np.float32), np.ascontiguousarray(cur_kl_un, KEYLINE_DTYPE),
            np.ascontiguousarray(cur_desc, np.uint8), np.ascontiguousarray(valid, np.uint8),
            np.ascontiguousarray(ml_xyz6, np.float32), np.ascontiguousarray(ml_desc, np.uint8)]
    cn = None if cur_nobs is None else np.ascontiguousarray(cur_nobs, np.int32)
    ncur = len(keep[1])
    match = np.zeros(max(1, ncur), np.int32)
    nm, wiped = C.c_int(0), C.c_int(0)
    check(lib().orbl_search_by_projection_list(
        C.byref(camera), _ptr(keep[0]), ncur, _ptr(keep[1]), _ptr(keep[2]),
        None if cn is None else _ptr(cn), len(keep[3]), _ptr(keep[3]), _ptr(keep[4]),
        _ptr(keep[5]), _ptr(match), C.byref(nm), C.byref(wiped)), "orbl_search_by_projection_list")
    return match[:ncur].copy(), nm.value, bool(wiped.value)


class Tracker:
    """Batched RGB-D / stereo tracker (orbpl_tracker_*): one
    TrackWithMotionModel step for n_streams independent streams per call.
    lines=True selects the point-and-line variant (ORBPL_TRACK_LINES),
    stereo=True the stereo Frame (ORBPL_TRACK_STEREO); both = the defined
    stereo points+lines mode."""

    TRACK_LINES = 1
    TRACK_STEREO = 2
    TRACK_LOCAL_MAP = 4
    TRACK_FIXED_LINE_JAC = 8
    TRACK_REFKF = 16
    TRACK_MAP = 32

    def __init__(self, orb_params, camera, n_streams, device=0, lines=False, stereo=False,
                 local_map=False, fixed_line_jac=False, refkf=False, map=False):
        h = C.c_void_p()
        self.camera, self.S, self.device, self.use_lines = camera, n_streams, device, bool(lines)
        self.stereo = bool(stereo)
        flags = ((self.TRACK_LINES if lines else 0) | (self.TRACK_STEREO if stereo else 0) |
                 (self.TRACK_LOCAL_MAP if local_map else 0) |
                 (self.TRACK_FIXED_LINE_JAC if fixed_line_jac else 0) |
                 (self.TRACK_REFKF if refkf else 0) | (self.TRACK_MAP if map else 0))
        self.map = bool(map)
        check(lib().orbpl_tracker_create_ex(C.byref(orb_params), C.byref(camera), n_streams, device,
                                            flags, C.byref(h)),
              "orbpl_tracker_create_ex")
        self._h = h
        self.kp_cap = lib().orbpl_tracker_kp_capacity(h)

    def close(self):
        if getattr(self, "_h", None):
            lib().orbpl_tracker_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, Tcw0=None):
        T = None if Tcw0 is None else _c(Tcw0, np.float32)
        check(lib().orbpl_tracker_reset(self._h, None if T is None else _ptr(T)), "reset")

    def clear_velocity(self, mask):
        """mVelocity = cv::Mat() for the streams where mask != 0: their next
        step runs TrackReferenceKeyFrame (orbpl_tracker_clear_velocity)."""
        m = np.ascontiguousarray(np.asarray(mask).astype(np.uint8).reshape(-1))
        if m.size != self.S:
            raise ValueError("clear_velocity: one mask byte per stream")
        check(lib().orbpl_tracker_clear_velocity(self._h, _ptr(m)), "orbpl_tracker_clear_velocity")

    def set_fps(self, fps):
        """Camera.fps of the settings: mMaxFrames (map trackers; 0 -> 30)."""
        check(lib().orbpl_tracker_set_fps(self._h, C.c_float(fps)), "orbpl_tracker_set_fps")

    def step_device(self, d_gray, d_depth):
        check(lib().orbpl_tracker_step(self._h, C.c_void_p(d_gray), C.c_void_p(d_depth)), "step")

    def step_host(self, h_gray, h_depth16, depth_map_factor=5000.0):
        """GrabImageRGBD from host memory: h_gray / h_depth16 = host pointers
        (HostBuffer.ptr) to n_streams u8 frames and u16 depth maps."""
        check(lib().orbpl_tracker_step_host(self._h, C.c_void_p(h_gray), C.c_void_p(h_depth16),
                                            C.c_float(depth_map_factor)), "orbpl_tracker_step_host")

    def step_stereo_device(self, d_left, d_right):
        """Stereo step: device pointers to n_streams left / right frames."""
        check(lib().orbpl_tracker_step_stereo(self._h, C.c_void_p(d_left), C.c_void_p(d_right)),
              "orbpl_tracker_step_stereo")

    def synchronize(self):
        check(lib().orbpl_tracker_synchronize(self._h), "orbpl_tracker_synchronize")

    def set_pipelined(self, on=True):
        """Overlap extraction of step t+1 with tracking of step t (2 streams)."""
        check(lib().orbpl_tracker_set_pipelined(self._h, int(bool(on))), "orbpl_tracker_set_pipelined")

    def state(self):
        S = self.S
        T = np.zeros((S, 4, 4), np.float32)
        nk, nm, ni, nmm = (np.zeros(S, np.int32) for _ in range(4))
        check(lib().orbpl_tracker_get_state(self._h, _ptr(T), _ptr(nk), _ptr(nm), _ptr(ni),
                                            _ptr(nmm)), "orbpl_tracker_get_state")
        return dict(Tcw=T, nkeypoints=nk, nmatches=nm, ninliers=ni, nmatches_map=nmm)

    def status(self):
        """ok, nlines, line_matches, line_nmatches_map per stream (last step)."""
        S = self.S
        ok, nl, lm, lnm = (np.zeros(S, np.int32) for _ in range(4))
        check(lib().orbpl_tracker_get_status(self._h, _ptr(ok), _ptr(nl), _ptr(lm), _ptr(lnm)),
              "orbpl_tracker_get_status")
        return dict(ok=ok, nlines=nl, line_matches=lm, line_nmatches_map=lnm)

    def set_vocabulary(self, voc, levelsup=4):
        """KeyFrame::ComputeBoW of every step's frame with an ORBVocabulary
        (None: off). The tracker keeps a reference so the vocabulary outlives
        its use."""
        check(lib().orbpl_tracker_set_vocabulary(self._h, voc._h if voc is not None else None,
                                                 levelsup), "orbpl_tracker_set_vocabulary")
        self._voc = voc

    def trk(self):
        """Per stream: 1 when the last step ran TrackReferenceKeyFrame."""
        out = np.zeros(self.S, np.int32)
        check(lib().orbpl_tracker_get_trk(self._h, _ptr(out)), "orbpl_tracker_get_trk")
        return out

    def bow(self, stream):
        """The last step's (bow_words, bow_values, feat_node) of one stream."""
        K = self.kp_cap
        w = np.zeros(K, np.uint32)
        v = np.zeros(K, np.float64)
        node = np.zeros(K, np.int32)
        bn, n = C.c_int(0), C.c_int(0)
        check(lib().orbpl_tracker_get_bow(self._h, stream, _ptr(w), _ptr(v), C.byref(bn),
                                          _ptr(node), C.byref(n)), "orbpl_tracker_get_bow")
        return w[:bn.value].copy(), v[:bn.value].copy(), node[:n.value].copy()

    def local_stats(self):
        """TrackLocalMap counts per stream of the last step (local_map=True)."""
        S = self.S
        a, b, c, d = (np.zeros(S, np.int32) for _ in range(4))
        check(lib().orbpl_tracker_get_local_stats(self._h, _ptr(a), _ptr(b), _ptr(c), _ptr(d)),
              "orbpl_tracker_get_local_stats")
        return dict(local_matches=a, local_inliers=b, local_line_matches=c, local_line_inliers=d)

    def lines(self, stream):
        """Undistorted KeyLines, LBD rows, line match, line outlier of one stream."""
        K = 80
        kl = np.zeros(K, KEYLINE_DTYPE)
        d = np.zeros((K, 32), np.uint8)
        m = np.zeros(K, np.int32)
        o = np.zeros(K, np.uint8)
        n = C.c_int(0)
        check(lib().orbpl_tracker_get_lines(self._h, stream, _ptr(kl), _ptr(d), _ptr(m), _ptr(o),
                                            C.byref(n)), "orbpl_tracker_get_lines")
        k = n.value
        return kl[:k], d[:k], m[:k], o[:k]

    LINE_STAGES = ("lsd", "keylines_lbd", "line_match")

    @staticmethod
    def timing_counts():
        """Floats per step of timings / line_timings / lsd_timings /
        stereo_timings as the library writes them (orbpl_tracker_timing_counts)."""
        c = np.zeros(5, np.int32)
        check(lib().orbpl_tracker_timing_counts(_ptr(c)), "orbpl_tracker_timing_counts")
        return tuple(int(x) for x in c)

    def _stage_buf(self, which, names, max_steps):
        k = self.timing_counts()[which]
        if k != len(names):
            raise RuntimeError(f"liborbpl writes {k} timing entries per step, the mirror names "
                               f"{len(names)}: library and package out of step")
        return np.zeros((max_steps, k), np.float32)

    def line_timings(self, max_steps=64):
        """(n_steps, 3) line-stage ms of the last steps (hipEvents in-stream)."""
        ms = self._stage_buf(1, self.LINE_STAGES, max_steps)
        n = C.c_int(0)
        check(lib().orbpl_tracker_line_timings(self._h, max_steps, _ptr(ms), C.byref(n)),
              "orbpl_tracker_line_timings")
        return ms[:n.value]

    LSD_STAGES = ("lsd_prep", "lsd_sort", "lsd_seed", "lsd_validate", "keylines", "lbd",
                  "line_prepare")
    # the kernels each LSD stage event pair brackets
    LSD_KERNELS = {"lsd_prep": "k_lsd_blur+k_lsd_resize+k_lsd_grad",
                   "lsd_sort": "k_lsd_sort+k_lsd_sort_local", "lsd_seed": "k_lsd_spec",
                   "lsd_validate": "k_lsd_validate+k_lsd_compact", "keylines": "k_keylines",
                   "lbd": "k_lsd_blur+k_sobel+k_lbd", "line_prepare": "k_line_prepare"}

    def launch_frames(self):
        """(orb, lsd): frames one extraction / LSD stage launch processes (the
        first half when the tracker splits that batch; lsd 0 without lines)."""
        o, l = C.c_int(0), C.c_int(0)
        check(lib().orbpl_tracker_launch_frames(self._h, C.byref(o), C.byref(l)),
              "orbpl_tracker_launch_frames")
        return o.value, l.value

    def lsd_timings(self, max_steps=64):
        """(n_steps, 7) LSD / LineExtractor kernel ms of the last steps."""
        ms = self._stage_buf(2, self.LSD_STAGES, max_steps)
        n = C.c_int(0)
        check(lib().orbpl_tracker_lsd_timings(self._h, max_steps, _ptr(ms), C.byref(n)),
              "orbpl_tracker_lsd_timings")
        return ms[:n.value]

    def set_history(self, max_steps):
        """Record every stream's pose and counts for the next max_steps steps."""
        check(lib().orbpl_tracker_set_history(self._h, int(max_steps)), "orbpl_tracker_set_history")

    def history(self, stream, max_steps=4096):
        """(Tcw (n,4,4), counts (n,12)) of one stream's recorded steps; counts in
        the oracle's order (nkeypoints, nmatches, ninliers, nmatches_map, ok,
        nlines, line_matches, line_nmatches_map, local_matches, local_inliers,
        local_line_matches, local_line_inliers)."""
        T = np.zeros((max_steps, 4, 4), np.float32)
        cnt = np.zeros((max_steps, 12), np.int32)
        n = C.c_int(0)
        check(lib().orbpl_tracker_get_history(self._h, stream, max_steps, _ptr(T), _ptr(cnt),
                                              C.byref(n)), "orbpl_tracker_get_history")
        return T[:n.value], cnt[:n.value]

    MAP_COUNTS = ("nkeypoints", "nmatches", "ninliers", "nmatches_map", "ok", "nlines",
                  "line_matches", "line_nmatches_map", "local_matches", "local_inliers",
                  "local_line_matches", "local_line_inliers", "keyframe", "keyframes",
                  "map_points", "map_lines", "temporal_points", "trk", "ref_kf", "state",
                  "local_keyframes", "local_points", "local_lines", "temporal_lines")

    def map_history(self, stream, max_steps=4096):
        """(n, 24) counts of one stream's recorded steps (map=True trackers), in
        the order of MAP_COUNTS (the oracle's MapVO.step dictionary)."""
        cnt = np.zeros((max_steps, 24), np.int32)
        n = C.c_int(0)
        check(lib().orbpl_tracker_get_map_history(self._h, stream, max_steps, _ptr(cnt),
                                                  C.byref(n)), "orbpl_tracker_get_map_history")
        return cnt[:n.value]

    def map_errors(self):
        """Per stream: capacity flags since the last reset (1 keyframe table
        full, 2 point / line pool full, 4 local list full); 0 = exact."""
        out = np.zeros(self.S, np.int32)
        check(lib().orbpl_tracker_get_map_errors(self._h, _ptr(out)), "orbpl_tracker_get_map_errors")
        return out

    def map_keyframes(self, stream, cap=64):
        """(parent (n,), [ordered connections per keyframe]) of one stream's map."""
        par = np.zeros(64, np.int32)
        ord_ = np.zeros((64, cap), np.int32)
        nord = np.zeros(64, np.int32)
        n = C.c_int(0)
        check(lib().orbpl_tracker_get_map_keyframes(self._h, stream, _ptr(par), _ptr(ord_), cap,
                                                    _ptr(nord), C.byref(n)),
              "orbpl_tracker_get_map_keyframes")
        k = n.value
        return par[:k].copy(), [ord_[j, :min(nord[j], cap)].copy() for j in range(k)]

    def map_points(self, stream, cap=1 << 17):
        """dict(nobs, desc, xyz, normal, dist) of one stream's map points."""
        nobs = np.zeros(cap, np.int32)
        desc = np.zeros((cap, 32), np.uint8)
        xyz = np.zeros((cap, 3), np.float32)
        nrm = np.zeros((cap, 3), np.float32)
        d2 = np.zeros((cap, 2), np.float32)
        n = C.c_int(0)
        check(lib().orbpl_tracker_get_map_points(self._h, stream, cap, _ptr(nobs), _ptr(desc),
                                                 _ptr(xyz), _ptr(nrm), _ptr(d2), C.byref(n)),
              "orbpl_tracker_get_map_points")
        k = min(n.value, cap)
        return dict(nobs=nobs[:k], desc=desc[:k], xyz=xyz[:k], normal=nrm[:k], dist=d2[:k])

    def map_lines(self, stream, cap=1 << 14):
        """dict(nobs, desc, pos) of one stream's map lines."""
        nobs = np.zeros(cap, np.int32)
        desc = np.zeros((cap, 32), np.uint8)
        pos = np.zeros((cap, 6), np.float32)
        n = C.c_int(0)
        check(lib().orbpl_tracker_get_map_lines(self._h, stream, cap, _ptr(nobs), _ptr(desc),
                                                _ptr(pos), C.byref(n)), "orbpl_tracker_get_map_lines")
        k = min(n.value, cap)
        return dict(nobs=nobs[:k], desc=desc[:k], pos=pos[:k])

    STEREO_STAGES = ("right_extract", "stereo_match", "right_lines", "stereo_lines")

    def stereo_timings(self, max_steps=64):
        """(n_steps, 4) stereo-stage ms of the last steps (hipEvents in-stream);
        the line stages are 0 without lines."""
        ms = self._stage_buf(3, self.STEREO_STAGES, max_steps)
        n = C.c_int(0)
        check(lib().orbpl_tracker_stereo_timings(self._h, max_steps, _ptr(ms), C.byref(n)),
              "orbpl_tracker_stereo_timings")
        return ms[:n.value]

    def stage_ms(self):
        ms = np.zeros(5, np.float32)
        check(lib().orbpl_tracker_stage_ms(self._h, _ptr(ms)), "orbpl_tracker_stage_ms")
        return ms

    STAGES = ("pyramid", "blur", "fast", "octree", "orient_desc", "glue", "match", "pose",
              "finish", "local_map", "bow")

    def timings(self, max_steps=64):
        """(n_steps, 11) per-kernel ms of the last steps (hipEvents in-stream)."""
        ms = self._stage_buf(0, self.STAGES, max_steps)
        n = C.c_int(0)
        check(lib().orbpl_tracker_timings(self._h, max_steps, _ptr(ms), C.byref(n)),
              "orbpl_tracker_timings")
        return ms[:n.value]

    KERNEL_STAGES = ("pose_motion", "pose_refkf", "pose_local", "match_local")

    def kernel_timings(self, max_steps=64):
        """(n_steps, 4) ms of every k_pose launch (motion model, reference
        keyframe, local map) and of k_match_local, each launch alone."""
        ms = self._stage_buf(4, self.KERNEL_STAGES, max_steps)
        n = C.c_int(0)
        check(lib().orbpl_tracker_kernel_timings(self._h, max_steps, _ptr(ms), C.byref(n)),
              "orbpl_tracker_kernel_timings")
        return ms[:n.value]

    def timings_reset(self):
        check(lib().orbpl_tracker_timings_reset(self._h), "orbpl_tracker_timings_reset")

    def frame(self, stream):
        K = self.kp_cap
        ku = np.zeros(K, KP_DTYPE)
        d = np.zeros((K, 32), np.uint8)
        m = np.zeros(K, np.int32)
        o = np.zeros(K, np.uint8)
        n = C.c_int(0)
        check(lib().orbpl_tracker_get_frame(self._h, stream, _ptr(ku), _ptr(d), _ptr(m), _ptr(o),
                                            C.byref(n)), "orbpl_tracker_get_frame")
        k = n.value
        return ku[:k], d[:k], m[:k], o[:k]


# ---------------------------------------------------------------------------
# Line features: LineExtractor::ExtractLineSegment (LineExtractor.cpp:12-74)
# ---------------------------------------------------------------------------
KEYLINE_DTYPE = np.dtype([("angle", "<f4"), ("class_id", "<i4"), ("octave", "<i4"),
                          ("pt_x", "<f4"), ("pt_y", "<f4"), ("response", "<f4"), ("size", "<f4"),
                          ("startPointX", "<f4"), ("startPointY", "<f4"), ("endPointX", "<f4"),
                          ("endPointY", "<f4"), ("sPointInOctaveX", "<f4"),
                          ("sPointInOctaveY", "<f4"), ("ePointInOctaveX", "<f4"),
                          ("ePointInOctaveY", "<f4"), ("lineLength", "<f4"),
                          ("numOfPixels", "<i4")])

_declare_points = _declare


def _declare(L):  # noqa: F811
    _declare_points(L)
    vp, i, ip = C.c_void_p, C.c_int, C.POINTER(C.c_int)
    L.lsdx_create.argtypes = [i, i, i, i, C.POINTER(vp)]
    L.lsdx_destroy.argtypes = [vp]
    L.lsdx_detect.argtypes = [vp, vp, i, i, i, vp, i, ip]
    L.lsdx_detect_batch_device.argtypes = [vp, vp, i, i, C.c_int64]
    L.lsdx_synchronize.argtypes = [vp]
    L.lsdx_get_lines.argtypes = [vp, i, vp, i, ip]
    L.lsdx_get_stages.argtypes = [vp, i, vp, vp, vp, ip, ip, ip]
    L.orbpl_test_introsort.argtypes = [vp, i, vp]
    L.lsdx_debug_profile.argtypes = [vp, vp]
    L.lsdx_set_serial_grow.argtypes = [vp, i]
    L.lsdx_extract.argtypes = [vp, vp, i, i, i, vp, vp, vp, i, ip]
    L.lsdx_extract_batch_device.argtypes = [vp, vp, i, i, C.c_int64]
    L.lsdx_get_keylines.argtypes = [vp, i, vp, vp, vp, i, ip]
    L.lsdx_device_outputs.argtypes = [vp, vp, vp, vp, vp]


class LineSegmentDetector:
    """cv::LineSegmentDetector(LSD_REFINE_ADV) as LSDDetector::detect(img, kl, 1, 1)
    runs it (LineExtractor.cpp:20-21): 0.8 Gaussian sub-sampling, region
    growing, rectangle refinement, NFA validation. detect() returns the
    segments (x1, y1, x2, y2) in detection order."""

    def __init__(self, width, height, max_batch=1, device=0):
        self.W, self.H, self.max_batch, self.device = width, height, max_batch, device
        h = C.c_void_p()
        check(lib().lsdx_create(width, height, max_batch, device, C.byref(h)), "lsdx_create")
        self._h = h

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().lsdx_destroy(self._h)
                self._h = None
        except Exception:
            pass

    def detect(self, img, cap=4096):
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        out = np.zeros((cap, 4), np.float32)
        n = C.c_int(0)
        check(lib().lsdx_detect(self._h, _ptr(img), w, h, w, _ptr(out), cap, C.byref(n)),
              "lsdx_detect")
        return out[:n.value].copy()

    def detect_batch_device(self, d_imgs, batch, stride=None, frame_pitch=None):
        stride = self.W if stride is None else stride
        frame_pitch = self.W * self.H if frame_pitch is None else frame_pitch
        check(lib().lsdx_detect_batch_device(self._h, C.c_void_p(d_imgs), batch, stride,
                                             frame_pitch), "lsdx_detect_batch_device")

    def synchronize(self):
        check(lib().lsdx_synchronize(self._h), "lsdx_synchronize")

    def lines(self, frame, cap=4096):
        out = np.zeros((cap, 4), np.float32)
        n = C.c_int(0)
        check(lib().lsdx_get_lines(self._h, frame, _ptr(out), cap, C.byref(n)), "lsdx_get_lines")
        return out[:n.value].copy()

    def set_serial_grow(self, on=True):
        """Wave-serial seed loop (restatement order) instead of the
        speculative lane-parallel one; identical lines."""
        check(lib().lsdx_set_serial_grow(self._h, int(bool(on))), "lsdx_set_serial_grow")

    def debug_profile(self):
        out = np.zeros(8, np.int64)
        check(lib().lsdx_debug_profile(self._h, _ptr(out)), "lsdx_debug_profile")
        keys = ("grow_cyc", "rounds", "spec_regions", "total_cyc", "fit_cyc", "validate_commit_cyc",
                "max_steps", "candidates")
        d = dict(zip(keys, out.tolist()))
        d["coop_regions"] = d["max_steps"] >> 40
        d["max_steps"] &= (1 << 40) - 1
        return d

    def stages(self, frame=0):
        sw, sh = int(round(self.W * 0.8)), int(round(self.H * 0.8))
        scaled = np.zeros((sh, sw), np.uint8)
        deg = np.zeros((sh, sw), np.float32)
        order = np.zeros((sw - 1) * (sh - 1), np.uint32)
        a, b, n = C.c_int(0), C.c_int(0), C.c_int(0)
        check(lib().lsdx_get_stages(self._h, frame, _ptr(scaled), _ptr(deg), _ptr(order),
                                    C.byref(a), C.byref(b), C.byref(n)), "lsdx_get_stages")
        return scaled, deg, order[:n.value]


def test_introsort(keys):
    """Device replica of std::sort(records, key greater): record order."""
    k = np.ascontiguousarray(keys, np.int32)
    perm = np.zeros(len(k), np.int32)
    check(lib().orbpl_test_introsort(_ptr(k), len(k), _ptr(perm)), "orbpl_test_introsort")
    return perm


class LineExtractor(LineSegmentDetector):
    """ORB_SLAM2::LineExtractor (include/LineExtractor.h:21-56):
    ExtractLineSegment(img) -> (key_lines, line_descriptor, keyline_coefficients)
    with scale = 1, num_octaves = 1 as Frame::ExtractLine calls it (Frame.cc:326-328)."""

    def ExtractLineSegment(self, img):
        img, stride = _rows_u8(img)
        h, w = img.shape
        kl = np.zeros(80, KEYLINE_DTYPE)
        desc = np.zeros((80, 32), np.uint8)
        coef = np.zeros((80, 3), np.float64)
        n = C.c_int(0)
        check(lib().lsdx_extract(self._h, _ptr(img), w, h, stride, _ptr(kl), _ptr(desc), _ptr(coef),
                                 80, C.byref(n)), "lsdx_extract")
        k = n.value
        return kl[:k].copy(), desc[:k].copy(), coef[:k].copy()

    def extract_batch_device(self, d_imgs, batch, stride=None, frame_pitch=None):
        stride = self.W if stride is None else stride
        frame_pitch = self.W * self.H if frame_pitch is None else frame_pitch
        check(lib().lsdx_extract_batch_device(self._h, C.c_void_p(d_imgs), batch, stride,
                                              frame_pitch), "lsdx_extract_batch_device")

    def keylines(self, frame):
        kl = np.zeros(80, KEYLINE_DTYPE)
        desc = np.zeros((80, 32), np.uint8)
        coef = np.zeros((80, 3), np.float64)
        n = C.c_int(0)
        check(lib().lsdx_get_keylines(self._h, frame, _ptr(kl), _ptr(desc), _ptr(coef), 80,
                                      C.byref(n)), "lsdx_get_keylines")
        k = n.value
        return kl[:k].copy(), desc[:k].copy(), coef[:k].copy()


# ---------------------------------------------------------------------------
# DBoW2 ORB vocabulary (ORBVocabulary, Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h)
# ---------------------------------------------------------------------------
def _declare_voc(L):
    vp, i, ip = C.c_void_p, C.c_int, C.POINTER(C.c_int)
    L.orbv_load_text.argtypes = [C.c_char_p, C.POINTER(vp)]
    L.orbv_create.argtypes = [i, i, i, i, i, vp, vp, vp, vp, C.POINTER(vp)]
    L.orbv_destroy.argtypes = [vp]
    L.orbv_info.argtypes = [vp, vp]
    L.orbv_export.argtypes = [vp, vp, vp, vp, vp]
    L.orbv_upload.argtypes = [vp, i]
    L.orbv_transform.argtypes = [vp, i, vp, i, i, vp, vp, ip, vp]
    L.orbv_transform_batch_device.argtypes = [vp, vp, C.c_int64, vp, i, i, i, vp, vp, vp, vp, vp,
                                              vp, C.c_int64, vp, vp]


_declare_prev_voc = _declare


def _declare(L):  # noqa: F811
    _declare_prev_voc(L)
    _declare_voc(L)


class ORBVocabulary:
    """TemplatedVocabulary<FORB::TDescriptor, FORB>: loadFromTextFile (host),
    transform on the GPU. Construct with `path` (the reference's text format)
    or `arrays` (dict from to_arrays(): parent, leaf, desc, weight, k, L,
    scoring, weighting) - e.g. a rank's copy of rank 0's broadcast."""

    def __init__(self, path=None, arrays=None, device=0):
        h = C.c_void_p()
        if path is not None:
            check(lib().orbv_load_text(str(path).encode(), C.byref(h)), "orbv_load_text")
        else:
            a = arrays
            par = _c(a["parent"], np.int32)
            leaf = _c(a["leaf"], np.uint8)
            desc = _c(a["desc"], np.uint8)
            wt = _c(a["weight"], np.float64)
            check(lib().orbv_create(int(a["k"]), int(a["L"]), int(a["scoring"]),
                                    int(a["weighting"]), len(par), _ptr(par), _ptr(leaf),
                                    _ptr(desc), _ptr(wt), C.byref(h)), "orbv_create")
        self._h = h
        self.device = device
        info = np.zeros(6, np.int32)
        check(lib().orbv_info(self._h, _ptr(info)), "orbv_info")
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words = map(int, info)

    @classmethod
    def loadFromTextFile(cls, path, device=0):
        return cls(path=path, device=device)

    def to_arrays(self):
        n = self.n_nodes
        a = dict(parent=np.zeros(n, np.int32), leaf=np.zeros(n, np.uint8),
                 desc=np.zeros((n, 32), np.uint8), weight=np.zeros(n, np.float64))
        check(lib().orbv_export(self._h, _ptr(a["parent"]), _ptr(a["leaf"]), _ptr(a["desc"]),
                                _ptr(a["weight"])), "orbv_export")
        a.update(k=self.k, L=self.L, scoring=self.scoring, weighting=self.weighting)
        return a

    def upload(self):
        check(lib().orbv_upload(self._h, self.device), "orbv_upload")

    def transform(self, desc, levelsup=4):
        """-> (bow_words u32, bow_values f64, feat_node i32 per feature, -1 = stopped)"""
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(desc)
        words = np.zeros(max(1, n), np.uint32)
        vals = np.zeros(max(1, n), np.float64)
        node = np.zeros(max(1, n), np.int32)
        bn = C.c_int(0)
        check(lib().orbv_transform(self._h, self.device, _ptr(desc), n, levelsup, _ptr(words),
                                   _ptr(vals), C.byref(bn), _ptr(node)), "orbv_transform")
        k = bn.value
        return words[:k].copy(), vals[:k].copy(), node[:n].copy()

    def transform_batch_device(self, d_desc, desc_pitch, d_n, nframes, max_n, levelsup, out,
                               stream=None):
        """out: dict of DeviceBuffers feat_node, feat_word, feat_weight,
        bow_words, bow_vals, bow_n, err (pitch out['pitch'])."""
        check(lib().orbv_transform_batch_device(
            self._h, C.c_void_p(d_desc), desc_pitch, C.c_void_p(d_n), nframes, max_n, levelsup,
            C.c_void_p(out["feat_node"].ptr), C.c_void_p(out["feat_word"].ptr),
            C.c_void_p(out["feat_weight"].ptr), C.c_void_p(out["bow_words"].ptr),
            C.c_void_p(out["bow_vals"].ptr), C.c_void_p(out["bow_n"].ptr), out["pitch"],
            C.c_void_p(out["err"].ptr), None if stream is None else C.c_void_p(stream)),
            "orbv_transform_batch_device")

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orbv_destroy(self._h)
            self._h = None
