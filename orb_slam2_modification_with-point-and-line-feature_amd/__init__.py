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
LIB_PATH = PKG_DIR / "liborbpl.so"

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

    def upload(self, arr):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        check(lib().orbpl_memcpy_htod(self.device, C.c_void_p(self.ptr), _ptr(arr), arr.nbytes),
              "orbpl_memcpy_htod")

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
        img = np.ascontiguousarray(image, dtype=np.uint8)
        assert img.ndim == 2, "CV_8UC1 image expected (ORBextractor.cc:1050)"
        h, w = img.shape
        cap = self.max_keypoints
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        check(lib().orbx_extract(self._h, _ptr(img), w, h, w, _ptr(kps), _ptr(desc), cap,
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
