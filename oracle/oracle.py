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
