"""Boundary behaviour of the C-ABI on the GPU: cv::Mat ROI inputs (row pitch
> width) give the same results as contiguous frames, caller buffers that are
too small report ORBPL_ERR_CAPACITY with the needed count, bad geometry and
over-capacity configurations are rejected with ORBPL_ERR_ARG."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _roi(synth, seed=4):
    big = synth.textured_image(760, 600, seed=seed)
    return big, big[50:530, 40:680]          # 480 x 640 view, row pitch 760


def test_orb_roi_stride(orbpl, oracle, synth):
    big, roi = _roi(synth)
    assert roi.strides[0] == 760 and not roi.flags["C_CONTIGUOUS"]
    ex = orbpl.ORBextractor(1000, 1.2, 8, 20, 7, width=640, height=480)
    kr, dr = ex(roi)
    kc, dc = ex(np.ascontiguousarray(roi))
    assert kr.tobytes() == kc.tobytes() and np.array_equal(dr, dc)
    ok, od, _ = oracle.extract(oracle.params(), np.ascontiguousarray(roi))
    assert np.array_equal(dr, od) and len(kr) == len(ok)


def test_lsd_roi_stride(orbpl, oracle, synth):
    big, roi = _roi(synth, seed=6)
    lx = orbpl.LineExtractor(640, 480)
    a = lx.ExtractLineSegment(roi)
    b = lx.ExtractLineSegment(np.ascontiguousarray(roi))
    assert a[0].tobytes() == b[0].tobytes() and np.array_equal(a[1], b[1])
    okl, od, oc, _ = oracle.line_extract(np.ascontiguousarray(roi))
    assert a[0].tobytes() == okl.tobytes() and np.array_equal(a[1], od)


def test_orb_capacity_and_arguments(orbpl, synth):
    img = synth.textured_image(640, 480, seed=3)
    ex = orbpl.ORBextractor(1000, 1.2, 8, 20, 7, width=640, height=480)
    kps, _ = ex(img)
    L = orbpl.lib()
    n = C.c_int(0)
    small = np.zeros(10, orbpl.KP_DTYPE)
    d = np.zeros((10, 32), np.uint8)
    rc = L.orbx_extract(ex._h, orbpl._ptr(img), 640, 480, 640, orbpl._ptr(small), orbpl._ptr(d),
                        10, C.byref(n))
    assert rc == orbpl.ORBPL_ERR_CAPACITY and n.value == len(kps)
    rc = L.orbx_extract(ex._h, orbpl._ptr(img), 640, 480, 600, orbpl._ptr(small), orbpl._ptr(d),
                        10, C.byref(n))
    assert rc == orbpl.ORBPL_ERR_ARG                  # stride < width
    wrong = np.zeros((400, 600), np.uint8)
    with pytest.raises(orbpl.OrbplError):
        ex(wrong)                                     # not the size given at construction
    # an empty image returns no keypoints (ORBextractor.cc:1049: _image.empty())
    k0, d0 = ex(np.zeros((0, 0), np.uint8))
    assert len(k0) == 0 and d0 is None


def test_tracker_rejects_over_capacity(orbpl, synth):
    cam = orbpl.make_camera(synth.TUM1)
    with pytest.raises(orbpl.OrbplError, match="2048"):
        orbpl.Tracker(orbpl.OrbParams(4000, 1.2, 8, 20, 7), cam, 1)
    tr = orbpl.Tracker(orbpl.OrbParams(1000, 1.2, 8, 20, 7), cam, 1, refkf=True)
    g = orbpl.DeviceBuffer(640 * 480)
    d = orbpl.DeviceBuffer(640 * 480 * 4)
    with pytest.raises(orbpl.OrbplError, match="vocabulary"):
        tr.step_device(g.ptr, d.ptr)                  # ORBPL_TRACK_REFKF without a vocabulary
