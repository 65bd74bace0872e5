"""CPU tests of the C-ABI boundary: the library loads, exports every symbol
include/orbpl.h declares, and its device-free entry points agree with the
oracle. No GPU calls."""
import re
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def _declared_functions():
    src = (ROOT / "include" / "orbpl.h").read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[\w]+\s*\**\s+(\w+)\s*\(", src, flags=re.M)
    return sorted(set(n for n in names if n not in ("if",)))


def test_library_exports_every_declared_symbol(orbpl):
    lib = orbpl.lib()
    names = _declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_describe_matches_oracle(orbpl, oracle):
    for (w, h, nf) in ((640, 480, 1000), (1241, 376, 2000), (1280, 720, 2000), (320, 240, 500)):
        d = orbpl.describe(nfeatures=nf, width=w, height=h)
        lw, lh, nfl, sc, _ = oracle.level_sizes(oracle.params(nf), w, h)
        assert np.array_equal(d["width"], lw)
        assert np.array_equal(d["height"], lh)
        assert np.array_equal(d["nfeatures"], nfl)
        assert np.array_equal(d["scale"], sc)
        assert d["max_keypoints"] >= nf + 3 * 8


def test_describe_rejects_bad_geometry(orbpl):
    import pytest
    with pytest.raises(orbpl.OrbplError):
        orbpl.describe(width=40, height=30)          # levels below 20 px
    with pytest.raises(orbpl.OrbplError):
        orbpl.describe(nfeatures=0)


def test_descriptor_distance(orbpl):
    rng = np.random.default_rng(0)
    for _ in range(50):
        a = rng.integers(0, 256, 32, dtype=np.uint8)
        b = rng.integers(0, 256, 32, dtype=np.uint8)
        ref = int(np.unpackbits(a ^ b).sum())
        assert orbpl.DescriptorDistance(a, b) == ref
    z = np.zeros(32, np.uint8)
    assert orbpl.DescriptorDistance(z, z) == 0
    assert orbpl.DescriptorDistance(z, np.full(32, 255, np.uint8)) == 256


def test_timing_layout_and_version(orbpl):
    """The timing buffers the mirror allocates match what the library writes
    (orbpl_tracker_stage_ms wrote 11 floats into 10)."""
    T = orbpl.Tracker
    assert T.timing_counts() == (len(T.STAGES), len(T.LINE_STAGES), len(T.LSD_STAGES),
                                 len(T.STEREO_STAGES), len(T.KERNEL_STAGES))
    assert orbpl.lib().orbpl_version().decode() == "orbpl gfx950 r4"


def test_dropin_classes_build_with_the_reference_signatures():
    """The g++-built drop-in library exports the reference's class methods
    (ORBextractor.h:51-85, LineExtractor.h:25-30, ORBmatcher.h, LineMatcher.h,
    Optimizer.h:121,234) and links against liborbpl.so."""
    import subprocess
    pkg = ROOT / "orb_slam2_modification_with-point-and-line-feature_amd"
    subprocess.run(["make", "-s", "-C", str(pkg / "dropin")], check=True)
    syms = subprocess.run(["nm", "-DC", "--defined-only", str(pkg / "liborbpl_dropin.so")],
                          check=True, capture_output=True, text=True).stdout
    for s in ("ORB_SLAM2::ORBextractor::ORBextractor(int, float, int, int, int)",
              "ORB_SLAM2::ORBextractor::operator()(cv::InputArray, cv::InputArray, "
              "std::vector<cv::KeyPoint, std::allocator<cv::KeyPoint> >&, cv::OutputArray)",
              "ORB_SLAM2::LineExtractor::ExtractLineSegment(cv::Mat const&",
              "ORB_SLAM2::ORBmatcher::SearchByProjection(ORB_SLAM2::Frame&, ORB_SLAM2::Frame const&, "
              "float, bool)",
              "ORB_SLAM2::ORBmatcher::DescriptorDistance(cv::Mat const&, cv::Mat const&)",
              "ORB_SLAM2::LineMatcher::SearchByProjection(ORB_SLAM2::Frame&, ORB_SLAM2::Frame const&)",
              "ORB_SLAM2::Optimizer::PoseOptimization(ORB_SLAM2::Frame*)",
              "ORB_SLAM2::Optimizer::PoseOptimizationWithLines(ORB_SLAM2::Frame*)"):
        assert s in syms, s
    ldd = subprocess.run(["ldd", str(pkg / "dropin_driver")], check=True, capture_output=True,
                         text=True).stdout
    assert "liborbpl_dropin.so" in ldd and "liborbpl.so" in ldd and "not found" not in ldd
