"""Regenerate the committed oracle fixtures in tests/golden/.

The reference ships no golden vectors for this path and cannot be built here
(SURVEY.md §8c), so these fixtures pin the CPU oracle's own output on seeded
synthetic frames ("parity unpinned" against the real reference binary). The
inputs are regenerated from the seed by orbpl.synth; the image sha256 is stored
so a drift of the generator is detected rather than silently absorbed.

Usage:  python tests/golden/make_golden.py
"""
import hashlib
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
from _pkg import load_oracle, load_pkg  # noqa: E402

CASES = [
    # name, width, height, seed, orb params (nfeatures, scale, levels, ini, min)
    ("vga_s1", 640, 480, 1, (1000, 1.2, 8, 20, 7)),
    ("vga_s2", 640, 480, 2, (1000, 1.2, 8, 20, 7)),
    ("qvga_s3", 320, 240, 3, (500, 1.2, 6, 20, 7)),
    ("kitti_s4", 1241, 376, 4, (2000, 1.2, 8, 20, 7)),
]


def image_for(name, w, h, seed):
    load_pkg()
    import orbpl.synth as synth
    return synth.textured_image(w, h, seed=seed)


LINE_CASES = [
    # name, width, height, seed: LineExtractor::ExtractLineSegment (LSD + top-80 + LBD)
    ("vga_s1", 640, 480, 1),
    ("kitti_s4", 1241, 376, 4),
]


def main():
    O = load_oracle()
    for name, w, h, seed in LINE_CASES:
        img = image_for(name, w, h, seed)
        lines = O.lsd_detect(img)
        kl, desc, coef, nd = O.line_extract(img)
        np.savez_compressed(
            HERE / f"lines_{name}.npz", sha256=hashlib.sha256(img.tobytes()).hexdigest(),
            width=w, height=h, seed=seed, lsd_lines=lines, keylines=kl.view(np.uint8),
            desc=desc, coef=coef, n_detected=nd)
        print("lines", name, len(lines), len(kl))
    for name, w, h, seed, pp in CASES:
        img = image_for(name, w, h, seed)
        p = O.params(*pp)
        kps, desc, cnt = O.extract(p, img)
        cands = O.candidates(p, img)
        np.savez_compressed(
            HERE / f"orb_{name}.npz", sha256=hashlib.sha256(img.tobytes()).hexdigest(),
            width=w, height=h, seed=seed, params=np.array(pp, np.float64),
            kps=kps, desc=desc, level_counts=cnt,
            cand_counts=np.array([len(c) for c in cands], np.int32))
        print(name, len(kps), cnt.tolist())


if __name__ == "__main__":
    main()
