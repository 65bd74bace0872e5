"""Seeded synthetic ORB vocabularies for the DBoW2 parity tests and the bench
(the reference's ORBvoc.txt is not in its checkout): trained on the oracle's
ORB descriptors of rendered frames by orbpl.synth.vocabulary_tree, written in
DBoW2's text format. Deterministic: the text's sha256 is pinned in the tests."""
import hashlib
import tempfile
from pathlib import Path

import numpy as np

from _pkg import load_oracle, load_pkg
from _scenes import sequence

_CACHE = {}


def training_descriptors(n_frames=12, seed=7, cam_name="TUM1"):
    O = load_oracle()
    cfg, traj, frames = sequence(n_frames, seed, cam_name)
    p = O.params()
    return [O.extract(p, g)[1] for g, _ in frames]


def vocabulary(k=10, L=5, seed=1, n_frames=12, scoring=0, weighting=0, trailing_newline=True):
    """-> (path, sha256 of the text); cached per process."""
    key = (k, L, seed, n_frames, scoring, weighting, trailing_newline)
    if key in _CACHE:
        return _CACHE[key]
    load_pkg()
    import orbpl.synth as synth
    tree = synth.vocabulary_tree(training_descriptors(n_frames), k=k, L=L, seed=seed)
    txt = synth.vocabulary_text(tree, scoring=scoring, weighting=weighting)
    if not trailing_newline:
        txt = txt.rstrip("\n")
    d = Path(tempfile.mkdtemp(prefix="orbvoc_"))
    path = d / f"voc_k{k}_L{L}_s{seed}_{scoring}{weighting}.txt"
    path.write_text(txt)
    out = (path, hashlib.sha256(txt.encode()).hexdigest())
    _CACHE[key] = out
    return out


def tiny_vocabulary_text():
    """Known-answer vocabulary (k = 2, L = 2): node 1 = zeros, node 2 = ones;
    leaves 3 (byte0 0x0F, w 0.5), 4 (byte0 0xF0, w 1), 5 (ones, w 0: stopped),
    6 (ones but byte0 0x00, w 2)."""
    def row(b0, fill):
        return " ".join([str(b0)] + [str(fill)] * 31)
    lines = ["2 2  0 0",
             f"0 0 {row(0, 0)}  0",
             f"0 0 {row(255, 255)}  0",
             f"1 1 {row(15, 0)}  0.5",
             f"1 1 {row(240, 0)}  1",
             f"2 1 {row(255, 255)}  0",
             f"2 1 {row(0, 255)}  2"]
    return "\n".join(lines) + "\n"


def tiny_features():
    f = np.zeros((5, 32), np.uint8)
    f[1, 0] = 0xF0
    f[2, :] = 0xFF
    f[3, :] = 0xFF
    f[3, 0] = 0
    return f
