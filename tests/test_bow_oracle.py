"""DBoW2 vocabulary on the CPU: the product's host loader
(orbv_load_text, no device needed) against the oracle's restatement of
TemplatedVocabulary::loadFromTextFile, and the oracle's transform against a
hand-computed known answer (TemplatedVocabulary.h:1127-1262, BowVector.cpp)."""
import numpy as np
import pytest

from _vocab import tiny_features, tiny_vocabulary_text, vocabulary


def _write(tmp_path, txt, name="v.txt"):
    p = tmp_path / name
    p.write_text(txt)
    return p


def test_tiny_known_answer(oracle, tmp_path):
    v = oracle.Vocabulary(_write(tmp_path, tiny_vocabulary_text()))
    assert (v.k, v.L, v.n_nodes, v.n_words) == (2, 2, 7, 4)
    f = tiny_features()
    # f0, f4 -> leaf 3 (tie 4 / 4 at level 2: the first child), f1 -> 4,
    # f2 -> 5 (stopped), f3 -> 6; BowVector {0: 0.5 + 0.5, 1: 1, 3: 2} / L1 4
    words, vals, node, fw, fwt = v.transform(f, levelsup=1)
    assert words.tolist() == [0, 1, 3]
    assert vals.tolist() == [0.25, 0.25, 0.5]
    assert node.tolist() == [1, 1, -1, 2, 1]     # level L - 1
    assert fw.tolist() == [0, 1, 2, 3, 0]
    assert fwt.tolist() == [0.5, 1.0, 0.0, 2.0, 0.5]
    _, _, node0, _, _ = v.transform(f, levelsup=0)
    assert node0.tolist() == [3, 4, -1, 6, 3]    # leaves
    _, _, node4, _, _ = v.transform(f, levelsup=4)
    assert node4.tolist() == [0, 0, -1, 0, 0]    # L - levelsup <= 0: the root


@pytest.mark.parametrize("trailing", [True, False])
def test_loader_matches_oracle(orbpl, oracle, tmp_path, trailing):
    txt = tiny_vocabulary_text()
    if not trailing:
        txt = txt.rstrip("\n")
    p = _write(tmp_path, txt)
    g = orbpl.ORBVocabulary(p).to_arrays()
    o = oracle.Vocabulary(p).nodes()
    assert len(g["parent"]) == 7        # P19: the empty last line makes no node
    for k in ("parent", "leaf", "desc", "weight"):
        assert np.array_equal(g[k], o[k]), k


def test_loader_rejects_bad_files(orbpl, tmp_path):
    bad = [_write(tmp_path, "30 2  0 0\n", "a.txt"),           # k > 20
           _write(tmp_path, "2 2  0 0\n5 1 " + "0 " * 32 + "1\n", "b.txt"),   # parent after
           _write(tmp_path, "", "c.txt")]
    for p in bad:
        with pytest.raises(orbpl.OrbplError):
            orbpl.ORBVocabulary(p)
    with pytest.raises(orbpl.OrbplError):
        orbpl.ORBVocabulary(tmp_path / "missing.txt")


def test_synthetic_vocabulary_pinned(orbpl, oracle):
    """The seeded synthetic vocabulary (k 10, L 4) is reproducible, both
    loaders read the same tree, and the oracle transform is a normalised
    BowVector whose FeatureVector nodes sit at level L - levelsup."""
    path, sha = vocabulary(k=10, L=4, seed=1, n_frames=6)
    path2, sha2 = vocabulary(k=10, L=4, seed=1, n_frames=6, trailing_newline=False)
    assert sha != sha2 and path != path2
    g = orbpl.ORBVocabulary(path).to_arrays()
    o = oracle.Vocabulary(path)
    on = o.nodes()
    for k in ("parent", "leaf", "desc", "weight"):
        assert np.array_equal(g[k], on[k]), k
    assert o.n_nodes == 11111 and o.n_words == 10000
    assert (on["weight"][on["leaf"] == 1] > 0).sum() > 9000   # nearly every word weighted
    from _vocab import training_descriptors
    desc = training_descriptors(2, seed=9)[1]
    words, vals, node, fw, fwt = o.transform(desc, levelsup=2)
    assert abs(vals.sum() - 1.0) < 1e-12 and np.all(np.diff(words.astype(np.int64)) > 0)
    kept = node >= 0
    assert np.array_equal(kept, fwt > 0)
    assert np.all((node[kept] >= 11) & (node[kept] < 111))   # level-2 node ids (BFS)
