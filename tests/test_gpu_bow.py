"""DBoW2 transform on the GPU (k_bow_words / k_bow_vector) against the
oracle's TemplatedVocabulary::transform: BowVector words and values and the
FeatureVector node of every feature bit-exact, single frame (Frame::
ComputeBoW, levelsup 4) and batched; the weighting / scoring variants; and
SearchByBoW fed with the transform's real node ids."""
import numpy as np
import pytest

from _vocab import tiny_features, tiny_vocabulary_text, training_descriptors, vocabulary

pytestmark = pytest.mark.gpu


def test_tiny_known_answer_gpu(orbpl, tmp_path):
    p = tmp_path / "tiny.txt"
    p.write_text(tiny_vocabulary_text())
    v = orbpl.ORBVocabulary(p)
    words, vals, node = v.transform(tiny_features(), levelsup=1)
    assert words.tolist() == [0, 1, 3] and vals.tolist() == [0.25, 0.25, 0.5]
    assert node.tolist() == [1, 1, -1, 2, 1]
    w0, v0, n0 = v.transform(np.zeros((0, 32), np.uint8))
    assert len(w0) == 0 and len(n0) == 0


@pytest.mark.parametrize("k,L,levelsup,scoring,weighting", [
    (10, 5, 4, 0, 0),    # ORBvoc's kind (L1, TF-IDF) as Frame::ComputeBoW calls it
    (10, 4, 2, 0, 0),
    (8, 4, 1, 1, 1),     # L2 norm, TF
    (10, 4, 2, 5, 2),    # dot product (no normalisation), IDF: addIfNotExist
    (10, 4, 6, 0, 3),    # BINARY; levelsup > L: the root
])
def test_transform_bit_exact(orbpl, oracle, k, L, levelsup, scoring, weighting):
    path, _ = vocabulary(k=k, L=L, seed=3, n_frames=8, scoring=scoring, weighting=weighting)
    g = orbpl.ORBVocabulary(path)
    o = oracle.Vocabulary(path)
    for desc in training_descriptors(3, seed=11):
        gw, gv, gn = g.transform(desc, levelsup=levelsup)
        ow, ov, on, _, _ = o.transform(desc, levelsup=levelsup)
        assert np.array_equal(gw, ow)
        assert np.array_equal(gv.view(np.uint64), ov.view(np.uint64))
        assert np.array_equal(gn, on)
        assert len(gw) > 50


def test_transform_batch_device(orbpl, oracle):
    path, _ = vocabulary(k=10, L=5, seed=3, n_frames=8)
    g = orbpl.ORBVocabulary(path)
    g.upload()
    o = oracle.Vocabulary(path)
    frames = training_descriptors(4, seed=13) + [np.zeros((0, 32), np.uint8)]
    F, P = len(frames), 2048
    desc = np.zeros((F, P, 32), np.uint8)
    n = np.zeros(F, np.int32)
    for f, d in enumerate(frames):
        desc[f, :len(d)] = d
        n[f] = len(d)
    dd = orbpl.DeviceBuffer.from_array(desc)
    dn = orbpl.DeviceBuffer.from_array(n)
    out = dict(pitch=P, feat_node=orbpl.DeviceBuffer(F * P * 4), feat_word=orbpl.DeviceBuffer(F * P * 4),
               feat_weight=orbpl.DeviceBuffer(F * P * 8), bow_words=orbpl.DeviceBuffer(F * P * 4),
               bow_vals=orbpl.DeviceBuffer(F * P * 8), bow_n=orbpl.DeviceBuffer(F * 4),
               err=orbpl.DeviceBuffer(4))
    out["err"].zero()
    g.transform_batch_device(dd.ptr, P, dn.ptr, F, int(n.max()), 4, out)
    orbpl.lib().orbpl_device_synchronize(0)
    node = out["feat_node"].download(np.int32, (F, P))
    words = out["bow_words"].download(np.uint32, (F, P))
    vals = out["bow_vals"].download(np.float64, (F, P))
    bn = out["bow_n"].download(np.int32, F)
    assert out["err"].download(np.int32, 1)[0] == 0
    for f, d in enumerate(frames):
        ow, ov, on, _, _ = o.transform(d, levelsup=4)
        assert bn[f] == len(ow), f
        assert np.array_equal(words[f, :bn[f]], ow)
        assert np.array_equal(vals[f, :bn[f]].view(np.uint64), ov.view(np.uint64))
        assert np.array_equal(node[f, :len(d)], on)


def test_search_by_bow_real_nodes(orbpl, oracle):
    """ORBmatcher(0.7, true).SearchByBoW between two frames of a sequence with
    the FeatureVectors from the transform (TrackReferenceKeyFrame's call,
    Tracking.cc:947-955)."""
    from _scenes import sequence
    path, _ = vocabulary(k=10, L=5, seed=3, n_frames=8)
    g = orbpl.ORBVocabulary(path)
    cfg, traj, frames = sequence(2, 21)
    p = oracle.params()
    (k0, d0, _), (k1, d1, _) = [oracle.extract(p, fr[0]) for fr in frames]
    _, _, n0 = g.transform(d0, levelsup=4)
    _, _, n1 = g.transform(d1, levelsup=4)
    valid = (np.arange(len(d0)) % 5 != 0).astype(np.uint8)
    m = orbpl.ORBmatcher(0.7, True)
    gm, gn = m.SearchByBoW(n0, valid, d0, k0["angle"], n1, d1, k1["angle"])
    om, on = oracle.search_by_bow(n0, valid, d0, k0["angle"], n1, d1, k1["angle"], 0.7, True)
    assert np.array_equal(gm, om) and gn == on
    assert gn > 100


@pytest.mark.parametrize("pipelined", [False, True])
def test_tracker_keyframe_bow(orbpl, oracle, pipelined):
    """orbpl_tracker_set_vocabulary: every step's frame gets KeyFrame::
    ComputeBoW (levelsup 4) on the device, bit-exact with the oracle's
    transform of the oracle's descriptors of the same frame."""
    from _scenes import sequence
    path, _ = vocabulary(k=10, L=5, seed=3, n_frames=8)
    voc = orbpl.ORBVocabulary(path)
    o = oracle.Vocabulary(path)
    S, F = 2, 3
    seqs = [sequence(F, 40 + s) for s in range(S)]
    cfg = seqs[0][0]
    tr = orbpl.Tracker(orbpl.OrbParams(1000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S)
    tr.set_pipelined(pipelined)
    tr.set_vocabulary(voc, 4)
    T0 = np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs])
    tr.reset(T0.reshape(S, 16))
    g = orbpl.DeviceBuffer(F * S * 640 * 480)
    d = orbpl.DeviceBuffer(F * S * 640 * 480 * 4)
    p = oracle.params()
    for f in range(F):
        g.upload(np.stack([sq[2][f][0] for sq in seqs]), offset=f * S * 640 * 480)
        d.upload(np.stack([sq[2][f][1] for sq in seqs]), offset=f * S * 640 * 480 * 4)
        tr.step_device(g.ptr + f * S * 640 * 480, d.ptr + f * S * 640 * 480 * 4)
        for s in range(S):
            gw, gv, gn = tr.bow(s)
            _, desc, _ = oracle.extract(p, seqs[s][2][f][0])
            ow, ov, on, _, _ = o.transform(desc, levelsup=4)
            assert np.array_equal(gw, ow) and np.array_equal(gv.view(np.uint64), ov.view(np.uint64))
            assert np.array_equal(gn, on)
