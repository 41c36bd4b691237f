"""DBoW2 ORBVocabulary: text loader + transform(features, BowVector, FeatureVector, levelsup)
(Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1259, 1338-1420; Frame::ComputeBoW
src/Frame.cc:462-469 calls it with levelsup = 4).

CPU: the oracle (oracle/voc.cpp) against a literal pure-Python transform on small synthetic
vocabularies for every scoring/weighting pair the text format allows and several levelsup
values -- bit-exact, including the double weights.  GPU: word ids, FeatureVector CSR and the
BowVector values bit-exact against the oracle on single and batched sets, and the transform's
FeatureVector driving SearchByBoW end to end.  ORBvoc.txt is not in the image: the
vocabularies are synthetic (synth.vocabulary), so parity is unpinned against the genuine file.
"""
import math

import numpy as np
import pytest

import oracle
from orb_slam2_commit_amd import synth


# ------------------------------------------------------------ literal restatement (KAT)
def parse_text(text):
    lines = text.split("\n")
    k, L, sc, wt = (int(x) for x in lines[0].split())
    nodes = [dict(parent=-1, children=[], desc=None, weight=0.0, word=-1)]
    nw = 0
    for ln in lines[1:]:
        if not ln.strip():
            break
        t = ln.split()
        pid, leaf = int(t[0]), int(t[1])
        nid = len(nodes)
        nodes.append(dict(parent=pid, children=[], desc=np.array([int(x) for x in t[2:34]], np.uint8),
                          weight=float(t[34]), word=-1))
        nodes[pid]["children"].append(nid)
        if leaf > 0:
            nodes[nid]["word"] = nw
            nw += 1
    return dict(k=k, L=L, scoring=sc, weighting=wt, nodes=nodes)


def hamming(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def literal_transform(V, desc, levelsup):
    nodes = V["nodes"]
    if not nodes[0]["children"]:
        return {}, {}
    bow, fv = {}, {}
    nid_level = V["L"] - levelsup
    for i, f in enumerate(desc):
        nid = 0 if nid_level <= 0 else None
        final, level = 0, 0
        while True:
            level += 1
            ch = nodes[final]["children"]
            final = ch[0]
            best = float(hamming(f, nodes[final]["desc"]))
            for c in ch[1:]:
                d = float(hamming(f, nodes[c]["desc"]))
                if d < best:
                    best, final = d, c
            if level == nid_level:
                nid = final
            if not nodes[final]["children"]:
                break
        if nid_level > level:
            nid = final
        w = nodes[final]["weight"]
        word = nodes[final]["word"]
        if w > 0:
            if V["weighting"] in (0, 1):
                bow[word] = bow[word] + w if word in bow else w
            else:
                bow.setdefault(word, w)
            fv.setdefault(nid, []).append(i)
    must = V["scoring"] != 5
    if V["weighting"] in (0, 1) and bow and not must:
        nd = float(len(bow))
        bow = {k: v / nd for k, v in bow.items()}
    if must:
        norm = 0.0
        if V["scoring"] != 1:
            for k in sorted(bow):
                norm += abs(bow[k])
        else:
            for k in sorted(bow):
                norm += bow[k] * bow[k]
            norm = math.sqrt(norm)
        if norm > 0.0:
            bow = {k: v / norm for k, v in bow.items()}
    return bow, fv


def as_maps(words, values, fv_nodes, fv_off, fv_feat):
    bow = {int(w): float(v) for w, v in zip(words, values)}
    fv = {int(n): [int(x) for x in fv_feat[fv_off[j]:fv_off[j + 1]]] for j, n in enumerate(fv_nodes)}
    return bow, fv


@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 0), (5, 0), (0, 1), (5, 1), (0, 2), (1, 3), (2, 0),
                                               (5, 3)])
@pytest.mark.parametrize("levelsup", [4, 0, 2, 7])
def test_oracle_transform_matches_literal(scoring, weighting, levelsup):
    text, vd, leaf = synth.vocabulary(seed=3 + scoring + 7 * weighting, k=5, L=3, scoring=scoring,
                                      weighting=weighting)
    V = parse_text(text)
    desc = synth.voc_descriptors(11, vd, leaf, n=120)
    o = oracle.Vocabulary(text)
    assert (o.k, o.L, o.scoring, o.weighting) == (5, 3, scoring, weighting)
    bow_o, fv_o = as_maps(*o.transform(desc, levelsup))
    bow_l, fv_l = literal_transform(V, desc, levelsup)
    assert list(bow_o) == sorted(bow_l) and list(fv_o) == sorted(fv_l)
    for k in bow_l:
        assert bow_o[k] == bow_l[k]  # bit-exact doubles
    assert fv_o == fv_l


def test_oracle_loader_rules():
    text, vd, leaf = synth.vocabulary(seed=1, k=4, L=2)
    assert oracle.Vocabulary(text).n_nodes == len(vd)
    # a blank line ends the node list (defined behaviour; see oracle/voc.cpp)
    cut = text.split("\n")
    assert oracle.Vocabulary("\n".join(cut[:6] + [""] + cut[6:])).n_nodes == 6
    for bad in ("21 3 0 0\n", "5 0 0 0\n", "5 3 6 0\n", "5 3 0 4\n"):
        with pytest.raises(ValueError):
            oracle.Vocabulary(bad)


def test_oracle_empty_vocabulary_and_stopped_words():
    o = oracle.Vocabulary("10 6 0 0\n")
    w, v, fn, fo, ff = o.transform(np.zeros((5, 32), np.uint8))
    assert len(w) == 0 and len(fn) == 0
    text, vd, leaf = synth.vocabulary(seed=2, k=4, L=2, p_stop=1.0)  # every word stopped
    w, v, fn, fo, ff = oracle.Vocabulary(text).transform(synth.voc_descriptors(2, vd, leaf, 40))
    assert len(w) == 0 and len(fn) == 0


# ---------------------------------------------------------------- GPU parity
def _same(g, o):
    for a, b in zip(g, o):
        np.testing.assert_array_equal(np.asarray(a).astype(np.float64), np.asarray(b).astype(np.float64))


@pytest.fixture(scope="module")
def orb_voc():
    """ORB-SLAM2's configuration (k = 10, L1 norm, TF-IDF) at L = 5 (L = 6 does not fit a test)."""
    text, vd, leaf = synth.vocabulary(seed=17, k=10, L=5, p_short=0.02)
    return text, vd, leaf


@pytest.mark.gpu
@pytest.mark.parametrize("levelsup", [4, 0, 2, 6])
def test_gpu_transform_bit_exact(gpu, orb_voc, levelsup):
    from orb_slam2_commit_amd import ORBVocabulary
    text, vd, leaf = orb_voc
    o = oracle.Vocabulary(text)
    g = ORBVocabulary()
    assert g.loadFromText(text)
    assert (g.k, g.L, g.n_nodes, g.n_words) == (o.k, o.L, o.n_nodes, o.n_words)
    for seed, n in [(1, 2000), (2, 1), (3, 777), (4, 8192)]:
        desc = synth.voc_descriptors(seed, vd, leaf, n)
        _same(g.transform(desc, levelsup), o.transform(desc, levelsup))
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scoring,weighting", [(1, 0), (5, 1), (0, 2), (5, 3), (2, 0)])
def test_gpu_transform_weightings(gpu, scoring, weighting):
    from orb_slam2_commit_amd import ORBVocabulary
    text, vd, leaf = synth.vocabulary(seed=40 + scoring, k=8, L=3, scoring=scoring, weighting=weighting)
    o = oracle.Vocabulary(text)
    g = ORBVocabulary()
    g.loadFromText(text)
    desc = synth.voc_descriptors(5, vd, leaf, 600)
    _same(g.transform(desc, 2), o.transform(desc, 2))
    g.close()


@pytest.mark.gpu
def test_gpu_transform_batch_sets(gpu, orb_voc):
    """Many frames in one call (ragged, including empty sets) == one call per frame."""
    from orb_slam2_commit_amd import ORBVocabulary
    text, vd, leaf = orb_voc
    o = oracle.Vocabulary(text)
    g = ORBVocabulary()
    g.loadFromText(text)
    sets = [synth.voc_descriptors(100 + i, vd, leaf, n) for i, n in enumerate([2000, 0, 5, 1500, 0, 1999, 64])]
    for got, d in zip(g.transform_sets(sets, 4), sets):
        _same(got, o.transform(d, 4))
    g.close()


@pytest.mark.gpu
def test_gpu_transform_edge_cases(gpu):
    from orb_slam2_commit_amd import ORBVocabulary, OrbxError
    g = ORBVocabulary()
    g.loadFromText("10 6 0 0\n")  # empty vocabulary: empty vectors
    w, v, fn, fo, ff = g.transform(np.zeros((9, 32), np.uint8))
    assert len(w) == 0 and len(fn) == 0
    text, vd, leaf = synth.vocabulary(seed=2, k=4, L=2, p_stop=1.0)  # all words stopped
    g.loadFromText(text)
    w, v, fn, fo, ff = g.transform(synth.voc_descriptors(2, vd, leaf, 40))
    assert len(w) == 0 and len(fn) == 0
    with pytest.raises(OrbxError):
        g.loadFromText("21 3 0 0\n")
    text, vd, leaf = synth.vocabulary(seed=3, k=4, L=2)
    g.loadFromText(text)
    with pytest.raises(OrbxError):  # more rows per set than the LDS sort holds
        g.transform(np.zeros((8193, 32), np.uint8))
    g.close()


@pytest.mark.gpu
def test_gpu_transform_feeds_search_by_bow(gpu, orb_voc):
    """transform's FeatureVector is SearchByBoW's input: KF-F matching on the GPU from GPU
    FeatureVectors equals the oracle chain (oracle transform -> oracle SearchByBoW)."""
    from orb_slam2_commit_amd import ORBmatcher, ORBVocabulary
    text, vd, leaf = orb_voc
    rng = np.random.default_rng(9)
    da = synth.voc_descriptors(31, vd, leaf, 1500)
    db = da.copy()  # the frame re-observes the KF's features with a few flipped bits
    flips = rng.integers(0, 256, (1500, 3))
    for i in range(1500):
        for b in flips[i]:
            db[i, b // 8] ^= np.uint8(1 << (b % 8))
    db = db[rng.permutation(1500)]
    ang_a = rng.uniform(0, 360, 1500).astype(np.float32)
    ang_b = rng.uniform(0, 360, 1500).astype(np.float32)
    valid = (rng.random(1500) < 0.85).astype(np.uint8)
    o = oracle.Vocabulary(text)
    g = ORBVocabulary()
    g.loadFromText(text)

    def side(desc, ang, t, valid=None):
        _, _, fn, fo, ff = t
        return dict(desc=desc, angle=ang, valid=valid, node_id=fn.astype(np.uint32), node_off=fo.astype(np.int32),
                    feat=ff.astype(np.int32))

    ga, gb = g.transform_sets([da, db], 4)
    oa, ob = o.transform(da, 4), o.transform(db, 4)
    _same(ga, oa)
    _same(gb, ob)
    m = ORBmatcher(0.75, True)
    got = m.SearchByBoW(side(da, ang_a, ga, valid), side(db, ang_b, gb))
    ref = oracle.search_by_bow(side(da, ang_a, oa, valid), side(db, ang_b, ob), 0.75, True, kf_kf=False)
    np.testing.assert_array_equal(np.asarray(got[0]), np.asarray(ref[0]))
    assert got[1] == ref[1] and got[1] > 100
    g.close()


@pytest.mark.gpu
def test_gpu_transform_device_queued_while_host_transforms(gpu, orb_voc):
    """One vocabulary shared by two threads (Tracking's Frame::ComputeBoW and LocalMapping's
    KeyFrame::ComputeBoW): a device transform still queued behind other work on its stream must not
    see its scratch overwritten by host transforms issued meanwhile (each call owns its scratch)."""
    import ctypes as C

    import torch
    from orb_slam2_commit_amd import ORBVocabulary, _lib
    from orb_slam2_commit_amd._lib import check, ptr
    text, vd, leaf = orb_voc
    o = oracle.Vocabulary(text)
    g = ORBVocabulary()
    g.loadFromText(text)
    S, cap = 12, 2000
    sets = [synth.voc_descriptors(300 + i, vd, leaf, cap - 37 * i) for i in range(S)]
    host = np.zeros((S, cap, 32), np.uint8)
    for i, d in enumerate(sets):
        host[i, :len(d)] = d
    d_desc = torch.from_numpy(host).to(gpu)
    d_cnt = torch.tensor([len(d) for d in sets], dtype=torch.int32, device=gpu)
    t = lambda n, dt=torch.int32: torch.zeros(n, dtype=dt, device=gpu)  # noqa: E731
    bw, bv, nb = t(S * cap), t(S * cap, torch.float64), t(S)
    fn, fo, ff, nf = t(S * cap), t(S * (cap + 1)), t(S * cap), t(S)
    st = torch.cuda.Stream(gpu)
    with torch.cuda.stream(st):  # keep the stream busy: the transform's kernels stay queued
        a = torch.randn(4096, 4096, device=gpu)
        for _ in range(24):
            a = torch.tanh(a @ a)
    check(_lib.lib().orbx_voc_transform_device(g._h, ptr(d_desc), cap, cap, ptr(d_cnt), 1, S, 4, ptr(bw), ptr(bv),
                                               ptr(nb), ptr(fn), ptr(fo), ptr(ff), ptr(nf),
                                               C.c_void_p(st.cuda_stream)), "orbx_voc_transform_device")
    other = synth.voc_descriptors(999, vd, leaf, 8192)  # larger than the device call: forces scratch growth
    want = o.transform(other, 4)
    for _ in range(3):
        _same(g.transform(other, 4), want)
    st.synchronize()
    bw, bv, nb, fn, fo, ff, nf = (x.cpu().numpy() for x in (bw, bv, nb, fn, fo, ff, nf))
    for s, d in enumerate(sets):
        b, q = int(nb[s]), int(nf[s])
        foff = fo[s * (cap + 1):s * (cap + 1) + q + 1]
        got = (bw[s * cap:s * cap + b], bv[s * cap:s * cap + b], fn[s * cap:s * cap + q], foff,
               ff[s * cap:s * cap + int(foff[-1] if q else 0)])
        _same(got, o.transform(d, 4))
    g.close()
