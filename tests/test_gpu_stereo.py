"""GPU parity of Frame::ComputeStereoMatches and ORBmatcher::DescriptorDistance."""
import numpy as np
import pytest

import oracle
from orb_slam2_commit_amd import ORBextractor, ORBmatcher, compute_stereo_matches, synth

pytestmark = pytest.mark.gpu

KITTI_BF, KITTI_FX = 386.1448, 718.856
EUROC_BF, EUROC_FX = 47.9064, 435.2047


@pytest.mark.parametrize("seed,w,h,nf,bf,fx", [(0, 1241, 376, 2000, KITTI_BF, KITTI_FX),
                                               (7, 1241, 376, 2000, KITTI_BF, KITTI_FX),
                                               (2, 752, 480, 1200, EUROC_BF, EUROC_FX)])
def test_stereo_bitexact(gpu, seed, w, h, nf, bf, fx):
    L, R = synth.stereo_pair(seed, w, h)
    exL, exR = ORBextractor(nf, 1.2, 8, 20, 7), ORBextractor(nf, 1.2, 8, 20, 7)
    kL, dL = exL(L)
    kR, dR = exR(R)
    uR, dep = compute_stereo_matches(exL, exR, kL, dL, kR, dR, bf, bf / fx)
    p = oracle.params(nf, 1.2, 8, 20, 7)
    oL, oR = oracle.extract(p, L), oracle.extract(p, R)
    ouR, odep = oracle.stereo_match(p, oL, oR, bf, bf / fx)
    assert (ouR >= 0).sum() > 50
    assert np.array_equal(uR.view(np.uint32), ouR.view(np.uint32))
    assert np.array_equal(dep.view(np.uint32), odep.view(np.uint32))


@pytest.mark.parametrize("seed,w,h,nf,bf,fx,pad", [(3, 1241, 376, 2000, KITTI_BF, KITTI_FX, 0),
                                                   (4, 752, 480, 1200, EUROC_BF, EUROC_FX, 13)])
def test_frame_stereo_bitexact(gpu, seed, w, h, nf, bf, fx, pad):
    """orbx_frame_stereo (Frame's stereo constructor, src/Frame.cc:62-123, in one call: both images as a
    batch of two, the matcher behind them, one copy back): keypoints, descriptors, uRight and depth bit
    for bit the oracle's, with row-padded host images (pad bytes per row); afterwards the handle's
    pyramid_level(l, image 0 / 1) is the left / right pyramid, and orbx_stereo_match refuses the handle
    (its last call is no single orbx_extract any more)."""
    from orb_slam2_commit_amd import frame_stereo
    from orb_slam2_commit_amd._lib import ORBX_ERR_STATE, OrbxError
    L, R = synth.stereo_pair(seed, w, h)
    if pad:
        Lp, Rp = np.zeros((h, w + pad), np.uint8), np.full((h, w + pad), 77, np.uint8)
        Lp[:, :w], Rp[:, :w] = L, R
        L, R = Lp[:, :w], Rp[:, :w]  # strided views
    ex = ORBextractor(nf, 1.2, 8, 20, 7)
    kL, dL, kR, dR, uR, dep = frame_stereo(ex, L, R, bf, bf / fx)
    p = oracle.params(nf, 1.2, 8, 20, 7)
    oL, oR = oracle.extract(p, np.ascontiguousarray(L)), oracle.extract(p, np.ascontiguousarray(R))
    ouR, odep = oracle.stereo_match(p, oL, oR, bf, bf / fx)
    assert np.array_equal(kL.view(np.uint8), oL.keypoints.view(np.uint8))
    assert np.array_equal(dL, oL.descriptors)
    assert np.array_equal(kR.view(np.uint8), oR.keypoints.view(np.uint8))
    assert np.array_equal(dR, oR.descriptors)
    assert (ouR >= 0).sum() > 50
    assert np.array_equal(uR.view(np.uint32), ouR.view(np.uint32))
    assert np.array_equal(dep.view(np.uint32), odep.view(np.uint32))
    for l in (0, 3, 7):
        assert np.array_equal(ex.pyramid_level(l, image=0), oL.level(l))
        assert np.array_equal(ex.pyramid_level(l, image=1), oR.level(l))
    with pytest.raises(OrbxError) as ei:
        compute_stereo_matches(ex, ex, kL, dL, kR, dR, bf, bf / fx)
    assert ei.value.code == ORBX_ERR_STATE
    # the same handle serves orbx_extract afterwards, and a second frame_stereo repeats the first
    kx, dx = ex(np.ascontiguousarray(L))
    assert np.array_equal(kx.view(np.uint8), oL.keypoints.view(np.uint8)) and np.array_equal(dx, oL.descriptors)
    again = frame_stereo(ex, L, R, bf, bf / fx)
    assert np.array_equal(again[4].view(np.uint32), uR.view(np.uint32))


def test_frame_stereo_empty_side(gpu):
    """A flat right image has no keypoints: every left keypoint stays unmatched (-1), as
    ComputeStereoMatches leaves it; a flat left image returns nothing at all."""
    from orb_slam2_commit_amd import frame_stereo
    L, _ = synth.stereo_pair(9, 640, 480)
    flat = np.full_like(L, 128)
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    kL, dL, kR, dR, uR, dep = frame_stereo(ex, L, flat, KITTI_BF, KITTI_BF / KITTI_FX)
    assert len(kL) > 100 and len(kR) == 0 and dR is None
    assert (uR == -1).all() and (dep == -1).all()
    kL, dL, kR, dR, uR, dep = frame_stereo(ex, flat, L, KITTI_BF, KITTI_BF / KITTI_FX)
    assert len(kL) == 0 and dL is None and len(kR) > 100 and len(uR) == 0


def test_stereo_uses_only_the_last_extraction(gpu):
    """orbx_stereo_match reads each extractor's device-resident keypoints, descriptors and pyramid
    (no upload), so it accepts only exactly what that extractor's last orbx_extract returned:
    a changed descriptor bit, a changed keypoint, or a newer extraction on the right handle is
    ORBX_ERR_STATE; repeating the call on the true outputs is bit-identical."""
    from orb_slam2_commit_amd._lib import ORBX_ERR_STATE, OrbxError
    L, R = synth.stereo_pair(5, 1241, 376)
    exL, exR = ORBextractor(2000, 1.2, 8, 20, 7), ORBextractor(2000, 1.2, 8, 20, 7)
    kL, dL = exL(L)
    kR, dR = exR(R)
    bl = KITTI_BF / KITTI_FX
    uR1, d1 = compute_stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, bl)
    uR2, d2 = compute_stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, bl)
    assert np.array_equal(uR1.view(np.uint32), uR2.view(np.uint32)) and np.array_equal(d1, d2)
    dbad = dL.copy()
    dbad[7, 3] ^= 1
    kbad = kL.copy()
    kbad["x"][0] += 0.5
    for args in [(kL, dbad, kR, dR), (kbad, dL, kR, dR), (kL, dL, kR, dR[::-1].copy())]:
        with pytest.raises(OrbxError) as ei:
            compute_stereo_matches(exL, exR, *args, KITTI_BF, bl)
        assert ei.value.code == ORBX_ERR_STATE
    exR(synth.stereo_pair(6, 1241, 376)[1])  # a newer extraction on the right handle
    with pytest.raises(OrbxError) as ei:
        compute_stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, bl)
    assert ei.value.code == ORBX_ERR_STATE


def test_stereo_frames_device(gpu):
    import torch
    n = 3
    pairs = [synth.stereo_pair(40 + i, 1241, 376) for i in range(n)]
    imgs = np.stack([im for pr in pairs for im in pr])
    ex = ORBextractor(2000, 1.2, 8, 20, 7)
    cap = ex.max_keypoints(1241, 376)
    d = torch.from_numpy(imgs).to(gpu)
    kps = torch.zeros((2 * n, cap, 28), dtype=torch.uint8, device=gpu)
    desc = torch.zeros((2 * n, cap, 32), dtype=torch.uint8, device=gpu)
    cnt = torch.zeros(2 * n, dtype=torch.int32, device=gpu)
    uR = torch.zeros((n, cap), dtype=torch.float32, device=gpu)
    dep = torch.zeros((n, cap), dtype=torch.float32, device=gpu)
    nm = torch.zeros(n, dtype=torch.int32, device=gpu)
    ex.stereo_frames_device(d, kps, desc, cnt, KITTI_BF, KITTI_BF / KITTI_FX, uR, dep, nm,
                            torch.cuda.current_stream())
    torch.cuda.synchronize()
    p = oracle.params(2000, 1.2, 8, 20, 7)
    for f in range(n):
        oL, oR = oracle.extract(p, pairs[f][0]), oracle.extract(p, pairs[f][1])
        ouR, odep = oracle.stereo_match(p, oL, oR, KITTI_BF, KITTI_BF / KITTI_FX)
        nL = int(cnt[2 * f])
        assert nL == len(oL.keypoints)
        assert np.array_equal(uR[f, :nL].cpu().numpy().view(np.uint32), ouR.view(np.uint32))
        assert np.array_equal(dep[f, :nL].cpu().numpy().view(np.uint32), odep.view(np.uint32))
        assert int(nm[f]) == int((ouR >= 0).sum())


def test_descriptor_distance(gpu):
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, (10000, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (10000, 32), dtype=np.uint8)
    b[:10] = a[:10]
    b[10:20] = ~a[10:20]
    d = ORBmatcher.DescriptorDistance(a, b)
    assert np.array_equal(d, oracle.hamming_pairs(a, b))
    assert (d[:10] == 0).all() and (d[10:20] == 256).all()
    assert ORBmatcher.DescriptorDistance(a[0], b[0]) == int(oracle.hamming_pairs(a[:1], b[:1])[0])


def test_bench_batch_slots_match_oracle(gpu):
    """The bench's exact timed batch (B = 256 frames = 512 KITTI images, bench.py / synth.stereo_batch):
    the first, a middle and the last slot against the oracle -- L and R keypoints, descriptors, uR,
    depth and the match count (large-batch pyramid / candidate / output offsets)."""
    import torch
    B = 256
    host = synth.stereo_batch(0, B)
    ex = ORBextractor(2000, 1.2, 8, 20, 7)
    cap = ex.max_keypoints(1241, 376)
    d = torch.from_numpy(host).to(gpu)
    kps = torch.zeros((2 * B, cap, 28), dtype=torch.uint8, device=gpu)
    desc = torch.zeros((2 * B, cap, 32), dtype=torch.uint8, device=gpu)
    cnt = torch.zeros(2 * B, dtype=torch.int32, device=gpu)
    uR = torch.zeros((B, cap), dtype=torch.float32, device=gpu)
    dep = torch.zeros((B, cap), dtype=torch.float32, device=gpu)
    nm = torch.zeros(B, dtype=torch.int32, device=gpu)
    ex.stereo_frames_device(d, kps, desc, cnt, KITTI_BF, KITTI_BF / KITTI_FX, uR, dep, nm,
                            torch.cuda.current_stream())
    torch.cuda.synchronize()
    kps, desc, cnt = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
    uR, dep, nm = uR.cpu().numpy(), dep.cpu().numpy(), nm.cpu().numpy()
    p = oracle.params(2000, 1.2, 8, 20, 7)
    for f in (0, 1, B // 2 - 1, B // 2, B - 1):
        o = [oracle.extract(p, host[2 * f + k]) for k in (0, 1)]
        for k in (0, 1):
            n = int(cnt[2 * f + k])
            assert n == len(o[k].keypoints), (f, k)
            assert kps[2 * f + k, :n].tobytes() == o[k].keypoints.tobytes(), (f, k)
            assert np.array_equal(desc[2 * f + k, :n], o[k].descriptors), (f, k)
        ouR, odep = oracle.stereo_match(p, o[0], o[1], KITTI_BF, KITTI_BF / KITTI_FX)
        nL = int(cnt[2 * f])
        assert np.array_equal(uR[f, :nL].view(np.uint32), ouR.view(np.uint32)), f
        assert np.array_equal(dep[f, :nL].view(np.uint32), odep.view(np.uint32)), f
        assert int(nm[f]) == int((ouR >= 0).sum()), f


def test_stereo_frames_device_ragged(gpu):
    """A device batch with ragged and empty frames: a blank left image (no left keypoints), a blank
    right image (every left keypoint unmatched), a low-texture pair (a left count that is no multiple
    of the 16 keypoints a match block takes) beside a textured pair -- each frame equal to the oracle,
    the empty ones writing nothing past their counts and zero matches."""
    import torch
    w, h = 1241, 376
    blank = np.full((h, w), 128, np.uint8)
    L0, R0 = synth.stereo_pair(61, w, h)
    L3, R3 = synth.stereo_pair(62, w, h)
    rng = np.random.default_rng(9)
    soft = (blank.astype(np.int16) + rng.integers(-12, 13, (h, w))).clip(0, 255).astype(np.uint8)
    pairs = [(L0, R0), (blank, R0), (L0, blank), (soft, np.roll(soft, -7, axis=1)), (L3, R3)]
    n = len(pairs)
    imgs = np.stack([im for pr in pairs for im in pr])
    ex = ORBextractor(2000, 1.2, 8, 20, 7)
    cap = ex.max_keypoints(w, h)
    d = torch.from_numpy(imgs).to(gpu)
    kps = torch.zeros((2 * n, cap, 28), dtype=torch.uint8, device=gpu)
    desc = torch.zeros((2 * n, cap, 32), dtype=torch.uint8, device=gpu)
    cnt = torch.zeros(2 * n, dtype=torch.int32, device=gpu)
    uR = torch.full((n, cap), 7.0, dtype=torch.float32, device=gpu)
    dep = torch.full((n, cap), 7.0, dtype=torch.float32, device=gpu)
    nm = torch.full((n,), -5, dtype=torch.int32, device=gpu)
    ex.stereo_frames_device(d, kps, desc, cnt, KITTI_BF, KITTI_BF / KITTI_FX, uR, dep, nm,
                            torch.cuda.current_stream())
    torch.cuda.synchronize()
    p = oracle.params(2000, 1.2, 8, 20, 7)
    cnt_h, uR_h, dep_h, nm_h = cnt.cpu().numpy(), uR.cpu().numpy(), dep.cpu().numpy(), nm.cpu().numpy()
    counts = []
    for f in range(n):
        oL, oR = oracle.extract(p, pairs[f][0]), oracle.extract(p, pairs[f][1])
        nL = int(cnt_h[2 * f])
        assert nL == len(oL.keypoints) and int(cnt_h[2 * f + 1]) == len(oR.keypoints), f
        counts.append((nL, len(oR.keypoints)))
        if nL:
            ouR, odep = oracle.stereo_match(p, oL, oR, KITTI_BF, KITTI_BF / KITTI_FX)
            assert np.array_equal(uR_h[f, :nL].view(np.uint32), ouR.view(np.uint32)), f
            assert np.array_equal(dep_h[f, :nL].view(np.uint32), odep.view(np.uint32)), f
            assert int(nm_h[f]) == int((ouR >= 0).sum()), f
        else:
            assert int(nm_h[f]) == 0, f
        assert (uR_h[f, nL:] == 7.0).all() and (dep_h[f, nL:] == 7.0).all(), f  # nothing past the count
    assert counts[1][0] == 0 and counts[2][1] == 0 and int(nm_h[2]) == 0
    assert counts[3][0] % 16 != 0 or counts[0][0] % 16 != 0
