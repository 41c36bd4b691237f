"""CPU known-answer tests pinning the oracle (oracle/orb_oracle.cpp).

The reference ships no tests or golden vectors and cannot be built here
(SURVEY.md §0, §8c), so each OpenCV-3.2 primitive the oracle restates is
checked against an INDEPENDENT restatement (numpy / python) of its published
definition, plus structural invariants of ORBextractor's output.
"""
import math
import os

import numpy as np
import pytest

import oracle
from orb_slam2_commit_amd import synth

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2), (-3, -1),
        (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def np_fast_window(img, t):
    """Brute-force FAST-9 (OpenCV FAST_t<16> definition) with window-local 3x3 NMS."""
    img = img.astype(np.int32)
    h, w = img.shape
    score = np.zeros((h, w), np.int32)
    corner = np.zeros((h, w), bool)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            v = img[y, x]
            p = [img[y + dy, x + dx] for dx, dy in RING]
            d = [v - q for q in p]
            best = -10 ** 9
            is_c = False
            for k in range(16):
                arc = [d[(k + j) % 16] for j in range(9)]
                best = max(best, min(arc), -max(arc))
                if all(a > t for a in arc) or all(a < -t for a in arc):
                    is_c = True
            if is_c:
                corner[y, x] = True
                score[y, x] = best - 1
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            if not corner[y, x]:
                continue
            s = score[y, x]
            nb = [score[y + dy, x + dx] if corner[y + dy, x + dx] else 0
                  for dy in (-1, 0, 1) for dx in (-1, 0, 1) if (dx, dy) != (0, 0)]
            if all(s > n for n in nb):
                out.append((x, y, s))
    return np.array(out, np.int32).reshape(-1, 3)


@pytest.mark.parametrize("seed", range(6))
def test_fast_matches_bruteforce(seed):
    rng = np.random.default_rng(seed)
    if seed < 3:
        img = rng.integers(0, 256, (23, 29), dtype=np.uint8)
    else:
        img = synth.mono_image(seed, 64, 48)[5:30, 7:40].copy()
    for t in (7, 20):
        assert np.array_equal(oracle.fast_window(img, t), np_fast_window(img, t))


def test_fast_arc_lengths():
    # exactly 9 contiguous brighter ring pixels -> corner; 8 -> not
    for n_arc, expect in ((9, True), (8, False)):
        img = np.full((7, 7), 100, np.uint8)
        for k in range(n_arc):
            dx, dy = RING[k]
            img[3 + dy, 3 + dx] = 200
        got = oracle.fast_window(img, 20)
        assert (len(got) == 1) == expect
        if expect:
            # cornerScore = max over arcs of min |d| - 1 = 100 - 1
            assert got[0, 2] == 99
            assert oracle.fast_score(img, 3, 3) == 99


def test_gaussian_kernel_integers():
    # OpenCV getGaussianKernel(7, 2, CV_32F) scaled by 256 and cvRound'ed
    x = np.arange(7) - 3.0
    g = np.exp(-0.5 * x * x / 4.0).astype(np.float32)
    g = (g.astype(np.float64) * (1.0 / g.astype(np.float64).sum())).astype(np.float32)
    k = np.rint(g * np.float32(256)).astype(int)
    assert k.tolist() == [18, 34, 49, 55, 49, 34, 18] and k.sum() == 257
    # delta response of the oracle blur equals the outer product, rounded
    img = np.zeros((15, 17), np.uint8)
    img[7, 8] = 255
    out = oracle.gaussian_blur7(img).astype(np.int64)
    acc = np.outer(k, k) * 255
    w = img.shape[1]
    simd_w = w & ~3
    exp = np.zeros_like(out)
    for yy in range(7):
        for xx in range(7):
            X = 8 + xx - 3
            a = int(acc[yy, xx])
            v = int(np.rint(np.float32(a) * np.float32(1 / 65536))) if X < simd_w else (a + 32768) >> 16
            exp[7 + yy - 3, X] = min(max(v, 0), 255)
    assert np.array_equal(out, exp)


def test_blur_constant_and_border():
    img = np.full((40, 37), 77, np.uint8)
    b = oracle.gaussian_blur7(img)
    k_sum = 257  # the integer kernel sums to 257
    assert np.all(np.abs(b.astype(int) - 77 * k_sum * k_sum / 65536) <= 1)


def np_resize_linear(src, dw, dh):
    """Independent numpy restatement of OpenCV 3.2 INTER_LINEAR 8U fixed point."""
    sh, sw = src.shape
    sx_scale = 1.0 / (dw / sw)
    sy_scale = 1.0 / (dh / sh)
    out = np.zeros((dh, dw), np.uint8)
    xo, a0, a1 = [], [], []
    for dx in range(dw):
        fx = np.float32((dx + 0.5) * sx_scale - 0.5)
        sx = int(np.floor(fx))
        fx = np.float32(fx - np.float32(sx))
        if sx < 0:
            fx, sx = np.float32(0), 0
        if sx >= sw - 1:
            fx, sx = np.float32(0), sw - 1
        xo.append(sx)
        a0.append(int(np.rint((np.float32(1) - fx) * np.float32(2048))))
        a1.append(int(np.rint(fx * np.float32(2048))))
    S = src.astype(np.int64)
    for dy in range(dh):
        fy = np.float32((dy + 0.5) * sy_scale - 0.5)
        sy = int(np.floor(fy))
        fy = np.float32(fy - np.float32(sy))
        b0 = int(np.rint((np.float32(1) - fy) * np.float32(2048)))
        b1 = int(np.rint(fy * np.float32(2048)))
        r = [S[min(max(sy, 0), sh - 1)], S[min(max(sy + 1, 0), sh - 1)]]
        for dx in range(dw):
            sx = xo[dx]
            hs = [rr[sx] * a0[dx] + rr[min(sx + 1, sw - 1)] * a1[dx] for rr in r]
            out[dy, dx] = (((b0 * (hs[0] >> 4)) >> 16) + ((b1 * (hs[1] >> 4)) >> 16) + 2) >> 2
    return out


@pytest.mark.parametrize("shape,dst", [((48, 64), (53, 40)), ((37, 41), (34, 31)), ((20, 20), (17, 17))])
def test_resize_matches_numpy(shape, dst):
    rng = np.random.default_rng(1)
    src = rng.integers(0, 256, shape, dtype=np.uint8)
    assert np.array_equal(oracle.resize_linear(src, *dst), np_resize_linear(src, *dst))


def test_resize_constant():
    src = np.full((50, 70), 200, np.uint8)
    assert np.all(oracle.resize_linear(src, 58, 42) == 200)


def test_fast_atan2():
    for y, x in [(1, 1), (0, 1), (1, 0), (0, -1), (-1, 0), (-3, -4), (5, -2), (1e3, 7), (-7, 1e3), (0, 0)]:
        a = oracle.fast_atan2(y, x)
        ref = math.degrees(math.atan2(y, x)) % 360.0
        assert 0 <= a < 360.0 + 1e-3
        if (x, y) != (0, 0):
            diff = min(abs(a - ref), 360 - abs(a - ref))
            assert diff < 0.3, (y, x, a, ref)


def test_sincos_correctly_rounded():
    xs = np.linspace(0, 2 * np.pi, 20001).astype(np.float32)
    c = np.array([oracle.cosf(float(x)) for x in xs], np.float32)
    s = np.array([oracle.sinf(float(x)) for x in xs], np.float32)
    assert np.array_equal(c, np.cos(xs.astype(np.float64)).astype(np.float32))
    assert np.array_equal(s, np.sin(xs.astype(np.float64)).astype(np.float32))


def test_hamming_vs_numpy():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (500, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (500, 32), dtype=np.uint8)
    ref = np.unpackbits(a ^ b, axis=1).sum(axis=1)
    assert np.array_equal(oracle.hamming_pairs(a, b), ref)


def test_scale_tables():
    t = oracle.scale_tables(oracle.params(2000, 1.2, 8, 20, 7))
    assert t["features_per_level"].tolist() == [434, 362, 302, 251, 209, 175, 145, 122]
    assert abs(float(t["scale"][7]) - 1.2 ** 7) < 1e-5
    t = oracle.scale_tables(oracle.params(1000, 1.2, 8, 20, 7))
    assert t["features_per_level"].tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    t = oracle.scale_tables(oracle.params(1200, 1.2, 8, 20, 7))
    assert t["features_per_level"].tolist() == [261, 217, 181, 151, 126, 105, 87, 72]


def test_extraction_invariants():
    p = oracle.params(1000, 1.2, 8, 20, 7)
    img = synth.mono_image(2, 640, 480)
    ex = oracle.extract(p, img)
    k = ex.keypoints
    assert np.all(np.diff(k["octave"]) >= 0)  # level-major output
    t = oracle.scale_tables(p)
    nf = t["features_per_level"]
    counts = np.bincount(k["octave"], minlength=8)
    assert np.all(counts <= nf + 3)
    assert np.all(k["class_id"] == -1)
    assert np.all((k["angle"] >= 0) & (k["angle"] < 360))
    sizes = np.array([int(31 * s) for s in t["scale"]], np.float32)
    assert np.array_equal(k["size"], sizes[k["octave"]])
    wh = ex.level_wh
    assert wh[1].tolist() == [533, 400] and wh[7].tolist() == [179, 134]
    # deterministic
    ex2 = oracle.extract(p, img)
    assert np.array_equal(ex2.keypoints.view(np.uint8), k.view(np.uint8))
    assert np.array_equal(ex2.descriptors, ex.descriptors)


def test_stereo_recovers_disparity_bands():
    """Synthetic right view = left shifted by per-band integer disparities."""
    L, R = synth.stereo_pair(0, 1241, 376)
    p = oracle.params(2000, 1.2, 8, 20, 7)
    bf, fx = 386.1448, 718.856
    eL, eR = oracle.extract(p, L), oracle.extract(p, R)
    uR, depth = oracle.stereo_match(p, eL, eR, bf, bf / fx)
    ok = uR >= 0
    assert ok.sum() > 500
    disp = eL.keypoints["x"][ok] - uR[ok]
    assert np.median(np.abs(disp - np.rint(disp))) < 0.35
    assert np.allclose(depth[ok], bf / disp, rtol=1e-5)


# --- libm divergence of the keypoint rotation (src/ORBextractor.cc:117) -------------------------
# The reference calls the host libm's cosf/sinf; oracle and GPU share sincos_det (a double
# evaluation rounded once = correctly rounded cos/sin).  glibc's float cos/sin is not correctly
# rounded: over all 1,086,918,620 floats in [0, 2*pi] it differs from sincos_det on 446,486 (cos) /
# 1,020,963 (sin) inputs, and only 88 of those angles change any of the 512 rotated BRIEF offsets
# (tools/trig_census.py; tests/golden/trig_pattern_angles.npy).  These tests pin that census.

def test_trig_libm_census_sample():
    # every 257th float of [0, 2*pi]: same mismatch rate as the full census (~1.35e-3)
    dc, ds, n = oracle.trig_census(0.0, float(np.float32(2 * np.pi)), 257)
    rate = (dc + ds) / n
    assert 0.5e-3 < rate < 2.5e-3, (dc, ds, n)


def test_trig_libm_pattern_angles():
    """Each committed angle changes the rotated pattern under libm; a strided census finds no others."""
    ang = np.load(GOLDEN_DIR + "/trig_pattern_angles.npy")
    assert len(ang) == 88
    for a in ang[:16]:
        a = float(a)
        nt, npat, n, found = oracle.trig_pattern_census(a, a, 1)
        assert (nt, npat, n) == (1, 1, 1)
    # the measure of pattern-changing angles (uniform in radians): ~1.9e-6 per keypoint
    frac = float(np.spacing(ang).astype(np.float64).sum() / (2 * np.pi))
    assert frac < 5e-6


def test_trig_libm_descriptor_divergence():
    """Extraction with libm cosf/sinf vs sincos_det on the golden and KITTI/EuRoC/TUM/stress images:
    identical keypoints, and 0 differing descriptors (32,961 descriptors in the full sweep)."""
    cases = []
    for name in ("extract_a", "extract_b", "extract_noise"):
        d = np.load(GOLDEN_DIR + "/%s.npz" % name)
        cases.append((d["image"], oracle.params(int(d["params"][0]), float(d["params"][1]), *[int(v) for v in d["params"][2:]])))
    for s in range(2):
        cases.append((synth.stereo_pair(s)[0], oracle.params(2000, 1.2, 8, 20, 7)))
        cases.append((synth.stereo_pair(s, 752, 480)[0], oracle.params(1200, 1.2, 8, 20, 7)))
        cases.append((synth.mono_image(s), oracle.params(1000, 1.2, 8, 20, 7)))
    cases.append((synth.stereo_pair(0, stress=True)[0], oracle.params(2000, 1.2, 8, 20, 7)))
    n_desc = n_diff = 0
    try:
        for img, p in cases:
            oracle.set_trig_mode(0)
            a = oracle.extract(p, img)
            oracle.set_trig_mode(1)
            b = oracle.extract(p, img)
            assert a.keypoints.tobytes() == b.keypoints.tobytes()
            n_desc += len(a.descriptors)
            n_diff += int(np.any(a.descriptors != b.descriptors, axis=1).sum())
    finally:
        oracle.set_trig_mode(0)
    assert n_desc > 10000
    assert n_diff == 0
