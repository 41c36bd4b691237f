"""MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:249-320) and
Frame::UndistortKeyPoints (src/Frame.cc:471-506, cv::undistortPoints).

CPU: the C++ oracle against literal pure-Python restatements (the N x N
distance matrix with numpy row sorts and the strict `median < BestMedian`
scan; cvUndistortPoints' FP64 sequence written out in Python floats, which
are IEEE doubles), plus a round-trip property for the undistortion (the
forward Brown-Conrady model maps the undistorted point back onto the input).
GPU (-m gpu): HIP kernels vs the oracle bit for bit.  Parity against the
genuine OpenCV 3.2 is unpinned: no OpenCV here, and the
reference holds no fixtures.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402

f32 = np.float32

# Published calibrations the reference's example configurations use (TUM fr1 with k3, EuRoC
# cam0 with four coefficients) and KITTI-00 (rectified: mDistCoef = 0).
TUM1 = (np.array([[517.306408, 0, 318.643040], [0, 516.469215, 255.313989], [0, 0, 1]], np.float32),
        np.array([0.262383, -0.953104, -0.005358, 0.002628, 1.163314], np.float32), 640, 480)
EUROC = (np.array([[458.654, 0, 367.215], [0, 457.296, 248.375], [0, 0, 1]], np.float32),
         np.array([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05], np.float32), 752, 480)
KITTI = (np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]], np.float32),
         np.zeros(4, np.float32), 1241, 376)


# ------------------------------------------------------------------ restatements
def py_distinctive(descs):
    n = len(descs)
    if n == 0:
        return -1
    bits = np.unpackbits(descs, axis=1).astype(np.int32)
    D = np.zeros((n, n), np.float32)  # float Distances[N][N]
    for i in range(n):
        for j in range(i + 1, n):
            D[i, j] = D[j, i] = int(np.sum(bits[i] != bits[j]))
    best_median, best = 2 ** 31 - 1, 0
    for i in range(n):
        row = np.sort(D[i].astype(np.int32))
        median = int(row[int(0.5 * (n - 1))])
        if median < best_median:
            best_median, best = median, i
    return best


def py_undistort(K, d, x, y):
    k = [0.0] * 5
    for i, v in enumerate(d):
        k[i] = float(v)
    A = [float(v) for v in np.asarray(K, np.float32).reshape(9)]
    ifx, ify = 1.0 / A[0], 1.0 / A[4]
    x = (float(x) - A[2]) * ifx
    y = (float(y) - A[5]) * ify
    x0, y0 = x, y
    for _ in range(5):
        r2 = x * x + y * y
        icdist = 1 / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
        dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
        dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
        x = (x0 - dx) * icdist
        y = (y0 - dy) * icdist
    xx = A[0] * x + A[1] * y + A[2]
    yy = A[3] * x + A[4] * y + A[5]
    ww = 1.0 / (A[6] * x + A[7] * y + A[8])
    return f32(xx * ww), f32(yy * ww)


def observations(seed, n_points, max_obs=40, extra=()):
    """Synthetic MapPoints: each point's observed descriptors are a centre with a few bit flips
    (what a well-tracked MapPoint sees), some fully random (outlier observations)."""
    rng = np.random.default_rng(seed)
    counts = list(rng.integers(0, max_obs + 1, n_points)) + list(extra)
    rows = []
    for c in counts:
        centre = rng.integers(0, 256, 32, dtype=np.uint8)
        for _ in range(c):
            if rng.random() < 0.15:
                rows.append(rng.integers(0, 256, 32, dtype=np.uint8))
                continue
            b = np.unpackbits(centre)
            flip = rng.choice(256, int(rng.integers(0, 40)), replace=False)
            b[flip] ^= 1
            rows.append(np.packbits(b))
    desc = np.array(rows, np.uint8).reshape(-1, 32)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    return desc, off


def random_keys(seed, n, w, h):
    rng = np.random.default_rng(seed)
    k = np.zeros(n, oracle.KEYPOINT_DTYPE)
    k["x"] = rng.uniform(0, w, n).astype(np.float32)
    k["y"] = rng.uniform(0, h, n).astype(np.float32)
    k["x"][:4] = [0, w, 0, w]
    k["y"][:4] = [0, 0, h, h]
    k["size"] = 31
    k["angle"] = rng.uniform(0, 360, n)
    k["response"] = rng.uniform(0, 100, n)
    k["octave"] = rng.integers(0, 8, n)
    k["class_id"] = -1
    return k


# ------------------------------------------------------------------ CPU
def test_distinctive_oracle_vs_python():
    desc, off = observations(0, 150, extra=(0, 1, 2, 63, 64, 65, 130))
    best, out = oracle.distinctive_descriptors(desc, off)
    for p in range(len(off) - 1):
        want = py_distinctive(desc[off[p]:off[p + 1]])
        assert best[p] == want, p
        if want >= 0:
            assert np.array_equal(out[p], desc[off[p] + want])


def test_distinctive_ties_first_row_wins():
    d = np.zeros((4, 32), np.uint8)  # all identical: every median 0 -> row 0
    b, _ = oracle.distinctive_descriptors(d, [0, 4])
    assert b[0] == 0
    d = np.zeros((2, 32), np.uint8)
    d[1, 0] = 0xFF  # two rows: medians vDists[0] = 0 for both -> row 0
    assert oracle.distinctive_descriptors(d, [0, 2])[0][0] == 0


@pytest.mark.parametrize("cal", [TUM1, EUROC])
def test_undistort_oracle_vs_python(cal):
    K, d, w, h = cal
    keys = random_keys(1, 300, w, h)
    got = oracle.undistort_keypoints(keys, K, d)
    for i in range(len(keys)):
        x, y = py_undistort(K, d, keys["x"][i], keys["y"][i])
        assert got["x"][i].view(np.uint32) == x.view(np.uint32) and got["y"][i].view(np.uint32) == y.view(np.uint32)
    for f in ("size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(got[f], keys[f])


@pytest.mark.parametrize("cal", [TUM1, EUROC])
def test_undistort_round_trip(cal):
    """Distorting the undistorted point (Brown-Conrady forward model) lands back near the input:
    pins the model and coefficient order, not just the arithmetic."""
    K, d, w, h = cal
    keys = random_keys(2, 400, w, h)
    keys = keys[(np.abs(keys["x"] - w / 2) < 0.25 * w) & (np.abs(keys["y"] - h / 2) < 0.25 * h)]
    u = oracle.undistort_keypoints(keys, K, d)
    k = list(map(float, d)) + [0.0] * (5 - len(d))
    fx, fy, cx, cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    x = (u["x"].astype(np.float64) - cx) / fx
    y = (u["y"].astype(np.float64) - cy) / fy
    r2 = x * x + y * y
    rad = 1 + k[0] * r2 + k[1] * r2 ** 2 + k[4] * r2 ** 3
    xd = x * rad + 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
    yd = y * rad + k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
    assert np.max(np.abs(xd * fx + cx - keys["x"])) < 0.02
    assert np.max(np.abs(yd * fy + cy - keys["y"])) < 0.02


def test_undistort_zero_coefficients_copy():
    K, d, w, h = KITTI
    keys = random_keys(3, 100, w, h)
    assert np.array_equal(oracle.undistort_keypoints(keys, K, d).view(np.uint8), keys.view(np.uint8))


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_gpu_distinctive(gpu):
    from orb_slam2_commit_amd.orb import compute_distinctive_descriptors
    desc, off = observations(10, 3000, extra=(0, 1, 2, 63, 64, 65, 129, 300))
    rb, ro = oracle.distinctive_descriptors(desc, off)
    gb, go = compute_distinctive_descriptors(desc, off)
    assert np.array_equal(gb, rb)
    m = rb >= 0
    assert np.array_equal(go[m], ro[m])


@pytest.mark.gpu
def test_gpu_distinctive_device_and_empty(gpu):
    import ctypes as C
    import torch
    from orb_slam2_commit_amd import _lib
    desc, off = observations(11, 20000, max_obs=12)
    rb, ro = oracle.distinctive_descriptors(desc, off)
    dd, do = torch.from_numpy(desc).to(gpu), torch.from_numpy(off).to(gpu)
    n = len(off) - 1
    best = torch.full((n,), -9, dtype=torch.int32, device=gpu)
    out = torch.zeros((n, 32), dtype=torch.uint8, device=gpu)
    s = torch.cuda.current_stream()
    L = _lib.lib()
    _lib.check(L.orbx_distinctive_descriptors_device(dd.data_ptr(), do.data_ptr(), n, best.data_ptr(),
                                                     out.data_ptr(), C.c_void_p(s.cuda_stream)), "distinctive")
    torch.cuda.synchronize()
    assert np.array_equal(best.cpu().numpy(), rb)
    m = rb >= 0
    assert np.array_equal(out.cpu().numpy()[m], ro[m])
    assert L.orbx_distinctive_descriptors(None, None, 0, None, None, 0) == 0
    assert L.orbx_distinctive_descriptors(None, None, 3, None, None, 0) == _lib.ORBX_ERR_ARG


@pytest.mark.gpu
@pytest.mark.parametrize("cal", [TUM1, EUROC, KITTI])
def test_gpu_undistort(gpu, cal):
    from orb_slam2_commit_amd.orb import compute_image_bounds, undistort_keypoints
    K, d, w, h = cal
    keys = random_keys(20, 2000, w, h)
    ref = oracle.undistort_keypoints(keys, K, d)
    got = undistort_keypoints(keys, K, d)
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8))
    c = np.zeros(4, oracle.KEYPOINT_DTYPE)
    c["x"], c["y"] = [0, w, 0, w], [0, 0, h, h]
    u = oracle.undistort_keypoints(c, K, d)
    want = ((min(u["x"][0], u["x"][2]), max(u["x"][1], u["x"][3]), min(u["y"][0], u["y"][1]),
             max(u["y"][2], u["y"][3])) if d[0] != 0 else (0.0, w, 0.0, h))
    assert compute_image_bounds(w, h, K, d) == tuple(float(v) for v in want)


@pytest.mark.gpu
def test_gpu_undistort_frame_batch(gpu):
    import ctypes as C
    import torch
    from orb_slam2_commit_amd import _lib
    from orb_slam2_commit_amd.orb import camera
    cals = [TUM1, EUROC, KITTI, TUM1, EUROC]
    counts = [2000, 1200, 0, 777, 1]
    keys = [random_keys(30 + i, max(c, 4), cal[2], cal[3])[:c] for i, (c, cal) in enumerate(zip(counts, cals))]
    allk = np.concatenate(keys)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    cams = (_lib.Camera * len(cals))(*[camera(c[0], c[1]) for c in cals])
    cam_bytes = np.frombuffer(bytes(cams), np.uint8).copy()
    dk = torch.from_numpy(allk.view(np.uint8).copy()).to(gpu)
    dout = torch.zeros_like(dk)
    doff, dcam = torch.from_numpy(off).to(gpu), torch.from_numpy(cam_bytes).to(gpu)
    s = torch.cuda.current_stream()
    _lib.check(_lib.lib().orbx_undistort_keypoints_device(dk.data_ptr(), doff.data_ptr(), len(cals), max(counts),
                                                          dcam.data_ptr(), dout.data_ptr(), C.c_void_p(s.cuda_stream)),
               "undistort batch")
    torch.cuda.synchronize()
    got = dout.cpu().numpy().view(oracle.KEYPOINT_DTYPE)
    for f, (k, cal) in enumerate(zip(keys, cals)):
        ref = oracle.undistort_keypoints(k, cal[0], cal[1])
        assert np.array_equal(got[off[f]:off[f + 1]].view(np.uint8), ref.view(np.uint8)), f
