"""Seeded synthetic stereo imagery (SURVEY.md §8d "Synthetic inputs").

No datasets exist in the container, so every benchmark and parity case runs on
images generated here from ``numpy.random.default_rng(seed)``:

* left image: low-frequency background (uniform noise at 1/8 resolution,
  bilinearly upsampled) + random filled triangles/quads/ellipses with grey
  levels U[0,255] + Gaussian noise sigma=2, clipped to u8;
* right image: the left scene warped horizontally by a piecewise-constant
  disparity field d in [2, 60] px (per random vertical band) + independent
  noise sigma=2.

Shapes follow the BASELINE.json configs: KITTI 1241x376 (2000 features),
EuRoC 752x480 (1200), TUM 640x480 (1000).
"""
import numpy as np

CONFIGS = {
    "kitti": dict(width=1241, height=376, nfeatures=2000, fx=718.856, bf=386.1448),
    "euroc": dict(width=752, height=480, nfeatures=1200, fx=435.2047, bf=47.9064),
    "tum": dict(width=640, height=480, nfeatures=1000, fx=517.306408, bf=40.0),
}


def _upsample(small, h, w):
    sh, sw = small.shape
    ys = np.linspace(0, sh - 1, h)
    xs = np.linspace(0, sw - 1, w)
    y0 = np.floor(ys).astype(int)
    x0 = np.floor(xs).astype(int)
    y1 = np.minimum(y0 + 1, sh - 1)
    x1 = np.minimum(x0 + 1, sw - 1)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    a = small[y0][:, x0] * (1 - fx) + small[y0][:, x1] * fx
    b = small[y1][:, x0] * (1 - fx) + small[y1][:, x1] * fx
    return a * (1 - fy) + b * fy


def _scene(rng, h, w, n_shapes):
    img = _upsample(rng.uniform(40, 215, size=(h // 8 + 2, w // 8 + 2)), h, w)
    for _ in range(n_shapes):
        kind = rng.integers(0, 3)
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        r = rng.uniform(6, 70)
        x0, x1 = int(max(cx - r, 0)), int(min(cx + r + 1, w))
        y0, y1 = int(max(cy - r, 0)), int(min(cy + r + 1, h))
        if x1 <= x0 or y1 <= y0:
            continue
        yy, xx = np.mgrid[y0:y1, x0:x1]
        if kind == 0:  # ellipse
            ax, ay = r, r * rng.uniform(0.3, 1.0)
            m = ((xx - cx) / ax) ** 2 + ((yy - cy) / ay) ** 2 <= 1.0
        else:  # convex polygon (triangle or quad) via half-planes
            k = 3 if kind == 1 else 4
            ang = np.sort(rng.uniform(0, 2 * np.pi, k))
            px = cx + r * np.cos(ang)
            py = cy + r * np.sin(ang)
            m = np.ones(xx.shape, bool)
            for i in range(k):
                ax_, ay_ = px[i], py[i]
                bx_, by_ = px[(i + 1) % k], py[(i + 1) % k]
                m &= (bx_ - ax_) * (yy - ay_) - (by_ - ay_) * (xx - ax_) >= 0
        img[y0:y1, x0:x1][m] = rng.uniform(0, 255)
    return img


def stereo_pair(seed, width=1241, height=376, n_shapes=None, stress=False):
    """Return (left, right) uint8 arrays of shape (height, width)."""
    rng = np.random.default_rng(seed)
    if stress:
        return (rng.integers(0, 256, (height, width), dtype=np.uint8),
                rng.integers(0, 256, (height, width), dtype=np.uint8))
    if n_shapes is None:
        n_shapes = int(rng.integers(200, 600))
    pad = 64
    scene = _scene(rng, height, width + pad, n_shapes)
    left = scene[:, :width]
    # piecewise-constant disparity over random vertical bands
    n_bands = int(rng.integers(4, 12))
    cuts = np.sort(rng.integers(0, width, n_bands - 1))
    disp = np.empty(width, np.int64)
    edges = np.concatenate([[0], cuts, [width]])
    for i in range(n_bands):
        disp[edges[i]:edges[i + 1]] = rng.integers(2, 61)
    cols = np.arange(width) + disp  # right(x) = left(x + d): points shift left in the right view
    right = scene[:, cols]
    left = left + rng.normal(0, 2, left.shape)
    right = right + rng.normal(0, 2, right.shape)
    return (np.clip(np.rint(left), 0, 255).astype(np.uint8),
            np.clip(np.rint(right), 0, 255).astype(np.uint8))


def sequence_seeds(seq, n_unique):
    """Seeds of the n_unique distinct stereo scenes of synthetic sequence `seq` (KITTI 00..07 -> 0..7)."""
    return [1000 * seq + s for s in range(n_unique)]


def stereo_batch(seq, n_frames, n_unique=16, width=1241, height=376, pairs=None, first=0):
    """Frames first .. first+n_frames-1 of synthetic sequence `seq` as one (2*n_frames, height, width)
    u8 array ordered L0,R0,L1,R1,... (the orbx_stereo_frames_device layout).  Frame f is scene f % U
    rolled horizontally by 53*(f // U) px (left and right alike, so the disparity field is kept); 53
    is coprime with the KITTI width, so no two of the first U*width frames share bytes.  bench.py's
    in-flight batch k is first = k*B."""
    if pairs is None:
        pairs = [stereo_pair(s, width, height) for s in sequence_seeds(seq, n_unique)]
    U = len(pairs)
    return np.stack([np.roll(pairs[f % U][k], 53 * (f // U), axis=1)
                     for f in range(first, first + n_frames) for k in (0, 1)])


def mono_image(seed, width=640, height=480):
    return stereo_pair(seed, width, height)[0]


def bow_problem(seed, n_a=1500, n_b=1500, n_nodes=100, n_true=700, noise_bits=12, rot_deg=25.0, p_valid=0.8):
    """Synthetic SearchByBoW inputs: two feature sets sharing n_true noisy correspondences.

    Returns dict(a=..., b=...) of side dicts {desc, angle, valid, node_id, node_off, feat}.
    Corresponding features share a FeatureVector node and differ by `noise_bits`
    flipped descriptor bits and a global rotation of `rot_deg` (plus outliers),
    which exercises the ratio test, the TH_LOW gate and the rotation histogram.
    """
    rng = np.random.default_rng(seed)
    da = rng.integers(0, 256, (n_a, 32), dtype=np.uint8)
    db = rng.integers(0, 256, (n_b, 32), dtype=np.uint8)
    node_a = rng.integers(0, n_nodes, n_a)
    node_b = rng.integers(0, n_nodes, n_b)
    ang_a = rng.uniform(0, 360, n_a).astype(np.float32)
    ang_b = rng.uniform(0, 360, n_b).astype(np.float32)
    ia = rng.choice(n_a, n_true, replace=False)
    ib = rng.choice(n_b, n_true, replace=False)
    bits = np.unpackbits(da[ia], axis=1)
    for r in range(n_true):
        flip = rng.choice(256, int(rng.integers(0, noise_bits + 1)), replace=False)
        bits[r, flip] ^= 1
    db[ib] = np.packbits(bits, axis=1)
    node_b[ib] = node_a[ia]
    rot = np.where(rng.uniform(size=n_true) < 0.85, rot_deg, rng.uniform(0, 360, n_true))
    ang_b[ib] = np.mod(ang_a[ia] - rot + rng.normal(0, 2, n_true), 360).astype(np.float32)
    ids = np.sort(rng.choice(10 ** 6, n_nodes, replace=False)).astype(np.uint32)

    def side(desc, ang, node):
        order = np.argsort(node, kind="stable")  # feature indices grouped by node, ascending index inside
        counts = np.bincount(node, minlength=n_nodes)
        present = counts > 0
        off = np.concatenate([[0], np.cumsum(counts[present])]).astype(np.int32)
        return dict(desc=desc, angle=ang, valid=(rng.uniform(size=len(desc)) < p_valid).astype(np.uint8),
                    node_id=ids[present], node_off=off, feat=order.astype(np.int32))

    return dict(a=side(da, ang_a, node_a), b=side(db, ang_b, node_b))


def _rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _rot_small(rng, sigma):
    w = rng.normal(0, sigma, 3)
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def localba_problem(seed=7, n_local=20, n_fixed=6, n_points=8000, obs_per_point=5, outlier_frac=0.05,
                    fx=718.856, fy=718.856, cx=607.1928, cy=185.2157, bf=386.1448, width=1241, height=376,
                    th_depth=35.0, pose_noise=(0.01, 0.05), point_noise=0.1, z_range=(5.0, 80.0), pixel_noise=1.0):
    """KITTI-00-shaped LocalBundleAdjustment problem.

    n_local keyframes along +z at 1 m spacing with +-2 deg yaw jitter, n_fixed
    fixed keyframes behind them; n_points points observed by ~obs_per_point
    keyframes each; stereo edge when depth < ThDepth*baseline, else monocular;
    pixel noise sigma = 1.2^octave; outlier_frac of observations offset by 20 px;
    initial poses perturbed by (0.01 rad, 0.05 m), points by 0.1 m."""
    rng = np.random.default_rng(seed)
    base = bf / fx
    n_cams = n_local + n_fixed
    Rwc, twc = [], []
    for i in range(n_cams):
        z = float(i) if i < n_local else -float(i - n_local + 1)
        Rwc.append(_rot_y(np.deg2rad(rng.uniform(-2, 2))))
        twc.append(np.array([rng.uniform(-0.2, 0.2), rng.uniform(-0.05, 0.05), z]))
    Tcw_true = np.zeros((n_cams, 3, 4))
    for i in range(n_cams):
        R = Rwc[i].T
        Tcw_true[i, :, :3] = R
        Tcw_true[i, :, 3] = -R @ twc[i]
    X = np.stack([rng.uniform(-15, 15, n_points), rng.uniform(-3, 2, n_points),
                  rng.uniform(z_range[0], z_range[1], n_points)], axis=1)
    ep, ec, obs, isg = [], [], [], []
    for p in range(n_points):
        Pc = Tcw_true[:, :, :3] @ X[p] + Tcw_true[:, :, 3]
        z = Pc[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = fx * Pc[:, 0] / z + cx
            v = fy * Pc[:, 1] / z + cy
        vis = np.where((z > 0.5) & (u > 20) & (u < width - 20) & (v > 20) & (v < height - 20))[0]
        vis_local = vis[vis < n_local]
        if len(vis_local) == 0:
            continue
        k = min(len(vis), int(rng.integers(obs_per_point - 1, obs_per_point + 2)))
        chosen = set(rng.choice(vis, k, replace=False).tolist())
        chosen.add(int(rng.choice(vis_local)))
        for c in sorted(chosen):
            octave = int(rng.integers(0, 8))
            sigma = 1.2 ** octave
            uu = u[c] + rng.normal(0, sigma * pixel_noise)
            vv = v[c] + rng.normal(0, sigma * pixel_noise)
            ur = -1.0
            if z[c] < th_depth * base:
                ur = uu - bf / z[c] + rng.normal(0, sigma * 0.5 * pixel_noise)
            if rng.uniform() < outlier_frac:
                uu += 20.0
                if ur >= 0:
                    ur += 20.0
            ep.append(p)
            ec.append(c)
            obs.append((uu, vv, ur if ur >= 0 else -1.0))
            isg.append(1.0 / (sigma * sigma))
    Tcw = Tcw_true.copy()
    for i in range(n_local):
        dR = _rot_small(rng, pose_noise[0])
        Tcw[i, :, :3] = dR @ Tcw[i, :, :3]
        Tcw[i, :, 3] = dR @ Tcw[i, :, 3] + rng.normal(0, pose_noise[1], 3)
    Xn = X + rng.normal(0, point_noise, X.shape)
    intr = np.tile(np.array([fx, fy, cx, cy, bf], np.float32), (n_cams, 1))
    fixed = np.zeros(n_cams, np.uint8)
    fixed[n_local:] = 1
    return dict(Tcw=Tcw.reshape(n_cams, 12).astype(np.float32), fixed=fixed, intr=intr,
                Xw=Xn.astype(np.float32), edge_point=np.array(ep, np.int32), edge_cam=np.array(ec, np.int32),
                obs=np.array(obs, np.float32), inv_sigma2=np.array(isg, np.float32),
                Tcw_true=Tcw_true.reshape(n_cams, 12), Xw_true=X)


EUROC = dict(fx=435.2047, fy=435.2047, cx=367.4517, cy=252.2009, bf=47.9064, width=752, height=480)


def pnp_problem(seed=3, n=1200, outlier_frac=0.4, noise_px=1.0, z_range=(2.0, 20.0), scale_factor=1.2,
                nlevels=8, intr=EUROC):
    """PnP RANSAC problem: n 3D-2D matches, outlier_frac
    of them with a random image position, the rest projected by a random true
    pose plus sigma=noise_px pixel noise; octave per match -> sigma2 = sf^(2 octave).

    Returns dict(p3d[n,3] f32, p2d[n,2] f32, sigma2[n] f32, fx, fy, cx, cy, R_true, t_true, outlier[n])."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, W, H = intr["fx"], intr["fy"], intr["cx"], intr["cy"], intr["width"], intr["height"]
    ang = rng.normal(0, 0.3, 3)
    th = np.linalg.norm(ang)
    k = ang / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    t = rng.normal(0, 1.0, 3)
    z = rng.uniform(*z_range, n)
    u = rng.uniform(0, W, n)
    v = rng.uniform(0, H, n)
    Pc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], axis=1)
    Xw = (Pc - t) @ R  # R^T (Pc - t)
    octave = rng.integers(0, nlevels, n)
    sigma2 = (np.float32(scale_factor) ** (2 * octave)).astype(np.float32)
    obs = np.stack([u, v], axis=1) + rng.normal(0, noise_px, (n, 2))
    out = rng.random(n) < outlier_frac
    obs[out] = np.stack([rng.uniform(0, W, out.sum()), rng.uniform(0, H, out.sum())], axis=1)
    return dict(p3d=Xw.astype(np.float32), p2d=obs.astype(np.float32), sigma2=sigma2,
                fx=np.float32(fx), fy=np.float32(fy), cx=np.float32(cx), cy=np.float32(cy),
                R_true=R, t_true=t, outlier=out)


def vocabulary(seed=5, k=10, L=4, scoring=0, weighting=0, flip_p=0.22, p_short=0.05, p_stop=0.03):
    """Synthetic DBoW2 vocabulary in the text format of TemplatedVocabulary::saveToTextFile
    (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1429-1455): header `k L scoring weighting`,
    then one line per node in node-id order: `parent isLeaf d0 .. d31 weight`.  Node ids follow
    DBoW2's HKmeansStep creation order (siblings consecutive, then depth first).  A child's
    descriptor is its parent's with each bit flipped with probability flip_p; some branches end
    early (fewer than k children, leaves above level L), some words are stopped (weight 0).
    Returns (text, node descriptors [n,32] u8, leaf flags) -- ORBvoc.txt is not in the image."""
    rng = np.random.default_rng(seed)
    desc = [np.zeros(32, np.uint8)]
    parent = [-1]
    depth = [0]
    children = [[]]

    def make_children(nid):
        kk = k if rng.random() > 0.15 else int(rng.integers(1, k + 1))
        ids = []
        for _ in range(kk):
            bits = np.unpackbits(desc[nid]) if nid else rng.integers(0, 2, 256).astype(np.uint8)
            flip = (rng.random(256) < (flip_p if nid else 0.5)).astype(np.uint8)
            d = np.packbits(bits ^ flip)
            desc.append(d)
            parent.append(nid)
            depth.append(depth[nid] + 1)
            children.append([])
            ids.append(len(desc) - 1)
        children[nid].extend(ids)
        for c in ids:
            if depth[c] < L and not (depth[c] >= 2 and rng.random() < p_short):
                make_children(c)

    make_children(0)
    lines = [f"{k} {L}  {scoring} {weighting}"]
    leaf = np.zeros(len(desc), bool)
    for nid in range(1, len(desc)):
        is_leaf = not children[nid]
        leaf[nid] = is_leaf
        w = 0.0
        if is_leaf and rng.random() > p_stop:
            w = float(rng.uniform(0.2, 6.0))
        lines.append(f"{parent[nid]} {1 if is_leaf else 0} " + " ".join(str(int(x)) for x in desc[nid]) +
                     f" {w!r}")
    return "\n".join(lines) + "\n", np.array(desc), leaf


def voc_descriptors(seed, voc_desc, leaf, n=800, noise_bits=24, p_random=0.15, p_dup=0.1):
    """Descriptors near random vocabulary leaves (noise_bits flipped), some uniform random, some
    exact duplicates of earlier ones (same word twice)."""
    rng = np.random.default_rng(seed)
    leaves = np.flatnonzero(leaf)
    out = np.zeros((n, 32), np.uint8)
    for i in range(n):
        r = rng.random()
        if i and r < p_dup:
            out[i] = out[rng.integers(0, i)]
        elif r < p_dup + p_random:
            out[i] = rng.integers(0, 256, 32, dtype=np.uint8)
        else:
            bits = np.unpackbits(voc_desc[rng.choice(leaves)])
            bits[rng.choice(256, noise_bits, replace=False)] ^= 1
            out[i] = np.packbits(bits)
    return out


# --------------------------------------------------------------- SearchByProjection
KITTI_K = dict(fx=718.856, fy=718.856, cx=607.1928, cy=185.2157, bf=386.1448)
_LEVEL_SHARE = np.array([434, 362, 302, 251, 209, 175, 145, 122], np.float64)


def scale_factors(scale_factor=1.2, nlevels=8):
    """mvScaleFactor as the ORBextractor ctor builds it (float, x double)."""
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(np.float64(s[-1]) * scale_factor))
    return np.array(s, np.float32)


def _flip_bits(rng, desc, nbits):
    out = desc.copy()
    for k in range(len(out)):
        if nbits[k] > 0:
            pos = rng.choice(256, size=int(nbits[k]), replace=False)
            bits = np.unpackbits(out[k])
            bits[pos] ^= 1
            out[k] = np.packbits(bits)
    return out


def _pose(rng, rot_sigma=0.05, t_sigma=0.5):
    R = _rot_small(rng, rot_sigma)
    t = rng.normal(0, t_sigma, 3)
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T.astype(np.float32)


def projection_frame(seed, width=1241, height=376, n=2000, p_stereo=0.6, p_occ=(0.05, 0.10), cell_crowd=0.0):
    """A current Frame for SearchByProjection: keypoints (mvKeysUn), descriptors,
    mvuRight, mvpMapPoints occupancy, image bounds, grid and KITTI intrinsics.
    cell_crowd > 0 piles that fraction of the keypoints into a few small spots
    (many features per grid cell)."""
    rng = np.random.default_rng(seed)
    from ._lib import KEYPOINT_DTYPE
    keys = np.zeros(n, KEYPOINT_DTYPE)
    keys["x"] = rng.uniform(0, width - 1, n).astype(np.float32)
    keys["y"] = rng.uniform(0, height - 1, n).astype(np.float32)
    if cell_crowd > 0:
        m = rng.random(n) < cell_crowd
        spots = rng.uniform([0, 0], [width - 1, height - 1], size=(4, 2))
        pick = rng.integers(0, 4, m.sum())
        keys["x"][m] = np.clip(spots[pick, 0] + rng.normal(0, 3, m.sum()), 0, width - 1)
        keys["y"][m] = np.clip(spots[pick, 1] + rng.normal(0, 3, m.sum()), 0, height - 1)
    keys["octave"] = rng.choice(8, size=n, p=_LEVEL_SHARE / _LEVEL_SHARE.sum())
    keys["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    keys["size"] = 31
    keys["response"] = rng.uniform(7, 80, n).astype(np.float32)
    keys["class_id"] = -1
    desc = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    u_right = np.full(n, -1.0, np.float32)
    st = rng.random(n) < p_stereo
    u_right[st] = (keys["x"][st] - rng.uniform(1, 60, st.sum())).astype(np.float32)
    r = rng.random(n)
    occ = np.zeros(n, np.int8)
    occ[r < p_occ[0] + p_occ[1]] = 2
    occ[r < p_occ[0]] = 1
    sf = scale_factors()
    K = KITTI_K
    Tcw = _pose(rng)
    return dict(keys_un=keys, desc=desc, u_right=u_right, occ=occ, min_x=np.float32(0), max_x=np.float32(width),
                min_y=np.float32(0), max_y=np.float32(height),
                grid_inv_w=np.float32(64) / np.float32(width), grid_inv_h=np.float32(48) / np.float32(height),
                nlevels=8, scale_factors=sf, log_scale_factor=np.float32(np.log(np.float32(1.2))),
                fx=np.float32(K["fx"]), fy=np.float32(K["fy"]), cx=np.float32(K["cx"]), cy=np.float32(K["cy"]),
                bf=np.float32(K["bf"]), b=np.float32(K["bf"] / K["fx"]), Tcw=Tcw)


def projection_points(seed, frame, kind, n_points=3000, pool=0.5, noise_px=1.5, max_flip=70, p_random=0.15,
                      p_take=0.9, p_obs=0.75, rot_sigma=8.0, p_rot_random=0.2):
    """MapPoints projected into `frame`.  Each point is built from a frame
    keypoint (drawn with repetition from a pool of pool*N keypoints, so several
    points compete for one feature): world position back-projected at a random
    depth with pixel noise, descriptor = the keypoint's with U[0,max_flip] bits
    flipped (p_random: a random descriptor), source angle near the keypoint's.
    Every kind gets world positions, normals, distance bounds, octaves and angles;
    kind 0 (local map) also the precomputed track fields."""
    rng = np.random.default_rng(seed)
    keys, n = frame["keys_un"], len(frame["keys_un"])
    pool_idx = rng.choice(n, size=max(1, int(pool * n)), replace=False)
    src = pool_idx[rng.integers(0, len(pool_idx), n_points)]
    T = frame["Tcw"].astype(np.float64)
    R, t = T[:3, :3], T[:3, 3]
    Ow = -R.T @ t
    fx, fy, cx, cy = (float(frame[k]) for k in ("fx", "fy", "cx", "cy"))
    z = rng.uniform(2.0, 40.0, n_points)
    u = keys["x"][src] + rng.normal(0, noise_px, n_points)
    v = keys["y"][src] + rng.normal(0, noise_px, n_points)
    Xc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
    Xw = (Xc - t) @ R  # R^T (Xc - t)
    nb = rng.integers(0, max_flip + 1, n_points)
    desc = _flip_bits(rng, frame["desc"][src], nb)
    rnd = rng.random(n_points) < p_random
    desc[rnd] = rng.integers(0, 256, size=(rnd.sum(), 32), dtype=np.uint8)
    flags = ((rng.random(n_points) < p_take).astype(np.uint8) | ((rng.random(n_points) < p_obs).astype(np.uint8) << 1))
    ang = (keys["angle"][src] + rng.normal(0, rot_sigma, n_points)) % 360.0
    rr = rng.random(n_points) < p_rot_random
    ang[rr] = rng.uniform(0, 360, rr.sum())
    sf = frame["scale_factors"].astype(np.float64)
    oct_ = np.clip(keys["octave"][src] + rng.integers(-1, 2, n_points), 0, 7).astype(np.int32)
    dist = np.linalg.norm(Xw - Ow, axis=1)
    dmax = dist * sf[oct_] * rng.uniform(0.9, 1.1, n_points)
    dmin = dmax / sf[7]
    far = rng.random(n_points) < 0.05
    dmax[far] *= 0.3
    pts = dict(kind=kind, desc=desc, flags=flags, pos=Xw.astype(np.float32),
               dist_minmax=np.stack([dmin, dmax], 1).astype(np.float32), angle=ang.astype(np.float32),
               octave=oct_)
    nrm = (Xw - Ow) / dist[:, None] + rng.normal(0, 0.3, (n_points, 3))
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    pts["normal"] = nrm.astype(np.float32)
    if kind == 0:
        track = np.zeros((n_points, 4), np.float32)
        track[:, 0] = u
        track[:, 1] = v
        track[:, 2] = u - float(frame["bf"]) / z
        track[:, 3] = np.where(rng.random(n_points) < 0.5, 0.9995, 0.99)
        pts["track"] = track
        pts["track_level"] = oct_.copy()
    return pts


# --------------------------------------------------------------- PoseOptimization
def pose_problem(seed, n=1000, p_stereo=0.6, outlier_frac=0.1, rot_sigma=0.01, t_sigma=0.05, width=1241,
                 height=376, scale_factor=1.2, nlevels=8):
    """A frame's PoseOptimization input: n MapPoint matches (feature order), KITTI intrinsics,
    observations with pixel noise sigma = scale[octave], stereo ur for p_stereo of them, a
    fraction of gross outliers (+/-20..60 px), and the initial Tcw perturbed from the truth."""
    rng = np.random.default_rng(seed)
    K = KITTI_K
    sf = scale_factors(scale_factor, nlevels).astype(np.float64)
    Ttrue = _pose(rng, 0.05, 0.5).astype(np.float64)
    u = rng.uniform(5, width - 5, n)
    v = rng.uniform(5, height - 5, n)
    z = rng.uniform(2.0, 40.0, n)
    Xc = np.stack([(u - K["cx"]) * z / K["fx"], (v - K["cy"]) * z / K["fy"], z], 1)
    R, t = Ttrue[:3, :3], Ttrue[:3, 3]
    Xw = (Xc - t) @ R
    octv = rng.choice(nlevels, size=n, p=_LEVEL_SHARE[:nlevels] / _LEVEL_SHARE[:nlevels].sum())
    sig = sf[octv]
    obs = np.zeros((n, 3))
    obs[:, 0] = u + rng.normal(0, 1, n) * sig
    obs[:, 1] = v + rng.normal(0, 1, n) * sig
    st = rng.random(n) < p_stereo
    obs[:, 2] = np.where(st, u - K["bf"] / z + rng.normal(0, 1, n) * sig, -1.0)
    bad = rng.random(n) < outlier_frac
    off = rng.uniform(20, 60, (bad.sum(), 2)) * rng.choice([-1, 1], (bad.sum(), 2))
    obs[bad, 0] += off[:, 0]
    obs[bad, 1] += off[:, 1]
    obs[bad & st, 2] += off[st[bad], 0]
    T0 = Ttrue.copy()
    T0[:3, :3] = _rot_small(rng, rot_sigma) @ R
    T0[:3, 3] = t + rng.normal(0, t_sigma, 3)
    inv_s2 = (1.0 / (sig * sig)).astype(np.float32)
    return dict(obs=obs.astype(np.float32), Xw=Xw.astype(np.float32), inv_sigma2=inv_s2, fx=np.float32(K["fx"]),
                fy=np.float32(K["fy"]), cx=np.float32(K["cx"]), cy=np.float32(K["cy"]), bf=np.float32(K["bf"]),
                Tcw=T0.astype(np.float32), Ttrue=Ttrue.astype(np.float32), is_outlier=bad)


# --------------------------------------------------------------- SearchForTriangulation
def triangulation_problem(seed, n1=1500, n2=1500, n_true=700, n_nodes=100, noise_bits=20, p_mp=0.35,
                          p_stereo=0.6, baseline=(0.8, 0.0, 0.3), width=1241, height=376):
    """Two KeyFrames observing a shared scene: n_true features of KF1 have a true correspondence in
    KF2 (same FeatureVector node, descriptor with noise bits flipped, pixel noise), the rest are
    random.  F12 = K^-T [t12]x R12 K^-1 as LocalMapping::ComputeF12 (src/LocalMapping.cc:672-690)."""
    rng = np.random.default_rng(seed)
    K = KITTI_K
    Km = np.array([[K["fx"], 0, K["cx"]], [0, K["fy"], K["cy"]], [0, 0, 1]])
    T1 = _pose(rng, 0.02, 0.2).astype(np.float64)
    T2 = T1.copy()
    T2[:3, :3] = _rot_small(rng, 0.03) @ T1[:3, :3]
    T2[:3, 3] = T1[:3, 3] - T2[:3, :3] @ np.array(baseline, np.float64) @ np.eye(3)
    from ._lib import KEYPOINT_DTYPE

    def keys(n):
        k = np.zeros(n, KEYPOINT_DTYPE)
        k["x"] = rng.uniform(0, width - 1, n)
        k["y"] = rng.uniform(0, height - 1, n)
        k["octave"] = rng.choice(8, size=n, p=_LEVEL_SHARE / _LEVEL_SHARE.sum())
        k["angle"] = rng.uniform(0, 360, n)
        k["size"] = 31
        k["class_id"] = -1
        return k

    k1, k2 = keys(n1), keys(n2)
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    d2 = rng.integers(0, 256, (n2, 32), dtype=np.uint8)
    node1 = rng.integers(0, n_nodes, n1)
    node2 = rng.integers(0, n_nodes, n2)
    i1 = rng.choice(n1, n_true, replace=False)
    i2 = rng.choice(n2, n_true, replace=False)
    # true 3D points seen by KF1 at its keypoints, reprojected into KF2
    z = rng.uniform(3, 40, n_true)
    Xc1 = np.stack([(k1["x"][i1] - K["cx"]) * z / K["fx"], (k1["y"][i1] - K["cy"]) * z / K["fy"], z], 1)
    Xw = (Xc1 - T1[:3, 3]) @ T1[:3, :3]
    Xc2 = Xw @ T2[:3, :3].T + T2[:3, 3]
    u2 = K["fx"] * Xc2[:, 0] / Xc2[:, 2] + K["cx"] + rng.normal(0, 0.7, n_true)
    v2 = K["fy"] * Xc2[:, 1] / Xc2[:, 2] + K["cy"] + rng.normal(0, 0.7, n_true)
    k2["x"][i2], k2["y"][i2] = u2, v2
    k2["octave"][i2] = k1["octave"][i1]
    k2["angle"][i2] = np.mod(k1["angle"][i1] - 10 + rng.normal(0, 3, n_true), 360)
    d2[i2] = _flip_bits(rng, d1[i1], rng.integers(0, noise_bits + 1, n_true))
    node2[i2] = node1[i1]
    ids = np.sort(rng.choice(10 ** 6, n_nodes, replace=False)).astype(np.uint32)

    def side(kp, desc, node):
        order = np.argsort(node, kind="stable")
        counts = np.bincount(node, minlength=n_nodes)
        present = counts > 0
        off = np.concatenate([[0], np.cumsum(counts[present])]).astype(np.int32)
        n = len(kp)
        ur = np.where(rng.random(n) < p_stereo, kp["x"] - rng.uniform(1, 60, n), -1.0).astype(np.float32)
        return dict(keys_un=kp, desc=desc, u_right=ur, has_mp=(rng.random(n) < p_mp).astype(np.uint8),
                    node_id=ids[present], node_off=off, feat=order.astype(np.int32))

    R1, t1, R2, t2 = T1[:3, :3], T1[:3, 3], T2[:3, :3], T2[:3, 3]
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    F12 = np.linalg.inv(Km).T @ tx @ R12 @ np.linalg.inv(Km)
    sf = scale_factors()
    return dict(kf1=side(k1, d1, node1), kf2=side(k2, d2, node2), F12=F12.astype(np.float32),
                C1w=(-R1.T @ t1).astype(np.float32), T2w=T2.astype(np.float32), fx=np.float32(K["fx"]),
                fy=np.float32(K["fy"]), cx=np.float32(K["cx"]), cy=np.float32(K["cy"]), scale_factors2=sf,
                level_sigma2_2=(sf * sf).astype(np.float32), true_pairs=(i1, i2))
