"""Host-side mirror of the reference's hot-path classes over liborbx.so.

Names, argument meaning and error behaviour follow the reference:

* ``ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)``
  (include/ORBextractor.h:77) with ``__call__(image, mask)`` ==
  ``operator()`` (src/ORBextractor.cc:1138-1211), ``GetLevels``,
  ``GetScaleFactor(s)``, ``GetInverseScaleFactors``, ``GetScaleSigmaSquares``,
  ``GetInverseScaleSigmaSquares`` and ``mvImagePyramid``.
* ``ORBmatcher.DescriptorDistance`` (src/ORBmatcher.cc:1844-1860), batched.
* ``compute_stereo_matches`` == ``Frame::ComputeStereoMatches``
  (src/Frame.cc:547-788).
* ``ORBmatcher.SearchByBoW`` (src/ORBmatcher.cc:175-325, 589-736).
* ``Optimizer.LocalBundleAdjustment`` (src/Optimizer.cc:530-885) on an
  explicit problem (cameras, points, observations) gathered like the
  reference gathers it from the covisibility graph.

Every result is computed by the HIP kernels; this module only moves bytes.
"""
import contextlib
import ctypes as C

import numpy as np

from . import _lib
from ._lib import KEYPOINT_DTYPE, check, ptr

TH_HIGH = 100  # src/ORBmatcher.cc:37
TH_LOW = 50    # src/ORBmatcher.cc:38
HISTO_LENGTH = 30  # src/ORBmatcher.cc:39


class ORBextractor:
    """GPU ORB extractor with the reference constructor signature."""

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device=0):
        L = _lib.lib()
        self.params = _lib.ExtractorParams(int(nfeatures), float(scaleFactor), int(nlevels), int(iniThFAST),
                                           int(minThFAST))
        h = C.c_void_p()
        check(L.orbx_extractor_create(C.byref(self.params), int(device), C.byref(h)), "orbx_extractor_create")
        self._h = h
        self.nfeatures = int(nfeatures)
        self.scaleFactor = float(scaleFactor)
        self.nlevels = int(nlevels)
        self.device = int(device)
        n = self.nlevels
        self._tables = [np.zeros(n, np.float32) for _ in range(4)]
        check(L.orbx_extractor_scale_tables(h, *[ptr(t) for t in self._tables]), "orbx_extractor_scale_tables")
        self._last_shape = None

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().orbx_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- reference accessors (include/ORBextractor.h:82-104)
    def GetLevels(self):
        return _lib.lib().orbx_extractor_get_levels(self._h)

    def GetScaleFactor(self):
        return self.scaleFactor

    def GetScaleFactors(self):
        return self._tables[0].copy()

    def GetInverseScaleFactors(self):
        return self._tables[1].copy()

    def GetScaleSigmaSquares(self):
        return self._tables[2].copy()

    def GetInverseScaleSigmaSquares(self):
        return self._tables[3].copy()

    def max_keypoints(self, width, height):
        n = _lib.lib().orbx_extractor_max_keypoints(self._h, int(width), int(height))
        if n < 0:
            check(n, "orbx_extractor_max_keypoints")
        return n

    # --- ORBextractor::operator()
    def __call__(self, image, mask=None):
        """Returns (keypoints structured array [cv::KeyPoint layout], descriptors uint8[n,32] or None).

        ``mask`` is accepted and ignored, as in the reference."""
        if image is None or getattr(image, "size", 0) == 0:
            return np.zeros(0, KEYPOINT_DTYPE), None
        img = np.asarray(image)
        assert img.dtype == np.uint8 and img.ndim == 2, "image must be CV_8UC1"  # src/ORBextractor.cc:1146
        h, w = img.shape
        if img.strides[1] != 1:
            img = np.ascontiguousarray(img)
        cap = self.max_keypoints(w, h)
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        check(_lib.lib().orbx_extract(self._h, ptr(img), w, h, img.strides[0], ptr(kps), cap, ptr(desc), C.byref(n)),
              "orbx_extract")
        self._last_shape = (w, h)
        n = n.value
        if n == 0:
            return kps[:0].copy(), None  # descriptors.release(), src/ORBextractor.cc:1163-1164
        return kps[:n].copy(), desc[:n].copy()

    @property
    def mvImagePyramid(self):
        return [self.pyramid_level(l) for l in range(self.nlevels)]

    def pyramid_level(self, level, image=0):
        L = _lib.lib()
        w, h = C.c_int(0), C.c_int(0)
        check(L.orbx_pyramid_level(self._h, image, level, None, 0, C.byref(w), C.byref(h)), "orbx_pyramid_level")
        out = np.zeros((h.value, w.value), np.uint8)
        check(L.orbx_pyramid_level(self._h, image, level, ptr(out), w.value, C.byref(w), C.byref(h)),
              "orbx_pyramid_level")
        return out

    # --- device batch API (inputs/outputs are torch CUDA tensors)
    def extract_batch_device(self, images, kps, desc, counts, stream=None):
        """images: uint8 [n,H,W] device tensor; kps: uint8 [n,cap,28]; desc: uint8 [n,cap,32]; counts: int32 [n]."""
        n, h, w = images.shape
        cap = kps.shape[1]
        check(_lib.lib().orbx_extract_batch_device(self._h, n, ptr(images), w, h, h * w, ptr(kps), ptr(desc),
                                                   ptr(counts), cap, _stream_ptr(stream, True)),
              "orbx_extract_batch_device")

    def stereo_frames_device(self, images, kps, desc, counts, bf, baseline, uright, depth, nmatches, stream=None):
        """images: uint8 [2n,H,W] ordered L0,R0,L1,R1...; uright/depth: float32 [n,cap]; nmatches: int32 [n]."""
        n2, h, w = images.shape
        cap = kps.shape[1]
        check(_lib.lib().orbx_stereo_frames_device(self._h, n2 // 2, ptr(images), w, h, h * w, ptr(kps), ptr(desc),
                                                   ptr(counts), cap, C.c_float(bf), C.c_float(baseline),
                                                   ptr(uright), ptr(depth), ptr(nmatches), _stream_ptr(stream, True)),
              "orbx_stereo_frames_device")


def _stream_ptr(stream, handle_api=False):
    """hipStream_t of a torch stream.  For the handle-owning entry points (extractor, vocabulary) NULL
    would pick the handle's own non-blocking stream, so torch's legacy default stream (cuda_stream 0) is
    passed as ORBX_STREAM_NULL to keep the caller's work on that stream ordered with the library's."""
    if stream is None:
        return None
    s = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
    if s == 0 and handle_api:
        return C.c_void_p(1)  # ORBX_STREAM_NULL
    return C.c_void_p(s)


def compute_stereo_matches(extractor_left, extractor_right, kps_left, desc_left, kps_right, desc_right, bf,
                           baseline):
    """Frame::ComputeStereoMatches on the pyramids of the extractors' last calls.

    Returns (mvuRight float32[N], mvDepth float32[N]) with -1 for no match."""
    nL, nR = len(kps_left), len(kps_right)
    uR = np.full(nL, -1.0, np.float32)
    depth = np.full(nL, -1.0, np.float32)
    if nL == 0:
        return uR, depth
    kL = np.ascontiguousarray(kps_left, KEYPOINT_DTYPE)
    kR = np.ascontiguousarray(kps_right, KEYPOINT_DTYPE)
    dL = np.ascontiguousarray(desc_left, np.uint8)
    dR = np.ascontiguousarray(desc_right if desc_right is not None else np.zeros((0, 32), np.uint8), np.uint8)
    check(_lib.lib().orbx_stereo_match(extractor_left._h, extractor_right._h, ptr(kL), ptr(dL), nL, ptr(kR),
                                       ptr(dR), nR, C.c_float(bf), C.c_float(baseline), ptr(uR), ptr(depth)),
          "orbx_stereo_match")
    return uR, depth


def frame_stereo(extractor, image_left, image_right, bf, baseline):
    """The ORB part of Frame's stereo constructor (src/Frame.cc:62-123: ExtractORB(0/1) + ComputeStereoMatches)
    in one call through `extractor` (both images as one batch of two, one copy back).

    Returns (kps_left, desc_left, kps_right, desc_right, mvuRight, mvDepth) as ``extractor(image)`` and
    ``compute_stereo_matches`` return them (descriptors None for an empty side)."""
    L = np.asarray(image_left)
    R = np.asarray(image_right)
    assert L.dtype == np.uint8 and L.ndim == 2 and R.dtype == np.uint8 and R.shape == L.shape, "two CV_8UC1 images"
    if L.strides[1] != 1:
        L = np.ascontiguousarray(L)
    if R.strides[1] != 1:
        R = np.ascontiguousarray(R)
    h, w = L.shape
    cap = extractor.max_keypoints(w, h)
    kL, kR = np.zeros(cap, KEYPOINT_DTYPE), np.zeros(cap, KEYPOINT_DTYPE)
    dL, dR = np.zeros((cap, 32), np.uint8), np.zeros((cap, 32), np.uint8)
    uR, depth = np.full(cap, -1.0, np.float32), np.full(cap, -1.0, np.float32)
    nL, nR = C.c_int(0), C.c_int(0)
    check(_lib.lib().orbx_frame_stereo(extractor._h, ptr(L), L.strides[0], ptr(R), R.strides[0], w, h, C.c_float(bf),
                                       C.c_float(baseline), ptr(kL), ptr(dL), cap, C.byref(nL), ptr(kR), ptr(dR), cap,
                                       C.byref(nR), ptr(uR), ptr(depth)),
          "orbx_frame_stereo")
    extractor._last_shape = (w, h)
    nL, nR = nL.value, nR.value
    return (kL[:nL].copy(), dL[:nL].copy() if nL else None, kR[:nR].copy(), dR[:nR].copy() if nR else None,
            uR[:nL].copy(), depth[:nL].copy())


def compute_distinctive_descriptors(desc, obs_off, device=0):
    """MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:249-320) for a batch of MapPoints:
    desc[obs_off[p]:obs_off[p+1]] are point p's observed descriptors in mObservations order.
    Returns (best[n_points] int32, -1 where a point has no observation; mDescriptor[n_points, 32])."""
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    off = np.ascontiguousarray(obs_off, np.int32)
    n = len(off) - 1
    best = np.zeros(max(n, 1), np.int32)
    out = np.zeros((max(n, 1), 32), np.uint8)
    check(_lib.lib().orbx_distinctive_descriptors(ptr(d), ptr(off), n, ptr(best), ptr(out), int(device)),
          "orbx_distinctive_descriptors")
    return best[:n], out[:n]


def camera(K, dist_coef):
    """orbx_camera from mK (3x3) and mDistCoef (4 or 5 coefficients)."""
    d = np.asarray(dist_coef, np.float32).reshape(-1)
    cam = _lib.Camera()
    cam.K[:] = _f32(K).reshape(9).tolist()
    dd = np.zeros(5, np.float32)
    dd[:len(d)] = d
    cam.dist[:] = dd.tolist()
    cam.n_dist = len(d)
    return cam


def undistort_keypoints(keys, K, dist_coef, device=0):
    """Frame::UndistortKeyPoints (src/Frame.cc:471-506): mvKeysUn from mvKeys, mK and mDistCoef."""
    k = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    out = np.zeros(max(len(k), 1), KEYPOINT_DTYPE)
    cam = camera(K, dist_coef)
    check(_lib.lib().orbx_undistort_keypoints(ptr(k), len(k), C.byref(cam), ptr(out), int(device)),
          "orbx_undistort_keypoints")
    return out[:len(k)]


def compute_image_bounds(cols, rows, K, dist_coef, device=0):
    """Frame::ComputeImageBounds (src/Frame.cc:508-537): (mnMinX, mnMaxX, mnMinY, mnMaxY)."""
    if float(np.float32(np.asarray(dist_coef, np.float32).reshape(-1)[0])) == 0.0:
        return 0.0, float(cols), 0.0, float(rows)
    c = np.zeros(4, KEYPOINT_DTYPE)
    c["x"] = [0.0, cols, 0.0, cols]
    c["y"] = [0.0, 0.0, rows, rows]
    u = undistort_keypoints(c, K, dist_coef, device)
    return (float(min(u["x"][0], u["x"][2])), float(max(u["x"][1], u["x"][3])),
            float(min(u["y"][0], u["y"][1])), float(max(u["y"][2], u["y"][3])))


def bow_side(side):
    """dict(desc, angle, valid, node_id, node_off, feat) -> (orbx_bow_side, keep-alive arrays)."""
    arrs = dict(desc=np.ascontiguousarray(side["desc"], np.uint8),
                angle=np.ascontiguousarray(side["angle"], np.float32),
                valid=None if side.get("valid") is None else np.ascontiguousarray(side["valid"], np.uint8),
                node_id=np.ascontiguousarray(side["node_id"], np.uint32),
                node_off=np.ascontiguousarray(side["node_off"], np.int32),
                feat=np.ascontiguousarray(side["feat"], np.int32))
    s = _lib.BowSide(len(arrs["desc"]), ptr(arrs["desc"]), ptr(arrs["angle"]), ptr(arrs["valid"]),
                     len(arrs["node_id"]), ptr(arrs["node_id"]), ptr(arrs["node_off"]), ptr(arrs["feat"]))
    return s, arrs


class ORBmatcher:
    """ORBmatcher(nnratio=0.6, checkOri=True) -- include/ORBmatcher.h:47."""

    def __init__(self, nnratio=0.6, checkOri=True, device=0):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self.device = int(device)

    def SearchByBoW(self, side_a, side_b, kf_kf=False):
        """SearchByBoW(KeyFrame*, Frame&) (kf_kf=False) or SearchByBoW(KeyFrame*, KeyFrame*) (kf_kf=True).

        Sides are dicts (desc, angle, valid, node_id, node_off, feat).  Returns (match, nmatches):
        KF-F: match[i_frame] = KF feature index or -1; KF-KF: match[i_kf1] = KF2 feature index or -1."""
        A, ka = bow_side(side_a)
        B, kb = bow_side(side_b)
        nout = A.n if kf_kf else B.n
        match = np.zeros(nout, np.int32)
        n = C.c_int(0)
        fn = _lib.lib().orbx_search_by_bow_kf_kf if kf_kf else _lib.lib().orbx_search_by_bow_kf_f
        check(fn(C.byref(A), C.byref(B), C.c_float(self.mfNNratio), int(self.mbCheckOrientation), ptr(match),
                 C.byref(n), self.device), "orbx_search_by_bow")
        return match, n.value

    def SearchByProjection(self, F, vpMapPoints, th=3.0, frustum=False, viewingCosLimit=0.5):
        """SearchByProjection(Frame&, const vector<MapPoint*>&, th) -- src/ORBmatcher.cc:46-142.

        F: frame dict (synth.projection_frame layout); vpMapPoints: points dict with the track
        fields (track = mTrackProjX/Y/XR/ViewCos, track_level) or, with frustum=True, the
        isInFrustum inputs (pos, normal, dist_minmax) of Tracking::SearchLocalPoints.  Returns
        (nmatches, frame_out, point_match[, track, track_level]); frame_out[i] = point now held by
        feature i, -1 unchanged."""
        o = _run_projection(self, F, vpMapPoints, PROJ_LOCAL, th=th, frustum=frustum,
                            view_cos_limit=viewingCosLimit)
        res = (int(o["nmatches"][0]), o["frame_out"], o["point_match"])
        return res + ((o["track"], o["track_level"]) if frustum else ())

    def SearchByProjectionLastFrame(self, CurrentFrame, LastFramePoints, LastTcw, th, bMono):
        """SearchByProjection(Frame&, const Frame&, th, bMono) -- src/ORBmatcher.cc:1489-1646.
        LastFramePoints: the last frame's MapPoints (pos, desc, octave, angle, flags bit0 =
        pMP && !mvbOutlier, bit1 = Observations() > 0).  frame_out[i] = -2 where the rotation
        check reset the feature to NULL."""
        o = _run_projection(self, CurrentFrame, LastFramePoints, PROJ_LAST_FRAME, th=th, mono=bMono,
                            last_Tcw=LastTcw)
        return int(o["nmatches"][0]), o["frame_out"], o["point_match"]

    def SearchByProjectionKeyFrame(self, CurrentFrame, KFPoints, th, ORBdist):
        """SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>& sAlreadyFound, th, ORBdist) --
        src/ORBmatcher.cc:1648-1795.  KFPoints flags bit0 = pMP && !isBad() && not already found."""
        o = _run_projection(self, CurrentFrame, KFPoints, PROJ_KEYFRAME, th=th, orb_dist=ORBdist)
        return int(o["nmatches"][0]), o["frame_out"], o["point_match"]

    def Fuse(self, pKF, vpMapPoints, th=3.0):
        """The matching half of Fuse(KeyFrame*, const vector<MapPoint*>&, th) --
        src/ORBmatcher.cc:944-1054.  pKF: frame dict of the KeyFrame (bounds = its int mnMinX..);
        vpMapPoints: points dict (pos, normal, dist_minmax, desc, flags bit0 = pMP && !isBad() &&
        !IsInKeyFrame(pKF)).  Returns (nFused, bestIdx[n_points] (-1 = no fuse)); the caller applies
        Replace / AddObservation in point order (:1057-1086)."""
        o = _run_projection(self, pKF, vpMapPoints, PROJ_FUSE, th=th)
        return int(o["nmatches"][0]), o["point_match"]

    def SearchByProjectionSim3(self, pKF, Scw, vpPoints, th=10):
        """SearchByProjection(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&, vector<MapPoint*>&
        vpMatched, th) -- src/ORBmatcher.cc:327-440 (LoopClosing::ComputeSim3, src/LoopClosing.cc:504).
        pKF: frame dict of the KeyFrame (bounds = its int mnMinX.., occ[i] != 0 = vpMatched[i] on
        entry); Scw: 4x4 Sim3; vpPoints: points dict (pos, normal, dist_minmax, desc, flags bit0 =
        !isBad() && not already in vpMatched).  Returns (nmatches, frame_out, point_match);
        frame_out[i] = k: vpMatched[i] = point k, -1 unchanged."""
        F = dict(pKF)
        F["Tcw"] = np.asarray(Scw, np.float32).reshape(4, 4)
        o = _run_projection(self, F, vpPoints, PROJ_SIM3, th=float(th))
        return int(o["nmatches"][0]), o["frame_out"], o["point_match"]

    def FuseSim3(self, pKF, Scw, vpPoints, th=4.0):
        """The matching half of Fuse(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&, th,
        vector<MapPoint*>& vpReplacePoint) -- src/ORBmatcher.cc:1094-1236 (LoopClosing::SearchAndFuse).
        vpPoints flags bit0 = !isBad() && not in pKF->GetMapPoints().  Returns (nFused,
        bestIdx[n_points] (-1 = none)); the caller applies the replace / AddMapPoint block
        (:1210-1229) in point order."""
        F = dict(pKF)
        F["Tcw"] = np.asarray(Scw, np.float32).reshape(4, 4)
        o = _run_projection(self, F, vpPoints, PROJ_FUSE_SIM3, th=float(th))
        return int(o["nmatches"][0]), o["point_match"]

    def SearchForInitialization(self, F1, F2, vbPrevMatched, windowSize=10):
        """SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
        vector<int>& vnMatches12, windowSize) -- src/ORBmatcher.cc:442-587 (Tracking::
        MonocularInitialization: ORBmatcher(0.9, true), windowSize 100).  F1, F2: frame dicts
        (keys_un, desc; F2's grid fields).  Returns (nmatches, vnMatches12[N1], vbPrevMatched[N1, 2]
        updated)."""
        f1, k1 = _host_proj_frame(F1)
        f2, k2 = _host_proj_frame(F2)
        p = _lib.InitProblem()
        p.f1, p.f2 = f1, f2
        prev = np.ascontiguousarray(vbPrevMatched, np.float32).reshape(-1, 2).copy()
        assert len(prev) == f1.n
        m = np.zeros(max(1, f1.n), np.int32)
        nm = np.zeros(1, np.int32)
        p.prev_matched, p.window = ptr(prev), int(windowSize)
        p.nnratio, p.check_ori = float(self.mfNNratio), int(bool(self.mbCheckOrientation))
        p.match12, p.nmatches = ptr(m), ptr(nm)
        check(_lib.lib().orbx_search_for_initialization(C.byref(p), self.device), "orbx_search_for_initialization")
        return int(nm[0]), m[:f1.n], prev

    def SearchBySim3(self, pKF1, pKF2, pts1, pts2, s12, R12, t12, th=7.5):
        """SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12, s12, R12, t12, th)
        -- src/ORBmatcher.cc:1238-1487 (LoopClosing::ComputeSim3).  pKFj: frame dicts (Tcw = GetPose());
        ptsj: the KeyFrame's GetMapPointMatches() as per-feature arrays (desc, pos, dist_minmax, flags bit0
        = pMP && !vbAlreadyMatched && !isBad()).  Returns (nFound, match12[N1]: the KF2 feature whose
        MapPoint becomes vpMatches12[i1], -1 none)."""
        f1, k1 = _host_proj_frame(pKF1)
        f2, k2 = _host_proj_frame(pKF2)
        p = _lib.Sim3Problem()
        p.kf1, p.kf2 = f1, f2
        keep = [k1, k2]
        for j, pts in ((1, pts1), (2, pts2)):
            for k, dt in (("desc", np.uint8), ("pos", np.float32), ("dist_minmax", np.float32), ("flags", np.uint8)):
                a = np.ascontiguousarray(pts[k], dt)
                keep.append(a)
                setattr(p, "%s%d" % (k, j), ptr(a))
        p.s12, p.th = float(s12), float(th)
        p.R12[:] = _f32(R12).reshape(9).tolist()
        p.t12[:] = _f32(t12).reshape(3).tolist()
        m = np.zeros(max(1, f1.n), np.int32)
        nf = np.zeros(1, np.int32)
        p.match12, p.nfound = ptr(m), ptr(nf)
        check(_lib.lib().orbx_search_by_sim3(C.byref(p), self.device), "orbx_search_by_sim3")
        return int(nf[0]), m[:f1.n]

    def SearchForTriangulation(self, prob, bOnlyStereo=False):
        """SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo) --
        src/ORBmatcher.cc:738-925.  prob: dict(kf1, kf2 (keys_un, desc, u_right, has_mp, node_id,
        node_off, feat), F12[3,3], C1w[3], T2w[4,4], fx, fy, cx, cy (pKF2), scale_factors2,
        level_sigma2_2).  Returns (nmatches, vMatchedPairs as an [m,2] int array)."""
        p, keep = tri_problem(prob, bOnlyStereo, self.mbCheckOrientation)
        m12 = np.zeros(max(1, p.kf1.n), np.int32)
        nm = np.zeros(1, np.int32)
        p.match12, p.nmatches = ptr(m12), ptr(nm)
        check(_lib.lib().orbx_search_for_triangulation(C.byref(p), self.device), "orbx_search_for_triangulation")
        m12 = m12[:p.kf1.n]
        i = np.nonzero(m12 >= 0)[0]
        return int(nm[0]), np.stack([i, m12[i]], 1).astype(np.int64)

    @staticmethod
    def DescriptorDistance(a, b):
        """Hamming distance of 32-byte descriptors; a, b: [32] or [n,32] uint8 (computed on the GPU)."""
        import torch
        a = np.atleast_2d(np.ascontiguousarray(a, np.uint8))
        b = np.atleast_2d(np.ascontiguousarray(b, np.uint8))
        assert a.shape == b.shape and a.shape[1] == 32
        n = a.shape[0]
        da = torch.from_numpy(a).cuda()
        db = torch.from_numpy(b).cuda()
        out = torch.empty(n, dtype=torch.int32, device=da.device)
        s = torch.cuda.current_stream()
        check(_lib.lib().orbx_descriptor_distance_device(ptr(da), ptr(db), n, ptr(out), _stream_ptr(s)),
              "orbx_descriptor_distance_device")
        d = out.cpu().numpy()
        return int(d[0]) if n == 1 else d


PROJ_LOCAL, PROJ_LAST_FRAME, PROJ_KEYFRAME, PROJ_FUSE, PROJ_SIM3, PROJ_FUSE_SIM3 = 0, 1, 2, 3, 4, 5


def _f32(x):
    return np.ascontiguousarray(x, np.float32)


def proj_problem(frame, points, kind, th, nnratio=0.6, check_ori=True, mono=False, orb_dist=100, last_Tcw=None,
                 frustum=False, view_cos_limit=0.5, outputs=None):
    """Fill an orbx_proj_problem from a frame dict and a points dict (synth.projection_frame /
    projection_points layout).  Arrays may be host numpy arrays (for orbx_search_by_projection) or
    device tensors (for orbx_search_by_projection_device); the caller keeps them alive.  `outputs`
    = dict(frame_out, point_match, nmatches[, track, track_level]); numpy arrays are allocated when
    absent.  Returns (problem, outputs)."""
    n, npnt = len(frame["desc"]), len(points["desc"])
    if outputs is None:
        outputs = dict(frame_out=np.zeros(n, np.int32), point_match=np.zeros(npnt, np.int32),
                       nmatches=np.zeros(1, np.int32))
        if kind == PROJ_LOCAL:
            outputs["track"] = (np.zeros((npnt, 4), np.float32) if frustum
                                else np.ascontiguousarray(points["track"], np.float32))
            outputs["track_level"] = (np.zeros(npnt, np.int32) if frustum
                                      else np.ascontiguousarray(points["track_level"], np.int32))
    f = _lib.ProjFrame()
    f.n = n
    f.keys_un, f.desc = ptr(frame["keys_un"]), ptr(frame["desc"])
    f.u_right = ptr(frame.get("u_right"))
    f.occ = ptr(frame.get("occ"))
    for k in ("min_x", "max_x", "min_y", "max_y", "grid_inv_w", "grid_inv_h", "log_scale_factor", "fx", "fy",
              "cx", "cy", "bf", "b"):
        setattr(f, k, float(frame[k]))
    if frame.get("grid_min_x") is not None:  # a KeyFrame's grid: the Frame's float bounds
        f.grid_min_x, f.grid_min_y, f.grid_min_set = float(frame["grid_min_x"]), float(frame["grid_min_y"]), 1
    f.nlevels = int(frame["nlevels"])
    sf = np.zeros(16, np.float32)
    sf[:f.nlevels] = frame["scale_factors"][:f.nlevels]
    f.scale_factors[:] = sf.tolist()
    isg = np.zeros(16, np.float32)
    if frame.get("inv_level_sigma2") is not None:
        isg[:f.nlevels] = frame["inv_level_sigma2"][:f.nlevels]
    else:  # mvInvLevelSigma2 = 1 / (s*s) in float (ORBextractor ctor)
        isg[:f.nlevels] = np.float32(1.0) / (sf[:f.nlevels] * sf[:f.nlevels])
    f.inv_level_sigma2[:] = isg.tolist()
    f.Tcw[:] = _f32(frame["Tcw"]).reshape(16).tolist()
    p = _lib.ProjProblem()
    p.kind, p.frustum, p.f, p.n_points = int(kind), int(bool(frustum)), f, npnt
    p.desc, p.flags = ptr(points["desc"]), ptr(points["flags"])
    for k in ("pos", "normal", "dist_minmax", "angle", "octave"):
        setattr(p, k, ptr(points.get(k)))
    p.track = ptr(outputs.get("track"))
    p.track_level = ptr(outputs.get("track_level"))
    p.th, p.nnratio, p.view_cos_limit = float(th), float(nnratio), float(view_cos_limit)
    p.check_ori, p.mono, p.orb_dist = int(bool(check_ori)), int(bool(mono)), int(orb_dist)
    p.last_Tcw[:] = (_f32(last_Tcw).reshape(16) if last_Tcw is not None else np.eye(4, dtype=np.float32).reshape(16)).tolist()
    p.frame_out, p.point_match, p.nmatches = (ptr(outputs["frame_out"]), ptr(outputs["point_match"]),
                                              ptr(outputs["nmatches"]))
    return p, outputs


def _host_proj_frame(frame):
    """An orbx_proj_frame over host copies of a frame dict's arrays; returns (frame, keep-alive)."""
    fr = _host_frame(frame)
    p, _ = proj_problem(fr, dict(desc=np.zeros((0, 32), np.uint8), flags=np.zeros(0, np.uint8)), PROJ_KEYFRAME,
                        th=1.0, outputs=dict(frame_out=None, point_match=None, nmatches=None))
    return p.f, fr


def _host_points(points):
    out = dict(points)
    for k, dt in (("desc", np.uint8), ("flags", np.uint8), ("pos", np.float32), ("normal", np.float32),
                  ("dist_minmax", np.float32), ("angle", np.float32), ("octave", np.int32)):
        if points.get(k) is not None:
            out[k] = np.ascontiguousarray(points[k], dt)
    return out


def _host_frame(frame):
    out = dict(frame)
    out["keys_un"] = np.ascontiguousarray(frame["keys_un"], KEYPOINT_DTYPE)
    out["desc"] = np.ascontiguousarray(frame["desc"], np.uint8)
    if frame.get("u_right") is not None:
        out["u_right"] = np.ascontiguousarray(frame["u_right"], np.float32)
    if frame.get("occ") is not None:
        out["occ"] = np.ascontiguousarray(frame["occ"], np.int8)
    return out


def _run_projection(matcher, frame, points, kind, **kw):
    fr, pts = _host_frame(frame), _host_points(points)
    p, out = proj_problem(fr, pts, kind, nnratio=matcher.mfNNratio, check_ori=matcher.mbCheckOrientation, **kw)
    check(_lib.lib().orbx_search_by_projection(C.byref(p), matcher.device), "orbx_search_by_projection")
    return out


def tri_problem(prob, only_stereo=False, check_ori=True):
    """orbx_tri_problem from a dict whose arrays are host numpy arrays or device tensors (the caller
    keeps them alive; numpy inputs are made contiguous here and returned in `keep`).  match12 and
    nmatches are left for the caller to point at its outputs."""
    keep = []

    def arr(x, dt):
        if x is None or not isinstance(x, np.ndarray):
            return x
        a = np.ascontiguousarray(x, dt)
        keep.append(a)
        return a

    def kf(d):
        k = _lib.TriKF()
        keys = arr(d["keys_un"], KEYPOINT_DTYPE)
        k.n = len(d["desc"])
        k.keys_un, k.desc = ptr(keys), ptr(arr(d["desc"], np.uint8))
        k.u_right, k.has_mp = ptr(arr(d.get("u_right"), np.float32)), ptr(arr(d.get("has_mp"), np.uint8))
        k.n_nodes = len(d["node_id"])
        k.node_id, k.node_off = ptr(arr(d["node_id"], np.uint32)), ptr(arr(d["node_off"], np.int32))
        k.feat = ptr(arr(d["feat"], np.int32))
        return k

    p = _lib.TriProblem()
    p.kf1, p.kf2 = kf(prob["kf1"]), kf(prob["kf2"])
    p.F12[:] = _f32(prob["F12"]).reshape(9).tolist()
    p.C1w[:] = _f32(prob["C1w"]).reshape(3).tolist()
    p.T2w[:] = _f32(prob["T2w"]).reshape(16).tolist()
    for k in ("fx", "fy", "cx", "cy"):
        setattr(p, k, float(prob[k]))
    sf = np.zeros(16, np.float32)
    sg = np.zeros(16, np.float32)
    nl = len(prob["scale_factors2"])
    sf[:nl], sg[:nl] = prob["scale_factors2"], prob["level_sigma2_2"]
    p.scale_factors2[:] = sf.tolist()
    p.level_sigma2_2[:] = sg.tolist()
    p.only_stereo, p.check_ori = int(bool(only_stereo)), int(bool(check_ori))
    return p, keep


def _ba_arrays(prob):
    """Problem dict -> contiguous arrays in the orbx_ba_problem layout."""
    nc = len(prob["Tcw"])
    fixed = prob.get("fixed")
    return dict(Tcw=np.ascontiguousarray(np.asarray(prob["Tcw"], np.float32).reshape(nc, 12)),
                fixed=np.ascontiguousarray(np.zeros(nc, np.uint8) if fixed is None else fixed, np.uint8),
                intr=np.ascontiguousarray(np.asarray(prob["intr"], np.float32).reshape(nc, 5)),
                Xw=np.ascontiguousarray(np.asarray(prob["Xw"], np.float32).reshape(-1, 3)),
                edge_point=np.ascontiguousarray(prob["edge_point"], np.int32),
                edge_cam=np.ascontiguousarray(prob["edge_cam"], np.int32),
                obs=np.ascontiguousarray(np.asarray(prob["obs"], np.float32).reshape(-1, 3)),
                inv_sigma2=np.ascontiguousarray(prob["inv_sigma2"], np.float32))


class Optimizer:
    """Optimizer::LocalBundleAdjustment (include/Optimizer.h:46) on the GPU.

    The solver handle keeps device buffers between calls (the local mapping
    thread runs one LocalBA per new keyframe)."""

    def __init__(self, device=0, priority=0, cu_mask=None):
        """priority: HIP stream priority of the handle's stream (0 default, < 0 higher; see
        orbx_ba_create_priority) -- the LocalMapping thread's handle runs high beside extraction.
        cu_mask: optional sequence of 32-bit words restricting the handle's stream to a CU set
        (orbx_ba_create_masked; the priority is then the default)."""
        h = C.c_void_p()
        if cu_mask is not None:
            m = np.ascontiguousarray(cu_mask, np.uint32)
            check(_lib.lib().orbx_ba_create_masked(int(device), ptr(m), len(m), C.byref(h)), "orbx_ba_create_masked")
        else:
            check(_lib.lib().orbx_ba_create_priority(int(device), int(priority), C.byref(h)), "orbx_ba_create_priority")
        self._h = h
        self.device = int(device)
        f = C.POINTER(C.c_int)()
        check(_lib.lib().orbx_ba_stop_flag(h, C.byref(f)), "orbx_ba_stop_flag")
        self._stop = f  # the handle's pinned flag (the device polls it without registration)

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().orbx_ba_destroy(self._h)
            self._h = None
            self._stop = None

    def set_debug_options(self, **kw):
        """Test options of this solver handle (include/orbx_debug.h, orbx_ba_debug_options: ldlt,
        nan_trial, raise_stop_after, trace, fused_ctl); no arguments restore the production defaults."""
        o = _lib.BaDebugOptions(0, -1, -1, 0)
        for k, v in kw.items():
            if k not in dict(o._fields_):
                raise TypeError("unknown LocalBA debug option %r" % k)
            setattr(o, k, int(v))
        check(_lib.lib().orbx_debug_ba_options(self._h, C.byref(o)), "orbx_debug_ba_options")

    @contextlib.contextmanager
    def debug_options(self, **kw):
        self.set_debug_options(**kw)
        try:
            yield self
        finally:
            self.set_debug_options()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def PoseOptimization(self, frame):
        """Optimizer::PoseOptimization(Frame*) -- src/Optimizer.cc:287-528.  frame: dict(obs[n,3]
        (u, v, ur; ur < 0 = monocular), Xw[n,3], inv_sigma2[n], fx, fy, cx, cy, bf, Tcw[4,4]) with
        one row per feature that has a MapPoint, in feature order.  Returns (nGood, Tcw[4,4],
        outlier[n] (mvbOutlier), iterations[4])."""
        pr = dict(frame)
        pr["obs"] = np.ascontiguousarray(frame["obs"], np.float32).reshape(-1, 3)
        pr["Xw"] = np.ascontiguousarray(frame["Xw"], np.float32).reshape(-1, 3)
        pr["inv_sigma2"] = np.ascontiguousarray(frame["inv_sigma2"], np.float32)
        p, out = pose_problem_struct(pr)
        check(_lib.lib().orbx_pose_optimization(C.byref(p), self.device), "orbx_pose_optimization")
        return int(out["ngood"][0]), out["Tcw_out"], out["outlier"][:len(pr["obs"])], out["iterations"]

    def LocalBundleAdjustment(self, prob, stop=False):
        """prob: dict(Tcw[n,12], fixed[n], intr[n,5] fx,fy,cx,cy,bf, Xw[m,3], edge_point, edge_cam,
        obs[e,3] (u, v, ur; ur<0 mono), inv_sigma2[e]).  ``stop`` mirrors *pbStopFlag: a bool, or
        a one-element int32 array another thread may set while the call runs (the LM loop polls
        it between iterations and trials, src/Optimizer.cc:749-762).

        Returns dict(Tcw, Xw, edge_outlier, Tcw_d, Xw_d, iterations, trials, chi2)."""
        a = _ba_arrays(prob)
        nc, npt, ne = len(a["Tcw"]), len(a["Xw"]), len(a["edge_point"])
        P = _lib.BaProblem(nc, ptr(a["Tcw"]), ptr(a["fixed"]), ptr(a["intr"]), npt, ptr(a["Xw"]), ne,
                           ptr(a["edge_point"]), ptr(a["edge_cam"]), ptr(a["obs"]), ptr(a["inv_sigma2"]))
        # (every output element is written by the call: no zero fill)
        out = dict(Tcw=np.empty((nc, 12), np.float32), Xw=np.empty((npt, 3), np.float32),
                   edge_outlier=np.empty(ne, np.uint8), Tcw_d=np.empty((nc, 12)), Xw_d=np.empty((npt, 3)))
        R = _lib.BaResult(ptr(out["Tcw"]), ptr(out["Xw"]), ptr(out["edge_outlier"]), ptr(out["Tcw_d"]),
                          ptr(out["Xw_d"]))
        if isinstance(stop, np.ndarray):
            if stop.dtype != np.int32 or stop.size != 1 or not stop.flags.c_contiguous:
                raise ValueError("stop flag array must be one contiguous int32")
            flag = C.c_void_p(stop.ctypes.data)
        else:
            self._stop[0] = 1 if stop else 0
            flag = C.cast(self._stop, C.c_void_p)
        check(_lib.lib().orbx_ba_run(self._h, C.byref(P), C.byref(R), flag), "orbx_ba_run")
        out.update(iterations=tuple(R.iterations), trials=R.trials, chi2=tuple(R.chi2))
        return out

    def LocalBundleAdjustmentMany(self, probs, stop=False):
        """K independent problems through one batched LM loop (orbx_ba_run_many); returns the
        list of result dicts, each bit-identical to LocalBundleAdjustment on that problem."""
        K = len(probs)
        keep, outs = [], []
        Ps, Rs = (_lib.BaProblem * K)(), (_lib.BaResult * K)()
        for k, prob in enumerate(probs):
            a = _ba_arrays(prob)
            nc, npt, ne = len(a["Tcw"]), len(a["Xw"]), len(a["edge_point"])
            Ps[k] = _lib.BaProblem(nc, ptr(a["Tcw"]), ptr(a["fixed"]), ptr(a["intr"]), npt, ptr(a["Xw"]), ne,
                                   ptr(a["edge_point"]), ptr(a["edge_cam"]), ptr(a["obs"]), ptr(a["inv_sigma2"]))
            out = dict(Tcw=np.empty((nc, 12), np.float32), Xw=np.empty((npt, 3), np.float32),
                       edge_outlier=np.empty(ne, np.uint8), Tcw_d=np.empty((nc, 12)), Xw_d=np.empty((npt, 3)))
            Rs[k] = _lib.BaResult(ptr(out["Tcw"]), ptr(out["Xw"]), ptr(out["edge_outlier"]), ptr(out["Tcw_d"]),
                                  ptr(out["Xw_d"]))
            keep.append(a)
            outs.append(out)
        self._stop[0] = 1 if stop else 0
        check(_lib.lib().orbx_ba_run_many(self._h, K, Ps, Rs, C.cast(self._stop, C.c_void_p)), "orbx_ba_run_many")
        for k in range(K):
            outs[k].update(iterations=tuple(Rs[k].iterations), trials=Rs[k].trials, chi2=tuple(Rs[k].chi2))
        return outs


def pose_problem_struct(prob, outputs=None):
    """orbx_pose_problem from a dict (host numpy or device tensors); outputs allocated on the host
    when absent.  Returns (struct, outputs)."""
    n = len(prob["obs"])
    if outputs is None:
        outputs = dict(Tcw_out=np.zeros((4, 4), np.float32), outlier=np.zeros(max(n, 1), np.uint8),
                       ngood=np.zeros(1, np.int32), iterations=np.zeros(4, np.int32))
    p = _lib.PoseProblem()
    p.n = n
    p.obs, p.Xw, p.inv_sigma2 = ptr(prob["obs"]), ptr(prob["Xw"]), ptr(prob["inv_sigma2"])
    for k in ("fx", "fy", "cx", "cy", "bf"):
        setattr(p, k, float(prob[k]))
    p.Tcw[:] = _f32(prob["Tcw"]).reshape(16).tolist()
    p.Tcw_out, p.outlier, p.ngood = ptr(outputs["Tcw_out"]), ptr(outputs["outlier"]), ptr(outputs["ngood"])
    p.iterations = ptr(outputs.get("iterations"))
    return p, outputs


class PnPsolver:
    """PnPsolver (include/PnPsolver.h:66-77) over orbx_pnp_*.

    Correspondences are given in the constructor's gather order
    (src/PnPsolver.cc:67-125): world points, undistorted keypoints and
    mvLevelSigma2[octave] of the matched keypoints.  Like the reference the
    constructor applies SetRansacParameters() with its defaults."""

    def __init__(self, p3d, p2d, sigma2, fx, fy, cx, cy, device=0):
        self.p3d = np.ascontiguousarray(p3d, np.float32).reshape(-1, 3)
        self.p2d = np.ascontiguousarray(p2d, np.float32).reshape(-1, 2)
        self.sigma2 = np.ascontiguousarray(sigma2, np.float32)
        self.n = len(self.p3d)
        self.intr = (float(fx), float(fy), float(cx), float(cy))
        self.device = int(device)
        self._h = None
        self.SetRansacParameters()

    def SetRansacParameters(self, probability=0.99, minInliers=8, maxIterations=300, minSet=4, epsilon=0.4,
                            th2=5.991):
        """src/PnPsolver.cc:136-179.  May be called at any time: after iterate() the derived parameters
        and maxError are recomputed in place and the iteration count / best set are kept, as in the
        reference."""
        prm = _lib.PnpParams(float(probability), int(minInliers), int(maxIterations), int(minSet), float(epsilon),
                             float(th2))
        if self._h:
            check(_lib.lib().orbx_pnp_set_ransac_parameters(self._h, ptr(self.sigma2), C.byref(prm)),
                  "orbx_pnp_set_ransac_parameters")
            self.min_set = int(minSet)
            a, b, c = C.c_int(), C.c_int(), C.c_float()
            check(_lib.lib().orbx_pnp_get_params(self._h, C.byref(a), C.byref(b), C.byref(c)), "orbx_pnp_get_params")
            self.min_inliers, self.max_its, self.epsilon = a.value, b.value, c.value
            return
        self.close()
        prob = _lib.PnpProblem(self.n, ptr(self.p3d), ptr(self.p2d), ptr(self.sigma2), *self.intr)
        prm = _lib.PnpParams(float(probability), int(minInliers), int(maxIterations), int(minSet), float(epsilon),
                             float(th2))
        h = C.c_void_p()
        check(_lib.lib().orbx_pnp_create(C.byref(prob), C.byref(prm), self.device, C.byref(h)), "orbx_pnp_create")
        self._h = h
        self.min_set = int(minSet)
        a, b, c = C.c_int(), C.c_int(), C.c_float()
        check(_lib.lib().orbx_pnp_get_params(h, C.byref(a), C.byref(b), C.byref(c)), "orbx_pnp_get_params")
        self.min_inliers, self.max_its, self.epsilon = a.value, b.value, c.value
        self._done = 0

    @classmethod
    def create_many(cls, problems, probability=0.99, minInliers=8, maxIterations=300, minSet=4, epsilon=0.4,
                    th2=5.991, device=0):
        """len(problems) solvers (dicts p3d, p2d, sigma2, fx, fy, cx, cy) with one parameter set, created by
        one orbx_pnp_create_many call (one upload for all correspondences)."""
        n = len(problems)
        objs, structs = [], (_lib.PnpProblem * max(n, 1))()
        for i, P in enumerate(problems):
            o = cls.__new__(cls)
            o.p3d = np.ascontiguousarray(P["p3d"], np.float32).reshape(-1, 3)
            o.p2d = np.ascontiguousarray(P["p2d"], np.float32).reshape(-1, 2)
            o.sigma2 = np.ascontiguousarray(P["sigma2"], np.float32)
            o.n = len(o.p3d)
            o.intr = (float(P["fx"]), float(P["fy"]), float(P["cx"]), float(P["cy"]))
            o.device = int(device)
            o._h = None
            structs[i] = _lib.PnpProblem(o.n, ptr(o.p3d), ptr(o.p2d), ptr(o.sigma2), *o.intr)
            objs.append(o)
        prm = _lib.PnpParams(float(probability), int(minInliers), int(maxIterations), int(minSet), float(epsilon),
                             float(th2))
        hs = (C.c_void_p * max(n, 1))()
        check(_lib.lib().orbx_pnp_create_many(structs, n, C.byref(prm), int(device), hs), "orbx_pnp_create_many")
        for o, h in zip(objs, hs):
            o._h = C.c_void_p(h)
            o.min_set = int(minSet)
            a, b, c = C.c_int(), C.c_int(), C.c_float()
            check(_lib.lib().orbx_pnp_get_params(o._h, C.byref(a), C.byref(b), C.byref(c)), "orbx_pnp_get_params")
            o.min_inliers, o.max_its, o.epsilon = a.value, b.value, c.value
            o._done = 0
        return objs

    @classmethod
    def create_many_device(cls, p3d, p2d, sigma2, offsets, intr, probability=0.99, minInliers=8,
                           maxIterations=300, minSet=4, epsilon=0.4, th2=5.991, device=0):
        """Solvers over device-resident correspondences: p3d [M,3], p2d [M,2], sigma2 [M] float32 device
        tensors holding the problems back to back (problem i = rows offsets[i]..offsets[i+1]-1), intr [n,4]
        (fx, fy, cx, cy) on the host -- one orbx_pnp_create_many_device call."""
        offs = np.ascontiguousarray(offsets, np.int32)
        it = np.ascontiguousarray(intr, np.float32).reshape(-1, 4)
        n = len(offs) - 1
        prm = _lib.PnpParams(float(probability), int(minInliers), int(maxIterations), int(minSet), float(epsilon),
                             float(th2))
        hs = (C.c_void_p * max(n, 1))()
        check(_lib.lib().orbx_pnp_create_many_device(C.c_void_p(p3d.data_ptr()), C.c_void_p(p2d.data_ptr()),
                                                     C.c_void_p(sigma2.data_ptr()), ptr(offs), ptr(it), n,
                                                     C.byref(prm), int(device), hs), "orbx_pnp_create_many_device")
        objs = []
        for i in range(n):
            o = cls.__new__(cls)
            o.n = int(offs[i + 1] - offs[i])
            o.device = int(device)
            o._h = C.c_void_p(hs[i])
            o.min_set = int(minSet)
            a, b, c = C.c_int(), C.c_int(), C.c_float()
            check(_lib.lib().orbx_pnp_get_params(o._h, C.byref(a), C.byref(b), C.byref(c)), "orbx_pnp_get_params")
            o.min_inliers, o.max_its, o.epsilon = a.value, b.value, c.value
            o._done = 0
            objs.append(o)
        return objs

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().orbx_pnp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def iterate(self, nIterations, rng):
        """rng: a rand() stream with peek(k)/advance(k) (e.g. glibc_rand.GlibcRand(1), the
        unseeded process rand() of the reference).  Returns (Tcw[4,4] or None, bNoMore,
        vbInliers[n] bool, nInliers); the stream advances by exactly what was drawn."""
        need = self.min_set * max(self.max_its - self._done, int(nIterations), 0)
        vals = np.ascontiguousarray(rng.peek(need), np.int32) if need else np.zeros(0, np.int32)
        used, nm, ni, found = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        T = np.zeros(16, np.float32)
        inl = np.zeros(max(self.n, 1), np.uint8)
        check(_lib.lib().orbx_pnp_iterate(self._h, int(nIterations), ptr(vals), len(vals), C.byref(used),
                                          C.byref(nm), ptr(T), ptr(inl), C.byref(ni), C.byref(found)),
              "orbx_pnp_iterate")
        rng.advance(used.value)
        self._done += used.value // self.min_set
        return (T.reshape(4, 4) if found.value else None), bool(nm.value), inl[:self.n].astype(bool), ni.value


def _rand_state(rng):
    st = _lib.RandState()
    w = rng.state_words()
    for k in range(34):
        st.r[k] = w[k]
    st.i = 34
    return st


def _rand_restore(rng, st):
    i = st.i
    rng.set_state_words([st.r[(i - 34 + k) % 34] for k in range(34)])


def _pnp_outputs(solvers, res, inl):
    out = []
    for s, r, b in zip(solvers, res, inl):
        s._done += r.used // s.min_set
        T = np.ctypeslib.as_array(r.Tcw).reshape(4, 4).copy() if r.found else None
        out.append((T, bool(r.no_more), b[:s.n].astype(bool), int(r.n_inliers)))
    return out


def pnp_iterate_candidates(solvers, nIterations, rng, raw_results=None):
    """Tracking::Relocalization's candidate loop (src/Tracking.cc:1738-1757) in one call:
    solvers[0].iterate(n), solvers[1].iterate(n), ... on the shared stream `rng` (GlibcRand),
    stopping after the first that returns a pose.  Returns (stopped, [(Tcw|None, bNoMore,
    vbInliers, nInliers)] for solvers[0..stopped]); rng advances by exactly what was drawn.
    raw_results: optional list that receives every solver's orbx_pnp_result (tests)."""
    n = len(solvers)
    hs = (C.c_void_p * max(n, 1))(*[s._h for s in solvers])
    res = (_lib.PnpResult * max(n, 1))()
    inl = [np.zeros(max(s.n, 1), np.uint8) for s in solvers]
    ip = (C.c_void_p * max(n, 1))(*[ptr(b) for b in inl])
    st = _rand_state(rng)
    stopped = C.c_int()
    check(_lib.lib().orbx_pnp_iterate_candidates(hs, n, int(nIterations), C.byref(st), res, ip, C.byref(stopped)),
          "orbx_pnp_iterate_candidates")
    _rand_restore(rng, st)
    if raw_results is not None:
        raw_results.extend(res[i] for i in range(n))
    k = min(stopped.value + 1, n)
    return stopped.value, _pnp_outputs(solvers[:k], res[:k], inl[:k])


def pnp_iterate_many(solvers, nIterations, rngs):
    """iterate(n) on independent solvers, rngs[i] its own GlibcRand stream; one batched call."""
    n = len(solvers)
    hs = (C.c_void_p * max(n, 1))(*[s._h for s in solvers])
    res = (_lib.PnpResult * max(n, 1))()
    inl = [np.zeros(max(s.n, 1), np.uint8) for s in solvers]
    ip = (C.c_void_p * max(n, 1))(*[ptr(b) for b in inl])
    sts = [_rand_state(r) for r in rngs]
    sp = (C.c_void_p * max(n, 1))(*[C.addressof(x) for x in sts])
    check(_lib.lib().orbx_pnp_iterate_many(hs, n, int(nIterations), sp, res, ip), "orbx_pnp_iterate_many")
    for r, x in zip(rngs, sts):
        _rand_restore(r, x)
    return _pnp_outputs(solvers, res[:n], inl)


class ORBVocabulary:
    """DBoW2 TemplatedVocabulary<FORB> (include/ORBVocabulary.h) on the GPU:
    loadFromTextFile (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1420) and
    transform(features, BowVector, FeatureVector, levelsup) (:1125-1196) over liborbx.so."""

    def __init__(self, device=0):
        self.device = device
        self._h = None

    def loadFromText(self, text):
        """The text of a vocabulary file (ORBvoc.txt format).  Returns True like the reference."""
        self.close()
        raw = text.encode() if isinstance(text, str) else bytes(text)
        h = C.c_void_p()
        check(_lib.lib().orbx_voc_load_text(raw, len(raw), self.device, C.byref(h)), "orbx_voc_load_text")
        self._h = h
        info = np.zeros(6, np.int32)
        check(_lib.lib().orbx_voc_info(h, ptr(info)), "orbx_voc_info")
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words = (int(x) for x in info)
        return True

    def loadFromTextFile(self, path):
        with open(path, "rb") as f:
            return self.loadFromText(f.read())

    def transform_sets(self, desc_sets, levelsup=4):
        """Batch form: list of (n_i, 32) uint8 descriptor arrays -> list of
        (bow_words, bow_values, fv_nodes, fv_off, fv_feat) per set (std::map order)."""
        sets = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in desc_sets]
        off = np.zeros(len(sets) + 1, np.int32)
        off[1:] = np.cumsum([len(d) for d in sets])
        total = int(off[-1])
        desc = np.concatenate(sets) if total else np.zeros((1, 32), np.uint8)
        m = max(total, 1)
        bw, bv = np.zeros(m, np.uint32), np.zeros(m, np.float64)
        fn, fo, ff = np.zeros(m, np.uint32), np.zeros(m + len(sets), np.int32), np.zeros(m, np.int32)
        nb, nf = np.zeros(len(sets), np.int32), np.zeros(len(sets), np.int32)
        check(_lib.lib().orbx_voc_transform(self._h, ptr(desc), ptr(off), len(sets), int(levelsup), ptr(bw), ptr(bv),
                                            ptr(nb), ptr(fn), ptr(fo), ptr(ff), ptr(nf)), "orbx_voc_transform")
        out = []
        for s in range(len(sets)):
            o, b, q = int(off[s]), int(nb[s]), int(nf[s])
            foff = fo[o + s:o + s + q + 1].copy()
            out.append((bw[o:o + b].copy(), bv[o:o + b].copy(), fn[o:o + q].copy(), foff,
                        ff[o:o + int(foff[-1] if q else 0)].copy()))
        return out

    def transform(self, desc, levelsup=4):
        """(BowVector as (words, values), FeatureVector as CSR (nodes, off, feat))."""
        return self.transform_sets([desc], levelsup)[0]

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().orbx_voc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
