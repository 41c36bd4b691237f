"""Tracking::TrackReferenceKeyFrame's per-frame front end on a device frame batch
(src/Tracking.cc:910-969), after the batch's extraction + stereo matching:

    mCurrentFrame.ComputeBoW();                                           orbx_voc_transform_device
    nmatches = ORBmatcher(0.7, true).SearchByBoW(mpReferenceKF, mCurrentFrame, vpMapPointMatches)
                                                                          orbx_search_by_bow_device
    mCurrentFrame.mvpMapPoints = vpMapPointMatches; SetPose(mLastFrame.mTcw)
    Optimizer::PoseOptimization(&mCurrentFrame)                           orbx_track_gather_device +
                                                                          orbx_pose_optimization_device

for every (reference KeyFrame, current frame) pair of the batch at once.  The reference KeyFrame is
an earlier frame of the same batch whose MapPoints are its stereo points (mvDepth > 0, the map that
StereoInitialization / CreateNewKeyFrame build), at Frame::UnprojectStereo (src/Frame.cc:823-839) with
pose Twc.  Frame::UnprojectStereo and PoseOptimization read mvKeysUn; the batch passes the extractor's
keypoints (mvKeys), which ARE mvKeysUn for rectified input without distortion (UndistortKeyPoints copies
them when mDistCoef(0) == 0, src/Frame.cc:471-476) -- KITTI and rectified EuRoC.  Distorted input must
be undistorted first (orbx_undistort_keypoints) and the undistorted keypoints passed instead.  All
data stays in HBM and every launch is sized on the device (the counts the previous kernels wrote,
read through the problems' *_dev pointers): the host reads back only the results, once per batch.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, ptr


class TrackBatch:
    """Device buffers and problem descriptors for tracking `n_frames` frames of a batch of B stereo
    frames laid out as orbx_stereo_frames_device writes them (image 2f = left of frame f)."""

    def __init__(self, voc, B, cap, inv_level_sigma2, fx, fy, cx, cy, bf, device, levelsup=4, nnratio=0.7,
                 check_ori=True):
        import torch
        self.voc, self.B, self.cap = voc, int(B), int(cap)
        self.levelsup, self.nnratio, self.check_ori = int(levelsup), float(nnratio), int(bool(check_ori))
        self.cam = (float(fx), float(fy), float(cx), float(cy), float(bf))
        dev = device
        t = lambda *shape, dt=torch.int32: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731
        n = self.B * self.cap
        # ComputeBoW outputs of the B left images (set f at f * cap)
        self.bow_words, self.bow_values, self.n_bow = t(n), t(n, dt=torch.float64), t(self.B)
        self.fv_nodes, self.fv_off, self.fv_feat, self.n_fv = t(n), t(self.B * (self.cap + 1)), t(n), t(self.B)
        # SearchByBoW / gather / PoseOptimization per tracked frame slot
        self.match, self.nmatch = t(self.B, self.cap), t(self.B)
        self.obs, self.Xw = t(self.B, self.cap, 3, dt=torch.float32), t(self.B, self.cap, 3, dt=torch.float32)
        self.isig, self.edge_feat, self.n_edges = t(self.B, self.cap, dt=torch.float32), t(self.B, self.cap), t(self.B)
        self.Tcw_out, self.outlier = t(self.B, 16, dt=torch.float32), t(self.B, self.cap, dt=torch.uint8)
        self.ngood, self.iters = t(self.B), t(self.B, 4)
        self.level_isig = torch.as_tensor(np.asarray(inv_level_sigma2, np.float32)).to(dev)
        self.device = dev

    def run(self, kps, desc, counts, uright, depth, pairs, stream=None, Twc=None, Tcw0=None, timings=None):
        """pairs: list of (reference KeyFrame frame index, current frame index) within the batch.
        kps/desc/counts/uright/depth: the orbx_stereo_frames_device outputs.  Returns host arrays
        (nmatches, n_edges, ngood) per pair; the poses / outlier flags stay on the device
        (self.Tcw_out, self.outlier, in pair order)."""
        import time

        import torch
        if len(pairs) > self.B:
            raise ValueError("TrackBatch.run: %d pairs but the per-pair buffers hold B = %d" % (len(pairs), self.B))
        L = _lib.lib()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        sp = C.c_void_p(st.cuda_stream)
        B, cap = self.B, self.cap
        t0 = time.perf_counter()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)] if timings is not None else None
        if ev:
            ev[0].record(st)
        # 1. Frame::ComputeBoW on every left image (src/Frame.cc ComputeBoW)
        check(L.orbx_voc_transform_device(self.voc._h, ptr(desc), cap, 2 * cap, ptr(counts), 2, B, self.levelsup,
                                          ptr(self.bow_words), ptr(self.bow_values), ptr(self.n_bow),
                                          ptr(self.fv_nodes), ptr(self.fv_off), ptr(self.fv_feat), ptr(self.n_fv),
                                          C.c_void_p(st.cuda_stream or 1)),  # 1 = ORBX_STREAM_NULL
              "orbx_voc_transform_device")
        if ev:
            ev[1].record(st)
        with torch.cuda.stream(st):
            kp32 = kps.view(torch.float32).reshape(2 * B, cap, 7)
            angle = kp32[:, :, 3].contiguous()  # keypoint angles as the matcher's SoA input
            valid = (depth > 0).to(torch.uint8)  # KeyFrame MapPoints: its stereo points
        t1 = time.perf_counter()
        # 2. SearchByBoW(KF, F) per pair (src/ORBmatcher.cc:175-325), nnratio 0.7 (src/Tracking.cc:918): the
        # sides are sized on the device (feature counts of the extraction, node counts of ComputeBoW)
        K = len(pairs)
        probs = (_lib.BowProblem * max(K, 1))()
        es = 4  # int32 bytes

        def side(img, f):
            return _lib.BowSide(cap, desc.data_ptr() + img * cap * 32, angle.data_ptr() + img * cap * 4,
                                valid.data_ptr() + f * cap, cap, self.fv_nodes.data_ptr() + f * cap * es,
                                self.fv_off.data_ptr() + f * (cap + 1) * es, self.fv_feat.data_ptr() + f * cap * es)

        for j, (kf, f) in enumerate(pairs):
            probs[j].a = side(2 * kf, kf)
            probs[j].b = side(2 * f, f)
            probs[j].b.valid = None
            probs[j].a_n_dev, probs[j].a_nodes_dev = counts.data_ptr() + 2 * kf * es, self.n_fv.data_ptr() + kf * es
            probs[j].b_n_dev, probs[j].b_nodes_dev = counts.data_ptr() + 2 * f * es, self.n_fv.data_ptr() + f * es
            probs[j].nnratio, probs[j].check_ori, probs[j].mode = self.nnratio, self.check_ori, 0
            probs[j].match = self.match.data_ptr() + j * cap * es
            probs[j].nmatches = self.nmatch.data_ptr() + j * es
        if ev:
            ev[2].record(st)
        check(L.orbx_search_by_bow_device(probs, K, sp), "orbx_search_by_bow_device")
        # 3. the PoseOptimization edges of every pair (src/Optimizer.cc:318-410)
        fx, fy, cx, cy, bf = self.cam
        I34 = (C.c_float * 12)(*(np.eye(3, 4, dtype=np.float32).ravel() if Twc is None else np.asarray(Twc).ravel()))
        gs = (_lib.TrackGather * max(K, 1))()
        for j, (kf, f) in enumerate(pairs):
            g = gs[j]
            g.f_kps, g.f_uright, g.f_count = kps.data_ptr() + 2 * f * cap * 28, uright.data_ptr() + f * cap * 4, \
                counts.data_ptr() + 2 * f * es
            g.match = self.match.data_ptr() + j * cap * es
            g.kf_kps, g.kf_depth = kps.data_ptr() + 2 * kf * cap * 28, depth.data_ptr() + kf * cap * 4
            g.Twc = I34
            g.fx, g.fy, g.cx, g.cy = fx, fy, cx, cy
            g.inv_level_sigma2 = self.level_isig.data_ptr()
            g.obs, g.Xw = self.obs.data_ptr() + j * cap * 12, self.Xw.data_ptr() + j * cap * 12
            g.inv_sigma2, g.edge_feature = self.isig.data_ptr() + j * cap * 4, self.edge_feat.data_ptr() + j * cap * es
            g.n_edges = self.n_edges.data_ptr() + j * es
        check(L.orbx_track_gather_device(gs, K, sp), "orbx_track_gather_device")
        if ev:
            ev[3].record(st)
        t2 = time.perf_counter()
        # 4. PoseOptimization from mLastFrame's pose (identity here), four rounds on the device
        T0 = np.eye(4, dtype=np.float32).ravel() if Tcw0 is None else np.asarray(Tcw0, np.float32).ravel()
        pp = (_lib.PoseProblem * max(K, 1))()
        for j in range(K):
            p = pp[j]
            p.n, p.n_dev = cap, self.n_edges.data_ptr() + j * es  # sized on the device by the gather
            p.obs, p.Xw = self.obs.data_ptr() + j * cap * 12, self.Xw.data_ptr() + j * cap * 12
            p.inv_sigma2 = self.isig.data_ptr() + j * cap * 4
            p.fx, p.fy, p.cx, p.cy, p.bf = fx, fy, cx, cy, bf
            for i in range(16):
                p.Tcw[i] = float(T0[i])
            p.Tcw_out = self.Tcw_out.data_ptr() + j * 64
            p.outlier = self.outlier.data_ptr() + j * cap
            p.ngood = self.ngood.data_ptr() + j * es
            p.iterations = self.iters.data_ptr() + j * 16
        if ev:
            ev[4].record(st)
        check(L.orbx_pose_optimization_device(pp, K, sp), "orbx_pose_optimization_device")
        if ev:
            ev[5].record(st)
        with torch.cuda.stream(st):
            res = torch.stack([self.nmatch[:K], self.n_edges[:K], self.ngood[:K]]).cpu().numpy()
        t3 = time.perf_counter()
        if timings is not None:
            # host wall per phase (incl. waiting for earlier work on the stream and the readbacks), then
            # the GPU time of each phase's launches (HIP events on the launch stream)
            # (contiguous: ComputeBoW | angle/valid prep + SearchByBoW + edge gather | PoseOptimization)
            timings.append((t1 - t0, t2 - t1, t3 - t2, ev[0].elapsed_time(ev[1]) / 1e3,
                            ev[1].elapsed_time(ev[3]) / 1e3, ev[3].elapsed_time(ev[5]) / 1e3))
        return res[0], res[1], res[2]


# ---------------------------------------------------------------------------------------------------
# Tracking::TrackWithMotionModel + Tracking::TrackLocalMap (src/Tracking.cc:1049-1170, 1403-1468) on a
# device batch, every phase sized on the device (no host readback between launches):
#
#   UpdateLastFrame: the last frame's MapPoints = its stereo points        orbx_frame_points_device
#   SearchByProjection(F, LastFrame, th=7, bMono=false) (ORBmatcher 0.9)  orbx_search_by_projection_device
#   if nmatches < 20: again with 2*th                                      (same launch, gated on the count)
#   if nmatches < 20: lost; PoseOptimization edges                         orbx_track_step_device AFTER_MOTION
#   Optimizer::PoseOptimization(&F)                                         orbx_pose_optimization_device
#   outliers leave F, nmatchesMap >= 10; SearchLocalPoints' inputs         orbx_track_step_device AFTER_POSE
#   SearchLocalPoints: isInFrustum(0.5) + SearchByProjection(F, local, th=1) (ORBmatcher 0.8)
#                                                                          orbx_search_by_projection_device
#   TrackLocalMap's PoseOptimization edges                                 orbx_track_step_device AFTER_LOCAL
#   Optimizer::PoseOptimization(&F); mnMatchesInliers                      orbx_pose_optimization_device
#
# The local map is the last frame's MapPoints (the reference KeyFrame's, which this batch's last frame
# is): the points the motion model matched are "seen" (mnLastFrameSeen = current) and skipped, the rest
# go through the frustum test and the local search, as UpdateLocalMap + SearchLocalPoints do.
class MotionTrackBatch:
    """Device buffers for K = max_pairs (last frame, current frame) pairs of a stereo batch laid out as
    orbx_stereo_frames_device writes it (image 2f = left of frame f)."""

    def __init__(self, max_pairs, cap, width, height, scale_factors, inv_level_sigma2, fx, fy, cx, cy, bf, device,
                 th=7.0, th_local=1.0, min_matches=20, min_good=10):
        import torch
        self.K, self.cap = int(max_pairs), int(cap)
        self.cam = (float(fx), float(fy), float(cx), float(cy), float(bf))
        self.W, self.H = float(width), float(height)
        self.th, self.th_local = float(th), float(th_local)
        self.min_matches, self.min_good = int(min_matches), int(min_good)
        self.sf = np.asarray(scale_factors, np.float32)
        self.isg = np.asarray(inv_level_sigma2, np.float32)
        self.device = device
        K, c = self.K, self.cap
        t = lambda *shape, dt=torch.int32: torch.zeros(shape, dtype=dt, device=device)  # noqa: E731
        f32, u8 = torch.float32, torch.uint8
        # the last frames' MapPoints (orbx_frame_points)
        self.pos, self.normal, self.dist = t(K, c, 3, dt=f32), t(K, c, 3, dt=f32), t(K, c, 2, dt=f32)
        self.angle, self.octave, self.flags = t(K, c, dt=f32), t(K, c), t(K, c, dt=u8)
        # searches
        self.fout1, self.pm1, self.nm1 = t(K, c), t(K, c), t(K)
        self.fout2, self.pm2, self.nm2 = t(K, c), t(K, c), t(K)
        self.track, self.track_level = t(K, c, 4, dt=f32), t(K, c)
        # frame map and bookkeeping
        self.fmap, self.seen, self.lflags = t(K, c), t(K, c, dt=u8), t(K, c, dt=u8)
        self.occ, self.lost = t(K, c, dt=torch.int8), t(K)
        # PoseOptimization edges and results
        self.obs, self.Xw, self.isig = t(K, c, 3, dt=f32), t(K, c, 3, dt=f32), t(K, c, dt=f32)
        self.edge_feat, self.n_edges = t(K, c), t(K)
        self.T1, self.out1, self.ng1 = t(K, 16, dt=f32), t(K, c, dt=u8), t(K)
        self.T2, self.out2, self.ng2 = t(K, 16, dt=f32), t(K, c, dt=u8), t(K)
        self.level_isig = torch.as_tensor(self.isg).to(device)

    def _frame(self, kps, desc, uright, counts, f, Tcw, occ=None):
        cap = self.cap
        fr = _lib.ProjFrame()
        fr.n = cap
        fr.keys_un = kps.data_ptr() + 2 * f * cap * 28
        fr.desc = desc.data_ptr() + 2 * f * cap * 32
        fr.u_right = uright.data_ptr() + f * cap * 4
        fr.occ = occ
        fr.min_x, fr.max_x, fr.min_y, fr.max_y = 0.0, self.W, 0.0, self.H
        fr.grid_inv_w = float(np.float32(64) / np.float32(self.W))
        fr.grid_inv_h = float(np.float32(48) / np.float32(self.H))
        nl = len(self.sf)
        fr.nlevels = nl
        sf, isg = np.zeros(16, np.float32), np.zeros(16, np.float32)
        sf[:nl], isg[:nl] = self.sf, self.isg
        fr.scale_factors[:] = sf.tolist()
        fr.inv_level_sigma2[:] = isg.tolist()
        fr.log_scale_factor = float(log_scale_factor(self.sf[1] if nl > 1 else 1.0))
        fx, fy, cx, cy, bf = self.cam
        fr.fx, fr.fy, fr.cx, fr.cy, fr.bf = fx, fy, cx, cy, bf
        fr.b = float(np.float32(bf) / np.float32(fx))
        fr.Tcw[:] = np.asarray(Tcw, np.float32).reshape(16).tolist()
        return fr

    def run(self, kps, desc, counts, uright, depth, pairs, last_kps=None, last_Twc=None, Tcw_guess=None,
            stream=None, timings=None):
        """pairs: (last frame index, current frame index) within the batch.  last_kps: optional (K, cap, 28)
        device keypoints standing for the last frames' mvKeysUn (default: the batch's own); last_Twc:
        (K, 3, 4) poses of the last frames (default identity); Tcw_guess: (K, 4, 4) mVelocity*LastTcw
        (default identity).  Returns host arrays per pair: nmatches (motion model, after the retry), ngood
        of PoseOptimization 1, lost, local-search matches, mnMatchesInliers."""
        import torch
        K = len(pairs)
        if K > self.K:
            raise ValueError("MotionTrackBatch.run: %d pairs but max_pairs = %d" % (K, self.K))
        L = _lib.lib()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        sp = C.c_void_p(st.cuda_stream)
        cap = self.cap
        fx, fy, cx, cy, bf = self.cam
        I4 = np.eye(4, dtype=np.float32)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)] if timings is not None else None

        def rec(k):
            if ev:
                ev[k].record(st)
        es = 4
        rec(0)
        # 1. UpdateLastFrame: the last frames' MapPoints
        fp = (_lib.FramePoints * max(K, 1))()
        for j, (lf, f) in enumerate(pairs):
            p = fp[j]
            p.kps = (last_kps.data_ptr() + j * cap * 28) if last_kps is not None else kps.data_ptr() + 2 * lf * cap * 28
            p.depth = depth.data_ptr() + lf * cap * 4
            p.count = counts.data_ptr() + 2 * lf * es
            p.cap = cap
            Twc = np.eye(3, 4, dtype=np.float32) if last_Twc is None else np.asarray(last_Twc[j], np.float32)
            p.Twc[:] = Twc.reshape(12).tolist()
            p.fx, p.fy, p.cx, p.cy = fx, fy, cx, cy
            p.nlevels = len(self.sf)
            sf = np.zeros(16, np.float32)
            sf[:len(self.sf)] = self.sf
            p.scale_factors[:] = sf.tolist()
            p.pos, p.normal, p.dist_minmax = (self.pos.data_ptr() + j * cap * 12, self.normal.data_ptr() + j * cap * 12,
                                              self.dist.data_ptr() + j * cap * 8)
            p.angle, p.octave, p.flags = (self.angle.data_ptr() + j * cap * 4, self.octave.data_ptr() + j * cap * es,
                                          self.flags.data_ptr() + j * cap)
        check(L.orbx_frame_points_device(fp, K, sp), "orbx_frame_points_device")
        # 2. SearchByProjection(F, LastFrame, th, bMono=false), then again with 2*th when < 20 matched
        probs = [(_lib.ProjProblem * max(K, 1))(), (_lib.ProjProblem * max(K, 1))()]
        for j, (lf, f) in enumerate(pairs):
            T0 = I4 if Tcw_guess is None else np.asarray(Tcw_guess[j], np.float32)
            for r in range(2):
                q = probs[r][j]
                q.kind, q.frustum = 1, 0
                q.f = self._frame(kps, desc, uright, counts, f, T0)
                q.f_n_dev = counts.data_ptr() + 2 * f * es
                q.n_points, q.n_points_dev = cap, counts.data_ptr() + 2 * lf * es
                q.desc = desc.data_ptr() + 2 * lf * cap * 32
                q.flags, q.pos = self.flags.data_ptr() + j * cap, self.pos.data_ptr() + j * cap * 12
                q.angle, q.octave = self.angle.data_ptr() + j * cap * 4, self.octave.data_ptr() + j * cap * es
                q.th = self.th * (2 if r else 1)
                q.nnratio, q.view_cos_limit, q.check_ori, q.mono, q.orb_dist = 0.9, 0.5, 1, 0, 100
                q.last_Tcw[:] = (np.eye(4, dtype=np.float32) if last_Twc is None else
                                 _inv_pose(np.asarray(last_Twc[j], np.float32))).reshape(16).tolist()
                q.frame_out, q.point_match = self.fout1.data_ptr() + j * cap * es, self.pm1.data_ptr() + j * cap * es
                q.nmatches = self.nm1.data_ptr() + j * es
                if r:  # src/Tracking.cc:1071-1076
                    q.gate, q.gate_below = self.nm1.data_ptr() + j * es, self.min_matches
        check(L.orbx_search_by_projection_device(probs[0], K, sp), "orbx_search_by_projection_device")
        check(L.orbx_search_by_projection_device(probs[1], K, sp), "orbx_search_by_projection_device (2*th)")
        rec(1)
        # 3. lost / edges, PoseOptimization, outliers, SearchLocalPoints' inputs
        steps = (_lib.TrackStep * max(K, 1))()

        def step(op, frame_out):
            for j, (lf, f) in enumerate(pairs):
                s = steps[j]
                s.op, s.cap = op, cap
                s.count = counts.data_ptr() + 2 * f * es
                s.kps, s.u_right = kps.data_ptr() + 2 * f * cap * 28, uright.data_ptr() + f * cap * 4
                s.inv_level_sigma2 = self.level_isig.data_ptr()
                s.n_points = counts.data_ptr() + 2 * lf * es
                s.pos, s.flags = self.pos.data_ptr() + j * cap * 12, self.flags.data_ptr() + j * cap
                s.frame_out = frame_out.data_ptr() + j * cap * es
                s.nmatches, s.min_matches = self.nm1.data_ptr() + j * es, self.min_matches
                s.outlier, s.ngood, s.min_good = (self.out1.data_ptr() + j * cap, self.ng1.data_ptr() + j * es,
                                                  self.min_good)
                s.fmap, s.seen = self.fmap.data_ptr() + j * cap * es, self.seen.data_ptr() + j * cap
                s.local_flags, s.occ = self.lflags.data_ptr() + j * cap, self.occ.data_ptr() + j * cap
                s.lost = self.lost.data_ptr() + j * es
                s.obs, s.Xw = self.obs.data_ptr() + j * cap * 12, self.Xw.data_ptr() + j * cap * 12
                s.inv_sigma2 = self.isig.data_ptr() + j * cap * 4
                s.edge_feature, s.n_edges = self.edge_feat.data_ptr() + j * cap * es, self.n_edges.data_ptr() + j * es
            check(L.orbx_track_step_device(steps, K, sp), "orbx_track_step_device")

        def pose(Tout, outl, ngood, Tcw_dev=None):
            pp = (_lib.PoseProblem * max(K, 1))()
            for j in range(K):
                p = pp[j]
                p.n, p.n_dev = cap, self.n_edges.data_ptr() + j * es
                p.obs, p.Xw = self.obs.data_ptr() + j * cap * 12, self.Xw.data_ptr() + j * cap * 12
                p.inv_sigma2 = self.isig.data_ptr() + j * cap * 4
                p.fx, p.fy, p.cx, p.cy, p.bf = fx, fy, cx, cy, bf
                T0 = I4 if Tcw_guess is None else np.asarray(Tcw_guess[j], np.float32)
                p.Tcw[:] = T0.reshape(16).tolist()
                p.Tcw_dev = (Tcw_dev.data_ptr() + j * 64) if Tcw_dev is not None else None
                p.Tcw_out, p.outlier, p.ngood = Tout.data_ptr() + j * 64, outl.data_ptr() + j * cap, ngood.data_ptr() + j * es
            check(L.orbx_pose_optimization_device(pp, K, sp), "orbx_pose_optimization_device")

        step(0, self.fout1)  # ORBX_TRACK_AFTER_MOTION
        rec(2)
        pose(self.T1, self.out1, self.ng1)
        rec(3)
        step(1, self.fout1)  # ORBX_TRACK_AFTER_POSE
        # 4. SearchLocalPoints: isInFrustum + SearchByProjection(F, local map points, th) from the new pose
        lp = (_lib.ProjProblem * max(K, 1))()
        for j, (lf, f) in enumerate(pairs):
            q = lp[j]
            q.kind, q.frustum = 0, 1
            q.f = self._frame(kps, desc, uright, counts, f, I4, occ=self.occ.data_ptr() + j * cap)
            q.f_n_dev, q.Tcw_dev = counts.data_ptr() + 2 * f * es, self.T1.data_ptr() + j * 64
            q.n_points, q.n_points_dev = cap, counts.data_ptr() + 2 * lf * es
            q.desc, q.flags = desc.data_ptr() + 2 * lf * cap * 32, self.lflags.data_ptr() + j * cap
            q.pos, q.normal = self.pos.data_ptr() + j * cap * 12, self.normal.data_ptr() + j * cap * 12
            q.dist_minmax = self.dist.data_ptr() + j * cap * 8
            q.track, q.track_level = self.track.data_ptr() + j * cap * 16, self.track_level.data_ptr() + j * cap * es
            q.th, q.nnratio, q.view_cos_limit, q.check_ori = self.th_local, 0.8, 0.5, 1
            q.frame_out, q.point_match = self.fout2.data_ptr() + j * cap * es, self.pm2.data_ptr() + j * cap * es
            q.nmatches = self.nm2.data_ptr() + j * es
            q.gate, q.gate_below = self.lost.data_ptr() + j * es, 1  # a lost frame does not TrackLocalMap
        check(L.orbx_search_by_projection_device(lp, K, sp), "orbx_search_by_projection_device (local)")
        rec(4)
        step(2, self.fout2)  # ORBX_TRACK_AFTER_LOCAL
        pose(self.T2, self.out2, self.ng2, Tcw_dev=self.T1)
        rec(5)
        with torch.cuda.stream(st):
            res = torch.stack([self.nm1[:K], self.ng1[:K], self.lost[:K], self.nm2[:K], self.ng2[:K]]).cpu().numpy()
        if timings is not None:  # GPU time per phase: search (last frame), gather+pose 1, local search, pose 2
            timings.append((ev[0].elapsed_time(ev[1]) / 1e3, ev[1].elapsed_time(ev[3]) / 1e3,
                            ev[3].elapsed_time(ev[4]) / 1e3, ev[4].elapsed_time(ev[5]) / 1e3))
        # a lost frame skipped the local search (its gate), so its nm2 slot still holds an older call's
        # count: report 0 for it, as the reference never runs TrackLocalMap on it
        local = np.where(res[2] != 0, 0, res[3])
        return dict(nmatches=res[0], ngood_motion=res[1], lost=res[2], local_matches=local, inliers=res[4])


def log_scale_factor(scale_factor):
    """Frame::mfLogScaleFactor = log(mfScaleFactor) on a float (the float overload, correctly rounded)."""
    import math
    return np.float32(math.log(float(np.float32(scale_factor))))


def _inv_pose(Twc34):
    """Tcw (4x4) of a camera-to-world 3x4 pose."""
    R, t = Twc34[:, :3].astype(np.float64), Twc34[:, 3].astype(np.float64)
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = R.T
    T[:3, 3] = -R.T @ t
    return T
