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
data stays in HBM; the host reads back only the per-frame counts that size the next call's
problem descriptors (FeatureVector node counts, edge counts): two small copies per batch.
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
                                          ptr(self.fv_nodes), ptr(self.fv_off), ptr(self.fv_feat), ptr(self.n_fv), sp),
              "orbx_voc_transform_device")
        if ev:
            ev[1].record(st)
        with torch.cuda.stream(st):
            kp32 = kps.view(torch.float32).reshape(2 * B, cap, 7)
            angle = kp32[:, :, 3].contiguous()  # keypoint angles as the matcher's SoA input
            valid = (depth > 0).to(torch.uint8)  # KeyFrame MapPoints: its stereo points
            host = torch.cat([self.n_fv, counts]).cpu().numpy()  # the one readback before SearchByBoW
        n_fv, cnt = host[:B], host[B:]
        t1 = time.perf_counter()
        # 2. SearchByBoW(KF, F) per pair (src/ORBmatcher.cc:175-325), nnratio 0.7 (src/Tracking.cc:918)
        K = len(pairs)
        probs = (_lib.BowProblem * max(K, 1))()
        es = 4  # int32 bytes

        def side(img, f):
            return _lib.BowSide(int(cnt[img]), desc.data_ptr() + img * cap * 32, angle.data_ptr() + img * cap * 4,
                                valid.data_ptr() + f * cap, int(n_fv[f]), self.fv_nodes.data_ptr() + f * cap * es,
                                self.fv_off.data_ptr() + f * (cap + 1) * es, self.fv_feat.data_ptr() + f * cap * es)

        for j, (kf, f) in enumerate(pairs):
            probs[j].a = side(2 * kf, kf)
            probs[j].b = side(2 * f, f)
            probs[j].b.valid = None
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
        with torch.cuda.stream(st):
            ne = self.n_edges[:K].cpu().numpy()  # the second readback: edge counts size the pose problems
        t2 = time.perf_counter()
        # 4. PoseOptimization from mLastFrame's pose (identity here), four rounds on the device
        T0 = np.eye(4, dtype=np.float32).ravel() if Tcw0 is None else np.asarray(Tcw0, np.float32).ravel()
        pp = (_lib.PoseProblem * max(K, 1))()
        for j in range(K):
            p = pp[j]
            p.n = int(ne[j])
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
            timings.append((t1 - t0, t2 - t1, t3 - t2, ev[0].elapsed_time(ev[1]) / 1e3,
                            ev[2].elapsed_time(ev[3]) / 1e3, ev[4].elapsed_time(ev[5]) / 1e3))
        return res[0], res[1], res[2]
