"""ctypes loader for liborbx.so (the HIP kernels + C ABI of include/orbx.h).

There is no CPU fallback: if the shared library is missing or cannot be
loaded, or no gfx950 device is visible when a handle is created, the call
raises.  Build with ``python -c "import __graft_entry__ as g; g.build()"`` or
``make -C orb_slam2_commit_amd/csrc``.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ORBX_LIB_OVERRIDE") or os.path.join(_HERE, "liborbx.so")  # override: A/B experiments only

ORBX_OK = 0
ORBX_ERR_ARG = -1
ORBX_ERR_CAPACITY = -2
ORBX_ERR_HIP = -3
ORBX_ERR_NODEV = -4
ORBX_ERR_SIZE = -5
ORBX_ERR_STATE = -6
_ERRS = {ORBX_ERR_ARG: "bad argument", ORBX_ERR_CAPACITY: "capacity", ORBX_ERR_HIP: "HIP runtime error",
         ORBX_ERR_NODEV: "no HIP device", ORBX_ERR_SIZE: "unsupported geometry", ORBX_ERR_STATE: "no extraction yet"}

# Layout-identical to cv::KeyPoint / orbx_keypoint (28 bytes).
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28


class OrbxError(RuntimeError):
    def __init__(self, code, what):
        super().__init__("%s failed: %s (%d)" % (what, _ERRS.get(code, "error"), code))
        self.code = code


class ExtractorParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int)]


class BowSide(C.Structure):
    _fields_ = [("n", C.c_int), ("desc", C.c_void_p), ("angle", C.c_void_p), ("valid", C.c_void_p),
                ("n_nodes", C.c_int), ("node_id", C.c_void_p), ("node_off", C.c_void_p), ("feat", C.c_void_p)]


class BowProblem(C.Structure):
    _fields_ = [("a", BowSide), ("b", BowSide), ("nnratio", C.c_float), ("check_ori", C.c_int), ("mode", C.c_int),
                ("match", C.c_void_p), ("nmatches", C.c_void_p), ("a_n_dev", C.c_void_p), ("a_nodes_dev", C.c_void_p),
                ("b_n_dev", C.c_void_p), ("b_nodes_dev", C.c_void_p)]


class BaProblem(C.Structure):
    _fields_ = [("n_cams", C.c_int), ("Tcw", C.c_void_p), ("fixed", C.c_void_p), ("intr", C.c_void_p),
                ("n_points", C.c_int), ("Xw", C.c_void_p), ("n_edges", C.c_int), ("edge_point", C.c_void_p),
                ("edge_cam", C.c_void_p), ("obs", C.c_void_p), ("inv_sigma2", C.c_void_p)]


class BaResult(C.Structure):
    _fields_ = [("Tcw", C.c_void_p), ("Xw", C.c_void_p), ("edge_outlier", C.c_void_p), ("Tcw_d", C.c_void_p),
                ("Xw_d", C.c_void_p), ("iterations", C.c_int * 2), ("trials", C.c_int), ("chi2", C.c_double * 2),
                ("ran", C.c_int)]


class PnpProblem(C.Structure):
    _fields_ = [("n", C.c_int), ("p3d", C.c_void_p), ("p2d", C.c_void_p), ("sigma2", C.c_void_p),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float)]


class PnpParams(C.Structure):
    _fields_ = [("probability", C.c_double), ("min_inliers", C.c_int), ("max_iterations", C.c_int),
                ("min_set", C.c_int), ("epsilon", C.c_float), ("th2", C.c_float)]


class ProjFrame(C.Structure):
    _fields_ = [("n", C.c_int), ("keys_un", C.c_void_p), ("desc", C.c_void_p), ("u_right", C.c_void_p),
                ("occ", C.c_void_p), ("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float),
                ("max_y", C.c_float), ("grid_inv_w", C.c_float), ("grid_inv_h", C.c_float), ("nlevels", C.c_int),
                ("scale_factors", C.c_float * 16), ("inv_level_sigma2", C.c_float * 16),
                ("log_scale_factor", C.c_float), ("fx", C.c_float),
                ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float), ("b", C.c_float),
                ("Tcw", C.c_float * 16), ("grid_min_x", C.c_float), ("grid_min_y", C.c_float),
                ("grid_min_set", C.c_int)]


class ProjProblem(C.Structure):
    _fields_ = [("kind", C.c_int), ("frustum", C.c_int), ("f", ProjFrame), ("n_points", C.c_int),
                ("desc", C.c_void_p), ("flags", C.c_void_p), ("pos", C.c_void_p), ("normal", C.c_void_p),
                ("dist_minmax", C.c_void_p), ("angle", C.c_void_p), ("octave", C.c_void_p), ("track", C.c_void_p),
                ("track_level", C.c_void_p), ("th", C.c_float), ("nnratio", C.c_float),
                ("view_cos_limit", C.c_float), ("check_ori", C.c_int), ("mono", C.c_int), ("orb_dist", C.c_int),
                ("last_Tcw", C.c_float * 16), ("frame_out", C.c_void_p), ("point_match", C.c_void_p),
                ("nmatches", C.c_void_p), ("f_n_dev", C.c_void_p), ("n_points_dev", C.c_void_p),
                ("Tcw_dev", C.c_void_p), ("gate", C.c_void_p), ("gate_below", C.c_int)]


class Sim3Problem(C.Structure):
    _fields_ = [("kf1", ProjFrame), ("kf2", ProjFrame)] + \
               [(k, C.c_void_p) for k in ("desc1", "pos1", "dist_minmax1", "flags1", "desc2", "pos2", "dist_minmax2",
                                          "flags2")] + \
               [("s12", C.c_float), ("R12", C.c_float * 9), ("t12", C.c_float * 3), ("th", C.c_float),
                ("match12", C.c_void_p), ("nfound", C.c_void_p)]


class InitProblem(C.Structure):
    _fields_ = [("f1", ProjFrame), ("f2", ProjFrame), ("prev_matched", C.c_void_p), ("window", C.c_int),
                ("nnratio", C.c_float), ("check_ori", C.c_int), ("match12", C.c_void_p), ("nmatches", C.c_void_p)]


class PoseProblem(C.Structure):
    _fields_ = [("n", C.c_int), ("obs", C.c_void_p), ("Xw", C.c_void_p), ("inv_sigma2", C.c_void_p),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("Tcw", C.c_float * 16), ("Tcw_out", C.c_void_p), ("outlier", C.c_void_p), ("ngood", C.c_void_p),
                ("iterations", C.c_void_p), ("n_dev", C.c_void_p), ("Tcw_dev", C.c_void_p)]


class TriKF(C.Structure):
    _fields_ = [("n", C.c_int), ("keys_un", C.c_void_p), ("desc", C.c_void_p), ("u_right", C.c_void_p),
                ("has_mp", C.c_void_p), ("n_nodes", C.c_int), ("node_id", C.c_void_p), ("node_off", C.c_void_p),
                ("feat", C.c_void_p)]


class TriProblem(C.Structure):
    _fields_ = [("kf1", TriKF), ("kf2", TriKF), ("F12", C.c_float * 9), ("C1w", C.c_float * 3),
                ("T2w", C.c_float * 16), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("scale_factors2", C.c_float * 16), ("level_sigma2_2", C.c_float * 16), ("only_stereo", C.c_int),
                ("check_ori", C.c_int), ("match12", C.c_void_p), ("nmatches", C.c_void_p)]


class FramePoints(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("depth", C.c_void_p), ("count", C.c_void_p), ("cap", C.c_int),
                ("Twc", C.c_float * 12), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("nlevels", C.c_int), ("scale_factors", C.c_float * 16), ("pos", C.c_void_p), ("normal", C.c_void_p),
                ("dist_minmax", C.c_void_p), ("angle", C.c_void_p), ("octave", C.c_void_p), ("flags", C.c_void_p)]


class TrackStep(C.Structure):
    _fields_ = [("op", C.c_int), ("cap", C.c_int), ("count", C.c_void_p), ("kps", C.c_void_p), ("u_right", C.c_void_p),
                ("inv_level_sigma2", C.c_void_p), ("n_points", C.c_void_p), ("pos", C.c_void_p),
                ("flags", C.c_void_p), ("frame_out", C.c_void_p), ("nmatches", C.c_void_p), ("min_matches", C.c_int),
                ("outlier", C.c_void_p), ("ngood", C.c_void_p), ("min_good", C.c_int), ("fmap", C.c_void_p),
                ("seen", C.c_void_p), ("local_flags", C.c_void_p), ("occ", C.c_void_p), ("lost", C.c_void_p),
                ("obs", C.c_void_p), ("Xw", C.c_void_p), ("inv_sigma2", C.c_void_p), ("edge_feature", C.c_void_p),
                ("n_edges", C.c_void_p)]


class TrackGather(C.Structure):
    _fields_ = [("f_kps", C.c_void_p), ("f_uright", C.c_void_p), ("f_count", C.c_void_p), ("match", C.c_void_p),
                ("kf_kps", C.c_void_p), ("kf_depth", C.c_void_p), ("Twc", C.c_float * 12), ("fx", C.c_float),
                ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("inv_level_sigma2", C.c_void_p),
                ("obs", C.c_void_p), ("Xw", C.c_void_p), ("inv_sigma2", C.c_void_p), ("edge_feature", C.c_void_p),
                ("n_edges", C.c_void_p)]


class BaDebugOptions(C.Structure):  # include/orbx_debug.h orbx_ba_debug_options
    _fields_ = [("ldlt", C.c_int), ("nan_trial", C.c_int), ("raise_stop_after", C.c_int), ("trace", C.c_int),
                ("fused_ctl", C.c_int)]


class Camera(C.Structure):
    _fields_ = [("K", C.c_float * 9), ("dist", C.c_float * 5), ("n_dist", C.c_int)]


class RandState(C.Structure):
    _fields_ = [("r", C.c_uint32 * 34), ("i", C.c_int32)]


class PnpResult(C.Structure):
    _fields_ = [("no_more", C.c_int), ("found", C.c_int), ("n_inliers", C.c_int), ("used", C.c_int),
                ("Tcw", C.c_float * 16)]


# Every entry point of include/orbx.h with its ctypes signature.
P = C.c_void_p
SIGNATURES = {
    "orbx_extractor_create": ([C.POINTER(ExtractorParams), C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "orbx_extractor_destroy": ([P], None),
    "orbx_extractor_get_levels": ([P], C.c_int),
    "orbx_extractor_scale_tables": ([P, P, P, P, P], C.c_int),
    "orbx_extractor_tables": ([P, P, P, P], C.c_int),
    "orbx_extractor_set_pyramid_readback": ([P, C.c_int], C.c_int),
    "orbx_extractor_max_keypoints": ([P, C.c_int, C.c_int], C.c_int),
    "orbx_extract": ([P, P, C.c_int, C.c_int, C.c_size_t, P, C.c_int, P, C.POINTER(C.c_int)], C.c_int),
    "orbx_pyramid_level": ([P, C.c_int, C.c_int, P, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)], C.c_int),
    "orbx_extract_batch_device": ([P, C.c_int, P, C.c_int, C.c_int, C.c_size_t, P, P, P, C.c_int, P], C.c_int),
    "orbx_stereo_match": ([P, P, P, P, C.c_int, P, P, C.c_int, C.c_float, C.c_float, P, P], C.c_int),
    "orbx_frame_stereo": ([P, P, C.c_size_t, P, C.c_size_t, C.c_int, C.c_int, C.c_float, C.c_float, P, P, C.c_int, P,
                           P, P, C.c_int, P, P, P], C.c_int),
    "orbx_stereo_frames_device": ([P, C.c_int, P, C.c_int, C.c_int, C.c_size_t, P, P, P, C.c_int, C.c_float,
                                   C.c_float, P, P, P, P], C.c_int),
    "orbx_descriptor_distance_device": ([P, P, C.c_int, P, P], C.c_int),
    "orbx_search_by_bow_kf_f": ([C.POINTER(BowSide), C.POINTER(BowSide), C.c_float, C.c_int, P,
                                 C.POINTER(C.c_int), C.c_int], C.c_int),
    "orbx_search_by_bow_kf_kf": ([C.POINTER(BowSide), C.POINTER(BowSide), C.c_float, C.c_int, P,
                                  C.POINTER(C.c_int), C.c_int], C.c_int),
    "orbx_search_by_bow_device": ([C.POINTER(BowProblem), C.c_int, P], C.c_int),
    "orbx_pnp_create": ([C.POINTER(PnpProblem), C.POINTER(PnpParams), C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "orbx_pnp_create_many": ([P, C.c_int, C.POINTER(PnpParams), C.c_int, P], C.c_int),
    "orbx_pnp_create_many_device": ([P, P, P, P, P, C.c_int, C.POINTER(PnpParams), C.c_int, P], C.c_int),
    "orbx_pnp_destroy": ([P], C.c_int),
    "orbx_pnp_get_params": ([P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_float)], C.c_int),
    "orbx_pnp_set_ransac_parameters": ([P, P, C.POINTER(PnpParams)], C.c_int),
    "orbx_pnp_iterate": ([P, C.c_int, P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), P, P,
                          C.POINTER(C.c_int), C.POINTER(C.c_int)], C.c_int),
    "orbx_pnp_iterate_stream": ([P, C.c_int, C.POINTER(RandState), C.POINTER(C.c_int), P, P, C.POINTER(C.c_int),
                                 C.POINTER(C.c_int)], C.c_int),
    "orbx_voc_load_text": ([C.c_char_p, C.c_size_t, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "orbx_voc_destroy": ([P], C.c_int),
    "orbx_voc_info": ([P, P], C.c_int),
    "orbx_voc_transform": ([P, P, P, C.c_int, C.c_int, P, P, P, P, P, P, P], C.c_int),
    "orbx_voc_transform_device": ([P, P, C.c_int, C.c_longlong, P, C.c_int, C.c_int, C.c_int, P, P, P, P, P, P, P, P],
                                  C.c_int),
    "orbx_track_gather_device": ([C.POINTER(TrackGather), C.c_int, P], C.c_int),
    "orbx_frame_points_device": ([C.POINTER(FramePoints), C.c_int, P], C.c_int),
    "orbx_track_step_device": ([C.POINTER(TrackStep), C.c_int, P], C.c_int),
    "orbx_search_by_projection": ([C.POINTER(ProjProblem), C.c_int], C.c_int),
    "orbx_search_by_sim3": ([C.POINTER(Sim3Problem), C.c_int], C.c_int),
    "orbx_search_for_initialization": ([C.POINTER(InitProblem), C.c_int], C.c_int),
    "orbx_search_by_projection_device": ([C.POINTER(ProjProblem), C.c_int, P], C.c_int),
    "orbx_pose_optimization": ([C.POINTER(PoseProblem), C.c_int], C.c_int),
    "orbx_pose_optimization_device": ([C.POINTER(PoseProblem), C.c_int, P], C.c_int),
    "orbx_search_for_triangulation": ([C.POINTER(TriProblem), C.c_int], C.c_int),
    "orbx_search_for_triangulation_device": ([C.POINTER(TriProblem), C.c_int, P], C.c_int),
    "orbx_distinctive_descriptors": ([P, P, C.c_int, P, P, C.c_int], C.c_int),
    "orbx_distinctive_descriptors_device": ([P, P, C.c_int, P, P, P], C.c_int),
    "orbx_undistort_keypoints": ([P, C.c_int, C.POINTER(Camera), P, C.c_int], C.c_int),
    "orbx_undistort_keypoints_device": ([P, P, C.c_int, C.c_int, P, P, P], C.c_int),
    "orbx_pnp_iterate_candidates": ([P, C.c_int, C.c_int, C.POINTER(RandState), P, P, C.POINTER(C.c_int)], C.c_int),
    "orbx_pnp_iterate_many": ([P, C.c_int, C.c_int, P, P, P], C.c_int),
    "orbx_rand_seed":([C.POINTER(RandState), C.c_uint32], None),
    "orbx_rand_next": ([C.POINTER(RandState)], C.c_int32),
    "orbx_ba_create": ([C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "orbx_ba_create_priority": ([C.c_int, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "orbx_ba_create_masked": ([C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "orbx_stream_create": ([C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "orbx_stream_destroy": ([C.c_void_p], None),
    "orbx_ba_destroy": ([P], C.c_int),
    "orbx_ba_run": ([P, C.POINTER(BaProblem), C.POINTER(BaResult), P], C.c_int),
    "orbx_ba_run_bool": ([P, C.POINTER(BaProblem), C.POINTER(BaResult), P], C.c_int),
    "orbx_ba_stop_flag": ([P, C.POINTER(C.POINTER(C.c_int))], C.c_int),
    "orbx_ba_run_many": ([P, C.c_int, C.POINTER(BaProblem), C.POINTER(BaResult), P], C.c_int),
    "orbx_local_ba": ([C.POINTER(BaProblem), C.POINTER(BaResult), P, C.c_int], C.c_int),
    "orbx_device_count": ([], C.c_int),
    "orbx_version": ([], C.c_char_p),
    "orbx_sizeof": ([C.c_char_p], C.c_longlong),
    "orbx_profile_enable": ([P, C.c_int], C.c_int),
    "orbx_profile_reset": ([P], C.c_int),
    "orbx_profile_read": ([P, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_longlong),
                           C.POINTER(C.c_char_p)], C.c_int),
    # include/orbx_debug.h
    "orbx_debug_copy": ([P, C.c_int, C.c_int, C.c_int, P, C.c_size_t], C.c_longlong),
    "orbx_debug_ldlt": ([P, P, C.c_int, P, C.c_int, C.POINTER(C.c_float)], C.c_int),
    "orbx_debug_ldlt_ex": ([P, P, C.c_int, P, C.c_int, C.POINTER(C.c_float), C.c_int, P], C.c_int),
    "orbx_debug_ba_options": ([P, C.POINTER(BaDebugOptions)], C.c_int),
    "orbx_debug_hbm_copy": ([P, P, C.c_size_t, C.c_int, C.POINTER(C.c_float)], C.c_int),
}

_lib = None


def lib():
    """Load liborbx.so (raises if it is absent: no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("liborbx.so not found at %s -- build it first (make -C orb_slam2_commit_amd/csrc)"
                               % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(code, what):
    if code != ORBX_OK:
        raise OrbxError(code, what)


def ptr(a):
    """Host numpy array or torch tensor (host or device) -> void*."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        # a writable buffer's address through ctypes.from_buffer (~1 us; ctypes.data_as ~4 us), else
        # (read-only, empty, non-contiguous) the array interface's data pointer
        try:
            return C.c_void_p(C.addressof(C.c_char.from_buffer(a)))
        except (TypeError, ValueError, BufferError):
            return C.c_void_p(a.__array_interface__["data"][0])
    if hasattr(a, "data_ptr"):
        return C.c_void_p(a.data_ptr())
    raise TypeError(type(a))
