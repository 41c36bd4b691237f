"""orb_slam2_commit_amd -- MI355X-native (gfx950 HIP) ORB-SLAM2 hot path.

The product is liborbx.so (HIP kernels + C ABI, include/orbx.h); this package
is the thin host-side mirror of the reference classes over it.
"""
from ._lib import KEYPOINT_DTYPE, OrbxError  # noqa: F401
from .orb import ORBextractor, ORBmatcher, ORBVocabulary, Optimizer, PnPsolver, compute_stereo_matches, frame_stereo  # noqa: F401

__all__ = ["ORBextractor", "ORBmatcher", "ORBVocabulary", "Optimizer", "PnPsolver", "compute_stereo_matches", "frame_stereo", "KEYPOINT_DTYPE", "OrbxError"]
