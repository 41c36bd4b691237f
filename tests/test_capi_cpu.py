"""CPU checks of the C-ABI library: it loads, exports every declared entry
point, and refuses (loudly) to run without a GPU -- no compute calls here."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "orb_slam2_commit_amd", "liborbx.so")


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(orbx_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "orb_slam2_commit_amd", "csrc")])
    from orb_slam2_commit_amd import _lib
    return _lib.lib()


def test_exports_every_declared_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r" T (orbx_\w+)", out))
    for h in ("orbx.h", "orbx_debug.h"):
        names = declared(h)
        assert names, h
        missing = [n for n in names if n not in exported]
        assert not missing, (h, missing)


def test_python_signatures_cover_abi(lib):
    from orb_slam2_commit_amd import _lib
    for h in ("orbx.h", "orbx_debug.h"):
        for n in declared(h):
            assert n in _lib.SIGNATURES, n


def test_no_gpu_fails_loudly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from orb_slam2_commit_amd import ORBextractor, OrbxError
    assert lib.orbx_device_count() == 0
    with pytest.raises(OrbxError) as e:
        ORBextractor(1000, 1.2, 8, 20, 7)
    assert e.value.code == -4


def test_version(lib):
    assert b"gfx950" in lib.orbx_version()


def test_keypoint_layout():
    import numpy as np
    from orb_slam2_commit_amd import KEYPOINT_DTYPE
    assert KEYPOINT_DTYPE.itemsize == 28  # cv::KeyPoint
    assert [KEYPOINT_DTYPE.fields[f][1] for f in KEYPOINT_DTYPE.names] == [0, 4, 8, 12, 16, 20, 24]
    assert np.dtype(KEYPOINT_DTYPE)


def test_ctypes_layouts_match_the_c_abi():
    """Every ctypes mirror of an include/orbx.h struct has the C size (orbx_sizeof, no GPU needed)."""
    import ctypes as C
    from orb_slam2_commit_amd import _lib
    L = _lib.lib()
    pairs = {"orbx_extractor_params": _lib.ExtractorParams, "orbx_bow_side": _lib.BowSide,
             "orbx_bow_problem": _lib.BowProblem, "orbx_ba_problem": _lib.BaProblem, "orbx_ba_result": _lib.BaResult,
             "orbx_pnp_problem": _lib.PnpProblem, "orbx_pnp_params": _lib.PnpParams,
             "orbx_pnp_result": _lib.PnpResult, "orbx_rand_state": _lib.RandState,
             "orbx_proj_frame": _lib.ProjFrame, "orbx_proj_problem": _lib.ProjProblem,
             "orbx_tri_kf": _lib.TriKF, "orbx_tri_problem": _lib.TriProblem, "orbx_pose_problem": _lib.PoseProblem,
             "orbx_track_gather": _lib.TrackGather, "orbx_frame_points": _lib.FramePoints,
             "orbx_track_step": _lib.TrackStep, "orbx_camera": _lib.Camera, "orbx_sim3_problem": _lib.Sim3Problem,
             "orbx_init_problem": _lib.InitProblem}
    for name, cls in pairs.items():
        assert L.orbx_sizeof(name.encode()) == C.sizeof(cls), name
    assert L.orbx_sizeof(b"orbx_keypoint") == _lib.KEYPOINT_DTYPE.itemsize == 28
    assert L.orbx_sizeof(b"no_such_type") == -1


def test_handle_stream_sentinel():
    """torch's legacy default stream (cuda_stream 0) reaches the handle-owning entry points as
    ORBX_STREAM_NULL (1), not NULL (= the handle's own non-blocking stream, unordered with the caller's
    work); other streams and the plain-stream entry points pass through unchanged."""
    from types import SimpleNamespace

    from orb_slam2_commit_amd.orb import _stream_ptr
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "orbx.h")).read()
    assert re.search(r"#define ORBX_STREAM_NULL \(\(void\*\)1\)", hdr)
    null, other = SimpleNamespace(cuda_stream=0), SimpleNamespace(cuda_stream=0x5000)
    assert _stream_ptr(null, True).value == 1
    assert _stream_ptr(null).value is None
    assert _stream_ptr(other, True).value == 0x5000 and _stream_ptr(other).value == 0x5000
    assert _stream_ptr(None, True) is None


def test_matcher_argument_checks_before_the_device():
    """orbx_search_for_initialization / orbx_search_by_sim3 reject bad arguments before any HIP call
    (ORBX_ERR_ARG / ORBX_ERR_CAPACITY), and a valid call without a GPU fails loudly (ORBX_ERR_NODEV)."""
    import ctypes as C

    import numpy as np
    from orb_slam2_commit_amd import _lib
    from orb_slam2_commit_amd._lib import KEYPOINT_DTYPE, ptr
    L = _lib.lib()
    assert L.orbx_search_for_initialization(None, 0) == -1
    assert L.orbx_search_by_sim3(None, 0) == -1

    def init_problem(n, octave=0):
        keys = np.zeros(n, KEYPOINT_DTYPE)
        keys["octave"] = octave
        desc = np.zeros((n, 32), np.uint8)
        prev = np.zeros((n, 2), np.float32)
        m = np.zeros(max(n, 1), np.int32)
        nm = np.zeros(1, np.int32)
        p = _lib.InitProblem()
        for f in (p.f1, p.f2):
            f.n, f.keys_un, f.desc = n, ptr(keys), ptr(desc)
            f.grid_inv_w = f.grid_inv_h = 0.05
        p.prev_matched, p.window, p.nnratio, p.check_ori, p.match12, p.nmatches = ptr(prev), 100, 0.9, 1, ptr(m), ptr(nm)
        return p, (keys, desc, prev, m, nm)

    p, keep = init_problem(8193)
    assert L.orbx_search_for_initialization(C.byref(p), 0) == -2
    p, keep = init_problem(10, octave=-1)
    assert L.orbx_search_for_initialization(C.byref(p), 0) == -1
    p, keep = init_problem(10)
    p.window = -1
    assert L.orbx_search_for_initialization(C.byref(p), 0) == -1
    p.window = 100
    assert L.orbx_search_for_initialization(C.byref(p), 0) == -4
    s = _lib.Sim3Problem()
    m12, nf = np.zeros(1, np.int32), np.zeros(1, np.int32)
    s.match12, s.nfound, s.s12 = ptr(m12), ptr(nf), 0.0
    assert L.orbx_search_by_sim3(C.byref(s), 0) == -1
