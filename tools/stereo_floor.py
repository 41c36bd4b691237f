"""Unique-sector floor of the stereo refinement's row reads (probe build; GPU box).

Runs the bench's stereo workload (B KITTI-sized stereo pairs per step through
ORBextractor.stereo_frames_device) with the ORBX_STEREO_ROWS_PROBE library
(ORBX_LIB_OVERRIDE=build_ab/rowsprobe/liborbx.so) and reads orbx_debug_stereo_floor after each
step: the 64-B sectors and 128-B lines the 11 + 11 SAD rows of every staged keypoint touch, each
counted once per step.  Prints per-step means beside SURVEY 8(d)'s B_st for the same step.
The probe's k_stereo_rows_only (the staging loads alone, in k_stereo_match's pattern) is measured
by a FETCH_SIZE pass of the same command (tools/traffic_now.sh with this script).
usage: ORBX_LIB_OVERRIDE=... python tools/stereo_floor.py [steps]
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main(steps=3):
    import torch

    from orb_slam2_commit_amd import ORBextractor, _lib, synth

    L = _lib.lib()
    if not hasattr(L, "orbx_debug_stereo_floor"):
        raise SystemExit("not a probe build (set ORBX_LIB_OVERRIDE to build_ab/rowsprobe/liborbx.so)")
    fn = L.orbx_debug_stereo_floor
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    fn.restype = C.c_int
    K = bench.KITTI
    W, H, B = K["width"], K["height"], 256
    dev = torch.device("cuda", 0)
    pairs = [synth.stereo_pair(s, W, H) for s in synth.sequence_seeds(0, 16)]
    images = torch.from_numpy(synth.stereo_batch(0, B, pairs=pairs)).to(dev)
    ex = ORBextractor(K["nfeatures"], 1.2, 8, 20, 7, device=0)
    cap = ex.max_keypoints(W, H)
    kps = torch.empty((2 * B, cap, 28), dtype=torch.uint8, device=dev)
    desc = torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    uR = torch.empty((B, cap), dtype=torch.float32, device=dev)
    depth = torch.empty((B, cap), dtype=torch.float32, device=dev)
    nmatch = torch.zeros(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    out = (C.c_ulonglong * 3)()
    ex.stereo_frames_device(images, kps, desc, counts, K["bf"], K["bf"] / K["fx"], uR, depth, nmatch, stream)
    torch.cuda.synchronize(dev)
    fn(out)  # discard the warm-up step
    tot = [0, 0, 0]
    for _ in range(steps):
        ex.stereo_frames_device(images, kps, desc, counts, K["bf"], K["bf"] / K["fx"], uR, depth, nmatch, stream)
        torch.cuda.synchronize(dev)
        if fn(out) != 0:
            raise SystemExit("orbx_debug_stereo_floor failed")
        for i in range(3):
            tot[i] += out[i]
    cnt = counts.cpu().numpy()
    nm = nmatch.cpu().numpy()
    n_frames = B
    kps_per_img = float(cnt.mean())
    acc = float(nm.mean())
    b_st = n_frames * bench.s8d_stereo_frame(kps_per_img, kps_per_img, acc)
    sec, lines, staged = (t / steps for t in tot)
    print(json.dumps(dict(
        frames_per_step=n_frames, keypoints_per_image=round(kps_per_img, 1), accepted_per_frame=round(acc, 1),
        staged_keypoints_per_step=round(staged), unique_sectors_64B_per_step=round(sec),
        unique_lines_128B_per_step=round(lines),
        floor_bytes_64B_sectors=round(sec * 64), floor_bytes_128B_lines=round(lines * 128),
        rows_bytes_compact=round(staged * 352), B_st_bytes=round(b_st),
        note="unique 64-B sectors / 128-B lines touched by the 11 left + 11 right SAD rows of every staged "
             "keypoint, each counted once per step (bitmaps over the input and pyramid buffers of both sides)")))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
