"""Time SearchByProjection (GPU, batched frames, device-resident) beside the oracle (one host thread).

One "frame" = one problem on a KITTI-shaped Frame (2000 keypoints):
  local : Tracking::SearchLocalPoints -- isInFrustum + SearchByProjection(F, localMapPoints, th=1)
          over 3000 local MapPoints (fused, frustum=1)
  last  : SearchByProjection(F, LastFrame, th=7, stereo) over 2000 last-frame MapPoints
  kf    : SearchByProjection(F, pKF, sFound, th=10, ORBdist=100) over 2000 KF MapPoints
B problems (16 distinct, tiled) run as one orbx_search_by_projection_device launch; the time is
HIP-event time on the launch stream over `reps` launches."""
import ctypes as C
import json
import sys
import time

import numpy as np

ROOT = __file__.rsplit("/tools/", 1)[0]
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/oracle")
from orb_slam2_commit_amd import _lib, synth  # noqa: E402
from orb_slam2_commit_amd.orb import proj_problem  # noqa: E402

KINDS = {
    "local": (0, dict(th=1.0, nnratio=0.8, frustum=True), 3000),
    "last": (1, dict(th=7.0, nnratio=0.6), 2000),
    "kf": (2, dict(th=10.0, nnratio=0.6, orb_dist=100), 2000),
}


def build(kind_name, distinct, batch, dev):
    import torch
    kind, kw, npnt = KINDS[kind_name]
    base = []
    for b in range(distinct):
        fr = synth.projection_frame(500 + b, n=2000)
        pts = synth.projection_points(600 + b, fr, kind, n_points=npnt)
        k = dict(kw)
        if kind == 1:
            k["last_Tcw"] = fr["Tcw"]
        base.append((fr, pts, k))
    probs, keep = [], []
    for b in range(batch):
        fr, pts, k = base[b % distinct]
        dfr = dict(fr)
        for key in ("keys_un", "desc", "u_right", "occ"):
            dfr[key] = torch.from_numpy(np.ascontiguousarray(fr[key]).view(np.uint8)).to(dev)
        dpts = {key: (torch.from_numpy(np.ascontiguousarray(v)).to(dev) if isinstance(v, np.ndarray) else v)
                for key, v in pts.items()}
        outs = dict(frame_out=torch.empty(2000, dtype=torch.int32, device=dev),
                    point_match=torch.empty(npnt, dtype=torch.int32, device=dev),
                    nmatches=torch.empty(1, dtype=torch.int32, device=dev),
                    track=torch.zeros((npnt, 4), dtype=torch.float32, device=dev),
                    track_level=torch.zeros(npnt, dtype=torch.int32, device=dev))
        p, _ = proj_problem(dfr, dpts, kind, outputs=outs, **k)
        probs.append(p)
        keep.append((dfr, dpts, outs))
    return base, (_lib.ProjProblem * batch)(*probs), keep


def main(batch=256, reps=20, cpu_frames=16):
    import torch
    dev = torch.device("cuda:0")
    torch.cuda.init()
    out = {}
    for name in KINDS:
        base, arr, keep = build(name, 16, batch, dev)
        s = torch.cuda.current_stream()
        sp = C.c_void_p(s.cuda_stream)
        L = _lib.lib()
        for _ in range(3):
            _lib.check(L.orbx_search_by_projection_device(arr, batch, sp), "warmup")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            L.orbx_search_by_projection_device(arr, batch, sp)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        nm = [int(k[2]["nmatches"].cpu()[0]) for k in keep[:16]]
        import oracle
        kind, kw, _ = KINDS[name]
        t0 = time.perf_counter()
        for i in range(cpu_frames):
            fr, pts, k = base[i % 16]
            r = oracle.search_by_projection(fr, pts, kind, **k)
            assert r["nmatches"] == nm[i % 16], (name, r["nmatches"], nm[i % 16])
        cpu_s = (time.perf_counter() - t0) / cpu_frames
        out[name] = dict(batch=batch, ms_per_launch=round(ms, 4), gpu_frames_per_s=round(batch / ms * 1e3, 1),
                         oracle_frames_per_s=round(1.0 / cpu_s, 1), mean_matches=float(np.mean(nm)),
                         note="oracle time includes ctypes marshalling of the frame (~5%)")
    print(json.dumps(out))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
