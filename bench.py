"""Benchmark: frames/sec ORB extract+match on KITTI-00-shaped stereo (BASELINE.json configs[1])
+ LocalBA iterations/sec on the KITTI-00 LocalBundleAdjustment problem (configs[3]).

One "step" = one pass of the hot path over one batch of B synthetic stereo
frames resident in HBM: ORB extraction of the 2B images (1241x376, 2000
features, 8 levels x1.2, FAST 20/7) + Frame::ComputeStereoMatches of the B
frames, all inside liborbx.so (orbx_stereo_frames_device).  `value` is that
frames/s.  The LocalBA leg then runs Optimizer::LocalBundleAdjustment
(orbx_ba_run) on a synthetic 20-KF / ~7.4k-point / ~43k-edge problem per rank,
--ba-calls times, and reports LM iterations/s (whole job) under "localba".

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

For N>1 the driver launches one rank per GPU with torch.distributed.run;
frames shard across ranks with no data-path collective ("weak" scaling), the
timed region is bracketed by barrier + synchronize and the max over ranks is
reported.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match (2k kp) + LocalBA iters/sec, KITTI-00 stereo"
KITTI = dict(width=1241, height=376, nfeatures=2000, fx=718.856, bf=386.1448)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="stereo frames per step per GPU")
    ap.add_argument("--unique", type=int, default=16, help="seeded synthetic stereo scenes per rank (slots are distinct rolls of them)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ba-calls", type=int, default=10, help="timed LocalBA calls per rank (0: skip)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (tools/profile.py); null if absent")
    return ap.parse_args()


def level_sizes(w, h, inv_scales):
    """ComputePyramid level sizes: cvRound((float)cols * mvInvScaleFactor[l]) (src/ORBextractor.cc:1219-1221)."""
    return [(int(np.rint(np.float32(w) * np.float32(s))), int(np.rint(np.float32(h) * np.float32(s))))
            for s in inv_scales]


def algorithmic_bytes(stage, n_img, n_frames, P, kps_per_img, acc_per_frame, cand_per_img):
    """Algorithmic HBM bytes of one launch of `stage` over the batch."""
    sP = sum(P)
    if stage == "k_resize":  # per launch average over the 7 level launches: read P_{l-1} + write P_l
        return n_img * sum(P[l - 1] + P[l] for l in range(1, len(P))) / (len(P) - 1)
    if stage == "k_fast":  # every level pixel read once + 4-B candidates written
        return n_img * (sP + 4 * cand_per_img)
    if stage == "k_blur":  # every level pixel read + written once
        return n_img * 2 * sP
    if stage == "k_octree":  # 4-B candidates read + 4-B selections written
        return n_img * (4 * cand_per_img + 4 * kps_per_img)
    if stage == "k_describe":  # raw + blurred levels read, 4-B selection read, 28-B kp + 32-B desc written
        return n_img * (2 * sP + 64 * kps_per_img)
    if stage == "k_stereo_match":  # per frame: NL*(32+28+8) + NR*(32+28) + Nacc*352
        return n_frames * (kps_per_img * 68 + kps_per_img * 60 + acc_per_frame * 352)
    if stage == "k_stereo_prep":
        return n_frames * kps_per_img * (28 + 8)
    if stage == "k_stereo_finalize":
        return n_frames * kps_per_img * 12
    return None


def cpu_baseline(pairs, seconds):
    """Single-thread CPU restatement (oracle/) on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    p = oracle.params(KITTI["nfeatures"], 1.2, 8, 20, 7)
    bf, fx = KITTI["bf"], KITTI["fx"]
    n = 0
    t0 = time.perf_counter()
    while True:
        L, R = pairs[n % len(pairs)]
        oL, oR = oracle.extract(p, L), oracle.extract(p, R)
        oracle.stereo_match(p, oL, oR, bf, bf / fx)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 3:
            break
    return dict(value=round(n / el, 3), unit="frames/s", cores=1, kind="port",
                sample="%d KITTI-shaped stereo frames (extract L + extract R + stereo match), oracle/ C++ "
                       "restatement, 1 thread, %.1f s" % (n, el))


def localba_leg(args, rank, world, dev, odist):
    """Optimizer::LocalBundleAdjustment on the config-4 problem: whole-job LM iterations/s."""
    import torch
    from orb_slam2_commit_amd import Optimizer, synth
    P = synth.localba_problem(seed=7 + 1000 * rank)
    opt = Optimizer(dev.index)
    r = opt.LocalBundleAdjustment(P)  # warm-up: allocations, code objects
    odist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    its = 0
    for _ in range(args.ba_calls):
        r = opt.LocalBundleAdjustment(P)
        its += sum(r["iterations"])
    torch.cuda.synchronize(dev)
    odist.barrier()
    el = odist.max_over_ranks(time.perf_counter() - t0, dev)
    its_all = odist.sum_over_ranks(float(its), dev)
    opt.close()
    out = dict(iters_per_s=round(its_all / el, 2), ms_per_call=round(el / args.ba_calls * 1e3, 3),
               calls_per_gpu=args.ba_calls, iterations=list(r["iterations"]), trials=r["trials"],
               problem=dict(keyframes=int(len(P["Tcw"])), fixed=int(np.sum(P["fixed"])),
                            points=int(len(P["Xw"])), edges=int(len(P["edge_point"])),
                            stereo_edges=int(np.sum(P["obs"][:, 2] >= 0))),
               dtype="f64", scaling="weak", cpu_baseline=None)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        n, t0 = 0, time.perf_counter()
        cits = 0
        while True:
            cr = oracle.local_ba(P)
            cits += sum(cr["iterations"])
            n += 1
            cel = time.perf_counter() - t0
            if cel >= 2.0 and n >= 2:
                break
        out["cpu_baseline"] = dict(value=round(cits / cel, 2), unit="LM iterations/s", cores=1, kind="port",
                                   sample="%d LocalBA calls on the same problem, oracle/localba.cpp, 1 thread, "
                                          "%.1f s" % (n, cel))
    return out


def main():
    args = parse()
    import torch

    from orb_slam2_commit_amd import dist as odist
    rank, local, world = odist.env_rank()
    # RCCL ("nccl") over xGMI; ORBX_DIST_BACKEND=gloo rehearses the multi-rank flow on a box with
    # fewer GPUs than ranks (ranks then wrap onto the available devices; collectives on CPU tensors)
    odist.init(os.environ.get("ORBX_DIST_BACKEND", "nccl"), rank, world)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from orb_slam2_commit_amd import ORBextractor, synth
    from orb_slam2_commit_amd import _lib

    W, H, B = KITTI["width"], KITTI["height"], args.batch
    # synthetic frames: distinct seeds per rank (frame shards), tiled into the batch
    pairs = [synth.stereo_pair(seed, W, H) for seed in odist.frame_seeds(rank, args.unique)]
    # every batch slot distinct: slot f is pair f % U rolled horizontally by 53 * (f // U) px
    # (L and R alike, so the disparity field is kept), so no two slots share bytes in HBM
    U = len(pairs)
    host = np.stack([np.roll(pairs[f % U][k], 53 * (f // U), axis=1) for f in range(B) for k in (0, 1)])
    images = torch.from_numpy(host).to(dev)
    ex = ORBextractor(KITTI["nfeatures"], 1.2, 8, 20, 7, device=local)
    cap = ex.max_keypoints(W, H)
    kps = torch.empty((2 * B, cap, 28), dtype=torch.uint8, device=dev)
    desc = torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    uR = torch.empty((B, cap), dtype=torch.float32, device=dev)
    depth = torch.empty((B, cap), dtype=torch.float32, device=dev)
    nmatch = torch.zeros(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    bf, baseline = KITTI["bf"], KITTI["bf"] / KITTI["fx"]

    def step():
        ex.stereo_frames_device(images, kps, desc, counts, bf, baseline, uR, depth, nmatch, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    L = _lib.lib()
    L.orbx_profile_reset(ex._h)
    L.orbx_profile_enable(ex._h, 1)
    odist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    odist.barrier()
    elapsed = time.perf_counter() - t0
    L.orbx_profile_enable(ex._h, 0)
    elapsed = odist.max_over_ranks(elapsed, dev)

    # per-stage live HIP-event timings on the stream the kernels ran on
    import ctypes as C
    stages = {}
    for s in range(L.orbx_profile_read(ex._h, -1, None, None, None)):
        ms, n, name = C.c_double(), C.c_longlong(), C.c_char_p()
        L.orbx_profile_read(ex._h, s, C.byref(ms), C.byref(n), C.byref(name))
        if n.value:
            stages[name.value.decode()] = (ms.value, n.value)
    cnt = counts.cpu().numpy()
    nm = nmatch.cpu().numpy()
    kps_per_img = float(cnt.mean())
    acc_per_frame = float(nm.mean())  # surviving matches (lower bound of SAD refinements)
    # candidates per image (FAST survivors) from the last batch
    ncand = L.orbx_debug_copy(ex._h, 2, 0, 0, None, 0) // 4
    cc = np.zeros(ncand, np.int32)
    L.orbx_debug_copy(ex._h, 2, 0, 0, _lib.ptr(cc), cc.nbytes)
    cand_per_img = float(cc.sum())
    P = [w * h for (w, h) in level_sizes(W, H, ex.GetInverseScaleFactors())]
    dom = max(stages, key=lambda k: stages[k][0]) if stages else None
    roofline = None
    if dom:
        ms_tot, nl = stages[dom]
        avg_s = ms_tot / nl / 1e3
        nbytes = algorithmic_bytes(dom, 2 * B, B, P, kps_per_img, acc_per_frame, cand_per_img)
        achieved = nbytes / avg_s / 1e9
        traffic = None
        if os.path.exists(args.traffic):
            try:
                traffic = json.load(open(args.traffic)).get("per_launch_bytes", {}).get(dom)
            except Exception:
                traffic = None
        roofline = dict(bound="hbm", kernel=dom, achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 5), traffic=traffic,
                        algorithmic_bytes_per_launch=int(nbytes), avg_launch_ms=round(avg_s * 1e3, 4))

    # every stage against the same HBM roofline (algorithmic bytes / average launch time)
    stage_hbm = {}
    for k, (ms_tot, nl) in stages.items():
        nb = algorithmic_bytes(k, 2 * B, B, P, kps_per_img, acc_per_frame, cand_per_img)
        if nb:
            gbs = nb / (ms_tot / nl / 1e3) / 1e9
            stage_hbm[k] = {"GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}

    value = odist.job_throughput(B, args.steps, world, elapsed)
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (%d seeded stereo scenes per rank, each batch slot a distinct horizontal roll of one)" % args.unique,
        "config": {"workload": "KITTI-00 stereo 1241x376, 2000 features, extract L+R + ComputeStereoMatches",
                   "batch_frames_per_gpu": B, "global_batch_frames": B * world, "nlevels": 8,
                   "scale_factor": 1.2, "fast_th": [20, 7], "parallelism": "frame-sharded x%d" % world},
        "roofline": roofline,
        "stage_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in stages.items()},
        "stage_hbm": stage_hbm,
        "keypoints_per_image": round(kps_per_img, 1),
        "stereo_matches_per_frame": round(acc_per_frame, 1),
        "localba_iters_per_s": None,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pairs, args.cpu_baseline_seconds)
    if args.ba_calls > 0:
        out["localba"] = localba_leg(args, rank, world, dev, odist)
        out["localba_iters_per_s"] = out["localba"]["iters_per_s"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
