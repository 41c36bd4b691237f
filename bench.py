"""Benchmark: frames/sec ORB extract+match on KITTI-00-shaped stereo (BASELINE.json configs[1])
+ LocalBA iterations/sec on the KITTI-00 LocalBundleAdjustment problem (configs[3])
+ the config-5 sequence pipeline with its RCCL all-gather (configs[4]).

One "step" = one pass of the hot path over one batch of B synthetic stereo
frames resident in HBM: ORB extraction of the 2B images (1241x376, 2000
features, 8 levels x1.2, FAST 20/7) + Frame::ComputeStereoMatches of the B
frames, all inside liborbx.so (orbx_stereo_frames_device).  `value` is that
frames/s, from an un-instrumented loop (HIP events around each batch only) with --inflight
batches in flight on their own extractor handles and HIP streams; the per-stage split and the
roofline come from a second, profiled pass of one handle alone.

Legs after the headline loop:
  config3   EuRoC-shaped stereo + PnP RANSAC per frame (configs[2]): extract+match of a frame batch
            (one frame per synthetic sequence) and one batched orbx_pnp_iterate_many over their solvers.
  localba   Optimizer::LocalBundleAdjustment (orbx_ba_run) on the config-4 problem
            per rank, --ba-calls times: LM iterations/s (whole job) + its roofline.
  config5   one synthetic sequence per rank: extract+match of --pipeline-steps
            batches of distinct frames into frame-record arenas, a keyframe every
            --kf-every frames whose config-4-sized LocalBA runs on the rank's
            LocalMapping thread (own stream) overlapping the extraction, then ONE
            all-gather of the records + LocalBA summaries (RCCL over xGMI); the
            sequence, its parts alone and the all-gather timed separately.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

Ranks: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) every rank checks
WORLD_SIZE == --gpus and fails otherwise.  Started plainly with --gpus N > 1 (no WORLD_SIZE), the
process is only a launcher: before any torch.cuda / HIP call it starts
`python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py
<same args>` as a CHILD process (never exec), lets the ranks' output through and exits with the
child's exit code.  Under RCCL (the default backend) N must not exceed the visible GPUs;
ORBX_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks wrap onto the devices).
Frames shard across ranks with no data-path collective in the headline loop ("weak" scaling),
the timed region is bracketed by barrier + synchronize and the max over ranks is reported.
Rank 0 prints ONE JSON line; `n_gpus` is the number of ranks that ran, `config.devices_used` the
distinct GPUs they used (gathered from the ranks), `config.dist_backend` the process-group backend.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match (2k kp) + LocalBA iters/sec, KITTI-00 stereo"
KITTI = dict(width=1241, height=376, nfeatures=2000, fx=718.856, bf=386.1448)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured float4 copy)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="stereo frames per step per GPU")
    ap.add_argument("--inflight", type=int, default=4, help="batches in flight (extractor handles / HIP streams)")
    ap.add_argument("--unique", type=int, default=16, help="seeded synthetic stereo scenes per rank (slots are distinct rolls of them)")
    ap.add_argument("--profile-steps", type=int, default=5, help="steps of the second, per-stage profiled pass")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ba-calls", type=int, default=40, help="timed LocalBA calls per rank (0: skip)")
    ap.add_argument("--ba-concurrent", type=int, default=8, help="LocalBA problems in flight per GPU for the "
                                                                  "throughput form (<=1: skip)")
    ap.add_argument("--pipeline-steps", type=int, default=4, help="config-5 batches of distinct frames per rank (0: skip)")
    ap.add_argument("--c5-ba-cus", type=int, default=0, help="config 5: CUs reserved for LocalMapping's LocalBA "
                                                                 "stream, the rest for extraction (0: shared)")
    ap.add_argument("--c5-cu-layout", default="contiguous", choices=["contiguous", "strided"])
    ap.add_argument("--c5-depth", type=int, default=0, help="config-5 batches queued ahead of the host "
                                                               "(0: all at once)")
    ap.add_argument("--kf-every", type=int, default=128, help="config-5 keyframe cadence: one keyframe (and its "
                                                                 "LocalBA) every K frames of a sequence (0: none)")
    ap.add_argument("--single-frames", type=int, default=200, help="frames of the single-frame drop-in leg (0: skip)")
    ap.add_argument("--track-steps", type=int, default=5, help="steps of the extract+match+track leg (0: skip)")
    ap.add_argument("--c1-batch", type=int, default=256, help="config-1 (TUM mono) images per batched launch (0: skip leg)")
    ap.add_argument("--c1-seconds", type=float, default=6.0, help="config-1 CPU reference sample length")
    ap.add_argument("--c3-steps", type=int, default=3, help="config-3 (EuRoC + PnP RANSAC) steps per rank (0: skip)")
    ap.add_argument("--c3-batch", type=int, default=128, help="config-3 frames (sequences) per step per GPU")
    ap.add_argument("--sq", default=os.path.join(ROOT, "profiles", "r06_sq_counters.json"),
                    help="SQ counter summary (tools/pmc_kernel.sh + tools/sq_summary.py) for issue fractions")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (tools/profile.sh + tools/parse_prof.py); null if absent")
    ap.add_argument("--rocprof", default=os.path.join(ROOT, "profiles", "r06_rocprof_stages.json"),
                    help="per-stage kernel time per step from rocprofv3 --stats (tools/rocprof_stages.py)")
    ap.add_argument("--ba-traffic", default=os.path.join(ROOT, "profiles", "r06_localba_traffic.json"),
                    help="LocalBA PMC bytes per LM iteration (tools/ba_traffic.py); null if absent")
    ap.add_argument("--stereo-floor", default=os.path.join(ROOT, "profiles", "r05_stereo_floor.json"),
                    help="measured sector floor of the stereo stage (tools/stereo_floor.py); null if absent")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(gpus, argv, port):
    """The torch.distributed.run command line that runs this script as `gpus` ranks on one node
    (the driver contract's own form: --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def rank_plan(args, env=None):
    """What this process is: ("rank", world) when it runs the benchmark itself, ("launch", N) when it
    must start N ranks.  Raises SystemExit when WORLD_SIZE and --gpus disagree (a driver that asked
    for N GPUs must never get a silent run of a different size).  Pure: reads no GPU state."""
    env = os.environ if env is None else env
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1 (got %d)" % args.gpus)
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != args.gpus:
            raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d: the launcher and the flag disagree"
                             % (world, args.gpus))
        return "rank", world
    if args.gpus == 1:
        return "rank", 1
    return "launch", args.gpus


def launch_ranks(args, argv):
    """Start the N-rank run as a child process (no exec: nothing here has touched the GPU, and the
    pool forbids replacing a process anyway) and return its exit code.  The ranks inherit stdout,
    so rank 0's JSON line is the launcher's output."""
    backend = os.environ.get("ORBX_DIST_BACKEND", "nccl")
    if backend != "gloo":
        import torch  # device_count() does not initialise the GPU on this image
        ndev = torch.cuda.device_count()
        if args.gpus > ndev:
            raise SystemExit("bench.py --gpus %d: only %d GPU(s) visible (RCCL needs one GPU per rank; "
                             "ORBX_DIST_BACKEND=gloo rehearses more ranks on fewer GPUs)" % (args.gpus, ndev))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    cmd = launcher_cmd(args.gpus, argv, _free_port())
    print("bench.py: launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def level_sizes(w, h, inv_scales):
    """ComputePyramid level sizes: cvRound((float)cols * mvInvScaleFactor[l]) (src/ORBextractor.cc:1219-1221)."""
    return [(int(np.rint(np.float32(w) * np.float32(s))), int(np.rint(np.float32(h) * np.float32(s))))
            for s in inv_scales]


def hbm_copy_peak(dev, nbytes=2 << 30, reps=10):
    """On-box HBM reference: a streaming 16-B copy kernel between two 2 GiB device buffers
    (orbx_debug_hbm_copy; read + write bytes per copy / time), the stream-copy figure the
    spec's 8 TB/s is compared against."""
    import ctypes as C
    import torch
    from orb_slam2_commit_amd import _lib
    try:
        with torch.cuda.device(dev):
            src = torch.ones(nbytes, dtype=torch.uint8, device=dev)
            dst = torch.empty_like(src)
            torch.cuda.synchronize(dev)
            ms = C.c_float(0)
            if _lib.lib().orbx_debug_hbm_copy(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()),
                                              nbytes, reps, C.byref(ms)) != 0:
                return None
            del src, dst
        return round(2 * nbytes / (ms.value / 1e3) / 1e9, 1)
    except Exception:
        return None


# SURVEY.md §8(d) algorithmic bytes.  Extraction, per image:
#   B_ext = 2*P0 + sum_{l=1..7}(P_{l-1} + P_l) + 4*sum(P) + 60*N
# (input read + L0 write; resize read + write; FAST read + orientation read + blur read/write +
# descriptor read; 28-B keypoint + 32-B descriptor written).  Stereo, per frame:
#   B_st = N_L*68 + N_R*60 + N_acc*352
# Each kernel is charged the §8(d) terms it performs and nothing else (its own intermediates --
# FAST candidates, octree selections, the stereo kernels' sorted copies and range tables -- are not
# algorithmic bytes).  The input copy 2*P0 is never performed (level 0 IS the caller's image), so no
# kernel carries it, but the whole-step figure keeps it, as §8(d) defines B_ext.
STAGE_EVENTS_PER_STEP = {"k_resize": 7}  # per-stage timer events per step (k_resize: one per level)


def s8d_stage_bytes(stage, n_img, n_frames, P, kps_per_img, acc_per_frame):
    """§8(d) bytes of ONE timer event of `stage` over the batch (None: no §8(d) term, e.g. k_octree)."""
    sP = sum(P)
    if stage == "k_resize":  # average over the 7 level launches: read P_{l-1} + write P_l
        return n_img * sum(P[l - 1] + P[l] for l in range(1, len(P))) / (len(P) - 1)
    if stage == "k_fast":  # the FAST read of every level
        return n_img * sP
    if stage == "k_blur":  # (debug launches only) blur read + write of every level
        return n_img * 2 * sP
    if stage == "k_describe":  # orientation read of the raw level + rBRIEF read of the blurred level + 60 B out
        return n_img * (2 * sP + 60 * kps_per_img)
    if stage == "stereo":  # k_stereo_prep + k_stereo_match + k_stereo_finalize together: B_st
        return n_frames * s8d_stereo_frame(kps_per_img, kps_per_img, acc_per_frame)
    return None


def s8d_stereo_frame(n_l, n_r, n_acc):
    return n_l * 68 + n_r * 60 + n_acc * 352


def s8d_frame_bytes(P, kps_per_img, acc_per_frame):
    """§8(d) bytes of one stereo frame: 2 * B_ext + B_st."""
    sP = sum(P)
    b_ext = 2 * P[0] + sum(P[l - 1] + P[l] for l in range(1, len(P))) + 4 * sP + 60 * kps_per_img
    return 2 * b_ext + s8d_stereo_frame(kps_per_img, kps_per_img, acc_per_frame)


STEREO_KERNELS = ("k_stereo_prep", "k_stereo_match", "k_stereo_finalize")


def rocprof_stage_ms(path):
    """Per-step kernel time of each bench stage from a committed rocprofv3 --stats summary
    (tools/rocprof_stages.py: TotalDurationNs of every dispatch of the stage / the profiled steps)."""
    if not path or not os.path.exists(path):
        return {}, None
    try:
        j = json.load(open(path))
        return {k: v["ms_per_step"] for k, v in j["stages"].items()}, dict(
            file=os.path.relpath(path, ROOT), head=j.get("head"), steps=j.get("steps"), command=j.get("command"))
    except Exception:  # noqa: BLE001 -- evidence is reported, never fatal
        return {}, None


def pct(xs, q):
    return float(np.percentile(np.asarray(xs, np.float64), q))


# ------------------------------------------------------------------ CPU baseline (oracle = checker)
def host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    return dict(cpu_model=model, nproc=os.cpu_count(), cpus_allowed=len(aff) or None), aff


def native_oracle():
    """Compile the oracle sources with -O3 -march=native -ffp-contract=off for THIS host into a temp dir
    (SURVEY §8d baseline flags; the committed build is -O2 and portable).  Returns (path, flags) or
    (None, reason)."""
    src = os.path.join(ROOT, "oracle")
    srcs = ["orb_oracle.cpp", "localba.cpp", "pnp.cpp", "voc.cpp", "projection.cpp", "poseopt.cpp",
            "triangulation.cpp", "mapping.cpp"]
    if not all(os.path.exists(os.path.join(src, s)) for s in srcs):
        return None, "oracle sources absent"
    flags = ["-O3", "-march=native", "-std=c++17", "-fPIC", "-ffp-contract=off"]
    d = tempfile.mkdtemp(prefix="orbx_oracle_native_")
    try:
        procs = [subprocess.Popen(["g++"] + flags + ["-c", os.path.join(src, s), "-o", os.path.join(d, s + ".o")],
                                  stdout=subprocess.DEVNULL, stderr=subprocess.PIPE) for s in srcs]
        if any(p.wait(timeout=300) != 0 for p in procs):
            return None, "native oracle compile failed"
        out = os.path.join(d, "liborb_oracle_native.so")
        subprocess.check_call(["g++", "-shared", "-o", out] + [os.path.join(d, s + ".o") for s in srcs])
        return out, " ".join(flags)
    except Exception as e:  # noqa: BLE001 -- the baseline is reported, never fatal
        return None, "native oracle build error: %s" % e


def load_oracle():
    path, flags = native_oracle()
    if path:
        os.environ["ORBX_ORACLE_LIB"] = path
    else:
        flags = "-O2 -ffp-contract=off (committed oracle/build; %s)" % flags
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    return oracle, flags


def cpu_baseline(oracle, flags, pairs, seconds, cpus):
    """oracle/ C++ restatement on a bounded sample of the same workload: 1 thread pinned to one core
    (median/p90 per frame), plus the reference's 2-thread form (L and R extraction concurrently on two
    cores, src/Frame.cc:80-84, then stereo matching)."""
    p = oracle.params(KITTI["nfeatures"], 1.2, 8, 20, 7)
    bf, fx = KITTI["bf"], KITTI["fx"]
    old = os.sched_getaffinity(0) if hasattr(os, "sched_setaffinity") else None
    c0 = cpus[0] if cpus else 0
    c1 = cpus[1] if len(cpus) > 1 else c0
    try:
        if old is not None:
            os.sched_setaffinity(0, {c0})
        L, R = pairs[0]
        oracle.stereo_match(p, oracle.extract(p, L), oracle.extract(p, R), bf, bf / fx)  # warm-up
        times = []
        t_start = time.perf_counter()
        n = 0
        while True:
            L, R = pairs[n % len(pairs)]
            t0 = time.perf_counter()
            oL, oR = oracle.extract(p, L), oracle.extract(p, R)
            oracle.stereo_match(p, oL, oR, bf, bf / fx)
            times.append(time.perf_counter() - t0)
            n += 1
            if time.perf_counter() - t_start >= seconds and n >= 3:
                break
        el = sum(times)
        one = dict(value=round(n / el, 3), unit="frames/s", cores=1, kind="port",
                   median_ms=round(pct(times, 50) * 1e3, 2), p90_ms=round(pct(times, 90) * 1e3, 2),
                   sample="%d KITTI-shaped stereo frames (extract L + extract R + stereo match), oracle/ C++ "
                          "restatement built %s, 1 thread pinned to cpu %d, %.1f s" % (n, flags, c0, el))
        # 2-thread L/R (ctypes releases the GIL inside the oracle calls)
        res = [None, None]

        def ext(k, img, cpu):
            if old is not None:
                os.sched_setaffinity(0, {cpu})
            res[k] = oracle.extract(p, img)

        times2 = []
        n2 = 0
        t_start = time.perf_counter()
        while True:
            L, R = pairs[n2 % len(pairs)]
            t0 = time.perf_counter()
            th = [threading.Thread(target=ext, args=(0, L, c0)), threading.Thread(target=ext, args=(1, R, c1))]
            for t in th:
                t.start()
            for t in th:
                t.join()
            oracle.stereo_match(p, res[0], res[1], bf, bf / fx)
            times2.append(time.perf_counter() - t0)
            n2 += 1
            if time.perf_counter() - t_start >= seconds / 2 and n2 >= 3:
                break
        one["two_thread"] = dict(value=round(n2 / sum(times2), 3), unit="frames/s", cores=2,
                                 median_ms=round(pct(times2, 50) * 1e3, 2), p90_ms=round(pct(times2, 90) * 1e3, 2),
                                 sample="%d frames, L and R extraction on two threads pinned to cpus %d,%d "
                                        "(src/Frame.cc:80-84), then stereo match" % (n2, c0, c1))
        return one
    finally:
        if old is not None:
            os.sched_setaffinity(0, old)


# ------------------------------------------------------------------ LocalBA leg
def localba_bytes_per_iteration(P):
    """E*512 + M*360 + (6K)^2*16 algorithmic bytes per LM outer iteration."""
    E = len(P["edge_point"])
    M = len(P["Xw"])
    K = int(len(P["fixed"]) - np.sum(P["fixed"]))
    return E * 512 + M * 360 + (6 * K) ** 2 * 16


def ba_traffic(args):
    """PMC HBM bytes per LM iteration of the config-4 call (tools/ba_traffic.py), with its source."""
    try:
        j = json.load(open(args.ba_traffic))
        return dict(bytes_per_iteration=j["bytes_per_iteration"], source=os.path.relpath(args.ba_traffic, ROOT),
                    head=j.get("head"))
    except Exception:  # noqa: BLE001 -- absent evidence is reported as null
        return None


def localba_leg(args, rank, world, dev, odist, oracle_mod=None, flags=None, cpus=None):
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
    call_ms = []
    for _ in range(args.ba_calls):
        c0 = time.perf_counter()
        r = opt.LocalBundleAdjustment(P)  # returns after its final readback (host-synchronous)
        call_ms.append((time.perf_counter() - c0) * 1e3)
        its += sum(r["iterations"])
    torch.cuda.synchronize(dev)
    odist.barrier()
    el_local = time.perf_counter() - t0
    el = odist.max_over_ranks(el_local, dev)
    its_all = odist.sum_over_ranks(float(its), dev)
    opt.close()
    bpi = localba_bytes_per_iteration(P)
    it_s_local = its / el_local
    achieved = bpi * it_s_local / 1e9
    out = dict(iters_per_s=round(its_all / el, 2), ms_per_call=round(el / args.ba_calls * 1e3, 3),
               median_ms_per_call=round(pct(call_ms, 50), 3), p90_ms_per_call=round(pct(call_ms, 90), 3),
               calls_per_gpu=args.ba_calls, iterations=list(r["iterations"]), trials=r["trials"],
               problem=dict(keyframes=int(len(P["Tcw"])), fixed=int(np.sum(P["fixed"])),
                            points=int(len(P["Xw"])), edges=int(len(P["edge_point"])),
                            stereo_edges=int(np.sum(P["obs"][:, 2] >= 0))),
               roofline=dict(bound="hbm", achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                             frac=round(achieved / HBM_PEAK_GBS, 5), traffic=ba_traffic(args),
                             algorithmic_bytes_per_iteration=int(bpi),
                             note="SURVEY 8d bytes per LM iteration (E*512 + M*360 + (6K)^2*16) x iterations/s "
                                  "of this rank; the trial is a chain of ~12 dependent small launches "
                                  "(latency-bound; per-kernel split in profiles/*localba_kernel_stats.csv)"),
               dtype="f64", scaling="weak", cpu_baseline=None)
    if args.ba_concurrent > 1:
        # throughput form: K independent LocalBA problems in flight on this GPU (one solver handle, HIP
        # stream and host thread each -- K maps / sequences per GPU); a single problem leaves most CUs
        # idle (its trial is a chain of small dependent launches)
        K = args.ba_concurrent
        probs = [synth.localba_problem(seed=7 + 1000 * rank + 17 * k) for k in range(K)]
        opts = [Optimizer(dev.index) for _ in range(K)]
        for o, Pk in zip(opts, probs):
            o.LocalBundleAdjustment(Pk)
        kits = [0] * K

        def run(k):
            for _ in range(args.ba_calls):
                kits[k] += sum(opts[k].LocalBundleAdjustment(probs[k])["iterations"])

        th = [threading.Thread(target=run, args=(k,)) for k in range(K)]
        odist.barrier()
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize(dev)
        odist.barrier()
        elk = odist.max_over_ranks(time.perf_counter() - t0, dev)
        its_k = odist.sum_over_ranks(float(sum(kits)), dev)
        for o in opts:
            o.close()
        out["concurrent"] = dict(problems_per_gpu=K, iters_per_s=round(its_k / elk, 2),
                                 ms_per_call=round(elk / args.ba_calls * 1e3, 3),
                                 note="K independent config-4-shaped problems (different seeds) in flight per GPU, "
                                      "one host thread + HIP stream each; aggregate LM iterations/s")
        # the same K problems through ONE batched call (orbx_ba_run_many: every trial kernel once for all K)
        ob = Optimizer(dev.index)
        ob.LocalBundleAdjustmentMany(probs)
        odist.barrier()
        t0 = time.perf_counter()
        bits = 0
        for _ in range(args.ba_calls):
            bits += sum(sum(r["iterations"]) for r in ob.LocalBundleAdjustmentMany(probs))
        torch.cuda.synchronize(dev)
        odist.barrier()
        elb = odist.max_over_ranks(time.perf_counter() - t0, dev)
        its_b = odist.sum_over_ranks(float(bits), dev)
        ob.close()
        out["batched"] = dict(problems_per_call=K, iters_per_s=round(its_b / elb, 2),
                              ms_per_call=round(elb / args.ba_calls * 1e3, 3),
                              note="the same K problems in one orbx_ba_run_many call per round (one host thread, "
                                   "one stream; results bit-identical to K single calls)")
    if rank == 0 and world == 1 and oracle_mod is not None:
        old = os.sched_getaffinity(0) if hasattr(os, "sched_setaffinity") else None
        try:
            if old is not None and cpus:
                os.sched_setaffinity(0, {cpus[0]})
            n, cits, ct = 0, 0, []
            t0 = time.perf_counter()
            while True:
                c0 = time.perf_counter()
                cr = oracle_mod.local_ba(P)
                ct.append(time.perf_counter() - c0)
                cits += sum(cr["iterations"])
                n += 1
                if time.perf_counter() - t0 >= 3.0 and n >= 3:
                    break
        finally:
            if old is not None:
                os.sched_setaffinity(0, old)
        cel = sum(ct)
        out["cpu_baseline"] = dict(value=round(cits / cel, 2), unit="LM iterations/s", cores=1, kind="port",
                                   median_ms_per_call=round(pct(ct, 50) * 1e3, 2),
                                   p90_ms_per_call=round(pct(ct, 90) * 1e3, 2),
                                   sample="%d LocalBA calls on the same problem, oracle/localba.cpp built %s, "
                                          "1 thread pinned, %.1f s" % (n, flags, cel))
    return out


# ------------------------------------------------------------------ single-frame (drop-in) leg
def single_frame_leg(args, pairs, cpu):
    """The drop-in path as ORB-SLAM2 drives it: one stereo Frame per TrackStereo call on the Tracking
    thread (Examples/Stereo/stereo_kitti.cc:82-99 times that call), i.e. the C++ shim's Frame stereo
    constructor -- two extraction threads on two ORBextractor handles (src/Frame.cc:80-84),
    UndistortKeyPoints, ComputeStereoMatches -- from host images to host vectors
    (shim/build/frame_bench, a separate process; the Frame makes one orbx_frame_stereo call).  Reported
    beside the oracle's per-frame time."""
    exe = os.path.join(ROOT, "shim", "build", "frame_bench")
    if not os.path.exists(exe):
        return dict(error="shim/build/frame_bench not built")
    W, H = KITTI["width"], KITTI["height"]
    fd, path = tempfile.mkstemp(prefix="orbx_frames_", suffix=".u8")
    try:
        with os.fdopen(fd, "wb") as f:
            for L, R in pairs:
                f.write(np.ascontiguousarray(L).tobytes())
                f.write(np.ascontiguousarray(R).tobytes())
        cmd = [exe, path, str(W), str(H), str(len(pairs)), str(args.single_frames), "20", str(KITTI["nfeatures"]),
               repr(KITTI["bf"]), repr(KITTI["fx"])]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            return dict(error="frame_bench rc %d: %s" % (r.returncode, (r.stderr or r.stdout)[-300:]))
        out = json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        os.unlink(path)
    out.update(unit="ms per stereo frame (Frame constructor, host images in, host keypoints/descriptors/"
                    "uRight/depth out)", warmup_frames=20,
               path="shim Frame(imLeft, imRight, ...) -> one orbx_frame_stereo call (both ExtractORB as one "
                    "batch of two + ComputeStereoMatches on the device, one copy back) + UndistortKeyPoints")
    if cpu:
        out["cpu_baseline"] = dict(median_ms=cpu.get("median_ms"), p90_ms=cpu.get("p90_ms"),
                                   two_thread_median_ms=(cpu.get("two_thread") or {}).get("median_ms"),
                                   kind=cpu.get("kind"), note="the oracle's per-frame time from cpu_baseline")
    return out


# ------------------------------------------------------------------ config-1 leg
TUM = dict(width=640, height=480, nfeatures=1000)


def config1_leg(args, dev, oracle_mod, flags, cpus):
    """BASELINE configs[0]: TUM fr1_xyz-shaped mono 640x480, 1,000 features -- the unit is Frame's
    monocular constructor's ExtractORB, i.e. one ORBextractor::operator() (src/Frame.cc:186-205,
    :273-279; mono extractor built at src/Tracking.cc:120,125).  Three numbers: the CPU reference path
    (oracle operator() on one pinned core: the config's own "CPU reference ORBextractor" number), the
    drop-in per-call latency through the shim's ORBextractor::operator() (host image in, host keypoints
    and descriptors out, shim/build/frame_bench mono), and batched device extraction (--c1-batch TUM
    images per orbx_extract_batch launch, inputs resident in HBM)."""
    import torch
    from orb_slam2_commit_amd import ORBextractor, synth
    W, H, NF = TUM["width"], TUM["height"], TUM["nfeatures"]
    imgs = [synth.mono_image(1000 * 9 + s, W, H) for s in range(8)]
    out = dict(config=dict(workload="TUM fr1_xyz-shaped mono 640x480, 1000 features, ORBextractor::operator()",
                           nlevels=8, scale_factor=1.2, fast_th=[20, 7]),
               data="synthetic (8 seeded mono scenes; batched slots are distinct horizontal rolls of them)")
    # CPU reference path: one pinned core
    if oracle_mod is not None:
        p = oracle_mod.params(NF, 1.2, 8, 20, 7)
        old = os.sched_getaffinity(0) if hasattr(os, "sched_setaffinity") else None
        try:
            if old is not None and cpus:
                os.sched_setaffinity(0, {cpus[0]})
            oracle_mod.extract(p, imgs[0])
            ts, n, t_start = [], 0, time.perf_counter()
            while True:
                t0 = time.perf_counter()
                o = oracle_mod.extract(p, imgs[n % len(imgs)])
                ts.append(time.perf_counter() - t0)
                n += 1
                if time.perf_counter() - t_start >= args.c1_seconds and n >= 5:
                    break
        finally:
            if old is not None:
                os.sched_setaffinity(0, old)
        out["cpu_baseline"] = dict(value=round(n / sum(ts), 3), unit="frames/s", cores=1, kind="port",
                                   median_ms=round(pct(ts, 50) * 1e3, 3), p90_ms=round(pct(ts, 90) * 1e3, 3),
                                   keypoints_per_frame=len(o.keypoints),
                                   sample="%d TUM-shaped mono images, oracle operator() built %s, 1 thread pinned"
                                          % (n, flags))
    # drop-in: the shim's ORBextractor::operator() per call (separate process)
    exe = os.path.join(ROOT, "shim", "build", "frame_bench")
    if os.path.exists(exe) and args.single_frames > 0:
        fd, path = tempfile.mkstemp(prefix="orbx_mono_", suffix=".u8")
        try:
            with os.fdopen(fd, "wb") as f:
                for im in imgs:
                    f.write(np.ascontiguousarray(im).tobytes())
            cmd = [exe, path, str(W), str(H), str(len(imgs)), str(args.single_frames), "20", str(NF), "0", "1", "mono"]
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            if r.returncode == 0:
                out["drop_in"] = json.loads(r.stdout.strip().splitlines()[-1])
                out["drop_in"].update(unit="ms per ORBextractor::operator() call (host image in, host keypoints + "
                                           "descriptors out, mvImagePyramid refreshed)")
            else:
                out["drop_in"] = dict(error="frame_bench rc %d: %s" % (r.returncode, (r.stderr or r.stdout)[-300:]))
        finally:
            os.unlink(path)
    # batched device extraction
    B1 = args.c1_batch
    ex = ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index)
    cap = ex.max_keypoints(W, H)
    batch = torch.from_numpy(np.stack([np.roll(imgs[i % len(imgs)], 37 * (i // len(imgs)), axis=1)
                                       for i in range(B1)])).to(dev)
    kps = torch.empty((B1, cap, 28), dtype=torch.uint8, device=dev)
    desc = torch.empty((B1, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(B1, dtype=torch.int32, device=dev)
    st = torch.cuda.Stream(dev)
    for _ in range(2):
        ex.extract_batch_device(batch, kps, desc, counts, st)
    torch.cuda.synchronize(dev)
    steps = max(args.steps // 2, 3)
    t0 = time.perf_counter()
    for _ in range(steps):
        ex.extract_batch_device(batch, kps, desc, counts, st)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ex.close()
    out["batched"] = dict(frames_per_s=round(B1 * steps / el, 1), ms_per_step=round(el / steps * 1e3, 4),
                          batch_images=B1, steps=steps, batches_in_flight=1,
                          keypoints_per_image=round(float(counts.float().mean()), 1))
    return out


# ------------------------------------------------------------------ tracking front-end leg
def track_leg(args, rank, world, dev, odist, ex, images, stream, pairs_host, oracle_mod=None, cpus=None):
    """Extract+match a batch, then Tracking::TrackReferenceKeyFrame's front end (src/Tracking.cc:910-969)
    for its frames: ComputeBoW -> SearchByBoW(KF, F) (nnratio 0.7) -> PoseOptimization, all on the
    device (orb_slam2_commit_amd/tracking.py).  Frame f is tracked against frame f-U (the same scene
    53 px earlier: the batch holds U scenes, rolled), so B-U of the B frames are tracked per step.
    Synthetic DBoW2 vocabulary k=10, L=5 (ORBvoc.txt is not in the image: k=10, L=6), FeatureVector
    at levelsup 3 (the reference's levelsup 4 on L=6: the same node level, <= 100 nodes)."""
    import torch
    from orb_slam2_commit_amd import ORBVocabulary, synth
    from orb_slam2_commit_amd.tracking import TrackBatch
    W, H, B, U = KITTI["width"], KITTI["height"], args.batch, args.unique
    cap = ex.max_keypoints(W, H)
    text = synth.vocabulary(seed=5, k=10, L=5)[0]
    voc = ORBVocabulary(dev.index)
    voc.loadFromText(text)
    fx, bf = KITTI["fx"], KITTI["bf"]
    cx, cy = 607.1928, 185.2157
    tb = TrackBatch(voc, B, cap, ex.GetInverseScaleSigmaSquares(), fx, fx, cx, cy, bf, dev, levelsup=3)
    kps = torch.empty((2 * B, cap, 28), dtype=torch.uint8, device=dev)
    desc = torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    uR = torch.empty((B, cap), dtype=torch.float32, device=dev)
    depth = torch.empty((B, cap), dtype=torch.float32, device=dev)
    nmatch = torch.zeros(B, dtype=torch.int32, device=dev)
    pairs = [(f - U, f) for f in range(U, B)]
    bl = bf / fx

    def step(tim=None):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ex.stereo_frames_device(images, kps, desc, counts, bf, bl, uR, depth, nmatch, stream)
        e1.record(stream)
        r = tb.run(kps, desc, counts, uR, depth, pairs, stream, timings=tim)
        return r, (e0, e1)

    step()
    torch.cuda.synchronize(dev)
    odist.barrier()
    tim, evs = [], []
    t0 = time.perf_counter()
    for _ in range(args.track_steps):
        r, ev = step(tim)
        evs.append(ev)
    torch.cuda.synchronize(dev)
    odist.barrier()
    el = odist.max_over_ranks(time.perf_counter() - t0, dev)
    nmat, nedge, ngood = r
    em_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    tim = np.asarray(tim) * 1e3
    split = dict(extract_match_gpu=round(em_ms, 3), compute_bow_gpu=round(float(tim[:, 3].mean()), 3),
                 search_by_bow_and_gather_gpu=round(float(tim[:, 4].mean()), 3),
                 pose_optimization_gpu=round(float(tim[:, 5].mean()), 3))
    step_ms = el / args.track_steps * 1e3
    gpu_sum = sum(v for v in split.values())
    split.update(sum_gpu=round(gpu_sum, 3), frac_of_step=round(gpu_sum / step_ms, 4),
                 note="GPU time of contiguous phases (HIP events on the launch stream); every launch is sized on "
                      "the device, the host reads the results back once per step")
    out = dict(frames_per_s=round(B * args.track_steps * world / el, 2),
               tracked_frames_per_s=round(len(pairs) * args.track_steps * world / el, 2),
               ms_per_step=round(step_ms, 3), batch_frames=B, tracked_per_step=len(pairs), split_ms=split,
               matches_per_frame=round(float(np.mean(nmat)), 1), edges_per_frame=round(float(np.mean(nedge)), 1),
               good_per_frame=round(float(np.mean(ngood)), 1),
               vocabulary="synthetic DBoW2 text vocabulary k=10 L=5, FeatureVector at levelsup 3",
               note="Tracking::TrackReferenceKeyFrame: one batch in flight: extract+match (device batch) then "
                    "ComputeBoW, SearchByBoW(KF=f-%d, F=f), PoseOptimization edge gather and PoseOptimization for "
                    "every tracked frame" % U)
    voc.close()
    out["motion_model"] = motion_leg(args, world, dev, odist, ex, images, stream, pairs, kps, desc, counts, uR, depth,
                                     nmatch)
    return out


def motion_leg(args, world, dev, odist, ex, images, stream, pairs, kps, desc, counts, uR, depth, nmatch):
    """Tracking::TrackWithMotionModel + TrackLocalMap (src/Tracking.cc:1049-1170, 1403-1468) for every tracked
    frame of the batch (tracking.MotionTrackBatch): the last frame's MapPoints, SearchByProjection(F, LastFrame)
    (+ the 2*th retry), PoseOptimization, outlier removal, SearchLocalPoints (frustum + SearchByProjection) and
    PoseOptimization again, every launch sized on the device.  Frame f is tracked from frame f-U, the same
    scene 53 px earlier: the last frame's keypoints are moved by the roll (a 'virtual' last frame), and the
    motion-model pose guess is the identity."""
    import torch
    from orb_slam2_commit_amd.tracking import MotionTrackBatch
    W, H, B = KITTI["width"], KITTI["height"], args.batch
    cap = ex.max_keypoints(W, H)
    fx, bf = KITTI["fx"], KITTI["bf"]
    mt = MotionTrackBatch(len(pairs), cap, W, H, ex.GetScaleFactors(), ex.GetInverseScaleSigmaSquares(), fx, fx,
                          607.1928, 185.2157, bf, dev)
    lf_idx = torch.tensor([2 * lf for lf, _ in pairs], device=dev)
    bl = bf / fx

    def step(tim=None):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(stream)
        ex.stereo_frames_device(images, kps, desc, counts, bf, bl, uR, depth, nmatch, stream)
        with torch.cuda.stream(stream):
            last = kps.index_select(0, lf_idx)
            last.view(torch.float32).view(len(pairs), cap, 7)[:, :, 0] += 53.0
        e1.record(stream)
        r = mt.run(kps, desc, counts, uR, depth, pairs, last_kps=last, stream=stream, timings=tim)
        e2.record(stream)
        return r, (e0, e1, e2)

    step()
    torch.cuda.synchronize(dev)
    odist.barrier()
    tim, evs = [], []
    t0 = time.perf_counter()
    for _ in range(args.track_steps):
        r, ev = step(tim)
        evs.append(ev)
    torch.cuda.synchronize(dev)
    odist.barrier()
    el = odist.max_over_ranks(time.perf_counter() - t0, dev)
    step_ms = el / args.track_steps * 1e3
    tim = np.asarray(tim) * 1e3
    split = dict(extract_match_and_last_frame_gpu=round(float(np.mean([a.elapsed_time(b) for a, b, _ in evs])), 3),
                 search_last_frame_gpu=round(float(tim[:, 0].mean()), 3),
                 edges_and_pose_1_gpu=round(float(tim[:, 1].mean()), 3),
                 search_local_points_gpu=round(float(tim[:, 2].mean()), 3),
                 edges_and_pose_2_gpu=round(float(tim[:, 3].mean()), 3))
    gpu_sum = sum(split.values())
    split.update(sum_gpu=round(gpu_sum, 3), frac_of_step=round(gpu_sum / step_ms, 4),
                 note="GPU time of contiguous phases (HIP events on the launch stream); no host readback between "
                      "launches, results read once per step")
    return dict(frames_per_s=round(B * args.track_steps * world / el, 2),
                tracked_frames_per_s=round(len(pairs) * args.track_steps * world / el, 2),
                ms_per_step=round(step_ms, 3), tracked_per_step=len(pairs), split_ms=split,
                motion_matches_per_frame=round(float(np.mean(r["nmatches"])), 1),
                motion_inliers_per_frame=round(float(np.mean(r["ngood_motion"])), 1),
                local_matches_per_frame=round(float(np.mean(r["local_matches"])), 1),
                inliers_per_frame=round(float(np.mean(r["inliers"])), 1), lost_frames=int(np.sum(r["lost"])),
                note="Tracking::TrackWithMotionModel + TrackLocalMap for every tracked frame, one batch in flight")


# ------------------------------------------------------------------ config-3 leg
def config3_leg(args, rank, world, dev, odist, stream, oracle_mod=None, flags=None, cpus=None):
    """EuRoC MH_01-shaped stereo (752x480, 1200 features) + PnP RANSAC per frame (BASELINE configs[2]):
    a step = extract L+R + stereo match of B3 frames (one per synthetic sequence, device batch) and, per
    frame, a fresh PnPsolver over its device-resident correspondences (1,200 matches, 40 % outliers,
    Tracking's (0.99,10,300,4,0.5,5.991)) run by
    iterate(5) on that sequence's own rand() stream -- all B3 solvers in one orbx_pnp_iterate_many call.
    Returns whole-job frames/s (+ the split) and a single-core oracle baseline of the same unit."""
    import torch
    from orb_slam2_commit_amd import ORBextractor, PnPsolver, synth
    from orb_slam2_commit_amd.glibc_rand import GlibcRand
    from orb_slam2_commit_amd.orb import pnp_iterate_many
    E = synth.EUROC
    W, H, B3, NF = E["width"], E["height"], args.c3_batch, 1200
    pairs = [synth.stereo_pair(s, W, H) for s in synth.sequence_seeds(100 + rank, 8)]
    host = synth.stereo_batch(100 + rank, B3, width=W, height=H, pairs=pairs)
    images = torch.from_numpy(host).to(dev)
    ex = ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index)
    cap = ex.max_keypoints(W, H)
    kps = torch.empty((2 * B3, cap, 28), dtype=torch.uint8, device=dev)
    desc = torch.empty((2 * B3, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(2 * B3, dtype=torch.int32, device=dev)
    uR = torch.empty((B3, cap), dtype=torch.float32, device=dev)
    depth = torch.empty((B3, cap), dtype=torch.float32, device=dev)
    nmatch = torch.zeros(B3, dtype=torch.int32, device=dev)
    bf, baseline = E["bf"], E["bf"] / E["fx"]
    probs = [synth.pnp_problem(seed=3000 * (rank + 1) + f, n=1200, outlier_frac=0.4) for f in range(B3)]
    rngs = [GlibcRand(1 + f + 1000 * rank) for f in range(B3)]  # one process rand() per sequence
    prm = (0.99, 10, 300, 4, 0.5, 5.991)
    # the frames' 3D-2D correspondences resident in HBM back to back (as a device matcher leaves them)
    offs = np.concatenate([[0], np.cumsum([len(P["p3d"]) for P in probs])]).astype(np.int32)
    d_p3d = torch.from_numpy(np.concatenate([P["p3d"] for P in probs]).astype(np.float32)).to(dev)
    d_p2d = torch.from_numpy(np.concatenate([P["p2d"] for P in probs]).astype(np.float32)).to(dev)
    d_s2 = torch.from_numpy(np.concatenate([P["sigma2"] for P in probs]).astype(np.float32)).to(dev)
    intr = np.array([[P["fx"], P["fy"], P["cx"], P["cy"]] for P in probs], np.float32)

    def step():
        ex.stereo_frames_device(images, kps, desc, counts, bf, baseline, uR, depth, nmatch, stream)
        t_e = time.perf_counter()
        # a new PnPsolver per frame, from the device-resident correspondences
        solvers = PnPsolver.create_many_device(d_p3d, d_p2d, d_s2, offs, intr, *prm, device=dev.index)
        t_c = time.perf_counter()
        res = pnp_iterate_many(solvers, 5, rngs)
        t_r = time.perf_counter()
        for sv in solvers:
            sv.close()
        return res, t_c - t_e, t_r - t_c

    step()
    torch.cuda.synchronize(dev)
    odist.barrier()
    t0 = time.perf_counter()
    found, t_create, t_ransac = 0, 0.0, 0.0
    for _ in range(args.c3_steps):
        res, tc, tr = step()
        found += sum(1 for r in res if r[0] is not None)
        t_create += tc
        t_ransac += tr
    torch.cuda.synchronize(dev)
    odist.barrier()
    el = odist.max_over_ranks(time.perf_counter() - t0, dev)
    frames = B3 * args.c3_steps * world
    out = dict(frames_per_s=round(frames / el, 2), ms_per_step=round(el / args.c3_steps * 1e3, 3),
               batch_frames_per_gpu=B3, steps=args.c3_steps,
               ms_per_step_solver_create=round(t_create / args.c3_steps * 1e3, 3),
               ms_per_step_ransac=round(t_ransac / args.c3_steps * 1e3, 3),
               poses_found_frac=round(found / (B3 * args.c3_steps), 4),
               keypoints_per_image=round(float(counts.float().mean()), 1),
               config=dict(workload="EuRoC MH_01 stereo 752x480, 1200 features, extract L+R + ComputeStereoMatches "
                                    "+ PnPsolver RANSAC (1200 matches, 40% outliers) per frame",
                           rand_streams="one glibc rand() stream per frame slot (independent sequences)"),
               data="synthetic (seeded stereo scenes, seeded PnP correspondence sets)", cpu_baseline=None)
    if rank == 0 and world == 1 and oracle_mod is not None:
        p = oracle_mod.params(NF, 1.2, 8, 20, 7)
        old = os.sched_getaffinity(0) if hasattr(os, "sched_setaffinity") else None
        try:
            if old is not None and cpus:
                os.sched_setaffinity(0, {cpus[0]})
            g = GlibcRand(1)
            n, ct = 0, []
            t0 = time.perf_counter()
            while True:
                L, R = pairs[n % len(pairs)]
                P = probs[n % len(probs)]
                c0 = time.perf_counter()
                oL, oR = oracle_mod.extract(p, L), oracle_mod.extract(p, R)
                oracle_mod.stereo_match(p, oL, oR, bf, baseline)
                sv = oracle_mod.PnPsolver(P["p3d"], P["p2d"], P["sigma2"], P["fx"], P["fy"], P["cx"], P["cy"], *prm)
                sv.iterate(5, g)
                ct.append(time.perf_counter() - c0)
                n += 1
                if time.perf_counter() - t0 >= max(2.0, args.cpu_baseline_seconds / 3) and n >= 3:
                    break
        finally:
            if old is not None:
                os.sched_setaffinity(0, old)
        out["cpu_baseline"] = dict(value=round(n / sum(ct), 3), unit="frames/s", cores=1, kind="port",
                                   median_ms=round(pct(ct, 50) * 1e3, 2), p90_ms=round(pct(ct, 90) * 1e3, 2),
                                   sample="%d EuRoC-shaped frames (extract L+R + stereo match + PnP RANSAC), "
                                          "oracle built %s, 1 thread pinned" % (n, flags))
    return out


# ------------------------------------------------------------------ config-5 leg
def config5_leg(args, rank, world, dev, odist, exs, batch_images, pairs):
    """One synthetic KITTI sequence per rank (configs[4]): the rank's Tracking loop steps through
    --pipeline-steps batches of DISTINCT frames (frames 0 .. steps*B-1 of its sequence, in order,
    --inflight batches in flight), and every --kf-every frames inserts a keyframe into the rank's
    LocalMapping thread, which runs a config-4-sized LocalBundleAdjustment for it (its own solver
    handle and HIP stream; the keyframe's local map = synth.localba_problem(seed 7 + 1000*rank + kf))
    once the batch holding the keyframe's frame is extracted -- overlapping the next batches'
    extraction as LocalMapping overlaps Tracking (src/LocalMapping.cc:51-101,
    Examples/Stereo/stereo_kitti.cc:68-110).  Then ONE all-gather of the last batch's frame records and
    every LocalBA summary.  Timed: the sequence with LocalMapping (barrier + synchronize around it,
    max over ranks), the same batches' extraction alone, the LocalBA calls alone, and the all-gather."""
    import torch
    from orb_slam2_commit_amd import pipeline, synth
    W, H, B = KITTI["width"], KITTI["height"], args.batch
    steps, K = args.pipeline_steps, args.kf_every
    batches = [batch_images[k] if k < len(batch_images) else
               torch.from_numpy(synth.stereo_batch(rank, B, pairs=pairs, first=k * B)).to(dev) for k in range(steps)]
    n_kf_rank = (steps * B) // K if K > 0 else 0
    n_kf = pipeline.agree_max(n_kf_rank)
    probs = [synth.localba_problem(seed=7 + 1000 * rank + kf) for kf in range(n_kf_rank)]
    ms, ba_mask = None, None
    if args.c5_ba_cus > 0:  # LocalMapping and Tracking on disjoint CU sets
        n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
        ba_mask, ex_mask = pipeline.cu_partition(n_cus, args.c5_ba_cus, args.c5_cu_layout)
        ms = pipeline.CUMaskedStreams(dev, len(exs), ex_mask)
    sh = pipeline.SequenceShard(exs[0], B, W, H, KITTI["bf"], KITTI["bf"] / KITTI["fx"], dev, extractors=exs[1:],
                                streams=ms.streams if ms else None)
    lm = pipeline.LocalMapping(probs, dev, cu_mask=ba_mask)
    # warm-up: the shard's arenas and the LocalMapping handle (one LocalBA on a keyframe problem)
    sh.run_sequence(batches[:len(sh.exs)])
    if probs:
        lm.opt.LocalBundleAdjustment(probs[0])
    torch.cuda.synchronize(dev)

    def timed(fn):
        odist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize(dev)
        odist.barrier()
        return odist.max_over_ranks(time.perf_counter() - t0, dev), out

    # the sequence: Tracking (this thread) + LocalMapping (its thread), frames numbered from 0
    sh.frames_done = 0

    depth = args.c5_depth if args.c5_depth > 0 else None

    def sequence():
        n = sh.run_sequence(batches, lm, K, depth=depth)
        return n, lm.finish()
    t_seq, (n_ins, res) = timed(sequence)
    # the same work apart: extraction alone (the same batches), LocalBA calls alone (one after another)
    sh.frames_done = 0
    t_ext, _ = timed(lambda: sh.run_sequence(batches, depth=depth))
    t_ba, _ = timed(lambda: [lm.opt.LocalBundleAdjustment(P) for P in probs])
    lm.opt.close()
    cu_split = None
    if ms is not None:
        cu_split = dict(localba_cus=args.c5_ba_cus, layout=args.c5_cu_layout)
    rec = pipeline.ba_summaries([r for _, r in res], [len(P["Tcw"]) for P in probs], n_kf=n_kf)
    t_gather, (recs, bas) = timed(lambda: sh.gather(rec))
    own_ok = bool(torch.equal(recs[rank].to(sh.arena.device), sh.arena)) and bool(np.array_equal(bas[rank], rec))
    ok_all = odist.sum_over_ranks(1.0 if own_ok else 0.0, dev) == world
    if ms is not None:
        torch.cuda.synchronize(dev)
        ms.close()
    its = sum(sum(r["iterations"]) for _, r in res)
    trials = sum(r["trials"] for _, r in res)
    its_all = odist.sum_over_ranks(float(its), dev)
    nbytes = sh.layout.nbytes
    frames = B * steps * world
    backend = pipeline._backend() or "none (1 rank)"
    return dict(sequences=world, unique_frames_per_sequence=B * steps, batch_frames=B, batches_in_flight=len(sh.exs),
                kf_every=K, tracking_depth=depth, cu_split=cu_split, keyframes_per_sequence=n_ins, localba_calls_per_sequence=len(res),
                localba_problem="config-4 sized per keyframe (26 KFs of which 6 fixed, 8,000 points, ~43k edges; "
                                "seed 7 + 1000*rank + kf)",
                lm_iterations_per_sequence=its, lm_trials_per_sequence=trials,
                sequence_s=round(t_seq, 5), extract_alone_s=round(t_ext, 5), localba_alone_s=round(t_ba, 5),
                overlap_gain=round((t_ext + t_ba) / t_seq, 3) if t_seq > 0 else None,
                frames_per_s_sequence=round(frames / t_seq, 2),
                localba_iters_per_s_sequence=round(its_all / t_seq, 1),
                frames_per_s_extract_alone=round(frames / t_ext, 2),
                allgather_ms=round(t_gather * 1e3, 3), allgather_backend=backend,
                record_bytes_per_rank=int(nbytes), record_bytes_per_frame=int(sh.layout.frame_bytes()),
                allgather_bytes_received_per_rank=int(nbytes * (world - 1)),
                allgather_algbw_GBps=round(nbytes * (world - 1) / t_gather / 1e9, 2) if world > 1 else None,
                frames_per_s_with_allgather=round(frames / (t_seq + t_gather), 2),
                localba_summary_ranks=[[pipeline.parse_ba_summary(r)["iterations"]
                                        for r in np.asarray(b).reshape(max(n_kf, 1), -1)[:n_kf]] for b in bas],
                gathered_slots_match=ok_all,
                note="frames_per_s_sequence = unique frames of all ranks / the sequence's wall time with every "
                     "keyframe's LocalBA done (max over ranks); the all-gather carries the LAST batch's records "
                     "(earlier batches are consumed in place) and every LocalBA summary")


def main():
    args = parse()
    kind, n = rank_plan(args)
    if kind == "launch":
        sys.exit(launch_ranks(args, sys.argv[1:]))
    import torch

    from orb_slam2_commit_amd import dist as odist
    rank, local, world = odist.env_rank()
    assert world == n
    backend = os.environ.get("ORBX_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "gloo":
        # one-GPU rehearsal of the multi-rank flow: ranks wrap onto the available devices
        local = local % max(ndev, 1)
    elif local >= ndev:
        raise SystemExit("LOCAL_RANK %d but only %d GPU(s): one rank per GPU under RCCL" % (local, ndev))
    torch.cuda.set_device(local)  # before the process group, so RCCL binds this rank's GPU
    odist.init(backend, rank, world)
    dev = torch.device("cuda", local)
    devices_used = odist.distinct_devices(local, dev)  # distinct GPUs the ranks actually use

    from orb_slam2_commit_amd import ORBextractor, synth
    from orb_slam2_commit_amd import _lib

    W, H, B = KITTI["width"], KITTI["height"], args.batch
    # synthetic frames: sequence = rank (distinct seeds per rank: frame shards); every frame of every
    # in-flight batch distinct (batch k holds frames k*B .. k*B+B-1 of the rank's sequence)
    pairs = [synth.stereo_pair(s, W, H) for s in synth.sequence_seeds(rank, args.unique)]
    # S = --inflight extractor handles, each with its own HIP stream, input batch and output buffers:
    # step i runs on slot i % S, so consecutive batches overlap (one batch's latency-bound stages --
    # octree, small pyramid levels, stereo finalize -- fill in beside the next batch's bandwidth-bound ones)
    S = max(1, args.inflight)
    batch_images = [torch.from_numpy(synth.stereo_batch(rank, B, pairs=pairs, first=k * B)).to(dev) for k in range(S)]
    images = batch_images[0]
    exs = [ORBextractor(KITTI["nfeatures"], 1.2, 8, 20, 7, device=local) for _ in range(S)]
    ex = exs[0]
    cap = ex.max_keypoints(W, H)
    slots = []
    for _ in range(S):
        slots.append(dict(kps=torch.empty((2 * B, cap, 28), dtype=torch.uint8, device=dev),
                          desc=torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev),
                          counts=torch.zeros(2 * B, dtype=torch.int32, device=dev),
                          uR=torch.empty((B, cap), dtype=torch.float32, device=dev),
                          depth=torch.empty((B, cap), dtype=torch.float32, device=dev),
                          nmatch=torch.zeros(B, dtype=torch.int32, device=dev),
                          stream=torch.cuda.Stream(dev)))
    kps, desc, counts = slots[0]["kps"], slots[0]["desc"], slots[0]["counts"]
    uR, depth, nmatch = slots[0]["uR"], slots[0]["depth"], slots[0]["nmatch"]
    # dedicated streams for the whole run: the library launches on them (the legacy null stream would be
    # replaced by the handle's own stream), and the step events / torch ops are ordered with the kernels
    stream = slots[0]["stream"]
    torch.cuda.set_stream(stream)
    torch.cuda.synchronize(dev)
    bf, baseline = KITTI["bf"], KITTI["bf"] / KITTI["fx"]

    def step(i=0):
        k = i % S
        sl = slots[k]
        exs[k].stereo_frames_device(batch_images[k], sl["kps"], sl["desc"], sl["counts"], bf, baseline, sl["uR"],
                                    sl["depth"], sl["nmatch"], sl["stream"])

    for i in range(max(args.warmup, S)):
        step(i)
    torch.cuda.synchronize(dev)
    L = _lib.lib()

    # ---- headline: un-instrumented timed loop (events around each step on its slot's stream)
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    odist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        st_i = slots[i % S]["stream"]
        ev0[i].record(st_i)
        step(i)
        ev1[i].record(st_i)
    torch.cuda.synchronize(dev)
    odist.barrier()
    elapsed = odist.max_over_ranks(time.perf_counter() - t0, dev)
    step_ms = [ev0[i].elapsed_time(ev1[i]) for i in range(args.steps)]  # per-batch latency on its stream

    # ---- second pass: per-stage HIP events (orbx_profile_*, recorded on the kernels' stream)
    L.orbx_profile_reset(ex._h)
    L.orbx_profile_enable(ex._h, 1)
    for _ in range(args.profile_steps):
        step()
    torch.cuda.synchronize(dev)
    L.orbx_profile_enable(ex._h, 0)
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
    ncand = L.orbx_debug_copy(ex._h, 2, 0, 0, None, 0) // 4  # FAST survivors per cell of the last batch
    cc = np.zeros(ncand, np.int32)
    L.orbx_debug_copy(ex._h, 2, 0, 0, _lib.ptr(cc), cc.nbytes)
    cand_per_img = float(cc.sum())  # noqa: F841 -- FAST survivors (reported)
    P = [w * h for (w, h) in level_sizes(W, H, ex.GetInverseScaleFactors())]
    # the dominant stage among those with SURVEY 8(d) bytes (k_octree has none; the three stereo
    # kernels are one stage, charged B_st together with their summed time)
    dom = None
    traffic_all, traffic_src = {}, None
    if os.path.exists(args.traffic):
        try:
            tj = json.load(open(args.traffic))
            traffic_all = tj.get("per_launch_bytes", {})
            traffic_src = dict(file=os.path.relpath(args.traffic, ROOT), head=tj.get("head"), batch=tj.get("batch"))
        except Exception:
            traffic_all = {}
    # issue fractions of the same kernels from the committed SQ counter profile (PMC cannot run live)
    sq_all, sq_src = {}, None
    if os.path.exists(args.sq):
        try:
            sj = json.load(open(args.sq))
            sq_all = sj.get("kernels", {})
            sq_src = os.path.relpath(args.sq, ROOT)
        except Exception:
            sq_all = {}
    rp_ms, rp_src = rocprof_stage_ms(args.rocprof)
    copy_gbs = hbm_copy_peak(dev) if rank == 0 else None

    # every stage against the HBM roofline with its §8(d) bytes: live = HIP events on the launch stream
    # (profiled pass), rocprof = the committed rocprofv3 --stats summary of the same stage
    def stage_entry(name, ev_s_live, events_per_step, rp_step_ms, traffic):
        nb = s8d_stage_bytes(name, 2 * B, B, P, kps_per_img, acc_per_frame)
        e = {"ms_per_step": round(ev_s_live * events_per_step * 1e3, 4), "events_per_step": events_per_step,
             "rocprof_ms_per_step": round(rp_step_ms, 4) if rp_step_ms else None,
             "s8d_bytes_per_event": int(nb) if nb else None, "traffic_per_event": traffic}
        if nb:
            gbs = nb / ev_s_live / 1e9
            e.update({"GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)})
            if rp_step_ms:
                e["frac_rocprof"] = round(nb * events_per_step / (rp_step_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
        return e

    stage_hbm = {}
    for k, (ms_tot, nl) in stages.items():
        if k in STEREO_KERNELS:
            continue
        ev_s = ms_tot / nl / 1e3
        stage_hbm[k] = stage_entry(k, ev_s, STAGE_EVENTS_PER_STEP.get(k, 1), rp_ms.get(k), traffic_all.get(k))
        stage_hbm[k]["valu_issue_frac"] = sq_all.get(k, {}).get("valu_issue_frac")
    st_k = [k for k in STEREO_KERNELS if k in stages]
    if st_k:  # ComputeStereoMatches is three launches: charged B_st together (§8(d))
        ev_s = sum(stages[k][0] / stages[k][1] for k in st_k) / 1e3
        rp = sum(rp_ms.get(k, 0.0) for k in st_k) or None
        tr = sum(traffic_all.get(k, 0) for k in st_k) or None
        stage_hbm["stereo"] = stage_entry("stereo", ev_s, 1, rp, tr)
        stage_hbm["stereo"]["kernels"] = {k: round(stages[k][0] / stages[k][1], 4) for k in st_k}
        # the measured floor (unique 64-B sectors of the staged keypoints' 22 SAD rows + the non-row
        # part of B_st), per frame from its profile run, scaled to this step's frames
        try:
            with open(args.stereo_floor) as f:
                fl = json.load(f)["floor"]
            per_frame = (fl["floor_bytes_64B_sectors"] + fl["B_st_bytes"] - fl["rows_bytes_compact"]) / fl["frames_per_step"]
            floor_b = per_frame * B
            stage_hbm["stereo"]["sector_floor_bytes_per_event"] = int(floor_b)
            stage_hbm["stereo"]["traffic_vs_sector_floor"] = round(tr / floor_b, 3) if tr else None
            # the same floor at the L2's 128-B line granularity (what a miss fetches on gfx950): the SAD
            # rows' distinct lines + the non-row part of B_st
            per_frame_l = (fl["floor_bytes_128B_lines"] + fl["B_st_bytes"] - fl["rows_bytes_compact"]) / fl["frames_per_step"]
            stage_hbm["stereo"]["line_floor_bytes_per_event"] = int(per_frame_l * B)
            stage_hbm["stereo"]["traffic_vs_line_floor"] = round(tr / (per_frame_l * B), 3) if tr else None
            stage_hbm["stereo"]["sector_floor_source"] = os.path.relpath(args.stereo_floor, ROOT)
        except (OSError, KeyError, ValueError):
            stage_hbm["stereo"]["sector_floor_bytes_per_event"] = None
    cands = {k: v for k, v in stage_hbm.items() if v.get("s8d_bytes_per_event")}
    if cands:
        dom = max(cands, key=lambda k: cands[k]["ms_per_step"])
        if dom == "stereo":
            stages = dict(stages, stereo=(sum(stages[k][0] / stages[k][1] for k in st_k), 1))
    roofline = None
    if dom:
        ms_tot, nl = stages[dom]
        avg_s = ms_tot / nl / 1e3
        ent = stage_hbm[dom]
        nbytes = ent["s8d_bytes_per_event"]
        achieved = nbytes / avg_s / 1e9
        roofline = dict(bound="hbm", kernel=dom, achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 5), frac_rocprof=ent.get("frac_rocprof"),
                        traffic=ent.get("traffic_per_event"), traffic_source=traffic_src, rocprof_source=rp_src,
                        algorithmic_bytes_per_launch=int(nbytes), avg_launch_ms=round(avg_s * 1e3, 4),
                        bytes_definition="SURVEY 8(d) terms of this kernel only, per timer event over the batch "
                                         "(k_fast: sum(P) per image; no intermediates)")
        if copy_gbs:
            roofline.update(measured_copy_peak=copy_gbs, frac_of_measured_peak=round(achieved / copy_gbs, 5))
        if dom in sq_all:
            roofline.update(valu_issue_frac=sq_all[dom].get("valu_issue_frac"),
                            salu_issue_frac=sq_all[dom].get("salu_issue_frac"),
                            wait_over_active=sq_all[dom].get("wait_over_active"), sq_source=sq_src)
    # the whole step against §8(d): (2 B_ext + B_st) per frame x frames/s
    frame_b = s8d_frame_bytes(P, kps_per_img, acc_per_frame)
    step_gbs = frame_b * B / (elapsed / args.steps) / 1e9
    whole_step = dict(s8d_bytes_per_frame=int(frame_b), GBps=round(step_gbs, 1),
                      frac=round(step_gbs / HBM_PEAK_GBS, 4),
                      note="SURVEY 8(d): 2*B_ext + B_st per stereo frame x frames/s of this rank (timed loop); "
                           "N_acc = surviving stereo matches per frame (a lower bound of the keypoints that reach "
                           "the SAD, so the figure is conservative)")
    value = odist.job_throughput(B, args.steps, world, elapsed)
    info, cpus = host_info()
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "median_ms_per_step": round(pct(step_ms, 50) / S, 4),
        "p90_ms_per_step": round(pct(step_ms, 90) / S, 4),
        "batch_latency_ms": {"median": round(pct(step_ms, 50), 4), "p90": round(pct(step_ms, 90), 4),
                             "note": "one batch on its stream with %d batches in flight" % S},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (%d seeded stereo scenes per rank; every frame of the %d in-flight batches a distinct "
                "horizontal roll of one)" % (args.unique, S),
        "config": {"workload": "KITTI-00 stereo 1241x376, 2000 features, extract L+R + ComputeStereoMatches",
                   "batch_frames_per_gpu": B, "global_batch_frames": B * world, "nlevels": 8,
                   "scale_factor": 1.2, "fast_th": [20, 7], "parallelism": "frame-sharded x%d" % world,
                   "devices_used": devices_used, "dist_backend": odist.backend(),
                   "batches_in_flight": S},
        "roofline": roofline,
        "whole_step_roofline": whole_step,
        "stage_ms_per_step": {k: round(v[0] / args.profile_steps, 4) for k, v in stages.items()},
        "stage_hbm": stage_hbm,
        "keypoints_per_image": round(kps_per_img, 1),
        "stereo_matches_per_frame": round(acc_per_frame, 1),
        "fast_candidates_per_image": round(cand_per_img, 1),
        "level_pixels": P,
        "localba_iters_per_s": None,
        "host": info,
        "cpu_baseline": None,
    }
    oracle_mod, flags = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        oracle_mod, flags = load_oracle()
        out["cpu_baseline"] = cpu_baseline(oracle_mod, flags, pairs, args.cpu_baseline_seconds, cpus)
    if args.single_frames > 0 and rank == 0 and world == 1:
        out["single_frame"] = single_frame_leg(args, pairs, out["cpu_baseline"])
    if args.ba_calls > 0:
        out["localba"] = localba_leg(args, rank, world, dev, odist, oracle_mod, flags, cpus)
        out["localba_iters_per_s"] = out["localba"]["iters_per_s"]
    if args.track_steps > 0:
        out["track"] = track_leg(args, rank, world, dev, odist, ex, images, stream, pairs)
    if args.pipeline_steps > 0:
        out["config5"] = config5_leg(args, rank, world, dev, odist, exs, batch_images, pairs)
    if args.c1_batch > 0 and rank == 0 and world == 1:
        out["config1"] = config1_leg(args, dev, oracle_mod, flags, cpus)
    if args.c3_steps > 0:
        out["config3"] = config3_leg(args, rank, world, dev, odist, stream, oracle_mod, flags, cpus)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
