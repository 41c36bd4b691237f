"""Config-5 sequence pipeline (orb_slam2_commit_amd/pipeline.py): one sequence per rank,
extract + stereo-match + LocalBA per rank, one all-gather of per-frame records and LocalBA summaries.

CPU (gloo, world 2): the records are filled by the oracle (test infrastructure), so this pins the record
layout, the sharding of sequences over ranks, the gather and the unpacking: the gathered records are
byte-equal to a single-process build of the same sequences.
GPU (gloo rehearsal of two ranks on one MI355X): the same exchange over the HIP path, gathered records
byte-equal to a single-process run of the same frames, and every frame equal to the oracle; and the
config-5 per-rank workload at full size -- a 256-frame KITTI batch per rank with a config-4-sized
LocalBA on the rank's LocalMapping thread, overlapping the extraction -- against the oracle."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from orb_slam2_commit_amd import pipeline, synth

W, H, NF, B = 320, 240, 500, 2
KITTI_BF, KITTI_FX = 386.1448, 718.856


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ba_problem(seq):
    return synth.localba_problem(seed=7 + 1000 * seq, n_local=5, n_fixed=2, n_points=300, obs_per_point=4)


def oracle_records(seq, n_frames=B, w=W, h=H, nf=NF):
    """The frame-record arena of sequence `seq` computed by the oracle (what the HIP path must write)."""
    p = oracle.params(nf, 1.2, 8, 20, 7)
    imgs = synth.stereo_batch(seq, n_frames, n_unique=2, width=w, height=h)
    cap = nf + 8 * 8 + 64
    lay = pipeline.FrameRecords(n_frames, cap)
    arena = np.zeros(lay.nbytes, np.uint8)
    v = lay.views(arena)
    for f in range(n_frames):
        o = [oracle.extract(p, imgs[2 * f + k]) for k in (0, 1)]
        for k in (0, 1):
            n = len(o[k].keypoints)
            v["counts"][2 * f + k] = n
            v["kps"][2 * f + k, :n] = o[k].keypoints.view(np.uint8).reshape(n, 28)
            v["desc"][2 * f + k, :n] = o[k].descriptors
        uR, dep = oracle.stereo_match(p, o[0], o[1], KITTI_BF, KITTI_BF / KITTI_FX)
        v["uR"][f, :len(uR)] = uR
        v["depth"][f, :len(dep)] = dep
        v["nmatch"][f] = int((uR >= 0).sum())
    return lay, arena


def _cpu_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from orb_slam2_commit_amd import dist as odist
    odist.init("gloo", rank, world)
    seq = rank  # one sequence per rank
    lay, arena = oracle_records(seq)
    P = _ba_problem(seq)
    rec = pipeline.ba_summary(oracle.local_ba(P), len(P["Tcw"]))
    recs, bas = pipeline.gather_sequence_results(torch.from_numpy(arena), rec)
    q.put((rank, recs.numpy().tobytes(), bas.tobytes(), recs.shape))
    dist.destroy_process_group()


def test_gloo_world2_gathered_records_equal_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process: the same sequences one after another
    single = [oracle_records(s)[1] for s in range(world)]
    lay = oracle_records(0)[0]
    P = [_ba_problem(s) for s in range(world)]
    single_ba = [pipeline.ba_summary(oracle.local_ba(p), len(p["Tcw"])) for p in P]
    for rank, rb, bb, shape in res:
        assert tuple(shape) == (world, lay.nbytes)
        assert rb == np.stack(single).tobytes()  # every rank holds every rank's records, byte-equal
        assert bb == np.stack(single_ba).tobytes()
    # the unpacked records are the oracle's frames
    g = np.frombuffer(res[0][1], np.uint8).reshape(world, -1)
    fr = lay.unpack(g[1])
    assert len(fr) == B and all(len(f["kpsL"]) > 0 for f in fr)
    s = pipeline.parse_ba_summary(np.frombuffer(res[0][2], np.float64).reshape(world, -1)[1])
    assert s["iterations"] == tuple(oracle.local_ba(P[1])["iterations"])


def _ragged_worker(rank, world, port, q):
    """Ranks with different image sizes (KITTI 00 1241x376 vs 04 1226x370, scaled down) and
    different local maps: the layout and the BA record size are agreed before the all-gather."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from orb_slam2_commit_amd import dist as odist
    odist.init("gloo", rank, world)
    nf = 500
    w, h = (320, 240) if rank == 0 else (300, 230)
    own_cap = nf + 8 * 8 + (64 if rank == 0 else 16)  # per-rank capacity (as max_keypoints(w, h) differs)
    lay = pipeline.FrameRecords(pipeline.agree_max(B), pipeline.agree_max(own_cap))
    arena = np.zeros(lay.nbytes, np.uint8)
    v = lay.views(arena)
    p = oracle.params(nf, 1.2, 8, 20, 7)
    imgs = synth.stereo_batch(rank, B, n_unique=2, width=w, height=h)
    o = oracle.extract(p, imgs[0])
    n = len(o.keypoints)
    v["counts"][0] = n
    v["kps"][0, :n] = o.keypoints.view(np.uint8).reshape(n, 28)
    P = synth.localba_problem(seed=7 + rank, n_local=4 + 3 * rank, n_fixed=2, n_points=200, obs_per_point=4)
    rec = pipeline.ba_summary(oracle.local_ba(P), len(P["Tcw"]))
    recs, bas = pipeline.gather_sequence_results(torch.from_numpy(arena), rec)
    bad = None
    try:  # a rank that skips the agreement fails loudly instead of hanging in the collective
        pipeline.gather_sequence_results(torch.zeros(lay.nbytes + 256 * rank, dtype=torch.uint8), rec)
    except ValueError as e:
        bad = str(e)
    q.put((rank, recs.numpy().tobytes(), bas.tobytes(), lay.nbytes, n, len(P["Tcw"]), bad))
    dist.destroy_process_group()


def test_gloo_world2_ragged_sequences():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ragged_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nbytes = res[0][3]
    assert res[1][3] == nbytes  # same agreed layout on both ranks
    lay = pipeline.FrameRecords(B, 500 + 8 * 8 + 64)
    assert lay.nbytes == nbytes
    for rank, rb, bb, _, _, _, bad in res:
        g = np.frombuffer(rb, np.uint8).reshape(world, nbytes)
        ba = np.frombuffer(bb, np.float64).reshape(world, -1)
        for r in range(world):
            assert int(lay.views(g[r])["counts"][0]) == res[r][4]
            assert pipeline.parse_ba_summary(ba[r])["Tcw"].shape == (res[r][5], 12)
        assert bad is not None and "differs between ranks" in bad


def test_record_layout():
    lay = pipeline.FrameRecords(256, 2024)
    assert all(o % 256 == 0 for o in lay.offsets.values())
    # ~ (2*60 + 8) B per keypoint slot per frame
    assert lay.frame_bytes() == pytest.approx(2 * 2024 * 60 + 2024 * 8 + 12, rel=0.01)
    a = np.zeros(lay.nbytes, np.uint8)
    v = lay.views(a)
    v["counts"][3] = 7
    v["uR"][1, 0] = 1.5
    assert v["kps"].shape == (512, 2024, 28) and v["uR"].shape == (256, 2024)
    fr = lay.unpack(a)
    assert len(fr[1]["kpsR"]) == 7 and fr[1]["uR"].shape == (0,)


class _OracleOptimizer:
    """Stands in for the GPU solver handle in the CPU test of the LocalMapping thread."""

    def __init__(self):
        self.calls = []

    def LocalBundleAdjustment(self, P):
        self.calls.append(len(P["Tcw"]))
        return oracle.local_ba(P)


def test_local_mapping_thread_runs_every_keyframe_in_order():
    """pipeline.LocalMapping: every inserted keyframe's LocalBA runs once, in insertion order, on the
    thread; finish() returns them; ba_summaries pads to the agreed keyframe count."""
    probs = {kf: _ba_problem(kf) for kf in range(3)}
    fake = _OracleOptimizer()
    lm = pipeline.LocalMapping(probs, "cpu", optimizer=fake)
    for kf in range(3):
        lm.insert_keyframe(kf)
    res = lm.finish()
    assert [kf for kf, _ in res] == [0, 1, 2]
    for kf, r in res:
        o = oracle.local_ba(probs[kf])
        assert tuple(r["iterations"]) == tuple(o["iterations"])
    rec = pipeline.ba_summaries([r for _, r in res], [len(probs[k]["Tcw"]) for k in range(3)], n_kf=4)
    rows = rec.reshape(4, -1)
    assert not rows[3].any()
    assert pipeline.parse_ba_summary(rows[1])["iterations"] == tuple(res[1][1]["iterations"])
    with pytest.raises(ValueError):
        pipeline.ba_summaries([r for _, r in res], 7, n_kf=2)
    bad = pipeline.LocalMapping(lambda kf: 1 / 0, "cpu", optimizer=fake)  # errors surface on finish()
    bad.insert_keyframe(0)
    with pytest.raises(ZeroDivisionError):
        bad.finish()


def test_cu_partition_masks_are_disjoint_and_cover():
    for n_cus, n_ba, layout in ((256, 64, "contiguous"), (256, 32, "strided"), (304, 48, "strided"), (80, 1, "contiguous")):
        ba, ex = pipeline.cu_partition(n_cus, n_ba, layout)
        bits = lambda m: {32 * w + b for w, v in enumerate(m) for b in range(32) if v >> b & 1}
        A, E = bits(ba), bits(ex)
        assert len(A) == n_ba and not (A & E) and A | E == set(range(n_cus))
    with pytest.raises(ValueError):
        pipeline.cu_partition(256, 0)
    with pytest.raises(ValueError):
        pipeline.cu_partition(256, 64, "diagonal")


def test_ba_summary_roundtrip():
    P = _ba_problem(3)
    r = oracle.local_ba(P)
    rec = pipeline.ba_summary(r, len(P["Tcw"]))
    assert len(rec) == pipeline.BA_HEAD + 12 * pipeline.MAX_BA_CAMS  # fixed size whatever the map
    s = pipeline.parse_ba_summary(rec)
    assert s["iterations"] == tuple(r["iterations"]) and s["trials"] == r["trials"]
    np.testing.assert_array_equal(s["Tcw"], np.asarray(r["Tcw_d"]).reshape(-1, 12))
    with pytest.raises(ValueError):
        pipeline.ba_summary(r, len(P["Tcw"]), max_cams=len(P["Tcw"]) - 1)


# ----------------------------------------------------------------- GPU rehearsal (two ranks, one card)
GW, GH, GNF, GB = 1241, 376, 2000, 4


def _gpu_records(seq, dev):
    import torch
    from orb_slam2_commit_amd import ORBextractor
    ex = ORBextractor(GNF, 1.2, 8, 20, 7, device=dev.index)
    sh = pipeline.SequenceShard(ex, GB, GW, GH, KITTI_BF, KITTI_BF / KITTI_FX, dev)
    imgs = torch.from_numpy(synth.stereo_batch(seq, GB, n_unique=2)).to(dev)
    sh.step(imgs, torch.cuda.current_stream(dev))
    torch.cuda.synchronize(dev)
    return sh


def _gpu_ba(seq, dev):
    from orb_slam2_commit_amd import Optimizer
    P = _ba_problem(seq)
    opt = Optimizer(dev.index)
    r = opt.LocalBundleAdjustment(P)
    opt.close()
    return pipeline.ba_summary(r, len(P["Tcw"]))


def _gpu_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from orb_slam2_commit_amd import dist as odist
    odist.init("gloo", rank, world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sh = _gpu_records(rank, dev)
    recs, bas = sh.gather(_gpu_ba(rank, dev))
    q.put((rank, recs.cpu().numpy().tobytes(), bas.tobytes()))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_two_rank_rehearsal_gathered_records(gpu):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = [_gpu_records(s, gpu) for s in range(world)]
    single = np.stack([s.arena.cpu().numpy() for s in shards])
    single_ba = np.stack([_gpu_ba(s, gpu) for s in range(world)])
    for rank, rb, bb in res:
        assert rb == single.tobytes()
        assert bb == single_ba.tobytes()
    # and the records are the oracle's frames (first and last frame of each sequence)
    p = oracle.params(GNF, 1.2, 8, 20, 7)
    lay = shards[0].layout
    for s in range(world):
        imgs = synth.stereo_batch(s, GB, n_unique=2)
        fr = lay.unpack(single[s])
        for f in (0, GB - 1):
            oL, oR = oracle.extract(p, imgs[2 * f]), oracle.extract(p, imgs[2 * f + 1])
            assert fr[f]["kpsL"].tobytes() == oL.keypoints.tobytes()
            assert fr[f]["descR"].tobytes() == oR.descriptors.tobytes()
            ouR, _ = oracle.stereo_match(p, oL, oR, KITTI_BF, KITTI_BF / KITTI_FX)
            assert fr[f]["uR"].tobytes() == ouR.tobytes()


@pytest.mark.gpu
def test_gpu_bench_launcher_gloo_two_ranks(gpu):
    """`ORBX_DIST_BACKEND=gloo python bench.py --gpus 2` (no WORLD_SIZE): the launcher starts two ranks
    under torch.distributed.run as a child process; rank 0's line says n_gpus 2, backend gloo, and the
    config-5 all-gather ran over 2 ranks with every gathered slot equal to its rank's arena."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["ORBX_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "8", "--inflight", "1", "--unique", "2", "--profile-steps", "1", "--no-cpu-baseline",
           "--ba-calls", "0", "--single-frames", "0", "--track-steps", "0", "--c3-steps", "0",
           "--pipeline-steps", "1", "--kf-every", "8"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["dist_backend"] == "gloo"
    assert out["config"]["devices_used"] == 1  # both ranks wrapped onto the one card
    assert out["config5"]["sequences"] == 2
    assert out["config5"]["allgather_backend"] == "gloo"
    assert out["config5"]["gathered_slots_match"] is True
    assert out["config5"]["localba_calls_per_sequence"] == 1 and out["config5"]["unique_frames_per_sequence"] == 8
    assert out["value"] > 0


# ----------------------------------------------------------------- config-5 per-rank workload, full size
C5_B = 256  # bench.py's batch: one full KITTI batch per rank
C5_SLOTS = (0, C5_B // 2, C5_B - 1)  # sampled slots checked against the oracle


def _c5_problem(seq):
    return synth.localba_problem(seed=7 + 1000 * seq)  # config 4's size (26 KFs, 8,000 points, ~43k edges)


def _c5_run(seq, dev):
    """One rank's config-5 workload: the sequence's first 256 frames in one batch, and the keyframe at
    frame 255 (kf_every = 256) whose config-4-sized LocalBA runs on the LocalMapping thread once the
    batch is extracted.  Returns (shard, LocalBA summaries, [(kf, result)])."""
    import torch
    from orb_slam2_commit_amd import ORBextractor
    ex = ORBextractor(GNF, 1.2, 8, 20, 7, device=dev.index)
    sh = pipeline.SequenceShard(ex, C5_B, GW, GH, KITTI_BF, KITTI_BF / KITTI_FX, dev)
    imgs = torch.from_numpy(synth.stereo_batch(seq, C5_B)).to(dev)
    P = _c5_problem(seq)
    lm = pipeline.LocalMapping({0: P}, dev)
    n_kf = sh.run_sequence([imgs], lm, kf_every=C5_B)
    res = lm.finish()
    lm.close()
    torch.cuda.synchronize(dev)
    assert n_kf == 1 and len(res) == 1
    rec = pipeline.ba_summaries([r for _, r in res], len(P["Tcw"]), n_kf=pipeline.agree_max(len(res)))
    return sh, rec, res


def _c5_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from orb_slam2_commit_amd import dist as odist
    odist.init("gloo", rank, world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sh, rec, _ = _c5_run(rank, dev)
    recs, bas = sh.gather(rec)
    rb = recs.cpu().numpy()
    q.put((rank, hashlib.sha256(rb.tobytes()).hexdigest(), rb.shape, bas.tobytes()))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_config5_rank_workload_full_size(gpu):
    """Config 5 per rank at full size, two gloo ranks on the one card: each rank extracts + stereo-matches
    256 distinct KITTI frames (1241x376, 2,000 features) into its record arena while its LocalMapping
    thread runs a config-4-sized LocalBundleAdjustment (its own handle and stream) for the batch's
    keyframe; then one all-gather of the records and LocalBA summaries.  Checked: the gathered records
    and summaries are byte-equal to single-process runs of the same sequences; slots 0, 128 and 255
    of each sequence are bit-exact against the oracle (keypoints, descriptors, uR, depth); each
    rank's LocalBA matches the oracle within 1e-4 with identical iterations, trials and outliers."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c5_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    runs = [_c5_run(s, gpu) for s in range(world)]
    single = np.stack([sh.arena.cpu().numpy() for sh, _, _ in runs])
    single_ba = np.stack([rec for _, rec, _ in runs])
    for rank, digest, shape, bb in res:
        assert tuple(shape) == single.shape
        assert digest == hashlib.sha256(single.tobytes()).hexdigest()
        assert bb == single_ba.tobytes()
    p = oracle.params(GNF, 1.2, 8, 20, 7)
    lay = runs[0][0].layout
    for s in range(world):
        fr = lay.unpack(single[s])
        imgs = synth.stereo_batch(s, C5_B)
        for f in C5_SLOTS:
            oL, oR = oracle.extract(p, imgs[2 * f]), oracle.extract(p, imgs[2 * f + 1])
            assert fr[f]["kpsL"].tobytes() == oL.keypoints.tobytes(), (s, f)
            assert fr[f]["descL"].tobytes() == oL.descriptors.tobytes(), (s, f)
            assert fr[f]["kpsR"].tobytes() == oR.keypoints.tobytes(), (s, f)
            assert fr[f]["descR"].tobytes() == oR.descriptors.tobytes(), (s, f)
            ouR, odep = oracle.stereo_match(p, oL, oR, KITTI_BF, KITTI_BF / KITTI_FX)
            assert fr[f]["uR"].tobytes() == ouR.tobytes(), (s, f)
            assert fr[f]["depth"].tobytes() == odep.tobytes(), (s, f)
        r = runs[s][2][0][1]
        o = oracle.local_ba(_c5_problem(s))
        assert tuple(r["iterations"]) == tuple(o["iterations"]) and r["trials"] == o["trials"]
        np.testing.assert_array_equal(r["edge_outlier"], o["edge_outlier"])
        np.testing.assert_allclose(r["Tcw_d"], o["Tcw_d"], atol=1e-4, rtol=0)
        np.testing.assert_allclose(r["Xw_d"], o["Xw_d"], atol=1e-4, rtol=0)
        summ = pipeline.parse_ba_summary(single_ba[s].reshape(1, -1)[0])
        assert summ["iterations"] == tuple(o["iterations"]) and summ["outliers"] == int(o["edge_outlier"].sum())
