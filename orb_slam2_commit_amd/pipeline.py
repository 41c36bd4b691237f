"""Config-5 sequence pipeline (BASELINE.json configs[4]).

One synthetic KITTI stereo sequence per rank (KITTI 00..07 -> rank 0..7): the rank
extracts and stereo-matches its frames in device batches (the reference's per-frame
unit is the stereo Frame constructor, src/Frame.cc:62-123, driven by the sequence
loop of Examples/Stereo/stereo_kitti.cc:68-124), runs Optimizer::LocalBundleAdjustment
on its own map (replicas: one problem per rank), and then the ranks exchange results
with ONE all-gather each:

* per-frame records: a rank's batch of B frames is a single byte arena
  (``FrameRecords``) whose sections are exactly the buffers the extraction writes --
  keypoints (cv::KeyPoint layout, 28 B), descriptors (32 B), per-image counts,
  uRight / depth (f32) padded to the keypoint capacity, per-frame match counts -- so
  the all-gather moves the arena as it lies in HBM (no packing kernel);
* per-rank LocalBA summaries (``ba_summary``): LM iterations per phase, trials,
  final chi2 per phase, outlier count and the optimised poses (FP64).

A rank's sequence is stepped in order through distinct frame batches
(``SequenceShard.run_sequence``); every ``kf_every`` frames a keyframe is inserted into
the rank's ``LocalMapping`` thread, which runs one LocalBundleAdjustment per keyframe on
its own solver handle and HIP stream once the batch holding the keyframe's frame is done,
concurrently with the extraction of the following batches (Tracking and LocalMapping as
the reference's two threads: src/Tracking.cc:1147-1179 InsertKeyFrame,
src/LocalMapping.cc:51-101).

torch.distributed backend "nccl" is RCCL over xGMI (device tensors); "gloo" moves
CPU tensors (CPU tests, and the one-GPU multi-rank rehearsal).
"""
import queue
import threading

import numpy as np

KP_BYTES = 28
DESC_BYTES = 32
_ALIGN = 256


def _align(n):
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


class FrameRecords:
    """Byte layout of one rank's batch of ``n_frames`` stereo frames (capacity ``cap`` keypoints
    per image).  Sections (each 256-B aligned), image 2f = left and 2f+1 = right of frame f:

        kps    (2B, cap, 28) u8    desc  (2B, cap, 32) u8    counts (2B,) i32
        uR     (B, cap) f32        depth (B, cap) f32        nmatch (B,) i32
    """

    SECTIONS = ("kps", "desc", "counts", "uR", "depth", "nmatch")

    def __init__(self, n_frames, cap):
        self.n_frames = int(n_frames)
        self.cap = int(cap)
        B, c = self.n_frames, self.cap
        sizes = dict(kps=2 * B * c * KP_BYTES, desc=2 * B * c * DESC_BYTES, counts=2 * B * 4, uR=B * c * 4,
                     depth=B * c * 4, nmatch=B * 4)
        self.offsets = {}
        off = 0
        for k in self.SECTIONS:
            self.offsets[k] = off
            off = _align(off + sizes[k])
        self.sizes = sizes
        self.nbytes = off

    def frame_bytes(self):
        """Bytes one frame contributes to the record (its slices of every section)."""
        return self.nbytes / self.n_frames

    # ---- views over an arena (numpy array or torch tensor of nbytes uint8)
    def views(self, arena):
        B, c = self.n_frames, self.cap
        shapes = dict(kps=((2 * B, c, KP_BYTES), "u8"), desc=((2 * B, c, DESC_BYTES), "u8"),
                      counts=((2 * B,), "i32"), uR=((B, c), "f32"), depth=((B, c), "f32"), nmatch=((B,), "i32"))
        out = {}
        for k in self.SECTIONS:
            o, n = self.offsets[k], self.sizes[k]
            shape, dt = shapes[k]
            out[k] = _typed(arena[o:o + n], dt).reshape(shape)
        return out

    def unpack(self, arena):
        """Valid entries of every frame as host numpy: list of dicts (kpsL, descL, kpsR, descR, uR, depth,
        nmatch); uR/depth hold the left keypoints' results."""
        v = self.views(arena)
        v = {k: (t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)) for k, t in v.items()}
        frames = []
        for f in range(self.n_frames):
            nL, nR = int(v["counts"][2 * f]), int(v["counts"][2 * f + 1])
            frames.append(dict(kpsL=v["kps"][2 * f, :nL].copy(), descL=v["desc"][2 * f, :nL].copy(),
                               kpsR=v["kps"][2 * f + 1, :nR].copy(), descR=v["desc"][2 * f + 1, :nR].copy(),
                               uR=v["uR"][f, :nL].copy(), depth=v["depth"][f, :nL].copy(),
                               nmatch=int(v["nmatch"][f])))
        return frames


def _typed(a, dt):
    if hasattr(a, "view") and not isinstance(a, np.ndarray):  # torch tensor
        import torch
        return a.view({"u8": torch.uint8, "i32": torch.int32, "f32": torch.float32}[dt])
    return a.view({"u8": np.uint8, "i32": np.int32, "f32": np.float32}[dt])


def new_arena(layout, device):
    """Zeroed record arena on `device`; the padding beyond each image's count stays zero, so two
    runs of the same frames give byte-identical arenas."""
    import torch
    return torch.zeros(layout.nbytes, dtype=torch.uint8, device=device)


def agree_max(value):
    """The maximum of an integer over every rank of the process group (the value itself without
    one).  all_gather_into_tensor / gloo all_gather need the same tensor size on every rank, and
    sequences differ in image size (KITTI 00-02 1241x376, 03 1242x375, 04-10 1226x370) and in
    local-map size, so every size that shapes an exchanged buffer is agreed on first."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return int(value)
    dev = "cpu"
    if dist.get_backend() != "gloo":
        dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


class SequenceShard:
    """One rank's share of config 5: extract + stereo-match its sequence's frames batch by batch into
    a FrameRecords arena (orbx_stereo_frames_device writes straight into the arena's sections).  The
    layout (frames per batch, keypoint capacity) is the maximum over the ranks, so every rank's arena
    has the same size for the all-gather whatever its sequence's image size."""

    def __init__(self, extractor, n_frames, width, height, bf, baseline, device, extractors=None, streams=None):
        """extractors: optional further extractor handles (each with its own record arena and HIP
        stream) so that consecutive batches of the sequence are in flight together; batch k runs on
        slot k % S and writes arena k % S.  `arena` is the arena of the last batch stepped.
        streams: the slots' torch streams (e.g. CUMaskedStreams' ExternalStreams); default: new ones."""
        import torch
        self.exs = [extractor] + list(extractors or [])
        self.ex = extractor
        self.layout = FrameRecords(agree_max(n_frames), agree_max(extractor.max_keypoints(width, height)))
        self.arenas = [new_arena(self.layout, device) for _ in self.exs]
        self.views_ = [self.layout.views(a) for a in self.arenas]
        self.streams = list(streams) if streams is not None else [torch.cuda.Stream(device) for _ in self.exs]
        if len(self.streams) < len(self.exs):
            raise ValueError("SequenceShard: %d streams for %d extractor slots" % (len(self.streams), len(self.exs)))
        self.bf, self.baseline = float(bf), float(baseline)
        self.stream = self.streams[0]
        self.slot = 0
        self.frames_done = 0
        self.last_stream = None

    @property
    def arena(self):
        return self.arenas[self.slot]

    @property
    def v(self):
        return self.views_[self.slot]

    def step(self, images, stream=None, clear=True, slot=0):
        """images: (2B, H, W) u8 device tensor ordered L0,R0,L1,R1,...  clear=True zeroes the arena first
        (canonical padding: the records of a batch do not depend on the previous batch).  The zeroing and
        the extraction are ordered on ONE stream: `stream` (a torch.cuda.Stream other than the legacy null
        stream, which the library would replace by its handle's own stream) or the slot's own."""
        import torch
        self.slot = slot % len(self.exs)
        if stream is None or getattr(stream, "cuda_stream", 0) == 0:
            stream = self.streams[self.slot]
        self.last_stream = stream
        if clear:
            with torch.cuda.stream(stream):
                self.arena.zero_()
        v = self.v
        self.exs[self.slot].stereo_frames_device(images, v["kps"], v["desc"], v["counts"], self.bf, self.baseline,
                                                 v["uR"], v["depth"], v["nmatch"], stream)

    def run_sequence(self, batches, local_mapping=None, kf_every=0, depth=None):
        """Step the rank's sequence through `batches` in order (frame numbers continue across calls), the
        batches in flight over the shard's slots.  With a LocalMapping thread, frame f is a keyframe when
        (f + 1) % kf_every == 0: it is inserted (keyframe id f // kf_every) together with an event
        recorded after its batch, so its LocalBA starts once that batch's extraction has finished on
        the device while later batches keep extracting.  depth: at most this many batches queued on the
        device ahead of the host (the host waits for batch k - depth before launching batch k, as a
        tracker that consumes its frames in order would), so earlier keyframes' LocalBA can start while
        later batches extract; None: every batch launched at once.  Returns the keyframes inserted."""
        import torch
        n_kf = 0
        done = []
        for k, images in enumerate(batches):
            if depth is not None and k >= depth:
                done[k - depth].synchronize()
            self.step(images, slot=k)
            ev_b = torch.cuda.Event()
            ev_b.record(self.last_stream)
            done.append(ev_b)
            nf = int(images.shape[0]) // 2
            f0, self.frames_done = self.frames_done, self.frames_done + nf
            if local_mapping is not None and kf_every > 0:
                kfs = [f // kf_every for f in range(f0, f0 + nf) if (f + 1) % kf_every == 0]
                for kf in kfs:
                    local_mapping.insert_keyframe(kf, ev_b)
                n_kf += len(kfs)
        return n_kf


    def gather(self, ba_record):
        """The config-5 exchange for this shard: the collective is ordered after the shard's last step
        (the current stream waits for the step's stream)."""
        import torch
        if getattr(self, "last_stream", None) is not None:
            torch.cuda.current_stream(self.arena.device).wait_stream(self.last_stream)
        return gather_sequence_results(self.arena, ba_record, self.arena.device)


# ------------------------------------------------------------------ LocalBA summary record
MAX_BA_CAMS = 64  # local window KFs + fixed KFs of one LocalBA call, far above ORB-SLAM2's usual ~30
BA_HEAD = 7


def ba_summary(result, n_cams, max_cams=MAX_BA_CAMS):
    """Fixed-size FP64 record of one LocalBundleAdjustment call (the same length on every rank,
    whatever its local map): [iterations phase 1, phase 2, trials, chi2 phase 1, chi2 phase 2, outlier
    edges, n_cams, Tcw (max_cams x 12, row-major 3x4; rows past n_cams zero)]."""
    if n_cams > max_cams:
        raise ValueError("LocalBA summary: %d cameras > max_cams %d" % (n_cams, max_cams))
    its = list(result["iterations"]) + [0, 0]
    chi = list(result.get("chi2", (0.0, 0.0))) + [0.0, 0.0]
    head = [its[0], its[1], result["trials"], chi[0], chi[1], float(np.sum(result["edge_outlier"])), n_cams]
    rec = np.zeros(BA_HEAD + 12 * max_cams, np.float64)
    rec[:BA_HEAD] = head
    T = np.asarray(result["Tcw_d"], np.float64).reshape(-1)
    rec[BA_HEAD:BA_HEAD + 12 * n_cams] = T[:12 * n_cams]
    return rec


def parse_ba_summary(rec):
    rec = np.asarray(rec, np.float64)
    n = int(rec[6])
    return dict(iterations=(int(rec[0]), int(rec[1])), trials=int(rec[2]), chi2=(rec[3], rec[4]),
                outliers=int(rec[5]), Tcw=rec[BA_HEAD:BA_HEAD + 12 * n].reshape(n, 12))


# ------------------------------------------------------------------ LocalMapping thread
class LocalMapping:
    """One rank's LocalMapping thread (src/LocalMapping.cc:51-101): keyframes arrive from the sequence
    loop (`insert_keyframe`, as Tracking::InsertKeyFrame hands them over); for each, after the event of
    the batch that produced its frame, Optimizer::LocalBundleAdjustment runs on this thread's own solver
    handle -- its own HIP stream -- on `problems(kf)` (the keyframe's local map), concurrently with the
    extraction the sequence loop keeps launching.  Every keyframe's LocalBA runs: the cadence is the
    caller's stated kf_every, with no mbAbortBA interruption (the reference aborts a running BA when a
    keyframe arrives so that a real-time tracker never waits; here throughput is measured instead).
    The LocalBA calls release the GIL (ctypes), so the two threads overlap on the host too."""

    def __init__(self, problems, device, optimizer=None, priority=-1, cu_mask=None):
        """priority: the solver handle's HIP stream priority (default high: the LocalBA trial chain is a
        series of short dependent launches that otherwise queue behind the extraction's blocks).
        cu_mask: restrict the handle's stream to a CU set instead (see cu_partition)."""
        from .orb import Optimizer
        self.problems = problems  # callable kf -> problem dict, or a sequence indexed by kf
        self.own = optimizer is None
        self.opt = optimizer if optimizer is not None else Optimizer(
            device.index if hasattr(device, "index") else int(device), priority=priority, cu_mask=cu_mask)
        self.q = queue.Queue()
        self.results = []  # (kf, result dict) in insertion order
        self.error = None
        self.t = threading.Thread(target=self._run, name="LocalMapping", daemon=True)
        self.t.start()

    def insert_keyframe(self, kf, event=None):
        self.q.put((int(kf), event))

    def _problem(self, kf):
        return self.problems(kf) if callable(self.problems) else self.problems[kf]

    def _run(self):
        try:
            while True:
                item = self.q.get()
                if item is None:
                    return
                kf, ev = item
                if ev is not None:
                    ev.synchronize()  # the keyframe's frame is extracted (releases the GIL while it waits)
                self.results.append((kf, self.opt.LocalBundleAdjustment(self._problem(kf))))
        except BaseException as e:  # noqa: BLE001 -- re-raised by finish() on the caller's thread
            self.error = e

    def finish(self):
        """Wait until every inserted keyframe's LocalBA has finished; returns [(kf, result)]."""
        self.q.put(None)
        self.t.join()
        if self.error is not None:
            raise self.error
        return list(self.results)

    def close(self):
        if self.t.is_alive():
            self.finish()
        if self.own:
            self.opt.close()


def cu_partition(n_cus, n_ba, layout="contiguous"):
    """Two disjoint CU masks (lists of 32-bit words) over n_cus compute units: n_ba for LocalMapping's
    LocalBA stream, the rest for Tracking's extraction streams.  layout "contiguous": CUs 0..n_ba-1;
    "strided": every (n_cus // n_ba)-th CU (spread over the shader engines / XCDs)."""
    if not 0 < n_ba < n_cus:
        raise ValueError("cu_partition: need 0 < n_ba < n_cus (%d, %d)" % (n_ba, n_cus))
    if layout == "contiguous":
        ba = set(range(n_ba))
    elif layout == "strided":
        step = n_cus // n_ba
        ba = set(range(0, step * n_ba, step))
    else:
        raise ValueError("cu_partition: layout %r" % layout)
    words = (n_cus + 31) // 32
    m_ba, m_ex = [0] * words, [0] * words
    for c in range(n_cus):
        (m_ba if c in ba else m_ex)[c >> 5] |= 1 << (c & 31)
    return m_ba, m_ex


class CUMaskedStreams:
    """n HIP streams restricted to one CU set (orbx_stream_create), wrapped as torch ExternalStreams."""

    def __init__(self, device, n, cu_mask):
        import ctypes as C
        import torch
        from . import _lib
        m = np.ascontiguousarray(cu_mask, np.uint32)
        self._raw = []
        self.streams = []
        dev = device.index if hasattr(device, "index") else int(device)
        for _ in range(n):
            h = C.c_void_p()
            _lib.check(_lib.lib().orbx_stream_create(dev, _lib.ptr(m), len(m), C.byref(h)), "orbx_stream_create")
            self._raw.append(h)
            self.streams.append(torch.cuda.ExternalStream(h.value, device=torch.device("cuda", dev)))

    def close(self):
        from . import _lib
        for h in self._raw:
            _lib.lib().orbx_stream_destroy(h)
        self._raw, self.streams = [], []


def ba_summaries(results, n_cams, n_kf=None, max_cams=MAX_BA_CAMS):
    """The fixed-size records of a rank's LocalBA calls, concatenated in keyframe order; `n_kf` (agreed
    over the ranks with agree_max) pads with zero records so every rank sends the same length."""
    n_kf = len(results) if n_kf is None else int(n_kf)
    if len(results) > n_kf:
        raise ValueError("LocalBA summaries: %d calls > n_kf %d" % (len(results), n_kf))
    rec = np.zeros((n_kf, BA_HEAD + 12 * max_cams), np.float64)
    for i, r in enumerate(results):
        rec[i] = ba_summary(r, n_cams[i] if hasattr(n_cams, "__len__") else n_cams, max_cams)
    return rec.reshape(-1)


# ------------------------------------------------------------------ collectives
def all_gather_bytes(t):
    """All-gather a 1-D tensor over the process group: returns (world, n) with row r = rank r's tensor.
    nccl (RCCL over xGMI): device tensors, one all_gather_into_tensor; gloo: CPU tensors.  Without an
    initialised group (one rank) the result is the tensor itself as one row."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t.reshape(1, -1)
    world = dist.get_world_size()
    if dist.get_backend() == "gloo":
        src = t.detach().cpu().contiguous()
        out = [torch.empty_like(src) for _ in range(world)]
        dist.all_gather(out, src)
        return torch.stack(out)
    out = torch.empty((world, t.numel()), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous())
    return out


def gather_sequence_results(shard_arena, ba_record, device=None):
    """The config-5 exchange: every rank's frame-record arena and LocalBA summary to every rank.
    Both must have the same size on every rank (SequenceShard / ba_summary make them so); a mismatch
    is an error here rather than a hang inside the collective."""
    import torch
    for what, n in (("frame-record arena", shard_arena.numel()), ("LocalBA summary", len(ba_record))):
        mx, mn = agree_max(n), -agree_max(-n)  # both collectives on every rank, then the verdict
        if mx != mn:
            raise ValueError("config-5 exchange: %s size differs between ranks (%d here)" % (what, n))
    recs = all_gather_bytes(shard_arena)
    ba = torch.as_tensor(np.asarray(ba_record, np.float64))
    if device is not None and _backend() != "gloo":
        ba = ba.to(device)
    bas = all_gather_bytes(ba)
    return recs, bas.cpu().numpy()


def _backend():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_backend()
    return None
