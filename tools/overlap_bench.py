"""Throughput of extract+match batches with S extractor handles on S HIP streams in flight
(double buffering), against one handle on one stream.  Same synthetic batch as bench.py."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

from orb_slam2_commit_amd import ORBextractor, synth  # noqa: E402

W, H, NF, BF, FX = 1241, 376, 2000, 386.1448, 718.856


def run(S, B, steps=20):
    dev = torch.device("cuda", 0)
    pairs = [synth.stereo_pair(s, W, H) for s in synth.sequence_seeds(0, 16)]
    images = torch.from_numpy(synth.stereo_batch(0, B, pairs=pairs)).to(dev)
    exs = [ORBextractor(NF, 1.2, 8, 20, 7) for _ in range(S)]
    cap = exs[0].max_keypoints(W, H)
    bufs = []
    for _ in range(S):
        bufs.append(dict(kps=torch.empty((2 * B, cap, 28), dtype=torch.uint8, device=dev),
                         desc=torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev),
                         counts=torch.zeros(2 * B, dtype=torch.int32, device=dev),
                         uR=torch.empty((B, cap), dtype=torch.float32, device=dev),
                         depth=torch.empty((B, cap), dtype=torch.float32, device=dev),
                         nm=torch.zeros(B, dtype=torch.int32, device=dev)))
    streams = [torch.cuda.Stream(dev) for _ in range(S)]

    def step(i):
        k = i % S
        b = bufs[k]
        exs[k].stereo_frames_device(images, b["kps"], b["desc"], b["counts"], BF, BF / FX, b["uR"], b["depth"],
                                    b["nm"], streams[k])

    for i in range(2 * S):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return dict(S=S, B=B, frames_per_s=round(B * steps / el, 1), ms_per_step=round(el / steps * 1e3, 3))


if __name__ == "__main__":
    combos = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(1, 256), (2, 256), (2, 128), (3, 128), (4, 128)]
    for S, B in combos:
        print(json.dumps(run(S, B)), flush=True)
