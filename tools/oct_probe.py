"""Per-phase cycles of the k_octree blocks on the bench batch (probe build:
tools/build_variant.sh oprobe -DORBX_OCT_PROBE; run with ORBX_LIB_OVERRIDE=build_ab/oprobe/liborbx.so)."""
import ctypes as C
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

from orb_slam2_commit_amd import ORBextractor, _lib, synth  # noqa: E402

W, H, B = 1241, 376, 256
dev = torch.device("cuda", 0)
pairs = [synth.stereo_pair(s, W, H) for s in synth.sequence_seeds(0, 16)]
images = torch.from_numpy(synth.stereo_batch(0, B, pairs=pairs)).to(dev)
ex = ORBextractor(2000, 1.2, 8, 20, 7)
cap = ex.max_keypoints(W, H)
kps = torch.empty((2 * B, cap, 28), dtype=torch.uint8, device=dev)
desc = torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev)
counts = torch.zeros(2 * B, dtype=torch.int32, device=dev)
uR = torch.empty((B, cap), dtype=torch.float32, device=dev)
dep = torch.empty((B, cap), dtype=torch.float32, device=dev)
nm = torch.zeros(B, dtype=torch.int32, device=dev)
L = _lib.lib()
st = torch.cuda.current_stream()
ex.stereo_frames_device(images, kps, desc, counts, 386.1448, 386.1448 / 718.856, uR, dep, nm, st)
torch.cuda.synchronize()
buf = torch.zeros((2 * B * 8, 8), dtype=torch.int32, device=dev)
L.orbx_debug_oct_probe.argtypes = [C.c_void_p]
L.orbx_debug_oct_probe(C.c_void_p(buf.data_ptr()))
ex.stereo_frames_device(images, kps, desc, counts, 386.1448, 386.1448 / 718.856, uR, dep, nm, st)
torch.cuda.synchronize()
L.orbx_debug_oct_probe(None)
import numpy as np  # noqa: E402
a = buf.cpu().numpy().astype(np.int64).reshape(2 * B, 8, 8)
names = ["load", "roots", "phase-1 rounds", "phase-2 rounds", "best + write (rest)"]
for l in range(8):
    x = a[:, l]
    rest = x[:, 6] - x[:, 0] - x[:, 1] - x[:, 2] - x[:, 4]
    print("level %d: T %6.0f  total %7.0f | load %6.0f roots %5.0f p1 %7.0f (%.1f rounds) p2 %7.0f (%.1f rounds) rest %6.0f"
          % (l, x[:, 7].mean(), x[:, 6].mean(), x[:, 0].mean(), x[:, 1].mean(), x[:, 2].mean(), x[:, 3].mean(),
             x[:, 4].mean(), x[:, 5].mean(), rest.mean()))
tot = a[:, :, 6].sum()
print("share of block-ticks: load %.1f%% roots %.1f%% p1 %.1f%% p2 %.1f%%" % tuple(
    100.0 * a[:, :, i].sum() / tot for i in (0, 1, 2, 4)))
