"""Per-phase cycles of the k_fast cell waves on the bench batch (probe build:
tools/build_variant.sh fprobe -DORBX_FAST_PROBE; run with ORBX_LIB_OVERRIDE=build_ab/fprobe/liborbx.so)."""
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
ncells = int(ex._plan_cells) if hasattr(ex, "_plan_cells") else 2000
buf = torch.zeros((2 * B * 2000, 8), dtype=torch.int32, device=dev)
L.orbx_debug_fast_probe.argtypes = [C.c_void_p]
L.orbx_debug_fast_probe(C.c_void_p(buf.data_ptr()))
ex.stereo_frames_device(images, kps, desc, counts, 386.1448, 386.1448 / 718.856, uR, dep, nm, st)
torch.cuda.synchronize()
L.orbx_debug_fast_probe(None)
import numpy as np  # noqa: E402
a = buf.cpu().numpy().astype(np.int64)
a = a[a[:, 0] > 0]
names = ["window load", "compass at iniThFAST", "score at iniThFAST", "NMS count", "minThFAST pass", "NMS + writes"]
tot = a[:, :6].sum(1)
print("waves %d, empty cells %.1f %%, compass survivors per cell %.1f, s_memtime ticks per wave mean %.0f median %.0f"
      % (len(a), 100.0 * a[:, 6].mean(), a[:, 7].mean(), tot.mean(), np.median(tot)))
for i, n in enumerate(names):
    print("%-22s mean %8.0f median %8.0f  %5.1f %%" % (n, a[:, i].mean(), np.median(a[:, i]), 100.0 * a[:, i].sum() / tot.sum()))
