"""Per-phase cycles of the k_fast cell waves (s_memtime probe build build_ab/fprobe), on the bench batch."""
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
ex.extract_batch_device(images, kps, desc, counts) if hasattr(ex, "extract_batch_device") else None
torch.cuda.synchronize()
L = _lib.lib()
buf = (C.c_ulonglong * 16)()
L.orbx_debug_fast_probe(buf, 1)
uR = torch.empty((B, cap), dtype=torch.float32, device=dev)
dep = torch.empty((B, cap), dtype=torch.float32, device=dev)
nm = torch.zeros(B, dtype=torch.int32, device=dev)
ex.stereo_frames_device(images, kps, desc, counts, 386.1448, 386.1448 / 718.856, uR, dep, nm)
torch.cuda.synchronize()
import numpy as np  # noqa: E402
ph = np.zeros(5 << 20, np.uint32)
L.orbx_debug_fast_phases(ph.ctypes.data_as(C.c_void_p))
ph = ph.reshape(5, 1 << 20)[:, :int(ex.ncells() if hasattr(ex, "ncells") else 1220) * 2 * B].astype(np.float64)
names = ["window load", "compass", "score", "nms count", "nms write"]
tot = ph.sum(0)
print("waves", ph.shape[1], "cycles/wave mean %.0f median %.0f p90 %.0f" % (tot.mean(), np.median(tot), np.percentile(tot, 90)))
for k, nmk in enumerate(names):
    print("%-12s mean %8.0f median %8.0f  %5.1f %%" % (nmk, ph[k].mean(), np.median(ph[k]), 100.0 * ph[k].sum() / tot.sum()))
