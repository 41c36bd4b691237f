"""Per-phase cycles of the k_describe keypoint waves (s_memtime probe build build_ab/dprobe)."""
import ctypes as C
import sys

import numpy as np

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
ex.stereo_frames_device(images, kps, desc, counts, 386.1448, 386.1448 / 718.856, uR, dep, nm)
torch.cuda.synchronize()
ph = np.zeros(6 << 21, np.uint32)
_lib.lib().orbx_debug_describe_phases(ph.ctypes.data_as(C.c_void_p))
ph = ph.reshape(6, 1 << 21)
cnt = counts.cpu().numpy()
sel = np.concatenate([np.arange(c) + i * cap for i, c in enumerate(cnt)])
sel = sel[sel < (1 << 21)]
ph = ph[:, sel].astype(np.float64)
names = ["prologue", "patch loads issue", "IC_Angle loads+sums", "atan/sincos", "patch->LDS + rBRIEF", "stores"]
tot = ph.sum(0)
print("waves", ph.shape[1], "cycles/kp mean %.0f median %.0f" % (tot.mean(), np.median(tot)))
for k, n in enumerate(names):
    print("%-22s mean %7.0f  %5.1f %%" % (n, ph[k].mean(), 100 * ph[k].sum() / tot.sum()))
