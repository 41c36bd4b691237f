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
buf = (C.c_ulonglong * 8)()
L.orbx_debug_fast_probe(buf, 1)
ex.stereo_frames_device(images, kps, desc, counts, 386.1448, 386.1448 / 718.856, uR, dep, nm, st)
torch.cuda.synchronize()
L.orbx_debug_fast_probe(buf, 0)
waves = buf[5]
names = ["window load", "detect at iniThFAST", "NMS count", "minThFAST pass", "NMS + writes"]
tot = sum(buf[i] for i in range(5))
print("waves %d, empty cells %d (%.1f %%), cycles per wave %.0f" % (waves, buf[6], 100.0 * buf[6] / waves, tot / waves))
for i, n in enumerate(names):
    print("%-22s %8.0f cycles/wave  %5.1f %%" % (n, buf[i] / waves, 100.0 * buf[i] / tot))
