"""Per-level census of the k_fast cell waves on the bench batch (probe build:
tools/build_variant.sh fprobe -DORBX_FAST_PROBE; run with ORBX_LIB_OVERRIDE=build_ab/fprobe/liborbx.so).

For every cell at iniThFAST: compass survivors (the quick test that feeds ring_score1), survivors of
the stronger necessary condition "4 contiguous of the 8 even ring points beyond t" (probe only),
corners (cornerScore > t) and NMS survivors; plus the per-phase s_memtime split.  Writes JSON to
argv[1] (default gpurun_out/fast_census.json)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import numpy as np  # noqa: E402
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
ncells = L.orbx_debug_copy(ex._h, 2, 0, 0, None, 0) // 4
tab = np.zeros((ncells, 8), np.int32)
L.orbx_debug_copy(ex._h, 3, 0, 0, _lib.ptr(tab), tab.nbytes)
level = tab[:, 0]
buf = torch.zeros((2 * B * ncells, 8), dtype=torch.int32, device=dev)
L.orbx_debug_fast_probe.argtypes = [C.c_void_p]
L.orbx_debug_fast_probe(C.c_void_p(buf.data_ptr()))
ex.stereo_frames_device(images, kps, desc, counts, 386.1448, 386.1448 / 718.856, uR, dep, nm, st)
torch.cuda.synchronize()
L.orbx_debug_fast_probe(None)
a = buf.cpu().numpy().astype(np.int64).reshape(2 * B, ncells, 8)
w6, w7 = a[..., 6], a[..., 7]
empty = w6 & 1
corners = (w6 >> 1) & 0x7FFF
surv = (w6 >> 16) & 0xFFFF
compass = w7 & 0xFFFF
even8 = (w7 >> 16) & 0xFFFF
names = ["window load", "compass at iniThFAST", "score at iniThFAST", "NMS count", "minThFAST pass", "NMS + writes"]
tot = a[..., :6].sum(-1)
out = dict(images=2 * B, cells_per_image=int(ncells), levels={}, phases={})
for i, n in enumerate(names):
    out["phases"][n] = round(float(a[..., i].sum() / tot.sum()), 4)
for lv in range(int(level.max()) + 1):
    m = level == lv
    rw = tab[m, 3] - tab[m, 1] + 1
    rh = tab[m, 4] - tab[m, 2] + 1
    out["levels"][lv] = dict(cells=int(m.sum()), region_px_per_cell=round(float((rw * rh).mean()), 1),
                             compass_per_cell=round(float(compass[:, m].mean()), 2),
                             even8_per_cell=round(float(even8[:, m].mean()), 2),
                             corners_per_cell=round(float(corners[:, m].mean()), 2),
                             nms_survivors_per_cell=round(float(surv[:, m].mean()), 2),
                             empty_frac=round(float(empty[:, m].mean()), 4))
tc, te, tk = compass.sum(), even8.sum(), corners.sum()
out["totals_per_image"] = dict(compass=round(float(tc) / (2 * B), 1), even8=round(float(te) / (2 * B), 1),
                               corners=round(float(tk) / (2 * B), 1), nms=round(float(surv.sum()) / (2 * B), 1))
out["ratios"] = dict(compass_over_corners=round(float(tc / max(tk, 1)), 3),
                     even8_over_corners=round(float(te / max(tk, 1)), 3),
                     even8_over_compass=round(float(te / max(tc, 1)), 3))
out["ticks_per_wave_mean"] = round(float(tot.mean()), 1)
path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fast_census.json"
os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out["totals_per_image"]), json.dumps(out["ratios"]), json.dumps(out["phases"]))
