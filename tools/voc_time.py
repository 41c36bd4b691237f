"""Time ORBVocabulary.transform (GPU, batched frames) beside the oracle (one host thread).
Synthetic vocabulary in ORB-SLAM2's configuration (k = 10, TF-IDF, L1) at L = 5 (ORBvoc.txt is
L = 6 and not in the image; L = 5 keeps generation to seconds).  One frame = 2000 descriptors,
levelsup = 4 (Frame::ComputeBoW)."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/oracle")
from orb_slam2_commit_amd import ORBVocabulary, synth  # noqa: E402


def main(frames=64, reps=5, cpu_frames=8):
    text, vd, leaf = synth.vocabulary(seed=17, k=10, L=5, p_short=0.02)
    sets = [synth.voc_descriptors(1000 + i, vd, leaf, 2000) for i in range(frames)]
    g = ORBVocabulary()
    g.loadFromText(text)
    g.transform_sets(sets, 4)  # warm-up
    t0 = time.perf_counter()
    for _ in range(reps):
        g.transform_sets(sets, 4)
    gpu_s = (time.perf_counter() - t0) / reps
    out = dict(frames=frames, descriptors_per_frame=2000, nodes=g.n_nodes, words=g.n_words,
               gpu_ms_per_batch=round(gpu_s * 1e3, 3), gpu_frames_per_s=round(frames / gpu_s, 1),
               note="host arrays in/out (PCIe included)")
    import oracle
    o = oracle.Vocabulary(text)
    t0 = time.perf_counter()
    for d in sets[:cpu_frames]:
        o.transform(d, 4)
    out["oracle_frames_per_s"] = round(cpu_frames / (time.perf_counter() - t0), 1)
    print(json.dumps(out))
    g.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
