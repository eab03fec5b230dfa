"""Diagnose a vocabulary parity mismatch on the bench workload (batched device path)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
from orbslam2commentedbyxcm_amd import ORBextractor, synth
from orbslam2commentedbyxcm_amd.vocabulary import ORBVocabulary
from oracle import oracle as O

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
frames_np, _ = synth.sequence(2000, B, 640, 480)
ex = ORBextractor(1000, 1.2, 8, 20, 7, device=0)
cap = ex.max_keypoints(640, 480)
d_frames = torch.from_numpy(frames_np).cuda()
d_kps = torch.empty((B, cap, 7), dtype=torch.int32, device="cuda")
d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
d_n = torch.empty((B,), dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
ex.extract_batch_device(d_frames, d_kps, d_desc, d_n)
torch.cuda.synchronize()
n_host = d_n.cpu().numpy(); desc = d_desc.cpu().numpy()
text = synth.vocabulary_text(7, 10, 6, 0, 0, centres=desc[0, :n_host[0]])
V = ORBVocabulary(0); assert V.loadFromText(text)
OV = O.Vocab(text)
out = ORBVocabulary.alloc_batch_outputs(B, cap, "cuda")
for mode in ("own-stream", "torch-stream+feat"):
    for t in out.values():
        t.fill_(-1)
    torch.cuda.synchronize()
    if mode == "own-stream":
        V.transform_batch_device(d_desc, d_n, cap, 4, out, stream=V.stream)
    else:
        fw = torch.empty((B, cap), dtype=torch.int32, device="cuda"); fn_ = torch.empty_like(fw)
        V.transform_batch_device(d_desc, d_n, cap, 4, out, stream=torch.cuda.current_stream().cuda_stream,
                                 feat_word=fw, feat_node=fn_)
    torch.cuda.synchronize()
    h = {k: v.cpu().numpy() for k, v in out.items()}
    nbad = 0
    for b in range(min(B, 8)):
        n = int(min(n_host[b], cap))
        e = OV.transform(desc[b, :n], 4)
        g1 = V.transform_arrays(desc[b, :n], 4)
        nb, nf = int(h["nbow"][b]), int(h["nfv"][b])
        g = (h["bow_word"][b, :nb], h["bow_value"][b, :nb], h["fv_node"][b, :nf], h["fv_off"][b, :nf + 1],
             h["fv_idx"][b, :h["fv_off"][b, nf] if nf >= 0 else 0])
        flags = [a.shape == c.shape and np.array_equal(a.view(np.uint8), c.view(np.uint8)) for a, c in zip(g, e)]
        flags1 = [a.shape == c.shape and np.array_equal(a.view(np.uint8), c.view(np.uint8)) for a, c in zip(g1, e)]
        print(mode, b, n, nb, len(e[0]), nf, len(e[2]), flags, "single:", flags1)
        if not all(flags):
            nbad += 1
            for name, a, c in zip(["bw", "bv", "fn", "fo", "fi"], g, e):
                m = min(len(a), len(c))
                d = np.nonzero(a[:m] != c[:m])[0]
                if len(d):
                    print("   ", name, d[:8], a[d[:4]], c[d[:4]])
print("done")
