"""Diagnostic: k_learn_multi (fused multi-update launch) against the split path, field by field after
each vector step; prints the first differing fields."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_selfplay as T  # noqa: E402


def golden(name, cache={}):
    if name not in cache:
        cache[name] = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz")))
    return cache[name]


U = int(sys.argv[1]) if len(sys.argv) > 1 else 2
kw = dict(n=1024, batch=256, cap=4096, seed=8, updates_per_step=U)
A = T._learner(golden, **kw)
B = T._learner(golden, fuse_apply=False, overlap=False, **kw)
names = ("idx", "isw", "grad", "paramsB", "paramsT", "adam_m", "adam_v", "prios", "per_work", "w_B", "learn_heads",
         "trans", "f64", "aB")
for k in range(int(sys.argv[2]) if len(sys.argv) > 2 else 6):
    A.step()
    T._drive_split(B, U)
    torch.cuda.synchronize()
    bad = []
    for nm in names:
        a, b = getattr(A, nm), getattr(B, nm)
        if not torch.equal(a, b):
            d = (a != b).nonzero()
            bad.append(f"{nm}: {d.shape[0]} differ, first {d[:4].flatten().tolist()}")
    ca, cb = A.counters(), B.counters()
    diffc = {kk: (ca[kk], cb[kk]) for kk in ca if ca[kk] != cb[kk]}
    print(f"step {k}: frow_ready={A.sp.frow_ready} {bad} ctrl {diffc}", flush=True)
    if bad:
        ia, ib = A.idx.cpu().numpy(), B.idx.cpu().numpy()
        print(" idx A", ia[:8], "B", ib[:8])
        ga, gb = A.grad.cpu().numpy(), B.grad.cpu().numpy()
        print(" grad A", ga[:4], ga[520:522], "B", gb[:4], gb[520:522])
        wa, wb = A.isw.cpu().numpy(), B.isw.cpu().numpy()
        print(" isw A", wa[:4], "B", wb[:4])
        break
