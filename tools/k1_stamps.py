"""Per-wave phase timeline of K1 (pm_env_step, autoreset 'done', production serves) from the
diagnostic library's s_memtime stamps (libpongmi_diag.so; never the product library).

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/k1_stamps.py [n]

Phases (lane 0 of every wave): 0 start | 1 every load landed (a vmcnt(0) drain: diag only) |
2 draw + tick done | 3 reset select + state/reward stores issued | 4 LDS staging + barrier |
5 observation rows + term rows issued | 6 every store drained. PONGMI_K1_PRO=0 selects round 4's
prologue (A/B)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PONGMI_LIB"] = os.path.join(ROOT, "pingpong-selfplay-ai_amd", "pongmi", "libpongmi_diag.so")
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from pongmi import _lib  # noqa: E402
from pongmi.env import PongEnv2PBatch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
lib = _lib.load()
lib.pm_k1_diag_read.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
env = PongEnv2PBatch(n, seed=3, autoreset="done", **bench.ENV_KW)
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
aA = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=g)
aB = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=g)
for _ in range(200):
    env.step(aA, aB)
torch.cuda.synchronize()
nw = min(4096, (n + 63) // 64)
names = ["loads landed", "draw + tick", "reset + state stores issued", "LDS + barrier", "obs/term stores issued",
         "stores drained"]
acc = [[] for _ in names]
starts, spans = [], []
buf = (ctypes.c_uint64 * (8 * 4096))()
for rep in range(20):
    env.step(aA, aB)
    torch.cuda.synchronize()
    lib.pm_k1_diag_read(buf)
    s = np.frombuffer(buf, np.uint64).reshape(8, 4096)[:, :nw].astype(np.int64)
    t0 = s[0].min()
    starts.append(np.percentile(s[0] - t0, [50, 90, 100]))
    spans.append(s[6].max() - t0)
    for k in range(6):
        acc[k].append(s[k + 1] - s[k])
print(f"n={n} waves={nw}  (s_memtime cycles)")
st = np.mean(starts, 0)
print(f"{'wave start offset':30s} median {st[0]:7.0f}  p90 {st[1]:7.0f}  max {st[2]:7.0f}")
for k, nm in enumerate(names):
    v = np.concatenate(acc[k])
    print(f"{nm:30s} median {np.median(v):7.0f}  p90 {np.percentile(v, 90):7.0f}  max {v.max():7.0f}")
print(f"{'span first start -> last drain':30s} mean {np.mean(spans):7.0f}")
# event-timed launch of the diag kernel, to convert cycles to us
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(100):
    env.step(aA, aB)
e1.record()
e1.synchronize()
print(f"diag kernel back-to-back (eager): {e0.elapsed_time(e1) * 10:.2f} us per launch")
