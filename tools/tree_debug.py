"""Debug: step a learner and compare its incrementally maintained PER sum tree with a full rebuild
after every step; print the first mismatching nodes. Diagnostic only.

    python tools/tree_debug.py [n] [cap] [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    n, cap = int(sys.argv[1]) if len(sys.argv) > 1 else 1000, int(sys.argv[2]) if len(sys.argv) > 2 else 2500
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3 * cap // n + 7
    import test_gpu_selfplay as T
    gdir = os.path.join(ROOT, "tests", "golden")
    golden = lambda name: dict(np.load(os.path.join(gdir, name + ".npz"), allow_pickle=False))  # noqa: E731
    L = T._learner(golden, n=n, batch=256, cap=cap, seed=4, epsilon=0.5)
    nch, nsub = (cap + 1023) // 1024, (cap + 63) // 64
    pad = lambda k: ((k * 8 + 255) // 256) * 256  # noqa: E731
    for k in range(steps):
        c0 = L.counters()
        L.step()
        torch.cuda.synchronize()
        inc = L.per_work.clone()
        L.prepare()
        torch.cuda.synchronize()
        reb = L.per_work.clone()
        L.per_work.copy_(inc)
        torch.cuda.synchronize()
        if torch.equal(inc, reb):
            continue
        ci, cr = inc[:nch * 8].view(torch.float64).cpu().numpy(), reb[:nch * 8].view(torch.float64).cpu().numpy()
        si = inc[pad(nch):pad(nch) + nsub * 8].view(torch.float64).cpu().numpy()
        sr = reb[pad(nch):pad(nch) + nsub * 8].view(torch.float64).cpu().numpy()
        c = L.counters()
        print(f"step {k}: pos {c0['pos']} -> {c['pos']} size {c['size']} train {c['train_steps']}")
        print("  chunk mismatches:", [(int(j), ci[j], cr[j]) for j in np.nonzero(ci != cr)[0][:8]])
        print("  sub mismatches:", [(int(j), si[j], sr[j]) for j in np.nonzero(si != sr)[0][:8]])
        lo = pad(nch) + pad(nsub)
        li = inc[lo:lo + cap * 4].view(torch.float32).cpu().numpy()
        lr = reb[lo:lo + cap * 4].view(torch.float32).cpu().numpy()
        print("  leaf mismatches:", np.nonzero(li != lr)[0][:8])
        print("  idx:", sorted(set((L.idx.cpu().numpy() // 64).tolist()))[:40])
        snap = lo + ((cap * 4 + 255) // 256) * 256
        snl = inc[snap:snap + 256 * 64 * 4].view(torch.float32).cpu().numpy().reshape(256, 64)
        sns = inc[snap + 256 * 64 * 4:snap + 256 * 64 * 4 + 256 * 16 * 8].view(torch.float64).cpu().numpy().reshape(256, 16)
        idx = L.idx.cpu().numpy()
        for ch in np.nonzero(ci != cr)[0][:2]:
            subs = si[ch * 16:(ch + 1) * 16] if (ch + 1) * 16 <= nsub else np.concatenate([si[ch * 16:], np.zeros((ch + 1) * 16 - nsub)])
            acc = 0.0
            for v in subs:
                acc += v
            print(f"  chunk {ch}: inc {ci[ch]!r} reb {cr[ch]!r} seq-sum of inc subs {acc!r}")
            print("    inc subs:", subs.tolist())
            js = np.nonzero(idx // 1024 == ch)[0]
            if len(js):
                print(f"    snapshot subs (sample {js[0]}):", sns[js[0]].tolist())
        return
    print("all steps equal")


if __name__ == "__main__":
    main()
