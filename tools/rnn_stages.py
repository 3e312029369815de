"""Per-stage timeline of the QNetRNN ring tile (K5) from the diagnostic library's PM_STG stamps.

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/rnn_stages.py [--n 65536]

Runs pm_rnn_q once over n arenas (n/128 blocks, one 128-row group each) and prints, over the first
1024 blocks, the median / p90 time between consecutive stamps: prologue, F2 stages, the 8 gate
stages + cell update + shared-head stage of each hidden block, heads epilogue. Diagnostic only.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PONGMI_LIB"] = os.path.join(ROOT, "pingpong-selfplay-ai_amd", "pongmi", "libpongmi_diag.so")
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES = {0: "begin", 1: "prologue (inputs, L1, h_prev)", 2: "F2 stage 0", 3: "F2 stage 1"}
for m in range(4):
    for t in range(8):
        NAMES[4 + 9 * m + t] = f"m{m} gate stage t{t}"
    NAMES[42 + m] = f"m{m} cell update"
    NAMES[12 + 9 * m] = f"m{m} shared-head stage"
NAMES[46] = "heads + outputs"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    a = ap.parse_args()
    from models.qnet_rnn import QNetRNN
    from pongmi import _lib, rnn
    lib = _lib.load()
    lib.pm_diag_read_rnn.argtypes = [ctypes.c_void_p]
    torch.manual_seed(0)
    w = rnn.fold(rnn.pack_state_dict(QNetRNN(7, 3).state_dict()), _lib.PM_FOLD_TRAIN)[0]
    n = a.n
    x = torch.rand(n, 7, device="cuda")
    h, c = rnn.init_state(n)
    for _ in range(3):
        rnn.q_step(w, x, h, c)
    torch.cuda.synchronize()
    lib.pm_diag_clear_rnn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rnn.q_step(w, x, h, c)
    e1.record()
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * (64 * 1024))()
    lib.pm_diag_read_rnn(buf)
    st = np.array(buf[:], dtype=np.int64).reshape(64, 1024)[:48]
    nb = min(1024, (n + 127) // 128)
    st = st[:, :nb]
    # chronological order of the stamps within a group
    order = [0, 1, 2, 3]
    for m in range(4):
        order += [4 + 9 * m + t for t in range(8)] + [42 + m, 12 + 9 * m]
    order += [46]
    t0 = st[0].min()
    print(f"kernel {e0.elapsed_time(e1) * 1e3:.1f} us, {nb} blocks; block span median "
          f"{np.median(st[46] - st[0]) * 0.01:.2f} us, first begin -> last end {(st[46].max() - t0) * 0.01:.2f} us")
    span_rt = (st[46] - st[0]) * 10e-9
    clk = (st[47] - st[40]) / span_rt
    print(f"shader clock during the blocks (s_memtime / s_memrealtime): median {np.median(clk) / 1e9:.3f} GHz, "
          f"min {clk.min() / 1e9:.3f}, max {clk.max() / 1e9:.3f}")
    print(f"begin times (us): min 0, median {np.median(st[0] - t0) * 0.01:.2f}, max {(st[0].max() - t0) * 0.01:.2f}")
    tot = 0.0
    for prev, k in zip(order[:-1], order[1:]):
        d = (st[k] - st[prev]) * 0.01
        tot += np.median(d)
        print(f"  {NAMES[k]:<32s} median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f}")
    print(f"  sum of medians {tot:.2f} us")


if __name__ == "__main__":
    main()
