"""Per-step phase split of k_rollout16 (configs[1], diagnostic library): waves 0 (heads + tick) and 1
(a layer wave) of block 0 add the s_memtime cycles between the kernel's phase points over a launch.

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/roll_stamps.py [--steps 4000]

The per-step total is also timed with HIP events over the same launch, which turns cycles into us.
Diagnostic only (libpongmi_diag.so, never the product library).
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PONGMI_LIB"] = os.path.join(ROOT, "pingpong-selfplay-ai_amd", "pongmi", "libpongmi_diag.so")
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

PHASES = ["layer 1 (MFMA + LDS stores)", "barrier A", "layer 2 (16 MFMA) + ReLU stores", "barrier B",
          "heads + actions (wave 0)", "tick + observations (wave 0)", "barrier C"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--arenas", type=int, default=4096)
    args = ap.parse_args()
    import bench
    from pongmi import _lib
    from pongmi.env import PongEnv2PBatch
    from pongmi.qnet import fold, pack_state_dict
    from pongmi.rollout import SelfPlayRollout
    lib = _lib.load()
    lib.pm_diag_read_roll.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    sdB, sdA, _, _ = bench.bench_nets("reference", 0)
    pB = pack_state_dict(sdB).reshape(-1)
    wA = fold(pack_state_dict(sdA), _lib.PM_FOLD_TRAIN).reshape(-1)
    env = PongEnv2PBatch(args.arenas, seed=0x5EED, autoreset=True, **bench.ENV_KW)
    env.reset()
    R = SelfPlayRollout(env, wA, pB, epsilon=0.02, seed_net=0x5EED)
    R.reserve(args.steps)
    R.run(args.steps)  # warm-up (clocks)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    R.run(args.steps, sync=False)
    e1.record()
    e1.synchronize()
    us_step = e0.elapsed_time(e1) * 1e3 / args.steps
    buf = (ctypes.c_uint64 * 16)()
    lib.pm_diag_read_roll(buf)
    print(f"k_rollout16, {args.arenas} arenas, {args.steps} steps per launch: {us_step:.3f} us per step (events, "
          f"incl. the heads fold)")
    for w in range(2):
        cyc = [buf[8 * w + k] / max(1, buf[8 * w + 7]) for k in range(7)]
        tot = sum(cyc)
        print(f"wave {w}: {tot:.0f} cycles per step ({buf[8 * w + 7]} steps)")
        for k, name in enumerate(PHASES):
            print(f"  {name:34s} {cyc[k]:8.1f} cycles  {cyc[k] / tot * 100:5.1f} %  ~{cyc[k] / tot * us_step:.3f} us")


if __name__ == "__main__":
    main()
