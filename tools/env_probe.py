#!/usr/bin/env python3
"""K1 probe: k_env_step duration vs arena count and output mode, against a plain device copy of the
same byte count (the practical HBM ceiling at that size). Timing = HIP events around M back-to-back
launches on one stream (average launch duration on a full queue).

    python tools/env_probe.py [--n 65536 262144 1048576 4194304] [--reps 200]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import ENV_KW  # noqa: E402
from pongmi._lib import check, ptr, stream_ptr  # noqa: E402
from pongmi.env import PongEnv2PBatch, ctypes_ref  # noqa: E402


def timed(fn, reps):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def probe(n, reps):
    env = PongEnv2PBatch(n, seed=3, autoreset=True, **ENV_KW)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    aA = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=g)
    aB = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=g)
    lib = env.lib

    def step(term, autoreset):
        def f():
            check(lib.pm_env_step(ctypes_ref(env.params), ctypes_ref(env.state), ptr(aA), ptr(aB), ptr(env.obsA),
                                  ptr(env.obsB), ptr(env.rA), ptr(env.rB), ptr(env.done),
                                  ptr(env.term_obsA) if term else None, ptr(env.term_obsB) if term else None,
                                  int(autoreset), None, 0, env.seed, env.counter, None, n, stream_ptr()),
                  "pm_env_step")
        return f

    out = {"n": n}
    out["autoreset_term_us"] = timed(step(True, True), reps)
    out["autoreset_us"] = timed(step(False, True), reps)
    out["noreset_us"] = timed(step(False, False), reps)
    nbytes = n * 203
    src = torch.empty(nbytes // 2 // 4, dtype=torch.float32, device="cuda")
    dst = torch.empty_like(src)
    out["copy_same_bytes_us"] = timed(lambda: dst.copy_(src), reps)
    for k in ("autoreset_us", "noreset_us", "copy_same_bytes_us"):
        out[k.replace("_us", "_GBs")] = round(nbytes / (out[k] * 1e-6) / 1e9, 1)
    out["autoreset_term_GBs"] = round(n * 259 / (out["autoreset_term_us"] * 1e-6) / 1e9, 1)
    for k in list(out):
        if k.endswith("_us"):
            out[k] = round(out[k], 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[65536, 262144, 1048576, 4194304])
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    for n in a.n:
        print(json.dumps(probe(n, a.reps)), flush=True)


if __name__ == "__main__":
    main()
