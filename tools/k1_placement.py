"""Diagnostic: K1 (pm_env_step, 65 536 arenas, autoreset='done') timed on envs allocated at shifted
device addresses in one process, to test whether the per-process swing of env_step_roofline
(profiles/r3b_k1_runs.txt) follows where the SoA rows land."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
import bench  # noqa: E402

keep = []
for shift_kb in (0, 64, 256, 1024, 4096, 12288, 0, 64):
    keep.append(torch.empty(shift_kb * 1024 + 1, dtype=torch.uint8, device="cuda"))
    r = bench.time_env_step(65536)
    print(f"shift {shift_kb:6d} KB  K1 {r['avg_us']:.2f} us  frac {r['frac']:.3f}  dispatch {r['dispatch_us']:.2f} us",
          flush=True)
