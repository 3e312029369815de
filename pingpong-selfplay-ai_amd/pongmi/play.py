"""Host side of K8 (pm_play, csrc/pm_play.hip): whole greedy matches in one launch.

The kernel plays every arena from its serve to the end of the episode with both players' nets
staged once per block of 128 arena slots; the host groups the arenas by (net A, net B) pair and
pads each group to whole blocks (pairs in first-appearance order, arenas ascending within a pair).
Net id FOLLOWER (-1) is the HardcodedBallFollower. Used by pongmi.evaluate (eval_vs_model /
eval_vs_pool) and pongmi.tournament (QNet / ball-follower pairs).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import PM_QNET_NW, check, ptr, stream_ptr
from .env import env_params

FOLLOWER = -1
BLOCK = 128


def plan_blocks(netA, netB):
    """(blk_nets int32 [nb, 2], arenas int32 [nb * BLOCK], -1 = padding) for per-arena net ids."""
    netA = np.asarray(netA, np.int64).reshape(-1)
    netB = np.asarray(netB, np.int64).reshape(-1)
    if netA.shape != netB.shape:
        raise ValueError("netA / netB must have one id per arena")
    key = (netA + 1) * (1 << 32) + (netB + 1)
    _, first, inv = np.unique(key, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")  # pairs in first-appearance order
    blk_nets, slots = [], []
    for g in order:
        idx = np.nonzero(inv == g)[0].astype(np.int32)
        nb = (len(idx) + BLOCK - 1) // BLOCK
        pad = np.full(nb * BLOCK, -1, np.int32)
        pad[:len(idx)] = idx
        slots.append(pad)
        blk_nets += [(int(netA[idx[0]]), int(netB[idx[0]]))] * nb
    if not blk_nets:
        return np.zeros((0, 2), np.int32), np.zeros(0, np.int32)
    return np.asarray(blk_nets, np.int32), np.concatenate(slots)


def play(env_kw, w_nets, netA, netB, serves, device="cuda", max_steps=1_000_000):
    """Play one greedy episode per arena. w_nets: effective weights [nets, PM_QNET_NW] (or None when
    every id is FOLLOWER); netA / netB: per-arena net ids; serves [E, 3] (vx, vy, spin).
    Returns host arrays (scoreA int32 [E], scoreB int32 [E], length int32 [E], last int8 [E]:
    sign(rB - rA) of the final tick)."""
    lib = _lib.load()
    dev = torch.device(device)
    serves = np.ascontiguousarray(np.asarray(serves, np.float64).reshape(-1, 3))
    E = serves.shape[0]
    out = [torch.zeros(E, dtype=torch.int32, device=dev) for _ in range(3)]
    last = torch.zeros(E, dtype=torch.int8, device=dev)
    if E == 0:
        return tuple(o.cpu().numpy() for o in out) + (last.cpu().numpy(),)
    blk_nets, slots = plan_blocks(netA, netB)
    if w_nets is None:
        w = torch.zeros((1, PM_QNET_NW), dtype=torch.float32, device=dev)
        n_nets = 0
    else:
        w = w_nets.to(dev, torch.float32).reshape(-1, PM_QNET_NW).contiguous()
        n_nets = int(w.shape[0])
    if int(blk_nets.max(initial=-1)) >= n_nets:
        raise ValueError(f"net id {int(blk_nets.max())} but only {n_nets} nets given")
    d_blk = torch.from_numpy(blk_nets).to(dev)
    d_slots = torch.from_numpy(slots).to(dev)
    d_serves = torch.from_numpy(serves).to(dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    prm = env_params(**env_kw)
    check(lib.pm_play(ctypes.byref(prm), ptr(w), n_nets, ptr(d_blk), ptr(d_slots), int(blk_nets.shape[0]),
                      ptr(d_serves), E, int(max_steps), ptr(out[0]), ptr(out[1]), ptr(out[2]), ptr(last), ptr(status),
                      stream_ptr()), "pm_play")
    st = int(status.item())
    if st:
        raise RuntimeError(f"pm_play: {st} arenas did not finish within {max_steps} steps (or had invalid ids)")
    return tuple(o.cpu().numpy() for o in out) + (last.cpu().numpy(),)
