"""Host side of K8 (pm_play, csrc/pm_play.hip): whole greedy matches in one launch.

The kernel plays every arena from its serve to the end of the episode with both players' nets
staged once per block; a block works through a range of slots (arenas of one (net A, net B) pair)
128 columns at a time, a column taking the next slot when its episode ends. The host groups the
arenas by pair (first-appearance order, arenas ascending within a pair), splits each group into
block ranges, and hands the serves over in slot order. Net id FOLLOWER (-1) is the
HardcodedBallFollower. Used by pongmi.evaluate (eval_vs_model / eval_vs_pool) and
pongmi.tournament (QNet / ball-follower pairs).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import PM_QNET_NW, check, ptr, stream_ptr
from .env import env_params

FOLLOWER = -1
COLUMNS = 128        # arenas a block plays at once
MAX_SLOTS = 1024     # slots per block range (the kernel stages them in LDS)
TARGET_BLOCKS = 512  # 2 blocks (8 waves) per CU on 256 CUs before ranges grow past one slot per column


def plan_blocks(netA, netB, per_block=None):
    """(blk_nets int32 [nb, 2], blk_range int32 [nb, 2] = (start, count), order int32 [E]: arena of
    each slot) for per-arena net ids. per_block: slots per block (default: COLUMNS, or more once the
    arenas would need more than TARGET_BLOCKS blocks, so columns refill instead of adding waves)."""
    netA = np.asarray(netA, np.int64).reshape(-1)
    netB = np.asarray(netB, np.int64).reshape(-1)
    if netA.shape != netB.shape:
        raise ValueError("netA / netB must have one id per arena")
    E = netA.shape[0]
    if per_block is None:
        per_block = min(MAX_SLOTS, COLUMNS * max(1, -(-E // (COLUMNS * TARGET_BLOCKS))))
    if not 0 < per_block <= MAX_SLOTS:
        raise ValueError(f"per_block must be in [1, {MAX_SLOTS}]")
    if E == 0:
        return np.zeros((0, 2), np.int32), np.zeros((0, 2), np.int32), np.zeros(0, np.int32)
    ka, kb = netA + 1, netB + 1
    width = int(kb.max()) + 1
    key = ka * width + kb
    span = int(key.max()) + 1
    if span <= (1 << 22):  # dense pair ids: first appearance by a scatter-min, no sort
        first_of = np.full(span, E, np.int64)
        np.minimum.at(first_of, key, np.arange(E))
        present = np.nonzero(first_of < E)[0]
        first = first_of[present]
        lut = np.empty(span, np.int64)
        lut[present] = np.arange(len(present))
        inv = lut[key]
    else:
        _, first, inv = np.unique(key, return_index=True, return_inverse=True)
    rank = np.empty(len(first), np.int64)
    rank[np.argsort(first, kind="stable")] = np.arange(len(first))  # pairs in first-appearance order
    grp = rank[inv.reshape(-1)]
    # stable sort by pair (radix sort for < 65536 pairs): ascending arena index within a pair
    order = np.argsort(grp.astype(np.uint16) if len(first) < (1 << 16) else grp, kind="stable").astype(np.int32)
    sizes = np.bincount(grp, minlength=len(first))
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    nblk = -(-sizes // per_block)
    g = np.repeat(np.arange(len(first)), nblk)                      # group of each block
    j = np.arange(len(g)) - np.repeat(np.cumsum(nblk) - nblk, nblk)  # block index within its group
    lo = starts[g] + j * per_block
    cnt = np.minimum(per_block, sizes[g] - j * per_block)
    head = order[starts[g]]
    blk_nets = np.stack([netA[head], netB[head]], 1).astype(np.int32)
    return blk_nets, np.stack([lo, cnt], 1).astype(np.int32), order


def play(env_kw, w_nets, netA, netB, serves, device="cuda", max_steps=1_000_000, per_block=None):
    """Play one greedy episode per arena. w_nets: effective weights [nets, PM_QNET_NW] (or None when
    every id is FOLLOWER); netA / netB: per-arena net ids; serves [E, 3] (vx, vy, spin).
    Returns host arrays (scoreA int32 [E], scoreB int32 [E], length int32 [E], last int8 [E]:
    sign(rB - rA) of the final tick)."""
    lib = _lib.load()
    dev = torch.device(device)
    serves = np.ascontiguousarray(np.asarray(serves, np.float64).reshape(-1, 3))
    E = serves.shape[0]
    sA = torch.zeros(E, dtype=torch.int32, device=dev)
    sB = torch.zeros(E, dtype=torch.int32, device=dev)
    length = torch.full((E,), -1, dtype=torch.int32, device=dev)
    last = torch.zeros(E, dtype=torch.int8, device=dev)
    if E == 0:
        return sA.cpu().numpy(), sB.cpu().numpy(), length.cpu().numpy(), last.cpu().numpy()
    blk_nets, blk_range, order = plan_blocks(netA, netB, per_block)
    if w_nets is None:
        w = torch.zeros((1, PM_QNET_NW), dtype=torch.float32, device=dev)
        n_nets = 0
    else:
        w = w_nets.to(dev, torch.float32).reshape(-1, PM_QNET_NW).contiguous()
        n_nets = int(w.shape[0])
    if int(blk_nets.max(initial=-1)) >= n_nets:
        raise ValueError(f"net id {int(blk_nets.max())} but only {n_nets} nets given")
    host = np.concatenate([blk_nets.reshape(-1), blk_range.reshape(-1), order]).astype(np.int32)
    d_int = torch.from_numpy(host).to(dev)  # one copy: nets | ranges | order
    nb = blk_nets.shape[0]
    d_serves = torch.from_numpy(np.ascontiguousarray(serves[order])).to(dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    prm = env_params(**env_kw)
    # the kernel bounds a wave's ticks over all its slots: max_steps per episode x slots per column
    per_col = -(-int(blk_range[:, 1].max()) // COLUMNS)
    wave_steps = min(int(max_steps) * per_col + per_col, 2**31 - 1)
    check(lib.pm_play(ctypes.byref(prm), ptr(w), n_nets, ptr(d_int), ptr(d_int[2 * nb:]), nb, ptr(d_int[4 * nb:]),
                      ptr(d_serves), E, wave_steps, ptr(sA), ptr(sB), ptr(length), ptr(last), ptr(status),
                      stream_ptr()), "pm_play")
    out = (sA.cpu().numpy(), sB.cpu().numpy(), length.cpu().numpy(), last.cpu().numpy())
    st = int(status.item())
    if st or (out[2] < 0).any():
        raise RuntimeError(f"pm_play: {int((out[2] < 0).sum())} arenas did not finish within {max_steps} steps "
                           f"({st} invalid ids or cut episodes)")
    return out
