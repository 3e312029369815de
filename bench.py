#!/usr/bin/env python3
"""Headline benchmark: env-steps/sec of the batched self-play DQN learner (BASELINE.json configs[2]:
65 536 arenas per GPU, the full train_iterative loop — both players acting, env tick, PER replay
push + proportional sample, double-DQN update with target net, Adam), weak-scaled over N GPUs
(configs[3]: one RCCL all-reduce of the 520 head gradients + counters per update).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--arenas 65536] [--pool 8]
    torchrun --nproc-per-node N bench.py --gpus N ...

--gpus N is authoritative (launch_plan): without a launcher (WORLD_SIZE unset) and N > 1 the bench
starts `torch.distributed.run --nproc-per-node N bench.py ...` as a child before any GPU call and
exits with its code; WORLD_SIZE != N, or fewer visible GPUs than N, exits 2 with an error line.

A step = one vector step: every arena on every rank advances one env step and every rank runs one
PER update of batch 256. value = total env-steps (all ranks) / max-over-ranks wall time of K steps.
Rank 0 prints one JSON line. Also reported:
  roofline      the step's dominant launch, k_learn + its extra blocks (pm_selfplay_learn_act): the
                single-workgroup double-DQN update (+ Adam + sum-tree refresh) and, on the other CUs,
                the next vector step's update-independent QNet work on the matrix cores: the
                opponents' act (a full forward per arena) and modelB's frozen feature layers (the
                forward up to the heads). Timed by the launch's own dispatch (pm_timer_arm:
                hipExtLaunchKernel begin/end events, no marker packets in the stream, the same
                interval rocprofv3 --kernel-trace reports) on every 20th production step of an
                instrumented run after the timed region: FP32 FLOP/s of that QNet work vs the
                157.3 TF dense FP32 matrix peak; `traffic` = its HBM bytes per
                launch from the committed counter profile (profiles/r3_pmc.json, same workload), null
                without it
  env_roofline  the first launch, k_actenv (pm_selfplay_actenv): modelB's heads on the features
                computed ahead, the env tick, replay push and bookkeeping, plus the PER sample +
                batch-forward blocks, as HBM work: 282 B of env traffic + 256 B of features read per
                arena vs 8 TB/s
  learn_us / actenv_us  the two launches' own durations (pm_timer_*)
  act_full_roofline  k_act_sp with both players' act (+ the PER sample blocks) in one launch
                (PM_ACT_ALL), back to back after the timed region (N=1 only)
  env_step_roofline  K1 (pm_env_step, autoreset of done arenas) alone at the same n: 203 B / env-step
                vs 8 TB/s, timed over graph-replayed back-to-back launches (N=1 only)
  cpu_baseline  the oracle's CPU port of the same vector step, 1 core, bounded sample (N=1 only)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

ENV_KW = dict(paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_spin=True, magnus_factor=0.025,
              restitution=1, friction=0.6, ball_mass=1.0, world_ball_radius=0.03, ball_speed_range=[0.03, 0.05],
              spin_range=[-5, 5], ball_angle_intervals=[[-60, -30], [30, 60]], speed_scale_every=1,
              speed_increment=0.1)  # config.yaml env (render keys dropped)
FLOP_PER_ARENA = 2 * (7 * 64 + 64 * 64 + 64 * 4)  # one QNet forward (MACs x 2)
FEAT_FLOP_PER_ARENA = 2 * (7 * 64 + 64 * 64)  # modelB's feature layers (computed ahead in the learner launch)
FEAT_BYTES = 64 * 4  # features per arena, written by the learner launch and read by k_actenv
ENV_BYTES = 203  # K1 algorithmic bytes per env-step
# k_env (self-play tick): state 7x8 + 3x4 read and written (136), actions 2, opp 4 + ep_reward 4 read and
# written (16), replay row 64 + priority 4 + PER leaf 4 written, next observations 2x28 written
SP_ENV_BYTES = 136 + 2 + 16 + 72 + 56
PEAK_FP32_TFLOPS = 157.3
INSTR = 20  # after the timed region: one instrumented (timer-armed) step per INSTR production steps


def timed_region(one_step, steps, dist, n_events, after=None, at_end=None):
    """Time exactly `steps` production steps (barrier + synchronize on both sides, max over ranks),
    then run steps // INSTR (at least 5) instrumented steps, each after INSTR - 1 production steps,
    OUTSIDE the timed region (`after()` runs after each, e.g. to read the launch timers): it never
    counts towards `value`. `at_end()` runs right after the timed region, before any instrumented
    step (e.g. to read the counters the timed steps left). Returns (seconds, [event tuples], at_end's
    result)."""
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    end = at_end() if at_end is not None else None
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(n_events)) for _ in range(max(5, steps // INSTR))]
    for ev in evs:
        for _ in range(INSTR - 1):
            one_step()
        one_step(ev)
        if after is not None:
            after()
    torch.cuda.synchronize()
    return dt, evs, end


PEAK_HBM_GBS = 8000.0


def pmc_traffic(kernel, profile="r3_pmc.json"):
    """HBM bytes per launch of `kernel` (`name`, or `name@grid` for one of its launch grids) from the
    committed rocprofv3 counter profile (profiles/r3_pmc.json: the default workload;
    profiles/r3_rnn_pmc.json: --workload rnn; profiles/r3_infer_pmc.json: --workload infer, 2 000-step
    launches), or None. The newest round's profile of the same name (r6_pmc.json, r5_pmc.json, …) wins
    when it holds the kernel."""
    stem = profile[3:] if profile.startswith("r3_") else profile
    for name in (f"r6_{stem}", f"r5_{stem}", f"r4_{stem}", profile):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as fh:
                return json.load(fh)["kernels"][kernel]["hbm_bytes"]
        except (OSError, KeyError, ValueError):
            continue
    return None


def replicas_identical(dist, params):
    """N > 1: every rank holds the same learner parameters after the timed region (the replicas apply
    the identical update to the all-reduced gradients). Compared as the float64 sum of the raw bit
    patterns and of the values, max == min over ranks."""
    if dist is None:
        return None
    bits = params.view(torch.int32).to(torch.float64)
    v = torch.stack([bits.sum(), params.to(torch.float64).sum()])
    hi, lo = v.clone(), -v
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MAX)
    return bool(torch.equal(hi, -lo))


def shard_proof(dist, rank, world, n, steps_done, status, comm, grad=None):
    """N > 1: what every rank saw, gathered to rank 0 so the line can only be produced by N live
    ranks: RCCL's own view of the communicator (pm_comm_info: ncclCommCount / ncclCommUserRank /
    device), the arenas and vector steps this rank ran, its device status word, and — for the DQN
    learner — the packed buffer's updated-flag after the last SUM all-reduce (= the number of ranks
    whose update entered it). Returns (per-rank list, ok)."""
    if dist is None:
        return None, True
    nr, rr, dev = comm.info() if comm is not None else (dist.get_world_size(), dist.get_rank(), torch.cuda.current_device())
    upd = float(grad[521].item()) if grad is not None else -1.0
    row = torch.zeros((world, 8), dtype=torch.float64, device="cuda")
    row[rank] = torch.tensor([rank, nr, rr, dev, n, steps_done, status, upd], dtype=torch.float64)
    dist.all_reduce(row)
    rows = [dict(rank=int(r[0]), rccl_nranks=int(r[1]), rccl_rank=int(r[2]), device=int(r[3]), arenas=int(r[4]),
                 vector_steps=int(r[5]), status=int(r[6]), **({"allreduce_updated_sum": r[7]} if grad is not None else {}))
            for r in row.cpu().tolist()]
    ok = all(r["rccl_nranks"] == world and r["rccl_rank"] == r["rank"] and r["status"] == 0 for r in rows)
    ok = ok and len({r["vector_steps"] for r in rows}) == 1
    if grad is not None:
        ok = ok and all(r["allreduce_updated_sum"] == world for r in rows)
    return rows, ok


def synthetic_qnet(seed):
    from models.qnet import QNet
    torch.manual_seed(seed)
    return {k: v.clone() for k, v in QNet(7, 3).state_dict().items()}


def time_env_step(n, per_graph=50, replays=40, warm_replays=100):
    """K1 alone: pm_env_step with autoreset of done arenas (term rows for done arenas only: the
    203 B / env-step of SURVEY.md 8d). `per_graph` back-to-back launches are captured in one HIP
    graph so the host launch rate (ctypes, ~8 us per call) does not pace the queue; HIP events on
    the replay stream bracket `replays` replays. avg_us = elapsed / launches."""
    from pongmi.env import PongEnv2PBatch
    env = PongEnv2PBatch(n, seed=3, autoreset="done", **ENV_KW)
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(0)
    aA = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=gen)
    aB = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=gen)
    for _ in range(20):
        env.step(aA, aB)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        env.step(aA, aB)
        s.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(per_graph):
                env.step(aA, aB)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(warm_replays):  # ~20 ms of back-to-back K1 first: the clocks settle (a 3-replay
            g.replay()                 # warm-up read 4.64 us on one box where others gave 4.07-4.17)
        e0.record(s)
        for _ in range(replays):
            g.replay()
        e1.record(s)
    e1.synchronize()
    t = e0.elapsed_time(e1) * 1e-3 / (per_graph * replays)
    achieved = n * ENV_BYTES / t / 1e9
    # the same launch timed from its own dispatch (pm_timer_arm: the interval rocprofv3's kernel trace
    # reports, without the launch-to-launch gap the graph replay includes), eager launches
    from pongmi import _lib
    with torch.cuda.stream(s):
        for _ in range(per_graph):
            _lib.timer_arm(_lib.PM_TIMER_ENV_STEP)
            env.step(aA, aB)
    td = sum(_lib.timer_read(_lib.PM_TIMER_ENV_STEP) for _ in range(per_graph)) / per_graph
    return {"bound": "hbm", "kernel": "k_env_step", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
            "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": pmc_traffic("k_env_step"),
            "avg_us": round(t * 1e6, 2), "bytes_per_env_step": ENV_BYTES, "n": n,
            "timing": f"HIP events over {replays} graph replays x {per_graph} launches, autoreset='done'",
            "dispatch_us": round(td * 1e6, 2), "dispatch_frac": round(n * ENV_BYTES / td / 1e9 / PEAK_HBM_GBS, 4)}


def time_act_full(L, launches=50):
    """k_act_sp with both players in one launch (PM_ACT_ALL: what the plain step and pm_selfplay_act
    run, PER sample blocks included), back to back on the learner's state after the timed region
    (idempotent: same observations, same sample, same actions), HIP events on its stream: both QNet
    forwards per arena, 19 200 FLOP."""
    from pongmi import _lib
    featB, L.sp.featB = L.sp.featB, None  # both players' act alone (no features computed ahead)
    for _ in range(5):
        L.act(_lib.PM_ACT_ALL)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(launches):
        L.act(_lib.PM_ACT_ALL)
    e1.record()
    e1.synchronize()
    L.sp.featB = featB
    L._aA_ready = False
    t = e0.elapsed_time(e1) * 1e-3 / launches
    achieved = L.n * 2 * FLOP_PER_ARENA / t / 1e12
    return {"bound": "mfma", "kernel": "k_act_sp (PM_ACT_ALL: both players + the PER sample blocks)",
            "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "avg_us": round(t * 1e6, 2),
            "flop_per_arena": 2 * FLOP_PER_ARENA, "n": L.n, "traffic": pmc_traffic("k_act_sp"),
            "timing": f"HIP events over {launches} back-to-back launches"}


def time_scalar_dropin(seconds=1.0):
    """The scalar drop-ins a reference script uses unchanged: configs[0]'s
    loop — one PongEnv2P, random vs random (random.randint for A then B), reset on done — on
    envs/my_pong_env_2p.py (one pm_env_step1 / pm_env_reset1 launch per call, results polled from
    host-mapped memory), and envs/physics.py's scalar collide (one pm_collide1 launch per call).
    Per-call wall time on this host; the reference's own Python step is 10.6 us."""
    import random
    from envs.my_pong_env_2p import PongEnv2P
    from envs.physics import collide_sphere_with_moving_plane
    env = PongEnv2P(**ENV_KW)
    rng = random.Random(0)
    for _ in range(200):
        _, _, d, _ = env.step(rng.randint(0, 2), rng.randint(0, 2))
        if d:
            env.reset()
    steps = resets = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, _, d, _ = env.step(rng.randint(0, 2), rng.randint(0, 2))
        steps += 1
        if d:
            env.reset()
            resets += 1
    dt = time.perf_counter() - t0
    k = 2000
    t1 = time.perf_counter()
    for j in range(k):
        collide_sphere_with_moving_plane(-0.04, 0.01 * (j % 7), 0.03, 1.5, 1.0, 0.6, 1.0, 0.03)
    dc = time.perf_counter() - t1
    # round 5's drop-in step for comparison: the batch env at n = 1 (actions copied to the device,
    # K1, the outputs gathered and copied back)
    from pongmi.env import PongEnv2PBatch
    b = PongEnv2PBatch(1, **ENV_KW)
    b.reset()
    for _ in range(50):
        (oA, oB), (rA, rB), dn, _ = b.step(torch.tensor([1], dtype=torch.int8), torch.tensor([1], dtype=torch.int8))
    k2 = 0
    t2 = time.perf_counter()
    while time.perf_counter() - t2 < seconds / 2:
        aA = torch.tensor([rng.randint(0, 2)], dtype=torch.int8)
        aB = torch.tensor([rng.randint(0, 2)], dtype=torch.int8)
        (oA, oB), (rA, rB), dn, _ = b.step(aA, aB)
        torch.cat([oA[0], oB[0], rA, rB, dn.float()]).cpu().numpy()
        k2 += 1
    db = time.perf_counter() - t2
    return {"env_us_per_step": round(dt / steps * 1e6, 2), "env_steps_per_s": round(steps / dt, 1), "steps": steps,
            "resets": resets, "collide_us_per_call": round(dc / k * 1e6, 2),
            "round5_dropin_us_per_step": round(db / k2 * 1e6, 2),
            "reference_python_us_per_step": 10.6,
            "note": "PongEnv2P drop-in, random vs random with reset on done, wall time incl. the host's randint "
                    "draws; one launch per step / reset, results polled from host-mapped memory"}


def cpu_baseline(n, nets, seconds=12.0, epsilon=0.08):
    """The oracle's CPU port of the same vector step, acting with the GPU leg's nets (`nets` =
    bench_nets(...): modelB, modelA, pool, description) and its epsilon, so both legs play the same
    policies (episode lengths, hence reset and bookkeeping load, match)."""
    from threadpoolctl import threadpool_limits
    from oracle.cpu_selfplay import CpuSelfPlay
    sdB, sdA, pool, wdesc = nets
    np_sd = lambda s: {k: v.numpy() for k, v in s.items()}  # noqa: E731
    with threadpool_limits(1):
        cpu = CpuSelfPlay(ENV_KW, n, np_sd(sdB), np_sd(sdA), [np_sd(s) for s in pool], batch=256, cap=1_000_000,
                          epsilon=epsilon)
        for _ in range(2):
            cpu.step()
        t0 = time.perf_counter()
        steps = 0
        while time.perf_counter() - t0 < seconds:
            cpu.step()
            steps += 1
        dt = time.perf_counter() - t0
    v = n * steps / dt
    return {"value": round(v, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/cpu_selfplay.py: {steps} vector steps x {n} arenas (full DQN loop, PER cap 1e6, "
                      f"batch 256, eps {epsilon}, pool {len(pool)}), {dt:.1f} s on 1 host core",
            "weights": wdesc,
            # calibration to the reference's own loop (measured in the survey container, one
            # thread): train_iterative.py's step body = 1 env step + 1 PER update of 256 per env step
            "reference_python_measured": {"steps_per_s": {"small_buffer": 398, "fill_100k": 209, "fill_1e6": 75},
                                          "note": "train_iterative.py step body, 1 env step + 1 update per step, "
                                                  "1 CPU thread (SURVEY 6)"},
            "port_vs_reference_loop": {"small_buffer": round(v / 398, 1), "fill_100k": round(v / 209, 1),
                                       "fill_1e6": round(v / 75, 1),
                                       "note": "env-steps/s ratio; the port batches 65 536 arenas and runs one update "
                                               "per vector step (the bench's U = 1), the reference one update per env "
                                               "step"}}


def _config0_worker(seconds, seed, q):
    from oracle import oracle as orc
    P = orc.make_params(orc.env_params_from_kwargs(**ENV_KW))
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        orc.rollout_random(P, seed + steps, 200_000)
        steps += 200_000
    q.put((steps, time.perf_counter() - t0))


def cpu_config0(seconds=3.0, procs=None):
    """BASELINE configs[0]: ONE PongEnv2P arena, random vs random, the scalar CPU step loop
    (random.seed, randint actions for A then B, reset on done), as the oracle's C
    restatement (oracle/pong_oracle.c or_rollout_random, pinned to the reference's own loop output by
    tests/test_oracle_golden.py::test_rollout_random_matches_reference_loop) on 1 host core and on
    `procs` independent processes (one arena each, like the reference run once per core)."""
    import multiprocessing as mpr
    procs = procs or max(1, min(16, len(os.sched_getaffinity(0))))
    out = {}
    for k in (1, procs):
        ctx = mpr.get_context("fork")
        q = ctx.Queue()
        ps = [ctx.Process(target=_config0_worker, args=(seconds, 1000 * r, q)) for r in range(k)]
        for p in ps:
            p.start()
        res = [q.get() for _ in ps]
        for p in ps:
            p.join()
        out[f"cores_{k}"] = round(sum(st / dt for st, dt in res), 1)
    return {"workload": "configs[0]: 1 arena per process, random vs random, scalar step loop with reset on done",
            "unit": "env-steps/s", "value_1core": out["cores_1"], "value_all": out[f"cores_{procs}"], "cores": procs,
            "kind": "port", "sample": f"oracle/pong_oracle.c or_rollout_random, {seconds:.0f} s per process",
            "reference_python_measured": "94 k env-steps/s per core, 442 k on 8 processes (SURVEY 6, survey container)"}


ENV_KW_RNN = dict(ENV_KW, restitution=1.0, speed_scale_every=5, speed_increment=0.2)  # config_rnn.yaml:6-28
# QNetRNN multiply-adds per row: 7(+bias)x64 + 64x128 + 256x512 (LSTM gates) + 128x128 + 128x4 heads
RNN_MAC = 8 * 64 + 64 * 128 + 256 * 512 + 128 * 128 + 128 * 4
RNN_FLOP_PER_ARENA = 2 * 2 * RNN_MAC  # both players
# k_rsp_env: state 136, actions 2, opp 4 + ep_reward 4 + ep_len 4 read, + reset 1 + fin 4 written (21 B),
# ring record 64 written, next observations 2 x 28 written
RNN_ENV_BYTES = 136 + 2 + 12 + 21 + 64 + 56


def synthetic_rnn(seed):
    from models.qnet_rnn import QNetRNN
    torch.manual_seed(seed)
    return {k: v.clone() for k, v in QNetRNN(7, 3).state_dict().items()}


def cpu_baseline_rnn(seconds=12.0, n=2048):
    from threadpoolctl import threadpool_limits
    from oracle.cpu_rnn_selfplay import CpuRnnSelfPlay
    np_sd = lambda s: {k: v.numpy() for k, v in s.items()}  # noqa: E731
    with threadpool_limits(1):
        cpu = CpuRnnSelfPlay(ENV_KW_RNN, n, np_sd(synthetic_rnn(1)), np_sd(synthetic_rnn(2)),
                             [np_sd(synthetic_rnn(100 + k)) for k in range(4)], min_episodes=640)
        while cpu.t == 0:  # fill the sequence buffer until updates run
            cpu.step()
        t0 = time.perf_counter()
        steps = 0
        while time.perf_counter() - t0 < seconds:
            cpu.step()
            steps += 1
        dt = time.perf_counter() - t0
    return {"value": round(n * steps / dt, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/cpu_rnn_selfplay.py: {steps} vector steps x {n} arenas (QNetRNN acting both players "
                      f"+ env + sequence buffer + DRQN update 64x8 every step), {dt:.1f} s on 1 host core"}


def drqn_flop(B, T):
    """FLOPs of one DRQN update (2 x MACs): three forward streams through F1, F2, the LSTM input and
    recurrent projections (T*B columns each) and the shared head + heads on h_T (B columns); BPTT of
    the obs stream: dWih, dWhh, dF2 = Wih^T dZ, dh = Whh^T dz, dW2, dF1, dW1, and the head's dW_S,
    dh_T."""
    C0 = T * B
    fwd = 3 * C0 * (7 * 64 + 64 * 128 + 2 * 128 * 512) + 3 * B * (128 * 128 + 128 * 4)
    bwd = C0 * (4 * 128 * 512 + 2 * 64 * 128 + 7 * 64) + B * 2 * 128 * 128
    return 2 * (fwd + bwd)


def time_drqn_update(D, launches=50):
    """The DRQN update alone (pm_drqn_update, 4 launches) back to back on its last batch after the
    timed region (HIP events on the stream), and the persistent recurrence k_dq_recur by its own
    dispatch (pm_timer_arm). Restores nothing: it runs after the measured steps."""
    from pongmi import _lib
    for _ in range(5):
        D.update()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(launches):
        D.update()
    e1.record()
    e1.synchronize()
    t = e0.elapsed_time(e1) * 1e-3 / launches
    for _ in range(10):
        _lib.timer_arm(_lib.PM_TIMER_DRQN)
        D.update()
    rec = sum(_lib.timer_read(_lib.PM_TIMER_DRQN) for _ in range(10)) / 10
    flop = drqn_flop(D.batch, D.T)
    achieved = flop / t / 1e12
    ks = ("k_dq_embed", "k_dq_recur", "k_dq_wgrad", "k_drqn_apply")
    tr = [pmc_traffic(k, "r3_rnn_pmc.json") for k in ks]
    traffic = round(sum(tr), 1) if all(x is not None for x in tr) and (D.batch, D.T) == (64, 8) else None
    return {"bound": "mfma", "kernel": "pm_drqn_update (k_dq_embed + k_dq_recur + k_dq_wgrad + k_drqn_apply), "
                                       "the whole update",
            "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": traffic, "update_us": round(t * 1e6, 2),
            "recur_us": round(rec * 1e6, 2), "launches_per_update": 4, "flop_per_update": flop,
            "batch": D.batch, "T": D.T, "timing": f"HIP events over {launches} back-to-back updates"}


def run_rnn(args, dist, rank, world, allreduce):
    """configs[4]: 32768 arenas/GPU, the train_rnn_iterative loop (QNetRNN both players with (h, c)
    per arena, sequence buffer, DRQN update 64 x 8 with BPTT + clip + Adam every vector step)."""
    from pongmi.rnn_selfplay import RNNSelfPlayLearner
    n = args.arenas or 32768
    pool_n = 4 if args.pool is None else args.pool
    L = RNNSelfPlayLearner(ENV_KW_RNN, n, synthetic_rnn(1), synthetic_rnn(2),
                           [synthetic_rnn(100 + k) for k in range(pool_n)], epsilon=0.05, seed=7, rank=rank,
                           world=world, allreduce=allreduce)

    from pongmi import _lib
    overlap = dist is None and L.overlap

    def one_step(ev=None):
        if ev is None:
            L.step()
            return
        _lib.timer_arm(_lib.PM_TIMER_RNN_ACT)  # the step's first k_rnn_act: modelB's side (overlap) or both
        if overlap:  # the production step's two calls: modelB's fold + act, then env + update with the
            ev[0].record()  # next step's opponent act beside it (the production path's aA is always ready)
            L.act_part(_lib.PM_ACT_B)
            ev[1].record()
            L.finish_overlap()
            ev[2].record()
            ev[3].record()
            return
        ev[0].record()
        L.act()
        ev[1].record()
        L.env_step()
        ev[2].record()
        if dist is None:
            L.learner.update()
        else:
            L.learner.grads()
            allreduce(L.learner.grad)
            L.learner.apply()
        ev[3].record()

    warm = max(args.warmup, 60)  # the sequence buffer holds > 640 episodes (updates run) from ~step 20
    for _ in range(warm):
        one_step()
    torch.cuda.synchronize()
    c0 = L.counters()
    act_t = []
    dt, evs, c1 = timed_region(one_step, args.steps, dist, 4, lambda: act_t.append(_lib.timer_read(_lib.PM_TIMER_RNN_ACT)),
                               L.counters)
    same = replicas_identical(dist, L.learner.params)
    act_s = sum(act_t) / len(act_t)  # k_rnn_act's own dispatch (pm_timer_*), as rocprofv3 times it
    env_s = sum(e[1].elapsed_time(e[2]) for e in evs) * 1e-3 / len(evs)  # overlap: env + update
    upd_s = sum(e[2].elapsed_time(e[3]) for e in evs) * 1e-3 / len(evs)
    c = L.counters()
    shards, shards_ok = shard_proof(dist, rank, world, n, c["step"], c["status"] & 1, args.comm)
    dst = L.learner.stats()
    failed = (c["status"] & 1) != 0 or dst["status"] != 0 or not shards_ok or (dist is not None and not same)
    drqn = time_drqn_update(L.learner) if world == 1 else None
    if rank == 0:
        value = n * world * args.steps / dt
        fpa = RNN_FLOP_PER_ARENA // 2 if overlap else RNN_FLOP_PER_ARENA  # overlap: modelB's side only
        achieved = n * fpa / act_s / 1e12
        env_gbs = n * RNN_ENV_BYTES / env_s / 1e9
        out = {
            "metric": "env-steps/sec (whole node), QNetRNN self-play + DRQN (configs[4])",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": warm,
            "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64 env state / f32 QNetRNN",
            "data": "synthetic (random-init QNetRNN weights of the reference architecture, Philox serves)",
            "config": {"workload": "configs[4]: 32768 arenas/GPU, train_rnn_iterative loop (QNetRNN act both players "
                                   "with (h, c) per arena + env tick + sequence buffer + DRQN update 64x8 BPTT + "
                                   "clip + Adam every vector step)",
                       "arenas_per_gpu": n, "global_arenas": n * world, "pool": pool_n, "batch": 64, "trace_length": 8,
                       "memory_size": L.cap, "ring_depth": L.depth,
                       "updates_in_timed_region": c1["train_steps"] - c0["train_steps"],
                       "parallelism": f"dp{world} (arena shards, 1 all-reduce/update)",
                       "all_reduce": args.comm_used if world > 1 else None, "replicas_identical": same,
                       "shards": shards},
            "roofline": {"bound": "mfma",
                         "kernel": "k_rnn_act side B: the overlapped step's act for modelB" if overlap
                                   else "k_rnn_act (both players)",
                         "timing": "the launch's own begin/end (hipExtLaunchKernel events, pm_timer_arm) "
                                   "on instrumented production steps after the timed region",
                         "compute": "v_mfma_f32_32x32x2_f32 (exact fp32; dense FP32 matrix peak 157.3 TF)",
                         "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                         # modelB's side: 256 blocks x 256 lanes (the overlapped step's only k_rnn_act of
                         # that grid); the plain step's both-players launch has no committed pass
                         "traffic": pmc_traffic(f"k_rnn_act@{256 * 256}", "r3_rnn_pmc.json") if overlap and n == 32768 else None,
                         "avg_us": round(act_s * 1e6, 2), "flop_per_arena": fpa, "n": n},
        }
        if overlap:
            out["env_update_us"] = round(env_s * 1e6, 2)  # env + sample + DRQN update, the opponents' act beside
        else:
            out["env_roofline"] = {"bound": "hbm", "kernel": "k_rsp_env + k_rsp_append + k_rsp_sample",
                                   "achieved": round(env_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                   "frac": round(env_gbs / PEAK_HBM_GBS, 4), "avg_us": round(env_s * 1e6, 2),
                                   "bytes_per_env_step": RNN_ENV_BYTES}
            out["drqn_update_us"] = round(upd_s * 1e6, 2)
        out.update({
            "learner": {"train_steps": c["train_steps"], "episodes": c["episodes"], "epsilon": c["epsilon"],
                        "seq_size": c["seq_size"], **dst, "status": c["status"], "drqn_status": dst["status"]},
            "drqn_roofline": drqn,
        })
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_rnn(args.cpu_seconds)
        if failed:
            out["error"] = "device status bit 0 (overwritten ring read) / shard proof failed"
        emit(out)
    if dist is not None:
        dist.destroy_process_group()
    if failed:
        sys.exit(3)


def cpu_baseline_infer(seconds=12.0, n=4096, replay_cap=0):
    from threadpoolctl import threadpool_limits
    from oracle.cpu_selfplay import CpuRollout
    sdB, _, _, _ = bench_nets("reference", 0)
    np_sd = lambda s: {k: v.numpy() for k, v in s.items()}  # noqa: E731
    with threadpool_limits(1):
        cpu = CpuRollout(ENV_KW, n, np_sd(sdB), np_sd(sdB), epsilon=0.02, replay_cap=replay_cap)
        cpu.step()
        t0 = time.perf_counter()
        steps = 0
        while time.perf_counter() - t0 < seconds:
            cpu.step()
            steps += 1
        dt = time.perf_counter() - t0
    return {"value": round(n * steps / dt, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/cpu_selfplay.py CpuRollout: {steps} vector steps x {n} arenas (both players' QNet "
                      f"f32 + fresh noise per step + eps-greedy + C oracle tick + reset on done"
                      f"{f' + memory.push into a {replay_cap}-row ring' if replay_cap else ''}), {dt:.1f} s on 1 host core",
            "reference_python_measured": "4 600 env-steps/s, batch-1 QNet rollout, 1 thread (SURVEY 6)"}


def infer_traffic(n, chunk, pmc_steps=2000, kernel="k_rollout"):
    """`kernel`'s (k_rollout / k_rollout16) HBM bytes for a launch of `chunk` steps, scaled from the
    committed counter pass (profiles/r4_infer_pmc.json or r3_infer_pmc.json: launches of 2 000 steps
    at 4 096 arenas); None at other sizes."""
    b = pmc_traffic(kernel, "r3_infer_pmc.json")
    return None if b is None or n != 4096 else round(b * chunk / pmc_steps, 1)


def time_infer_stepped(wA, pB, n=4096, per_graph=100, replays=5):
    """The composition K9 replaces, for comparison: per vector step pm_qnet_fold (modelB, fresh noise)
    -> pm_qnet_act (both players) -> pm_env_step (autoreset), `per_graph` steps captured in one HIP
    graph (SURVEY 8d's configs[1] recipe), HIP events over `replays` replays."""
    from pongmi import _lib
    from pongmi.env import PongEnv2PBatch
    from pongmi.qnet import act, fold
    env = PongEnv2PBatch(n, seed=0x5EED, autoreset=True, **ENV_KW)
    env.reset()
    wA2 = wA.reshape(1, -1)

    def steps():
        for _ in range(per_graph):
            c = env.counter
            wB = fold(pB, _lib.PM_FOLD_TRAIN_FRESH, seed=0x5EED, counter=c)
            aA, aB = act(wA2, None, wB, env.obsA, env.obsB, 0.02, seed=env.seed, counter=c)
            env.step(aA, aB)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        steps()  # warm-up (allocations, lazy loads)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            steps()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(replays):
            g.replay()
        e1.record(s)
    e1.synchronize()
    t = e0.elapsed_time(e1) * 1e-3 / (per_graph * replays)
    return {"value": round(n / t, 1), "us_per_step": round(t * 1e6, 3), "launches_per_step": 3,
            "timing": f"{per_graph} vector steps per HIP graph, events over {replays} replays"}


REPLAY_BYTES = 16 * 4 + 4 + 4  # per pushed transition: the 64-B row, its priority and its PER leaf


def run_infer(args, dist, rank, world):
    """configs[1]: 4096 arenas/GPU, QNet inference-only self-play (both players act, modelB with fresh
    NoisyNet noise per vector step and eps = 0.02, autoreset), as the K9 megakernel (pm_rollout):
    `--infer-chunk` vector steps per launch, the arenas in registers in between. Shards are independent
    (per-rank env seed), no collective.

    --workload collect: the same launches at configs[2]'s 65 536 arenas with every
    transition pushed into a 1e6-row PER replay ring (pm_rollout_push; the sum tree's nodes rebuilt
    after each launch): as many vector steps per launch as the ring holds without a slot being
    written twice (15)."""
    from pongmi import _lib
    from pongmi.env import PongEnv2PBatch
    from pongmi.qnet import fold, pack_state_dict
    from pongmi.replay import DeviceReplay
    from pongmi.rollout import STATS, STATS_PUSH, SelfPlayRollout
    collect = args.workload == "collect"
    n = args.arenas or (65536 if collect else 4096)
    steps = args.steps
    chunk = max(1, min(args.infer_chunk, steps))
    replay = None
    if collect:
        replay = DeviceReplay(args.memory, "cuda")
        chunk = max(1, min(chunk, args.memory // n))
        STATS = STATS_PUSH  # noqa: N806
    sdB, sdA, _, wdesc = bench_nets(args.weights, 0)
    pB = pack_state_dict(sdB).reshape(-1)
    wA = fold(pack_state_dict(sdA), _lib.PM_FOLD_TRAIN).reshape(-1)  # modelA: mu + sigma * (its frozen eps)
    env = PongEnv2PBatch(n, seed=0x5EED + rank, autoreset=True, **ENV_KW)
    env.reset()
    R = SelfPlayRollout(env, wA, pB, epsilon=0.02, seed_net=0x5EED + 1000 * rank)
    # the warm-up runs long enough (>= 5000 vector steps, ~15 ms) for the clocks to settle: a 100-step
    # warm-up left the first ~30 ms of the timed launch at ramp-up clocks (timed region 2x the launch)
    warm = max(args.warmup, 5000 if not collect else 600)
    R.reserve(chunk if collect else max(chunk, warm))  # the heads workspace is allocated before the timed region
    tot = torch.zeros(len(STATS), dtype=torch.int64, device="cuda")

    def run(k):
        done = 0
        while done < k:
            c = min(chunk, k - done)
            tot.add_(R.run(c, sync=False, replay=replay)[:len(STATS)])
            done += c

    run(warm)  # the same calls as the timed region (torch loads its add kernel lazily on first use)
    torch.cuda.synchronize()
    tot.zero_()

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        dist.all_reduce(tot)
    # after the timed region: the megakernel's own dispatch (pm_timer_arm, as rocprofv3 times it) on
    # `reps` launches of `chunk` steps, and the same launches bracketed by HIP events on the stream
    reps = 3
    ks = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        _lib.timer_arm(_lib.PM_TIMER_ROLLOUT)
        R.run(chunk, sync=False, replay=replay)
    e1.record()
    e1.synchronize()
    ks = [_lib.timer_read(_lib.PM_TIMER_ROLLOUT) for _ in range(reps)]
    k_s = sum(ks) / reps
    ev_s = e0.elapsed_time(e1) * 1e-3 / reps
    st = dict(zip(STATS, tot.cpu().tolist()))
    r16 = int(os.environ.get("PONGMI_ROLL16", "1") or "1")  # the library's tile choice (pm_rollout.hip roll16)
    tile16 = bool(r16 & (2 if collect else 1))
    if rank == 0:
        value = n * world * steps / dt
        flop = n * chunk * 2 * FLOP_PER_ARENA
        achieved = flop / k_s / 1e12
        out = {
            "metric": "env-steps/sec (whole node), QNet inference-only self-play rollout (configs[1])",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": steps, "warmup": warm,
            "ms_per_step": round(dt / steps * 1e3, 5), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64 env state / f32 QNet",
            "data": f"synthetic: the env's own Philox serves; {wdesc}",
            "config": {"workload": "configs[1]: 4096 arenas/GPU, QNet inference-only self-play rollout (modelA "
                                   "greedy on mu + sigma*eps, modelB fresh noise every vector step + eps-greedy "
                                   "0.02, autoreset)",
                       "arenas_per_gpu": n, "global_arenas": n * world, "steps_per_launch": chunk,
                       "launches_in_timed_region": -(-steps // chunk), "parallelism": f"dp{world} (independent "
                       "arena shards, no collective)"},
            "roofline": {"bound": "mfma", "kernel": (f"k_rollout16 (K9 on 16-arena tiles, v_mfma_f32_16x16x4_f32" if tile16
                                                     else "k_rollout (K9 on 32-arena tiles") +
                                                    f": both players' QNet forward + env tick, {chunk} vector steps per launch)",
                         "compute": f"{'v_mfma_f32_16x16x4_f32' if tile16 else 'v_mfma_f32_32x32x2_f32'} (exact fp32; "
                                    "dense FP32 matrix peak 157.3 TF)",
                         "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": infer_traffic(n, chunk, kernel="k_rollout16" if tile16 else "k_rollout"),
                         "avg_us": round(k_s * 1e6, 1), "avg_us_per_step": round(k_s / chunk * 1e6, 4),
                         "flop_per_env_step": 2 * FLOP_PER_ARENA, "n": n,
                         "waves": 8 * (-(-n // 16)) if tile16 else 4 * (-(-n // 32)), "wave_slots": 256 * 4,
                         "timing": f"pm_timer_arm dispatch of {reps} launches after the timed region; "
                                   f"HIP events incl. the heads fold: {ev_s * 1e6:.1f} us per launch"},
            "rollout": st,
            "stepped": time_infer_stepped(wA, pB, n) if world == 1 else None,
        }
        if world == 1 and not args.no_cpu_baseline:
            # collect: the port at 4 096 arenas with the push (the 65 536-arena vector step would take
            # most of the bounded sample per step)
            out["cpu_baseline"] = cpu_baseline_infer(args.cpu_seconds, 4096 if collect else n,
                                                     replay_cap=args.memory if collect else 0)
        if collect:
            rb = n * chunk * REPLAY_BYTES / k_s / 1e9
            out["metric"] = ("env-steps/sec (whole node), collecting self-play rollout: every transition pushed "
                             "into the PER replay ring (SURVEY 8f3)")
            out["config"]["workload"] = (f"8f3 at configs[2]'s arena count: {n} arenas/GPU, the configs[1] rollout "
                                         f"(eps 0.02 held, learner off) + memory.push of every transition into a "
                                         f"{args.memory}-row PER ring, {chunk} vector steps per launch")
            out["config"]["replay_cap"] = args.memory
            out["roofline"]["kernel"] = (f"{'k_rollout16_push' if tile16 else 'k_rollout_push'} (both players' QNet "
                                         f"forward + env tick + replay push, {chunk} vector steps per launch)")
            # HBM bytes per launch from the committed counter passes (profiles/r3_collect_pmc.json,
            # round 3: 65 536 arenas, 15-step launches); None at other shapes
            tb = pmc_traffic("k_rollout_push", "r3_collect_pmc.json")
            out["roofline"]["traffic"] = tb if (n, chunk) == (65536, 15) else None
            out["roofline"]["algorithmic_bytes"] = n * chunk * REPLAY_BYTES + n * (136 + 56)
            out["replay_roofline"] = {"bound": "hbm", "achieved": round(rb, 2), "peak": PEAK_HBM_GBS,
                                      "unit": "GB/s", "frac": round(rb / PEAK_HBM_GBS, 4),
                                      "bytes_per_transition": REPLAY_BYTES,
                                      "note": "replay-write bytes (row 64 + priority 4 + PER leaf 4) per launch / "
                                              "k_rollout_push dispatch time; the launch is MFMA-latency bound"}
            out["stepped"] = None
            out["replay"] = {"pos": replay.pos, "size": replay.size}
        emit(out)
    if dist is not None:
        dist.destroy_process_group()


REF_LOOP_STEPS_PER_S = {"small_buffer": 398, "fill_100k": 209, "fill_1e6": 75}  # SURVEY 6, 1 CPU thread


def run_train(args, dist, rank, world):
    """The real training path at the reference's replay ratio: one
    config.yaml generation try as pongmi.generations.QNetGenerations runs it — `episodes_per_generation`
    (2 400) episodes of self-play on `--arenas` (512) arenas with U = replay_ratio x arenas updates per
    vector step (1.0: one PER update of batch 256 per pushed transition, the reference's one update per
    env step, scripts/train_iterative.py:239-245), PER cap 1e6 starting empty, target sync every 1 000
    updates, then the try's evaluation (eval_vs_model + eval_vs_pool, 1 000 episodes each,
    :171-196). value = env-steps/s over the play phase (wall clock, from an empty replay as a
    generation starts); also updates/s, the play / evaluation / try wall seconds, and k_learn_multi's
    per-update time from its own dispatch. Shards (N > 1) would be independent tries: the controller
    is single-GPU (U > 1 steps are unsharded, pm_selfplay_step_multi)."""
    import yaml
    from pongmi import _lib
    from pongmi.evaluate import eval_vs_model, eval_vs_pool
    from pongmi.generations import _env_kw, _play_episodes, updates_for
    from pongmi.selfplay import SelfPlayLearner
    if world > 1:
        raise SystemExit("--workload train is a single-GPU generation try (the reference's controller); use --gpus 1")
    with open(os.path.join(ROOT, "pingpong-selfplay-ai_amd", "config.yaml")) as fh:
        cfg = yaml.safe_load(fh)
    t = cfg["training"]
    env_kw = _env_kw(cfg)
    n = args.arenas or 512
    U = updates_for(n, args.replay_ratio)
    pool_n = 8 if args.pool is None else args.pool
    sdB, _, pool, wdesc = bench_nets(args.weights, pool_n)
    episodes = int(args.episodes or t["episodes_per_generation"])
    eval_eps = int(t["eval_episodes"])

    def learner(seed):
        return SelfPlayLearner(env_kw, n, sdB, sdB, pool, batch=t["batch_size"], memory_size=t["memory_size"],
                               gamma=t["gamma"], lr=t["lr"], epsilon=t["min_epsilon"], min_epsilon=t["min_epsilon"],
                               epsilon_decay=t["epsilon_decay"], target_update_interval=t["target_update_interval"],
                               pool_ratio=t["opponent_pool_ratio"], seed=seed, updates_per_step=U)

    class _Quiet:  # _play_episodes' progress hook without console lines
        def tick(self, c):
            pass

    # warm-up on a throwaway learner (module load, lazy allocations), so the try starts like a
    # generation does: empty replay, episode count 0
    W = learner(99)
    for _ in range(max(2, args.warmup)):
        W.step()
    torch.cuda.synchronize()
    del W
    import random as _random
    rng = _random.Random(5)
    L = learner(7)
    c0 = L.counters()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c1 = _play_episodes(L, episodes, _Quiet(), 4)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    B = (L.modelB_state_dict(), _lib.PM_FOLD_TRAIN)
    wA = eval_vs_model(env_kw, (L.modelA_state_dict(), _lib.PM_FOLD_TRAIN), B, eval_eps, rng=rng)
    wP = eval_vs_pool(env_kw, B, [(sd, _lib.PM_FOLD_EVAL) for sd in pool], eval_eps, rng=rng)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    L.check_status(c1)
    # k_learn_multi (updates 1..U-1 of a vector step) by its own dispatch, after the try
    um = []
    for _ in range(5):
        _lib.timer_arm(_lib.PM_TIMER_LEARN_MULTI)
        L.step()
        um.append(_lib.timer_read(_lib.PM_TIMER_LEARN_MULTI))
    multi_s = sum(um) / len(um)
    play_s, eval_s = t1 - t0, t2 - t1
    vsteps = c1["step"] - c0["step"]
    env_steps = vsteps * n
    upd = c1["train_steps"] - c0["train_steps"]
    if rank == 0:
        value = env_steps / play_s
        out = {
            "metric": "env-steps/sec, one config.yaml generation try of the train_iterative loop at the reference's "
                      "replay ratio (1 update of 256 per env step)",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": vsteps, "warmup": args.warmup,
            "ms_per_step": round(play_s / max(vsteps, 1) * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64 env state / f32 QNet",
            "data": f"synthetic (env Philox serves; {wdesc})",
            "config": {"workload": f"train: config.yaml generation try, {episodes} episodes on {n} arenas, U = {U} "
                                   f"updates per vector step (replay ratio {args.replay_ratio}), PER cap "
                                   f"{t['memory_size']} from empty, batch {t['batch_size']}, target sync every "
                                   f"{t['target_update_interval']}, then eval 2 x {eval_eps} episodes",
                       "arenas": n, "updates_per_vector_step": U, "pool": pool_n, "episodes": c1["episodes"] - c0["episodes"],
                       "learn_multi": L.frow is not None},
            "updates": upd, "updates_per_s": round(upd / play_s, 1), "play_s": round(play_s, 3),
            "eval_s": round(eval_s, 3), "generation_try_s": round(play_s + eval_s, 3),
            "eval": {"vs_A": wA, "vs_pool": wP},
            "learn_multi_us_per_update": round(multi_s / max(U - 1, 1) * 1e6, 3),
            "learn_multi_launch_us": round(multi_s * 1e6, 1),
            "reference_python_measured": {"steps_per_s": REF_LOOP_STEPS_PER_S,
                                          "note": "train_iterative.py step body (1 env step + 1 update of 256), 1 CPU "
                                                  "thread (SURVEY 6); a 2 400-episode try is ~91 k steps"},
            "vs_reference_loop": {k: round(value / v, 1) for k, v in REF_LOOP_STEPS_PER_S.items()},
        }
        emit(out)


def emit(out):
    """Rank 0's one JSON line (marked when the ranks are a rehearsal sharing GPUs, see rehearsal())."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and rehearsal(os.environ):
        out["rehearsal"] = ("N ranks sharing the visible GPU(s) over gloo (PONGMI_BENCH_REHEARSE=1): a check of the "
                            "multi-rank path, not a scaling number")
    print(json.dumps(out), flush=True)


def rehearsal(env):
    """PONGMI_BENCH_REHEARSE=1 (a test hook the driver never sets): N > 1 ranks may share the visible
    GPUs (rank r on device r mod count) and talk over gloo, so the multi-rank path (spawn, barriers,
    max-over-ranks timing, the shard proof, replica identity, the sharded steps) runs end to end on a
    1-GPU box. The line says so ("rehearsal") and is no scaling number: the ranks share one device."""
    return env.get("PONGMI_BENCH_REHEARSE", "0") not in ("", "0")


def launch_plan(argv, env, device_count):
    """What `python bench.py --gpus N ...` does before any GPU call. Returns
    ("run", None) when this process is the (only or torchrun-launched) rank that should run, ("spawn",
    cmd) when N > 1 ranks are asked for and no launcher started us (WORLD_SIZE unset): cmd starts
    torch.distributed.run with N ranks on this same bench, which this process then waits on as a
    child (never exec: the parent exits with the child's code), or ("error", message) when the
    request cannot be honoured — WORLD_SIZE set and != --gpus, or fewer visible devices than ranks.
    `device_count` is torch.cuda.device_count() (which does not initialise the GPU on this image)
    or None to skip that check."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    ns, _ = ap.parse_known_args(argv)
    n = ns.gpus
    if n < 1:
        return "error", f"--gpus {n}: need at least one GPU"
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != n:
            return "error", (f"--gpus {n} but WORLD_SIZE={ws}: the launcher started a different number of ranks "
                             f"than the bench was asked to report")
        if device_count is not None and int(env.get("LOCAL_RANK", "0")) >= device_count and not rehearsal(env):
            return "error", f"LOCAL_RANK {env.get('LOCAL_RANK')} but only {device_count} visible GPU(s)"
        return "run", None
    if n == 1:
        return "run", None
    if device_count is not None and device_count < n and not rehearsal(env):
        return "error", f"--gpus {n} but only {device_count} visible GPU(s) on this node"
    import socket
    with socket.socket() as s:  # a free rendezvous port on the loopback (the hostname may not resolve)
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return "spawn", cmd


def main():
    plan, what = launch_plan(sys.argv[1:], os.environ, torch.cuda.device_count())
    if plan == "error":
        print(json.dumps({"error": what, "argv": sys.argv[1:]}), flush=True)
        sys.exit(2)
    if plan == "spawn":
        import subprocess
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        sys.exit(subprocess.call(what, env=env))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="vector steps timed (200; infer: 10000)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed vector steps first (30; infer: 100)")
    ap.add_argument("--workload", choices=("dqn", "rnn", "infer", "collect", "train"), default="dqn",
                    help="dqn: configs[2] (the headline); rnn: configs[4], the QNetRNN / DRQN loop; infer: "
                         "configs[1], the inference-only rollout megakernel; collect: 8f3, that megakernel "
                         "pushing every transition into the PER replay ring at 65 536 arenas; train: one config.yaml "
                         "generation try at the reference's replay ratio (QNetGenerations' loop)")
    ap.add_argument("--replay-ratio", type=float, default=1.0, help="train: updates per pushed transition")
    ap.add_argument("--episodes", type=int, default=None, help="train: episodes per try (config.yaml: 2400)")
    ap.add_argument("--infer-chunk", type=int, default=10000, help="infer: vector steps per pm_rollout launch")
    ap.add_argument("--arenas", type=int, default=None, help="arenas per GPU (65536 dqn, 32768 rnn)")
    ap.add_argument("--pool", type=int, default=None, help="opponent pool size (synthetic nets; 8 dqn, 4 rnn)")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--memory", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--updates-per-step", type=int, default=1,
                    help="dqn: PER updates of `batch` per vector step (U; SURVEY 8d: 1 default, 64 the stress "
                         "variant; the reference's own ratio is one update per env step, i.e. U = arenas)")
    ap.add_argument("--no-learn-multi", action="store_true",
                    help="dqn, U > 1: updates 1..U-1 as three launches each (resample, batch forward, learn) "
                         "instead of one single-workgroup launch for all of them (k_learn_multi)")
    ap.add_argument("--weights", choices=("reference", "random"), default="reference",
                    help="reference: model5-5_fault.pth's QNet weights (tests/golden/qnet.npz) for modelB and modelA "
                         "(SURVEY 8d); random: random-init nets of the reference architecture")
    ap.add_argument("--no-overlap", action="store_true", help="dqn: plain step (opponent act in k_act_sp, not in the learner launch)")
    ap.add_argument("--no-features-ahead", action="store_true",
                    help="dqn: k_actenv's env blocks run modelB's whole forward (features + heads) themselves instead "
                         "of reading the features the previous learner launch computed ahead (featB): the A/B of the "
                         "featB round trip")
    ap.add_argument("--comm", choices=("native", "torch"), default="native",
                    help="N > 1: the gradient all-reduce as libpongmi's own RCCL communicator inside one library "
                         "call per vector step (native), or torch.distributed.all_reduce between launches (torch)")
    args = ap.parse_args()
    infer = args.workload in ("infer", "collect")
    collect = args.workload == "collect"
    args.steps = args.steps if args.steps is not None else (3000 if collect else 10000 if infer else 200)
    args.warmup = args.warmup if args.warmup is not None else (100 if infer else 4 if args.workload == "train" else 30)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    assert world == args.gpus, (world, args.gpus)  # launch_plan guarantees it
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # configs[0]'s scalar CPU loop runs in forked worker processes: before this process touches the GPU
    args.cpu_config0 = cpu_config0() if world == 1 and args.workload == "dqn" and not args.no_cpu_baseline else None
    rehearse = world > 1 and rehearsal(os.environ)
    if rehearse:  # ranks share the visible devices; gloo, torch.distributed all-reduce (RCCL wants one GPU per rank)
        local = local % max(torch.cuda.device_count(), 1)
        args.comm = "torch"
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    comm = None
    if dist is not None and args.comm == "native" and not infer:
        from pongmi.dist import NativeComm
        comm = NativeComm()  # raises on every rank if RCCL cannot be bound: no silent fallback
    args.comm_used = ("native RCCL, in-stream" if comm is not None
                      else "torch.distributed (gloo)" if rehearse else "torch.distributed")
    args.comm = comm
    allreduce = comm if comm is not None else ((lambda t: dist.all_reduce(t)) if dist else None)

    if args.workload == "rnn":
        return run_rnn(args, dist, rank, world, allreduce)
    if args.workload == "train":
        return run_train(args, dist, rank, world)
    if infer:
        return run_infer(args, dist, rank, world)
    args.arenas = args.arenas or 65536
    args.pool = 8 if args.pool is None else args.pool
    from pongmi import _lib
    from pongmi.selfplay import SelfPlayLearner

    U = max(1, int(args.updates_per_step))
    nets = bench_nets(args.weights, args.pool)
    sdB, sdA, pool, wdesc = nets
    L = SelfPlayLearner(ENV_KW, args.arenas, sdB, sdA, pool, batch=args.batch, memory_size=args.memory,
                        epsilon=0.08, seed=7, rank=rank, world=world, allreduce=allreduce,
                        overlap=not args.no_overlap, updates_per_step=U, learn_multi=not args.no_learn_multi,
                        features_ahead=not args.no_features_ahead)

    def one_step(ev=None):
        # the production path: the overlapped vector step (L.step); an instrumented step is the same
        # call with both of its launches armed (pm_timer_arm: each dispatch records its own begin/end,
        # no marker packets join the stream)
        if ev is not None:
            _lib.timer_arm(_lib.PM_TIMER_ACTENV)
            _lib.timer_arm(_lib.PM_TIMER_LEARN)
        L.step()

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    c0 = L.counters()
    ae_t, learn_t = [], []

    def read_timers():
        ae_t.append(_lib.timer_read(_lib.PM_TIMER_ACTENV))
        learn_t.append(_lib.timer_read(_lib.PM_TIMER_LEARN))

    dt, _, c1 = timed_region(one_step, args.steps, dist, 0, read_timers, L.counters)
    same = replicas_identical(dist, L.paramsB)
    ae_s = sum(ae_t) / len(ae_t)  # the launches' own durations, as rocprofv3 --kernel-trace times them
    learn_s = sum(learn_t) / len(learn_t)
    c = L.counters()
    shards, shards_ok = shard_proof(dist, rank, world, args.arenas, c["step"], c["status"], args.comm, L.grad)
    failed = c["status"] != 0 or not shards_ok or (dist is not None and not same)

    if rank == 0:
        total = args.arenas * world * args.steps
        value = total / dt
        ahead = L.featB is not None
        learn_flop = FLOP_PER_ARENA + (FEAT_FLOP_PER_ARENA if ahead else 0)
        achieved = args.arenas * learn_flop / learn_s / 1e12
        env_bytes = SP_ENV_BYTES + (FEAT_BYTES if ahead else 0)
        env_gbs = args.arenas * env_bytes / ae_s / 1e9
        ae_grid = (args.batch + 63) // 64 + (args.arenas + 255) // 256
        out = {
            "metric": "env-steps/sec (whole node) at 65536 arenas, 1/2/4/8 GPUs; CPU-ref baseline",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64 env state / f32 QNet",
            "data": f"synthetic observations from the env itself (Philox serves); {wdesc}",
            "config": {"workload": "configs[2]: 65536 arenas/GPU, full DQN train_iterative loop (act both players + "
                                   "env tick + PER push/sample + double-DQN update + Adam + target sync)",
                       "arenas_per_gpu": args.arenas, "global_arenas": args.arenas * world,
                       "pool": args.pool, "batch": args.batch, "updates_per_vector_step": U,
                       "updates_in_timed_region": c1["train_steps"] - c0["train_steps"],
                       "memory_size": args.memory, "parallelism": f"dp{world} (arena shards, 1 all-reduce/update)",
                       "all_reduce": args.comm_used if world > 1 else None, "replicas_identical": same,
                       "shards": shards},
            "roofline": {"bound": "mfma",
                         "kernel": "k_learn launch: the double-DQN update (one workgroup) + the next step's "
                                   "opponents' act and modelB's feature layers on the other CUs",
                         "compute": "v_mfma_f32_32x32x2_f32 (exact fp32; dense FP32 matrix peak 157.3 TF)",
                         "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": pmc_traffic("k_learn") if U == 1 else None,
                         "avg_us": round(learn_s * 1e6, 2), "flop_per_arena": learn_flop, "n": args.arenas},
            "env_roofline": {"bound": "hbm",
                             "kernel": "k_actenv (modelB's heads + env tick + replay push + PER sample / batch "
                                       "forward)" if ahead else "k_actenv (modelB's act + env tick + replay push + "
                                                                "PER sample / batch forward)",
                             "achieved": round(env_gbs, 1), "peak": PEAK_HBM_GBS,
                             "unit": "GB/s", "frac": round(env_gbs / PEAK_HBM_GBS, 4),
                             "traffic": pmc_traffic(f"k_actenv@{ae_grid * 256}") if U == 1 else None,
                             "avg_us": round(ae_s * 1e6, 2), "bytes_per_env_step": env_bytes},
            "learn_us": round(learn_s * 1e6, 2), "actenv_us": round(ae_s * 1e6, 2),
            "learner": {"train_steps": c["train_steps"], "episodes": c["episodes"], "epsilon": c["epsilon"],
                        "last_loss": c["last_loss"], "status": c["status"]},
        }
        if U > 1:
            out["us_per_update"] = round(dt / args.steps / U * 1e6, 3)
            out["learn_multi"] = L.frow is not None
        if world == 1:
            out["act_full_roofline"] = time_act_full(L)
            out["env_step_roofline"] = time_env_step(args.arenas)
            out["scalar_dropin"] = time_scalar_dropin()
            if not args.no_cpu_baseline:
                out["cpu_baseline"] = cpu_baseline(args.arenas, nets, args.cpu_seconds)
                out["cpu_config0"] = args.cpu_config0
        if failed:
            out["error"] = "device status / shard proof failed: see learner.status and config.shards"
        emit(out)
    if dist is not None:
        dist.destroy_process_group()
    if failed:
        sys.exit(3)


def bench_nets(which, n_pool):
    """(modelB, modelA, pool, description). reference: SURVEY 8d's acting nets, model5-5_fault.pth's
    QNet (tests/golden/qnet.npz holds its modelB / modelA state_dicts, written by make_golden.py from
    the reference checkpoint) for modelB and for modelA; the pool is its modelA plus random-init nets
    (the reference's pool loads its legacy fc.* files with strict=False, i.e. as random nets)."""
    if which == "random":
        return (synthetic_qnet(1), synthetic_qnet(2), [synthetic_qnet(100 + k) for k in range(n_pool)],
                "random-init QNet weights of the reference architecture")
    g = np.load(os.path.join(ROOT, "tests", "golden", "qnet.npz"))
    sd = {who: {k[len(who) + 1:]: torch.from_numpy(g[k].copy()) for k in g.files
                if k.startswith(who + ".") and "q_" not in k} for who in ("modelB", "modelA")}
    pool = ([sd["modelA"]] if n_pool else []) + [synthetic_qnet(100 + k) for k in range(max(0, n_pool - 1))]
    return (sd["modelB"], sd["modelB"], pool,
            "model5-5_fault.pth QNet weights (modelB for both players; pool = its modelA + random-init nets)")


if __name__ == "__main__":
    main()
