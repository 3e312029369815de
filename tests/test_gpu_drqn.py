"""K6 — the DRQN update (pm_drqn_update) against train_step_rnn run on the reference QNetRNN with
torch autograd (tests/golden/drqn.npz) and against the float64 oracle (oracle.drqn_update).

Tolerances (fp32 on the device; exact-f32 MFMA sums in a different order than torch's CPU GEMMs):
loss / pre-clip norm rtol 1e-4; gradients rtol 1e-3 with atol 1e-5 x the tensor's largest
magnitude (the same bar the oracle meets against the reference). Parameters after clipped Adam
steps, as a band check: Adam normalises every element's step to ~lr = 1e-4 x sign(m), so an element
whose float64 gradient at some step is within the gradient tolerance of zero (|g| <= 2e-5 x the
tensor's largest |g|: the sign is a rounding decision) may move by up to 2 lr per step the other
way — the band, counted and printed; every other element must be within 1e-6 + 1e-5 |ref|, with no
fraction allowed to escape. The apply itself (clip + Adam given the device's gradient and norm) is
pinned bit for bit by test_drqn_clip_adam_exact.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sd(g):
    return {k[7:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("params.")}


def _batch(gd, k):
    return tuple(gd[f"b{k}_{n}"] for n in ("obs", "act", "rew", "next", "done"))


def _grads(L):
    from pongmi.rnn import PARAM_LAYOUT
    out, o = {}, 0
    g = L.grad.cpu().numpy()
    for k, s in PARAM_LAYOUT:
        n = int(np.prod(s))
        if "epsilon" not in k:
            out[k] = g[o:o + n].reshape(s)
        o += n
    return out


BAND_REL = 2e-5  # twice the gradient check's atol (1e-5 x the tensor's largest |g|)


def _band(grads_per_step, k):
    """Elements of parameter k whose float64 gradient at any step is within BAND_REL x the tensor's
    largest |g| of zero: their Adam direction is a rounding decision."""
    band = None
    for g in grads_per_step:
        g = np.asarray(g[k], np.float64)
        b = np.abs(g) <= BAND_REL * np.abs(g).max()
        band = b if band is None else band | b
    return band


def _assert_params(got, ref, what, steps, band, tally=None):
    got, ref = np.asarray(got, np.float64).reshape(-1), np.asarray(ref, np.float64).reshape(-1)
    band = np.asarray(band).reshape(-1)
    np.testing.assert_allclose(got[band], ref[band], rtol=0, atol=steps * 2e-4 * 1.01, err_msg=f"{what} (band)")
    np.testing.assert_allclose(got[~band], ref[~band], rtol=1e-5, atol=1e-6, err_msg=what)
    if tally is not None:
        tally[0] += int(band.sum())
        tally[1] += band.size
        err = np.abs(got - ref) / (1e-6 + 1e-5 * np.abs(ref))
        tally[2] = max(tally[2], float(np.max(err[~band], initial=0.0)))
        tally[3] += int((err[band] > 1.0).sum())  # band elements that did use the band


def _assert_grads(got, ref, what):
    worst = 0.0
    for k, r in ref.items():
        tol = 1e-5 * np.abs(r).max() + 1e-9
        np.testing.assert_allclose(got[k], r, rtol=1e-3, atol=tol, err_msg=f"{what}: {k}")
        worst = max(worst, float(np.max(np.abs(got[k] - r) / (tol + 1e-3 * np.abs(r)))))
    print(f"\n{what}: gradient error / tolerance (rtol 1e-3, atol 1e-5 max|g|) max {worst:.4f}")


def test_drqn_update_matches_reference(golden, orc):
    from pongmi.drqn import DRQNLearner
    gr, gd = golden("rnn"), golden("drqn")
    L = DRQNLearner(_sd(gr), batch=64, T=8)
    for k in range(3):
        L.update(*(torch.from_numpy(x) for x in _batch(gd, k)))
        st = L.stats()
        assert st["steps"] == k + 1
        np.testing.assert_allclose(st["loss"], gd[f"u{k}_loss"], rtol=1e-4)
        np.testing.assert_allclose(st["norm"], gd[f"u{k}_norm"], rtol=1e-4)
        if k == 0:
            _assert_grads(_grads(L), {k2[len("u0_grad."):]: v for k2, v in gd.items() if k2.startswith("u0_grad.")},
                          "update 0")
    # the band: the float64 oracle's gradients of the same three updates
    p64 = {k: v.numpy().astype(np.float64) for k, v in _sd(gr).items()}
    adam, gsteps = {}, []
    for k in range(3):
        p64, info = orc.drqn_update(p64, {k2: v.numpy().astype(np.float64) for k2, v in _sd(gr).items()}, adam, k + 1,
                                    _batch(gd, k))
        gsteps.append(info["grads"])
    sd = L.state_dict()
    tally = [0, 0, 0.0, 0]
    for k in (n[len("final_sub."):] for n in gd if n.startswith("final_sub.")):
        _assert_params(sd[k].numpy().reshape(-1)[::8], gd["final_sub." + k], k, 3, _band(gsteps, k).reshape(-1)[::8],
                       tally)
    print(f"\nparameters after 3 updates: {tally[0]} of {tally[1]} elements in the sign band, {tally[3]} of them "
          f"beyond 1e-6 + 1e-5 |ref|; worst off-band error / (1e-6 + 1e-5 |ref|) {tally[2]:.4f}")
    # targetB untouched (interval 2000), epsilon buffers unchanged
    assert torch.equal(L.target_state_dict()["lstm.weight_hh_l0"], _sd(gr)["lstm.weight_hh_l0"])
    assert torch.equal(sd["fc_A.weight_epsilon"], _sd(gr)["fc_A.weight_epsilon"])


@pytest.mark.parametrize("B,T", [(32, 3), (96, 5), (64, 1), (256, 8), (32, 64)])
def test_drqn_against_oracle_ragged(golden, orc, B, T):
    """Other batch / sequence sizes against the oracle, with a target net that differs from modelB.
    (256, 8) is the largest batch: k_dq_recur's 3 x 256 workgroups of 1024 threads are more than the
    chip holds at once, so the waits on lower-indexed workgroups (target Q, BPTT's dz) run with later
    workgroups not yet resident; (32, 64) is the longest sequence (T <= 64)."""
    from pongmi.drqn import DRQNLearner
    gr = golden("rnn")
    sd = {k[7:]: v for k, v in gr.items() if k.startswith("params.")}
    rng = np.random.default_rng(B * 100 + T)
    tsd = {k: (v + rng.normal(0, 0.02, v.shape).astype(np.float32)) if "epsilon" not in k else v for k, v in sd.items()}
    obs = rng.uniform(0, 1, (B, T, 7)).astype(np.float32)
    nxt = rng.uniform(0, 1, (B, T, 7)).astype(np.float32)
    act = rng.integers(0, 3, (B, T)).astype(np.int64)
    rew = rng.choice(np.array([-1, 0, 1], np.float32), (B, T)).astype(np.float32)
    done = rng.random((B, T)) < 0.3
    L = DRQNLearner({k: torch.from_numpy(v) for k, v in sd.items()}, {k: torch.from_numpy(v) for k, v in tsd.items()},
                    batch=B, T=T)
    L.grads(torch.from_numpy(obs), torch.from_numpy(act), torch.from_numpy(rew), torch.from_numpy(nxt),
            torch.from_numpy(done))
    info = orc.drqn_grads({k: v.astype(np.float64) for k, v in sd.items()},
                          {k: v.astype(np.float64) for k, v in tsd.items()}, obs, act, rew, nxt, done)
    np.testing.assert_allclose(L.stats()["loss"], info["loss"], rtol=1e-4)
    L.apply()  # the sigma gradients (mu gradient x epsilon) are formed after the all-reduce, in apply
    _assert_grads(_grads(L), info["grads"], f"B={B} T={T}")
    new, _ = orc.drqn_update({k: v.astype(np.float64) for k, v in sd.items()},
                             {k: v.astype(np.float64) for k, v in tsd.items()}, {}, 1, (obs, act, rew, nxt, done))
    got = L.state_dict()
    tally = [0, 0, 0.0, 0]
    for k in orc.RNN_PARAM_KEYS:
        _assert_params(got[k].numpy(), new[k], k, 1, _band([info["grads"]], k), tally)
    print(f"B={B} T={T}: {tally[0]} of {tally[1]} parameters in the sign band, {tally[3]} of them beyond "
          f"1e-6 + 1e-5 |ref|; worst off-band error / (1e-6 + 1e-5 |ref|) {tally[2]:.4f}")


def test_drqn_deterministic_world_and_target_sync(golden):
    """Bit-identical across runs; a gradient summed over 2 ranks with world = 2 gives the same step;
    targetB <- modelB (all of it, epsilon buffers included) at every target_update_interval-th step."""
    from pongmi.drqn import DRQNLearner
    gr, gd = golden("rnn"), golden("drqn")
    b = tuple(torch.from_numpy(x) for x in _batch(gd, 1))
    runs = []
    for world in (1, 1, 2):
        L = DRQNLearner(_sd(gr), batch=64, T=8, target_update_interval=2)
        for step in (1, 2):
            L.grads(*b)
            if world == 2:
                L.grad.mul_(2.0)  # what the all-reduce of two identical replicas leaves (flag slot: 2 ranks)
            L.apply()
            assert torch.equal(L.params, L.target) == (step == 2)  # synced at step 2
        runs.append((L.params.clone(), L.adam_m.clone(), L.adam_v.clone(), L.stats()))
    for r in runs[1:]:
        assert torch.equal(r[0], runs[0][0]) and torch.equal(r[1], runs[0][1]) and torch.equal(r[2], runs[0][2])
        assert r[3] == runs[0][3]


def test_drqn_disabled_replica_contributes_nothing(golden):
    """enable = 0: grads() zeroes the gradient and the rank count; apply() then leaves everything
    untouched — a rank whose sequence buffer is not ready yet sits out an all-reduce."""
    from pongmi.drqn import DRQNLearner
    gr, gd = golden("rnn"), golden("drqn")
    en = torch.zeros(1, dtype=torch.int32, device="cuda")
    L = DRQNLearner(_sd(gr), batch=64, T=8, enable=en)
    p0 = L.params.clone()
    L.grad.fill_(3.0)
    L.update(*(torch.from_numpy(x) for x in _batch(gd, 0)))
    assert torch.count_nonzero(L.grad) == 0 and torch.equal(L.params, p0) and L.stats()["steps"] == 0
    en.fill_(1)
    L.update()
    assert L.grad[-4].item() == 1.0 and L.stats()["steps"] == 1 and not torch.equal(L.params, p0)
    np.testing.assert_allclose(L.stats()["loss"], gd["u0_loss"], rtol=1e-4)


def _adam_f32(p, m, v, g, norm, at, lr=1e-4, b1=0.9, b2=0.999, eps=1e-8, max_norm=1.0):
    """torch's clip_grad_norm_ + Adam step restated in float32 in the kernel's operation order (the
    clip coefficient from the device's own pre-clip norm, which is an fp64 sum in a fixed tree)."""
    f = np.float32
    coef = f(max_norm / (np.float64(f(norm)) + 1e-6))
    coef = min(coef, f(1.0))
    bc1, bc2 = 1.0 - b1 ** at, 1.0 - b2 ** at
    step_size, bc2s = f(lr / bc1), f(np.sqrt(bc2))
    gc = g.astype(f) * coef
    m = m + f(1.0 - b1) * (gc - m)
    v = v * f(b2) + f(1.0 - b2) * gc * gc
    denom = np.sqrt(v) / bc2s + f(eps)
    return p - step_size * (m / denom), m, v


def test_drqn_clip_adam_exact(golden):
    """The clip + Adam half of train_step_rnn is exact: given the update's own gradient (read back
    after apply, sigma slots formed) and its pre-clip norm, every parameter and both Adam moments
    equal a float32 restatement bit for bit, over three updates; the norm equals the fp64 norm of
    that gradient. With the gradients checked against autograd / the oracle above, this pins the
    parameters without the Adam sign-of-rounding escape (_assert_params)."""
    from pongmi._lib import PM_RNN_NPARAM
    from pongmi.drqn import DRQNLearner
    gr, gd = golden("rnn"), golden("drqn")
    L = DRQNLearner(_sd(gr), batch=64, T=8)
    for k in range(3):
        p0 = L.params.cpu().numpy()[:PM_RNN_NPARAM].copy()
        m0, v0 = L.adam_m.cpu().numpy().copy(), L.adam_v.cpu().numpy().copy()
        L.update(*(torch.from_numpy(x) for x in _batch(gd, k)))
        st = L.stats()
        g = L.grad.cpu().numpy()[:PM_RNN_NPARAM]
        np.testing.assert_allclose(st["norm"], np.sqrt(np.sum(g.astype(np.float64) ** 2)), rtol=1e-6)
        p, m, v = _adam_f32(p0, m0, v0, g, st["norm"], k + 1)
        np.testing.assert_array_equal(L.adam_m.cpu().numpy(), m, err_msg=f"exp_avg, update {k}")
        np.testing.assert_array_equal(L.adam_v.cpu().numpy(), v, err_msg=f"exp_avg_sq, update {k}")
        np.testing.assert_array_equal(L.params.cpu().numpy()[:PM_RNN_NPARAM], p, err_msg=f"params, update {k}")


def test_drqn_timeout_voids_update(golden):
    """A hand-off timeout inside pm_drqn_grads voids the update: forced with the poll_limit test hook
    (< 0: every in-launch wait times out at once), the update leaves parameters, target, Adam moments
    and the step counters untouched, latches status bits 2 (timed out) and 8 (voided), and
    check_status raises (RNNSelfPlayLearner.check_status calls it). Restoring the limit, the
    next update runs normally and equals a fresh learner's first update bit for bit."""
    from pongmi import _lib
    from pongmi.drqn import DRQNLearner
    gr, gd = golden("rnn"), golden("drqn")
    b = tuple(torch.from_numpy(x) for x in _batch(gd, 0))
    L = DRQNLearner(_sd(gr), batch=64, T=8, poll_limit=-1, target_update_interval=1)
    p0, t0 = L.params.clone(), L.target.clone()
    L.update(*b)
    st = L.stats()
    assert st["status"] & 2 and st["status"] & 8, st
    assert st["steps"] == 0 and st["adam_t"] == 0
    assert torch.equal(L.params, p0) and torch.equal(L.target, t0)  # interval 1: a sync would have copied
    assert torch.count_nonzero(L.adam_m) == 0 and torch.count_nonzero(L.adam_v) == 0
    assert L.grad[-3].item() > 0  # the void count that rides the all-reduce
    with pytest.raises(_lib.PongmiError):
        L.check_status()
    L.desc.poll_limit = 0
    L._set_stats(status=0)
    L.update(*b)
    assert L.stats()["status"] == 0 and L.stats()["steps"] == 1 and L.grad[-3].item() == 0
    R = DRQNLearner(_sd(gr), batch=64, T=8, target_update_interval=1)
    R.update(*b)
    assert torch.equal(L.params, R.params) and torch.equal(L.adam_v, R.adam_v) and torch.equal(L.target, R.target)
