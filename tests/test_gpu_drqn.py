"""K6 — the DRQN update (pm_drqn_update) against train_step_rnn run on the reference QNetRNN with
torch autograd (tests/golden/drqn.npz) and against the float64 oracle (oracle.drqn_grads).

Tolerances (fp32 on the device; exact-f32 MFMA sums in a different order than torch's CPU GEMMs):
loss / pre-clip norm rtol 1e-4; gradients rtol 5e-4 with atol 1e-5 x the tensor's largest magnitude
(round 5: the kernel's measured worst was 0.40 of the round-4 bar of rtol 1e-3), every update, every
tensor, except that the atol of a tensor is widened to 1.5x the error of the reference's own float32
autograd (torch, CPU, the reference module tree at the same parameters and batch) when that error is
larger (_assert_grads_conditioned): the device must be as close to float64 as the reference itself
is. Both errors are printed. Parameters are
pinned by composition, with no sign band: every update's gradient is checked against the oracle run
from the device's OWN pre-update parameters (so Adam's sign-of-rounding cannot drift the two apart),
and clip + Adam given that gradient and the device's pre-clip norm is checked bit for bit against
the float32 restatement oracle.clip_adam_f32 — every parameter, both moments, every update. The
parameters after the three fixture updates are also compared with the reference's own autograd run
(final_sub.*) under the sign band that Adam's normalised step needs there (_assert_final_sub).
"""
import os

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


def _assert_grads(got, ref, what, atol_rel=1e-5):
    worst = 0.0
    for k, r in ref.items():
        tol = atol_rel * np.abs(r).max() + 1e-9
        np.testing.assert_allclose(got[k], r, rtol=GRAD_RTOL, atol=tol, err_msg=f"{what}: {k}")
        worst = max(worst, float(np.max(np.abs(got[k] - r) / (tol + GRAD_RTOL * np.abs(r)))))
    print(f"\n{what}: gradient error / tolerance (rtol {GRAD_RTOL}, atol {atol_rel:g} max|g|) max {worst:.4f}")
    return worst


def _grad_err(got, ref, atol_rel=1e-5):
    """max over tensors of |got - ref| / (atol_rel max|ref| + GRAD_RTOL |ref|): <= 1 passes the bar."""
    worst = 0.0
    for k, r in ref.items():
        tol = atol_rel * np.abs(r).max() + 1e-9
        worst = max(worst, float(np.max(np.abs(got[k] - r) / (tol + GRAD_RTOL * np.abs(r)))))
    return worst


def ref32_grads(sd, tsd, obs, act, rew, nxt, done, gamma=0.99):
    """train_step_rnn's gradient (scripts/train_rnn_iterative.py:424-513) by torch autograd in
    float32 on the CPU, on the reference's module tree (models.qnet_rnn.QNetRNN's torch path, pinned
    to the reference module's outputs by tests/test_rnn_host.py): what the reference itself computes
    at these parameters. Its distance from the float64 oracle measures how well-conditioned the
    update is in float32."""
    from models.qnet_rnn import QNetRNN

    def net(state, train):
        m = QNetRNN(7, 3)
        m.load_state_dict({k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in state.items()})
        m.train(train)
        return m

    B = obs.shape[0]
    h0 = (torch.zeros(1, B, 128), torch.zeros(1, B, 128))
    mB, mT = net(sd, True), net(tsd, False)
    q = mB(torch.from_numpy(np.asarray(obs, np.float32)), h0)[0]
    with torch.no_grad():
        nx = torch.from_numpy(np.asarray(nxt, np.float32))
        a = mB(nx, h0)[0].argmax(1)
        y = torch.from_numpy(np.asarray(rew[:, -1], np.float32)) + gamma * mT(nx, h0)[0].gather(1, a[:, None])[:, 0] * \
            (1.0 - torch.from_numpy(np.asarray(done[:, -1], np.float32)))
    qa = q.gather(1, torch.from_numpy(np.asarray(act[:, -1], np.int64))[:, None])[:, 0]
    torch.nn.functional.smooth_l1_loss(qa, y).backward()
    return {k: v.grad.double().numpy() for k, v in mB.named_parameters()}


REF32_FACTOR = 1.5


def _assert_grads_conditioned(got, orc, sd, tsd, batch, what):
    """The device's gradient vs the float64 oracle, per tensor at atol = max(1e-5 x max|g|,
    REF32_FACTOR x the reference's own float32 error there) with rtol GRAD_RTOL: the bar widens only
    where the reference's float32 autograd (ref32_grads, same parameters, same batch) is itself that
    far from float64. Round 5's failing update (update 1 of the fixture: the device 4.5e-5 x max|g|
    off on the LSTM / feature gradients) is such a case: the reference's float32 autograd is 5.6e-5 x
    max|g| off there, 20x its error on update 0, with no ReLU or argmax decision near a tie (a
    conditioning effect of the batch, not a device defect). Prints both errors per tensor class."""
    info = orc.drqn_grads(sd, tsd, *batch)
    ref, r32 = info["grads"], ref32_grads(sd, tsd, *batch)
    worst = 0.0
    lines = []
    for k, r in ref.items():
        m = np.abs(r).max()
        e32 = float(np.abs(r32[k] - r).max())
        atol = max(1e-5 * m, REF32_FACTOR * e32) + 1e-9
        np.testing.assert_allclose(got[k], r, rtol=GRAD_RTOL, atol=atol, err_msg=f"{what}: {k}")
        worst = max(worst, float(np.max(np.abs(got[k] - r) / (atol + GRAD_RTOL * np.abs(r)))))
        if k in ("lstm.weight_hh_l0", "features_extractor.2.weight", "fc_shared_head.0.weight_mu"):
            lines.append(f"{k}: device {np.abs(got[k] - r).max() / m:.2e}, reference f32 {e32 / m:.2e} x max|g|")
    print(f"\n{what}: vs float64 — " + "; ".join(lines) + f"; error / bar max {worst:.4f}")
    return worst, ref


def _f64(sd):
    return {k: np.asarray(v, np.float64) for k, v in sd.items()}


def _assert_apply_exact(L, p0, m0, v0, at, what):
    """clip + Adam of the update just applied, given its own gradient (L.grad after apply: sigma slots
    formed) and pre-clip norm, equals oracle.clip_adam_f32 bit for bit; the norm is the fp64 norm of
    that gradient."""
    from pongmi._lib import PM_RNN_NPARAM
    st = L.stats()
    g = L.grad.cpu().numpy()[:PM_RNN_NPARAM]
    np.testing.assert_allclose(st["norm"], np.sqrt(np.sum(g.astype(np.float64) ** 2)), rtol=1e-6, err_msg=what)
    p, m, v, _ = orc_mod().clip_adam_f32(p0, m0, v0, g, st["norm"], at, max_norm=L.desc.max_norm, lr=L.desc.lr)
    np.testing.assert_array_equal(L.adam_m.cpu().numpy(), m, err_msg=f"exp_avg, {what}")
    np.testing.assert_array_equal(L.adam_v.cpu().numpy(), v, err_msg=f"exp_avg_sq, {what}")
    np.testing.assert_array_equal(L.params.cpu().numpy()[:PM_RNN_NPARAM], p, err_msg=f"params, {what}")


def orc_mod():
    from oracle import oracle
    return oracle


def _snap(L):
    from pongmi._lib import PM_RNN_NPARAM
    return (L.params.cpu().numpy()[:PM_RNN_NPARAM].copy(), L.adam_m.cpu().numpy().copy(),
            L.adam_v.cpu().numpy().copy())


GRAD_RTOL = 5e-4


def _assert_final_sub(L, gd, refs):
    """The parameters after the three fixture updates vs the reference's own autograd run
    (drqn.npz final_sub.*: every 8th element, make_golden_drqn.py). Adam normalises each element's
    step to ~lr x sign(m), so an element whose gradient at some update is within the gradient bar of
    zero (|g| <= 2e-5 x the tensor's max |g| in `refs`, the oracle gradients the updates were checked
    against) may step the other way: that sign band gets 2 lr per update and is counted; every other
    element must be within 1e-6 + 1e-5 |ref| (the round-4 check, kept beside the per-update
    composition checks: ADVICE r5)."""
    sd = L.state_dict()
    nband = ntot = 0
    worst = 0.0
    for name in (n[len("final_sub."):] for n in gd if n.startswith("final_sub.")):
        got = sd[name].numpy().astype(np.float64).reshape(-1)[::8]
        ref = gd["final_sub." + name].astype(np.float64).reshape(-1)
        band = np.zeros(ref.shape, bool)
        for g in refs:
            g = np.abs(np.asarray(g[name], np.float64))
            band |= (g <= 2e-5 * g.max()).reshape(-1)[::8]
        np.testing.assert_allclose(got[band], ref[band], rtol=0, atol=len(refs) * 2e-4 * 1.01, err_msg=f"{name} (band)")
        np.testing.assert_allclose(got[~band], ref[~band], rtol=1e-5, atol=1e-6, err_msg=name)
        nband += int(band.sum())
        ntot += band.size
        worst = max(worst, float(np.max(np.abs(got - ref)[~band] / (1e-6 + 1e-5 * np.abs(ref[~band])), initial=0.0)))
    print(f"parameters after {len(refs)} updates vs the reference's autograd run: {nband} of {ntot} elements in the "
          f"sign band; worst off-band error / (1e-6 + 1e-5 |ref|) {worst:.4f}")


def test_drqn_update_matches_reference(golden, orc):
    """Three updates on the reference's fixture batches: loss and pre-clip norm vs the reference's
    autograd run every update, update 0's gradients vs autograd; every update's gradient vs the float64
    oracle from the device's own pre-update parameters, and its clip + Adam bit for bit."""
    from pongmi.drqn import DRQNLearner
    gr, gd = golden("rnn"), golden("drqn")
    L = DRQNLearner(_sd(gr), batch=64, T=8)
    worst, refs = 0.0, []
    for k in range(3):
        p0, m0, v0 = _snap(L)
        sd_before = _f64(L.state_dict())
        L.update(*(torch.from_numpy(x) for x in _batch(gd, k)))
        st = L.stats()
        assert st["steps"] == k + 1
        np.testing.assert_allclose(st["loss"], gd[f"u{k}_loss"], rtol=1e-4)
        np.testing.assert_allclose(st["norm"], gd[f"u{k}_norm"], rtol=1e-4)
        if k == 0:
            _assert_grads(_grads(L), {k2[len("u0_grad."):]: v for k2, v in gd.items() if k2.startswith("u0_grad.")},
                          "update 0 vs autograd")
        # every update at the full bar, widened only where the reference's own float32 autograd is
        # farther from float64 (update 1: an ill-conditioned batch, see _assert_grads_conditioned)
        dump = os.environ.get("PONGMI_DRQN_DUMP")  # diagnosis: the device's parameters and gradient per update
        if dump:
            os.makedirs(dump, exist_ok=True)
            np.savez(os.path.join(dump, f"drqn_u{k}.npz"), **{"p." + n: v for n, v in sd_before.items()},
                     **{"g." + n: v for n, v in _grads(L).items()})
        w, ref = _assert_grads_conditioned(_grads(L), orc, sd_before, _f64(_sd(gr)), _batch(gd, k),
                                    f"update {k} vs oracle (device's own parameters)")
        worst, refs = max(worst, w), refs + [ref]
        _assert_apply_exact(L, p0, m0, v0, k + 1, f"update {k}")
    _assert_final_sub(L, gd, refs)
    # targetB untouched (interval 2000), epsilon buffers unchanged
    sd = L.state_dict()
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
    p0, m0, v0 = _snap(L)
    L.apply()  # the sigma gradients (mu gradient x epsilon) are formed after the all-reduce, in apply
    _assert_grads_conditioned(_grads(L), orc, {k: v.astype(np.float64) for k, v in sd.items()},
                       {k: v.astype(np.float64) for k, v in tsd.items()}, (obs, act, rew, nxt, done), f"B={B} T={T}")
    _assert_apply_exact(L, p0, m0, v0, 1, f"B={B} T={T}")


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


def test_drqn_clip_adam_exact(golden):
    """The clip + Adam half of train_step_rnn is exact: given the update's own gradient (read back
    after apply, sigma slots formed) and its pre-clip norm, every parameter and both Adam moments
    equal a float32 restatement bit for bit, over three updates; the norm equals the fp64 norm of
    that gradient. With the gradients checked against autograd / the oracle above, this pins the
    parameters with no sign-of-rounding band."""
    from pongmi._lib import PM_RNN_NPARAM
    from pongmi.drqn import DRQNLearner
    gr, gd = golden("rnn"), golden("drqn")
    L = DRQNLearner(_sd(gr), batch=64, T=8)
    for k in range(3):
        p0, m0, v0 = _snap(L)
        L.update(*(torch.from_numpy(x) for x in _batch(gd, k)))
        _assert_apply_exact(L, p0, m0, v0, k + 1, f"update {k}")


def test_drqn_clip_active_both_norm_paths(golden, orc):
    """max_norm small enough that the clip scales every gradient: the single-replica
    update (pm_drqn_update: the clip norm's shares summed by k_dq_wgrad's tiles) and the replica path
    (pm_drqn_grads -> pm_drqn_apply: k_dq_norm forms the same shares of the (all-reduced) gradient in
    the same order, round 6) each equal the float32 clip + Adam restatement bit for bit given their
    own gradient and norm, and with one rank the two are bit-identical: norm, parameters, moments."""
    from pongmi._lib import PM_RNN_NPARAM
    from pongmi.drqn import DRQNLearner
    gr, gd = golden("rnn"), golden("drqn")
    outs = []
    for split in (False, True):
        L = DRQNLearner(_sd(gr), batch=64, T=8, max_norm=0.01)
        for k in range(2):
            b = tuple(torch.from_numpy(x) for x in _batch(gd, k))
            p0, m0, v0 = _snap(L)
            if split:
                L.grads(*b)
                L.apply()
            else:
                L.update(*b)
            st = L.stats()
            assert 0.01 / (st["norm"] + 1e-6) < 1.0  # the clip is active
            _assert_apply_exact(L, p0, m0, v0, k + 1, ("split" if split else "fused") + f" update {k}")
        outs.append((st["norm"], L.params.clone(), L.adam_m.clone(), L.adam_v.clone(), L.grad.clone()))
    assert outs[0][0] == outs[1][0]
    for a, b in zip(outs[0][1:], outs[1][1:]):
        assert torch.equal(a, b)


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
