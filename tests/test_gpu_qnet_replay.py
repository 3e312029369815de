"""K2 (QNet fold / Q / fused two-player act) and K4 (PER sample / update) against the reference's
golden outputs and the oracle, on the device."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sd(g, who):
    return {k[len(who) + 1:]: torch.from_numpy(v) for k, v in g.items() if k.startswith(who + ".") and "q_" not in k}


def _obs(rng, n):
    lo = np.array([0, 0, -0.08, -0.08, 0, 0, -5], np.float32)
    hi = np.array([1, 1, 0.08, 0.08, 1, 1, 5], np.float32)
    return (lo + (hi - lo) * rng.random_sample((n, 7))).astype(np.float32)


def test_qnet_q_matches_reference_golden(golden):
    from pongmi import _lib
    from pongmi.qnet import fold, pack_state_dict, q_values

    g = golden("qnet")
    x = torch.from_numpy(g["obs"]).cuda()
    for who in ("modelB", "modelA"):
        blk = pack_state_dict(_sd(g, who))
        for mode, key in ((_lib.PM_FOLD_EVAL, "q_eval"), (_lib.PM_FOLD_TRAIN, "q_train")):
            q = q_values(fold(blk, mode)[0], x).cpu().numpy()
            np.testing.assert_allclose(q, g[f"{who}.{key}"], rtol=0, atol=2e-5)


def test_qnet_q_matches_oracle_at_scale(orc, golden):
    """65 536 rows: the device's Q equals the float32 restatement of its evaluation order bit for bit
    (oracle.qnet_forward_f32), the folded weights equal torch's mu + sigma*eps float32 fold bit for
    bit, and the float64 forward of the reference's formula stays within 3e-5."""
    from pongmi import _lib
    from pongmi.qnet import fold, pack_state_dict, q_values

    g = golden("qnet")
    sd = _sd(g, "modelB")
    x = _obs(np.random.RandomState(3), 65536)
    sdn = {k: v.numpy() for k, v in sd.items()}
    for mode, name in ((_lib.PM_FOLD_TRAIN, "train"), (_lib.PM_FOLD_EVAL, "eval")):
        w = fold(pack_state_dict(sd), mode)[0]
        assert np.array_equal(w[:4932].cpu().numpy(), orc.fold_heads_f32(sdn, name)), name
        q = q_values(w, torch.from_numpy(x).cuda()).cpu().numpy()
        q32 = orc.qnet_forward_f32(w.cpu().numpy(), x)
        assert np.array_equal(q.view(np.int32), q32.view(np.int32)), f"{name}: {(q != q32).sum()} Q values differ"
        ref = orc.qnet_forward(orc.qnet_effective(sdn, noisy=name == "train"), x)
        np.testing.assert_allclose(q, ref, rtol=0, atol=3e-5)


def test_fold_fresh_noise_matches_restatement(orc, golden):
    """reset_noise on the device: eps_w = f(out) (x) f(in), eps_b = f(out) with f = sign*sqrt|.|,
    values equal to the Philox restatement; written back into the block's epsilon slots."""
    from pongmi import _lib
    from pongmi.qnet import fold, pack_state_dict, unpack_state_dict

    g = golden("qnet")
    blk = pack_state_dict(_sd(g, "modelB"))
    out = blk.clone()
    seed, ctr = 77, 5
    w = fold(blk, _lib.PM_FOLD_TRAIN_FRESH, seed=seed, counter=ctr, params_out=out)
    sd = unpack_state_dict(out)
    fVi, fVo, fAi, fAo = orc.philox_noise(seed, orc.TAG_NOISE_ACT, ctr)
    assert np.array_equal(sd["fc_V.weight_epsilon"].numpy(), np.outer(fVo, fVi))  # the draws bit for bit
    assert np.array_equal(sd["fc_A.weight_epsilon"].numpy(), np.outer(fAo, fAi))
    assert np.array_equal(sd["fc_A.bias_epsilon"].numpy(), fAo)
    # effective heads = mu + sigma*eps from the written-back eps
    sd0 = unpack_state_dict(blk)
    wh = w[0, 4672:4672 + 256].cpu().numpy().reshape(4, 64)
    expA = sd0["fc_A.weight_mu"].numpy() + sd0["fc_A.weight_sigma"].numpy() * sd["fc_A.weight_epsilon"].numpy()
    assert np.array_equal(wh[1:], expA.astype(np.float32))
    # the raw draws are N(0,1): recover them over many counters
    raws = []
    for c in range(40):
        fold(blk, _lib.PM_FOLD_TRAIN_FRESH, seed=seed, counter=1000 + c, params_out=out)
        e = unpack_state_dict(out)["fc_V.weight_epsilon"].numpy()[0] / unpack_state_dict(out)["fc_V.bias_epsilon"].numpy()[0]
        raws.append(np.sign(e) * e ** 2)
    r = np.concatenate(raws)
    assert abs(r.mean()) < 0.1 and abs(r.var() - 1) < 0.15


def test_act_both_players(orc, golden):
    """A greedy on its per-arena opponent, B eps-greedy; the eps draws and random actions are
    the Philox restatement's, the greedy ones argmax of the oracle Q (first index on ties)."""
    from pongmi import _lib
    from pongmi.qnet import act, fold, pack_state_dict

    g = golden("qnet")
    sdB, sdA = _sd(g, "modelB"), _sd(g, "modelA")
    n = 50000
    rng = np.random.RandomState(9)
    oA, oB = _obs(rng, n), _obs(rng, n)
    opp = rng.randint(0, 3, n).astype(np.int32)
    w_opp = torch.cat([fold(pack_state_dict(sdA), _lib.PM_FOLD_TRAIN), fold(pack_state_dict(sdB), _lib.PM_FOLD_EVAL),
                       fold(pack_state_dict(sdA), _lib.PM_FOLD_EVAL)])
    w_B = fold(pack_state_dict(sdB), _lib.PM_FOLD_TRAIN)[0]
    effs = [orc.qnet_effective({k: v.numpy() for k, v in s.items()}, noisy=m)
            for s, m in ((sdA, True), (sdB, False), (sdA, False))]
    # the float32 restatement of the device's order: every Q bitwise, so every action exactly
    qa32 = np.zeros((n, 3), np.float32)
    for k in range(3):
        sel = opp == k
        qa32[sel] = orc.qnet_forward_f32(w_opp[k].cpu().numpy(), oA[sel])
    qb32 = orc.qnet_forward_f32(w_B.cpu().numpy(), oB)
    qa_ref = np.zeros((n, 3))
    for k in range(3):
        sel = opp == k
        qa_ref[sel] = orc.qnet_forward(effs[k], oA[sel])
    for eps in (0.0, 0.3, 1.0):
        seed, ctr = 11, 3
        aA, aB, qA, qB = act(w_opp, torch.from_numpy(opp), w_B, torch.from_numpy(oA).cuda(), torch.from_numpy(oB).cuda(),
                             epsilon=eps, seed=seed, counter=ctr, want_q=True)
        aA, aB = aA.cpu().numpy(), aB.cpu().numpy()
        assert np.array_equal(qA.cpu().numpy(), qa32) and np.array_equal(qB.cpu().numpy(), qb32)
        np.testing.assert_allclose(qA.cpu().numpy(), qa_ref, atol=3e-5)  # the reference's formula, float64
        assert np.array_equal(aA, np.argmax(qa32, 1))  # first max on ties, every arena
        r = orc.philox64(np.arange(n), orc.TAG_ACT, np.full(n, ctr, np.uint64), seed)
        explore = orc.u53(r[0], r[1]) < eps
        rnd = orc.below(r[2], 3)
        assert np.array_equal(aB, np.where(explore, rnd, np.argmax(qb32, 1)))
        assert abs(explore.mean() - eps) < 0.01
        if eps == 1.0:
            counts = np.bincount(aB, minlength=3)
            assert np.all(np.abs(counts / n - 1 / 3) < 0.01)


def test_per_matches_reference_golden(golden):
    from pongmi.replay import per_sample, per_update

    g = golden("per")
    for ph in range(int(g["n_phases"])):
        u = 0
        while f"p{ph}.u{u}.idxs" in g:
            k = f"p{ph}.u{u}."
            prios = torch.from_numpy(g[k + "prios_before"].copy()).cuda()
            idx, w = per_sample(prios, int(g[k + "size"]), 64, float(g[k + "beta"]), uniforms=g[k + "uniforms"])
            assert np.array_equal(idx.cpu().numpy(), g[k + "idxs"])
            np.testing.assert_allclose(w.cpu().numpy(), g[k + "weights"], rtol=2e-5)
            per_update(prios, torch.from_numpy(g[k + "upd_idx"]), torch.from_numpy(g[k + "upd_err"]))
            assert np.array_equal(prios.cpu().numpy(), g[k + "prios_after"])
            u += 1


@pytest.mark.parametrize("size", [1, 1023, 1025, 700_000, 1_000_000])
def test_per_sample_matches_oracle_at_scale(orc, size):
    from pongmi.replay import per_sample

    cap = 1_000_000
    rng = np.random.RandomState(size)
    pr = rng.uniform(0, 3, cap).astype(np.float32)
    pr[rng.rand(cap) < 0.1] = 0.0  # unfilled / zero-priority entries are never drawn
    if size == 1:
        pr[0] = 0.5
    u = rng.random_sample(256)
    idx, w = per_sample(torch.from_numpy(pr).cuda(), size, 256, 0.55, uniforms=u)
    idx, w = idx.cpu().numpy(), w.cpu().numpy()
    # the device's descent restated in its own summation order: every index and weight exactly
    tidx, tw = orc.per_sample_tree(pr, size, size, 0.55, u)
    assert np.array_equal(idx, tidx)
    np.testing.assert_allclose(w, tw / tw.max(), rtol=5e-7)  # the device normalises by its own float32 max
    # np.random.choice's own algorithm (float32-normalised CDF): identical on every draw outside the
    # rounding band of a CDF boundary (oracle.per_boundary_band); the band's size is reported
    ref_idx, ref_w = orc.per_sample(pr, size, 256, 0.55, u)
    band = orc.per_boundary_band(pr, size, u)
    assert np.array_equal(idx[~band], ref_idx[~band])
    print(f"size {size}: {band.sum()} of 256 draws in the boundary band, {(idx != ref_idx).sum()} differ there")
    assert np.all(pr[idx] > 0) and np.all(idx < size)
    np.testing.assert_allclose(w, ref_w, rtol=2e-5)


def test_per_philox_sampling_distribution():
    """Production uniforms: sampled frequencies follow p_i^alpha (chi-square)."""
    from pongmi.replay import per_sample

    pr = torch.tensor([0.0, 1.0, 2.0, 0.5, 4.0, 0.0, 1e-6, 3.0], device="cuda")
    counts = np.zeros(8)
    for c in range(400):
        idx, _ = per_sample(pr, 8, 256, 0.4, counter=c, seed=99)
        counts += np.bincount(idx.cpu().numpy(), minlength=8)
    p = pr.cpu().numpy().astype(np.float64) ** 0.6
    p /= p.sum()
    exp = p * counts.sum()
    assert counts[0] == 0 and counts[5] == 0
    m = exp > 5
    chi2 = ((counts[m] - exp[m]) ** 2 / exp[m]).sum()
    assert chi2 < 30, (counts, exp)
