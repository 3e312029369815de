"""QNetRNN host side (no GPU): the packed parameter layout and the drop-in module's torch path."""
import numpy as np
import torch


def _sd(g):
    return {k[7:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("params.")}


def test_packed_layout_matches_header_offsets(golden):
    """pongmi.rnn.PARAM_LAYOUT against the R_P_* offsets of pm_rnn.h and modelB.parameters() order."""
    from models.qnet_rnn import QNetRNN
    from pongmi import rnn
    from pongmi._lib import PM_RNN_NP, PM_RNN_NPARAM
    offs, o = {}, 0
    for k, s in rnn.PARAM_LAYOUT:
        offs[k] = o
        o += int(np.prod(s))
    assert o == PM_RNN_NP
    assert offs["lstm.weight_ih_l0"] == 8832 and offs["fc_shared_head.0.weight_mu"] == 140928
    assert offs["fc_A.bias_sigma"] == 174981 and offs["fc_shared_head.0.weight_epsilon"] == PM_RNN_NPARAM
    assert offs["fc_A.bias_epsilon"] == 192009
    net = QNetRNN(7, 3)
    assert [n for n, _ in net.named_parameters()] == list(rnn.PARAM_KEYS)
    assert list(net.state_dict()) == list(rnn.STATE_KEYS)
    g = golden("rnn")
    block = rnn.pack_state_dict(_sd(g), "cpu")
    back = rnn.unpack_state_dict(block)
    assert list(back) == list(rnn.STATE_KEYS)
    for k, v in back.items():
        assert torch.equal(v, torch.from_numpy(g["params." + k])), k


def test_dropin_torch_path_matches_reference(golden):
    """models.qnet_rnn.QNetRNN loads the reference checkpoint's state_dict and, on CPU, reproduces
    the reference module's outputs (tests/golden/rnn.npz)."""
    from models.qnet_rnn import QNetRNN
    g = golden("rnn")
    net = QNetRNN(7, 3)
    net.load_state_dict(_sd(g))
    with torch.no_grad():
        for mode in ("train", "eval"):
            net.train(mode == "train")
            q, (h, c) = net(torch.from_numpy(g["act_x"]), (torch.from_numpy(g["act_h0"]), torch.from_numpy(g["act_c0"])))
            np.testing.assert_allclose(q.numpy(), g[f"act_q_{mode}"], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(c.numpy(), g[f"act_c1_{mode}"], rtol=1e-5, atol=1e-6)
            q, (h, c) = net(torch.from_numpy(g["seq_x"]), net.init_hidden(16, "cpu"))
            np.testing.assert_allclose(q.numpy(), g[f"seq_q_{mode}"], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(h.numpy(), g[f"seq_h_{mode}"], rtol=1e-5, atol=1e-6)

