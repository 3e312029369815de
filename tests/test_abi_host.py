"""CPU-only checks of the drop-in boundary: libpongmi.so loads without a GPU, exports exactly the
entry points include/pongmi.h declares, its struct layouts match the ctypes mirror, and the host
logic (derived env constants, parity-mode serves, parameter packing, chunk sizing) is right."""
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "pongmi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from pongmi import _lib
    L = _lib.load()
    decl = _declared()
    assert len(decl) >= 18
    for name in decl:
        assert hasattr(L, name), name
    assert set(decl) == set(_lib.EXPORTED), set(decl) ^ set(_lib.EXPORTED)
    nm = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    exported = set(re.findall(r" T (pm_[a-z0-9_]+)", nm))
    assert exported == set(decl), exported ^ set(decl)


def test_struct_layouts_and_constants_match_header():
    from pongmi import _lib
    L = _lib.load()
    assert L.pm_abi_version() == _lib.ABI_VERSION
    for which, cls in ((0, _lib.EnvParams), (1, _lib.EnvState), (2, _lib.Ctrl), (3, _lib.SelfPlay),
                       (8, _lib.RollReplay)):
        assert L.pm_sizeof(which) == __import__("ctypes").sizeof(cls)
    hdr = open(os.path.join(ROOT, "include", "pongmi.h")).read()
    for k in ("PM_QNET_NP", "PM_QNET_NHEAD", "PM_QNET_HEAD_OFF", "PM_QNET_EPS_OFF", "PM_QNET_NW", "PM_TRANS_F",
              "PM_MAX_BATCH", "PM_GRAD_EPISODES", "PM_GRAD_UPDATED", "PM_GRAD_LEN"):
        v = int(re.search(rf"#define {k} (\d+)", hdr).group(1))
        assert getattr(_lib, k) == v, k


def test_entry_points_reject_bad_arguments_without_a_gpu():
    from pongmi import _lib
    L = _lib.load()
    assert L.pm_env_step(None, None, None, None, None, None, None, None, None, None, None, 0, None, 0, 0, 0, None, 4,
                         None) == -1
    assert L.pm_qnet_fold(None, None, 7, 0, 0, None, None, 1, None) == -1
    assert b"mode" in L.pm_last_error()
    assert L.pm_selfplay_step(None, None) == -1
    # 977 fp64 chunk sums (1024 leaves) + 15625 fp64 sub-block sums (64 leaves) + 1e6 fp32 leaves,
    # each 256-byte rounded
    assert L.pm_per_work_bytes(1_000_000) == 7936 + 125184 + 4_000_000
    assert L.pm_env_reset(None, None, None, None, 0, 0, None, None, None, 0, None) == 0  # n = 0 is a no-op


def test_env_params_derived_constants_use_python_expressions():
    from pongmi.env import env_params
    p = env_params(ball_mass=1.3, world_ball_radius=0.031, paddle_width=0.21, speed_increment=0.1)
    assert p.inertia == (2 / 5) * 1.3 * 0.031 ** 2
    assert p.jt_coef == 2 * 1.3 / 7.0
    assert p.half_width == 0.21 / 2 and p.speed_scale == 1.0 + 0.1
    d = env_params()  # constructor defaults (envs/my_pong_env_2p.py:19-37)
    assert (d.paddle_speed, d.magnus_factor, d.restitution, d.friction, d.speed_scale_every) == (0.02, 0.01, 0.9, 0.2, 3)
    assert (d.ang0_lo, d.ang0_hi, d.ang1_lo, d.ang1_hi) == (-60, -30, 30, 60)
    with pytest.raises(ZeroDivisionError):
        env_params(speed_scale_every=0)


def test_parity_serves_equal_reference_resets(golden):
    """serve_table_from_random reproduces the reference's reset() draws (global random stream)."""
    from pongmi.env import serve_table_from_random
    g = golden("env_cfg")
    names = [str(n) for n in g["param_names"]]
    pv = dict(zip(names, g["param_values"].tolist()))
    kw = dict(ball_speed_range=(pv["speed_lo"], pv["speed_hi"]), spin_range=(pv["spin_lo"], pv["spin_hi"]))
    tab = serve_table_from_random(g["seeds"], int(g["done"].sum(1).max()) + 1, **kw)
    assert np.array_equal(tab[:, 0, 0], g["init"][:, 2]) and np.array_equal(tab[:, 0, 2], g["init"][:, 4])
    for i in range(tab.shape[0]):
        k = 1
        for t in np.nonzero(g["done"][i])[0]:
            assert np.array_equal(tab[i, k], g["reset_state"][i, t, [2, 3, 4]])
            k += 1


def test_qnet_pack_roundtrip_and_layout(golden):
    from pongmi.qnet import PARAM_LAYOUT, pack_state_dict, unpack_state_dict
    from models.qnet import QNet
    g = golden("qnet")
    sd = {k[7:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("modelB.") and "q_" not in k}
    blk = pack_state_dict(sd, "cpu")
    assert blk.numel() == 5452
    back = unpack_state_dict(blk)
    assert list(back.keys()) == list(QNet(7, 3).state_dict().keys())
    for k in sd:
        assert torch.equal(back[k], sd[k].float()), k
    # head block order is the order train_iterative.py hands the params to Adam (:101-104)
    net = QNet(7, 3)
    adam_order = [n for n, _ in list(net.fc_V.named_parameters(prefix="fc_V")) +
                  list(net.fc_A.named_parameters(prefix="fc_A"))]
    assert [k for k, _ in PARAM_LAYOUT[4:12]] == adam_order
    with pytest.raises(KeyError):
        pack_state_dict({k: v for k, v in sd.items() if "features.0" not in k}, "cpu")


def test_act_chunk_sizing():
    from pongmi.selfplay import act_chunk
    assert act_chunk(1.0) == 256 and act_chunk(0.67) == 256  # >= 256: the env kernel's per-block lists
    assert act_chunk(0.33 / 8) == 4096 and act_chunk(0.0) == 4096
    assert act_chunk(1.0, lo=64) == 128
    for p in (0.5, 0.1, 0.01):
        c = act_chunk(p)
        assert c <= 4096 and c % 256 == 0 and (c * p >= 96 or c == 4096)


def test_drop_in_modules_import_with_reference_names():
    import envs.my_pong_env_2p as e
    import envs.physics as ph
    import models.qnet as q
    assert hasattr(e, "PongEnv2P") and hasattr(ph, "collide_sphere_with_moving_plane")
    net = q.QNet(7, 3)
    x = torch.rand(5, 7)
    y = net(x)  # CPU tensors: the module keeps the reference's tensor semantics
    assert y.shape == (5, 3)


def test_integration_stub_runs(monkeypatch):
    """INTEGRATION.md section 1's ctypes stub (the binding a reference maintainer would add) runs
    as written against the built library: its ABI assertion holds, its pm_env_step argtypes have as
    many entries as the header's prototype, and a bad call surfaces pm_last_error as RuntimeError."""
    from pongmi import _lib
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 1."):text.index("## 2.")]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    hdr = open(os.path.join(ROOT, "include", "pongmi.h")).read()
    abi = re.search(r"#define PM_ABI_VERSION (\d+)", hdr).group(1)
    assert f"== {abi}" in code
    os.environ["PONGMI_LIB"] = _lib.LIB_PATH
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    proto = re.search(r"int pm_env_step\((.*?)\);", hdr, re.S).group(1)
    assert len(ns["_lib"].pm_env_step.argtypes) == len(proto.split(","))
    # n = 4 with a state of null device pointers: the library rejects the call before any HIP work
    # and the stub raises its message
    from pongmi.env import env_params
    T = torch.zeros(4, dtype=torch.int8)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda: type("S", (), {"cuda_stream": 0})())  # no GPU here
    with pytest.raises(RuntimeError, match="pm_env_step"):
        ns["env_step"](env_params(), _lib.EnvState(), T, T, T, T, T, T, T)
