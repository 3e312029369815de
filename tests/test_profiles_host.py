"""Host-only checks that bench.py's `roofline.traffic` fields resolve against the committed counter
profiles (profiles/r2_pmc.json, profiles/r2_rnn_pmc.json), and that tools/pmc_summary.py keys
namespaced kernel names by their bare name. No GPU."""
import csv
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_traffic_keys_resolve():
    b = _bench()
    # the default workload's launches (bench.py quotes these keys)
    for k in ("k_learn", "k_env_step", "k_act_sp"):
        v = b.pmc_traffic(k)
        assert v is not None and v > 0, k
    # --workload rnn: modelB's side of the overlapped step, 256 blocks x 256 lanes
    v = b.pmc_traffic("k_rnn_act@65536", "r2_rnn_pmc.json")
    assert v is not None and 32768 * 2048 * 0.9 < v < 32768 * 2048 * 1.5
    assert b.pmc_traffic("no_such_kernel") is None
    assert b.pmc_traffic("k_learn", "no_such_profile.json") is None


def test_pmc_summary_bare_names(tmp_path):
    d = tmp_path / "pmc_t_fetch"
    d.mkdir()
    rows = [
        ("(anonymous namespace)::k_rnn_act(pm::ActGrid, (anonymous namespace)::X)", "65536", "FETCH_SIZE", "10"),
        ("void (anonymous namespace)::k_env_step<2, false, true>(pm_env_params, float*)", "65536", "FETCH_SIZE", "4"),
        ("k_learn(pm_selfplay, int, int, int)", "82432", "FETCH_SIZE", "2"),
        ("(anonymous namespace)::k_rnn_act(pm::ActGrid, (anonymous namespace)::X)", "65536", "WRITE_SIZE", "5"),
        ("pm::k_gemm(pm::GemmBatch)", "1024", "WRITE_SIZE", "3"),
    ]
    with open(d / "p_counter_collection.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
        w.writerows(rows)
    out = tmp_path / "s.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), "t", str(tmp_path),
                    "--json", str(out)], check=True, capture_output=True)
    ks = json.load(open(out))["kernels"]
    for k in ("k_rnn_act", "k_rnn_act@65536", "k_env_step", "k_learn@82432", "k_gemm"):
        assert k in ks, (k, sorted(ks))
    # FETCH_SIZE doubled (gfx950 wide reads, MI355X_MICROARCH.md) + WRITE_SIZE, both in KB
    assert ks["k_rnn_act"]["hbm_bytes"] == 10 * 1024 * 2 + 5 * 1024
