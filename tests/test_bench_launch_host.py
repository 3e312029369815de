"""bench.py --gpus N is authoritative: with WORLD_SIZE unset and N > 1 the bench
starts torch.distributed.run with N ranks as a child process (before any GPU call), a launcher that
started a different number of ranks than --gpus is refused, and so is a request for more ranks than
visible GPUs. Host only: launch_plan is pure, and the refusals are checked end to end on this
GPU-less container (torch.cuda.device_count() == 0)."""
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


def test_default_is_one_rank_in_process():
    b = _bench()
    assert b.launch_plan([], {}, 1) == ("run", None)
    assert b.launch_plan(["--gpus", "1", "--steps", "5"], {}, 8) == ("run", None)
    assert b.launch_plan(["--workload", "rnn"], {"WORLD_SIZE": "1", "LOCAL_RANK": "0"}, 1) == ("run", None)


def test_gpus_n_spawns_torchrun_child():
    b = _bench()
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5", "--workload", "rnn"]
    plan, cmd = b.launch_plan(argv, {}, 8)
    assert plan == "spawn"
    assert cmd[0] == sys.executable and cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv  # every flag passes through, --gpus included: each rank then sees WORLD_SIZE == N
    # the ranks torchrun starts are consistent with the request and run in-process
    assert b.launch_plan(argv, {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}, 8) == ("run", None)
    assert b.launch_plan(["--gpus=2"], {}, 2)[0] == "spawn"


def test_mismatches_are_refused():
    b = _bench()
    plan, msg = b.launch_plan(["--gpus", "2"], {"WORLD_SIZE": "4", "LOCAL_RANK": "0"}, 8)
    assert plan == "error" and "WORLD_SIZE=4" in msg
    plan, msg = b.launch_plan([], {"WORLD_SIZE": "2", "LOCAL_RANK": "0"}, 8)  # torchrun N=2 without --gpus 2
    assert plan == "error"
    plan, msg = b.launch_plan(["--gpus", "2"], {}, 1)  # a 1-GPU box: never a silent 1-rank line
    assert plan == "error" and "only 1 visible" in msg
    plan, msg = b.launch_plan(["--gpus", "2"], {"WORLD_SIZE": "2", "LOCAL_RANK": "1"}, 1)
    assert plan == "error" and "LOCAL_RANK" in msg
    assert b.launch_plan(["--gpus", "0"], {}, 8)[0] == "error"


def _run(args, extra_env):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


def test_bench_refuses_end_to_end():
    # this container has no GPU: --gpus 2 must fail loudly (non-zero, an error line), not print a
    # 1-rank measurement
    r = _run(["--gpus", "2", "--no-cpu-baseline"], {})
    assert r.returncode == 2, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert "visible GPU" in line["error"] and "value" not in line
    r = _run(["--gpus", "1", "--no-cpu-baseline"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in json.loads(r.stdout.strip().splitlines()[-1])["error"]


def test_rehearsal_lets_ranks_share_a_gpu():
    # PONGMI_BENCH_REHEARSE=1 (never set by the driver): the 1-GPU refusals are lifted so the N-rank
    # path can be exercised on one device; without it they stand (test_mismatches_are_refused)
    b = _bench()
    env = {"PONGMI_BENCH_REHEARSE": "1"}
    assert b.launch_plan(["--gpus", "2"], env, 1)[0] == "spawn"
    assert b.launch_plan(["--gpus", "2"], dict(env, WORLD_SIZE="2", LOCAL_RANK="1"), 1) == ("run", None)
    assert b.launch_plan(["--gpus", "2"], dict(env, WORLD_SIZE="4", LOCAL_RANK="1"), 1)[0] == "error"
    assert b.launch_plan(["--gpus", "2"], {"PONGMI_BENCH_REHEARSE": "0"}, 1)[0] == "error"
