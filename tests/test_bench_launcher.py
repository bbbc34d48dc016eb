"""bench.py's own rank launcher (``bench.py --gpus N`` with no torch.distributed.run) and the
TcpHub harness, on the CPU: ``--harness-only`` never opens a device."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "RSAMD_BENCH_FAIL_RANK", "RSAMD_BENCH_FAKE_RCCL", "RSAMD_BENCH_DEVICE")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks_and_prints_one_line(n):
    p = _run(["--gpus", str(n), "--harness-only", "--no-cpu-baseline"])
    assert p.returncode == 0, p.stderr
    lines = [s for s in p.stdout.splitlines() if s.strip()]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["harness_only"]
    assert [r["rank"] for r in rec["ranks"]] == list(range(n))
    assert [r["local_rank"] for r in rec["ranks"]] == list(range(n))
    assert all(r["launched"] for r in rec["ranks"])
    assert len({r["pid"] for r in rec["ranks"]}) == n       # n distinct processes
    assert rec["max_rank"] == n - 1                          # the hub's max-reduce
    assert rec["harness"].startswith("tcp hub")


def test_single_rank_runs_in_process():
    p = _run(["--gpus", "1", "--harness-only", "--no-cpu-baseline"])
    assert p.returncode == 0, p.stderr
    rec = json.loads(p.stdout.strip())
    assert rec["n_gpus"] == 1 and not rec["ranks"][0]["launched"]


def test_failing_rank_fails_the_launcher():
    p = _run(["--gpus", "3", "--harness-only", "--no-cpu-baseline"], {"RSAMD_BENCH_FAIL_RANK": "1"})
    assert p.returncode != 0
    assert "rank 1 of 3 exited with status 3" in p.stderr
    assert not p.stdout.strip()


def test_world_mismatch_is_an_error():
    # an external launcher that formed a different world than --gpus asks for
    p = _run(["--gpus", "4", "--harness-only", "--no-cpu-baseline"],
             {"WORLD_SIZE": "2", "RANK": "0", "MASTER_ADDR": "127.0.0.1",
              "MASTER_PORT": "29777"})
    assert p.returncode != 0
    assert "WORLD_SIZE=2 but --gpus=4" in p.stderr


def test_rccl_failure_on_distinct_devices_exits_nonzero():
    # ranks on distinct GPUs (RSAMD_BENCH_DEVICE unset) whose RCCL init failed: no line at all,
    # a non-zero exit (the launcher reports the first failing rank)
    p = _run(["--gpus", "2", "--harness-only", "--no-cpu-baseline"],
             {"RSAMD_BENCH_FAKE_RCCL": "fail"})
    assert p.returncode != 0
    assert "RCCL communicator init failed" in p.stderr
    assert not p.stdout.strip()


def test_rccl_failure_in_one_device_rehearsal_uses_the_hub():
    p = _run(["--gpus", "2", "--harness-only", "--no-cpu-baseline"],
             {"RSAMD_BENCH_FAKE_RCCL": "fail", "RSAMD_BENCH_DEVICE": "0"})
    assert p.returncode == 0, p.stderr
    rec = json.loads(p.stdout.strip())
    assert rec["exchange"].startswith("tcp-hub all-gather")
    p = _run(["--gpus", "2", "--harness-only", "--no-cpu-baseline"],
             {"RSAMD_BENCH_FAKE_RCCL": "ok"})
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout.strip())["exchange"] == "rccl all-gather"


def test_cpu_baseline_is_reported_at_world_two():
    # rank 0 times the oracle before any HIP call also when the world has several ranks
    p = _run(["--gpus", "2", "--harness-only", "--cpu-seconds", "0.6", "--cpu-procs", "2"])
    assert p.returncode == 0, p.stderr
    cb = json.loads(p.stdout.strip())["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 2 and cb["value"] > 0


def test_under_torch_distributed_run_as_the_driver_launches_it():
    """The driver's multi-GPU invocation: python -m torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N; every rank
    prints nothing but rank 0's single line, and the world is the launcher's."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), BENCH, "--gpus", "2", "--harness-only", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [x for x in p.stdout.splitlines() if x.strip().startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and [r["rank"] for r in rec["ranks"]] == [0, 1]
    assert not any(r["launched"] for r in rec["ranks"])   # the external launcher's processes
