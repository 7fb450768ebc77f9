"""The driver contract of ``bench.py`` (task spec): ONE JSON line from rank 0 with the BASELINE.json
metric, the whole-job aggregate ``value`` (total turns / max-over-ranks time), ``n_gpus`` =
WORLD_SIZE, weak scaling and the dp parallelism label -- exercised on CPU with tiny models, single
process and 2 ranks over gloo (the 8-GPU scaling run uses the same code path with RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--device", "cpu", "--model", "llama-tiny", "--embed-model", "bert-tiny", "--corpus", "2000", "--users",
        "20", "--convs", "3", "--steps", "1", "--warmup", "1", "--respond-tokens", "4", "--max-model-len", "1024"]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out: str):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def _clean_env(**kw):
    """The environment of a plain shell: no launcher variables leaking in from the test runner."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _check(d, n):
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == n and d["steps"] == 1 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["unit"] == "turns/s"
    assert d["config"]["parallelism"] == f"dp{n}" and d["config"]["global_batch"] == 3 * n
    assert d["turn_errors"] == 0 and d["value"] > 0
    # value = whole-job turns / max-over-ranks wall time of the K timed steps
    assert abs(d["ms_per_step"] - 1e3 * (3 * n) / d["value"]) / d["ms_per_step"] < 0.02


@pytest.mark.timeout(300)
def test_bench_single_process_json_contract():
    r = subprocess.run([sys.executable, "bench.py", *ARGS], cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    _check(lines[0], 1)


@pytest.mark.timeout(400)
def test_bench_self_spawns_ranks_without_launcher():
    """a plain ``bench.py --gpus 2`` (no torchrun) starts its own 2 ranks and reports
    them -- the driver's 1->8 scaling run must never silently measure one GPU."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=ROOT, capture_output=True, text=True,
                       timeout=380, env=_clean_env(OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    _check(lines[0], 2)
    assert lines[0]["host"]["world_size"] == 2 and lines[0]["host"]["launcher"].startswith("bench.py self-spawn")


@pytest.mark.timeout(400)
def test_bench_self_spawns_tensor_parallel_without_launcher():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--tp", "2", *ARGS], cwd=ROOT, capture_output=True,
                       text=True, timeout=380, env=_clean_env(OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["host"]["world_size"] == 2 and d["config"]["parallelism"] == "dp1tp2"
    assert d["turn_errors"] == 0 and d["value"] > 0


def test_bench_world_mismatch_fails_loudly():
    """--gpus disagreeing with the launcher's WORLD_SIZE is an error, not a warning."""
    env = _clean_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=ROOT, capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE 1" in r.stderr
    assert _json_lines(r.stdout) == []


@pytest.mark.timeout(400)
def test_bench_two_ranks_gloo_json_contract():
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", *ARGS]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=380, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1          # rank 0 only
    _check(lines[0], 2)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_two_ranks_on_one_gpu_json_contract():
    """The dpN bench path on the device: two ranks share cuda:0 (gloo control plane, each engine takes
    a slice of HBM through PENNY_KV_FRACTION), tiny models through the HIP kernels."""
    env = dict(os.environ, OMP_NUM_THREADS="2", PENNY_DIST_BACKEND="gloo", PENNY_KV_FRACTION="0.05")
    gpu_args = ["--device" if a == "--device" else ("cuda" if a == "cpu" else a) for a in ARGS]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", *gpu_args]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    _check(lines[0], 2)


@pytest.mark.timeout(400)
def test_bench_tensor_parallel_replica_gloo_json_contract():
    """--tp 2 over 2 ranks (config 4's process model at small scale): one replica whose TP follower
    replays the leader's steps; the JSON counts both GPUs and the replica's conversations."""
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--tp", "2", *ARGS]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=380, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp1tp2" and d["config"]["global_batch"] == 3
    assert d["turn_errors"] == 0 and d["value"] > 0
    assert abs(d["ms_per_step"] - 1e3 * 3 / d["value"]) / d["ms_per_step"] < 0.02


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_self_spawn_on_one_gpu():
    """``bench.py --gpus 2`` with no launcher on the device (two ranks share cuda:0 over gloo)."""
    env = _clean_env(OMP_NUM_THREADS="2", PENNY_DIST_BACKEND="gloo", PENNY_KV_FRACTION="0.05")
    gpu_args = ["--device" if a == "--device" else ("cuda" if a == "cpu" else a) for a in ARGS]
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *gpu_args], cwd=ROOT, capture_output=True,
                       text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    _check(lines[0], 2)
    assert lines[0]["host"]["world_size"] == 2


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_tensor_parallel_replica_on_one_gpu_json_contract():
    """--tp 2 on the device: leader and follower share cuda:0 (gloo control plane, the TP all-reduces
    on the custom IPC kernels inside the captured decode graphs)."""
    env = dict(os.environ, OMP_NUM_THREADS="2", PENNY_DIST_BACKEND="gloo", PENNY_KV_FRACTION="0.05")
    gpu_args = ["--device" if a == "--device" else ("cuda" if a == "cpu" else a) for a in ARGS]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--tp", "2", *gpu_args]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert d["config"]["parallelism"] == "dp1tp2" and d["turn_errors"] == 0 and d["value"] > 0


@pytest.mark.timeout(300)
def test_bench_tp_shard_estimate_mode():
    """``--tp-shard-estimate N``: one process runs rank 0's TP=N shard with its
    collectives stubbed and projects the all-reduce time at stated xGMI rates."""
    r = subprocess.run([sys.executable, "bench.py", *ARGS, "--tp-shard-estimate", "2"], cwd=ROOT, capture_output=True,
                       text=True, timeout=280, env=_clean_env())
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_lines(r.stdout)[0]
    e = d["tp_shard_estimate"]
    assert e["tp"] == 2 and e["all_reduces_per_step"] == 1 + 2 * 2          # llama-tiny: 2 layers
    assert e["prefill_tokens"] > 0 and e["all_reduce_bytes"] > 0
    for k in ("optimistic", "pessimistic"):
        assert e[k]["projected_s"] >= e["compute_only_s"]
    assert "stubbed" in d["config"]["parallelism"]
