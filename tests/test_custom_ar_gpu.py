"""Custom one-shot / two-shot all-reduce (C1 custom path) on the GPU box.

Only one MI355X is available to the test runner, so 2, 4 or 8 processes share cuda:0: each
exports its IPC buffers, maps every peer's, and runs the real kernel protocol (flags,
double-buffered rounds, bounded waits, automatic one-shot / two-shot choice at > 2 ranks).
Cross-GPU xGMI transport is the same code with peers on other devices.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _timeout_worker(rank, world, port, q):
    """Rank 1 misses an all-reduce: rank 0's bounded wait expires and the kernel FAILS the
    collective -- NaN output (never a sum of stale peer buffers), the error flag set, its slots in
    the peer poisoned -- and the engine's per-step sync (PendingStep) raises CollectiveTimeout.
    Rank 0's next call fails at once (a dead rank never publishes again); the late rank 1 polls a
    poisoned slot and fails at once too (allreduce.hip)."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import time

        import torch.distributed as dist

        from financial_chatbot_llm_amd.engine.model_runner import CollectiveTimeout, PendingStep
        from financial_chatbot_llm_amd.parallel.custom_ar import CustomAllReduce
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        try:
            ar = CustomAllReduce(None, torch.device("cuda", 0), max_bytes=1 << 20, buffer_bytes=1 << 20)
        except RuntimeError as e:
            q.put((rank, "SKIP", str(e)))
            return
        x = torch.ones(4096, dtype=torch.bfloat16, device="cuda")
        ar.all_reduce(x)                        # a healthy round first
        torch.cuda.synchronize()
        ar.check()
        dist.barrier()
        out = {}
        if rank == 0:
            y = ar.all_reduce(x)                # the peer never arrives
            host = torch.zeros(3, dtype=torch.int32).pin_memory()
            host[2:3].copy_(ar.err, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            try:
                PendingStep(None, 2, host, ev, check_err=True).result()
            except CollectiveTimeout as e:
                out["raised"] = str(e)
            out["nan"] = bool(torch.isnan(y.float()).all())
            t0 = time.perf_counter()
            y2 = ar.all_reduce(x)               # dead rank: fails without waiting
            torch.cuda.synchronize()
            out["dead_s"] = time.perf_counter() - t0
            out["dead_nan"] = bool(torch.isnan(y2.float()).all())
        dist.barrier()
        if rank == 1:
            t0 = time.perf_counter()
            y = ar.all_reduce(x)                # the late peer: rank 0's slots are poisoned
            torch.cuda.synchronize()
            out["late_s"] = time.perf_counter() - t0
            out["late_nan"] = bool(torch.isnan(y.float()).all())
            out["late_err"] = int(ar.err.item())
        dist.barrier()
        ar.close()
        q.put((rank, "OK", out))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch.distributed as dist

        from financial_chatbot_llm_amd.parallel.custom_ar import CustomAllReduce
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        try:
            ar = CustomAllReduce(None, torch.device("cuda", 0), max_bytes=1 << 20, buffer_bytes=1 << 20)
        except RuntimeError as e:
            q.put((rank, "SKIP", str(e)))
            return
        results = []
        for i, n in enumerate([8, 4096, 4096 * 3 + 8, 262144, 524288]):
            g = torch.Generator().manual_seed(1000 * i + rank)
            x = torch.randn(n, generator=g).to(torch.bfloat16)
            xs = [torch.empty_like(x) for _ in range(world)]
            dist.all_gather(xs, x)
            ref = torch.stack([t.float() for t in xs]).sum(0)
            xd = x.cuda()
            out = ar.all_reduce(xd)
            ar.all_reduce(xd, out=xd)              # in-place form (what tp_all_reduce uses)
            torch.cuda.synchronize()
            results.append(((out.float().cpu() - ref).abs().max().item(),
                            (xd.float().cpu() - ref).abs().max().item(), ref.abs().max().item()))
        # two-shot form (reduce-scatter + all-gather): bit-identical to one-shot
        for i, n in enumerate([16 * world, 4096 * world + 8 * world, 65536 * world]):
            g = torch.Generator().manual_seed(7000 + 1000 * i + rank)
            xd = torch.randn(n, generator=g).to(torch.bfloat16).cuda()
            a = ar.all_reduce(xd, method="oneshot")
            b = ar.all_reduce(xd, method="twoshot")
            torch.cuda.synchronize()
            results.append((float((a.float() - b.float()).abs().max().item()), 0.0, 0.0))
        # all-gather (vocab-parallel logits): rank-major, exact
        for i, n in enumerate([8, 4096 + 8, 300000]):
            g = torch.Generator().manual_seed(9000 + 100 * i + rank)
            x = torch.randn(n, generator=g).to(torch.bfloat16)
            xs = [torch.empty_like(x) for _ in range(world)]
            dist.all_gather(xs, x)
            got = ar.all_gather(x.cuda()).cpu()
            results.append((float((got.float() - torch.stack(xs).float()).abs().max().item()), 0.0, 0.0))
        # hipGraph capture: the round counter advances on the device across replays
        x = torch.full((4096,), float(rank + 1), dtype=torch.bfloat16, device="cuda")
        ar.all_reduce(x)
        torch.cuda.synchronize()
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph):
            y = ar.all_reduce(x)
        for _ in range(5):
            gph.replay()
        torch.cuda.synchronize()
        results.append((float(y.float().mean().item()), float(world * (world + 1) / 2), 0.0))
        results.append((float(ar.counter.item()), 25.0, 0.0))   # 10 + 6 + 3 + 1 eager calls + 5 replays
        ar.check()
        # the engine's init-time first-contact check (one-shot, two-shot, all-gather vs the exact sum,
        # consensus over the group) passes on a healthy group.  Up to 4 ranks: with 8 processes
        # time-slicing ONE GPU the spinning peers can outlast the bounded wait (the engine would then
        # fall back to RCCL, which is the intended safe outcome, but not what this assertion checks)
        if world <= 4:
            ok, why = ar.self_test()
            assert ok, why
        results.append((1.0, 1.0, 0.0))
        dist.barrier()
        ar.close()
        q.put((rank, "OK", results))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


def _run(target, world):
    env_keep = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    assert env_keep in (None, "0")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, status, payload = q.get(timeout=200)
        res[r] = (status, payload)
    for p in procs:
        p.join(timeout=60)
    if any(s == "SKIP" for s, _ in res.values()):
        pytest.skip(f"IPC mapping unavailable on this box: {[p for s, p in res.values() if s == 'SKIP']}")
    for r, (status, payload) in res.items():
        assert status == "OK", payload
    return res


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_custom_all_reduce_processes(world):
    res = _run(_worker, world)
    for r, (status, payload) in res.items():
        *sizes, graph, rounds, selftest = payload
        for err, err_inplace, mag in sizes:
            assert err <= 0.02 * mag + 1e-2 and err_inplace <= 0.02 * mag + 1e-2, (err, err_inplace, mag)
        assert graph[0] == graph[1]
        assert rounds[0] == rounds[1]
        assert selftest[0] == 1.0


@pytest.mark.timeout(120)
def test_custom_all_reduce_missing_peer_fails_the_step():
    res = _run(_timeout_worker, 2)
    r0, r1 = res[0][1], res[1][1]
    assert "missed the bounded wait" in r0["raised"]
    assert r0["nan"] and r0["dead_nan"] and r0["dead_s"] < 1.0, r0
    assert r1["late_nan"] and r1["late_err"] == 1 and r1["late_s"] < 1.0, r1
