"""First-contact safety of the custom TP collectives (parallel/custom_ar.py ``self_test``,
``comm.verify_custom_all_reduce``), CPU + gloo, world 4.

Each rank checks the collective against the exact fp32 sum of every rank's seeded input and the
ranks agree by a MIN all-reduce: a corrupt peer (wrong sum on ONE rank), an expired bounded wait or
an exception on one rank sends EVERY rank to the RCCL path; a healthy collective keeps it.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 4


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_sum(x):
    xf = x.float()
    dist.all_reduce(xf)
    return xf.to(torch.bfloat16)


def _gloo_gather(x):
    parts = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, x)
    return torch.stack(parts)


class _FakeAR:
    """Stands in for CustomAllReduce: its collective is gloo, optionally broken on one rank."""

    def __init__(self, mode):
        self.mode, self.closed = mode, False

    def self_test(self):
        from financial_chatbot_llm_amd.parallel.custom_ar import self_test
        rank = dist.get_rank()

        def reduce_fn(x):
            y = _gloo_sum(x)
            if self.mode == "corrupt" and rank == 2:
                y[::97] += 1.0                       # a peer whose sum is silently wrong
            return y

        def check_fn():
            if self.mode == "timeout" and rank == 3:
                raise RuntimeError("custom all-reduce: a peer never arrived (bounded wait expired)")

        def gather_fn(x):
            g = _gloo_gather(x)
            if self.mode == "stale_gather" and rank == 1:
                g[0] = 0                              # stale peer buffer
            return g
        return self_test(reduce_fn, None, torch.device("cpu"), sizes=(512, 4096), gather_fn=gather_fn,
                         check_fn=check_fn)

    def close(self):
        self.closed = True


def _worker(rank, port, mode, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from financial_chatbot_llm_amd.parallel import comm
        fake = _FakeAR(mode)
        comm._CUSTOM_AR = fake
        kept = comm.verify_custom_all_reduce()
        q.put((rank, kept, comm._CUSTOM_AR is None, fake.closed, dict(comm.AR_STATUS)))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), None, None))


@pytest.mark.timeout(180)
@pytest.mark.parametrize("mode", ["ok", "corrupt", "timeout", "stale_gather"])
def test_custom_ar_self_test_consensus_fallback(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, mode, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        item = q.get(timeout=170)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=30)
    for r, v in res.items():
        assert v[0] != "ERR", v[1]
    if mode == "ok":
        assert all(v[0] and not v[1] and not v[2] and v[3]["self_test"] == "ok" for v in res.values())
    else:
        # every rank falls back together (a split decision would deadlock the next collective)
        assert all((not v[0]) and v[1] and v[2] and v[3]["self_test"].startswith("failed") for v in res.values())
        bad = {"corrupt": 2, "timeout": 3, "stale_gather": 1}[mode]
        assert "peer rank" not in res[bad][3]["self_test"]
        assert all("peer rank" in v[3]["self_test"] for r, v in res.items() if r != bad)
