"""C4 over the shared-memory step ring (``csrc/runtime/step_ring.h``, ``parallel/step_ring.py``).

* the native ring: every reader gets every message byte-identical and in order, a full ring
  back-pressures the writer, an oversize message is refused (the channel then goes over gloo),
  a reader's timeout returns None and a closed ring wakes blocked callers;
* a world-4 gloo group: followers replay the leader's packed ``StepInputs`` bit-identically
  through ``comm.broadcast_step`` -- ring messages, an oversize message through the gloo fallback,
  then stop -- and a follower with no leader times out instead of hanging.
"""
import os
import socket
import threading
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

rt = pytest.importorskip("financial_chatbot_llm_amd._penny_runtime")


def _name(tag):
    return f"/penny_test_{tag}_{os.getpid()}_{time.monotonic_ns() % 10**9}"


def test_ring_order_backpressure_oversize_timeout():
    w = rt.StepRing(_name("a"), True, 4, 4096, 3)
    r_ring = [rt.StepRing(w.name, False, 0, 0, 0) for _ in range(3)]
    rng = np.random.default_rng(0)
    msgs = [rng.integers(0, 256, size=int(rng.integers(0, 4096)), dtype=np.uint8) for _ in range(40)]
    got = {r: [] for r in range(3)}

    def reader(r):
        for _ in msgs:
            got[r].append(r_ring[r].get(r, 10.0))
    ts = [threading.Thread(target=reader, args=(r,)) for r in range(3)]
    for t in ts:
        t.start()
    for m in msgs:                                  # 40 messages through 4 slots: back-pressure
        assert w.put(m, 10.0)
    for t in ts:
        t.join(20)
    for r in range(3):
        assert len(got[r]) == len(msgs) and all(np.array_equal(a, b) for a, b in zip(got[r], msgs))
    assert w.head == len(msgs)
    assert not w.put(np.zeros(4097, np.uint8), 1.0)           # oversize: refused, nothing published
    assert r_ring[0].get(0, 0.05) is None                      # nothing pending: timeout -> None
    with pytest.raises(RuntimeError):                          # reader 0 never reads: writer times out
        for _ in range(5):
            w.put(np.zeros(8, np.uint8), 0.2)
    # a blocked reader wakes when the ring is closed
    err = []

    def blocked():
        try:
            while True:
                r_ring[1].get(1, 30.0)
        except RuntimeError as e:
            err.append(str(e))
    t = threading.Thread(target=blocked)
    t.start()
    time.sleep(0.3)
    w.close()
    t.join(10)
    assert err and "closed" in err[0]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _steps():
    """Packed StepInputs of a decode step, a prefill step and one too big for a 64 KiB slot."""
    from financial_chatbot_llm_amd.engine.model_runner import StepInputs
    rng = np.random.default_rng(1)

    def mk(T, S, W):
        i32 = lambda *s: rng.integers(0, 1000, size=s, dtype=np.int32)   # noqa: E731
        return StepInputs(i32(T), i32(T), i32(T), np.arange(S + 1, dtype=np.int32), i32(S), i32(S, W), 7, i32(3),
                          i32(3, W), i32(4), rng.random(4, dtype=np.float32), rng.integers(0, 2**40, 4),
                          i32(4), rng.random(4, dtype=np.float32), None)
    return [mk(4, 0, 5), mk(300, 3, 40), mk(20000, 2, 64)]


def _worker(rank, world, port, q, mode):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from financial_chatbot_llm_amd.parallel import comm
        from financial_chatbot_llm_amd.parallel import step_ring
        from financial_chatbot_llm_amd.parallel.dist import init_distributed, shutdown, state
        init_distributed(tp_size=world, backend="gloo", device_type="cpu")
        s = state()
        group = s.tp_cpu_group if s.tp_cpu_group is not None else s.tp_group
        leader = s.tp_leader_rank
        followers = [r for r in range(world) if r != leader]
        timeout = 2.0 if mode == "timeout" else 60.0
        ch = step_ring.StepChannel(group, leader, rank == leader, followers.index(rank) if rank != leader else 0,
                                   len(followers), nslots=4, slot_bytes=64 << 10, timeout_s=timeout)
        comm._STEP_CHANNEL = ch
        out = None
        if mode == "replay":
            steps = _steps()
            if rank == leader:
                for si in steps * 3:
                    comm.broadcast_step(si)
                comm.broadcast_step(None)
                out = ch.fallbacks
            else:
                got = []
                while True:
                    si = comm.broadcast_step(None)
                    if si is None:
                        break
                    got.append(si.pack())
                want = [si.pack() for si in steps * 3]
                out = len(got) == len(want) and all(np.array_equal(a, b) for a, b in zip(got, want))
        else:                                        # the leader never sends: followers time out
            if rank != leader:
                try:
                    comm.broadcast_step(None)
                    out = "no timeout"
                except TimeoutError:
                    out = "timeout"
            else:
                time.sleep(4.0)
                out = "leader"
        comm._STEP_CHANNEL = None
        q.put((rank, out))
        shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("mode", ["replay", "timeout"])
def test_followers_replay_bit_identical_steps_through_the_ring(mode):
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=200) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not (isinstance(v, str) and v.startswith("ERR")), v
    if mode == "replay":
        assert res[0] == 3                           # the 20k-token step went over gloo, 3 times
        assert all(res[r] is True for r in range(1, world))
    else:
        assert all(res[r] == "timeout" for r in range(1, world))


def test_ring_slot_size_rounded_to_whole_lines():
    """a slot size that is not a multiple of 64 would misalign every SlotHeader after
    slot 0 (its atomic seq loses single-copy atomicity); the ring rounds it up to whole 64-B lines
    and records the rounded size, so writer and readers agree on the geometry."""
    w = rt.StepRing(_name("odd"), True, 3, 100, 1)
    assert w.slot_bytes == 128
    r = rt.StepRing(w.name, False, 0, 0, 0)
    assert r.slot_bytes == 128 and r.nslots == 3
    msgs = [np.arange(n, dtype=np.uint8) for n in (0, 1, 100, 127, 128, 64)]
    for m in msgs:
        assert w.put(m, 5.0)
        got = r.get(0, 5.0)
        assert bytes(got) == m.tobytes()
    assert not w.put(np.zeros(129, dtype=np.uint8), 5.0)   # larger than the rounded slot: refused
