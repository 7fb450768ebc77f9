"""Context parallelism (ring attention, SURVEY §2.D / §5.7 stretch) on CPU with gloo.

* zig-zag shard / unshard round-trips and balances causal work;
* the log-sum-exp block merge equals one softmax over the concatenated keys;
* ring attention over 2 and 3 gloo ranks (GQA, causal and bidirectional) equals single-process
  fp32 attention over the whole sequence.
"""
import os
import socket

import pytest
import torch
from mp_util import to_np, to_torch
import torch.multiprocessing as mp

from financial_chatbot_llm_amd.parallel import context as cpx


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _full(q, k, v, causal):
    pos = torch.arange(q.shape[0])
    o, _ = cpx.torch_block_attention(q, k, v, pos, pos, q.shape[-1] ** -0.5, causal)
    return o


def _inputs(T=48, Hq=4, Hkv=2, D=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(T, Hq, D, generator=g), torch.randn(T, Hkv, D, generator=g),
            torch.randn(T, Hkv, D, generator=g))


def test_zigzag_roundtrip_and_balance():
    x = torch.arange(24).float()[:, None]
    parts = [cpx.zigzag_shard(x, 3, r) for r in range(3)]
    assert torch.equal(cpx.zigzag_unshard(parts), x)
    # causal work (visible keys per rank) is identical across ranks
    work = [int((cpx.zigzag_positions(24, 3, r) + 1).sum()) for r in range(3)]
    assert len(set(work)) == 1
    with pytest.raises(ValueError):
        cpx.zigzag_positions(25, 3, 0)


def test_block_merge_equals_full_softmax():
    q, k, v = _inputs()
    pos = torch.arange(q.shape[0])
    ref, ref_lse = cpx.torch_block_attention(q, k, v, pos, pos, 0.25, True)
    h = q.shape[0] // 2
    oa, la = cpx.torch_block_attention(q, k[:h], v[:h], pos, pos[:h], 0.25, True)
    ob, lb = cpx.torch_block_attention(q, k[h:], v[h:], pos, pos[h:], 0.25, True)
    assert torch.isinf(lb[:, :h]).all()          # rows before the second half see none of it
    o, lse = cpx.merge_blocks(oa, la, ob, lb)
    assert torch.allclose(o, ref, atol=1e-5)
    assert torch.allclose(lse, ref_lse, atol=1e-5)


def _worker(rank, world, port, q_out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from financial_chatbot_llm_amd.parallel.dist import init_distributed, shutdown
        init_distributed(tp_size=1, backend="gloo", device_type="cpu")
        import torch.distributed as dist
        res = {}
        for causal in (True, False):
            q, k, v = _inputs(T=12 * world)
            shard = lambda t: cpx.zigzag_shard(t, world, rank)  # noqa: E731
            res[causal] = cpx.ring_attention(shard(q), shard(k), shard(v), q.shape[0], causal=causal)
        q_out.put((rank, to_np(res)))
        dist.barrier()
        shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q_out.put((rank, traceback.format_exc()))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 3])
def test_ring_attention_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q_out)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: to_torch(v) for r, v in (q_out.get(timeout=200) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    q, k, v = _inputs(T=12 * world)
    for causal in (True, False):
        got = cpx.zigzag_unshard([res[r][causal] for r in range(world)])
        assert torch.allclose(got, _full(q, k, v, causal), atol=1e-5), causal


def _cp_model_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch.distributed as dist

        from financial_chatbot_llm_amd.models.configs import get_model_config
        from financial_chatbot_llm_amd.models.llama import LlamaModel
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cfg = get_model_config("llama-tiny")
        m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=9, std=0.05)
        total = 24 * world
        ids = torch.arange(7, 7 + total, dtype=torch.int32)
        local = cpx.zigzag_shard(ids, world, rank)
        shards = {}
        h = m.forward_cp(local, total, kv_sink=lambda i, k, v: shards.setdefault(i, (k, v)))
        parts = [torch.empty_like(h) for _ in range(world)]
        dist.all_gather(parts, h.contiguous())
        full_h = cpx.zigzag_unshard(parts)
        q.put((rank, m.logits(full_h).detach().numpy(), tuple(tuple(t.shape) for t in shards[0])))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 3])
def test_model_forward_cp_matches_single_process_prefill(world):
    """A whole Llama decoder prefilled context-parallel (zig-zag shards, ring attention per layer,
    RoPE at global positions) reproduces the single-process prefill logits of every token."""
    from financial_chatbot_llm_amd.models.configs import get_model_config
    from financial_chatbot_llm_amd.models.llama import LlamaModel
    from test_model_parity import _prefill_logits
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cp_model_worker, args=(r, world, port, qq)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = qq.get(timeout=200)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not (isinstance(v[0], str) and v[0] == "ERR"), v[1]
    cfg = get_model_config("llama-tiny")
    ref = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=9, std=0.05)
    want = _prefill_logits(ref, list(range(7, 7 + 24 * world)))
    for r in range(world):
        got = torch.from_numpy(res[r][0])
        assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (got - want).abs().max()
        assert res[r][1][0] == (24, cfg.num_kv_heads, cfg.head_dim)       # local K shard per layer
