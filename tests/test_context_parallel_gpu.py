"""Context parallelism on the HIP kernels (GPU box, one MI355X).

* the prefill kernel's log-sum-exp output equals the fp32 reference (both tile kernels, causal
  and bidirectional, D = 128 / 64);
* the HIP ring block (zig-zag chunk pairs on the paged MFMA prefill kernel) equals the fp32
  torch block for every (q shard, kv shard) pair;
* a whole decoder prefilled context-parallel over 2 ranks sharing the GPU (gloo carries the ring
  hops) reproduces the single-process prefill logits.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from financial_chatbot_llm_amd import ops
from financial_chatbot_llm_amd.ops.attention import KV_BS, _lse_ref, gather_kv_ref
from financial_chatbot_llm_amd.parallel import context as cpx

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("qlen,ctx,D,causal", [(300, 300, 128, True), (70, 500, 128, True), (20, 200, 64, False),
                                                (257, 600, 128, False)])
def test_prefill_lse_matches_reference(qlen, ctx, D, causal):
    g = torch.Generator().manual_seed(qlen)
    Hq, Hkv = 8, 2
    nb = (ctx + KV_BS - 1) // KV_BS
    kc = (torch.randn(nb + 1, Hkv, KV_BS * D, generator=g) * 0.5).to(torch.bfloat16)
    vc = torch.randn(nb + 1, Hkv, KV_BS * D, generator=g).to(torch.bfloat16)
    bt = torch.arange(1, nb + 1, dtype=torch.int32)[None]
    q = torch.randn(qlen, Hq, D, generator=g).to(torch.bfloat16)
    lse = torch.empty(qlen, Hq, device=DEV)
    ops.prefill(q.to(DEV), torch.tensor([0, qlen], dtype=torch.int32, device=DEV),
                torch.tensor([ctx], dtype=torch.int32, device=DEV), bt.to(DEV), kc.to(DEV), vc.to(DEV),
                D ** -0.5, causal, qlen, lse=lse)
    k, _ = gather_kv_ref(kc, vc, bt[0], ctx)
    ref = _lse_ref(q, k, D ** -0.5, ctx - qlen if causal else None)
    assert torch.allclose(lse.cpu(), ref, atol=2e-2, rtol=1e-3), (lse.cpu() - ref).abs().max()


def test_hip_ring_block_matches_torch_block():
    g = torch.Generator().manual_seed(4)
    T, Hq, Hkv, D, cp = 512, 8, 2, 128, 2
    q = torch.randn(T, Hq, D, generator=g).to(torch.bfloat16)
    k = (torch.randn(T, Hkv, D, generator=g) * 0.5).to(torch.bfloat16)
    v = torch.randn(T, Hkv, D, generator=g).to(torch.bfloat16)
    for rq in range(cp):
        for rk in range(cp):
            pq, pk = cpx.zigzag_positions(T, cp, rq), cpx.zigzag_positions(T, cp, rk)
            a = cpx.hip_block_attention(q[pq].to(DEV), k[pk].to(DEV), v[pk].to(DEV), pq.to(DEV), pk.to(DEV),
                                        D ** -0.5, True)
            b = cpx.torch_block_attention(q[pq], k[pk], v[pk], pq, pk, D ** -0.5, True)
            fin = torch.isfinite(b[1])
            assert torch.equal(torch.isfinite(a[1]).cpu(), fin)
            assert torch.allclose(a[1].cpu()[fin], b[1][fin], atol=2e-2)
            assert torch.allclose(a[0].cpu(), b[0], atol=3e-2, rtol=3e-2)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    from financial_chatbot_llm_amd.models.configs import get_model_config
    from financial_chatbot_llm_amd.models.llama import LlamaModel
    return LlamaModel(get_model_config("llama-tiny-tp"), device=DEV).init_random(seed=13, std=0.05)


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        m = _model()
        total = 512
        ids = torch.arange(11, 11 + total, dtype=torch.int32, device=DEV)
        h = m.forward_cp(cpx.zigzag_shard(ids, world, rank), total)
        parts = [torch.empty_like(h).cpu() for _ in range(world)]
        dist.all_gather(parts, h.cpu().contiguous())
        logits = m.logits(cpx.zigzag_unshard(parts).to(DEV)).float().cpu().numpy()
        torch.cuda.synchronize()
        q.put((rank, logits))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


@pytest.mark.timeout(240)
def test_forward_cp_two_ranks_matches_single_gpu_prefill():
    from financial_chatbot_llm_amd.models.common import AttentionMetadata, KVCache
    m = _model()
    T = 512
    nb = T // KV_BS
    kv = KVCache(m.cfg.num_layers, nb + 1, m.hkv, m.D, device=DEV)
    bt = torch.arange(1, nb + 1, dtype=torch.int32, device=DEV)[None]
    slots = torch.arange(KV_BS, KV_BS + T, dtype=torch.int32, device=DEV)
    meta = AttentionMetadata(slots=slots, num_prefill_tokens=T, cu_q=torch.tensor([0, T], dtype=torch.int32, device=DEV),
                             ctx_lens_p=torch.tensor([T], dtype=torch.int32, device=DEV), block_tables_p=bt, max_q_len=T)
    ref = m.logits(m.forward(torch.arange(11, 11 + T, dtype=torch.int32, device=DEV),
                             torch.arange(T, dtype=torch.int32, device=DEV), meta, kv)).float().cpu()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=200) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not (isinstance(v, str) and v.startswith("ERR")), v
    got = torch.from_numpy(res[0])
    # bf16 activations; the ring merges per-chunk partials: compare logits and greedy tokens
    err = (got - ref).abs()
    assert err.mean() < 0.02 * ref.abs().mean() + 1e-3, (err.mean(), ref.abs().mean())
    assert (got.argmax(-1) == ref.argmax(-1)).float().mean() > 0.9
