"""Expert parallelism on CPU with gloo, world_size 2.

* the all-to-all dispatch/combine of one token shard per rank equals the single-process MoE;
* Mixtral with ``moe_parallel="ep"`` under TP=2 (whole experts per rank, routed rows exchanged
  by all_to_all_single) reproduces the unsharded model's logits, in bf16-expert and fp8 form.
"""
import os
import socket

import pytest
import torch
from mp_util import to_np, to_torch
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ref_moe(x, logits, w13, w2, top_k):
    from financial_chatbot_llm_amd import ops
    from financial_chatbot_llm_amd.ops.moe import topk_softmax
    topw, topi = topk_softmax(logits, top_k)
    out = torch.zeros_like(x)
    for t in range(x.shape[0]):
        for j in range(top_k):
            e = int(topi[t, j])
            y = torch.nn.functional.linear(ops.silu_mul(torch.nn.functional.linear(x[t:t + 1], w13[e])), w2[e])
            out[t] += topw[t, j] * y[0]
    return out


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch.distributed as dist

        from financial_chatbot_llm_amd.models.configs import get_model_config
        from financial_chatbot_llm_amd.models.mixtral import MixtralModel
        from financial_chatbot_llm_amd.parallel.dist import init_distributed, shutdown
        from financial_chatbot_llm_amd.parallel.ep import ep_moe_shard, expert_range
        from test_model_parity import _prefill_logits
        init_distributed(tp_size=world, backend="gloo", device_type="cpu")
        # 1) raw dispatch/combine: each rank owns different tokens
        g = torch.Generator().manual_seed(5)
        E, H, F_, K = 4, 32, 48, 2
        w13, w2 = torch.randn(E, 2 * F_, H, generator=g) * 0.1, torch.randn(E, H, F_, generator=g) * 0.1
        xs = torch.randn(2, 9, H, generator=g)
        rw = torch.randn(E, H, generator=g)
        x = xs[rank][: 9 - 4 * rank]                      # uneven shards (9 and 5 tokens)
        lo, hi = expert_range(E, rank, world)
        f = lambda rows, e: torch.nn.functional.linear(  # noqa: E731
            __import__("financial_chatbot_llm_amd").ops.silu_mul(torch.nn.functional.linear(rows, w13[lo + e])),
            w2[lo + e])
        got = ep_moe_shard(x, x @ rw.t(), K, E, f)
        raw = (got, _ref_moe(x, x @ rw.t(), w13, w2, K))
        # 2) Mixtral EP under TP=2
        cfg = get_model_config("mixtral-tiny")
        m = MixtralModel(cfg, device="cpu", dtype=torch.float32, moe_parallel="ep").init_random(seed=4, std=0.05)
        ids = list(range(30, 101))
        logits = _prefill_logits(m, ids)
        m.quantize_experts()
        logits_fp8 = _prefill_logits(m, ids)
        q.put((rank, to_np(raw), to_np(logits), to_np(logits_fp8), m.w["layers.0.w13_t"].shape[0]))
        dist.barrier()
        shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), None, None))


@pytest.mark.timeout(300)
def test_expert_parallel_all_to_all_matches_single_process():
    from financial_chatbot_llm_amd.models.configs import get_model_config
    from financial_chatbot_llm_amd.models.mixtral import MixtralModel
    from test_model_parity import _prefill_logits

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        item = q.get(timeout=240)
        res[item[0]] = to_torch(item[1:])
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not (isinstance(v[0], str) and v[0] == "ERR"), v[1]
    for r in (0, 1):
        got, ref = res[r][0]
        assert torch.allclose(got, ref, atol=1e-5), (got - ref).abs().max()
        assert res[r][3] == 2                                    # 2 of 4 experts per rank
    cfg = get_model_config("mixtral-tiny")
    ref = MixtralModel(cfg, device="cpu", dtype=torch.float32, tp_rank=0, tp_size=1).init_random(seed=4, std=0.05)
    ids = list(range(30, 101))
    ref_logits = _prefill_logits(ref, ids)
    ref.quantize_experts()
    ref_fp8 = _prefill_logits(ref, ids)
    for r in (0, 1):
        assert torch.allclose(res[r][1], ref_logits, atol=1e-4, rtol=1e-4)
        assert torch.allclose(res[r][2], ref_fp8, atol=1e-4, rtol=1e-4)
