"""Context parallelism reachable from serving (engine/context_prefill.py), CPU + gloo.

A 2-rank CP replica (each rank with the full weights): the leader's engine prefills a long prompt
context-parallel -- zig-zag shards, ring attention, the K/V shards gathered to the leader's
paged pool -- and then decodes it as usual.  The paged K/V of the prompt must equal what a
single-process engine's ordinary prefill writes, and the greedy continuation must be produced.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
from mp_util import to_np, to_torch

PROMPT = [(37 * i + 11) % 20000 + 100 for i in range(301)]
CP_T = 300                       # (301 - 1) rounded down to a multiple of 2*cp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg(cp, device="cpu"):
    from financial_chatbot_llm_amd.config import EngineConfig
    return EngineConfig(model="llama-tiny", device=device, num_kv_blocks=64, max_model_len=1024, max_num_seqs=4,
                        use_cuda_graph=False, cp_size=cp, cp_min_tokens=64, seed=5, kv_mem_fraction=0.05)


def _run(eng, prompt, max_tokens=4):
    """Greedy-generate ``prompt``; returns (output ids, the prompt's first CP_T paged K/V per layer)."""
    from financial_chatbot_llm_amd.engine import SamplingParams
    from financial_chatbot_llm_amd.ops.attention import gather_kv_ref
    seq = eng.add_request("r0", prompt, SamplingParams(temperature=0.0, max_tokens=max_tokens, ignore_eos=True))
    kv = None
    while not seq.finished:
        eng.step()
        if kv is None and seq.num_computed >= CP_T and seq.block_table:
            bt = torch.tensor(seq.block_table, dtype=torch.int32)
            kv = [tuple(t.float().cpu().clone() for t in gather_kv_ref(eng.kv.k(i), eng.kv.v(i), bt.to(eng.device),
                                                                        CP_T))
                  for i in range(eng.model.cfg.num_layers)]
    while eng.has_work():
        eng.step()
    return list(seq.output_ids), kv


def _worker(rank, world, port, q, device):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from financial_chatbot_llm_amd.engine.llm_engine import LLMEngine
        from financial_chatbot_llm_amd.parallel.dist import init_cp_groups, init_distributed, shutdown
        init_distributed(tp_size=1, backend="gloo", device_type=device)
        init_cp_groups(world)
        eng = LLMEngine(_cfg(world, device))
        if rank == 0:
            out, kv = _run(eng, PROMPT)
            stats = eng.stats()
            eng.stop_followers()
            q.put((rank, to_np(kv), out, stats.get("cp_prefills", 0), stats.get("cp_tokens", 0)))
        else:
            eng.cp_follower_loop()
            q.put((rank, None, None, 0, 0))
        shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), 0, 0))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_engine_context_parallel_prefill_matches_single_process(device):
    """device=cuda: both ranks share cuda:0 -- QKV / O / MLP on the HIP GEMMs, q/k RoPE in one HIP
    pass, ring blocks on the HIP prefill kernel, the gathered K/V written by the HIP KV writer."""
    world = 2
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, qq, device)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = qq.get(timeout=280)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not (isinstance(v[0], str) and v[0] == "ERR"), v[1]
    kv_cp, out_cp, n_cp, tok_cp = res[0]
    assert n_cp == 1 and tok_cp == CP_T                 # the prompt went through the CP path
    from financial_chatbot_llm_amd.engine.llm_engine import LLMEngine
    ref_out, ref_kv = _run(LLMEngine(_cfg(1, device)), PROMPT)
    assert len(out_cp) == len(ref_out) == 4
    for (k, v), (rk, rv) in zip(to_torch(kv_cp), ref_kv):
        assert torch.allclose(k, rk, atol=3e-2, rtol=3e-2), (k - rk).abs().max()
        assert torch.allclose(v, rv, atol=3e-2, rtol=3e-2), (v - rv).abs().max()


PROMPT2 = PROMPT[:256] + [(53 * i + 7) % 20000 + 100 for i in range(101)]   # 256 cached + 101 new


def _worker_interleave(rank, world, port, q):
    """Leader: a short request decodes while the long prompt is prefilled context-parallel one
    layer per engine step; then a second long prompt that shares PROMPT's first 256 tokens runs
    the CP pass over its uncached suffix only (prefix K/V broadcast from the leader's pool)."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from financial_chatbot_llm_amd.engine import SamplingParams
        from financial_chatbot_llm_amd.engine.llm_engine import LLMEngine
        from financial_chatbot_llm_amd.ops.attention import gather_kv_ref
        from financial_chatbot_llm_amd.parallel.dist import init_cp_groups, init_distributed, shutdown
        init_distributed(tp_size=1, backend="gloo", device_type="cpu")
        init_cp_groups(world)
        cfg = _cfg(world)
        cfg.cp_layers_per_step = 1
        eng = LLMEngine(cfg)
        if rank == 0:
            short = eng.add_request("short", list(range(500, 540)),
                                    SamplingParams(temperature=0.0, max_tokens=40, ignore_eos=True))
            for _ in range(3):
                eng.step()
            long_ = eng.add_request("long", PROMPT, SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True))
            during = []
            while not long_.finished:
                active = eng.cp.active is not None
                n0 = len(short.output_ids)
                eng.step()
                if active:
                    during.append(len(short.output_ids) - n0)
            while eng.has_work():
                eng.step()
            seq2 = eng.add_request("long2", PROMPT2, SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True))
            kv2 = None
            while not seq2.finished:
                eng.step()
                if kv2 is None and seq2.num_computed >= 352 and seq2.block_table:
                    bt = torch.tensor(seq2.block_table, dtype=torch.int32)
                    kv2 = [tuple(t.float().clone() for t in gather_kv_ref(eng.kv.k(i), eng.kv.v(i), bt, 352))
                           for i in range(eng.model.cfg.num_layers)]
            stats = eng.stats()
            eng.stop_followers()
            q.put((rank, during, to_np(kv2), stats.get("cp_prefills", 0), stats.get("cp_prefix_tokens", 0)))
        else:
            eng.cp_follower_loop()
            q.put((rank, None, None, 0, 0))
        shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), 0, 0))


@pytest.mark.timeout(300)
def test_cp_prefill_interleaves_decode_and_reuses_the_prefix_cache():
    world = 2
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_interleave, args=(r, world, port, qq)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = qq.get(timeout=280)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not (isinstance(v[0], str) and v[0] == "ERR"), v[1]
    during, kv2, n_cp, pre = res[0]
    assert n_cp == 2 and pre == 256                # the second pass started after 256 cached tokens
    assert len(during) >= 2 and sum(during) >= 2   # the short request decoded during the CP slices
    from financial_chatbot_llm_amd.engine import SamplingParams
    from financial_chatbot_llm_amd.engine.llm_engine import LLMEngine
    from financial_chatbot_llm_amd.ops.attention import gather_kv_ref
    ref = LLMEngine(_cfg(1))
    s = ref.add_request("r", PROMPT2, SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True))
    ref_kv = None
    while not s.finished:
        ref.step()
        if ref_kv is None and s.num_computed >= 352 and s.block_table:
            bt = torch.tensor(s.block_table, dtype=torch.int32)
            ref_kv = [tuple(t.float().clone() for t in gather_kv_ref(ref.kv.k(i), ref.kv.v(i), bt, 352))
                      for i in range(ref.model.cfg.num_layers)]
    for (k, v), (rk, rv) in zip(to_torch(kv2), ref_kv):
        assert torch.allclose(k, rk, atol=3e-2, rtol=3e-2), (k - rk).abs().max()
        assert torch.allclose(v, rv, atol=3e-2, rtol=3e-2), (v - rv).abs().max()


def _worker_abort(rank, world, port, q):
    """Leader: abort the long request while its CP pass is in progress (one layer per step)."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from financial_chatbot_llm_amd.engine import SamplingParams
        from financial_chatbot_llm_amd.engine.llm_engine import LLMEngine
        from financial_chatbot_llm_amd.parallel.dist import init_cp_groups, init_distributed, shutdown
        init_distributed(tp_size=1, backend="gloo", device_type="cpu")
        init_cp_groups(world)
        cfg = _cfg(world)
        cfg.cp_layers_per_step = 1
        eng = LLMEngine(cfg)
        if rank == 0:
            free0 = eng.bm.num_free()
            long_ = eng.add_request("long", PROMPT, SamplingParams(temperature=0.0, max_tokens=50, ignore_eos=True))
            eng.step()
            mid = eng.cp.active is not None            # the pass is in progress
            eng.abort("long")
            steps = 0
            while eng.has_work() and steps < 200:
                eng.step()
                steps += 1
            # the same replica still serves: another long prompt goes through CP afterwards
            out = eng.generate([PROMPT2], SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True))
            stats = eng.stats()
            eng.stop_followers()
            q.put((rank, mid, len(long_.output_ids), long_ in eng.scheduler.running,
                   stats.get("cp_aborted", 0), (free0, eng.bm.num_free()), len(out[0])))
        else:
            eng.cp_follower_loop()
            q.put((rank, None, None, None, None, None, None))
        shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), None, None, None, None))


@pytest.mark.timeout(300)
def test_cp_prefill_abort_mid_pass_frees_blocks():
    """a request aborted while its context-parallel pass runs must not be handed to the
    scheduler when the pass ends (it would decode to max_tokens for nobody) and its KV blocks go back
    to the pool; the followers still finish the collective pass, and the replica keeps serving."""
    world = 2
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_abort, args=(r, world, port, qq)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = qq.get(timeout=280)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not (isinstance(v[0], str) and v[0] == "ERR"), v[1]
    mid, n_out, running, aborted, (free0, free1), n2 = res[0]
    assert mid and aborted == 1
    assert n_out == 0 and not running
    assert free1 == free0                          # nothing held by the aborted sequence
    assert n2 == 2
