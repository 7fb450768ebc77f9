"""Tensor parallelism on CPU with gloo, world_size 2 and 4 (SURVEY §4 'Distributed').

Each rank owns half the heads / half the MLP columns / half the vocabulary; row-parallel outputs
are all-reduced (C1), vocab-parallel logits all-gathered (C2), and the engine leader broadcasts
each step's packed inputs to the follower (C4).  TP=2 must reproduce TP=1, with and without
sequence parallelism (reduce-scatter / all-gather of the row-sharded residual stream).
"""
import os
import socket

import pytest
import torch
from mp_util import to_np, to_torch
import torch.multiprocessing as mp

from financial_chatbot_llm_amd.config import EngineConfig
from financial_chatbot_llm_amd.models.configs import get_model_config


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    # PENNY_TP_OVERLAP_MIN_ROWS=16: the engine's prefill steps (<= 64 rows here) run the micro-batch
    # pipeline with the all-reduces overlapped (rows cut inside a sequence and between sequences)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), PENNY_TP_OVERLAP_MIN_ROWS="16")
    try:
        from financial_chatbot_llm_amd.engine import LLMEngine, SamplingParams
        from financial_chatbot_llm_amd.engine.tokenizer import SyntheticLlamaTokenizer
        from financial_chatbot_llm_amd.models.llama import LlamaModel
        from financial_chatbot_llm_amd.parallel.dist import init_distributed, shutdown
        from test_model_parity import _prefill_logits
        init_distributed(tp_size=world, backend="gloo", device_type="cpu")
        cfg = get_model_config("llama-tiny-tp")
        tp = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=7, std=0.05)
        ids = list(range(3, 140))
        logits_tp = _prefill_logits(tp, ids)
        tp.sequence_parallel, tp.sp_min_tokens = True, 1     # 137 rows: not a multiple of 2 or 4
        assert tp.uses_sp(len(ids))
        logits_sp = _prefill_logits(tp, ids)
        tp.sequence_parallel = False
        logits_tp = (logits_tp, logits_sp)
        ecfg = EngineConfig(model="unused", device="cpu", num_kv_blocks=32, max_model_len=1024,
                            max_num_batched_tokens=64, use_cuda_graph=False)
        eng = LLMEngine(ecfg, model=tp, tokenizer=SyntheticLlamaTokenizer(cfg.vocab_size))
        out = None
        if rank == 0:
            out = eng.generate([list(range(10, 90)), list(range(200, 230))],
                               SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))
            # temperature sampling, vocab-parallel: per-shard Gumbel-max candidates gathered (C2)
            out = (out, eng.generate([list(range(10, 90)), list(range(200, 230))],
                                     SamplingParams(temperature=0.9, max_tokens=8, ignore_eos=True, seed=123)))
            eng.stop_followers()
            assert eng.runner.stats["overlap_steps"] >= 2, eng.runner.stats
            assert eng.runner.stats.get("vocab_parallel_sample_steps", 0) > 0, eng.runner.stats
            from financial_chatbot_llm_amd.parallel import comm
            ch = comm.step_channel()        # C4 went through the shared-memory ring
            assert ch is not None and ch.sent > 0 and ch.fallbacks == 0
        else:
            eng.follower_loop()
        q.put((rank, to_np(logits_tp), out))
        shutdown()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_tp_matches_tp1(world):
    from financial_chatbot_llm_amd.engine import LLMEngine, SamplingParams
    from financial_chatbot_llm_amd.engine.tokenizer import SyntheticLlamaTokenizer
    from financial_chatbot_llm_amd.models.llama import LlamaModel
    from test_model_parity import _prefill_logits

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, a, b = q.get(timeout=240)
        res[r] = (to_torch(a), b)
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert not (isinstance(res[r][0], str) and res[r][0] == "ERR"), res[r][1]

    cfg = get_model_config("llama-tiny-tp")
    ref = LlamaModel(cfg, device="cpu", tp_rank=0, tp_size=1, dtype=torch.float32).init_random(seed=7, std=0.05)
    ref_logits = _prefill_logits(ref, list(range(3, 140)))
    for r in range(world):
        plain, sp = res[r][0]
        assert torch.allclose(plain, ref_logits, atol=1e-4, rtol=1e-4)
        assert torch.allclose(sp, ref_logits, atol=1e-4, rtol=1e-4)      # sequence-parallel prefill
    ecfg = EngineConfig(model="unused", device="cpu", num_kv_blocks=32, max_model_len=1024,
                        max_num_batched_tokens=64, use_cuda_graph=False)
    eng = LLMEngine(ecfg, model=ref, tokenizer=SyntheticLlamaTokenizer(cfg.vocab_size))
    want = eng.generate([list(range(10, 90)), list(range(200, 230))],
                        SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))
    want_t = eng.generate([list(range(10, 90)), list(range(200, 230))],
                          SamplingParams(temperature=0.9, max_tokens=8, ignore_eos=True, seed=123))
    assert res[0][1][0] == want
    assert res[0][1][1] == want_t          # the TP = 1 sampler's tokens, same seeds
