"""Runtime failure of the custom TP all-reduce (VERDICT r5 missing #3), on CPU with gloo, TP = 2.

The device kernel's failure contract (csrc/kernels/allreduce.hip): a rank whose bounded wait
expires -- a peer stalled mid-run -- poisons its flag slots in every peer, so every rank's
collective returns NaN with the error flag set, and every later call fails fast.  Here a host-side
stand-in with exactly that contract replaces the custom instance on both ranks (the kernel path
itself is covered by ``test_custom_ar_gpu.py``); the engine must then

* fail every in-flight request -- the waiting turn sees an exception, which the serving worker
  turns into the reference's error event (main.py:112-122);
* switch the whole TP group to RCCL (gloo here) at one step boundary, the leader telling the
  follower over C4;
* keep serving: the next requests produce exactly the TP = 1 tokens.
"""
import asyncio
import os
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

from financial_chatbot_llm_amd.config import EngineConfig
from financial_chatbot_llm_amd.models.configs import get_model_config

PROMPTS = [list(range(10, 90)), list(range(200, 230))]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class StallingAllReduce:
    """The custom all-reduce's contract on the host: a real sum over the group until call
    ``fail_at``, where rank ``stall_rank`` stalls past the bounded wait; from then on every rank's
    calls return NaN with ``err`` set, without communicating (the kernels' poison + dead-rank exit)."""

    def __init__(self, group, fail_at: int, stall_rank: int = 1, max_bytes: int = 4 << 20):
        import torch.distributed as dist
        self.group, self.fail_at, self.stall_rank, self.max_bytes = group, fail_at, stall_rank, max_bytes
        self.rank = dist.get_rank(group)
        self.calls = 0
        self.err = torch.zeros(1, dtype=torch.int32)

    def eligible(self, x):
        return x.is_contiguous() and x.numel() * x.element_size() <= self.max_bytes

    def gather_eligible(self, x):
        return False

    def all_reduce(self, x, out=None, method=None):
        import torch.distributed as dist
        self.calls += 1
        out = x if out is None else out
        if self.calls == self.fail_at and self.rank == self.stall_rank:
            time.sleep(0.2)                      # the stall (the peer's bounded wait expires)
        if self.calls >= self.fail_at or int(self.err[0]):
            self.err[0] = 1
            out.fill_(float("nan"))
            return out
        dist.all_reduce(x, group=self.group)
        if out is not x:
            out.copy_(x)
        return out

    def close(self):
        pass


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from financial_chatbot_llm_amd.engine import LLMEngine, SamplingParams
        from financial_chatbot_llm_amd.engine.async_engine import AsyncEngine
        from financial_chatbot_llm_amd.engine.model_runner import CollectiveTimeout
        from financial_chatbot_llm_amd.engine.tokenizer import SyntheticLlamaTokenizer
        from financial_chatbot_llm_amd.models.llama import LlamaModel
        from financial_chatbot_llm_amd.parallel import comm
        from financial_chatbot_llm_amd.parallel.dist import init_distributed, shutdown
        ps = init_distributed(tp_size=world, backend="gloo", device_type="cpu")
        cfg = get_model_config("llama-tiny-tp")
        tp = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=7, std=0.05)
        ecfg = EngineConfig(model="unused", device="cpu", num_kv_blocks=32, max_model_len=1024,
                            max_num_batched_tokens=64, use_cuda_graph=False)
        eng = LLMEngine(ecfg, model=tp, tokenizer=SyntheticLlamaTokenizer(cfg.vocab_size))
        # a few decode steps in: well past the prefill of the first request pair
        comm._CUSTOM_AR = StallingAllReduce(ps.tp_group, fail_at=4 * cfg.num_layers + 40)
        out = None
        if rank == 0:
            aeng = AsyncEngine(engine=eng, warmup=False)
            params = SamplingParams(temperature=0.0, max_tokens=24, ignore_eos=True)

            async def turn(p):
                toks = []
                async for o in aeng.generate(p, params):
                    toks += o.new_token_ids
                return toks

            async def main():
                first = await asyncio.gather(*(turn(p) for p in PROMPTS), return_exceptions=True)
                second = await asyncio.gather(*(turn(p) for p in PROMPTS), return_exceptions=True)
                return first, second

            first, second = asyncio.run(main())
            aeng.shutdown()                       # stops the follower too
            out = ([type(e).__name__ for e in first], second, dict(comm.AR_STATUS),
                   comm.custom_all_reduce() is None)
        else:
            eng.follower_loop()
            out = (dict(comm.AR_STATUS), comm.custom_all_reduce() is None)
        q.put((rank, "OK", out))
        shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


@pytest.mark.timeout(300)
def test_stalled_peer_fails_requests_and_falls_back_to_rccl():
    from financial_chatbot_llm_amd.engine import LLMEngine, SamplingParams
    from financial_chatbot_llm_amd.engine.tokenizer import SyntheticLlamaTokenizer
    from financial_chatbot_llm_amd.models.llama import LlamaModel

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, status, payload = q.get(timeout=240)
        res[r] = (status, payload)
    for p in procs:
        p.join(timeout=60)
    for r, (status, payload) in res.items():
        assert status == "OK", payload

    errs, second, status0, gone0 = res[0][1]
    status1, gone1 = res[1][1]
    assert errs == ["CollectiveTimeout", "CollectiveTimeout"]          # both waiting turns were failed
    for st, gone in ((status0, gone0), (status1, gone1)):                # the whole group switched
        assert gone and st["custom"] is False and st["runtime_fallbacks"] == 1

    cfg = get_model_config("llama-tiny-tp")
    ref = LlamaModel(cfg, device="cpu", tp_rank=0, tp_size=1, dtype=torch.float32).init_random(seed=7, std=0.05)
    ecfg = EngineConfig(model="unused", device="cpu", num_kv_blocks=32, max_model_len=1024,
                        max_num_batched_tokens=64, use_cuda_graph=False)
    eng = LLMEngine(ecfg, model=ref, tokenizer=SyntheticLlamaTokenizer(cfg.vocab_size))
    want = eng.generate(PROMPTS, SamplingParams(temperature=0.0, max_tokens=24, ignore_eos=True))
    assert second == want                   # served on after the fallback, exactly the TP = 1 tokens
