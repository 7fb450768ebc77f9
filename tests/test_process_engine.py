"""Engine-core process (``engine/process_engine.py``) on CPU.

The child-process engine must be a drop-in for the in-process ``AsyncEngine``: identical tokens
for the same requests (greedy and seeded sampling, forced outputs), streamed per step, abort of an
abandoned stream, stats round trip, and a clean shutdown.
"""
import asyncio

import pytest

from financial_chatbot_llm_amd.config import EngineConfig
from financial_chatbot_llm_amd.engine import SamplingParams
from financial_chatbot_llm_amd.engine.async_engine import AsyncEngine
from financial_chatbot_llm_amd.engine.process_engine import ProcessAsyncEngine

CFG = dict(model="llama-tiny", device="cpu", max_model_len=1024, max_num_batched_tokens=256,
           use_cuda_graph=False, max_num_seqs=8, num_kv_blocks=64)


def _prompts(n, length=40):
    return [list(range(100 + 17 * i, 100 + 17 * i + length + 3 * i)) for i in range(n)]


async def _run_all(eng, prompts, params):
    outs = await asyncio.gather(*(eng.generate_all(p, sp) for p, sp in zip(prompts, params)))
    return [o.seq.output_ids for o in outs]


def _params():
    return [SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True),
            SamplingParams(temperature=0.7, max_tokens=9, ignore_eos=True, seed=3),
            SamplingParams(temperature=0.5, max_tokens=12, forced_output=[5, 6, 7, 8])]


@pytest.mark.timeout(240)
def test_process_engine_matches_in_process_engine():
    prompts, params = _prompts(3), _params()
    ref_eng = AsyncEngine(EngineConfig(**CFG))
    try:
        ref = asyncio.run(_run_all(ref_eng, prompts, params))
    finally:
        ref_eng.shutdown()
    eng = ProcessAsyncEngine(EngineConfig(**CFG))
    try:
        got = asyncio.run(_run_all(eng, prompts, params))
        assert got == ref
        assert got[2] == [5, 6, 7, 8]          # forced decode ends at the forced length
        s = eng.stats()
        assert s["engine_process"] == 1.0 and s["steps"] > 0 and s["running"] == 0
    finally:
        eng.shutdown()
    assert not eng._proc.is_alive()


@pytest.mark.timeout(240)
def test_process_engine_streams_and_aborts():
    eng = ProcessAsyncEngine(EngineConfig(**CFG))

    async def main():
        # streamed: one StepOutput per token, the last one finished
        items = [o async for o in eng.generate(_prompts(1)[0], SamplingParams(temperature=0.0, max_tokens=5,
                                                                               ignore_eos=True))]
        assert [len(o.new_token_ids) for o in items] == [1] * 5 and items[-1].finished
        assert items[-1].seq.output_ids == [t for o in items for t in o.new_token_ids]
        # a consumer that walks away mid-stream aborts the request in the child (KV freed)
        agen = eng.generate(_prompts(2)[1], SamplingParams(temperature=0.0, max_tokens=200, ignore_eos=True))
        await agen.__anext__()
        await agen.aclose()
        for _ in range(100):
            s = eng.stats()
            if s["running"] == 0 and s["waiting"] == 0:
                break
            await asyncio.sleep(0.05)
        assert s["running"] == 0 and s["kv_usage"] == 0.0
        # the engine keeps serving afterwards
        out = await eng.generate_all(_prompts(3)[2], SamplingParams(temperature=0.0, max_tokens=3, ignore_eos=True))
        assert out.finished and len(out.seq.output_ids) == 3
    try:
        asyncio.run(main())
    finally:
        eng.shutdown()


def test_process_engine_rejects_tp():
    with pytest.raises(ValueError):
        ProcessAsyncEngine(EngineConfig(tp_size=2, **CFG))
