"""End-to-end on CPU: the benchmark workload (full serving path) with tiny models."""
import asyncio

import torch

from financial_chatbot_llm_amd.bench.workload import RagWorkload, decide_script
from financial_chatbot_llm_amd.config import EngineConfig
from financial_chatbot_llm_amd.engine.async_engine import AsyncEngine
from financial_chatbot_llm_amd.engine.backend import EngineLLM
from financial_chatbot_llm_amd.retrieval import BgeEmbedder, DeviceVectorStore, RetrievalService


def test_rag_workload_cpu():
    emb = BgeEmbedder("bert-tiny", device="cpu")
    store = DeviceVectorStore(emb.dim, device="cpu")
    store.load_synthetic(5000, 50, seed=0)
    ret = RetrievalService(emb, store)
    ecfg = EngineConfig(model="llama-tiny", device="cpu", num_kv_blocks=256, max_model_len=4096,
                        max_num_batched_tokens=4096, use_cuda_graph=False, max_num_seqs=16)
    eng = AsyncEngine(ecfg)
    llm = EngineLLM(eng, max_model_len=4096, decide_script=decide_script, respond_ignore_eos=True, respond_tokens=8)

    async def main():
        wl = RagWorkload(llm, ret, num_convs=4, num_users=50, respond_tokens=8)
        wl.kafka.setup_consumer()
        task = asyncio.create_task(wl.worker.consume_messages())
        r1 = await wl.run_wave()
        r2 = await wl.run_wave()
        r3 = await wl.run_closed_loop(2)          # independent per-conversation clients
        assert r3.turns == 8 and r3.errors == 0 and wl.turn_of == [4, 4, 4, 4]
        assert len(r3.stages["respond_first_token"]) == 8
        wl.worker.stop()
        await task
        return wl, r1, r2

    try:
        wl, r1, r2 = asyncio.run(main())
    finally:
        eng.shutdown()
    assert r1.turns == 4 and r1.errors == 0 and r2.errors == 0
    assert r1.retrievals == 2 and r2.retrievals == 2
    assert len(r1.ttfts) == 4
    out = wl.broker.values("ai_response")
    assert sum(e.get("type") == "complete" for e in out) == 16
    # prefix cache: wave 2 prompts extend wave 1's and share the system prompt
    assert eng.engine.bm.hits > 0
    saved = list(wl.db.messages_collection.find({"sender": "AIMessage"}))
    assert len(saved) == 16 and all(isinstance(d["message"], str) for d in saved)


def test_multistep_agent_workload_cpu():
    """North-star config 4's agent loop on the bench workload: retrieve, then plot, then answer."""
    emb = BgeEmbedder("bert-tiny", device="cpu")
    store = DeviceVectorStore(emb.dim, device="cpu")
    store.load_synthetic(5000, 50, seed=0)
    ret = RetrievalService(emb, store)
    ecfg = EngineConfig(model="llama-tiny", device="cpu", num_kv_blocks=256, max_model_len=4096,
                        max_num_batched_tokens=4096, use_cuda_graph=False, max_num_seqs=16)
    eng = AsyncEngine(ecfg)
    llm = EngineLLM(eng, max_model_len=4096, decide_script=decide_script, respond_ignore_eos=True, respond_tokens=6)

    async def main():
        wl = RagWorkload(llm, ret, num_convs=4, num_users=50, respond_tokens=6, max_tool_steps=3)
        plot = wl.agent.tools["create_financial_plot"]
        real = plot.ainvoke

        async def counted(args):
            calls.append(args)
            return await real(args)
        plot.ainvoke = counted
        wl.kafka.setup_consumer()
        task = asyncio.create_task(wl.worker.consume_messages())
        r = await wl.run_closed_loop(1)
        wl.worker.stop()
        await task
        return r
    calls = []
    try:
        r = asyncio.run(main())
    finally:
        eng.shutdown()
    assert r.turns == 4 and r.errors == 0 and r.retrievals == 2
    assert len(calls) == 2 and all(c["plot_config"]["plot_type"] == "bar" for c in calls)
