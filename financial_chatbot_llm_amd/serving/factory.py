"""Build the serving stack (db, kafka, retrieval, LLM backend, agent) from config.

``backend="stub"`` is north-star config 1 (CPU plumbing: scripted LLM, hash embedder, numpy
brute-force store).  ``backend="engine"`` runs the MI355X stack: a local Llama-3 engine,
the bge encoder and the HBM-resident corpus searched by the HIP top-k kernel.
"""
from __future__ import annotations

import datetime as _dt
from typing import Any, Optional

from .. import config
from ..adapters import Database, InMemoryBroker, KafkaClient
from ..agent import LLMAgent, LLMService, StubLLM
from ..retrieval import HashEmbedder, NumpyVectorStore, RetrievalService
from ..tools import make_plot_tool, make_retrieval_tool
from .app import Services


def retrieval_limit_tokens() -> int:
    return config.RetrievalConfig.from_env().max_limit_tokens


def build_stub_services(broker: Optional[InMemoryBroker] = None, db: Optional[Database] = None,
                        llm=None, store=None, embedder=None, serving: Optional[config.ServingConfig] = None,
                        today_fn=_dt.date.today, max_tool_steps: int = 1) -> Services:
    serving = serving or config.ServingConfig(backend="stub")
    db = db or Database(uri="")
    kafka = KafkaClient(broker=broker or InMemoryBroker())
    embedder = embedder or HashEmbedder(768)
    store = store or NumpyVectorStore(embedder.dim)
    retrieval = RetrievalService(embedder, store)
    llm = llm or StubLLM()
    if not serving.tools:
        agent = LLMService(llm, temperature=serving.temperature, max_response_tokens=serving.max_response_tokens)
    else:
        agent = LLMAgent(llm, make_retrieval_tool(retrieval),
                         extra_tools=[make_plot_tool()], temperature=serving.temperature,
                         max_response_tokens=serving.max_response_tokens,
                         max_decide_tokens=serving.max_decide_tokens, max_tool_steps=max_tool_steps,
                         today_fn=today_fn, max_transaction_tokens=retrieval_limit_tokens())
    return Services(db=db, kafka=kafka, agent=agent, retrieval=retrieval, serving=serving)


def build_engine_services(engine_cfg: Optional[config.EngineConfig] = None,
                          retrieval_cfg: Optional[config.RetrievalConfig] = None,
                          serving: Optional[config.ServingConfig] = None,
                          broker: Optional[InMemoryBroker] = None, db: Optional[Database] = None,
                          max_tool_steps: int = 1) -> Services:
    from ..engine.async_engine import AsyncEngine
    from ..engine.backend import EngineLLM

    engine_cfg = engine_cfg or config.EngineConfig.from_env()
    retrieval_cfg = retrieval_cfg or config.RetrievalConfig.from_env()
    serving = serving or config.ServingConfig.from_env()
    from ..retrieval.ingest import build_store
    engine = AsyncEngine(engine_cfg)
    embedder, store = build_store(retrieval_cfg.embed_model, retrieval_cfg.device, retrieval_cfg.corpus_path,
                                  weights=retrieval_cfg.weights, vocab=retrieval_cfg.vocab)
    if retrieval_cfg.corpus_size and not retrieval_cfg.corpus_path:
        store.load_synthetic(retrieval_cfg.corpus_size, retrieval_cfg.num_users)
    retrieval = RetrievalService(embedder, store)
    llm = EngineLLM(engine, max_model_len=engine_cfg.max_model_len,
                    history_token_budget=serving.history_token_budget)
    if not serving.tools:
        agent = LLMService(llm, temperature=serving.temperature, max_response_tokens=serving.max_response_tokens)
    else:
        agent = LLMAgent(llm, make_retrieval_tool(retrieval), extra_tools=[make_plot_tool()],
                         temperature=serving.temperature, max_response_tokens=serving.max_response_tokens,
                         max_decide_tokens=serving.max_decide_tokens, max_tool_steps=max_tool_steps,
                         max_transaction_tokens=retrieval_cfg.max_limit_tokens)
    return Services(db=db or Database(), kafka=KafkaClient(broker=broker), agent=agent,
                    engine=engine, retrieval=retrieval, serving=serving)


def build_services_from_env() -> Services:
    serving = config.ServingConfig.from_env()
    if serving.backend == "stub":
        return build_stub_services(serving=serving)
    return build_engine_services(serving=serving)
