"""FastAPI surface (reference ``main.py:24-53``) plus the services factory.

Endpoints:
* ``GET /health`` -> ``{"status": "healthy"}`` (``main.py:51-53``; Docker HEALTHCHECK target).
* ``POST /process_message`` -- the reference's commented-out sync endpoint (``main.py:39-49``),
  re-enabled: ``{conversation_id, message, user_id}`` -> ``{response, retrieved_transactions_count}``;
  ``user_id`` must be the conversation's owner (403 otherwise) -- retrieval uses the stored id.
* ``POST /v1/chat/stream`` -- server-sent events of the agent's updates for one turn (no Kafka);
  used for latency probing.
* ``GET /metrics`` -- Prometheus text: turns/s, TTFT p50/p99, ITL, KV utilisation, ...
* ``POST /v1/transactions`` -- ingest ``{"documents": [{page_content, metadata{user_id, date,
  ...}}]}`` into the on-device collection (bge bulk embedding + append; the upstream Qdrant
  collection was populated outside the reference repo).  Operator-only: the route exists only
  when ``PENNY_INGEST_TOKEN`` is set and every call must send ``Authorization: Bearer <token>``
  (documents carry their own ``metadata.user_id``, so an open write path would let any caller
  plant rows in another user's retrieval results).  Batches of 1024 documents are embedded and
  appended under the retrieval lock one at a time, so concurrent searches interleave.  The write
  lands in THIS replica's collection only: with several DP replicas (serving/launch.py, one
  port per replica) the operator sends the same batch to every replica's port, or builds the
  collection offline (``retrieval.ingest`` CLI snapshot) and starts every replica from it.
* ``/docs``, ``/redoc``, ``/openapi.json`` come from FastAPI as in the reference.

The lifespan pings Mongo (raising aborts startup), subscribes the Kafka consumer and starts
the background consumer (``main.py:24-30``).  Unlike gunicorn-per-worker replicas of the
reference (``main.py:18-22``), ONE process owns the GPU engine and serves every connection.
"""
from __future__ import annotations

import asyncio
import hmac
import json
from contextlib import asynccontextmanager
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse
from pydantic import BaseModel

from .. import config
from ..utils.logging import get_logger
from ..utils.metrics import METRICS
from .worker import ChatWorker

logger = get_logger(__name__)


@dataclass
class Services:
    db: Any
    kafka: Any
    agent: Any
    engine: Any = None
    retrieval: Any = None
    serving: Optional[config.ServingConfig] = None


class IngestPayload(BaseModel):
    documents: List[Dict[str, Any]]


class MessagePayload(BaseModel):
    conversation_id: str
    message: str
    user_id: str


def create_app(services: Services, start_consumer: bool = True) -> FastAPI:
    serving = services.serving or config.ServingConfig()
    state = {"worker": None, "task": None}

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        await services.db.check_connection()
        worker = ChatWorker(services.db, services.kafka, services.agent,
                            max_concurrent_turns=serving.max_concurrent_turns,
                            message_timeout_s=serving.message_timeout_s)
        state["worker"] = worker
        app.state.worker = worker
        if start_consumer:
            services.kafka.setup_consumer()
            state["task"] = asyncio.create_task(worker.consume_messages())
        try:
            yield
        finally:
            worker.stop()
            if state["task"] is not None:
                state["task"].cancel()
                try:
                    await state["task"]
                except (asyncio.CancelledError, Exception):  # noqa: BLE001
                    pass
            services.kafka.close()
            if services.engine is not None and hasattr(services.engine, "shutdown"):
                services.engine.shutdown()

    app = FastAPI(title="Finance Chatbot LLM Worker",
                  description="A python worker for processing LLM requests",
                  version="1.0.0", lifespan=lifespan)
    app.state.services = services

    @app.get("/health")
    async def health_check():
        # reference body when healthy; 503 once the engine watchdog saw a wedged GPU step, so the
        # container HEALTHCHECK / orchestrator restarts the replica
        if getattr(services.engine, "stalled", False):
            return JSONResponse({"status": "unhealthy", "reason": "engine step stalled"}, status_code=503)
        return {"status": "healthy"}

    @app.get("/metrics", response_class=PlainTextResponse)
    async def metrics():
        if services.engine is not None and hasattr(services.engine, "stats"):
            for k, v in services.engine.stats().items():
                for kk, vv in (v.items() if isinstance(v, dict) else ((None, v),)):
                    METRICS.set_gauge(f"engine_{k}" if kk is None else f"engine_{k}_{kk}", float(vv))
        return METRICS.render_prometheus()

    @app.post("/process_message")
    async def process_message_endpoint(payload: MessagePayload):
        user_context, user_id = await services.db.get_context(payload.conversation_id)
        # retrieval is filtered by this id: it must be the conversation owner's (server-side,
        # as llm_agent.py:119-120 does for the tool args), never a caller-chosen one
        if payload.user_id != user_id:
            return JSONResponse({"detail": "user_id does not own this conversation"}, status_code=403)
        chat_history = await services.db.get_history(payload.conversation_id)
        res = await services.agent.query(payload.message, user_id, user_context, chat_history)
        return {"response": res["response"], "retrieved_transactions_count": res["retrieved_transactions_count"]}

    if serving.ingest_token:
        expected = f"Bearer {serving.ingest_token}".encode()

        @app.post("/v1/transactions")
        async def ingest_transactions(payload: IngestPayload, request: Request):
            got = request.headers.get("authorization", "").encode()
            if not hmac.compare_digest(got, expected):
                return JSONResponse({"detail": "operator token required"}, status_code=401)
            svc = services.retrieval
            if svc is None or not hasattr(svc.store, "add"):
                return JSONResponse({"detail": "no vector store configured"}, status_code=503)
            from ..retrieval.ingest import CorpusIngestor
            # the service lock is taken per 1024-document batch, never for the whole request
            ing = CorpusIngestor(svc.embedder, svc.store, lock=svc._lock)
            stats = await asyncio.to_thread(ing.ingest, payload.documents)
            return {**stats, "size": len(svc.store.corpus), "scope": "this replica"}

    @app.post("/v1/chat/stream")
    async def chat_stream(payload: MessagePayload):
        user_context, user_id = await services.db.get_context(payload.conversation_id)
        chat_history = await services.db.get_history(payload.conversation_id)

        async def gen():
            async for upd in services.agent.stream_with_status(payload.message, user_id, user_context, chat_history):
                yield f"data: {json.dumps(upd)}\n\n"

        return StreamingResponse(gen(), media_type="text/event-stream")

    return app
