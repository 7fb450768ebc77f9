"""Integration: Kafka-fake turn -> streamed chunks -> complete -> Mongo-fake save."""
import asyncio
import json

import httpx

from financial_chatbot_llm_amd import config
from financial_chatbot_llm_amd.adapters import InMemoryBroker
from financial_chatbot_llm_amd.agent import StubLLM
from financial_chatbot_llm_amd.serving import ChatWorker, create_app
from financial_chatbot_llm_amd.serving.factory import build_stub_services
from financial_chatbot_llm_amd.tools import ToolCall
from helpers import TODAY, seeded_db, seeded_store


def services(llm, convs=(("c1", "u1"),), **kw):
    emb, store = seeded_store()
    broker = InMemoryBroker()
    db = seeded_db(convs)
    return build_stub_services(broker=broker, db=db, llm=llm, store=store, embedder=emb, today_fn=lambda: TODAY, **kw)


def send(svc, cid, text, uid="u1", ts=1):
    svc.db.put_user_message(cid, text, uid, ts)
    svc.kafka.producer.produce(config.USER_MESSAGE_TOPIC, key=cid,
                               value=json.dumps({"message": text, "conversation_id": cid, "user_id": uid}))


async def run_worker(svc, n_msgs, timeout_s=100.0):
    svc.kafka.setup_consumer()
    w = ChatWorker(svc.db, svc.kafka, svc.agent, message_timeout_s=timeout_s)
    return w


def drive(svc, msgs, timeout_s=100.0):
    async def main():
        svc.kafka.setup_consumer()
        w = ChatWorker(svc.db, svc.kafka, svc.agent, message_timeout_s=timeout_s)
        task = asyncio.create_task(w.consume_messages())
        for m in msgs:
            send(svc, *m)
        for _ in range(400):
            await asyncio.sleep(0.01)
            if len(w.traces) >= len(msgs) and not w._tasks:
                break
        w.stop()
        await task
        return w
    return asyncio.run(main())


def out(svc, cid=None):
    return svc.kafka.broker.values(config.AI_RESPONSE_TOPIC, cid)


def test_full_turn_streams_then_completes_and_saves():
    svc = services(StubLLM(decisions=[ToolCall("retrieve_transactions", {"search_query": "grocery"})],
                           responses=["one two three four five"], chunk_words=2))
    drive(svc, [("c1", "What did I spend on groceries?")])
    ev = out(svc, "c1")
    assert [e.get("type") for e in ev] == ["response_chunk"] * 3 + ["complete"]
    assert "".join(e["message"] for e in ev[:-1]) == "one two three four five"
    assert ev[-1]["message"] == "What did I spend on groceries?" and ev[-1]["user_id"] == "u1"
    saved = list(svc.db.messages_collection.find({"conversation_id": "c1", "sender": "AIMessage"}))
    assert saved[0]["message"] == "one two three four five" and saved[0]["user_id"] == "u1"


def test_missing_context_sends_nothing():
    svc = services(StubLLM())
    drive(svc, [("nope", "hi", "u9")])
    assert out(svc) == []


def test_agent_error_sends_error_event():
    svc = services(StubLLM(decisions=[None], responses=["a b c d e f"], chunk_words=1, fail_stream=True))
    drive(svc, [("c1", "hello")])
    ev = out(svc, "c1")
    assert ev[-1]["error"] is True and ev[-1]["message"] == "" and "type" not in ev[-1]
    assert svc.db.messages_collection.count_documents({"sender": "AIMessage"}) == 0


def test_timeout_event():
    svc = services(StubLLM(decisions=[None], decide_delay_s=0.5))
    drive(svc, [("c1", "hello")], timeout_s=0.05)
    ev = out(svc, "c1")
    assert ev[-1]["message"] == "Request timed out. Please try again." and ev[-1]["error"] is True


def test_concurrent_conversations_and_per_key_order():
    convs = [(f"c{i}", f"u{i}") for i in range(6)]
    svc = services(StubLLM(stream_delay_s=0.005), convs=convs)
    msgs = [(c, "hello", u) for c, u in convs] + [("c0", "second", "u0", 2)]
    w = drive(svc, msgs)
    assert len(w.traces) == 7 and not any(t.error for t in w.traces)
    ev0 = out(svc, "c0")
    completes = [e for e in ev0 if e.get("type") == "complete"]
    assert [c["message"] for c in completes] == ["hello", "second"]
    # each turn's chunks arrive before its complete (no interleaving within a conversation)
    first_complete = ev0.index(completes[0])
    assert all(e.get("type") == "response_chunk" for e in ev0[:first_complete])


def test_http_surface():
    svc = services(StubLLM(responses=["answer text"]))
    svc.db.put_user_message("c1", "invest?", "u1", 1)
    app = create_app(svc, start_consumer=False)

    async def main():
        async with app.router.lifespan_context(app):
            transport = httpx.ASGITransport(app=app)
            async with httpx.AsyncClient(transport=transport, base_url="http://t") as cl:
                r = await cl.get("/health")
                assert r.json() == {"status": "healthy"}
                r = await cl.post("/process_message", json={"conversation_id": "c1", "message": "invest?", "user_id": "u1"})
                assert r.json()["response"] == "answer text"
                r = await cl.get("/openapi.json")
                assert r.json()["info"]["title"] == "Finance Chatbot LLM Worker"
                r = await cl.get("/metrics")
                assert r.status_code == 200
    asyncio.run(main())


def test_process_message_rejects_foreign_user_id():
    """A caller cannot read another user's transactions by naming their user_id (retrieval is
    filtered by the conversation owner's id, as the tool's server-side injection intends)."""
    llm = StubLLM(decisions=[ToolCall("retrieve_transactions", {"search_query": "grocery"})], responses=["x"])
    svc = services(llm, convs=(("c1", "u1"), ("c2", "u2")))
    svc.db.put_user_message("c2", "groceries?", "u2", 1)
    app = create_app(svc, start_consumer=False)

    async def main():
        async with app.router.lifespan_context(app):
            transport = httpx.ASGITransport(app=app)
            async with httpx.AsyncClient(transport=transport, base_url="http://t") as cl:
                r = await cl.post("/process_message", json={"conversation_id": "c2", "message": "What did I spend on groceries?",
                                                            "user_id": "u1"})
                assert r.status_code == 403
                assert not llm.calls                       # nothing ran, nothing retrieved
                r = await cl.post("/process_message", json={"conversation_id": "c2", "message": "What did I spend on groceries?",
                                                            "user_id": "u2"})
                assert r.status_code == 200 and r.json()["retrieved_transactions_count"] == 1   # u2's one row
    asyncio.run(main())


def test_conversation_lock_survives_saturated_semaphore():
    """Turns of one conversation never overlap, even when the second turn is still queued on the
    concurrency semaphore while the first finishes (lock entry dropped too early)."""
    active, overlaps = {}, []

    class Probe(StubLLM):
        async def agenerate(self, messages, tools=None, **kw):
            cid = messages[-1].content.split()[-1]
            active[cid] = active.get(cid, 0) + 1
            overlaps.append(active[cid])
            await asyncio.sleep(0.01)
            active[cid] -= 1
            return await super().agenerate(messages, tools, **kw)

    convs = [(f"c{i}", f"u{i}") for i in range(4)]
    svc = services(Probe(), convs=convs)

    async def main():
        svc.kafka.setup_consumer()
        w = ChatWorker(svc.db, svc.kafka, svc.agent, max_concurrent_turns=1)
        task = asyncio.create_task(w.consume_messages())
        msgs = [(c, f"hello {c}", u, k) for k in range(3) for c, u in convs]
        for m in msgs:
            send(svc, *m)
        for _ in range(1000):
            await asyncio.sleep(0.01)
            if len(w.traces) >= len(msgs) and not w._tasks:
                break
        w.stop()
        await task
        return w
    w = asyncio.run(main())
    assert len(w.traces) == 12 and not any(t.error for t in w.traces)
    assert max(overlaps) == 1 and not w._conv_locks


def test_no_tools_service_single_chain():
    """Legacy LLMService (llm_service.py:8-33): one respond call, no decide, SYSTEM_PROMPT verbatim."""
    from financial_chatbot_llm_amd.agent import LLMService
    llm = StubLLM(responses=["plain answer"])
    svc = services(llm)
    svc.agent = LLMService(llm, system_prompt="SYS")
    drive(svc, [("c1", "What did I spend on groceries?")])
    ev = out(svc, "c1")
    assert "".join(e["message"] for e in ev if e.get("type") == "response_chunk") == "plain answer"
    assert ev[-1]["type"] == "complete"
    assert [c["kind"] for c in llm.calls] == ["stream"]
    assert llm.calls[0]["messages"][0].content.startswith("SYS\nMy name is Ada.")


# ---- fault injection in the fakes (drop, delay, raise) ------------------------------
def test_fault_poll_errors_back_off_and_recover(monkeypatch):
    """Consumer-loop errors are logged and retried after the backoff (main.py:157-159); the turn
    is processed once polling recovers."""
    monkeypatch.setattr(config, "LOOP_ERROR_BACKOFF_S", 0.01)
    svc = services(StubLLM(responses=["ok"]))
    svc.kafka.broker.faults.raise_on_poll = True

    async def main():
        svc.kafka.setup_consumer()
        w = ChatWorker(svc.db, svc.kafka, svc.agent)
        task = asyncio.create_task(w.consume_messages())
        send(svc, "c1", "hello")
        await asyncio.sleep(0.1)
        assert not w.traces                     # nothing consumed while polling fails
        svc.kafka.broker.faults.raise_on_poll = False
        for _ in range(300):
            await asyncio.sleep(0.01)
            if w.traces:
                break
        w.stop()
        await task
        return w
    w = asyncio.run(main())
    assert len(w.traces) == 1 and not w.traces[0].error
    assert out(svc, "c1")[-1]["type"] == "complete"


def test_fault_dropped_chunks_still_save_the_reply():
    """A lossy producer (dropped records) does not break the turn: the reply is still saved."""
    svc = services(StubLLM(responses=["all the tokens"]))

    async def main():
        svc.kafka.setup_consumer()
        w = ChatWorker(svc.db, svc.kafka, svc.agent)
        send(svc, "c1", "q")                       # the request itself is delivered ...
        svc.kafka.broker.faults.drop_produce = 1.0  # ... every reply record is lost
        task = asyncio.create_task(w.consume_messages())
        for _ in range(300):
            await asyncio.sleep(0.01)
            if w.traces and not w._tasks:
                break
        w.stop()
        await task
        return w
    w = asyncio.run(main())
    assert len(w.traces) == 1 and not w.traces[0].error
    assert out(svc, "c1") == []
    saved = [d for d in svc.db.messages_collection.find({"conversation_id": "c1", "sender": "AIMessage"})]
    assert len(saved) == 1 and saved[0]["message"] == "all the tokens"


def test_fault_produce_raises_marks_turn_failed():
    """A producer that raises mid-stream: the worker reports the turn as failed, tries the
    error event (which also fails) and keeps consuming (next turn succeeds)."""
    svc = services(StubLLM(responses=["first", "second"]), convs=(("c1", "u1"), ("c2", "u1")))

    async def main():
        svc.kafka.setup_consumer()
        w = ChatWorker(svc.db, svc.kafka, svc.agent)
        send(svc, "c1", "q1")
        svc.kafka.broker.faults.raise_on_produce = True
        task = asyncio.create_task(w.consume_messages())
        for _ in range(300):
            await asyncio.sleep(0.01)
            if w.traces:
                break
        svc.kafka.broker.faults.raise_on_produce = False
        send(svc, "c2", "q2")
        for _ in range(300):
            await asyncio.sleep(0.01)
            if len(w.traces) >= 2:
                break
        w.stop()
        await task
        return w
    w = asyncio.run(main())
    assert len(w.traces) == 2 and w.traces[0].error and not w.traces[1].error
    assert out(svc, "c2")[-1]["type"] == "complete"


def test_fault_slow_producer_delays_but_delivers():
    """A slow (blocking) producer, like a congested librdkafka queue: every record is still
    delivered in order and the turn's latency absorbs the delay."""
    svc = services(StubLLM(responses=["slow answer here"]))

    async def main():
        svc.kafka.setup_consumer()
        w = ChatWorker(svc.db, svc.kafka, svc.agent)
        send(svc, "c1", "q")
        svc.kafka.broker.faults.delay_produce_s = 0.05
        task = asyncio.create_task(w.consume_messages())
        for _ in range(300):
            await asyncio.sleep(0.01)
            if w.traces and not w._tasks:
                break
        w.stop()
        await task
        return w
    w = asyncio.run(main())
    svc.kafka.broker.faults.delay_produce_s = 0.0
    tr = w.traces[0]
    assert not tr.error and tr.t_complete - tr.t_receive >= 0.1   # >= 2 delayed records
    ev = out(svc, "c1")
    assert [e.get("type") for e in ev] == ["response_chunk", "complete"]
