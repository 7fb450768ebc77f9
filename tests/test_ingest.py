"""Real-corpus retrieval: document loaders, bulk ingest, snapshots, WordPiece."""
import asyncio
import datetime as dt
import json
import random

import httpx
import numpy as np
import pytest

from financial_chatbot_llm_amd.retrieval import (BgeEmbedder, CorpusIngestor, DeviceVectorStore, HashEmbedder,
                                                 NumpyVectorStore, RetrievalService, iter_documents)
from financial_chatbot_llm_amd.tools import make_retrieval_tool

NOW = 1_760_000_000
CATS = ["Groceries", "Dining", "Rent", "Travel", "Utilities"]


def _docs(n, users=50, seed=0):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        cat = CATS[i % len(CATS)]
        day = NOW - rng.randrange(0, 365) * 86400
        amt = round(rng.uniform(1, 500), 2)
        out.append({"page_content": f"{dt.datetime.utcfromtimestamp(day):%Y-%m-%d} {cat} purchase number {i} ${amt}",
                    "metadata": {"user_id": f"user-{i % users}", "date": day, "amount": amt, "category": cat}})
    return out


def test_ingest_10k_then_filtered_score_ordered_queries():
    docs = _docs(10_000)
    emb = HashEmbedder(256)
    store = DeviceVectorStore(256, device="cpu")
    stats = CorpusIngestor(emb, store, batch_size=2048).ingest(docs)
    assert stats["ingested"] == 10_000 and stats["docs_per_s"] > 0 and store.size == 10_000
    ref = NumpyVectorStore(256)
    ref.add(emb.embed([d["page_content"] for d in docs]), [d["metadata"]["user_id"] for d in docs],
            [d["metadata"]["date"] for d in docs], docs)
    svc = RetrievalService(emb, store)
    floor = NOW - 30 * 86400
    hits = svc.search_sync("Groceries purchase", "user-7", floor, 25)
    want = ref.search_batch(emb.embed(["Groceries purchase"]), ["user-7"], [floor], [25])[0]
    assert [h.payload["page_content"] for h in hits] == [h.payload["page_content"] for h in want]
    assert all(h.payload["metadata"]["user_id"] == "user-7" and h.payload["metadata"]["date"] >= floor for h in hits)
    assert all(a.score >= b.score for a, b in zip(hits, hits[1:]))
    # the tool returns page_content in score order + structured rows for plotting
    tool = make_retrieval_tool(svc)
    out = tool.invoke({"user_id": "user-7", "search_query": "Groceries purchase", "num_transactions": 5})
    want5 = ref.search_batch(emb.embed(["Groceries purchase"]), ["user-7"], [None], [5])[0]
    assert list(out) == [h.payload["page_content"] for h in want5]
    assert {"date", "amount", "category"} <= set(out.records[0])


def test_snapshot_round_trip(tmp_path):
    docs = _docs(3000, seed=1)
    emb = HashEmbedder(128)
    store = DeviceVectorStore(128, device="cpu")
    CorpusIngestor(emb, store).ingest(docs)
    store.save(str(tmp_path / "snap"))
    back = DeviceVectorStore.load(str(tmp_path / "snap"), device="cpu")
    q = emb.embed(["Rent purchase"])
    a = store.search_batch(q, ["user-3"], [None], [10])[0]
    b = back.search_batch(q, ["user-3"], [None], [10])[0]
    assert [h.id for h in a] == [h.id for h in b] and [h.payload for h in a] == [h.payload for h in b]
    syn = DeviceVectorStore(64, device="cpu")
    syn.load_synthetic(5000, 20, seed=3)
    syn.save(str(tmp_path / "syn"))
    back = DeviceVectorStore.load(str(tmp_path / "syn"), device="cpu")
    assert back.size == 5000 and back.corpus.payload(17) == syn.corpus.payload(17)


def test_loaders_jsonl_json_parquet(tmp_path):
    docs = _docs(50)
    (tmp_path / "a.jsonl").write_text("\n".join(json.dumps(d) for d in docs))
    (tmp_path / "a.json").write_text(json.dumps(docs))
    import pyarrow as pa
    import pyarrow.parquet as pq
    table = pa.table({"page_content": [d["page_content"] for d in docs],
                      "user_id": [d["metadata"]["user_id"] for d in docs],
                      "date": [dt.datetime.utcfromtimestamp(d["metadata"]["date"]).isoformat() + "+00:00" for d in docs]})
    pq.write_table(table, tmp_path / "a.parquet")
    for name in ("a.jsonl", "a.json", "a.parquet"):
        got = list(iter_documents(str(tmp_path / name)))
        assert len(got) == 50 and got[3]["page_content"] == docs[3]["page_content"]
    store = NumpyVectorStore(64)
    st = CorpusIngestor(HashEmbedder(64), store).ingest(iter_documents(str(tmp_path / "a.parquet")))
    assert st["ingested"] == 50 and int(store.corpus.dates[3]) == docs[3]["metadata"]["date"]
    bad = CorpusIngestor(HashEmbedder(64), NumpyVectorStore(64)).ingest([{"page_content": "x"}, docs[0]])
    assert bad["ingested"] == 1 and bad["rejected"] == 1


def test_bge_bulk_encode_is_batch_invariant():
    emb = BgeEmbedder("bert-tiny", device="cpu")
    texts = [d["page_content"] for d in _docs(40)]
    one = np.stack([emb.embed([t])[0].numpy() for t in texts[:5]])
    bulk = emb.embed(texts)[:5].numpy()
    assert np.allclose(one, bulk, atol=2e-2)


def _vocab(tmp_path):
    words = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", "grocery", "purchase", "whole", "foods", "rent",
             "spent", "on", "the", "##s", "##ing", "a", "b", "c", "1", "2", "3", "$", ".", ","]
    p = tmp_path / "vocab.txt"
    p.write_text("\n".join(words) + "\n")
    return str(p)


def test_wordpiece_matches_transformers_and_keeps_sep(tmp_path):
    from transformers import BertTokenizer

    from financial_chatbot_llm_amd.engine.tokenizer import WordPieceTokenizer
    path = _vocab(tmp_path)
    ours = WordPieceTokenizer(path)
    ref = BertTokenizer(path, do_lower_case=True)
    for text in ["Grocery purchases on the Whole Foods $12.3", "rent", "spent spending xyz"]:
        assert ours.encode(text) == ref(text)["input_ids"]
    long = " ".join(["grocery"] * 100)
    ids = ours.encode(long, max_len=16)
    assert len(ids) == 16 and ids[0] == ours.CLS and ids[-1] == ours.SEP
    assert ref(long, truncation=True, max_length=16)["input_ids"] == ids
    emb = BgeEmbedder("bert-tiny", device="cpu", vocab=path, max_len=8)
    assert all(t[-1] == ours.SEP and len(t) <= 8 for t in emb.tokenize(["grocery " * 20, "rent"]))


def test_http_ingest_then_retrieve():
    from financial_chatbot_llm_amd.agent import StubLLM
    from financial_chatbot_llm_amd.serving import create_app
    from financial_chatbot_llm_amd.serving.factory import build_stub_services
    from financial_chatbot_llm_amd.tools import ToolCall
    from helpers import TODAY, seeded_db
    emb = HashEmbedder(64)
    store = NumpyVectorStore(64)
    llm = StubLLM(decisions=[ToolCall("retrieve_transactions", {"search_query": "Groceries purchase"})], responses=["ok"])
    from financial_chatbot_llm_amd.config import ServingConfig
    svc = build_stub_services(db=seeded_db((("c9", "user-9"),)), llm=llm, store=store, embedder=emb, today_fn=lambda: TODAY,
                              serving=ServingConfig(backend="stub", ingest_token="s3cret"))
    svc.db.put_user_message("c9", "groceries?", "user-9", 1)
    app = create_app(svc, start_consumer=False)

    async def main():
        async with app.router.lifespan_context(app):
            async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as cl:
                r = await cl.post("/v1/transactions", json={"documents": _docs(200)})
                assert r.status_code == 401 and len(store.corpus) == 0                    # no token
                r = await cl.post("/v1/transactions", json={"documents": _docs(200)},
                                  headers={"Authorization": "Bearer wrong"})
                assert r.status_code == 401 and len(store.corpus) == 0
                r = await cl.post("/v1/transactions", json={"documents": _docs(200)},
                                  headers={"Authorization": "Bearer s3cret"})
                assert r.status_code == 200 and r.json()["ingested"] == 200 and r.json()["size"] == 200
                r = await cl.post("/process_message", json={"conversation_id": "c9", "message": "What did I spend on groceries?",
                                                            "user_id": "user-9"})
                assert r.json()["retrieved_transactions_count"] == 4      # user-9 owns 4 of the 200
    asyncio.run(main())


def test_ingest_endpoint_absent_without_operator_token():
    from financial_chatbot_llm_amd.serving import create_app
    from financial_chatbot_llm_amd.serving.factory import build_stub_services
    app = create_app(build_stub_services(), start_consumer=False)

    async def main():
        async with app.router.lifespan_context(app):
            async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as cl:
                r = await cl.post("/v1/transactions", json={"documents": _docs(5)})
                assert r.status_code in (404, 405)
    asyncio.run(main())


def test_ingest_takes_the_search_lock_per_batch_only():
    """A search waiting on the retrieval lock runs between ingest batches, not after the whole
    ingest (the lock is held per 1024-document batch)."""
    import threading
    emb = HashEmbedder(32)
    store = NumpyVectorStore(32)
    lock = threading.Lock()
    events = []
    orig = store.add

    def add(*a, **k):
        events.append("add")
        return orig(*a, **k)
    store.add = add
    ing = CorpusIngestor(emb, store, batch_size=50, lock=lock)
    done = threading.Event()

    def searcher():
        while not done.is_set():
            with lock:
                if events and events[-1] == "add":
                    events.append("search")
    t = threading.Thread(target=searcher)
    t.start()
    import time as _t
    orig_flush = ing._flush_locked

    def slow(batch):
        orig_flush(batch)
        _t.sleep(0.01)
    ing._flush_locked = slow
    ing.ingest(_docs(300))
    done.set()
    t.join()
    assert events.count("add") == 6 and len(store.corpus) == 300
    assert "search" in events[:-1]           # a search got the lock before the last batch


@pytest.mark.gpu
def test_bulk_bge_ingest_on_gpu_reports_docs_per_s():
    """bge-base-en bulk encode of 20k transactions on the GPU (K14 bulk mode) into the HBM store;
    queries agree with an exact host search over the same vectors."""
    import torch
    emb = BgeEmbedder("bge-base-en", device="cuda")
    store = DeviceVectorStore(emb.dim, device="cuda")
    docs = _docs(20_000, users=200)
    CorpusIngestor(emb, store, batch_size=4096).ingest(docs[:4096])          # warm-up batch
    st = CorpusIngestor(emb, store, batch_size=4096).ingest(docs[4096:])
    print(f"bulk bge-base ingest: {st}")
    assert store.size == 20_000 and st["docs_per_s"] > 1000
    host = NumpyVectorStore(emb.dim)
    host.add(store.vectors[:store.size].float().cpu().numpy(), [d["metadata"]["user_id"] for d in docs],
             [d["metadata"]["date"] for d in docs], docs)
    q = emb.embed(["Dining purchase"]).float().cpu().numpy()
    got = store.search_batch(q, ["user-11"], [NOW - 90 * 86400], [20])[0]
    want = host.search_batch(q, ["user-11"], [NOW - 90 * 86400], [20])[0]
    assert len(got) == len(want) > 0
    assert np.allclose([h.score for h in got], [h.score for h in want], atol=2e-3)   # same ranking up to ties
    assert all(h.payload["metadata"]["user_id"] == "user-11" for h in got)
    torch.cuda.synchronize()
