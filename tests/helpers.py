"""Shared fixtures for the plumbing tests: seeded fakes and a frozen date."""
import datetime as dt
import time

from financial_chatbot_llm_amd.adapters import Database, InMemoryBroker
from financial_chatbot_llm_amd.retrieval import HashEmbedder, NumpyVectorStore

TODAY = dt.date(2026, 10, 15)


def ctx_doc(cid, uid, name="Ada"):
    return {"conversation_id": cid, "user_id": uid, "name": name, "income": 8000, "savings_goal": 1500,
            "accounts": [{"account_id": "a1", "balances": {"current": 1000.0, "iso_currency_code": "USD"},
                          "official_name": "Checking"}],
            "additional_monthly_expenses": [{"name": "Gym", "amount": 50, "description": ""}]}


def seeded_db(convs=(("c1", "u1"),)):
    db = Database(uri="")
    for cid, uid in convs:
        db.put_context(ctx_doc(cid, uid))
    return db


def seeded_store(now=None):
    emb = HashEmbedder(64)
    store = NumpyVectorStore(64)
    now = int(time.time()) if now is None else now
    texts = [("u1", "grocery store purchase Whole Foods $54.20", now - 86400, 54.20, "Groceries"),
             ("u1", "grocery purchase Safeway $12.00", now - 40 * 86400, 12.00, "Groceries"),
             ("u1", "Netflix subscription $15.99", now - 2 * 86400, 15.99, "Entertainment"),
             ("u2", "grocery purchase Trader Joes $33.00", now - 86400, 33.00, "Groceries")]
    store.add(emb.embed([t[1] for t in texts]), [t[0] for t in texts], [t[2] for t in texts],
              [{"page_content": t, "metadata": {"user_id": u, "date": d, "amount": a, "category": c}}
               for u, t, d, a, c in texts])
    return emb, store
