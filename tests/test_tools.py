"""Tool schema / semantics tests (reference tools/qdrant_tool.py, tools/plot_tool.py)."""
import json

from financial_chatbot_llm_amd.retrieval import RetrievalService
from financial_chatbot_llm_amd.tools import RetrievalIntent, create_financial_plot, make_retrieval_tool
from financial_chatbot_llm_amd.tools.retrieval import date_floor, effective_limit
from helpers import seeded_store


def test_schema_fields():
    props = RetrievalIntent.model_json_schema()["properties"]
    assert set(props) == {"user_id", "num_transactions", "time_period_days", "search_query"}
    assert props["search_query"]["default"] == "recent transactions"
    assert RetrievalIntent().num_transactions is None


def test_limit_and_date_floor():
    assert effective_limit(None) == 10000 and effective_limit(7) == 7
    assert date_floor(None) is None and date_floor(0) is None
    import datetime as dt
    now = dt.datetime(2026, 1, 31, 12, 0, 0)
    assert date_floor(30, now) == int(dt.datetime(2026, 1, 1, 12, 0, 0).timestamp())


def test_missing_user_returns_empty():
    emb, store = seeded_store()
    tool = make_retrieval_tool(RetrievalService(emb, store))
    assert tool.invoke({"search_query": "grocery"}) == []
    out = tool.invoke({"search_query": "grocery purchase", "user_id": "u1"})
    assert len(out) == 3 and all(isinstance(s, str) for s in out)


def test_score_order():
    emb, store = seeded_store()
    tool = make_retrieval_tool(RetrievalService(emb, store))
    out = tool.invoke({"search_query": "Netflix subscription", "user_id": "u1"})
    assert out[0].startswith("Netflix")


def test_plot_tool_kinds():
    data = json.dumps([{"cat": "a", "amt": 1.0, "x": 1}, {"cat": "b", "amt": 2.0, "x": 2}, {"cat": "a", "amt": 3.0, "x": 3}])
    for kind in ("line", "bar", "pie", "scatter", "histogram"):
        cfg = {"plot_type": kind, "x_axis": "x", "y_axis": "amt", "title": kind, "group_by": "cat" if kind != "scatter" else None}
        out = create_financial_plot(data, cfg)
        assert out.startswith("data:image/png;base64,"), out[:80]
    assert create_financial_plot("not json", {"plot_type": "bar", "x_axis": "x", "title": "t"}).startswith("Error creating plot:")
