"""Agent routing tests with a scripted LLM (SURVEY §4 'Unit: agent')."""
import asyncio

from financial_chatbot_llm_amd.agent import LLMAgent, StubLLM, parse_tool_calls, format_tool_call
from financial_chatbot_llm_amd.agent.graph import END, StateGraph
from financial_chatbot_llm_amd.retrieval import RetrievalService
from financial_chatbot_llm_amd.tools import ToolCall, make_plot_tool, make_retrieval_tool
from financial_chatbot_llm_amd.wire import HumanMessage
from helpers import TODAY, seeded_store


def make_agent(llm, **kw):
    emb, store = seeded_store()
    tool = make_retrieval_tool(RetrievalService(emb, store))
    return LLMAgent(llm, tool, extra_tools=[make_plot_tool()], today_fn=lambda: TODAY,
                    system_prompt="SYS", tool_prompt="TOOL", **kw)


def collect(agen):
    async def run():
        return [u async for u in agen]
    return asyncio.run(run())


def test_no_tool_route():
    llm = StubLLM(decisions=[None], responses=["Hello there friend"])
    ups = collect(make_agent(llm).stream_with_status("How should I invest?", "u1", "CTX", [HumanMessage("How should I invest?")]))
    types = [u["type"] for u in ups]
    assert "retrieval_complete" not in types and types[-1] == "complete"
    assert "".join(u["content"] for u in ups if u["type"] == "response_chunk") == "Hello there friend"
    dec, resp = llm.calls
    assert dec["tools"] == ["retrieve_transactions"]  # plot tool NOT bound (llm_agent.py:38)
    assert dec["messages"][0].content == "The current date is 2026-10-15.\nTOOL\nCTX"
    assert resp["messages"][0].content == "The current date is 2026-10-15.\n\nSYS\nCTX\n"
    assert dec["temperature"] == 0.5


def test_retrieve_route_injects_user_id_and_first_call_only():
    calls = [ToolCall("retrieve_transactions", {"search_query": "grocery purchase", "user_id": "u2",
                                                "num_transactions": 5})]
    llm = StubLLM(decisions=calls, responses=["ok"])
    ups = collect(make_agent(llm).stream_with_status("What did I spend on groceries?", "u1", "CTX", []))
    rc = [u for u in ups if u["type"] == "retrieval_complete"][0]
    assert rc["count"] == 3  # only u1's rows, despite the model asking for u2
    sysmsg = llm.calls[1]["messages"][0].content
    assert "Retrieved Transaction Data:\n" in sysmsg and "Trader Joes" not in sysmsg


def test_time_filter_and_limit():
    calls = [ToolCall("retrieve_transactions", {"search_query": "grocery", "time_period_days": 7, "num_transactions": 1})]
    llm = StubLLM(decisions=calls, responses=["ok"])
    res = asyncio.run(make_agent(llm).query("groceries last week?", "u1", "CTX", []))
    txns = res["state"]["retrieved_transactions"]
    assert len(txns) == 1 and "Whole Foods" in txns[0]


def test_retrieval_error_becomes_error_string():
    calls = [ToolCall("retrieve_transactions", {"num_transactions": 0})]  # violates ge=1 -> validation error
    llm = StubLLM(decisions=calls, responses=["ok"])
    res = asyncio.run(make_agent(llm).query("spend?", "u1", "CTX", []))
    assert res["state"]["retrieved_transactions"][0].startswith("Error: ")
    assert res["retrieved_transactions_count"] == 1


def test_empty_retrieval_no_block():
    calls = [ToolCall("retrieve_transactions", {"search_query": "x"})]
    llm = StubLLM(decisions=calls, responses=["ok"])
    res = asyncio.run(make_agent(llm).query("spend?", "nobody", "CTX", []))
    assert res["retrieved_transactions_count"] == 0
    assert "Retrieved Transaction Data" not in llm.calls[1]["messages"][0].content


def test_query_graph_path():
    llm = StubLLM(responses=["graph answer"])
    res = asyncio.run(make_agent(llm).query("What did I spend on groceries?", "u1", "CTX", []))
    assert res["response"] == "graph answer" and res["retrieved_transactions_count"] > 0


def test_multi_step_with_plot():
    cfg = {"plot_type": "bar", "x_axis": "category", "y_axis": "amount", "group_by": "category", "title": "t"}
    calls = [ToolCall("retrieve_transactions", {"search_query": "grocery"}),
             ToolCall("create_financial_plot", {"plot_config": cfg}), None]
    llm = StubLLM(decisions=calls, responses=["done"])
    agent = make_agent(llm, max_tool_steps=3)
    ups = collect(agent.stream_with_status("plot my groceries", "u1", "CTX", []))
    assert sum(u["type"] == "retrieval_complete" for u in ups) == 1
    plots = [u for u in ups if u["type"] == "tool_complete"]
    assert len(plots) == 1 and plots[0]["ok"], plots
    assert set(llm.calls[0]["tools"]) == {"retrieve_transactions", "create_financial_plot"}
    # the plot saw the hits' structured columns (reference plot_tool.py:29-63), not raw text
    res = asyncio.run(make_agent(StubLLM(decisions=list(calls), responses=["done"]), max_tool_steps=3)
                      .query("plot my groceries", "u1", "CTX", []))
    plot = [r for r in res["state"]["tool_results"] if r["name"] == "create_financial_plot"][0]
    assert plot["result"].startswith("data:image/png;base64,")
    import json
    rows = json.loads(plot["args"]["transactions_json"])
    assert {"date", "amount", "category"} <= set(rows[0]) and "user_id" not in rows[0]


def test_transaction_clamp_keeps_best_scoring_rows():
    calls = [ToolCall("retrieve_transactions", {"search_query": "grocery"})]
    llm = StubLLM(decisions=calls, responses=["ok"])
    agent = make_agent(llm, max_transaction_tokens=12)     # ~1 row at len/4 tokens per row
    res = asyncio.run(agent.query("What did I spend on groceries?", "u1", "CTX", []))
    assert res["retrieved_transactions_count"] == 3
    sysmsg = llm.calls[1]["messages"][0].content
    block = sysmsg.split("Retrieved Transaction Data:\n", 1)[1]
    assert block == res["state"]["retrieved_transactions"][0]     # only the top hit fits


def test_tool_call_parser():
    tools = [make_plot_tool()]
    emb, store = seeded_store()
    tools.append(make_retrieval_tool(RetrievalService(emb, store)))
    assert parse_tool_calls("No tool call", tools) == []
    c = parse_tool_calls('<|python_tag|>{"name": "retrieve_transactions", "parameters": {"search_query": "rent"}}', tools)
    assert c[0].name == "retrieve_transactions" and c[0].args == {"search_query": "rent"}
    c = parse_tool_calls('Call tool: retrieve_transactions({"search_query": "all purchases", "time_period_days": 2})', tools)
    assert c[0].args["time_period_days"] == 2
    c = parse_tool_calls('{"name": "retrieve_transactions", "arguments": "{\\"num_transactions\\": 3}"}', tools)
    assert c[0].args == {"num_transactions": 3}
    assert parse_tool_calls('{"name": "unknown", "parameters": {}}', tools) == []
    tc = ToolCall("retrieve_transactions", {"search_query": "rent"})
    assert parse_tool_calls(format_tool_call(tc), tools)[0].args == tc.args


def test_state_graph_validation():
    g = StateGraph()
    g.add_node("a", lambda s: s + 1)
    g.set_entry_point("a")
    g.add_edge("a", END)
    assert asyncio.run(g.compile().ainvoke(1)) == 2
