"""The Penny tool-calling agent (reference ``llm_agent.py:21-253``).

Same three steps and routing as the reference:

1. **decide** (``llm_agent.py:81-106``): one non-streaming generation over
   ``["The current date is D.\\n" + TOOL_PROMPT + "\\n" + context, *history, query]`` with the
   retrieval tool bound; only ``tool_calls[0]`` is kept.
2. **retrieve** (``llm_agent.py:108-133``): pops the call, **overwrites ``user_id`` with the
   server-side id**, runs the tool; an exception becomes ``["Error: ..."]``.
3. **respond** (``llm_agent.py:135-158`` / ``:234-250``): context + optional
   ``"Retrieved Transaction Data:\\n"`` block, system ``"The current date is D.\\n\\n" +
   SYSTEM_PROMPT``; streamed in ``stream_with_status``.

Differences by design (SURVEY §3.2 hazards): every step is ``async`` -- the decide call and
the tool no longer block the event loop, so concurrent turns batch inside the GPU engine.
``max_tool_steps > 1`` enables the multi-step agent of north-star config 4 (retrieval +
plotting, tool results fed back before the final answer).
"""
from __future__ import annotations

import datetime as _dt
import json
from collections import deque
from typing import Any, AsyncGenerator, Callable, Deque, Dict, List, Literal, Optional, Sequence, TypedDict

from .. import config
from ..prompts import system_prompt as _load_system_prompt, tool_prompt as _load_tool_prompt
from ..tools.base import Tool, ToolCall
from ..utils.logging import get_logger
from ..wire import ChatMessage, build_messages, decide_system_prompt, respond_context, respond_system_prompt
from .graph import END, StateGraph
from .llm import LLMBackend

logger = get_logger(__name__)


class AgentState(TypedDict):
    user_query: str
    user_id: str
    user_context: str
    chat_history: List[ChatMessage]
    tool_calls: Deque[ToolCall]
    retrieved_transactions: List[str]
    final_response: Optional[str]
    tool_results: List[Dict[str, Any]]
    transaction_records: List[Dict[str, Any]]   # structured rows of the hits (plot tool input)


def initial_state(user_query: str, user_id: str, user_context: str, chat_history: Sequence[ChatMessage]) -> AgentState:
    return {"user_query": user_query, "user_id": user_id, "tool_calls": deque(),
            "user_context": user_context, "chat_history": list(chat_history),
            "retrieved_transactions": [], "final_response": None, "tool_results": [],
            "transaction_records": []}


class LLMAgent:
    def __init__(self, llm: LLMBackend, retrieval_tool: Tool, extra_tools: Sequence[Tool] = (),
                 temperature: float = config.DEFAULT_TEMPERATURE, max_response_tokens: int = 512,
                 max_decide_tokens: int = 160, max_tool_steps: int = 1,
                 today_fn: Callable[[], _dt.date] = _dt.date.today,
                 system_prompt: Optional[str] = None, tool_prompt: Optional[str] = None,
                 max_transaction_tokens: Optional[int] = config.MAX_TRANSACTION_TOKENS):
        self.llm = llm
        self.retrieval_tool = retrieval_tool
        self.tools: Dict[str, Tool] = {retrieval_tool.name: retrieval_tool}
        for t in extra_tools:
            self.tools[t.name] = t
        # Reference binds ONLY the retrieval tool (llm_agent.py:38); extra tools only bind in
        # multi-step mode.
        self.bound_tools: List[Tool] = list(self.tools.values()) if max_tool_steps > 1 else [retrieval_tool]
        self.temperature = temperature
        self.max_response_tokens = max_response_tokens
        self.max_decide_tokens = max_decide_tokens
        self.max_tool_steps = max_tool_steps
        self.max_transaction_tokens = max_transaction_tokens
        self.today_fn = today_fn
        self.system_prompt = system_prompt if system_prompt is not None else _load_system_prompt()
        self.tool_prompt = tool_prompt if tool_prompt is not None else _load_tool_prompt()
        self.graph = self._build_graph()
        logger.info("Agent initialized with state graph")

    # -- graph ----------------------------------------------------------------------------
    def _build_graph(self):
        g = StateGraph()
        g.add_node("decide_retrieval", self._decide_retrieval_node)
        g.add_node("retrieve_data", self._retrieve_data_node)
        g.add_node("generate_response", self._generate_response_node)
        g.set_entry_point("decide_retrieval")
        g.add_conditional_edges("decide_retrieval", self._should_retrieve,
                                {"retrieve": "retrieve_data", "respond": "generate_response"})
        if self.max_tool_steps > 1:   # multi-step agent: tool results go back to the decider
            g.add_conditional_edges("retrieve_data", self._after_tool,
                                    {"decide": "decide_retrieval", "respond": "generate_response"})
        else:
            g.add_edge("retrieve_data", "generate_response")
        g.add_edge("generate_response", END)
        return g.compile()

    def decide_messages(self, state: AgentState) -> List[ChatMessage]:
        sp = decide_system_prompt(self.tool_prompt, self.today_fn())
        ctx = state["user_context"]
        if state["tool_results"]:
            ctx = ctx + "\n" + "\n".join(self._tool_result_lines(state))
        return build_messages(sp, ctx, state["chat_history"], state["user_query"])

    def respond_messages(self, state: AgentState) -> List[ChatMessage]:
        # token-budget step 1: the reference stuffs up to 10,000 hits
        # (qdrant_tool.py:145, llm_agent.py:234-236); keep the best-scoring ones that fit
        from ..engine.chat_template import clamp_transactions
        txns = clamp_transactions(state["retrieved_transactions"], self.max_transaction_tokens,
                                  self.llm.count_tokens)
        if len(txns) < len(state["retrieved_transactions"]):
            logger.info(f"Clamped {len(state['retrieved_transactions'])} transactions to {len(txns)} "
                        f"({self.max_transaction_tokens} tokens)")
        ctx = respond_context(state["user_context"], txns)
        if len(state["tool_results"]) > 1 or any(r["name"] != self.retrieval_tool.name for r in state["tool_results"]):
            extra = [l for l in self._tool_result_lines(state) if not l.startswith("[retrieve_transactions]")]
            if extra:
                ctx += "\n" + "\n".join(extra)
        sp = respond_system_prompt(self.system_prompt, self.today_fn())
        return build_messages(sp, ctx, state["chat_history"], state["user_query"])

    @staticmethod
    def _tool_result_lines(state: AgentState) -> List[str]:
        out = []
        for r in state["tool_results"]:
            res = r["result"]
            if isinstance(res, str) and res.startswith("data:image/png;base64,"):
                res = f"<plot image generated, {len(res)} bytes>"
            elif isinstance(res, list):
                res = f"{len(res)} transactions retrieved"
            out.append(f"[{r['name']}] {res}")
        return out

    async def _decide_retrieval_node(self, state: AgentState) -> AgentState:
        logger.info("Deciding if transaction retrieval is needed")
        result = await self.llm.agenerate(self.decide_messages(state), tools=self.bound_tools,
                                          temperature=self.temperature, max_tokens=self.max_decide_tokens,
                                          purpose="decide", ephemeral_kv=bool(state["tool_results"]))
        logger.info(f"Decide Retrieval Response: {result.text!r} tool_calls={[t.to_dict() for t in result.tool_calls]}")
        if result.tool_calls:
            tc = result.tool_calls[0]  # only the first call is honoured (llm_agent.py:100)
            state["tool_calls"].append(tc)
            logger.info(f"LLM requested retrieval with args: {tc.args}")
        else:
            logger.info("LLM decided no retrieval needed")
        return state

    async def _retrieve_data_node(self, state: AgentState) -> AgentState:
        logger.info("Retrieving transaction data")
        if len(state["tool_calls"]) == 0:
            return state
        try:
            tc = state["tool_calls"].popleft()
            tool = self.tools.get(tc.name)
            if tool is None:
                raise KeyError(f"unknown tool {tc.name}")
            args = dict(tc.args)
            if tool is self.retrieval_tool:
                args["user_id"] = state["user_id"]   # server-side id always wins (llm_agent.py:120)
            elif tc.name == "create_financial_plot" and "transactions_json" not in args:
                # the reference tool plots a transactions JSON with real columns
                # (plot_tool.py:29-63): hand it the structured rows of the retrieval hits
                args["transactions_json"] = json.dumps(state.get("transaction_records") or [])
            result = await tool.ainvoke(args)
            state["tool_results"].append({"name": tc.name, "args": args, "result": result})
            if tool is self.retrieval_tool:
                state["retrieved_transactions"] = list(result)
                state["transaction_records"] = list(getattr(result, "records", []) or [])
                logger.info(f"Retrieved {len(result)} transactions")
        except Exception as e:  # noqa: BLE001
            logger.error(f"Error retrieving transactions: {e}")
            state["retrieved_transactions"] = [f"Error: {e}"]
        return state

    async def _generate_response_node(self, state: AgentState) -> AgentState:
        logger.info("Generating final response")
        parts = []
        async for piece in self.llm.astream(self.respond_messages(state), temperature=self.temperature,
                                            max_tokens=self.max_response_tokens, purpose="respond",
                                            ephemeral_kv=bool(state["tool_results"])):
            parts.append(piece)
        state["final_response"] = "".join(parts)
        logger.info("Final response generated")
        return state

    def _after_tool(self, state: AgentState) -> Literal["decide", "respond"]:
        return "decide" if len(state["tool_results"]) < self.max_tool_steps else "respond"

    def _should_retrieve(self, state: AgentState) -> Literal["retrieve", "respond"]:
        if len(state["tool_calls"]) > 0:
            logger.info("Routing to retrieve_data")
            return "retrieve"
        logger.info("Routing to generate_response")
        return "respond"

    # -- public API -----------------------------------------------------------------------
    async def query(self, user_query: str, user_id: str, user_context: str = "",
                    chat_history: Sequence[ChatMessage] = ()) -> Dict[str, Any]:
        """Non-streaming graph run (``llm_agent.py:175-200``)."""
        logger.info(f"Processing query for user {user_id}: {user_query}")
        final = await self.graph.ainvoke(initial_state(user_query, user_id, user_context, chat_history))
        return {"response": final["final_response"],
                "retrieved_transactions_count": len(final["retrieved_transactions"]),
                "state": final}

    async def stream_with_status(self, user_query: str, user_id: str, user_context: str = "",
                                 chat_history: Sequence[ChatMessage] = ()) -> AsyncGenerator[Dict[str, Any], None]:
        """Live path (``llm_agent.py:202-253``): status events, chunks, then ``complete``."""
        logger.info(f"Processing query with status streaming for user {user_id}: {user_query}")
        yield {"type": "status", "message": "Starting query processing..."}
        state = initial_state(user_query, user_id, user_context, chat_history)
        yield {"type": "status", "message": "Analyzing query to determine if transaction data is needed..."}
        state = await self._decide_retrieval_node(state)
        steps = 0
        retrieved_any = False
        while self._should_retrieve(state) == "retrieve" and steps < self.max_tool_steps:
            yield {"type": "status", "message": "Retrieving relevant transaction data..."}
            n_results = len(state["tool_results"])
            state = await self._retrieve_data_node(state)
            steps += 1
            retrieved_any = True
            last = state["tool_results"][-1] if len(state["tool_results"]) > n_results else None
            if last is not None and last["name"] != self.retrieval_tool.name:
                res = last["result"]
                ok = isinstance(res, str) and res.startswith("data:image/png;base64,")
                yield {"type": "tool_complete", "name": last["name"], "ok": ok,
                       "message": f"{last['name']} {'succeeded' if ok else 'failed'}"}
            else:
                n = len(state["retrieved_transactions"])
                yield {"type": "retrieval_complete", "count": n, "message": f"Retrieved {n} transactions"}
            if steps < self.max_tool_steps:
                state = await self._decide_retrieval_node(state)
        if not retrieved_any:
            yield {"type": "status", "message": "No transaction data retrieval needed"}
        yield {"type": "status", "message": "Generating response..."}
        async for piece in self.llm.astream(self.respond_messages(state), temperature=self.temperature,
                                            max_tokens=self.max_response_tokens, purpose="respond",
                                            ephemeral_kv=bool(state["tool_results"])):
            if piece:
                yield {"type": "response_chunk", "content": piece}
        yield {"type": "complete", "message": "Query processing completed"}
        logger.info("Status streaming completed")
