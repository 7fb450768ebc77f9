"""Synthetic RAG chat workload driven through the FULL serving path.

One "step" = one wave of ``C`` concurrent chat turns (one per synthetic conversation):

    user message -> Mongo (history) + Kafka ``user_message``
      -> ChatWorker.process_message -> LLMAgent
           decide  : Llama-3 generation over the tool prompt (tool call teacher-forced: random
                     weights cannot emit valid JSON), prefix-cached
           retrieve: bge-base-en query embedding (GPU) + filtered top-k over a 1M-vector
                     HBM corpus (HIP K15)                          [every other turn]
           respond : streamed Llama-3 generation, fixed length (ignore EOS)
      -> Kafka ``ai_response`` chunks + complete, reply saved to Mongo

Turns/s counts completed turns (``complete`` event); TTFT is receipt -> first
``response_chunk`` (SURVEY §6 metric definitions).
"""
from __future__ import annotations

import asyncio
import datetime as _dt
import json
import os
import random
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .. import config
from ..adapters import Database, InMemoryBroker, KafkaClient
from ..agent import LLMAgent, LLMService, scripted_decision
from ..agent.toolcall import format_tool_call
from ..retrieval import RetrievalService
from ..retrieval.store import MERCHANTS, user_name
from ..serving.worker import ChatWorker
from ..tools import make_plot_tool, make_retrieval_tool
from ..tools.base import ToolCall

ADVICE_QUESTIONS = [
    "How should I invest for retirement given my income?",
    "Should I pay off my student loans faster or invest more?",
    "How big should my emergency fund be?",
    "Can you help me build a monthly budget plan?",
    "Is it a good idea to open a Roth IRA this year?",
]
SPEND_QUESTIONS = [
    "What did I spend on groceries last month?",
    "How much did I spend on dining in the last 30 days?",
    "Show me my recent transactions at Amazon.",
    "How much did I spend two days ago?",
    "What were my biggest purchases last week?",
]


def context_doc(i: int, user: str, rng: random.Random) -> Dict:
    accounts = [{"account_id": f"acc-{i}-{k}", "balances": {"available": None, "current": round(rng.uniform(100, 20000), 2),
                                                           "limit": None, "iso_currency_code": "USD"},
                 "mask": f"{rng.randint(1000, 9999)}", "name": n, "official_name": n, "subtype": s, "type": t}
                for k, (n, s, t) in enumerate([("Plaid Checking", "checking", "depository"),
                                               ("Plaid Saving", "savings", "depository"),
                                               ("Plaid Credit Card", "credit card", "credit")])]
    expenses = [{"name": n, "amount": a, "description": d} for n, a, d in
                [("Rent", rng.randint(1200, 3500), "apartment"), ("Car payment", rng.randint(200, 600), ""),
                 ("Gym", 45, ""), ("Phone", 70, "family plan")]]
    return {"conversation_id": f"conv-{i:05d}", "user_id": user, "name": f"User {i}",
            "income": rng.randint(3000, 15000), "savings_goal": rng.randint(200, 3000),
            "accounts": accounts, "additional_monthly_expenses": expenses}


@dataclass
class WaveResult:
    seconds: float
    ttfts: List[float]
    turns: int
    errors: int
    retrievals: int
    stages: Dict[str, List[float]] = field(default_factory=dict)   # TTFT anatomy per turn (s)
    plots_ok: int = 0
    plots_failed: int = 0


class RagWorkload:
    """Owns the fakes, the worker and the synthetic conversations for one GPU replica."""

    def __init__(self, llm, retrieval: RetrievalService, num_convs: int, num_users: int,
                 respond_tokens: int, seed: int = 0, rank: int = 0, max_tool_steps: int = 1,
                 tools: bool = True):
        self.rng = random.Random(seed * 7919 + rank)
        self.progress = None       # callable(str): heartbeat for long runs
        self.broker = InMemoryBroker(num_partitions=16)
        self.db = Database(uri="")
        self.kafka = KafkaClient(broker=self.broker)
        if tools:
            self.agent = LLMAgent(llm, make_retrieval_tool(retrieval), extra_tools=[make_plot_tool()],
                                  max_response_tokens=respond_tokens, max_tool_steps=max_tool_steps)
        else:   # BASELINE config 2: legacy single-chain chat (llm_service.py), no decide/retrieval
            self.agent = LLMService(llm, max_response_tokens=respond_tokens)
        self.worker = ChatWorker(self.db, self.kafka, self.agent, max_concurrent_turns=4 * num_convs)
        self.convs = []
        for i in range(num_convs):
            uid = user_name(self.rng.randrange(num_users))
            doc = context_doc(rank * 100000 + i, uid, self.rng)
            self.db.put_context(doc)
            self.convs.append(doc)
        self.turn_of = [0] * num_convs            # next turn index per conversation
        self.conv_index = {d["conversation_id"]: i for i, d in enumerate(self.convs)}

    def _send(self, i: int) -> None:
        """Conversation i's next user message (spend / advice questions alternate per turn)."""
        doc, k = self.convs[i], self.turn_of[i]
        pool = SPEND_QUESTIONS if (i + k) % 2 == 0 else ADVICE_QUESTIONS
        text = pool[(i // 2 + k) % len(pool)]
        # wall-clock seconds, like the AI replies saved by the worker (database.py:100): history is
        # sorted by timestamp (database.py:77), so a synthetic clock would misorder the two senders
        self.db.put_user_message(doc["conversation_id"], text, doc["user_id"], int(time.time()))
        self.kafka.producer.produce(config.USER_MESSAGE_TOPIC, key=doc["conversation_id"],
                                    value=json.dumps({"message": text, "conversation_id": doc["conversation_id"],
                                                      "user_id": doc["user_id"]}))
        self.turn_of[i] += 1

    async def _send_wave(self) -> None:
        for i in range(len(self.convs)):
            self._send(i)

    async def run_closed_loop(self, turns_per_conv: int) -> WaveResult:
        """Closed-loop load: every conversation is an independent client that sends its next
        message as soon as its previous turn completes (no cross-conversation lock-step, so no
        synchronised arrival bursts and no end-of-wave tail per turn).  Returns after every
        conversation completed ``turns_per_conv`` turns."""
        n0 = len(self.worker.traces)
        t0 = time.perf_counter()
        left = [turns_per_conv - 1] * len(self.convs)
        for i in range(len(self.convs)):
            self._send(i)
        seen, target = n0, n0 + turns_per_conv * len(self.convs)
        t_log = t0
        while seen < target:
            await asyncio.sleep(0.002)
            if self.progress is not None and time.perf_counter() - t_log > 30:
                t_log = time.perf_counter()
                self.progress(f"closed loop: {seen - n0}/{target - n0} turns in {t_log - t0:.0f}s")
            new = self.worker.traces[seen:]
            seen += len(new)
            for tr in new:
                i = self.conv_index[tr.conversation_id]
                if left[i] > 0:
                    left[i] -= 1
                    self._send(i)
        dt = time.perf_counter() - t0
        traces = self.worker.traces[n0:target]
        return _result(dt, traces)

    async def run_wave(self) -> WaveResult:
        n0 = len(self.worker.traces)
        t0 = time.perf_counter()
        await self._send_wave()
        target = n0 + len(self.convs)
        while len(self.worker.traces) < target:
            await asyncio.sleep(0.002)
        dt = time.perf_counter() - t0
        traces = self.worker.traces[n0:target]
        return _result(dt, traces)


def _result(dt: float, traces) -> WaveResult:
    return WaveResult(dt, [t.ttft for t in traces if t.ttft is not None], len(traces),
                      sum(t.error for t in traces), sum(t.retrieved > 0 for t in traces), ttft_stages(traces),
                      plots_ok=sum(t.tools_ok for t in traces), plots_failed=sum(t.tools_failed for t in traces))


def ttft_stages(traces) -> Dict[str, List[float]]:
    """Split each turn's TTFT: receive -> decide done (context fetch + LLM call 1), decide done ->
    respond start (retrieval, when taken), respond start -> first chunk (LLM call 2 prefill)."""
    out: Dict[str, List[float]] = {"decide": [], "retrieval": [], "respond_first_token": []}
    for t in traces:
        st = t.stages
        if "decide_done" in st:
            out["decide"].append(st["decide_done"] - t.t_receive)
            if "respond_start" in st:
                out["retrieval"].append(st["respond_start"] - st["decide_done"])
        if "respond_start" in st and t.t_first_chunk is not None:
            out["respond_first_token"].append(t.t_first_chunk - st["respond_start"])
    return out


# spending per category over the retrieved rows (the retrieval tool hands the plot tool the
# hits' structured columns: date, amount, merchant, category)
PLOT_CALL = ToolCall("create_financial_plot", {"plot_config": {"plot_type": "bar", "x_axis": "category",
                                                                "y_axis": "amount", "group_by": "category",
                                                                "title": "Spending by category"}})


def decide_script(messages, tools) -> str:
    """Scripted decision for random-weight benchmarking: the reference's few-shot rule set.

    Multi-step agent (plot tool bound, north-star config 4): once transactions were retrieved the
    next decision plots them, after the plot it answers."""
    names = {t.name for t in tools}
    system = messages[0].content if messages else ""
    if "[retrieve_transactions]" in system:
        nothing = "[retrieve_transactions] 0 transactions retrieved" in system   # nothing to plot
        if PLOT_CALL.name in names and f"[{PLOT_CALL.name}]" not in system and not nothing:
            return format_tool_call(PLOT_CALL)
        return "No tool call"
    # PENNY_DECIDE_ALWAYS_LIMIT=1 (bench.py --decide-always-limit): num_transactions on every call,
    # the round-2 workload; default: the reference few-shot (time windows carry no limit)
    always = os.environ.get("PENNY_DECIDE_ALWAYS_LIMIT", "0") == "1"
    call = scripted_decision(messages[-1].content, always_limit=always) if messages else None
    if call is None or not any(t.name == call.name for t in tools):
        return "No tool call"
    return format_tool_call(call)
