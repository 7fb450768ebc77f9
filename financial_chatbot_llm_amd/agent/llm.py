"""LLM backend protocol (replaces the LangChain ``prompt | ChatGoogleGenerativeAI`` chains).

Reference call sites: ``llm_agent.py:87-93`` (non-streaming decide call with the tool bound)
and ``llm_agent.py:243-250`` (streaming respond call).  Both become methods of an
:class:`LLMBackend`:

* ``agenerate(messages, tools, temperature, max_tokens)`` -> :class:`LLMResult` (text + parsed
  tool calls), used for the decide step;
* ``astream(messages, temperature, max_tokens)`` -> async iterator of text deltas, used for
  the respond step.

:class:`StubLLM` is the scripted backend of north-star config 1 (CPU plumbing, tests): it
emits a tool call or ``No tool call`` on cue and streams canned text.  The GPU engine backend
lives in ``engine.backend.EngineLLM``.
"""
from __future__ import annotations

import asyncio
import re
from dataclasses import dataclass, field
from typing import Any, AsyncIterator, Callable, Dict, List, Optional, Sequence

from ..tools.base import Tool, ToolCall
from ..wire import ChatMessage


@dataclass
class LLMResult:
    text: str = ""
    tool_calls: List[ToolCall] = field(default_factory=list)
    prompt_tokens: int = 0
    completion_tokens: int = 0


class LLMBackend:
    async def agenerate(self, messages: Sequence[ChatMessage], tools: Optional[Sequence[Tool]] = None,
                        temperature: float = 0.5, max_tokens: int = 256, **kw) -> LLMResult:
        raise NotImplementedError

    def astream(self, messages: Sequence[ChatMessage], temperature: float = 0.5,
                max_tokens: int = 512, **kw) -> AsyncIterator[str]:
        raise NotImplementedError

    def count_tokens(self, text: str) -> int:
        """Prompt-budget estimate of ``text`` (backends with a tokenizer count exactly)."""
        return len(text) // 4 + 1


_RETRIEVAL_CUES = re.compile(
    r"\b(spen[dt]|spending|transactions?|purchases?|bought|paid|charges?|groceries|grocery|"
    r"subscriptions?|expenses?|bills?|merchant|last (week|month)|yesterday|days? ago)\b", re.I)
_DAYS = re.compile(r"\b(\d+|one|two|three|four|five|six|seven|eight|nine|ten|fourteen|thirty)\s+days?\b", re.I)
_NUM_WORDS = {"one": 1, "two": 2, "three": 3, "four": 4, "five": 5, "six": 6, "seven": 7, "eight": 8, "nine": 9,
              "ten": 10, "fourteen": 14, "thirty": 30}


def scripted_decision(user_query: str, always_limit: bool = False) -> Optional[ToolCall]:
    """Heuristic tool decision mirroring the few-shot of ``tool_prompt.txt`` (reference
    ``tool_prompt.txt:15-23``): a topical query carries ``num_transactions: 20``; a time-window
    query ("two days ago") carries ``time_period_days`` and NO ``num_transactions``, so the tool's
    limit falls back to 10000 (``tools/qdrant_tool.py:145``) and the agent's transaction-token
    clamp decides how much of the window reaches the respond prompt.  ``always_limit=True`` keeps
    ``num_transactions: 20`` on every call (the round-2 benchmark workload)."""
    if not _RETRIEVAL_CUES.search(user_query):
        return None
    args: Dict[str, Any] = {"search_query": user_query.strip().rstrip("?.!") or "recent transactions"}
    m = _DAYS.search(user_query)
    low = user_query.lower()
    days = None
    if m:
        w = m.group(1).lower()
        days = int(w) if w.isdigit() else _NUM_WORDS[w]
    elif "yesterday" in low:
        days = 1
    elif "last week" in low:
        days = 7
    elif "last month" in low:
        days = 30
    if days is None or always_limit:
        args["num_transactions"] = 20
    if days is not None:
        args["time_period_days"] = days
    return ToolCall(name="retrieve_transactions", args=args, id="call_0")


class StubLLM(LLMBackend):
    """Scripted backend.  ``decisions``/``responses`` queues override the heuristics."""

    def __init__(self, decisions: Optional[List[Optional[ToolCall]]] = None,
                 responses: Optional[List[str]] = None, chunk_words: int = 3,
                 stream_delay_s: float = 0.0, fail_stream: bool = False, fail_generate: bool = False,
                 decide_delay_s: float = 0.0):
        self.decisions = list(decisions) if decisions is not None else None
        self.responses = list(responses) if responses is not None else None
        self.chunk_words = chunk_words
        self.stream_delay_s = stream_delay_s
        self.decide_delay_s = decide_delay_s
        self.fail_stream, self.fail_generate = fail_stream, fail_generate
        self.calls: List[Dict[str, Any]] = []

    async def agenerate(self, messages, tools=None, temperature=0.5, max_tokens=256, **kw) -> LLMResult:
        self.calls.append({"kind": "generate", "messages": list(messages),
                           "tools": [t.name for t in (tools or [])], "temperature": temperature})
        if self.decide_delay_s:
            await asyncio.sleep(self.decide_delay_s)
        if self.fail_generate:
            raise RuntimeError("injected generate failure")
        tool_names = {t.name for t in (tools or [])}
        if self.decisions is not None and self.decisions:
            tc = self.decisions.pop(0)
        else:
            tc = scripted_decision(messages[-1].content) if messages else None
        if tc is not None and tc.name in tool_names:
            return LLMResult(text="", tool_calls=[tc])
        return LLMResult(text="No tool call")

    async def astream(self, messages, temperature=0.5, max_tokens=512, **kw) -> AsyncIterator[str]:
        self.calls.append({"kind": "stream", "messages": list(messages), "temperature": temperature})
        if self.responses:
            text = self.responses.pop(0)
        else:
            sys = messages[0].content if messages else ""
            n = sys.split("Retrieved Transaction Data:\n", 1)
            k = len(n[1].splitlines()) if len(n) > 1 else 0
            text = (f"Thanks for the question! I looked at {k} of your transactions. "
                    "Here is a plan tailored to your situation.")
        words = text.split(" ")
        for i in range(0, len(words), self.chunk_words):
            if self.fail_stream and i > 0:
                raise RuntimeError("injected stream failure")
            if self.stream_delay_s:
                await asyncio.sleep(self.stream_delay_s)
            piece = " ".join(words[i:i + self.chunk_words])
            yield piece if i + self.chunk_words >= len(words) else piece + " "
