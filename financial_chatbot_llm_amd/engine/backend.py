"""Agent backend on the local engine (replaces ``ChatGoogleGenerativeAI`` chains, llm_agent.py:34-45).

* decide (``agenerate``): chat-templated prompt with the tool declarations, full generation,
  tool-call JSON parsed from the text (``agent.toolcall``).
* respond (``astream``): incremental detokenisation of the token stream into text deltas.

``decide_script`` (benchmarks / demos with random weights) supplies the decide step's text per
turn; the engine still runs every forward pass and teacher-forces those tokens (forced decoding),
so the compute matches a real model producing that output (SURVEY §6 'scripted tool decision').

Decide outputs follow the tool-call grammar (``agent.grammar``): tokens the grammar forces (the
JSON skeleton, the tool name, unambiguous keys, the closing braces) are appended without
sampling and computed as one chunk (jump-forward decoding) -- for scripted and sampled outputs
alike; ``jump_forward=False`` decodes them one step each.

Decide calls also decode with prompt-lookup speculation (``engine.speculative``, up to
``prompt_lookup`` draft tokens per step): a tool call's arguments mostly copy the user's words.

``ephemeral_kv`` (agent hint): the prompt carries this turn's tool results, which the next turn
will not repeat, so its freshly computed KV blocks are recycled before any other cached prefix
(``PyBlockManager.free``) -- the conversation prefixes that DO recur survive in HBM.
"""
from __future__ import annotations

import os
from typing import AsyncIterator, Callable, Optional, Sequence

from ..agent.grammar import ToolCallGrammar, jump_mask
from ..agent.llm import LLMBackend, LLMResult
from ..agent.toolcall import parse_tool_calls
from ..tools.base import Tool
from ..utils.profiling import marker
from ..wire import ChatMessage
from .async_engine import AsyncEngine
from .chat_template import ChatEncoder
from .sequence import TURN_START, SamplingParams
from .tokenizer import IncrementalDetokenizer


class EngineLLM(LLMBackend):
    def __init__(self, engine: AsyncEngine, max_model_len: int = 8192,
                 decide_script: Optional[Callable[[Sequence[ChatMessage], Sequence[Tool]], str]] = None,
                 respond_ignore_eos: bool = False, respond_tokens: Optional[int] = None,
                 stream_chunk_tokens: int = 1, history_token_budget: Optional[int] = None,
                 jump_forward: bool = True, prompt_lookup: Optional[int] = None):
        self.engine = engine
        self.tok = engine.tokenizer
        self.encoder = ChatEncoder(self.tok)
        self.max_model_len = max_model_len
        self.history_token_budget = history_token_budget
        self.jump_forward = jump_forward
        self.prompt_lookup = (int(os.environ.get("PENNY_PROMPT_LOOKUP", "8")) if prompt_lookup is None
                              else prompt_lookup)
        self.decide_script = decide_script
        self.respond_ignore_eos = respond_ignore_eos
        self.respond_tokens = respond_tokens
        self.stream_chunk_tokens = max(1, stream_chunk_tokens)
        self.eot = self.tok.special.get("<|eot_id|>")
        self.last_prompt_tokens = 0
        # per-purpose prompt accounting: calls, prompt tokens, tokens actually prefilled
        # (prompt - prefix-cache hits + preemption recomputes), generated tokens
        self.token_stats = {p: {"calls": 0, "prompt": 0, "prefilled": 0, "generated": 0}
                            for p in ("decide", "respond")}
        # engine-side latency anatomy per call (seconds): queued before admission, admission to the
        # first sampled token, and arrival to the last token
        self.latency = {p: {"queue": [], "to_first": [], "total": []} for p in ("decide", "respond")}

    def _account(self, purpose: str, prompt_len: int, seq) -> None:
        st = self.token_stats.setdefault(purpose, {"calls": 0, "prompt": 0, "prefilled": 0, "generated": 0})
        st["calls"] += 1
        st["prompt"] += prompt_len
        # prefill chunks also cover forced tokens appended after the prompt (jump-forward)
        st["prefilled"] += min(getattr(seq, "num_prefilled", 0), prompt_len)
        st["generated"] += len(seq.output_ids)
        lat = self.latency.setdefault(purpose, {"queue": [], "to_first": [], "total": []})
        import time as _t
        if getattr(seq, "admit_time", None) is not None:
            lat["queue"].append(seq.admit_time - seq.arrival)
            if seq.first_token_time is not None:
                lat["to_first"].append(seq.first_token_time - seq.admit_time)
        lat["total"].append(_t.perf_counter() - seq.arrival)

    def count_tokens(self, text: str) -> int:
        return self.encoder.count(text)

    def _encode(self, messages, tools, max_tokens) -> list:
        with marker("serve.encode"):
            ids = self.encoder.encode(messages, tools, max_prompt_tokens=self.max_model_len - max_tokens - 1,
                                      history_token_budget=self.history_token_budget)
        self.last_prompt_tokens = len(ids)
        return ids

    async def agenerate(self, messages, tools=None, temperature=0.5, max_tokens=256, **kw) -> LLMResult:
        tools = list(tools or [])
        ids = self._encode(messages, tools, max_tokens)
        forced = jump = None
        grammar = ToolCallGrammar(tools) if (tools and self.jump_forward) else None
        if self.decide_script is not None:
            text = self.decide_script(messages, tools)
            forced = self.tok.encode(text, allow_special=False)[: max_tokens - 1] + ([self.eot] if self.eot is not None else [])
            if grammar is not None:
                jump = jump_mask(forced, self.tok.decode, grammar, self.eot)
        params = SamplingParams(temperature=temperature, max_tokens=max_tokens, forced_output=forced,
                                forced_jump=jump, grammar=grammar, ephemeral_kv=bool(kw.get("ephemeral_kv")),
                                prompt_lookup=self.prompt_lookup, priority_ts=TURN_START.get())
        out = await self.engine.generate_all(ids, params)
        self._account(kw.get("purpose", "decide"), len(ids), out.seq)
        text = self.tok.decode(out.seq.output_ids)
        return LLMResult(text=text, tool_calls=parse_tool_calls(text, tools), prompt_tokens=len(ids),
                         completion_tokens=len(out.seq.output_ids))

    async def astream(self, messages, temperature=0.5, max_tokens=512, **kw) -> AsyncIterator[str]:
        n = self.respond_tokens or max_tokens
        ids = self._encode(messages, None, n)
        params = SamplingParams(temperature=temperature, max_tokens=n, ignore_eos=self.respond_ignore_eos,
                                ephemeral_kv=bool(kw.get("ephemeral_kv")), priority_ts=TURN_START.get())
        detok = IncrementalDetokenizer(self.tok)
        buf, k = [], 0
        async for o in self.engine.generate(ids, params):
            buf.append(detok.push(o.new_token_ids))
            k += 1
            if o.finished:
                self._account(kw.get("purpose", "respond"), len(ids), o.seq)
            if k % self.stream_chunk_tokens == 0 or o.finished:
                text = "".join(buf)
                buf = []
                if text:
                    yield text
        tail = detok.flush()
        if tail:
            yield tail
