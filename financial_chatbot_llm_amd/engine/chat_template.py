"""Llama-3 chat formatting of the agent's 3-part prompt and the token-budget
policy for long prompts.

The reference sends ``[system "{system_prompt}\\n{context}", *history, user "{input}"]`` to
Gemini with the tool declaration passed out-of-band.  For a local Llama-3 model the messages
are rendered with the Llama-3 header tokens; the tool declarations (JSON) go at the START of
the system turn, before the date line, so the longest possible prefix is shared by every
user's decide prompt (tools + date + TOOL_PROMPT) and respond prompt (date + SYSTEM_PROMPT):
the engine's prefix cache then serves those ~1k tokens from HBM for every turn of the day.

Token budget (:class:`ChatEncoder`).  The reference re-sends the ENTIRE history every turn
(``database.py:77``) and may stuff up to 10,000 transactions into the system turn
(``tools/qdrant_tool.py:145``, ``llm_agent.py:234-236``); an 8k-context model cannot take that.
Policy, applied in this order:

1. the agent clamps the stuffed transactions to ``max_limit_tokens`` (best-scoring first,
   ``LLMAgent.respond_messages``) -- retrieval can no longer crowd out the conversation;
2. the history is cut from the OLDEST message, in steps of ``history_quantum`` messages: the
   cut point moves once every ``quantum/2`` turns instead of every turn, so between moves the
   system+history prefix of consecutive turns is identical and the KV prefix cache keeps
   hitting (a per-turn sliding window would re-prefill the whole history every turn);
3. only if the system turn plus the query alone still overflow is the system turn's tail
   trimmed, then the query's tail; the ``<|eot_id|>`` terminators and the assistant generation
   header are never cut.

Every message is tokenised once and memoised (history messages and the per-day system turns
repeat every turn), so a turn's encode costs O(new text), not O(prompt) -- and never
O(messages x prompt) as a re-encode-per-dropped-message loop would.  Rendering pieces end and
start at special tokens, which every tokenizer here splits on first, so the concatenation of
per-piece ids equals the ids of the whole rendered prompt (tested).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

from ..agent.toolcall import render_tools_block
from ..tools.base import Tool
from ..wire import ChatMessage
from .tokenizer import BaseTokenizer

_ROLE = {"system": "system", "user": "user", "assistant": "assistant", "tool": "ipython"}
BOT = "<|begin_of_text|>"
GEN_HEADER = "<|start_header_id|>assistant<|end_header_id|>\n\n"


def _header(role: str) -> str:
    return f"<|start_header_id|>{_ROLE.get(role, role)}<|end_header_id|>\n\n"


def _content(i: int, m: ChatMessage, tools: Optional[Sequence[Tool]]) -> str:
    if i == 0 and m.role == "system" and tools:
        return "Environment: ipython\n" + render_tools_block(tools) + m.content
    return m.content


def render(messages: Sequence[ChatMessage], tools: Optional[Sequence[Tool]] = None,
           add_generation_prompt: bool = True) -> str:
    parts: List[str] = [BOT]
    for i, m in enumerate(messages):
        parts.append(f"{_header(m.role)}{_content(i, m, tools)}<|eot_id|>")
    if add_generation_prompt:
        parts.append(GEN_HEADER)
    return "".join(parts)


@dataclass
class EncodeInfo:
    """What the budget policy did to the last prompt (tests, logs, bench stats)."""
    tokens: int = 0
    dropped_messages: int = 0
    trimmed_system: int = 0      # tokens cut from the system turn's tail
    trimmed_query: int = 0


class ChatEncoder:
    """Memoising, budget-aware Llama-3 chat encoder (one per tokenizer)."""

    def __init__(self, tokenizer: BaseTokenizer, cache_size: int = 16384, history_quantum: int = 8):
        self.tok = tokenizer
        self.cache_size = cache_size
        self.history_quantum = max(1, history_quantum)
        self._cache: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
        self.last = EncodeInfo()

    def ids(self, text: str) -> Tuple[int, ...]:
        """Token ids of a rendering piece (special tokens allowed), memoised LRU."""
        hit = self._cache.get(text)
        if hit is not None:
            self._cache.move_to_end(text)
            return hit
        ids = tuple(self.tok.encode(text))
        self._cache[text] = ids
        if len(self._cache) > self.cache_size:
            self._cache.popitem(last=False)
        return ids

    def count(self, text: str) -> int:
        """Tokens of plain text (no special-token parsing); used for budget clamps."""
        return len(self.tok.encode(text, allow_special=False))

    def _piece(self, role: str, content: str) -> Tuple[Tuple[int, ...], Tuple[int, ...], Tuple[int, ...]]:
        return self.ids(_header(role)), self.ids(content), self.ids("<|eot_id|>")

    def encode(self, messages: Sequence[ChatMessage], tools: Optional[Sequence[Tool]] = None,
               max_prompt_tokens: Optional[int] = None,
               history_token_budget: Optional[int] = None) -> List[int]:
        msgs = list(messages)
        info = EncodeInfo()
        bot, gen = self.ids(BOT), self.ids(GEN_HEADER)
        pieces = [self._piece(m.role, _content(i, m, tools)) for i, m in enumerate(msgs)]
        lens = [len(h) + len(c) + len(e) for h, c, e in pieces]
        total = len(bot) + sum(lens) + len(gen)
        has_sys = bool(msgs) and msgs[0].role == "system"
        first_hist = 1 if has_sys else 0
        last_hist = len(msgs) - 1 if len(msgs) - first_hist >= 1 else len(msgs)   # final user turn kept
        hist_lens = lens[first_hist:last_hist]
        hist_total = sum(hist_lens)
        fixed = total - hist_total
        budget = hist_total
        if history_token_budget is not None:
            budget = min(budget, history_token_budget)
        if max_prompt_tokens is not None:
            budget = min(budget, max(0, max_prompt_tokens - fixed))
        start = 0
        if hist_total > budget:
            # smallest quantised cut whose suffix fits (whole history dropped in the worst case)
            suffix, s_min = hist_total, 0
            while s_min < len(hist_lens) and suffix > budget:
                suffix -= hist_lens[s_min]
                s_min += 1
            q = self.history_quantum
            start = min(len(hist_lens), -(-s_min // q) * q)
            info.dropped_messages = start
        keep = list(range(first_hist)) + list(range(first_hist + start, len(msgs)))
        out: List[int] = list(bot)
        used = len(bot) + len(gen) + sum(lens[i] for i in keep)
        over = 0 if max_prompt_tokens is None else max(0, used - max_prompt_tokens)
        for i in keep:
            h, c, e = pieces[i]
            if over and i == 0 and has_sys:
                cut = min(over, len(c))
                c = c[: len(c) - cut]
                over -= cut
                info.trimmed_system = cut
            elif over and i == len(msgs) - 1:
                cut = min(over, len(c))
                c = c[: len(c) - cut]
                over -= cut
                info.trimmed_query = cut
            out.extend(h)
            out.extend(c)
            out.extend(e)
        out.extend(gen)
        info.tokens = len(out)
        self.last = info
        return out


def encode_chat(tokenizer: BaseTokenizer, messages: Sequence[ChatMessage], tools: Optional[Sequence[Tool]] = None,
                max_prompt_tokens: Optional[int] = None, history_token_budget: Optional[int] = None) -> List[int]:
    """One-shot convenience wrapper of :meth:`ChatEncoder.encode` (no memo across calls)."""
    return ChatEncoder(tokenizer).encode(messages, tools, max_prompt_tokens, history_token_budget)


def clamp_transactions(transactions: Sequence[str], max_tokens: Optional[int], count) -> List[str]:
    """Leading (best-scoring) transactions whose joined text fits ``max_tokens`` -- counts only
    as many rows as fit, so a 10,000-hit retrieval costs O(budget), not O(hits)."""
    if max_tokens is None:
        return list(transactions)
    out: List[str] = []
    used = 0
    for t in transactions:
        n = count(t) + 1            # + the joining newline
        if used + n > max_tokens:
            break
        out.append(t)
        used += n
    return out
