"""Llama-3 chat formatting of the agent's 3-part prompt.

The reference sends ``[system "{system_prompt}\\n{context}", *history, user "{input}"]`` to
Gemini with the tool declaration passed out-of-band.  For a local Llama-3 model the messages
are rendered with the Llama-3 header tokens; the tool declarations (JSON) go at the START of
the system turn, before the date line, so the longest possible prefix is shared by every
user's decide prompt (tools + date + TOOL_PROMPT) and respond prompt (date + SYSTEM_PROMPT):
the engine's prefix cache then serves those ~1k tokens from HBM for every turn of the day.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

from ..agent.toolcall import render_tools_block
from ..tools.base import Tool
from ..wire import ChatMessage
from .tokenizer import BaseTokenizer

_ROLE = {"system": "system", "user": "user", "assistant": "assistant", "tool": "ipython"}


def render(messages: Sequence[ChatMessage], tools: Optional[Sequence[Tool]] = None,
           add_generation_prompt: bool = True) -> str:
    parts: List[str] = ["<|begin_of_text|>"]
    for i, m in enumerate(messages):
        content = m.content
        if i == 0 and m.role == "system" and tools:
            content = "Environment: ipython\n" + render_tools_block(tools) + content
        parts.append(f"<|start_header_id|>{_ROLE.get(m.role, m.role)}<|end_header_id|>\n\n{content}<|eot_id|>")
    if add_generation_prompt:
        parts.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
    return "".join(parts)


def encode_chat(tokenizer: BaseTokenizer, messages: Sequence[ChatMessage], tools: Optional[Sequence[Tool]] = None,
                max_prompt_tokens: Optional[int] = None) -> List[int]:
    """Tokenise the chat; if it exceeds ``max_prompt_tokens`` drop the OLDEST history messages
    first (system turn and the final user turn are kept), then trim the system turn's tail
    (the stuffed transactions) -- the token-budget policy of SURVEY §5.7."""
    msgs = list(messages)
    ids = tokenizer.encode(render(msgs, tools))
    if max_prompt_tokens is None or len(ids) <= max_prompt_tokens:
        return ids
    while len(msgs) > 2 and len(ids) > max_prompt_tokens:
        msgs.pop(1)
        ids = tokenizer.encode(render(msgs, tools))
    if len(ids) > max_prompt_tokens:
        sys_ids = tokenizer.encode(msgs[0].content)
        over = len(ids) - max_prompt_tokens
        keep = max(0, len(sys_ids) - over - 8)
        msgs[0] = ChatMessage("system", tokenizer.decode(sys_ids[:keep]))
        ids = tokenizer.encode(render(msgs, tools))[:max_prompt_tokens]
    return ids
