"""Tool-call rendering and parsing for a local Llama-3-family model.

Gemini receives the ``retrieve_transactions`` declaration out-of-band (``llm_agent.py:38``).
A local Llama-3.1-style model gets the JSON declarations in its prompt and answers with a
JSON object ``{"name": ..., "parameters": {...}}`` (optionally behind ``<|python_tag|>``).
The parser also accepts ``"arguments"`` instead of ``"parameters"``, a list of such objects,
and the call syntax of the reference's few-shot examples
(``retrieve_transactions({"search_query": ...})``, ``tool_prompt.txt:17-20``).  Anything else
-- including the literal ``No tool call`` -- yields no calls.
"""
from __future__ import annotations

import json
import re
from typing import Any, Dict, Iterable, List, Optional, Sequence

from ..tools.base import Tool, ToolCall

TOOL_INSTRUCTIONS = (
    "Given the following functions, respond with a JSON for a function call with its proper arguments "
    "that best answers the given prompt.\n"
    'Respond in the format {"name": function name, "parameters": dictionary of argument name and its value}. '
    "Do not use variables.\n\n"
)

_CALL_SYNTAX = re.compile(r"([A-Za-z_][A-Za-z0-9_]*)\s*\(\s*(\{.*\})\s*\)", re.S)


def render_tools_block(tools: Sequence[Tool]) -> str:
    return TOOL_INSTRUCTIONS + "\n\n".join(json.dumps(t.function_declaration(), indent=4) for t in tools) + "\n\n"


def _first_json_value(text: str) -> Optional[Any]:
    dec = json.JSONDecoder()
    for i, ch in enumerate(text):
        if ch in "{[":
            try:
                val, _ = dec.raw_decode(text[i:])
                return val
            except json.JSONDecodeError:
                continue
    return None


def _as_call(obj: Any, names: Iterable[str], idx: int) -> Optional[ToolCall]:
    if not isinstance(obj, dict):
        return None
    if "function" in obj and isinstance(obj["function"], dict):
        obj = obj["function"]
    name = obj.get("name")
    args = obj.get("parameters", obj.get("arguments", {}))
    if isinstance(args, str):
        try:
            args = json.loads(args)
        except json.JSONDecodeError:
            return None
    if not isinstance(name, str) or name not in names or not isinstance(args, dict):
        return None
    return ToolCall(name=name, args=args, id=f"call_{idx}")


def parse_tool_calls(text: str, tools: Sequence[Tool]) -> List[ToolCall]:
    names = {t.name for t in tools}
    if not text or not names:
        return []
    body = text.replace("<|python_tag|>", "").strip()
    if body.lower().startswith("no tool call"):
        return []
    m = _CALL_SYNTAX.search(body)
    if m and m.group(1) in names:
        try:
            return [ToolCall(name=m.group(1), args=json.loads(m.group(2)), id="call_0")]
        except json.JSONDecodeError:
            pass
    val = _first_json_value(body)
    objs = val if isinstance(val, list) else [val]
    calls = []
    for i, o in enumerate(objs):
        c = _as_call(o, names, i)
        if c is not None:
            calls.append(c)
    return calls


def format_tool_call(call: ToolCall) -> str:
    """Canonical text a model emits for ``call`` (used to force-decode scripted decisions)."""
    return json.dumps({"name": call.name, "parameters": call.args})
