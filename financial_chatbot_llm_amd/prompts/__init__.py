"""Prompt assets.

``penny_persona.prompt`` and ``retrieval_decision.prompt`` carry the reference's
``system_prompt.txt`` / ``tool_prompt.txt`` text byte-for-byte: the prompts are part of the
wire-compatible surface, so they are data shipped verbatim, not code.
"""
from __future__ import annotations

import os
from functools import lru_cache

_DIR = os.path.dirname(os.path.abspath(__file__))


@lru_cache(maxsize=None)
def load_prompt(name: str) -> str:
    with open(os.path.join(_DIR, name), "r", encoding="utf-8") as fh:
        return fh.read()


def system_prompt() -> str:
    """Penny persona (reference ``system_prompt.txt``, loaded at ``llm_agent.py:14-15``)."""
    return load_prompt(os.getenv("PENNY_SYSTEM_PROMPT_FILE", "penny_persona.prompt"))


def tool_prompt() -> str:
    """Retrieval-decision instructions (reference ``tool_prompt.txt``, ``llm_agent.py:17-18``)."""
    return load_prompt(os.getenv("PENNY_TOOL_PROMPT_FILE", "retrieval_decision.prompt"))
