"""Wire-compatible surfaces: Kafka events, Mongo docs, context string, prompts.

Everything in here is pure Python and byte-for-byte compatible with the reference:

* Kafka event payloads: ``main.py:86-93`` (chunk), ``main.py:101-107`` (complete),
  ``main.py:114-121`` (agent error), ``main.py:144-151`` (timeout).
* User-context string: ``database.py:33-68``.
* History mapping: ``database.py:83-87``.
* Prompt assembly: ``llm_agent.py:47-51`` (3-message layout), ``llm_agent.py:85`` (decide
  system prompt, single newline), ``llm_agent.py:146,238`` (respond, double newline) and
  ``llm_agent.py:234-236`` (retrieved-transactions block).
"""
from __future__ import annotations

import datetime as _dt
import json
import time
from dataclasses import dataclass
from typing import Any, Dict, Iterable, List, Mapping, Optional, Sequence

AI_SENDER = "AIMessage"
USER_SENDER = "UserMessage"
TIMEOUT_MESSAGE = "Request timed out. Please try again."


# ---------------------------------------------------------------------------------------
# Chat messages (replaces langchain_core HumanMessage / AIMessage)
# ---------------------------------------------------------------------------------------
@dataclass(frozen=True)
class ChatMessage:
    role: str       # "system" | "user" | "assistant"
    content: str


def HumanMessage(content: str) -> ChatMessage:  # noqa: N802 - mirrors the LangChain name
    return ChatMessage("user", content)


def AIMessage(content: str) -> ChatMessage:  # noqa: N802
    return ChatMessage("assistant", content)


def history_from_docs(docs: Iterable[Mapping[str, Any]]) -> List[ChatMessage]:
    """``sender == "UserMessage"`` -> user, anything else -> assistant (``database.py:83-87``)."""
    return [HumanMessage(d["message"]) if d.get("sender") == USER_SENDER else AIMessage(d["message"])
            for d in docs]


# ---------------------------------------------------------------------------------------
# Mongo documents
# ---------------------------------------------------------------------------------------
def normalize_account(a: Mapping[str, Any]) -> Dict[str, Any]:
    """Account defaults exactly as ``database.py:36-52``."""
    b = a.get("balances", {}) or {}
    return {
        "account_id": a.get("account_id", ""),
        "balances": {
            "available": b.get("available", None),
            "current": b.get("current", 0.0),
            "limit": b.get("limit", None),
            "iso_currency_code": b.get("iso_currency_code", ""),
        },
        "mask": a.get("mask", ""),
        "name": a.get("name", "Unnamed Account"),
        "official_name": a.get("official_name", "Unnamed Account"),
        "subtype": a.get("subtype", ""),
        "type": a.get("type", ""),
    }


def format_user_context(doc: Mapping[str, Any]) -> str:
    """Render the natural-language user context (``database.py:56-68``)."""
    accounts = [normalize_account(a) for a in (doc.get("accounts") if doc.get("accounts") is not None else [])]
    out = [f"My name is {doc['name']}.\nI make {doc['income']} dollars a month.\n"
           f"I want to save {doc['savings_goal']} a month.\n\n"]
    out.append("Here is a list of my current account balances:\n")
    for acc in accounts:
        out.append(f"{acc['official_name']} : {acc['balances']['current']} {acc['balances']['iso_currency_code']}\n")
    out.append("Here is a list of my recurring monthly expenses:\n")
    expenses = doc.get("additional_monthly_expenses")
    for e in (expenses if expenses is not None else []):
        line = f"Name: {e['name']} | Amount: {e['amount']}"
        desc = e.get("description", "")
        if desc != "":
            line += " | Description: " + f"{desc}"
        out.append(line + "\n")
    return "".join(out)


def ai_message_doc(conversation_id: str, message: str, user_id: str,
                   timestamp: Optional[int] = None) -> Dict[str, Any]:
    """Document persisted for an AI reply (``database.py:95-101``)."""
    return {
        "conversation_id": conversation_id,
        "sender": AI_SENDER,
        "user_id": user_id,
        "message": message,
        "timestamp": int(time.time()) if timestamp is None else int(timestamp),
    }


# ---------------------------------------------------------------------------------------
# Kafka events
# ---------------------------------------------------------------------------------------
def decode_user_message(raw: bytes) -> Dict[str, Any]:
    """UTF-8 JSON with required ``message`` and ``conversation_id`` (``main.py:57-60``)."""
    value = json.loads(raw.decode("utf-8"))
    _ = value["message"], value["conversation_id"]
    return value


def chunk_event(inbound: Mapping[str, Any], text: str) -> Dict[str, Any]:
    return {**inbound, "message": text, "last_message": False, "error": False,
            "sender": AI_SENDER, "type": "response_chunk"}


def complete_event(inbound: Mapping[str, Any]) -> Dict[str, Any]:
    # NB: "message" is intentionally NOT overridden (echoes the user's text), main.py:101-107.
    return {**inbound, "last_message": True, "error": False, "sender": AI_SENDER, "type": "complete"}


def error_event(inbound: Mapping[str, Any]) -> Dict[str, Any]:
    # No "type" key on the error path (main.py:114-121).
    return {**inbound, "message": "", "last_message": True, "error": True, "sender": AI_SENDER}


def timeout_event(inbound: Mapping[str, Any]) -> Dict[str, Any]:
    return {**inbound, "message": TIMEOUT_MESSAGE, "last_message": True, "error": True,
            "sender": AI_SENDER}


def encode_event(value: Mapping[str, Any]) -> bytes:
    """``json.dumps`` with default separators, as ``kafka_client.py:26``."""
    return json.dumps(value).encode("utf-8")


# ---------------------------------------------------------------------------------------
# Prompt assembly
# ---------------------------------------------------------------------------------------
def today_iso(today: Optional[_dt.date] = None) -> str:
    return (today or _dt.date.today()).isoformat()


def decide_system_prompt(tool_prompt: str, today: Optional[_dt.date] = None) -> str:
    return f"The current date is {today_iso(today)}.\n{tool_prompt}"


def respond_system_prompt(system_prompt: str, today: Optional[_dt.date] = None) -> str:
    return f"The current date is {today_iso(today)}.\n\n{system_prompt}"


def respond_context(user_context: str, transactions: Sequence[str]) -> str:
    ctx = f"{user_context}\n"
    if transactions:
        ctx += "Retrieved Transaction Data:\n" + "\n".join(transactions)
    return ctx


def build_messages(system_prompt: str, context: str, history: Sequence[ChatMessage],
                   user_input: str) -> List[ChatMessage]:
    """system ``"{system_prompt}\\n{context}"`` + history + user ``"{input}"`` (llm_agent.py:47-51).

    The current user message is normally already the last history entry (the upstream
    backend stores it before publishing), so it appears twice -- reproduced on purpose.
    """
    return [ChatMessage("system", f"{system_prompt}\n{context}"), *history, ChatMessage("user", user_input)]
