"""Golden-format tests for the wire-compatible surfaces (SURVEY §2.C, §4 'Unit: wire')."""
import datetime as dt
import json

from financial_chatbot_llm_amd import config
from financial_chatbot_llm_amd.wire import (AIMessage, ChatMessage, HumanMessage, build_messages, chunk_event,
                                            complete_event, decide_system_prompt, error_event, format_user_context,
                                            history_from_docs, respond_context, respond_system_prompt, timeout_event)

INBOUND = {"message": "How much did I spend?", "conversation_id": "c1", "user_id": "u1", "extra": 7}

CTX_DOC = {
    "conversation_id": "c1", "user_id": "u1", "name": "Ada", "income": 8000, "savings_goal": 1500.5,
    "accounts": [
        {"account_id": "a1", "balances": {"current": 1234.5, "iso_currency_code": "USD"}, "official_name": "Checking Plus"},
        {"account_id": "a2", "balances": {}},
    ],
    "additional_monthly_expenses": [
        {"name": "Gym", "amount": 50, "description": ""},
        {"name": "Rent", "amount": 2000, "description": "downtown apt"},
    ],
}


def test_context_string_exact():
    expect = ("My name is Ada.\nI make 8000 dollars a month.\nI want to save 1500.5 a month.\n\n"
              "Here is a list of my current account balances:\n"
              "Checking Plus : 1234.5 USD\n"
              "Unnamed Account : 0.0 \n"
              "Here is a list of my recurring monthly expenses:\n"
              "Name: Gym | Amount: 50\n"
              "Name: Rent | Amount: 2000 | Description: downtown apt\n")
    assert format_user_context(CTX_DOC) == expect


def test_context_none_lists():
    doc = dict(CTX_DOC, accounts=None, additional_monthly_expenses=None)
    s = format_user_context(doc)
    assert s.endswith("Here is a list of my current account balances:\nHere is a list of my recurring monthly expenses:\n")


def test_kafka_events():
    c = chunk_event(INBOUND, "Hi")
    assert c == {**INBOUND, "message": "Hi", "last_message": False, "error": False, "sender": "AIMessage",
                 "type": "response_chunk"}
    done = complete_event(INBOUND)
    assert done["message"] == INBOUND["message"] and done["type"] == "complete" and done["last_message"] is True
    err = error_event(INBOUND)
    assert "type" not in err and err["message"] == "" and err["error"] is True and err["extra"] == 7
    to = timeout_event(INBOUND)
    assert to["message"] == "Request timed out. Please try again." and to["error"] is True and "type" not in to
    assert json.loads(json.dumps(c)) == c


def test_prompt_assembly():
    d = dt.date(2026, 10, 15)
    assert decide_system_prompt("TOOL", d) == "The current date is 2026-10-15.\nTOOL"
    assert respond_system_prompt("SYS", d) == "The current date is 2026-10-15.\n\nSYS"
    assert respond_context("ctx", []) == "ctx\n"
    assert respond_context("ctx", ["t1", "t2"]) == "ctx\nRetrieved Transaction Data:\nt1\nt2"
    hist = [HumanMessage("q0"), AIMessage("a0"), HumanMessage("q1")]
    msgs = build_messages("SP", "CTX", hist, "q1")
    assert msgs[0] == ChatMessage("system", "SP\nCTX")
    assert msgs[-1] == ChatMessage("user", "q1") and msgs[-2] == ChatMessage("user", "q1")  # duplicated on purpose
    assert len(msgs) == 5


def test_history_mapping():
    docs = [{"sender": "UserMessage", "message": "a"}, {"sender": "AIMessage", "message": "b"},
            {"sender": "Other", "message": "c"}]
    assert [m.role for m in history_from_docs(docs)] == ["user", "assistant", "assistant"]


def test_kafka_config_switch(monkeypatch):
    monkeypatch.setenv("KAFKA_SERVER", "broker:9092")
    monkeypatch.delenv("KAFKA_USERNAME", raising=False)
    assert config.build_kafka_config() == {"bootstrap.servers": "broker:9092", "security.protocol": "PLAINTEXT"}
    monkeypatch.setenv("KAFKA_USERNAME", "u")
    monkeypatch.setenv("KAFKA_PASSWORD", "p")
    c = config.build_kafka_config()
    assert c["security.protocol"] == "SASL_SSL" and c["sasl.mechanisms"] == "PLAIN" and c["sasl.username"] == "u"


def test_constants():
    assert (config.USER_MESSAGE_TOPIC, config.AI_RESPONSE_TOPIC, config.GROUP_ID) == \
        ("user_message", "ai_response", "message_consumer")
    assert (config.CONTEXT_COLLECTION_NAME, config.MESSAGE_COLLECTION_NAME, config.QDRANT_COLLECTION_NAME) == \
        ("contexts", "messages", "transactions")


def test_logger_format():
    from financial_chatbot_llm_amd.utils.logging import LOG_FORMAT
    assert LOG_FORMAT == "[%(levelname)s] %(asctime)s |%(name)s| %(message)s"
