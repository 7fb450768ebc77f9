"""``retrieve_transactions`` tool (reference ``tools/qdrant_tool.py:39-177``).

Argument schema and semantics are kept exactly; the backend changes from remote
OpenAI-embeddings + Qdrant to the on-device :class:`~..retrieval.service.RetrievalService`
(bge encoder + filtered top-k HIP kernel over an HBM-resident corpus).

Semantics preserved:
* missing ``user_id`` -> ``[]`` (security check, ``qdrant_tool.py:89-91``);
* filter ``metadata.user_id == user_id`` always, plus ``metadata.date >= now - N days`` when
  ``time_period_days`` is truthy (``qdrant_tool.py:105-126``);
* ``limit = num_transactions or 10000`` (``qdrant_tool.py:145``);
* results re-checked against ``user_id`` and returned as ``page_content`` strings in
  descending score order (``qdrant_tool.py:159-172``);
* any exception -> ``[]`` (``qdrant_tool.py:175-177``).
"""
from __future__ import annotations

import datetime as _dt
from typing import Any, Dict, List, Optional

from pydantic import BaseModel, ConfigDict, Field

from .. import config
from ..utils.logging import get_logger
from .base import Tool

logger = get_logger(__name__)

RETRIEVAL_TOOL_DESCRIPTION = (
    "Retrieve relevant transactions from the database based on search intent.\n\n"
    "Args:\n    intent: RetrievalIntent object specifying search parameters\n\n"
    "Returns:\n    JSON string of retrieved transactions"
)


class RetrievalIntent(BaseModel):
    """Intent for retrieving user transactions with specific search criteria."""

    model_config = ConfigDict(json_schema_extra={"example": {
        "search_query": "monthly spending categories including rent and groceries",
        "num_transactions": None, "time_period_days": 30}})

    user_id: str = Field(default="", description="The ID of the user whose transactions to retrieve")
    num_transactions: Optional[int] = Field(
        default=None, ge=1, le=10000,
        description="Optional: Number of transactions to retrieve (between 1 and 500). "
                    "If not specified, defaults to 10000.")
    time_period_days: Optional[int] = Field(
        default=None,
        description="Optional: Limit to transactions from the last N days (e.g., 30 for last month, 7 for last week)")
    search_query: str = Field(
        default="recent transactions",
        description="Semantic search query describing what transactions to find (e.g., 'monthly spending "
                    "categories', 'grocery purchases', 'entertainment expenses', 'rent and housing costs')")


def date_floor(time_period_days: Optional[int], now: Optional[_dt.datetime] = None) -> Optional[int]:
    """Unix-seconds lower bound for ``metadata.date`` or None (truthiness test as the reference)."""
    if not time_period_days:
        return None
    start = (now or _dt.datetime.now()) - _dt.timedelta(days=time_period_days)
    return int(start.timestamp())


def effective_limit(num_transactions: Optional[int]) -> int:
    return num_transactions if num_transactions is not None else config.RETRIEVAL_DEFAULT_LIMIT


class TransactionList(list):
    """The tool's return value: a plain ``list`` of ``page_content`` strings, exactly as the
    reference (``qdrant_tool.py:159-172``), carrying the hits' structured metadata alongside in
    ``records`` (date as ``YYYY-MM-DD``, amount, merchant, category, ...; ``user_id`` dropped) so
    the plot tool gets real columns (``plot_tool.py:29-63``)."""

    records: List[Dict[str, Any]]


def transaction_record(payload: Dict[str, Any]) -> Dict[str, Any]:
    meta = dict(payload.get("metadata", {}))
    meta.pop("user_id", None)
    if isinstance(meta.get("date"), (int, float)):
        meta["date"] = _dt.datetime.fromtimestamp(int(meta["date"])).strftime("%Y-%m-%d")
    meta.setdefault("description", payload.get("page_content", ""))
    return meta


def make_retrieval_tool(service) -> Tool:
    """Bind the tool to a RetrievalService (sync ``invoke`` and async ``ainvoke`` paths)."""

    def _post(user_id: str, hits) -> List[str]:
        out, skipped = TransactionList(), 0
        out.records = []
        for h in hits:
            meta = (h.payload or {}).get("metadata", {}) if h.payload else {}
            if h.payload and meta.get("user_id") == user_id:
                out.append(h.payload["page_content"])
                out.records.append(transaction_record(h.payload))
            else:
                skipped += 1
        if skipped:
            logger.warning(f"Skipped {skipped} transactions due to user_id mismatch")
        logger.info(f"Successfully processed {len(out)} transactions")
        return out

    def retrieve_transactions(user_id: str = "", num_transactions: Optional[int] = None,
                              time_period_days: Optional[int] = None,
                              search_query: str = "recent transactions") -> List[str]:
        try:
            if not user_id:
                logger.error("Security violation: user_id not provided")
                return []
            hits = service.search_sync(search_query, user_id=user_id,
                                       date_gte=date_floor(time_period_days),
                                       limit=effective_limit(num_transactions))
            return _post(user_id, hits)
        except Exception as e:  # noqa: BLE001 - reference swallows all errors
            logger.error(f"Error retrieving transactions: {e}", exc_info=True)
            return []

    async def aretrieve_transactions(user_id: str = "", num_transactions: Optional[int] = None,
                                     time_period_days: Optional[int] = None,
                                     search_query: str = "recent transactions") -> List[str]:
        try:
            if not user_id:
                logger.error("Security violation: user_id not provided")
                return []
            hits = await service.search(search_query, user_id=user_id,
                                        date_gte=date_floor(time_period_days),
                                        limit=effective_limit(num_transactions))
            return _post(user_id, hits)
        except Exception as e:  # noqa: BLE001
            logger.error(f"Error retrieving transactions: {e}", exc_info=True)
            return []

    return Tool(name="retrieve_transactions", description=RETRIEVAL_TOOL_DESCRIPTION,
                args_schema=RetrievalIntent, func=retrieve_transactions,
                coroutine=aretrieve_transactions)
