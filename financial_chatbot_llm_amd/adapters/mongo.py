"""MongoDB data access (reference ``database.py``) with an in-memory backend.

Same surface and failure semantics as the reference:

* ``check_connection`` pings and raises on failure (``database.py:15-21``).
* ``get_context`` raises if the context doc or its ``user_id`` is missing and renders the
  SURVEY §2.C.4 string (``database.py:23-73``).
* ``get_history`` sorts by ``timestamp`` ascending and **raises on empty history**
  (``database.py:75-91``).
* ``save_ai_message`` inserts ``{conversation_id, sender:"AIMessage", user_id, message,
  timestamp}`` (``database.py:93-104``).

Unlike the reference, the blocking pymongo calls run in worker threads
(``asyncio.to_thread``) so ``/health`` and the other in-flight turns keep running (fixes the
event-loop stall noted in SURVEY §3.2).
"""
from __future__ import annotations

import asyncio
import copy
import threading
from typing import Any, Dict, Iterable, List, Mapping, Optional, Tuple

from .. import config
from ..utils.logging import get_logger
from ..wire import ChatMessage, ai_message_doc, format_user_context, history_from_docs

logger = get_logger(__name__)


def _match(doc: Mapping[str, Any], flt: Mapping[str, Any]) -> bool:
    for k, v in flt.items():
        cur: Any = doc
        for part in k.split("."):
            if not isinstance(cur, Mapping) or part not in cur:
                return False
            cur = cur[part]
        if cur != v:
            return False
    return True


class _Cursor:
    def __init__(self, docs: List[Dict[str, Any]]):
        self._docs = docs

    def sort(self, key: str, direction: int = 1) -> "_Cursor":
        self._docs = sorted(self._docs, key=lambda d: d.get(key, 0), reverse=direction < 0)
        return self

    def __iter__(self):
        return iter(self._docs)


class InMemoryCollection:
    """Dict-backed collection.  Documents are indexed by ``conversation_id`` (every DAO query
    filters on it), so a turn's ``find`` touches that conversation's documents only instead of
    scanning (and deep-copying) the whole collection -- the bench ends with thousands of them."""

    INDEXED = "conversation_id"

    def __init__(self):
        self._docs: List[Dict[str, Any]] = []
        self._by_key: Dict[Any, List[Dict[str, Any]]] = {}
        self._lock = threading.Lock()
        self._next_id = 0

    def insert_one(self, doc: Dict[str, Any]):
        with self._lock:
            d = copy.deepcopy(doc)
            d.setdefault("_id", self._next_id)
            self._next_id += 1
            self._docs.append(d)
            if self.INDEXED in d:
                self._by_key.setdefault(d[self.INDEXED], []).append(d)
        return d["_id"]

    def insert_many(self, docs: Iterable[Dict[str, Any]]):
        return [self.insert_one(d) for d in docs]

    def _candidates(self, flt: Mapping[str, Any]) -> List[Dict[str, Any]]:
        if self.INDEXED in flt:
            return self._by_key.get(flt[self.INDEXED], [])
        return self._docs

    def find_one(self, flt: Mapping[str, Any]) -> Optional[Dict[str, Any]]:
        with self._lock:
            for d in self._candidates(flt):
                if _match(d, flt):
                    return copy.deepcopy(d)
        return None

    def find(self, flt: Mapping[str, Any]) -> _Cursor:
        with self._lock:
            return _Cursor([copy.deepcopy(d) for d in self._candidates(flt) if _match(d, flt)])

    def count_documents(self, flt: Mapping[str, Any]) -> int:
        with self._lock:
            return sum(1 for d in self._candidates(flt) if _match(d, flt))


class InMemoryMongo:
    """Enough of ``pymongo.MongoClient`` for the DAO: ``client[db][coll]`` and ``admin.command``."""

    def __init__(self):
        self._dbs: Dict[str, Dict[str, InMemoryCollection]] = {}
        self.fail_ping = False

        class _Admin:
            def __init__(s, outer):
                s.outer = outer

            def command(s, name: str):
                if s.outer.fail_ping:
                    raise ConnectionError("injected ping failure")
                return {"ok": 1.0}

        self.admin = _Admin(self)

    def __getitem__(self, name: str) -> Dict[str, InMemoryCollection]:
        db = self._dbs.setdefault(name, {})

        class _DB(dict):
            def __getitem__(s, coll):
                if coll not in db:
                    db[coll] = InMemoryCollection()
                return db[coll]

        return _DB()


class Database:
    def __init__(self, client: Any = None, uri: Optional[str] = None):
        uri = config.MONGODB_URI if uri is None else uri
        if client is None:
            if uri:
                from pymongo import MongoClient  # type: ignore
                import certifi  # type: ignore
                client = MongoClient(uri, tls=True, tlsCAFile=certifi.where())
            else:
                logger.warning("MONGODB_URI unset: using in-memory MongoDB")
                client = InMemoryMongo()
        self.client = client
        self.db = client[config.MONGO_DATABASE_NAME]
        self.context_collection = self.db[config.CONTEXT_COLLECTION_NAME]
        self.messages_collection = self.db[config.MESSAGE_COLLECTION_NAME]
        self._inline = isinstance(client, InMemoryMongo)

    async def _run(self, fn, *args):
        if self._inline:
            return fn(*args)
        return await asyncio.to_thread(fn, *args)

    async def check_connection(self) -> None:
        try:
            await self._run(self.client.admin.command, "ping")
            logger.info("MongoDB connection successful!")
        except Exception as e:
            logger.error(f"MongoDB connection failed: {e}")
            raise Exception(f"MongoDB connection failed: {e}")

    def _get_context_sync(self, conversation_id: str) -> Tuple[str, str]:
        doc = self.context_collection.find_one({"conversation_id": conversation_id})
        if not doc:
            raise Exception(f"No context found for conversation_id: {conversation_id}")
        user_id = doc.get("user_id", "")
        if not user_id:
            raise Exception(f"No user_id found in context for conversation_id: {conversation_id}")
        return format_user_context(doc), user_id

    async def get_context(self, conversation_id: str) -> Tuple[str, str]:
        try:
            return await self._run(self._get_context_sync, conversation_id)
        except Exception as e:
            logger.error(f"Error retrieving context for conversation_id {conversation_id}: {e}")
            raise

    def _get_history_sync(self, conversation_id: str) -> List[ChatMessage]:
        docs = list(self.messages_collection.find({"conversation_id": conversation_id}).sort("timestamp", 1))
        if not docs:
            raise Exception(f"No chat history found for conversation_id: {conversation_id}")
        return history_from_docs(docs)

    async def get_history(self, conversation_id: str) -> List[ChatMessage]:
        try:
            return await self._run(self._get_history_sync, conversation_id)
        except Exception as e:
            logger.error(f"Error retrieving history for conversation_id {conversation_id}: {e}")
            raise

    async def save_ai_message(self, conversation_id: str, message: str, user_id: str) -> None:
        try:
            await self._run(self.messages_collection.insert_one, ai_message_doc(conversation_id, message, user_id))
        except Exception as e:
            logger.error(f"Error saving message to MongoDB: {e}")
            raise

    # -- seeding helpers used by tests / bench (the upstream backend does this in prod) --
    def put_context(self, doc: Dict[str, Any]) -> None:
        self.context_collection.insert_one(doc)

    def put_user_message(self, conversation_id: str, message: str, user_id: str, timestamp: int) -> None:
        self.messages_collection.insert_one({
            "conversation_id": conversation_id, "sender": "UserMessage", "user_id": user_id,
            "message": message, "timestamp": int(timestamp)})
