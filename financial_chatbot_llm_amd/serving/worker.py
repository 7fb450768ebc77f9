"""Kafka-driven chat worker (reference ``main.py:55-159``).

``process_message`` keeps the reference's wire behaviour exactly:

* decode JSON, read ``message``/``conversation_id`` (``main.py:57-60``);
* context/history failure -> log and return with **no Kafka reply** (``main.py:66-70``);
* every ``response_chunk`` -> one Kafka record, ``complete`` -> final record
  (``main.py:81-110``); any agent exception -> error record with flush (``main.py:112-122``);
* full reply saved to Mongo after completion (``main.py:125-129``);
* a turn exceeding 100 s -> timeout record (``main.py:138-153``).

The consumer loop no longer awaits each turn before polling the next message (the reference
processes strictly serially per worker, ``main.py:138``): turns run as concurrent tasks,
bounded by ``max_concurrent_turns``, so the GPU engine can batch them.  Turns of the SAME
conversation stay serialised (per-conversation lock) to keep Kafka's per-key ordering.
"""
from __future__ import annotations

import asyncio
import json
from typing import Any, Dict, Optional, Set

from .. import config
from ..engine.sequence import TURN_START
from ..utils.logging import get_logger
from ..utils.metrics import METRICS, TurnTrace, now
from ..wire import chunk_event, complete_event, decode_user_message, error_event, timeout_event

logger = get_logger(__name__)


class ChatWorker:
    def __init__(self, db, kafka, agent, max_concurrent_turns: int = 256,
                 message_timeout_s: float = config.MESSAGE_TIMEOUT_S, metrics=METRICS):
        self.db, self.kafka, self.agent = db, kafka, agent
        self.message_timeout_s = message_timeout_s
        self.metrics = metrics
        self._sem = asyncio.Semaphore(max_concurrent_turns)
        self._conv_locks: Dict[str, list] = {}   # cid -> [lock, users]
        self._tasks: Set[asyncio.Task] = set()
        self._stop = asyncio.Event()
        self.traces = []

    async def process_message(self, message, trace: Optional[TurnTrace] = None) -> None:
        value = decode_user_message(message.value())
        msg, conversation_id = value["message"], value["conversation_id"]
        trace = trace or TurnTrace(conversation_id=conversation_id)
        TURN_START.set(trace.t_receive)     # engine requests of this turn are scheduled by it
        full_message = ""
        logger.info(f"Received message from Kafka: |{conversation_id}| {msg}")
        try:
            trace.mark("mongo_start")
            context, user_id = await self.db.get_context(conversation_id)
            chat_history = await self.db.get_history(conversation_id)
            trace.mark("mongo_done")
        except Exception as e:  # noqa: BLE001
            logger.error(f"Error retrieving context or history for conversation {conversation_id}: {e}")
            trace.error = True
            return
        try:
            async for update in self.agent.stream_with_status(msg, user_id, context, chat_history):
                kind = update["type"]
                if kind == "response_chunk":
                    text = update["content"]
                    full_message += text
                    trace.on_chunk()
                    self.kafka.produce_message(config.AI_RESPONSE_TOPIC, conversation_id, chunk_event(value, text))
                elif kind == "complete":
                    self.kafka.produce_message(config.AI_RESPONSE_TOPIC, conversation_id, complete_event(value))
                    trace.t_complete = now()
                    logger.info(f"Complete message sent to Kafka for conversation {conversation_id}")
                elif kind == "tool_complete":
                    trace.tools_ok += int(bool(update.get("ok")))
                    trace.tools_failed += int(not update.get("ok"))
                elif kind == "retrieval_complete":
                    trace.retrieved = int(update.get("count", 0))
                    trace.mark("retrieval_done")
                elif kind == "status":
                    m = update.get("message", "")
                    if m.startswith("Analyzing"):
                        trace.mark("decide_start")
                    elif m.startswith("Retrieving") or m.startswith("No transaction"):
                        trace.mark("decide_done")
                    elif m.startswith("Generating"):
                        trace.mark("respond_start")
        except Exception as e:  # noqa: BLE001
            logger.error(f"Error streaming LLM response: {e}")
            trace.error = True
            self.kafka.produce_error_message(config.AI_RESPONSE_TOPIC, conversation_id, error_event(value))
            return
        try:
            await self.db.save_ai_message(conversation_id=conversation_id, message=full_message, user_id=user_id)
            logger.info(f"Message saved to DB for conversation {conversation_id}")
        except Exception as e:  # noqa: BLE001
            logger.error(f"Error saving AI message to DB: {e}")

    async def handle(self, message) -> None:
        """One turn with the 100 s deadline and timeout event (``main.py:136-153``)."""
        try:
            value = json.loads(message.value().decode("utf-8"))
            cid = value.get("conversation_id", "")
        except Exception:  # noqa: BLE001
            value, cid = None, ""
        # per-conversation lock, reference-counted: the entry lives while ANY task of the
        # conversation holds or awaits it (a waiter still queued on the semaphore is not in the
        # lock's waiter list, so "no waiters" is not "no users")
        entry = self._conv_locks.get(cid)
        if entry is None:
            entry = self._conv_locks[cid] = [asyncio.Lock(), 0]
        entry[1] += 1
        lock = entry[0]
        trace = TurnTrace(conversation_id=cid)
        try:
            async with lock, self._sem:
                await self._handle_locked(message, value, trace)
        finally:
            entry[1] -= 1
            if entry[1] == 0 and self._conv_locks.get(cid) is entry:
                del self._conv_locks[cid]

    async def _handle_locked(self, message, value, trace: TurnTrace) -> None:
        try:
            await asyncio.wait_for(self.process_message(message, trace), timeout=self.message_timeout_s)
        except asyncio.TimeoutError:
            logger.error(f"Message processing timed out after {self.message_timeout_s} seconds")
            trace.error = True
            try:
                if value is None:
                    raise ValueError("undecodable message")
                self.kafka.produce_error_message(config.AI_RESPONSE_TOPIC, value["conversation_id"],
                                                 timeout_event(value))
            except Exception as e:  # noqa: BLE001
                logger.error(f"Failed to send timeout error message: {e}")
        except Exception as e:  # noqa: BLE001
            logger.error(f"Error in message consumption: {e}")
            trace.error = True
        finally:
            self.metrics.record_turn(trace)
            self.traces.append(trace)

    async def consume_messages(self) -> None:
        blocking_poll = getattr(self.kafka, "backend", "memory") != "memory"
        while not self._stop.is_set():
            try:
                if blocking_poll:
                    msg = await asyncio.to_thread(self.kafka.poll_message)
                else:
                    msg = self.kafka.poll_message(0.0)
                if msg is not None:
                    t = asyncio.create_task(self.handle(msg))
                    self._tasks.add(t)
                    t.add_done_callback(self._tasks.discard)
                else:
                    await asyncio.sleep(config.IDLE_SLEEP_S)
            except Exception as e:  # noqa: BLE001
                logger.error(f"Error in message consumption: {e}")
                await asyncio.sleep(config.LOOP_ERROR_BACKOFF_S)

    async def drain(self) -> None:
        while self._tasks:
            await asyncio.gather(*list(self._tasks), return_exceptions=True)

    def stop(self) -> None:
        self._stop.set()
