"""Kafka ingest/egress (reference ``kafka_client.py``), plus an in-memory broker.

:class:`KafkaClient` keeps the reference's method surface (``setup_consumer``,
``produce_message``, ``produce_error_message``, ``poll_message``, ``close``) and consumer
settings (``kafka_client.py:12-22``: session timeout 45 s, client id ``python-client-1``,
group ``message_consumer``, ``auto.offset.reset=latest``).  It is backed either by
confluent-kafka (when importable and ``KAFKA_SERVER`` is set) or by :class:`InMemoryBroker`,
a partitioned, consumer-group-aware fake used by tests, the CPU plumbing config and the
benchmark harness.  Partitioning is by key hash, so per-conversation ordering holds exactly
as with a real broker keyed on ``conversation_id`` (``main.py:96``).

Fault injection: ``InMemoryBroker.faults`` can drop, delay or raise on produce.
"""
from __future__ import annotations

import json
import threading
import time
import zlib
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from .. import config
from ..utils.logging import get_logger

logger = get_logger(__name__)


@dataclass
class Message:
    """Duck-types ``confluent_kafka.Message`` for the fields the worker reads."""

    _topic: str
    _partition: int
    _offset: int
    _key: Optional[bytes]
    _value: bytes
    _error: Any = None
    _timestamp: float = field(default_factory=time.time)

    def value(self) -> bytes:
        return self._value

    def key(self) -> Optional[bytes]:
        return self._key

    def topic(self) -> str:
        return self._topic

    def partition(self) -> int:
        return self._partition

    def offset(self) -> int:
        return self._offset

    def error(self) -> Any:
        return self._error

    def timestamp(self) -> Tuple[int, int]:
        return (1, int(self._timestamp * 1000))


@dataclass
class Faults:
    drop_produce: float = 0.0      # probability a produced record is silently dropped
    delay_produce_s: float = 0.0
    raise_on_produce: bool = False
    raise_on_poll: bool = False


def _partition_for(key: Optional[bytes], n: int) -> int:
    if key is None:
        return 0
    return zlib.crc32(key) % n


class InMemoryBroker:
    """Thread-safe partitioned log with consumer groups (at-most-once, auto-commit on poll)."""

    def __init__(self, num_partitions: int = 8):
        self.num_partitions = num_partitions
        self._lock = threading.Condition()
        self._logs: Dict[str, List[List[Message]]] = {}
        self._offsets: Dict[Tuple[str, str, int], int] = {}
        self._members: Dict[Tuple[str, str], List["InMemoryConsumer"]] = defaultdict(list)
        self.faults = Faults()
        self._rng_state = 0x9E3779B9

    def _topic(self, topic: str) -> List[List[Message]]:
        if topic not in self._logs:
            self._logs[topic] = [[] for _ in range(self.num_partitions)]
        return self._logs[topic]

    def _rand(self) -> float:
        self._rng_state = (1103515245 * self._rng_state + 12345) & 0x7FFFFFFF
        return self._rng_state / 0x7FFFFFFF

    def produce(self, topic: str, key: Optional[bytes], value: bytes) -> None:
        if self.faults.raise_on_produce:
            raise RuntimeError("injected produce failure")
        if self.faults.delay_produce_s:
            time.sleep(self.faults.delay_produce_s)
        with self._lock:
            if self.faults.drop_produce and self._rand() < self.faults.drop_produce:
                return
            parts = self._topic(topic)
            p = _partition_for(key, self.num_partitions)
            parts[p].append(Message(topic, p, len(parts[p]), key, value))
            self._lock.notify_all()

    # -- consumer-group bookkeeping --------------------------------------------------
    def join(self, group: str, topic: str, consumer: "InMemoryConsumer", reset: str) -> None:
        with self._lock:
            parts = self._topic(topic)
            for p in range(self.num_partitions):
                k = (group, topic, p)
                if k not in self._offsets:
                    self._offsets[k] = len(parts[p]) if reset == "latest" else 0
            self._members[(group, topic)].append(consumer)

    def leave(self, group: str, topic: str, consumer: "InMemoryConsumer") -> None:
        with self._lock:
            members = self._members[(group, topic)]
            if consumer in members:
                members.remove(consumer)

    def _assigned(self, group: str, topic: str, consumer: "InMemoryConsumer") -> List[int]:
        members = self._members[(group, topic)]
        if consumer not in members:
            return []
        i, n = members.index(consumer), len(members)
        return [p for p in range(self.num_partitions) if p % n == i]

    def poll(self, group: str, topic: str, consumer: "InMemoryConsumer", timeout: float) -> Optional[Message]:
        if self.faults.raise_on_poll:
            raise RuntimeError("injected poll failure")
        deadline = time.monotonic() + max(timeout, 0.0)
        with self._lock:
            while True:
                parts = self._topic(topic)
                assigned = self._assigned(group, topic, consumer)
                # round-robin start so one hot partition cannot starve the others
                start = consumer._rr % max(len(assigned), 1)
                for j in range(len(assigned)):
                    p = assigned[(start + j) % len(assigned)]
                    k = (group, topic, p)
                    off = self._offsets[k]
                    if off < len(parts[p]):
                        self._offsets[k] = off + 1   # auto-commit (librdkafka default)
                        consumer._rr += 1
                        return parts[p][off]
                remaining = deadline - time.monotonic()
                if remaining <= 0:
                    return None
                self._lock.wait(remaining)

    # -- test helpers ----------------------------------------------------------------
    def messages(self, topic: str) -> List[Message]:
        with self._lock:
            parts = self._topic(topic)
            return sorted((m for p in parts for m in p), key=lambda m: m._timestamp)

    def values(self, topic: str, key: Optional[str] = None) -> List[Dict[str, Any]]:
        out = []
        for m in self.messages(topic):
            if key is None or m.key() == key.encode():
                out.append(json.loads(m.value()))
        return out


class InMemoryConsumer:
    def __init__(self, broker: InMemoryBroker, conf: Dict[str, Any]):
        self.broker, self.conf = broker, conf
        self.group = conf.get("group.id", config.GROUP_ID)
        self.topics: List[str] = []
        self._rr = 0

    def subscribe(self, topics: List[str]) -> None:
        for t in topics:
            self.broker.join(self.group, t, self, self.conf.get("auto.offset.reset", "latest"))
            self.topics.append(t)

    def poll(self, timeout: float = 0.1) -> Optional[Message]:
        per = timeout / max(len(self.topics), 1)
        for t in self.topics:
            m = self.broker.poll(self.group, t, self, per)
            if m is not None:
                return m
        return None

    def close(self) -> None:
        for t in self.topics:
            self.broker.leave(self.group, t, self)
        self.topics = []


class InMemoryProducer:
    def __init__(self, broker: InMemoryBroker):
        self.broker = broker

    def produce(self, topic: str, key: Any = None, value: Any = None) -> None:
        k = key.encode("utf-8") if isinstance(key, str) else key
        v = value.encode("utf-8") if isinstance(value, str) else value
        self.broker.produce(topic, k, v)

    def poll(self, timeout: float = 0) -> int:
        return 0

    def flush(self, timeout: float = -1) -> int:
        return 0


def _confluent():
    try:
        import confluent_kafka  # type: ignore
        return confluent_kafka
    except Exception:  # pragma: no cover - not in the image
        return None


class KafkaClient:
    """Reference-compatible Kafka client (``kafka_client.py:8-61``)."""

    def __init__(self, broker: Optional[InMemoryBroker] = None, kafka_config: Optional[Dict[str, str]] = None):
        self.kafka_config = dict(kafka_config or config.KAFKA_CONFIG)
        ck = _confluent()
        self.broker = broker
        if broker is None and ck is not None and self.kafka_config.get("bootstrap.servers"):
            self._backend = "confluent"
            self.producer = ck.Producer(self.kafka_config)
        else:
            if broker is None:
                broker = InMemoryBroker()
                logger.warning("confluent-kafka unavailable or KAFKA_SERVER unset: using in-memory broker")
            self.broker = broker
            self._backend = "memory"
            self.producer = InMemoryProducer(broker)
        self.consumer = None

    @property
    def backend(self) -> str:
        return self._backend

    def consumer_config(self) -> Dict[str, Any]:
        return {
            **self.kafka_config,
            "session.timeout.ms": config.KAFKA_SESSION_TIMEOUT_MS,
            "client.id": "python-client-1",
            "group.id": config.GROUP_ID,
            "auto.offset.reset": "latest",
        }

    def setup_consumer(self) -> None:
        conf = self.consumer_config()
        if self._backend == "confluent":
            self.consumer = _confluent().Consumer(conf)
        else:
            self.consumer = InMemoryConsumer(self.broker, conf)
        self.consumer.subscribe([config.USER_MESSAGE_TOPIC])
        logger.info("Kafka consumer started, waiting for messages...")

    def produce_message(self, topic: str, key: str, value: Dict[str, Any]) -> None:
        try:
            self.producer.produce(topic, key=key, value=json.dumps(value))
            self.producer.poll(0)
        except Exception as e:
            logger.error(f"Error producing message to Kafka: {e}")
            raise

    def produce_error_message(self, topic: str, key: str, value: Dict[str, Any]) -> None:
        try:
            self.producer.produce(topic, key=key, value=json.dumps(value))
            self.producer.flush()
        except Exception as e:
            logger.error(f"Failed to send error message to Kafka: {e}")
            raise

    def poll_message(self, timeout: float = config.KAFKA_POLL_TIMEOUT_S):
        if self.consumer is None:
            logger.error("Kafka consumer is not initialized.")
            return None
        try:
            msg = self.consumer.poll(timeout)
            if msg is None:
                return None
            if msg.error():
                logger.error(f"Consumer error: {msg.error()}")
                return None
            return msg
        except Exception as e:
            logger.error(f"Error in message consumption: {e}")
            return None

    def close(self) -> None:
        if self.consumer:
            self.consumer.close()
        self.producer.flush()
