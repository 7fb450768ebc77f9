"""I/O adapters: Kafka (reference kafka_client.py) and MongoDB (reference database.py)."""
from .kafka import InMemoryBroker, KafkaClient, Message
from .mongo import Database, InMemoryMongo

__all__ = ["InMemoryBroker", "KafkaClient", "Message", "Database", "InMemoryMongo"]
