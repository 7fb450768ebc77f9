"""Serving layer: FastAPI app, Kafka worker loop and the services factory."""
from .app import Services, create_app
from .worker import ChatWorker

__all__ = ["Services", "create_app", "ChatWorker"]
