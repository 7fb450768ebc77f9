"""On-device retrieval: embedders, vector stores and the micro-batched service (R2 + R3)."""
from .embedder import BgeEmbedder, HashEmbedder
from .ingest import CorpusIngestor, iter_documents
from .service import RetrievalService
from .store import Corpus, DeviceVectorStore, Hit, NumpyVectorStore, synthetic_payload, user_name

__all__ = ["BgeEmbedder", "HashEmbedder", "CorpusIngestor", "iter_documents", "RetrievalService", "Corpus", "DeviceVectorStore", "Hit",
           "NumpyVectorStore", "synthetic_payload", "user_name"]
