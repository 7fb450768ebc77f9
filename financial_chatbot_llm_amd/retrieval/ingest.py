"""Getting real transactions into the on-device collection (what Qdrant ingestion did upstream).

The reference queries a persistent, externally populated Qdrant collection ``transactions``
(``tools/qdrant_tool.py:24-28``, ``:147-153``) whose points follow langchain-qdrant's layout
``{page_content, metadata{user_id, date, ...}}``, embedded with the same model
as the queries (``tools/qdrant_tool.py:28,136-137``).  Here:

* :func:`iter_documents` streams documents from JSONL / JSON / Parquet files;
* :class:`CorpusIngestor` embeds ``page_content`` in large batches with the on-device bge encoder
  (K14, bulk mode: thousands of rows per forward) and appends vectors + metadata to the store;
* ``DeviceVectorStore.save`` / ``.load`` snapshot the collection (safetensors + JSON, no pickles);
* ``POST /v1/transactions`` (serving/app.py) ingests at runtime, in batches interleaved with searches.

CLI (bulk build + snapshot, reports docs/s)::

    python -m financial_chatbot_llm_amd.retrieval.ingest --input txns.jsonl --snapshot /data/penny_corpus
"""
from __future__ import annotations

import argparse
import datetime as _dt
import json
import os
import time
from typing import Any, Dict, Iterable, Iterator, List, Optional, Tuple

from ..utils.logging import get_logger

logger = get_logger(__name__)


def _to_unix(v: Any) -> int:
    """``metadata.date`` as unix seconds (the reference compares ints, qdrant_tool.py:116-126)."""
    if isinstance(v, (int, float)):
        return int(v)
    if isinstance(v, str):
        s = v.strip()
        if s.lstrip("-").isdigit():
            return int(s)
        d = _dt.datetime.fromisoformat(s.replace("Z", "+00:00"))
        return int(d.timestamp())
    raise ValueError(f"unsupported date {v!r}")


def normalise(doc: Dict[str, Any]) -> Dict[str, Any]:
    """Validate one point: ``page_content`` text and ``metadata.user_id``/``metadata.date``
    (flat ``user_id``/``date`` keys are accepted and moved under ``metadata``)."""
    text = doc.get("page_content")
    if not isinstance(text, str) or not text:
        raise ValueError("document without page_content")
    meta = dict(doc.get("metadata") or {})
    for k in ("user_id", "date"):
        if k not in meta and k in doc:
            meta[k] = doc[k]
    if not meta.get("user_id"):
        raise ValueError("document without metadata.user_id")
    meta["user_id"] = str(meta["user_id"])
    meta["date"] = _to_unix(meta.get("date", 0))
    return {"page_content": text, "metadata": meta}


def iter_documents(path: str, batch_rows: int = 65536) -> Iterator[Dict[str, Any]]:
    """Stream documents from ``.jsonl``/``.ndjson`` (one object a line), ``.json`` (a list) or
    ``.parquet`` (``page_content`` + a ``metadata`` struct column, or flat metadata columns)."""
    if path.endswith((".jsonl", ".ndjson")):
        with open(path) as fh:
            for line in fh:
                line = line.strip()
                if line:
                    yield json.loads(line)
    elif path.endswith(".json"):
        with open(path) as fh:
            data = json.load(fh)
        yield from (data if isinstance(data, list) else data.get("documents", []))
    elif path.endswith(".parquet"):
        # system allocator unless the deployment chose one: arrow's jemalloc pool segfaulted
        # intermittently next to torch in test workers (only applies if pyarrow is not loaded yet)
        os.environ.setdefault("ARROW_DEFAULT_MEMORY_POOL", "system")
        import pyarrow.parquet as pq
        f = pq.ParquetFile(path)
        for batch in f.iter_batches(batch_size=batch_rows):
            cols = batch.to_pydict()
            n = batch.num_rows
            names = [c for c in cols if c not in ("page_content", "metadata")]
            for i in range(n):
                meta = dict(cols["metadata"][i]) if "metadata" in cols and cols["metadata"][i] else {}
                for c in names:
                    meta.setdefault(c.split("metadata.", 1)[-1], cols[c][i])
                yield {"page_content": cols["page_content"][i], "metadata": meta}
    else:
        raise ValueError(f"unsupported corpus file {path} (jsonl/json/parquet)")


class CorpusIngestor:
    """Bulk-embed documents on the GPU and append them to a vector store."""

    def __init__(self, embedder, store, batch_size: int = 1024, max_len: int = 128, lock=None):
        """``lock`` (optional) is held around each batch's embed + append only, so a caller
        that serialises searches on the same store with it (the serving RetrievalService) can
        interleave its searches between batches instead of waiting for the whole ingest."""
        self.embedder, self.store = embedder, store
        self.batch_size, self.max_len = batch_size, max_len
        self.lock = lock
        self.docs = 0
        self.rejected = 0
        self.seconds = 0.0

    def _flush(self, batch: List[Dict[str, Any]]) -> None:
        if self.lock is not None:
            with self.lock:
                self._flush_locked(batch)
                self._sync()
        else:
            self._flush_locked(batch)

    def _flush_locked(self, batch: List[Dict[str, Any]]) -> None:
        texts = [d["page_content"] for d in batch]
        if hasattr(self.embedder, "tokenize"):
            vecs = self.embedder.embed(texts, max_len=self.max_len)
        else:
            vecs = self.embedder.embed(texts)
        self.store.add(vecs, [d["metadata"]["user_id"] for d in batch], [d["metadata"]["date"] for d in batch], batch)

    def ingest(self, docs: Iterable[Dict[str, Any]]) -> Dict[str, float]:
        t0 = time.perf_counter()
        batch: List[Dict[str, Any]] = []
        n0 = self.docs
        for d in docs:
            try:
                batch.append(normalise(d))
            except (ValueError, TypeError) as e:
                self.rejected += 1
                logger.warning(f"skipping document: {e}")
                continue
            if len(batch) >= self.batch_size:
                self._flush(batch)
                self.docs += len(batch)
                batch = []
        if batch:
            self._flush(batch)
            self.docs += len(batch)
        self._sync()
        dt = time.perf_counter() - t0
        self.seconds += dt
        n = self.docs - n0
        return {"ingested": n, "rejected": self.rejected, "seconds": round(dt, 3),
                "docs_per_s": round(n / dt, 1) if dt > 0 else 0.0}

    def _sync(self) -> None:
        dev = getattr(self.store, "device", None)
        if dev is not None and getattr(dev, "type", "") == "cuda":
            import torch
            torch.cuda.synchronize(dev)


def build_store(embed_model: str, device: str, corpus_path: Optional[str], weights: Optional[str] = None,
                vocab: Optional[str] = None) -> Tuple[Any, Any]:
    """(embedder, store) for serving: load a snapshot directory, or ingest a document file."""
    import os

    from .embedder import BgeEmbedder
    from .store import DeviceVectorStore
    embedder = BgeEmbedder(embed_model, device=device, weights=weights, vocab=vocab)
    if corpus_path and os.path.isdir(corpus_path):
        store = DeviceVectorStore.load(corpus_path, device=device)
        logger.info(f"loaded collection snapshot {corpus_path}: {store.size} points")
    else:
        store = DeviceVectorStore(embedder.dim, device=device)
        if corpus_path:
            stats = CorpusIngestor(embedder, store).ingest(iter_documents(corpus_path))
            logger.info(f"ingested {corpus_path}: {stats}")
    return embedder, store


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--input", required=True, help="jsonl / json / parquet documents")
    ap.add_argument("--snapshot", default="", help="directory to write the collection snapshot to")
    ap.add_argument("--embed-model", default="bge-base-en")
    ap.add_argument("--weights", default=None)
    ap.add_argument("--vocab", default=None)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args(argv)
    from .embedder import BgeEmbedder
    from .store import DeviceVectorStore
    emb = BgeEmbedder(a.embed_model, device=a.device, weights=a.weights, vocab=a.vocab)
    store = DeviceVectorStore(emb.dim, device=a.device)
    stats = CorpusIngestor(emb, store, batch_size=a.batch).ingest(iter_documents(a.input))
    if a.snapshot:
        store.save(a.snapshot)
    print(json.dumps({"input": a.input, **stats, "size": store.size, "snapshot": a.snapshot or None}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
