"""Vector stores replacing the remote Qdrant collection (reference ``tools/qdrant_tool.py:98-153``).

Point layout follows langchain-qdrant's default: each row has a dense
vector and a payload ``{"page_content": str, "metadata": {"user_id": str, "date": int, ...}}``.

Two implementations share one batched API, ``search_batch(qvecs, user_ids, date_gte, limits)``:

* :class:`NumpyVectorStore` -- exact brute force on the host (CPU plumbing config, tests).
* :class:`DeviceVectorStore` -- the corpus lives in HBM as L2-normalised bf16 rows with int32
  user codes and int64 dates; ``ops.retrieval.filtered_topk`` (HIP, K15) evaluates the
  ``user_id == u AND date >= t`` filter, scores only matching rows, and selects the top-k per
  query on the GPU.  Retrieval never leaves HBM except for the final (row, score) lists.

Both are exact (the reference uses HNSW with ``hnsw_ef=128, exact=False``; exact search is a
superset of its recall).  Similarity is the inner product of normalised vectors (cosine).
"""
from __future__ import annotations

import datetime as _dt
import hashlib
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np

from ..utils.logging import get_logger

logger = get_logger(__name__)

MERCHANTS = [
    ("Whole Foods", "Groceries"), ("Trader Joe's", "Groceries"), ("Safeway", "Groceries"),
    ("Shell", "Gas"), ("Chevron", "Gas"), ("Netflix", "Entertainment"), ("Spotify", "Entertainment"),
    ("AMC Theatres", "Entertainment"), ("Starbucks", "Dining"), ("Chipotle", "Dining"),
    ("Uber", "Transportation"), ("Lyft", "Transportation"), ("Amazon", "Shopping"),
    ("Target", "Shopping"), ("Costco", "Shopping"), ("PG&E", "Utilities"), ("Comcast", "Utilities"),
    ("Landlord LLC", "Rent"), ("CVS Pharmacy", "Health"), ("Equinox", "Fitness"),
    ("Delta Air Lines", "Travel"), ("Airbnb", "Travel"), ("Geico", "Insurance"), ("Venmo", "Transfer"),
]


@dataclass
class Hit:
    id: int
    score: float
    payload: Optional[Dict[str, Any]]


def synthetic_payload(row: int, user_id: str, date: int) -> Dict[str, Any]:
    """Deterministic plaid-like transaction text for synthetic corpora."""
    h = int.from_bytes(hashlib.blake2b(row.to_bytes(8, "little"), digest_size=8).digest(), "little")
    merchant, category = MERCHANTS[h % len(MERCHANTS)]
    amount = ((h >> 8) % 40000) / 100.0 + 1.0
    day = _dt.datetime.fromtimestamp(date).strftime("%Y-%m-%d")
    text = f"Date: {day} | Merchant: {merchant} | Amount: ${amount:.2f} | Category: {category}"
    return {"page_content": text, "metadata": {"user_id": user_id, "date": int(date),
                                               "merchant": merchant, "category": category,
                                               "amount": amount}}


class Corpus:
    """Host-side mirror of a collection: ids, user codes, dates, payload provider.

    Arrays grow by doubling (bulk ingest appends thousands of batches), payloads are stored
    per row or generated (``payload_fn``) for synthetic corpora."""

    def __init__(self, dim: int):
        self.dim = dim
        self.user_to_code: Dict[str, int] = {}
        self.code_to_user: List[str] = []
        self._codes = np.zeros((0,), np.int32)
        self._dates = np.zeros((0,), np.int64)
        self._n = 0
        self._payloads: List[Optional[Dict[str, Any]]] = []
        self.payload_fn: Optional[Callable[[int], Dict[str, Any]]] = None
        self.synthetic: Optional[Dict[str, int]] = None   # how payload_fn was built (snapshots)

    @property
    def user_codes(self) -> np.ndarray:
        return self._codes[: self._n]

    @user_codes.setter
    def user_codes(self, v) -> None:
        self._codes = np.asarray(v, np.int32)
        self._n = int(self._codes.shape[0])

    @property
    def dates(self) -> np.ndarray:
        return self._dates[: self._n]

    @dates.setter
    def dates(self, v) -> None:
        self._dates = np.asarray(v, np.int64)

    def __len__(self) -> int:
        return self._n

    def code(self, user_id: str, create: bool = False) -> int:
        c = self.user_to_code.get(user_id)
        if c is None and create:
            c = len(self.code_to_user)
            self.user_to_code[user_id] = c
            self.code_to_user.append(user_id)
        return -1 if c is None else c

    def append(self, user_ids: Sequence[str], dates: Sequence[int], payloads: Sequence[Optional[Dict[str, Any]]]) -> np.ndarray:
        codes = np.array([self.code(u, create=True) for u in user_ids], np.int32)
        n, start = len(codes), self._n
        if start + n > self._codes.shape[0]:
            cap = max(start + n, 2 * self._codes.shape[0], 1024)
            c2, d2 = np.zeros(cap, np.int32), np.zeros(cap, np.int64)
            c2[:start], d2[:start] = self._codes[:start], self._dates[:start]
            self._codes, self._dates = c2, d2
        self._codes[start:start + n] = codes
        self._dates[start:start + n] = np.asarray(dates, np.int64)
        self._n = start + n
        if len(self._payloads) < start:
            self._payloads.extend([None] * (start - len(self._payloads)))
        self._payloads.extend(payloads)
        return np.arange(start, start + n)

    def payload(self, row: int) -> Optional[Dict[str, Any]]:
        if row < len(self._payloads) and self._payloads[row] is not None:
            return self._payloads[row]
        if self.payload_fn is not None:
            return self.payload_fn(row)
        return None


def synthetic_metadata(n: int, num_users: int, seed: int = 0, now: Optional[int] = None,
                       horizon_days: int = 365):
    """Random user assignment and dates for an ``n``-row synthetic corpus."""
    rng = np.random.default_rng(seed)
    now = int(_dt.datetime.now().timestamp()) if now is None else now
    users = rng.integers(0, num_users, size=n).astype(np.int32)
    dates = (now - rng.integers(0, horizon_days * 86400, size=n)).astype(np.int64)
    return users, dates


def user_name(i: int) -> str:
    return f"user-{i:06d}"


class VectorStoreBase:
    corpus: Corpus

    def search_batch(self, qvecs, user_ids: Sequence[str], date_gte: Sequence[Optional[int]],
                     limits: Sequence[int]) -> List[List[Hit]]:
        raise NotImplementedError

    def _hits(self, rows, scores) -> List[Hit]:
        return [Hit(int(r), float(s), self.corpus.payload(int(r))) for r, s in zip(rows, scores)]


class NumpyVectorStore(VectorStoreBase):
    def __init__(self, dim: int):
        self.corpus = Corpus(dim)
        self.vectors = np.zeros((0, dim), np.float32)

    def add(self, vectors: np.ndarray, user_ids: Sequence[str], dates: Sequence[int],
            payloads: Sequence[Optional[Dict[str, Any]]]) -> None:
        v = np.asarray(vectors, np.float32)
        v = v / np.maximum(np.linalg.norm(v, axis=1, keepdims=True), 1e-12)
        self.vectors = np.concatenate([self.vectors, v])
        self.corpus.append(user_ids, dates, payloads)

    def search_batch(self, qvecs, user_ids, date_gte, limits):
        q = np.asarray(qvecs, np.float32)
        q = q / np.maximum(np.linalg.norm(q, axis=1, keepdims=True), 1e-12)
        out = []
        for i in range(q.shape[0]):
            code = self.corpus.code(user_ids[i])
            mask = self.corpus.user_codes == code
            if date_gte[i] is not None:
                mask &= self.corpus.dates >= date_gte[i]
            rows = np.nonzero(mask)[0]
            if code < 0 or rows.size == 0:
                out.append([])
                continue
            s = self.vectors[rows] @ q[i]
            order = np.argsort(-s, kind="stable")[: int(limits[i])]
            out.append(self._hits(rows[order], s[order]))
        return out


class DeviceVectorStore(VectorStoreBase):
    """HBM-resident corpus searched by the HIP filtered top-k kernel (K15)."""

    def __init__(self, dim: int, device: str = "cuda", capacity: int = 0):
        import torch
        self.torch = torch
        self.device = torch.device(device)
        self.corpus = Corpus(dim)
        self.vectors = torch.empty((capacity, dim), dtype=torch.bfloat16, device=self.device)
        self.user_codes = torch.empty((capacity,), dtype=torch.int32, device=self.device)
        self.dates = torch.empty((capacity,), dtype=torch.int64, device=self.device)
        self.size = 0

    def _ensure(self, n: int) -> None:
        torch = self.torch
        if n <= self.vectors.shape[0]:
            return
        cap = max(n, 2 * self.vectors.shape[0], 1024)
        for name, dt, shape in (("vectors", torch.bfloat16, (cap, self.corpus.dim)),
                                ("user_codes", torch.int32, (cap,)), ("dates", torch.int64, (cap,))):
            old = getattr(self, name)
            new = torch.empty(shape, dtype=dt, device=self.device)
            new[: self.size] = old[: self.size]
            setattr(self, name, new)

    def add(self, vectors, user_ids, dates, payloads) -> None:
        torch = self.torch
        v = torch.as_tensor(vectors, device=self.device, dtype=torch.float32)
        v = torch.nn.functional.normalize(v, dim=-1)
        rows = self.corpus.append(user_ids, dates, payloads)
        n = len(rows)
        self._ensure(self.size + n)
        self.vectors[self.size: self.size + n] = v.to(torch.bfloat16)
        self.user_codes[self.size: self.size + n] = torch.as_tensor(self.corpus.user_codes[rows], device=self.device)
        self.dates[self.size: self.size + n] = torch.as_tensor(self.corpus.dates[rows], device=self.device)
        self.size += n

    def load_synthetic(self, n: int, num_users: int, seed: int = 0, now: Optional[int] = None,
                       chunk: int = 1 << 18) -> None:
        """Fill the store with ``n`` random unit vectors (generated on device) and metadata."""
        torch = self.torch
        users, dates = synthetic_metadata(n, num_users, seed, now)
        self.corpus.user_to_code = {user_name(i): i for i in range(num_users)}
        self.corpus.code_to_user = [user_name(i) for i in range(num_users)]
        self.corpus.user_codes = users
        self.corpus.dates = dates
        self.corpus._payloads = []
        self.corpus.payload_fn = lambda r: synthetic_payload(r, user_name(int(users[r])), int(dates[r]))
        self.corpus.synthetic = {"n": int(n), "num_users": int(num_users), "seed": int(seed)}
        self._ensure(n)
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            x = torch.randn((e - s, self.corpus.dim), generator=g, device=self.device, dtype=torch.float32)
            self.vectors[s:e] = torch.nn.functional.normalize(x, dim=-1).to(torch.bfloat16)
        self.user_codes[:n] = torch.as_tensor(users, device=self.device)
        self.dates[:n] = torch.as_tensor(dates, device=self.device)
        self.size = n

    # -- snapshots (safetensors + JSON sidecars; no pickles) -----------------------------
    def save(self, path: str) -> None:
        """Write the collection to ``path/``: ``vectors.safetensors`` (bf16 rows, int32 user
        codes, int64 dates), ``corpus.json`` (user ids, synthetic recipe) and, for ingested
        rows, ``payloads.jsonl`` (one payload per row)."""
        import json
        import os

        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        n = self.size
        save_file({"vectors": self.vectors[:n].cpu().contiguous(), "user_codes": self.user_codes[:n].cpu().contiguous(),
                   "dates": self.dates[:n].cpu().contiguous()}, os.path.join(path, "vectors.safetensors"))
        meta = {"dim": self.corpus.dim, "size": n, "users": self.corpus.code_to_user,
                "synthetic": self.corpus.synthetic}
        with open(os.path.join(path, "corpus.json"), "w") as fh:
            json.dump(meta, fh)
        if self.corpus._payloads:
            with open(os.path.join(path, "payloads.jsonl"), "w") as fh:
                for r in range(n):
                    fh.write(json.dumps(self.corpus._payloads[r] if r < len(self.corpus._payloads) else None) + "\n")

    @classmethod
    def load(cls, path: str, device: str = "cuda") -> "DeviceVectorStore":
        import json
        import os

        from safetensors import safe_open
        with open(os.path.join(path, "corpus.json")) as fh:
            meta = json.load(fh)
        st = cls(meta["dim"], device=device)
        with safe_open(os.path.join(path, "vectors.safetensors"), framework="pt") as fh:
            vec, codes, dates = fh.get_tensor("vectors"), fh.get_tensor("user_codes"), fh.get_tensor("dates")
        n = int(meta["size"])
        st._ensure(n)
        st.vectors[:n] = vec.to(st.device)
        st.user_codes[:n] = codes.to(st.device)
        st.dates[:n] = dates.to(st.device)
        st.size = n
        c = st.corpus
        c.code_to_user = list(meta["users"])
        c.user_to_code = {u: i for i, u in enumerate(c.code_to_user)}
        c.user_codes, c.dates = codes.numpy(), dates.numpy()
        syn = meta.get("synthetic")
        if syn:
            users, ds = c.user_codes, c.dates
            c.payload_fn = lambda r: synthetic_payload(r, user_name(int(users[r])), int(ds[r]))
            c.synthetic = syn
        ppath = os.path.join(path, "payloads.jsonl")
        if os.path.exists(ppath):
            with open(ppath) as fh:
                c._payloads = [json.loads(line) for line in fh]
        return st

    def search_batch(self, qvecs, user_ids, date_gte, limits):
        from ..ops.retrieval import filtered_topk
        torch = self.torch
        q = torch.as_tensor(qvecs, device=self.device, dtype=torch.float32)
        q = torch.nn.functional.normalize(q, dim=-1).to(torch.bfloat16)
        codes = torch.tensor([self.corpus.code(u) for u in user_ids], dtype=torch.int32)
        floors = torch.tensor([(-(1 << 62)) if d is None else int(d) for d in date_gte], dtype=torch.int64)
        ks = torch.tensor([int(k) for k in limits], dtype=torch.int32)
        ids, scores, counts = filtered_topk(self.vectors[: self.size], self.user_codes[: self.size],
                                            self.dates[: self.size], q, codes.to(self.device),
                                            floors.to(self.device), ks.to(self.device), int(ks.max().item()))
        ids, scores, counts = ids.cpu().numpy(), scores.cpu().numpy(), counts.cpu().numpy()
        return [self._hits(ids[i, : counts[i]], scores[i, : counts[i]]) for i in range(q.shape[0])]
