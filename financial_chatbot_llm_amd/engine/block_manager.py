"""Paged-KV block allocator with automatic prefix caching.

HBM is carved into 64-token blocks (one attention KV tile each).  A FULL block is identified by
a chained hash ``h_i = H(h_{i-1}, tokens of block i)``, so equal prefixes map to equal block
sequences and are computed once: every turn's decide prompt (tools + date + TOOL_PROMPT) and
respond prompt (date + SYSTEM_PROMPT) share ~1k leading tokens across all users, and turn n+1
of a conversation re-uses turn n's KV (SURVEY §3.2 latency structure, §5.4).

Blocks whose reference count drops to zero keep their hash and stay resident in an LRU
"evictable" pool; they are only recycled when the free list is empty.  This is the Python
implementation; ``_penny_runtime.BlockManager`` (C++, csrc/runtime) implements the same
interface and is used when built (``make_block_manager``).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Sequence as Seq

from .sequence import Sequence


def block_hash(parent: int, tokens: Seq[int]) -> int:
    return hash((parent, tuple(tokens)))


class PyBlockManager:
    def __init__(self, num_blocks: int, block_size: int = 64, enable_prefix_caching: bool = True):
        self.num_blocks, self.block_size = num_blocks, block_size
        self.enable_prefix_caching = enable_prefix_caching
        self.ref = [0] * num_blocks
        self.hash_of: List[Optional[int]] = [None] * num_blocks
        self.cache: Dict[int, int] = {}
        self.evictable: "OrderedDict[int, None]" = OrderedDict()
        self.free_list: List[int] = list(range(num_blocks - 1, -1, -1))
        self.seq_hashes: Dict[int, List[int]] = {}
        self.hits = 0
        self.queries = 0
        self.evictions = 0          # cached blocks recycled (their prefix KV lost)

    # -- capacity ------------------------------------------------------------------------
    def num_free(self) -> int:
        return len(self.free_list) + len(self.evictable)

    def usage(self) -> float:
        return 1.0 - self.num_free() / max(self.num_blocks, 1)

    def blocks_needed(self, seq: Sequence, total_tokens: int) -> int:
        need = (total_tokens + self.block_size - 1) // self.block_size
        return max(0, need - len(seq.block_table))

    def _alloc(self) -> int:
        if self.free_list:
            b = self.free_list.pop()
        elif self.evictable:
            b, _ = self.evictable.popitem(last=False)
            self.evictions += 1
            h = self.hash_of[b]
            if h is not None and self.cache.get(h) == b:
                del self.cache[h]
            self.hash_of[b] = None
        else:
            raise MemoryError("out of KV blocks")
        self.ref[b] = 1
        return b

    # -- sequence lifecycle ----------------------------------------------------------------
    def match_prefix(self, seq: Sequence) -> int:
        """Attach cached full blocks of the prompt; returns the number of cached tokens.  At
        least one token is always left to compute (its logits start decoding)."""
        hashes: List[int] = []
        self.seq_hashes[seq.seq_id] = hashes
        if not self.enable_prefix_caching or seq.block_table:
            return 0
        ids = seq.all_ids
        bs = self.block_size
        max_full = (len(ids) - 1) // bs
        parent = 0
        self.queries += max_full
        for i in range(max_full):
            h = block_hash(parent, ids[i * bs:(i + 1) * bs])
            b = self.cache.get(h)
            if b is None:
                break
            if self.ref[b] == 0:
                self.evictable.pop(b, None)
            self.ref[b] += 1
            seq.block_table.append(b)
            hashes.append(h)
            parent = h
            self.hits += 1
        seq.num_computed = len(seq.block_table) * bs
        seq.num_cached_prompt = seq.num_computed
        return seq.num_computed

    def can_grow(self, seq: Sequence, total_tokens: int) -> bool:
        return self.blocks_needed(seq, total_tokens) <= self.num_free()

    def grow(self, seq: Sequence, total_tokens: int) -> bool:
        n = self.blocks_needed(seq, total_tokens)
        if n > self.num_free():
            return False
        for _ in range(n):
            seq.block_table.append(self._alloc())
        return True

    def commit(self, seq: Sequence) -> None:
        """Register hashes for blocks that became full and computed."""
        if not self.enable_prefix_caching:
            return
        hashes = self.seq_hashes.setdefault(seq.seq_id, [])
        bs = self.block_size
        full = min(seq.num_computed // bs, len(seq.block_table))
        if len(hashes) >= full:
            return
        ids = seq.all_ids
        parent = hashes[-1] if hashes else 0
        for i in range(len(hashes), full):
            h = block_hash(parent, ids[i * bs:(i + 1) * bs])
            b = seq.block_table[i]
            if h not in self.cache and self.hash_of[b] is None:
                self.cache[h] = b
                self.hash_of[b] = h
            hashes.append(h)
            parent = h

    def free(self, seq: Sequence, evict_first: bool = False) -> None:
        """Release ``seq``'s blocks.  ``evict_first``: the blocks it computed itself (everything
        after its prefix-cache hit) are KV nobody will ask for again -- a prompt built around a
        one-off retrieval context -- so they go to the FRONT of the eviction order (tail first)
        instead of pushing still-useful prefixes out (an LRU over a cyclic working set slightly
        larger than HBM would otherwise evict exactly what the next turn needs)."""
        table = seq.block_table
        keep = min(seq.num_cached_prompt // self.block_size, len(table)) if evict_first else len(table)
        for b in table[keep:]:
            self.ref[b] -= 1
            if self.ref[b] == 0:
                if self.hash_of[b] is not None:
                    self.evictable[b] = None
                    self.evictable.move_to_end(b, last=False)
                else:
                    self.free_list.append(b)
        for b in reversed(table[:keep]):
            self.ref[b] -= 1
            if self.ref[b] == 0:
                if self.hash_of[b] is not None:
                    self.evictable[b] = None
                else:
                    self.free_list.append(b)
        seq.block_table = []
        self.seq_hashes.pop(seq.seq_id, None)

    def hit_rate(self) -> float:
        return self.hits / max(self.queries, 1)


def make_block_manager(num_blocks: int, block_size: int = 64, enable_prefix_caching: bool = True,
                       prefer_native: bool = True):
    if prefer_native:
        try:
            from .native_block_manager import NativeBlockManager
            return NativeBlockManager(num_blocks, block_size, enable_prefix_caching)
        except Exception:  # noqa: BLE001 - native runtime not built
            pass
    return PyBlockManager(num_blocks, block_size, enable_prefix_caching)
