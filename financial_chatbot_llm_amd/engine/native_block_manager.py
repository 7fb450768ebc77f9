"""Engine-facing wrapper of the C++ block allocator (``csrc/runtime/block_manager.cpp``).

Same interface as :class:`~.block_manager.PyBlockManager` (the scheduler is agnostic), but the
allocator state, prefix-cache map and LRU live in C++.  Only O(new blocks) data crosses the
boundary per call: ``grow`` returns the appended block ids and ``commit`` ships just the tokens
of blocks that became full since the last commit.
"""
from __future__ import annotations

from .sequence import Sequence


class NativeBlockManager:
    def __init__(self, num_blocks: int, block_size: int = 64, enable_prefix_caching: bool = True):
        from .. import _penny_runtime as rt  # built in-tree by _build.build_runtime()
        self.core = rt.BlockAllocator(num_blocks, block_size, enable_prefix_caching)
        self.num_blocks, self.block_size = num_blocks, block_size
        self.enable_prefix_caching = enable_prefix_caching

    @property
    def hits(self) -> int:
        return self.core.hits

    @property
    def queries(self) -> int:
        return self.core.queries

    @property
    def evictions(self) -> int:
        return self.core.evictions

    def num_free(self) -> int:
        return self.core.num_free()

    def usage(self) -> float:
        return self.core.usage()

    def hit_rate(self) -> float:
        return self.core.hits / max(self.core.queries, 1)

    def blocks_needed(self, seq: Sequence, total_tokens: int) -> int:
        return self.core.blocks_needed(seq.seq_id, total_tokens)

    def can_grow(self, seq: Sequence, total_tokens: int) -> bool:
        return self.core.blocks_needed(seq.seq_id, total_tokens) <= self.core.num_free()

    def match_prefix(self, seq: Sequence) -> int:
        if seq.block_table:
            return 0
        seq.block_table = list(self.core.match_prefix(seq.seq_id, seq.all_ids))
        seq.num_computed = len(seq.block_table) * self.block_size
        seq.num_cached_prompt = seq.num_computed
        return seq.num_computed

    def grow(self, seq: Sequence, total_tokens: int) -> bool:
        added = self.core.grow(seq.seq_id, total_tokens)
        if added and added[0] < 0:
            return False
        seq.block_table.extend(added)
        return True

    def commit(self, seq: Sequence) -> None:
        if not self.enable_prefix_caching:
            return
        bs = self.block_size
        done = self.core.num_committed(seq.seq_id)
        full = min(seq.num_computed // bs, len(seq.block_table))
        if full > done:
            self.core.commit(seq.seq_id, done, seq.all_ids[done * bs:full * bs])

    def free(self, seq: Sequence, evict_first: bool = False) -> None:
        keep = seq.num_cached_prompt // self.block_size if evict_first else -1
        self.core.free(seq.seq_id, keep)
        seq.block_table = []
