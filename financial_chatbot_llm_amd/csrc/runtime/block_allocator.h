// Paged-KV block allocator with automatic prefix caching: pure C++ (no Python), shared by the
// pybind11 module (block_manager.cpp) and the sanitizer stress driver
// (tests/native/block_allocator_stress.cpp, built with -fsanitize=address,undefined).
//
// Native paged-KV block allocator with automatic prefix caching (host side of the engine).
//
// The scheduler calls into this every step for every running sequence (grow by a block, commit
// newly full blocks, free on finish), so it is C++: O(1) allocation from a free stack, an
// intrusive LRU list of evictable cached blocks, and an open hash map from chained block hashes
// to block ids.  Cached blocks keep their token ids so a hash hit is VERIFIED against the actual
// tokens (a collision can never alias two different prefixes' KV).
//
// Block lifecycle: free -> owned (ref >= 1) -> [committed: hashed + cached] -> ref 0 ->
// evictable (still cached, LRU) -> reclaimed when the free stack is empty.
//
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace penny {

inline uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t block_hash(uint64_t parent, const int32_t* toks, int n) {
  uint64_t h = mix(parent ^ 0x243F6A8885A308D3ull);
  for (int i = 0; i < n; ++i) h = mix(h ^ (uint64_t)(uint32_t)toks[i]);
  return h ? h : 1;  // 0 is reserved for "no hash"
}

struct Block {
  int ref = 0;
  uint64_t hash = 0;              // 0: not cached
  std::vector<int32_t> tokens;    // tokens of a cached block (verification)
  int lru_prev = -1, lru_next = -1;
  bool in_lru = false;
};

struct SeqState {
  std::vector<int> table;
  std::vector<uint64_t> hashes;   // chained hashes of committed full blocks
};

class BlockAllocator {
 public:
  BlockAllocator(int num_blocks, int block_size, bool prefix_caching)
      : bs_(block_size), caching_(prefix_caching), blocks_(num_blocks) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad allocator geometry");
    free_.reserve(num_blocks);
    for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
  }

  int num_blocks() const { return (int)blocks_.size(); }
  int num_free() const { return (int)free_.size() + lru_size_; }
  int block_size() const { return bs_; }
  long hits() const { return hits_; }
  long queries() const { return queries_; }
  long evictions() const { return evictions_; }

  int blocks_needed(int seq, int total_tokens) const {
    auto it = seqs_.find(seq);
    const int have = it == seqs_.end() ? 0 : (int)it->second.table.size();
    const int need = (total_tokens + bs_ - 1) / bs_;
    return need > have ? need - have : 0;
  }

  // Attach cached full blocks of `tokens` (never the whole prompt: >= 1 token left to compute).
  std::vector<int> match_prefix(int seq, const std::vector<int32_t>& tokens) {
    SeqState& s = seqs_[seq];
    if (!caching_ || !s.table.empty()) return s.table;
    const int max_full = ((int)tokens.size() - 1) / bs_;
    queries_ += max_full;
    uint64_t parent = 0;
    for (int i = 0; i < max_full; ++i) {
      const int32_t* t = tokens.data() + (size_t)i * bs_;
      const uint64_t h = block_hash(parent, t, bs_);
      auto it = cache_.find(h);
      if (it == cache_.end()) break;
      Block& blk = blocks_[it->second];
      if (!std::equal(blk.tokens.begin(), blk.tokens.end(), t)) break;  // verified hit only
      if (blk.ref == 0) lru_remove(it->second);
      blk.ref += 1;
      s.table.push_back(it->second);
      s.hashes.push_back(h);
      parent = h;
      ++hits_;
    }
    return s.table;
  }

  // Append blocks until the table covers total_tokens; returns the new block ids (empty + false
  // semantics: raises nothing, returns {-1} when the pool cannot satisfy the request).
  std::vector<int> grow(int seq, int total_tokens) {
    const int n = blocks_needed(seq, total_tokens);
    if (n > num_free()) return {-1};
    SeqState& s = seqs_[seq];
    std::vector<int> added;
    added.reserve(n);
    for (int i = 0; i < n; ++i) {
      const int b = alloc();
      s.table.push_back(b);
      added.push_back(b);
    }
    return added;
  }

  // Register hashes for the full blocks [first_block, first_block + nblocks) of `seq`, whose
  // tokens are given contiguously.
  void commit(int seq, int first_block, const std::vector<int32_t>& tokens) {
    if (!caching_) return;
    auto it = seqs_.find(seq);
    if (it == seqs_.end()) return;
    SeqState& s = it->second;
    const int nblocks = (int)tokens.size() / bs_;
    if (first_block != (int)s.hashes.size()) throw std::invalid_argument("commit out of order");
    uint64_t parent = s.hashes.empty() ? 0 : s.hashes.back();
    for (int i = 0; i < nblocks && first_block + i < (int)s.table.size(); ++i) {
      const int32_t* t = tokens.data() + (size_t)i * bs_;
      const uint64_t h = block_hash(parent, t, bs_);
      const int b = s.table[first_block + i];
      Block& blk = blocks_[b];
      if (blk.hash == 0 && cache_.find(h) == cache_.end()) {
        cache_[h] = b;
        blk.hash = h;
        blk.tokens.assign(t, t + bs_);
      }
      s.hashes.push_back(h);
      parent = h;
    }
  }

  int num_committed(int seq) const {
    auto it = seqs_.find(seq);
    return it == seqs_.end() ? 0 : (int)it->second.hashes.size();
  }

  std::vector<int> table(int seq) const {
    auto it = seqs_.find(seq);
    return it == seqs_.end() ? std::vector<int>{} : it->second.table;
  }

  // Release a sequence.  Cached blocks [0, keep_blocks) join the LRU tail (tail block first, so
  // a chain is evicted leaf-first); blocks [keep_blocks, end) -- KV the caller knows will not be
  // asked for again, e.g. a prompt around a one-off retrieval context -- join the LRU HEAD and
  // are recycled before any other cached block.  keep_blocks < 0: keep everything.
  void free(int seq, int keep_blocks = -1) {
    auto it = seqs_.find(seq);
    if (it == seqs_.end()) return;
    const std::vector<int>& t = it->second.table;
    const int n = (int)t.size();
    const int keep = keep_blocks < 0 ? n : std::min(keep_blocks, n);
    for (int i = keep; i < n; ++i) {  // forward + push-front: the tail ends up first in line
      Block& blk = blocks_[t[i]];
      if (--blk.ref == 0) {
        if (blk.hash) lru_push_front(t[i]);
        else free_.push_back(t[i]);
      }
    }
    for (int i = keep - 1; i >= 0; --i) {  // tail first: later blocks evict first
      Block& blk = blocks_[t[i]];
      if (--blk.ref == 0) {
        if (blk.hash) lru_push_back(t[i]);
        else free_.push_back(t[i]);
      }
    }
    seqs_.erase(it);
  }

  double usage() const { return 1.0 - (double)num_free() / (double)blocks_.size(); }

  // Full structural audit (tests / debug builds): "" when consistent, else the first violation.
  // Every block is exactly one of free (ref 0), evictable-cached (ref 0, hashed, in the LRU) or
  // owned (ref == number of sequence tables holding it); the hash map and LRU links agree.
  std::string check_invariants() const {
    const int nb = (int)blocks_.size();
    std::vector<int> refs(nb, 0), in_free(nb, 0);
    for (const auto& kv : seqs_)
      for (int b : kv.second.table) {
        if (b < 0 || b >= nb) return "table holds out-of-range block";
        ++refs[b];
      }
    for (int b : free_) {
      if (b < 0 || b >= nb) return "free stack holds out-of-range block";
      if (in_free[b]++) return "block twice on the free stack";
    }
    int lru_count = 0, prev = -1;
    for (int b = lru_head_; b >= 0; b = blocks_[b].lru_next) {
      if (++lru_count > nb) return "LRU cycle";
      if (!blocks_[b].in_lru || blocks_[b].lru_prev != prev) return "LRU links broken";
      prev = b;
    }
    if (prev != lru_tail_ || lru_count != lru_size_) return "LRU tail/size mismatch";
    for (int b = 0; b < nb; ++b) {
      const Block& blk = blocks_[b];
      if (blk.ref != refs[b]) return "refcount != table occurrences (block " + std::to_string(b) + ")";
      const int states = (in_free[b] ? 1 : 0) + (blk.in_lru ? 1 : 0) + (blk.ref > 0 ? 1 : 0);
      if (states != 1) return "block in " + std::to_string(states) + " states (block " + std::to_string(b) + ")";
      if (blk.in_lru && blk.hash == 0) return "unhashed block on the LRU";
      if (blk.hash) {
        auto it = cache_.find(blk.hash);
        if (it == cache_.end() || it->second != b) return "hashed block missing from the cache map";
        if ((int)blk.tokens.size() != bs_) return "cached block without its tokens";
      }
    }
    for (const auto& kv : cache_)
      if (kv.second < 0 || kv.second >= nb || blocks_[kv.second].hash != kv.first) return "stale cache entry";
    return "";
  }

 private:
  int alloc() {
    int b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else if (lru_head_ >= 0) {
      b = lru_head_;
      lru_remove(b);
      ++evictions_;
      Block& blk = blocks_[b];
      auto it = cache_.find(blk.hash);
      if (it != cache_.end() && it->second == b) cache_.erase(it);
      blk.hash = 0;
      blk.tokens.clear();
    } else {
      throw std::runtime_error("out of KV blocks");
    }
    blocks_[b].ref = 1;
    return b;
  }

  void lru_push_back(int b) {
    Block& blk = blocks_[b];
    blk.lru_prev = lru_tail_;
    blk.lru_next = -1;
    if (lru_tail_ >= 0) blocks_[lru_tail_].lru_next = b;
    else lru_head_ = b;
    lru_tail_ = b;
    blk.in_lru = true;
    ++lru_size_;
  }

  void lru_push_front(int b) {
    Block& blk = blocks_[b];
    blk.lru_prev = -1;
    blk.lru_next = lru_head_;
    if (lru_head_ >= 0) blocks_[lru_head_].lru_prev = b;
    else lru_tail_ = b;
    lru_head_ = b;
    blk.in_lru = true;
    ++lru_size_;
  }

  void lru_remove(int b) {
    Block& blk = blocks_[b];
    if (!blk.in_lru) return;
    if (blk.lru_prev >= 0) blocks_[blk.lru_prev].lru_next = blk.lru_next;
    else lru_head_ = blk.lru_next;
    if (blk.lru_next >= 0) blocks_[blk.lru_next].lru_prev = blk.lru_prev;
    else lru_tail_ = blk.lru_prev;
    blk.lru_prev = blk.lru_next = -1;
    blk.in_lru = false;
    --lru_size_;
  }

  int bs_;
  bool caching_;
  std::vector<Block> blocks_;
  std::vector<int> free_;
  std::unordered_map<uint64_t, int> cache_;
  std::unordered_map<int, SeqState> seqs_;
  int lru_head_ = -1, lru_tail_ = -1, lru_size_ = 0;
  long hits_ = 0, queries_ = 0, evictions_ = 0;
};

}  // namespace penny

