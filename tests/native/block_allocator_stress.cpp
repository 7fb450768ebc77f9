// Randomised stress of the native paged-KV block allocator (csrc/runtime/block_allocator.h),
// built by tests/test_native_sanitizers.py with -fsanitize=address,undefined (a
// sanitizer build of the C++ host code).  It drives the engine's call pattern -- match_prefix on
// admission, grow per step, commit of newly full blocks, free on finish/preemption -- over
// prompts that share random-length prefixes, and after every operation audits the allocator's
// invariants plus the two properties the engine relies on:
//   * a block is never owned by two sequences unless it is a verified shared-prefix hit;
//   * every prefix hit's block holds exactly the tokens of the prompt it was matched for.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <set>
#include <vector>

#include "block_allocator.h"

using penny::BlockAllocator;

struct Live {
  std::vector<int32_t> tokens;  // prompt + generated so far
  int computed = 0;             // tokens whose KV is "written"
  int committed = 0;            // full blocks registered with commit()
  std::map<int, std::vector<int32_t>> content;  // block id -> tokens this seq wrote/matched there
};

#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, "\n");                          \
      return 1;                                            \
    }                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  const int bs = 16, nblocks = 96;
  std::mt19937 rng(1234);
  BlockAllocator a(nblocks, bs, true);
  std::vector<std::vector<int32_t>> prefixes;
  for (int p = 0; p < 4; ++p) {
    std::vector<int32_t> t(bs * (2 + p));
    for (auto& x : t) x = (int32_t)(rng() % 1000);
    prefixes.push_back(t);
  }
  std::map<int, Live> live;
  int next_id = 0;
  long hits_seen = 0;
  for (int it = 0; it < iters; ++it) {
    const int op = rng() % 10;
    if (op < 3 && live.size() < 12) {  // admit
      Live s;
      const auto& pre = prefixes[rng() % prefixes.size()];
      s.tokens.assign(pre.begin(), pre.begin() + (rng() % (pre.size() + 1)));
      const int extra = 1 + rng() % 40;
      for (int i = 0; i < extra; ++i) s.tokens.push_back((int32_t)(rng() % 1000));
      const int id = next_id++;
      std::vector<int> table = a.match_prefix(id, s.tokens);
      for (size_t i = 0; i < table.size(); ++i) {
        s.content[table[i]] = std::vector<int32_t>(s.tokens.begin() + i * bs, s.tokens.begin() + (i + 1) * bs);
        ++hits_seen;
      }
      s.committed = (int)table.size();
      if (a.grow(id, (int)s.tokens.size()) == std::vector<int>{-1}) {
        a.free(id);  // admission fails: back out the prefix refs
      } else {
        s.computed = (int)s.tokens.size();
        live[id] = s;
      }
    } else if (op < 8 && !live.empty()) {  // decode step for a random seq
      auto itv = live.begin();
      std::advance(itv, rng() % live.size());
      Live& s = itv->second;
      s.tokens.push_back((int32_t)(rng() % 1000));
      if (a.grow(itv->first, (int)s.tokens.size()) == std::vector<int>{-1}) {
        a.free(itv->first);  // preempted
        live.erase(itv);
      } else {
        s.computed = (int)s.tokens.size();
        const int full = s.computed / bs;
        if (full > s.committed) {
          std::vector<int32_t> toks(s.tokens.begin() + s.committed * bs, s.tokens.begin() + full * bs);
          a.commit(itv->first, s.committed, toks);
          s.committed = full;
        }
      }
    } else if (!live.empty()) {  // finish
      auto itv = live.begin();
      std::advance(itv, rng() % live.size());
      a.free(itv->first);
      live.erase(itv);
    }
    const std::string err = a.check_invariants();
    CHECK(err.empty(), "iteration %d: %s", it, err.c_str());
    // ownership: a block held by two live seqs must be a shared prefix block with equal tokens
    std::map<int, int> owner;
    for (auto& kv : live) {
      const std::vector<int> t = a.table(kv.first);
      CHECK((int)t.size() * bs >= (int)kv.second.tokens.size(), "table too short");
      for (size_t i = 0; i < t.size(); ++i) {
        auto o = owner.find(t[i]);
        if (o == owner.end()) {
          owner[t[i]] = kv.first;
          continue;
        }
        const Live& other = live[o->second];
        const size_t lo = i * bs, hi = (i + 1) * bs;
        CHECK(hi <= kv.second.tokens.size() && hi <= other.tokens.size(), "shared block %d not full", t[i]);
        for (size_t j = lo; j < hi; ++j)
          CHECK(kv.second.tokens[j] == other.tokens[j], "shared block %d holds different tokens", t[i]);
      }
    }
    for (auto& kv : live)
      for (auto& bc : kv.second.content) {
        const std::vector<int> t = a.table(kv.first);
        bool found = false;
        for (size_t i = 0; i < t.size(); ++i)
          if (t[i] == bc.first) {
            found = true;
            for (int j = 0; j < bs; ++j) CHECK(kv.second.tokens[i * bs + j] == bc.second[j], "hit block content");
          }
        CHECK(found, "matched block vanished from the table");
      }
  }
  std::printf("ok iters=%d hits=%ld queries=%ld matched_blocks=%ld\n", iters, a.hits(), a.queries(), hits_seen);
  return hits_seen > 0 ? 0 : 2;
}
