// Native byte-pair-encoding merge loop (host C++).
//
// Python (engine/tokenizer.py) does the regex pre-tokenisation; this file
// merges each pre-token by rank exactly like tiktoken's `_byte_pair_merge`:
// repeatedly fuse the adjacent pair whose concatenation has the lowest rank.
// A per-handle piece cache makes repeated words O(1); the cache is guarded by
// a mutex so one tokenizer can be shared by several Python threads.
//
// C ABI (ctypes):
//   void*   mrsum_bpe_create(const char* blob, const int32_t* lens, const int32_t* ranks, int32_t n)
//   void    mrsum_bpe_destroy(void*)
//   int64_t mrsum_bpe_encode_pieces(void*, const char* blob, const int32_t* offsets /*n+1*/,
//                                   int32_t n, int32_t* out, int64_t cap)
// returns the number of ids written, or -1 if a byte is missing from the
// vocabulary / the output buffer is too small.

#include <cstdint>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace {

struct BPE {
  std::unordered_map<std::string, int32_t> ranks;
  std::unordered_map<std::string, std::vector<int32_t>> cache;
  std::mutex mu;
};

constexpr int32_t kNone = std::numeric_limits<int32_t>::max();

inline int32_t rank_of(const BPE& b, const char* p, size_t n) {
  auto it = b.ranks.find(std::string(p, n));
  return it == b.ranks.end() ? kNone : it->second;
}

// parts[i] = start byte of part i; parts.back() = piece length.
bool merge_piece(const BPE& b, const char* s, size_t n, std::vector<int32_t>& out) {
  if (n == 0) return true;
  int32_t whole = rank_of(b, s, n);
  if (whole != kNone) { out.push_back(whole); return true; }
  std::vector<size_t> start(n + 1);
  for (size_t i = 0; i <= n; ++i) start[i] = i;
  // pair_rank[i] = rank of parts i and i+1 fused
  std::vector<int32_t> pair_rank(n, kNone);
  auto pr = [&](size_t i) -> int32_t {
    if (i + 2 >= start.size()) return kNone;
    return rank_of(b, s + start[i], start[i + 2] - start[i]);
  };
  for (size_t i = 0; i + 1 < n; ++i) pair_rank[i] = pr(i);
  pair_rank.resize(start.size() - 1);
  while (start.size() > 2) {
    int32_t best = kNone;
    size_t bi = 0;
    for (size_t i = 0; i + 1 < start.size() - 1; ++i)
      if (pair_rank[i] < best) { best = pair_rank[i]; bi = i; }
    if (best == kNone) break;
    start.erase(start.begin() + bi + 1);
    pair_rank.erase(pair_rank.begin() + bi + 1);
    pair_rank[bi] = pr(bi);
    if (bi > 0) pair_rank[bi - 1] = pr(bi - 1);
  }
  for (size_t i = 0; i + 1 < start.size(); ++i) {
    int32_t r = rank_of(b, s + start[i], start[i + 1] - start[i]);
    if (r == kNone) return false;
    out.push_back(r);
  }
  return true;
}

}  // namespace

extern "C" {

void* mrsum_bpe_create(const char* blob, const int32_t* lens, const int32_t* ranks, int32_t n) {
  auto* b = new BPE();
  b->ranks.reserve(static_cast<size_t>(n) * 2);
  size_t off = 0;
  for (int32_t i = 0; i < n; ++i) {
    b->ranks.emplace(std::string(blob + off, lens[i]), ranks[i]);
    off += lens[i];
  }
  return b;
}

void mrsum_bpe_destroy(void* h) { delete static_cast<BPE*>(h); }

int64_t mrsum_bpe_encode_pieces(void* h, const char* blob, const int32_t* offsets, int32_t n, int32_t* out,
                                int64_t cap) {
  auto* b = static_cast<BPE*>(h);
  int64_t m = 0;
  std::vector<int32_t> tmp;
  for (int32_t i = 0; i < n; ++i) {
    const char* p = blob + offsets[i];
    size_t len = static_cast<size_t>(offsets[i + 1] - offsets[i]);
    std::string key(p, len);
    const std::vector<int32_t>* ids = nullptr;
    {
      std::lock_guard<std::mutex> g(b->mu);
      auto it = b->cache.find(key);
      if (it != b->cache.end()) ids = &it->second;
      if (ids) {
        if (m + static_cast<int64_t>(ids->size()) > cap) return -1;
        std::memcpy(out + m, ids->data(), ids->size() * sizeof(int32_t));
        m += static_cast<int64_t>(ids->size());
        continue;
      }
    }
    tmp.clear();
    if (!merge_piece(*b, p, len, tmp)) return -1;
    if (m + static_cast<int64_t>(tmp.size()) > cap) return -1;
    std::memcpy(out + m, tmp.data(), tmp.size() * sizeof(int32_t));
    m += static_cast<int64_t>(tmp.size());
    std::lock_guard<std::mutex> g(b->mu);
    if (b->cache.size() < 1000000) b->cache.emplace(std::move(key), tmp);
  }
  return m;
}

}  // extern "C"
