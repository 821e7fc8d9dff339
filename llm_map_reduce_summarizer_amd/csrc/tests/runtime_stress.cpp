// Multi-threaded stress of the host runtime (csrc/runtime: KV page allocator, BPE merge loop), built
// and run under AddressSanitizer + UndefinedBehaviorSanitizer and, separately, ThreadSanitizer by
// tests/test_runtime_sanitizers.py (SURVEY.md §5.2 race detection: the engine shares one allocator
// and one tokenizer across Python threads; both guard their state with a mutex -- this checks it).
//
//   pages: T threads allocate / free random page runs; a shared owner table (atomics) proves no page
//          is ever handed to two owners, foreign and double frees are rejected, and every page is
//          back on the free list at the end.
//   bpe:   T threads encode the same pre-tokens concurrently (cache hits and misses racing) and must
//          all produce the single-threaded ids.
// Exit status 0 = pass; the sanitizers abort with a report on any memory error or data race.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* mrsum_pages_create(int num_pages, int reserved);
int mrsum_pages_alloc(void* h, int n, int* out);
int mrsum_pages_free(void* h, int n, const int* ids);
int mrsum_pages_available(void* h);
void mrsum_pages_destroy(void* h);
void* mrsum_bpe_create(const char* blob, const int32_t* lens, const int32_t* ranks, int32_t n);
void mrsum_bpe_destroy(void* h);
int64_t mrsum_bpe_encode_pieces(void* h, const char* blob, const int32_t* offsets, int32_t n, int32_t* out,
                                int64_t cap);
}

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

static int stress_pages(int threads, int iters) {
  const int total = 4096, reserved = 1;
  void* h = mrsum_pages_create(total, reserved);
  CHECK(h != nullptr);
  std::vector<std::atomic<int>> owner(total);
  for (auto& o : owner) o.store(-1);
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) {
    ts.emplace_back([&, t] {
      std::mt19937 rng(1234 + t);
      std::vector<std::vector<int>> held;
      for (int it = 0; it < iters; ++it) {
        if (held.empty() || (rng() % 3 != 0 && held.size() < 8)) {
          const int n = 1 + static_cast<int>(rng() % 40);
          std::vector<int> ids(n);
          if (mrsum_pages_alloc(h, n, ids.data()) == 0) {
            for (int id : ids) {
              CHECK(id >= reserved && id < total);
              int expect = -1;
              CHECK(owner[id].compare_exchange_strong(expect, t));  // nobody else holds it
            }
            held.push_back(std::move(ids));
          }
        } else {
          const size_t k = rng() % held.size();
          std::vector<int> ids = std::move(held[k]);
          held.erase(held.begin() + static_cast<long>(k));
          for (int id : ids) owner[id].store(-1);
          CHECK(mrsum_pages_free(h, static_cast<int>(ids.size()), ids.data()) == 0);
        }
      }
      for (auto& ids : held) {
        for (int id : ids) owner[id].store(-1);
        CHECK(mrsum_pages_free(h, static_cast<int>(ids.size()), ids.data()) == 0);
      }
    });
  }
  for (auto& th : ts) th.join();
  // (single-threaded: concurrently another thread may legitimately own a page we just freed)
  int two[2];
  CHECK(mrsum_pages_alloc(h, 2, two) == 0);
  CHECK(mrsum_pages_free(h, 2, two) == 0);
  CHECK(mrsum_pages_free(h, 1, two) == -1);  // double free rejected, nothing freed
  int x;
  CHECK(mrsum_pages_alloc(h, 1, &x) == 0);
  const int dup[2] = {x, x};
  CHECK(mrsum_pages_free(h, 2, dup) == -1);  // duplicate ids in one call rejected, nothing freed
  CHECK(mrsum_pages_free(h, 1, &x) == 0);
  const int foreign[2] = {0, total + 5};
  CHECK(mrsum_pages_free(h, 1, &foreign[0]) == -1);
  CHECK(mrsum_pages_free(h, 1, &foreign[1]) == -1);
  CHECK(mrsum_pages_available(h) == total - reserved);
  mrsum_pages_destroy(h);
  return 0;
}

static int stress_bpe(int threads, int iters) {
  // vocabulary: the 256 single bytes + a few merges
  std::vector<std::string> toks;
  for (int b = 0; b < 256; ++b) toks.emplace_back(1, static_cast<char>(b));
  for (const char* m : {"th", "he", "the", "in", "ing", "an", "and", "er", "ere", "there", " t", " the"})
    toks.emplace_back(m);
  std::string blob;
  std::vector<int32_t> lens, ranks;
  for (size_t i = 0; i < toks.size(); ++i) {
    blob += toks[i];
    lens.push_back(static_cast<int32_t>(toks[i].size()));
    ranks.push_back(static_cast<int32_t>(i));
  }
  void* h = mrsum_bpe_create(blob.data(), lens.data(), ranks.data(), static_cast<int32_t>(toks.size()));
  CHECK(h != nullptr);
  std::vector<std::string> words = {" the", "there", "and", "singing", "anther", " theremin", "xyz", "inn"};
  std::string wb;
  std::vector<int32_t> off = {0};
  for (int r = 0; r < 64; ++r)
    for (auto& w : words) {
      wb += w + std::to_string(r % 7);
      off.push_back(static_cast<int32_t>(wb.size()));
    }
  const int32_t n = static_cast<int32_t>(off.size() - 1);
  std::vector<int32_t> ref(wb.size() + 1);
  const int64_t m = mrsum_bpe_encode_pieces(h, wb.data(), off.data(), n, ref.data(), static_cast<int64_t>(ref.size()));
  CHECK(m > 0);
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) {
    ts.emplace_back([&] {
      std::vector<int32_t> out(wb.size() + 1);
      for (int it = 0; it < iters; ++it) {
        const int64_t k = mrsum_bpe_encode_pieces(h, wb.data(), off.data(), n, out.data(),
                                                  static_cast<int64_t>(out.size()));
        CHECK(k == m);
        CHECK(std::memcmp(out.data(), ref.data(), static_cast<size_t>(m) * sizeof(int32_t)) == 0);
      }
    });
  }
  for (auto& th : ts) th.join();
  int32_t tiny[2];
  CHECK(mrsum_bpe_encode_pieces(h, wb.data(), off.data(), n, tiny, 2) == -1);  // output too small
  mrsum_bpe_destroy(h);
  return 0;
}

int main() {
  stress_pages(8, 4000);
  stress_bpe(8, 200);
  std::printf("runtime stress ok\n");
  return 0;
}
