// KV-cache page allocator (host C++), used by engine/kv_cache.py.
//
// LIFO free list over page ids [reserved, num_pages): recently freed pages
// are reused first (they are the most likely to still sit in the 256 MiB
// Infinity Cache / L2).  An allocation is all-or-nothing.  A per-page "in
// use" bitmap catches double frees and foreign ids.  Thread-safe.
//
// C ABI (ctypes):
//   void* mrsum_pages_create(int num_pages, int reserved)
//   int   mrsum_pages_alloc(void*, int n, int* out)      0 ok, -1 not enough pages
//   int   mrsum_pages_free(void*, int n, const int* ids) 0 ok, -1 bad / double free (nothing freed)
//   int   mrsum_pages_available(void*)
//   void  mrsum_pages_destroy(void*)

#include <cstdint>
#include <mutex>
#include <vector>

namespace {

struct Pages {
  std::vector<int> free_list;
  std::vector<uint8_t> used;
  int reserved = 0;
  std::mutex mu;
};

}  // namespace

extern "C" {

void* mrsum_pages_create(int num_pages, int reserved) {
  if (num_pages <= reserved || reserved < 0) return nullptr;
  auto* p = new Pages();
  p->reserved = reserved;
  p->used.assign(num_pages, 0);
  for (int i = 0; i < reserved; ++i) p->used[i] = 1;
  p->free_list.reserve(num_pages - reserved);
  for (int i = num_pages - 1; i >= reserved; --i) p->free_list.push_back(i);
  return p;
}

int mrsum_pages_alloc(void* h, int n, int* out) {
  auto* p = static_cast<Pages*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  if (n < 0 || static_cast<size_t>(n) > p->free_list.size()) return -1;
  for (int i = 0; i < n; ++i) {
    const int id = p->free_list.back();
    p->free_list.pop_back();
    p->used[id] = 1;
    out[i] = id;
  }
  return 0;
}

int mrsum_pages_free(void* h, int n, const int* ids) {
  auto* p = static_cast<Pages*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  const int total = static_cast<int>(p->used.size());
  for (int i = 0; i < n; ++i) {
    const int id = ids[i];
    if (id < p->reserved || id >= total || !p->used[id]) return -1;
    for (int j = 0; j < i; ++j)
      if (ids[j] == id) return -1;
  }
  for (int i = n - 1; i >= 0; --i) {
    p->used[ids[i]] = 0;
    p->free_list.push_back(ids[i]);
  }
  return 0;
}

int mrsum_pages_available(void* h) {
  auto* p = static_cast<Pages*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  return static_cast<int>(p->free_list.size());
}

void mrsum_pages_destroy(void* h) { delete static_cast<Pages*>(h); }

}  // extern "C"
