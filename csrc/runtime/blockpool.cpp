// Paged-KV block allocator and mbox message splitter (host C++ runtime).
//
// * BlockPool: thread-safe LIFO free list of KV-cache block ids (LIFO keeps recently freed,
//   still-L2/MALL-warm blocks hot for the next sequence).
// * cfc_mbox_split: finds the byte offsets of every "From " separator line of an mbox buffer
//   (the reference walks the file with Python's mailbox module, parsing/app/parser.py:42-62;
//   here the scan is one memchr pass so multi-GB archives split at memory bandwidth).
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#define CFC_API extern "C" __attribute__((visibility("default")))

namespace {
struct BlockPool {
  std::mutex mu;
  std::vector<int32_t> free_list;
  explicit BlockPool(int n) {
    free_list.reserve(n);
    for (int i = n - 1; i >= 0; --i) free_list.push_back(i);
  }
};
}  // namespace

CFC_API void* cfc_blockpool_create(int num_blocks) {
  if (num_blocks <= 0) return nullptr;
  return new BlockPool(num_blocks);
}

CFC_API int cfc_blockpool_destroy(void* p) {
  delete static_cast<BlockPool*>(p);
  return 0;
}

// Pops n blocks into out (in allocation order). Returns -1 (and allocates nothing) if short.
CFC_API int cfc_blockpool_alloc(void* p, int n, int32_t* out) {
  auto* bp = static_cast<BlockPool*>(p);
  std::lock_guard<std::mutex> g(bp->mu);
  if (n < 0 || (size_t)n > bp->free_list.size()) return -1;
  for (int i = 0; i < n; ++i) {
    out[i] = bp->free_list.back();
    bp->free_list.pop_back();
  }
  return 0;
}

CFC_API int cfc_blockpool_free(void* p, const int32_t* blocks, int n) {
  auto* bp = static_cast<BlockPool*>(p);
  std::lock_guard<std::mutex> g(bp->mu);
  for (int i = n - 1; i >= 0; --i) bp->free_list.push_back(blocks[i]);
  return 0;
}

CFC_API int cfc_blockpool_num_free(void* p) {
  auto* bp = static_cast<BlockPool*>(p);
  std::lock_guard<std::mutex> g(bp->mu);
  return (int)bp->free_list.size();
}

// Writes up to max_out message start offsets (offset of the "From " line) into out; returns the
// total number of messages found (may exceed max_out: call again with a bigger buffer).
// A separator is "From " at the start of the buffer or right after '\n'.
CFC_API int64_t cfc_mbox_split(const char* buf, int64_t len, int64_t* out, int max_out) {
  int64_t count = 0;
  auto emit = [&](int64_t off) {
    if (count < max_out) out[count] = off;
    ++count;
  };
  if (len >= 5 && std::memcmp(buf, "From ", 5) == 0) emit(0);
  const char* p = buf;
  const char* end = buf + len;
  while (p < end) {
    const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
    if (!nl) break;
    const char* s = nl + 1;
    if (end - s >= 5 && std::memcmp(s, "From ", 5) == 0) emit((int64_t)(s - buf));
    p = s;
  }
  return count;
}
