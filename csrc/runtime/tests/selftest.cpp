// Host self-test of the C++ runtime, built with sanitizers by tests/test_native_sanitizers.py:
//   * ASan + UBSan: BPE build/encode/decode/train, WordPiece, mbox splitting, block pool;
//   * TSan: the block pool under concurrent alloc/free from several threads (the engine, the
//     bench's prepare worker and the prefix cache can touch it from different threads).
// (GPU sanitizers / XNACK are not available on the GPU pool; the kernels are covered by the
// fp32-reference numerics tests instead.)
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* cfc_blockpool_create(int);
int cfc_blockpool_destroy(void*);
int cfc_blockpool_alloc(void*, int, int32_t*);
int cfc_blockpool_free(void*, const int32_t*, int);
int cfc_blockpool_num_free(void*);
int64_t cfc_mbox_split(const char*, int64_t, int64_t*, int);
void* cfc_bpe_create();
int cfc_bpe_destroy(void*);
int cfc_bpe_add_token(void*, const char*, int, int);
int cfc_bpe_add_merge(void*, int, int, int, int);
int cfc_bpe_finalize(void*);
int cfc_bpe_encode(void*, const char*, int, int32_t*, int);
int cfc_bpe_decode(void*, const int32_t*, int, char*, int);
int cfc_bpe_train(const char*, int, int, char*, int32_t*, int);
void* cfc_wp_create(int, int, int, int);
int cfc_wp_destroy(void*);
int cfc_wp_add_token(void*, const char*, int, int);
int cfc_wp_encode(void*, const char*, int, int32_t*, int);
}

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                           \
    }                                                                     \
  } while (0)

static int test_pool_threads() {
  void* p = cfc_blockpool_create(4096);
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([p, t] {
      std::vector<int32_t> got(37);
      for (int it = 0; it < 2000; ++it) {
        const int n = 1 + (it * 7 + t) % 37;
        if (cfc_blockpool_alloc(p, n, got.data()) == 0) cfc_blockpool_free(p, got.data(), n);
      }
    });
  for (auto& x : th) x.join();
  CHECK(cfc_blockpool_num_free(p) == 4096);
  std::vector<int32_t> all(4096);
  CHECK(cfc_blockpool_alloc(p, 4096, all.data()) == 0);
  CHECK(cfc_blockpool_alloc(p, 1, all.data()) == -1);
  std::vector<int> seen(4096, 0);
  for (int b : all) seen[b]++;
  for (int s : seen) CHECK(s == 1);
  cfc_blockpool_destroy(p);
  return 0;
}

static int test_mbox() {
  const std::string mb = "From a@x Mon\nSubject: s\n\nbody From x\nFrom b@y Tue\n\nFromage\nFrom c@z\n";
  int64_t off[8];
  const int64_t n = cfc_mbox_split(mb.data(), (int64_t)mb.size(), off, 8);
  CHECK(n == 3 && off[0] == 0 && mb.compare((size_t)off[1], 5, "From ") == 0);
  CHECK(cfc_mbox_split(mb.data(), (int64_t)mb.size(), off, 1) == 3);   // count beyond the buffer
  return 0;
}

static int test_bpe() {
  std::string corpus;
  for (int i = 0; i < 200; ++i) corpus += "the working group reached rough consensus on the draft ";
  std::vector<char> base(1 << 20, 0);
  std::vector<int32_t> merges(2 * 400);
  const int nm = cfc_bpe_train(corpus.data(), (int)corpus.size(), 400, base.data(), merges.data(), 400);
  CHECK(nm > 0 && nm <= 400);
  // hand-built vocabulary: bytes + "▁a", "▁ab"
  void* h = cfc_bpe_create();
  const char* sp = "\xe2\x96\x81";
  int id = 0;
  for (const char* s : {"<unk>", "<s>", "</s>"}) cfc_bpe_add_token(h, s, (int)std::strlen(s), id++);
  for (int b = 0; b < 256; ++b) {
    char t[8];
    std::snprintf(t, sizeof t, "<0x%02X>", b);
    cfc_bpe_add_token(h, t, 6, id++);
  }
  const int a = id++, bb = id++, spid = id++;
  cfc_bpe_add_token(h, "a", 1, a);
  cfc_bpe_add_token(h, "b", 1, bb);
  cfc_bpe_add_token(h, sp, 3, spid);
  const int spa = id++, spab = id++;
  cfc_bpe_add_token(h, (std::string(sp) + "a").c_str(), 4, spa);
  cfc_bpe_add_token(h, (std::string(sp) + "ab").c_str(), 5, spab);
  cfc_bpe_add_merge(h, spid, a, 0, spa);
  cfc_bpe_add_merge(h, spa, bb, 1, spab);
  cfc_bpe_finalize(h);
  int32_t out[64];
  const int n = cfc_bpe_encode(h, "ab ab \xc3\xa9", 8, out, 64);
  CHECK(n >= 3 && out[0] == spab && out[1] == spab);
  char txt[64];
  const int m = cfc_bpe_decode(h, out, n, txt, 63);
  CHECK(m == 8 && std::memcmp(txt, "ab ab \xc3\xa9", 8) == 0);
  CHECK(cfc_bpe_encode(h, "ab", 2, out, 0) == 1);   // size query with cap 0
  cfc_bpe_destroy(h);
  return 0;
}

static int test_wordpiece() {
  void* w = cfc_wp_create(100, 101, 102, 1);
  const char* toks[] = {"con", "##sen", "##sus", "rough", "[UNK]"};
  for (int i = 0; i < 5; ++i) cfc_wp_add_token(w, toks[i], (int)std::strlen(toks[i]), i);
  int32_t out[32];
  const int n = cfc_wp_encode(w, "Rough consensus zzz", 19, out, 32);
  // lower-cased greedy longest-match pieces, unknown word -> unk (CLS/SEP are added by the caller)
  CHECK(n == 5 && out[0] == 3 && out[1] == 0 && out[2] == 1 && out[3] == 2 && out[4] == 100);
  cfc_wp_destroy(w);
  return 0;
}

int main(int argc, char** argv) {
  const bool threads_only = argc > 1 && std::strcmp(argv[1], "threads") == 0;
  if (test_pool_threads()) return 1;
  if (!threads_only && (test_mbox() || test_bpe() || test_wordpiece())) return 1;
  std::puts("runtime selftest ok");
  return 0;
}
