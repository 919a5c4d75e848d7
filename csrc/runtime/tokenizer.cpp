// Host C++ tokenizers for the MI355X pipeline.
//
//  * BPE (SentencePiece-style, as used by Mistral / Llama-2): text is pre-split on spaces with the
//    U+2581 "▁" word marker (add-dummy-prefix), every word is greedily merged by merge RANK
//    (lowest rank first) over UTF-8 characters, unknown characters fall back to <0xXX> byte
//    tokens.  Vocab + merges come from an HF tokenizer.json (parsed in Python) or from the
//    built-in trainer below.
//  * WordPiece (BERT / MiniLM / BGE): lower-casing basic tokenizer (whitespace + punctuation
//    split, CJK isolated), greedy longest-match-first with "##" continuations, [UNK] for words
//    with no segmentation or > 100 characters.
//  * BPE trainer: the classic incremental pair-count algorithm (pair -> occurrence index, lazy
//    max-heap), so 32k merges over a multi-MB corpus take seconds, not hours.
//
// The reference tokenises inside HF `tokenizers` (Rust) / sentence-transformers and inside
// llama.cpp; these are the native replacements.  All entry points are extern "C".
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#define CFC_API extern "C" __attribute__((visibility("default")))

namespace {

const std::string kSpaceMark = "\xE2\x96\x81";  // U+2581

inline int utf8_len(unsigned char c) {
  if (c < 0x80) return 1;
  if ((c >> 5) == 0x6) return 2;
  if ((c >> 4) == 0xE) return 3;
  if ((c >> 3) == 0x1E) return 4;
  return 1;  // invalid lead byte: treat as a single byte
}

std::vector<std::string> utf8_chars(const std::string& s) {
  std::vector<std::string> out;
  for (size_t i = 0; i < s.size();) {
    int n = std::min<int>(utf8_len((unsigned char)s[i]), (int)(s.size() - i));
    out.emplace_back(s.substr(i, n));
    i += n;
  }
  return out;
}

struct PairHash {
  size_t operator()(const std::pair<int, int>& p) const {
    return std::hash<uint64_t>()(((uint64_t)(uint32_t)p.first << 32) | (uint32_t)p.second);
  }
};

// ------------------------------------------------------------------------------------------ BPE
struct BPE {
  std::unordered_map<std::string, int> tok2id;
  std::vector<std::string> id2tok;
  std::unordered_map<std::pair<int, int>, std::pair<int, int>, PairHash> merges;  // (a,b) -> (rank, merged id)
  int byte_tok[256];
  int unk_id = 0;
  std::unordered_map<std::string, std::vector<int>> cache;

  BPE() { std::fill(byte_tok, byte_tok + 256, -1); }

  void finalize() {
    char buf[8];
    for (int b = 0; b < 256; ++b) {
      snprintf(buf, sizeof(buf), "<0x%02X>", b);
      auto it = tok2id.find(buf);
      byte_tok[b] = it == tok2id.end() ? -1 : it->second;
    }
    auto u = tok2id.find("<unk>");
    unk_id = u == tok2id.end() ? 0 : u->second;
    cache.clear();
  }

  using WordCache = std::unordered_map<std::string, std::vector<int>>;

  void encode_word(const std::string& word, std::vector<int>& out) { encode_word(word, out, cache); }

  // `wc` is the caller's word cache: the member cache for the single-text API (serialised by the
  // Python binding's lock), a thread-local one per worker in encode_batch
  void encode_word(const std::string& word, std::vector<int>& out, WordCache& wc) const {
    auto hit = wc.find(word);
    if (hit != wc.end()) {
      out.insert(out.end(), hit->second.begin(), hit->second.end());
      return;
    }
    std::vector<int> sym;
    for (const auto& ch : utf8_chars(word)) {
      auto it = tok2id.find(ch);
      if (it != tok2id.end()) {
        sym.push_back(it->second);
      } else {
        for (unsigned char b : ch) sym.push_back(byte_tok[b] >= 0 ? byte_tok[b] : unk_id);
      }
    }
    // repeatedly merge the lowest-rank adjacent pair (words are short: O(n^2) is fine)
    while (sym.size() > 1) {
      int best = -1, best_rank = 0x7fffffff, best_id = -1;
      for (size_t i = 0; i + 1 < sym.size(); ++i) {
        auto m = merges.find({sym[i], sym[i + 1]});
        if (m != merges.end() && m->second.first < best_rank) {
          best_rank = m->second.first;
          best = (int)i;
          best_id = m->second.second;
        }
      }
      if (best < 0) break;
      sym[best] = best_id;
      sym.erase(sym.begin() + best + 1);
    }
    if (wc.size() < 1000000) wc.emplace(word, sym);
    out.insert(out.end(), sym.begin(), sym.end());
  }

  void encode(const std::string& text, std::vector<int>& out) { encode(text, out, cache); }

  // HF tokenizer.json semantics of the SentencePiece-style pipelines:
  //   split_mode 0 -- Metaspace(split=true): a new piece starts at EVERY "▁" ("▁▁▁a" -> ▁ ▁ ▁a);
  //   split_mode 1 -- no pre-tokenizer (Llama-2/Mistral files: Prepend + Replace normalizers):
  //                   the whole text is one sequence; splitting where a "▁" follows a non-"▁"
  //                   character is exact for SentencePiece vocabularies, whose pieces carry "▁"
  //                   only as a prefix (runs like "▁▁▁" still merge);
  //   prepend_mode 0 -- prepend "▁" unless the text already starts with one (Metaspace "always"),
  //                1 -- always (Prepend normalizer), 2 -- never.
  // Newlines are ordinary characters inside a piece (SentencePiece: "a\nb" -> ▁a <0x0A> b).
  int split_mode = 0, prepend_mode = 0;

  void encode(const std::string& text, std::vector<int>& out, WordCache& wc) const {
    if (text.empty()) return;
    std::string norm;
    norm.reserve(text.size() + text.size() / 2 + 3);
    if (prepend_mode == 1 || (prepend_mode == 0 && text[0] != ' ')) norm += kSpaceMark;
    for (char c : text) {
      if (c == ' ') norm += kSpaceMark;
      else norm.push_back(c);
    }
    // kSpaceMark's lead byte 0xE2 never occurs inside another UTF-8 sequence, so a byte scan is safe
    size_t start = 0;
    bool prev_mark = false;
    for (size_t p = 0; p < norm.size();) {
      const bool mark = norm.compare(p, 3, kSpaceMark) == 0;
      if (mark && p > start && (split_mode == 0 || !prev_mark)) {
        encode_word(norm.substr(start, p - start), out, wc);
        start = p;
      }
      prev_mark = mark;
      p += mark ? 3 : 1;
    }
    if (start < norm.size()) encode_word(norm.substr(start), out, wc);
  }
};

// ------------------------------------------------------------------------------------ WordPiece
struct WordPiece {
  std::unordered_map<std::string, int> vocab;
  int unk_id, cls_id, sep_id, max_chars;
  size_t max_piece = 0;   // longest vocabulary entry in bytes: longer substrings are never looked up
  bool lower;

  static bool is_punct(uint32_t cp) {
    if ((cp >= 33 && cp <= 47) || (cp >= 58 && cp <= 64) || (cp >= 91 && cp <= 96) || (cp >= 123 && cp <= 126))
      return true;
    return (cp >= 0x2000 && cp <= 0x206F) || (cp >= 0x3000 && cp <= 0x303F);
  }
  static bool is_cjk(uint32_t cp) {
    return (cp >= 0x4E00 && cp <= 0x9FFF) || (cp >= 0x3400 && cp <= 0x4DBF) || (cp >= 0xF900 && cp <= 0xFAFF) ||
           (cp >= 0x20000 && cp <= 0x2FA1F);
  }
  static uint32_t decode_cp(const unsigned char* s, int n) {
    switch (n) {
      case 1: return s[0];
      case 2: return ((s[0] & 0x1F) << 6) | (s[1] & 0x3F);
      case 3: return ((s[0] & 0x0F) << 12) | ((s[1] & 0x3F) << 6) | (s[2] & 0x3F);
      default: return ((s[0] & 0x07) << 18) | ((s[1] & 0x3F) << 12) | ((s[2] & 0x3F) << 6) | (s[3] & 0x3F);
    }
  }

  // Per-thread scratch: the encode loop allocates nothing once these have grown.
  struct Scratch {
    std::string word, sub;
    std::vector<int> bounds, pieces;
  };

  // Greedy longest-match-first pieces of one basic-split word (bytes in sc.word).
  void encode_word(Scratch& sc, std::vector<int>& out) const {
    const std::string& w = sc.word;
    sc.bounds.clear();
    for (size_t i = 0; i < w.size();) {
      sc.bounds.push_back((int)i);
      i += (size_t)std::min<int>(utf8_len((unsigned char)w[i]), (int)(w.size() - i));
    }
    const int nch = (int)sc.bounds.size();
    sc.bounds.push_back((int)w.size());
    if (nch > max_chars) { out.push_back(unk_id); return; }
    sc.pieces.clear();
    int start = 0;
    while (start < nch) {
      const size_t pre = start > 0 ? 2 : 0;
      int end = nch, found = -1;
      // substrings longer than the longest vocabulary entry cannot match: start below them
      while (end > start && (size_t)(sc.bounds[end] - sc.bounds[start]) + pre > max_piece) --end;
      for (; end > start; --end) {
        sc.sub.assign(start > 0 ? "##" : "");
        sc.sub.append(w, (size_t)sc.bounds[start], (size_t)(sc.bounds[end] - sc.bounds[start]));
        auto it = vocab.find(sc.sub);
        if (it != vocab.end()) { found = it->second; break; }
      }
      if (found < 0) { out.push_back(unk_id); return; }
      sc.pieces.push_back(found);
      start = end;
    }
    out.insert(out.end(), sc.pieces.begin(), sc.pieces.end());
  }

  // BERT basic split (whitespace, control characters dropped, punctuation and CJK as single
  // words, ASCII lower-casing) fused with the WordPiece pass; stops once out holds `limit` ids
  // (the callers truncate there), so a long chunk is not encoded past its model's max length.
  void encode(const std::string& text, std::vector<int>& out, Scratch& sc, size_t limit = SIZE_MAX) const {
    sc.word.clear();
    auto flush = [&] {
      if (!sc.word.empty()) { encode_word(sc, out); sc.word.clear(); }
    };
    const unsigned char* t = (const unsigned char*)text.data();
    const size_t n = text.size();
    for (size_t i = 0; i < n && out.size() < limit;) {
      const int len = std::min<int>(utf8_len(t[i]), (int)(n - i));
      const uint32_t cp = decode_cp(t + i, len);
      if (cp == ' ' || cp == '\t' || cp == '\n' || cp == '\r' || cp == 0xA0) {
        flush();
      } else if (cp == 0 || cp == 0xFFFD || cp < 32 || cp == 0x7F) {   // control characters dropped (HF: Cc)
      } else if (is_punct(cp) || is_cjk(cp)) {
        flush();
        sc.word.assign((const char*)t + i, (size_t)len);
        flush();
      } else if (lower && len == 1) {
        sc.word.push_back((char)std::tolower(t[i]));
      } else {
        sc.word.append((const char*)t + i, (size_t)len);
      }
      i += (size_t)len;
    }
    if (out.size() < limit) flush();
  }
  void encode(const std::string& text, std::vector<int>& out) const {
    Scratch sc;
    encode(text, out, sc);
  }
};

}  // namespace

// ----------------------------------------------------------------------------------------- BPE
CFC_API void* cfc_bpe_create() { return new BPE(); }
CFC_API int cfc_bpe_destroy(void* h) { delete static_cast<BPE*>(h); return 0; }

CFC_API int cfc_bpe_add_token(void* h, const char* tok, int len, int id) {
  auto* b = static_cast<BPE*>(h);
  std::string t(tok, len);
  b->tok2id[t] = id;
  if ((int)b->id2tok.size() <= id) b->id2tok.resize(id + 1);
  b->id2tok[id] = t;
  return 0;
}

CFC_API int cfc_bpe_add_merge(void* h, int a, int b, int rank, int merged) {
  static_cast<BPE*>(h)->merges[{a, b}] = {rank, merged};
  return 0;
}

CFC_API int cfc_bpe_finalize(void* h) { static_cast<BPE*>(h)->finalize(); return 0; }

CFC_API int cfc_bpe_set_mode(void* h, int split_mode, int prepend_mode) {
  if (split_mode < 0 || split_mode > 1 || prepend_mode < 0 || prepend_mode > 2) return -1;
  auto* b = static_cast<BPE*>(h);
  b->split_mode = split_mode;
  b->prepend_mode = prepend_mode;
  b->cache.clear();
  return 0;
}

// Returns the number of ids produced (may exceed cap: call again with a bigger buffer).
CFC_API int cfc_bpe_encode(void* h, const char* text, int len, int32_t* out, int cap) {
  std::vector<int> ids;
  static_cast<BPE*>(h)->encode(std::string(text, len), ids);
  const int n = (int)ids.size();
  for (int i = 0; i < std::min(n, cap); ++i) out[i] = ids[i];
  return n;
}

// Writes the UTF-8 detokenisation ("▁" -> space, <0xXX> -> byte) into out; returns its length.
CFC_API int cfc_bpe_decode(void* h, const int32_t* ids, int n, char* out, int cap) {
  auto* b = static_cast<BPE*>(h);
  std::string s;
  for (int i = 0; i < n; ++i) {
    if (ids[i] < 0 || ids[i] >= (int)b->id2tok.size()) continue;
    const std::string& t = b->id2tok[ids[i]];
    if (t.size() == 6 && t[0] == '<' && t[1] == '0' && t[2] == 'x' && t[5] == '>') {
      s.push_back((char)std::stoi(t.substr(3, 2), nullptr, 16));
      continue;
    }
    for (size_t p = 0; p < t.size();) {
      if (t.compare(p, 3, kSpaceMark) == 0) { s.push_back(' '); p += 3; }
      else { s.push_back(t[p]); ++p; }
    }
  }
  if (!s.empty() && s[0] == ' ') s.erase(0, 1);
  const int m = (int)s.size();
  std::memcpy(out, s.data(), std::min(m, cap));
  return m;
}

// Trains SentencePiece-style BPE merges on `corpus`.  Base symbols = the 256 byte tokens
// <0xXX> (ids 3..258, after <unk>=0 <s>=1 </s>=2) + every distinct UTF-8 character of the corpus;
// then merges until vocab_size.  Output: merges as (left id, right id) pairs in rank order into
// merge_out (2*cap ints) and the number of base characters in *n_chars... the token strings are
// reconstructible from the merge list, so only pairs are returned.  Returns the merge count.
// The first `n_base` ids are returned through base_out as a '\0'-separated UTF-8 string list.
CFC_API int cfc_bpe_train(const char* corpus, int len, int vocab_size, char* base_out, int32_t* merge_out,
                          int merge_cap) {
  std::string text(corpus, len);
  // word frequencies over "▁word" pieces
  std::unordered_map<std::string, int> wfreq;
  {
    size_t i = 0;
    while (i < text.size()) {
      while (i < text.size() && (text[i] == ' ' || text[i] == '\n')) ++i;
      size_t k = i;
      while (k < text.size() && text[k] != ' ' && text[k] != '\n') ++k;
      if (k > i) wfreq[kSpaceMark + text.substr(i, k - i)]++;
      i = k;
    }
  }
  std::vector<std::string> base;  // id order after the 3 specials + 256 bytes
  std::unordered_map<std::string, int> id_of;
  const int first_char_id = 3 + 256;
  std::vector<std::vector<int>> words;
  std::vector<int> freqs;
  words.reserve(wfreq.size());
  for (auto& kv : wfreq) {
    std::vector<int> sym;
    for (auto& ch : utf8_chars(kv.first)) {
      auto it = id_of.find(ch);
      if (it == id_of.end()) {
        it = id_of.emplace(ch, first_char_id + (int)base.size()).first;
        base.push_back(ch);
      }
      sym.push_back(it->second);
    }
    words.push_back(std::move(sym));
    freqs.push_back(kv.second);
  }
  // serialise base characters
  {
    size_t p = 0;
    for (auto& b : base) { std::memcpy(base_out + p, b.data(), b.size()); p += b.size(); base_out[p++] = '\0'; }
    base_out[p] = '\0';
  }
  int next_id = first_char_id + (int)base.size();
  std::unordered_map<std::pair<int, int>, long long, PairHash> cnt;
  std::unordered_map<std::pair<int, int>, std::unordered_set<int>, PairHash> where;
  for (int w = 0; w < (int)words.size(); ++w)
    for (size_t i = 0; i + 1 < words[w].size(); ++i) {
      auto pr = std::make_pair(words[w][i], words[w][i + 1]);
      cnt[pr] += freqs[w];
      where[pr].insert(w);
    }
  using HE = std::pair<long long, std::pair<int, int>>;
  auto cmp = [](const HE& a, const HE& b) {
    if (a.first != b.first) return a.first < b.first;
    return a.second > b.second;  // deterministic tie-break: smaller pair first
  };
  std::priority_queue<HE, std::vector<HE>, decltype(cmp)> heap(cmp);
  for (auto& kv : cnt) heap.push({kv.second, kv.first});
  int n_merges = 0;
  while (next_id < vocab_size && !heap.empty() && n_merges < merge_cap) {
    auto top = heap.top();
    heap.pop();
    auto it = cnt.find(top.second);
    const long long cur = it == cnt.end() ? 0 : it->second;
    if (cur != top.first) {  // stale heap entry: re-queue with the live count
      if (cur >= 2) heap.push({cur, top.second});
      continue;
    }
    if (cur < 2) break;  // nothing left worth merging
    const auto pr = top.second;
    const int nid = next_id++;
    merge_out[2 * n_merges] = pr.first;
    merge_out[2 * n_merges + 1] = pr.second;
    ++n_merges;
    auto ws = where[pr];  // copy: we mutate the index while iterating
    std::unordered_map<std::pair<int, int>, long long, PairHash> delta;
    for (int w : ws) {
      auto& sym = words[w];
      const int f = freqs[w];
      for (size_t i = 0; i + 1 < sym.size(); ++i) delta[{sym[i], sym[i + 1]}] -= f;
      std::vector<int> ns;
      ns.reserve(sym.size());
      for (size_t i = 0; i < sym.size();) {
        if (i + 1 < sym.size() && sym[i] == pr.first && sym[i + 1] == pr.second) { ns.push_back(nid); i += 2; }
        else { ns.push_back(sym[i]); ++i; }
      }
      sym.swap(ns);
      for (size_t i = 0; i + 1 < sym.size(); ++i) {
        auto np = std::make_pair(sym[i], sym[i + 1]);
        delta[np] += f;
        where[np].insert(w);
      }
    }
    for (auto& d : delta) {
      if (d.second == 0) continue;
      long long& c = cnt[d.first];
      c += d.second;
      if (c > 0 && d.second > 0) heap.push({c, d.first});
    }
    cnt.erase(pr);
    where.erase(pr);
  }
  return n_merges;
}

// ----------------------------------------------------------------------------------- WordPiece
CFC_API void* cfc_wp_create(int unk_id, int cls_id, int sep_id, int lowercase) {
  auto* w = new WordPiece();
  w->unk_id = unk_id; w->cls_id = cls_id; w->sep_id = sep_id; w->max_chars = 100; w->lower = lowercase != 0;
  return w;
}
CFC_API int cfc_wp_destroy(void* h) { delete static_cast<WordPiece*>(h); return 0; }
CFC_API int cfc_wp_add_token(void* h, const char* tok, int len, int id) {
  auto* w = static_cast<WordPiece*>(h);
  w->vocab[std::string(tok, len)] = id;
  w->max_piece = std::max(w->max_piece, (size_t)len);
  return 0;
}
CFC_API int cfc_wp_finalize(void*) { return 0; }
CFC_API int cfc_wp_encode(void* h, const char* text, int len, int32_t* out, int cap) {
  std::vector<int> ids;
  static_cast<WordPiece*>(h)->encode(std::string(text, len), ids);
  const int n = (int)ids.size();
  for (int i = 0; i < std::min(n, cap); ++i) out[i] = ids[i];
  return n;
}

// ------------------------------------------------------------------------------------ batch encode
// texts = buf[offs[i], offs[i+1]); ids of text i go to out[i*cap ...] (at most cap), its FULL length
// to lens[i] (re-encode singly when lens[i] > cap).  nthreads workers, text i on worker i % nthreads.
template <class F>
static void parallel_texts(int n, int nthreads, F&& fn) {
  nthreads = std::max(1, std::min(nthreads, n));
  if (nthreads == 1) {
    fn(0, 1);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) th.emplace_back([&fn, t, nthreads] { fn(t, nthreads); });
  for (auto& x : th) x.join();
}

CFC_API int cfc_bpe_encode_batch(void* h, const char* buf, const int64_t* offs, int n, int cap, int32_t* out,
                                 int32_t* lens, int nthreads) {
  const auto* b = static_cast<const BPE*>(h);
  parallel_texts(n, nthreads, [&](int t, int nt) {
    BPE::WordCache wc;
    std::vector<int> ids;
    for (int i = t; i < n; i += nt) {
      ids.clear();
      b->encode(std::string(buf + offs[i], (size_t)(offs[i + 1] - offs[i])), ids, wc);
      lens[i] = (int32_t)ids.size();
      const int m = std::min((int)ids.size(), cap);
      for (int k = 0; k < m; ++k) out[(size_t)i * cap + k] = ids[k];
    }
  });
  return 0;
}

// Byte-level BPE (GPT-2 / tiktoken / Llama-3 tokenizer.json): the caller has already split the text
// with the model's regex and mapped every byte to its printable stand-in character; each piece is
// merged independently (no "▁" handling, no byte fallback needed).  Concatenated ids into out;
// returns their count (may exceed cap).
CFC_API int cfc_bpe_encode_pieces(void* h, const char* buf, const int64_t* offs, int n, int32_t* out, int cap) {
  auto* b = static_cast<BPE*>(h);
  std::vector<int> ids;
  for (int i = 0; i < n; ++i)
    b->encode_word(std::string(buf + offs[i], (size_t)(offs[i + 1] - offs[i])), ids);
  const int m = (int)ids.size();
  for (int k = 0; k < std::min(m, cap); ++k) out[k] = ids[k];
  return m;
}

CFC_API int cfc_wp_encode_batch(void* h, const char* buf, const int64_t* offs, int n, int cap, int32_t* out,
                                int32_t* lens, int nthreads) {
  // every caller truncates to cap (the model's max length): encoding stops there, and lens[i]
  // holds at least min(full length, cap) -- callers use min(lens[i], cap)
  const auto* w = static_cast<const WordPiece*>(h);
  parallel_texts(n, nthreads, [&](int t, int nt) {
    std::vector<int> ids;
    WordPiece::Scratch sc;
    std::string text;
    for (int i = t; i < n; i += nt) {
      ids.clear();
      text.assign(buf + offs[i], (size_t)(offs[i + 1] - offs[i]));
      w->encode(text, ids, sc, (size_t)cap);
      lens[i] = (int32_t)ids.size();
      const int m = std::min((int)ids.size(), cap);
      for (int k = 0; k < m; ++k) out[(size_t)i * cap + k] = ids[k];
    }
  });
  return 0;
}
