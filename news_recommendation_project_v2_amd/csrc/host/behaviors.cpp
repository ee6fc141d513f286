// Native MIND behaviours parser, C-ABI in include/newsrec_host.h.
//
// Restates split_impressions_and_history (data_utils.py:168-232): rows in
// order; per row the history tokens are registered before the impression
// tokens; a news id gets the next position the first time it is seen; labels
// are the integer after "-".
//
// Parallel over rows without changing that order: the rows are cut into
// contiguous byte-balanced chunks, one thread each; a thread numbers the ids of
// its chunk in ITS first-appearance order (local ids) in a private table.  An
// id's first appearance overall lies in the first chunk that contains it, and
// inside that chunk its local order is the global order, so registering every
// chunk's local ids, chunk by chunk, into one global table yields exactly the
// sequential numbering; each thread then rewrites its tokens through its
// local -> global map into its slice of the outputs.  Tables are open
// addressing on 8-byte (tag, id) slots with ids of <= 16 bytes kept inline in
// a dense per-id array (MIND ids are "N" + digits), so a lookup touches one
// slot and one key and never the input text of the id's first occurrence.
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/newsrec_host.h"

namespace {

thread_local char g_err[256];

void set_err(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Python's str.split() whitespace restricted to ASCII (the caller guarantees ASCII):
// \t \n \v \f \r, 0x1c-0x1f and space.
inline bool is_ws(unsigned char c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f); }

inline uint64_t hash_bytes(const char* p, int64_t n) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a 64
  for (int64_t i = 0; i < n; ++i) h = (h ^ (unsigned char)p[i]) * 1099511628211ull;
  return h ^ (h >> 29);
}

constexpr int kInline = 16;

// Open addressing over 8-byte slots (hash tag << 32 | id + 1; 0 = empty) with
// the ids' bytes in dense per-id arrays: a lookup reads one slot and, on a tag
// match, one 16-byte inline key, so a table of ~72k MIND ids stays ~3 MiB.
struct IdTable {
  std::vector<uint64_t> slots;
  struct Key {
    char b[kInline];
  };
  std::vector<Key> keys;     // per id: bytes when n <= kInline
  std::vector<int32_t> lens;  // per id
  std::vector<std::pair<const char*, int64_t>> ids;  // first-appearance order (bytes in the input)
  uint64_t mask = 0;

  explicit IdTable(size_t cap = 1 << 12) { rehash(cap); }

  void rehash(size_t cap) {
    std::vector<uint64_t> old;
    old.swap(slots);
    slots.assign(cap, 0);
    mask = cap - 1;
    for (uint64_t v : old)
      if (v) {
        const int32_t id = (int32_t)(uint32_t)v - 1;
        const auto& k = ids[(size_t)id];
        uint64_t i = hash_bytes(k.first, k.second) & mask;
        while (slots[i]) i = (i + 1) & mask;
        slots[i] = v;
      }
  }
  int32_t get(const char* p, int64_t n) { return get_h(hash_bytes(p, n), p, n); }
  int32_t get_h(uint64_t h, const char* p, int64_t n) {
    const uint64_t tag = h >> 32;
    uint64_t i = h & mask;
    while (const uint64_t v = slots[i]) {
      if ((v >> 32) == tag) {
        const int32_t id = (int32_t)(uint32_t)v - 1;
        if (lens[(size_t)id] == n &&
            memcmp(n <= kInline ? keys[(size_t)id].b : ids[(size_t)id].first, p, (size_t)n) == 0)
          return id;
      }
      i = (i + 1) & mask;
    }
    const int32_t id = (int32_t)ids.size();
    slots[i] = tag << 32 | (uint64_t)(uint32_t)(id + 1);
    ids.emplace_back(p, n);
    lens.push_back((int32_t)n);
    Key k{};
    if (n <= kInline) memcpy(k.b, p, (size_t)n);
    keys.push_back(k);
    if (ids.size() * 2 > slots.size()) rehash(slots.size() * 2);
    return id;
  }
};

// One contiguous run of rows [r0, r1) parsed with a private id table.  Every
// buffer a worker writes is sized by the main thread before the workers start
// (counting pass first), so workers do not allocate: in a sandboxed process a
// worker's first malloc creates a glibc arena, and that cost 2-3x the parse.
struct Chunk {
  int64_t r0 = 0, r1 = 0;
  int64_t n_hist = 0, n_imp = 0, rows_h = 0;  // counting pass
  int64_t o_hist = 0, o_imp = 0, o_rows_h = 0;  // output offsets (prefix sums)
  IdTable table;
  std::vector<uint64_t> hashes;  // per local id, for the merge
  std::vector<int32_t> to_global;  // local id -> global id
  int rc = NRH_OK;
  char msg[256] = {0};
};

inline int64_t count_tokens(const char* p, const char* e) {
  int64_t n = 0;
  bool in = false;
  for (; p < e; ++p) {
    const bool w = is_ws((unsigned char)*p);
    n += (!w && !in);
    in = !w;
  }
  return n;
}

void count_chunk(Chunk& c, const char* imps, const int64_t* imp_off, const char* hist, const int64_t* hist_off,
                 const uint8_t* hist_skip) {
  for (int64_t r = c.r0; r < c.r1; ++r) {
    if (!(hist_skip && hist_skip[r])) {
      c.n_hist += count_tokens(hist + hist_off[r], hist + hist_off[r + 1]);
      ++c.rows_h;
    }
    c.n_imp += count_tokens(imps + imp_off[r], imps + imp_off[r + 1]);
  }
}

// Parse [r0, r1) into the chunk's slices of the outputs, as local ids.
void parse_chunk(Chunk& c, const char* imps, const int64_t* imp_off, const char* hist, const int64_t* hist_off,
                 const uint8_t* hist_skip, bool has_labels, int32_t* imp_idx, int32_t* imp_len, int32_t* hist_idx,
                 int32_t* hist_len, int8_t* labels) {
  int32_t* hi = hist_idx + c.o_hist;
  int32_t* hl = hist_len + c.o_rows_h;
  int32_t* ii = imp_idx + c.o_imp;
  int32_t* il = imp_len + c.r0;
  int8_t* lb = labels ? labels + c.o_imp : nullptr;
  auto token_id = [&](const char* t, int64_t n) {
    const uint64_t h = hash_bytes(t, n);
    const size_t before = c.table.ids.size();
    const int32_t id = c.table.get_h(h, t, n);
    if (c.table.ids.size() != before) c.hashes.push_back(h);
    return id;
  };
  for (int64_t r = c.r0; r < c.r1; ++r) {
    if (!(hist_skip && hist_skip[r])) {
      const char* p = hist + hist_off[r];
      const char* e = hist + hist_off[r + 1];
      int32_t cnt = 0;
      while (p < e) {
        while (p < e && is_ws((unsigned char)*p)) ++p;
        const char* t = p;
        while (p < e && !is_ws((unsigned char)*p)) ++p;
        if (p > t) {
          *hi++ = token_id(t, p - t);
          ++cnt;
        }
      }
      *hl++ = cnt;
    }
    const char* p = imps + imp_off[r];
    const char* e = imps + imp_off[r + 1];
    int32_t cnt = 0;
    while (p < e) {
      while (p < e && is_ws((unsigned char)*p)) ++p;
      const char* t = p;
      while (p < e && !is_ws((unsigned char)*p)) ++p;
      if (p == t) continue;
      int64_t n = p - t;
      if (has_labels) {
        // "<news>-<label>": k.split("-") -> (x[0], int(x[1])); only the plain
        // single-dash form with a 0/1..127 decimal label is handled natively.
        const char* dash = (const char*)memchr(t, '-', (size_t)n);
        if (!dash || memchr(dash + 1, '-', (size_t)(p - dash - 1)) || dash + 1 == p) {
          snprintf(c.msg, sizeof(c.msg), "row %lld: impression token without a plain '<id>-<label>' form",
                   (long long)r);
          c.rc = NRH_ERR_UNSUPPORTED;
          return;
        }
        int v = 0;
        for (const char* q = dash + 1; q < p; ++q) {
          if (*q < '0' || *q > '9' || v > 11) {
            snprintf(c.msg, sizeof(c.msg), "row %lld: label is not a small decimal integer", (long long)r);
            c.rc = NRH_ERR_UNSUPPORTED;
            return;
          }
          v = v * 10 + (*q - '0');
        }
        *lb++ = (int8_t)v;
        n = dash - t;
      }
      *ii++ = token_id(t, n);
      ++cnt;
    }
    if (cnt == 0 && has_labels) {  // zip(*[]) raises in the reference
      snprintf(c.msg, sizeof(c.msg), "row %lld: empty impression row", (long long)r);
      c.rc = NRH_ERR_UNSUPPORTED;
      return;
    }
    *il++ = cnt;
  }
}

template <typename F>
void parallel(int T, F&& f) {
  if (T == 1) {
    f(0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve((size_t)T - 1);
  for (int t = 1; t < T; ++t) th.emplace_back(f, t);
  f(0);
  for (auto& x : th) x.join();
}

int n_threads_for(int64_t n_rows, int64_t n_bytes) {
  int t = 16;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) t = std::min(t, CPU_COUNT(&set));
  if (const char* e = getenv("NRH_THREADS")) t = atoi(e);
  // >= 4 MiB of text per thread (NRH_CHUNK_BYTES overrides): small inputs stay sequential
  int64_t per = 1 << 22;
  if (const char* e = getenv("NRH_CHUNK_BYTES")) per = std::max<int64_t>(1, atoll(e));
  t = (int)std::min<int64_t>(t, std::max<int64_t>(1, n_bytes / per));
  t = (int)std::min<int64_t>(t, std::max<int64_t>(1, n_rows));
  return std::max(1, t);
}

}  // namespace

struct nrh_split {
  IdTable table{1 << 16};
  std::vector<int32_t> imp_idx, imp_len, hist_idx, hist_len;
  std::vector<int8_t> labels;
  bool has_labels = false;
  int64_t news_bytes = 0;
};

extern "C" const char* nrh_last_error(void) { return g_err; }

// sha256 of behaviors.cpp + include/newsrec_host.h (native.source_hash), set by the build
#ifndef NRH_BUILD_HASH
#define NRH_BUILD_HASH "unknown"
#endif
static const char kBuildTag[] __attribute__((used)) = "nrh-build-hash:" NRH_BUILD_HASH;

extern "C" const char* nrh_build_hash(void) { return kBuildTag + 15; }

extern "C" int nrh_split_behaviors(const char* imps, const int64_t* imp_off, const char* hist, const int64_t* hist_off,
                                   const uint8_t* hist_skip, int64_t n_rows, int label_present, nrh_split** out) {
  g_err[0] = 0;
  if (!out || n_rows < 0 || (n_rows > 0 && (!imps || !imp_off || !hist_off))) {
    set_err("nrh_split_behaviors: bad arguments");
    return NRH_ERR_INVALID;
  }
  std::unique_ptr<nrh_split> s(new nrh_split());
  s->has_labels = label_present != 0;
  const bool lab = s->has_labels;
  if (n_rows == 0) {
    *out = s.release();
    return NRH_OK;
  }
  // byte-balanced contiguous row chunks
  const int64_t total = (imp_off[n_rows] - imp_off[0]) + (hist_off[n_rows] - hist_off[0]);
  const int T = n_threads_for(n_rows, total);
  std::vector<Chunk> ch(T);
  {
    int64_t r = 0;
    for (int t = 0; t < T; ++t) {
      ch[t].r0 = r;
      if (t == T - 1) {
        r = n_rows;
      } else {
        const int64_t target = total * (t + 1) / T;
        while (r < n_rows && (imp_off[r] - imp_off[0]) + (hist_off[r] - hist_off[0]) < target) ++r;
      }
      ch[t].r1 = r;
    }
  }
  // 1. count tokens (workers: no allocation)
  parallel(T, [&](int t) { count_chunk(ch[t], imps, imp_off, hist, hist_off, hist_skip); });
  int64_t nh = 0, ni = 0, nrh = 0;
  for (Chunk& c : ch) {
    c.o_hist = nh;
    c.o_imp = ni;
    c.o_rows_h = nrh;
    nh += c.n_hist;
    ni += c.n_imp;
    nrh += c.rows_h;
    // a chunk's distinct ids: <= its tokens; a MIND-sized chunk sees up to ~10^5
    const size_t cap = (size_t)std::min<int64_t>(std::max<int64_t>(c.n_hist + c.n_imp, 1), 1 << 17);
    size_t pow2 = 1 << 12;
    while (pow2 < 2 * cap) pow2 <<= 1;
    c.table.rehash(pow2);
    c.table.ids.reserve(pow2 / 2);
    c.table.keys.reserve(pow2 / 2);
    c.table.lens.reserve(pow2 / 2);
    c.hashes.reserve(pow2 / 2);
  }
  s->imp_idx.resize((size_t)ni);
  s->hist_idx.resize((size_t)nh);
  s->hist_len.resize((size_t)nrh);
  s->imp_len.resize((size_t)n_rows);
  if (lab) s->labels.resize((size_t)ni);
  // 2. parse into the output slices as local ids
  parallel(T, [&](int t) {
    parse_chunk(ch[t], imps, imp_off, hist, hist_off, hist_skip, lab, s->imp_idx.data(), s->imp_len.data(),
                s->hist_idx.data(), s->hist_len.data(), lab ? s->labels.data() : nullptr);
  });
  for (const Chunk& c : ch)  // the first failing row overall is in the first failing chunk
    if (c.rc != NRH_OK) {
      set_err("%s", c.msg);
      return c.rc;
    }
  // 3. merge: register each chunk's ids, in chunk order and local first-appearance order
  for (Chunk& c : ch) {
    c.to_global.resize(c.table.ids.size());
    for (size_t i = 0; i < c.table.ids.size(); ++i)
      c.to_global[i] = s->table.get_h(c.hashes[i], c.table.ids[i].first, c.table.ids[i].second);
  }
  // 4. local -> global ids in place
  parallel(T, [&](int t) {
    const Chunk& c = ch[(size_t)t];
    const int32_t* g = c.to_global.data();
    int32_t* ii = s->imp_idx.data() + c.o_imp;
    for (int64_t k = 0; k < c.n_imp; ++k) ii[k] = g[ii[k]];
    int32_t* hi = s->hist_idx.data() + c.o_hist;
    for (int64_t k = 0; k < c.n_hist; ++k) hi[k] = g[hi[k]];
  });
  for (auto& id : s->table.ids) s->news_bytes += id.second;
  *out = s.release();
  return NRH_OK;
}

extern "C" int nrh_split_sizes(const nrh_split* s, int64_t sizes[6]) {
  if (!s || !sizes) return NRH_ERR_INVALID;
  sizes[0] = (int64_t)s->table.ids.size();
  sizes[1] = s->news_bytes;
  sizes[2] = (int64_t)s->imp_idx.size();
  sizes[3] = (int64_t)s->hist_idx.size();
  sizes[4] = (int64_t)s->hist_len.size();
  sizes[5] = (int64_t)s->labels.size();
  return NRH_OK;
}

extern "C" int nrh_split_copy(const nrh_split* s, char* news_bytes, int64_t* news_off, int32_t* imp_idx,
                              int32_t* imp_len, int32_t* hist_idx, int32_t* hist_len, int8_t* labels) {
  if (!s) return NRH_ERR_INVALID;
  int64_t o = 0;
  if (news_off) news_off[0] = 0;
  for (size_t i = 0; i < s->table.ids.size(); ++i) {
    const auto& id = s->table.ids[i];
    if (news_bytes) memcpy(news_bytes + o, id.first, (size_t)id.second);
    o += id.second;
    if (news_off) news_off[i + 1] = o;
  }
  auto cp = [](const auto& v, auto* dst) {
    if (dst && !v.empty()) memcpy(dst, v.data(), v.size() * sizeof(v[0]));
  };
  cp(s->imp_idx, imp_idx);
  cp(s->imp_len, imp_len);
  cp(s->hist_idx, hist_idx);
  cp(s->hist_len, hist_len);
  cp(s->labels, labels);
  return NRH_OK;
}

extern "C" void nrh_split_free(nrh_split* s) { delete s; }
