// Native MIND behaviours parser, C-ABI in include/newsrec_host.h.
//
// Restates split_impressions_and_history (data_utils.py:168-232): rows in
// order; per row the history tokens are registered before the impression
// tokens; a news id gets the next position the first time it is seen; labels
// are the integer after "-".  One pass over the bytes with an open-addressing
// table of (hash, offset, length) keyed on the id bytes (ids stay in the
// caller's input buffers, never copied until nrh_split_copy).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <memory>
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

struct IdTable {
  struct Slot {
    uint64_t h;
    const char* p;
    int64_t n;
    int32_t id;  // -1 = empty
  };
  std::vector<Slot> slots;
  std::vector<std::pair<const char*, int64_t>> ids;  // first-appearance order
  uint64_t mask = 0;

  IdTable() { rehash(1 << 16); }

  void rehash(size_t cap) {
    std::vector<Slot> old;
    old.swap(slots);
    slots.assign(cap, Slot{0, nullptr, 0, -1});
    mask = cap - 1;
    for (const Slot& s : old)
      if (s.id >= 0) place(s);
  }
  void place(const Slot& s) {
    uint64_t i = s.h & mask;
    while (slots[i].id >= 0) i = (i + 1) & mask;
    slots[i] = s;
  }
  int32_t get(const char* p, int64_t n) {
    const uint64_t h = hash_bytes(p, n);
    uint64_t i = h & mask;
    while (slots[i].id >= 0) {
      const Slot& s = slots[i];
      if (s.h == h && s.n == n && memcmp(s.p, p, (size_t)n) == 0) return s.id;
      i = (i + 1) & mask;
    }
    const int32_t id = (int32_t)ids.size();
    slots[i] = Slot{h, p, n, id};
    ids.emplace_back(p, n);
    if (ids.size() * 2 > slots.size()) rehash(slots.size() * 2);
    return id;
  }
};

}  // namespace

struct nrh_split {
  IdTable table;
  std::vector<int32_t> imp_idx, imp_len, hist_idx, hist_len;
  std::vector<int8_t> labels;
  bool has_labels = false;
  int64_t news_bytes = 0;
};

extern "C" const char* nrh_last_error(void) { return g_err; }

extern "C" int nrh_split_behaviors(const char* imps, const int64_t* imp_off, const char* hist, const int64_t* hist_off,
                                   const uint8_t* hist_skip, int64_t n_rows, int label_present, nrh_split** out) {
  g_err[0] = 0;
  if (!out || n_rows < 0 || (n_rows > 0 && (!imps || !imp_off || !hist_off))) {
    set_err("nrh_split_behaviors: bad arguments");
    return NRH_ERR_INVALID;
  }
  std::unique_ptr<nrh_split> s(new nrh_split());
  s->has_labels = label_present != 0;
  s->imp_len.reserve((size_t)n_rows);
  for (int64_t r = 0; r < n_rows; ++r) {
    if (!(hist_skip && hist_skip[r])) {
      const char* p = hist + hist_off[r];
      const char* e = hist + hist_off[r + 1];
      int32_t cnt = 0;
      while (p < e) {
        while (p < e && is_ws((unsigned char)*p)) ++p;
        const char* t = p;
        while (p < e && !is_ws((unsigned char)*p)) ++p;
        if (p > t) {
          s->hist_idx.push_back(s->table.get(t, p - t));
          ++cnt;
        }
      }
      s->hist_len.push_back(cnt);
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
      if (s->has_labels) {
        // "<news>-<label>": k.split("-") -> (x[0], int(x[1])); only the plain
        // single-dash form with a 0/1..127 decimal label is handled natively.
        const char* dash = (const char*)memchr(t, '-', (size_t)n);
        if (!dash || memchr(dash + 1, '-', (size_t)(p - dash - 1)) || dash + 1 == p) {
          set_err("row %lld: impression token without a plain '<id>-<label>' form", (long long)r);
          return NRH_ERR_UNSUPPORTED;
        }
        int v = 0;
        for (const char* q = dash + 1; q < p; ++q) {
          if (*q < '0' || *q > '9' || v > 11) {
            set_err("row %lld: label is not a small decimal integer", (long long)r);
            return NRH_ERR_UNSUPPORTED;
          }
          v = v * 10 + (*q - '0');
        }
        s->labels.push_back((int8_t)v);
        n = dash - t;
      }
      s->imp_idx.push_back(s->table.get(t, n));
      ++cnt;
    }
    if (cnt == 0 && s->has_labels) {  // zip(*[]) raises in the reference
      set_err("row %lld: empty impression row", (long long)r);
      return NRH_ERR_UNSUPPORTED;
    }
    s->imp_len.push_back(cnt);
  }
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
