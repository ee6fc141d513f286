// Sanitizer driver for the native behaviours parser (csrc/host/behaviors.cpp).
// Built by tests/test_sanitizers.py with -fsanitize=address,undefined and,
// separately, -fsanitize=thread (race detection / sanitizers).
//
// Every input is parsed sequentially (NRH_THREADS=1) and again with 2, 5 and
// 16 threads over 1-byte chunks (NRH_CHUNK_BYTES=1: every row its own chunk,
// so per-thread id tables are merged across many chunks); all outputs must be
// identical.  Inputs: ids first seen in later chunks, ids shared by every
// chunk, None / "" histories, labelled and unlabelled rows, a malformed row in
// a late chunk (must fail cleanly), and an empty result set of histories.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/newsrec_host.h"

struct Rows {
  std::string imps, hist;
  std::vector<int64_t> imp_off{0}, hist_off{0};
  std::vector<uint8_t> skip;
  void add(const std::string& imp, const std::string& h, bool none) {
    imps += imp;
    imp_off.push_back((int64_t)imps.size());
    hist += h;
    hist_off.push_back((int64_t)hist.size());
    skip.push_back(none || h.empty() ? 1 : 0);
  }
};

struct Result {
  int rc = 0;
  std::vector<int64_t> sizes = std::vector<int64_t>(6, 0);
  std::string news;
  std::vector<int64_t> news_off;
  std::vector<int32_t> imp_idx, imp_len, hist_idx, hist_len;
  std::vector<int8_t> labels;
  bool operator==(const Result& o) const {
    return rc == o.rc && sizes == o.sizes && news == o.news && news_off == o.news_off && imp_idx == o.imp_idx &&
           imp_len == o.imp_len && hist_idx == o.hist_idx && hist_len == o.hist_len && labels == o.labels;
  }
};

static Result parse(const Rows& r, int labels, const char* threads, const char* chunk) {
  setenv("NRH_THREADS", threads, 1);
  if (chunk) setenv("NRH_CHUNK_BYTES", chunk, 1); else unsetenv("NRH_CHUNK_BYTES");
  Result out;
  nrh_split* s = nullptr;
  out.rc = nrh_split_behaviors(r.imps.data(), r.imp_off.data(), r.hist.data(), r.hist_off.data(), r.skip.data(),
                               (int64_t)r.skip.size(), labels, &s);
  if (out.rc != NRH_OK) return out;
  nrh_split_sizes(s, out.sizes.data());
  out.news.resize(out.sizes[1]);
  out.news_off.resize(out.sizes[0] + 1);
  out.imp_idx.resize(out.sizes[2]);
  out.imp_len.resize(r.skip.size());
  out.hist_idx.resize(out.sizes[3]);
  out.hist_len.resize(out.sizes[4]);
  out.labels.resize(out.sizes[5]);
  nrh_split_copy(s, &out.news[0], out.news_off.data(), out.imp_idx.data(), out.imp_len.data(), out.hist_idx.data(),
                 out.hist_len.data(), labels ? out.labels.data() : nullptr);
  nrh_split_free(s);
  return out;
}

static Rows make_rows(std::mt19937_64& g, int n_rows, int n_ids, bool labels, bool malformed_late) {
  Rows r;
  std::vector<std::string> ids(n_ids);
  for (int i = 0; i < n_ids; ++i) ids[i] = "N" + std::to_string((i * 7919) % 100003);
  for (int row = 0; row < n_rows; ++row) {
    const int pool_h = std::min(n_ids, 20 + 3 * row), pool_c = std::min(n_ids, 30 + 2 * row);
    std::string h;
    const int nh = (int)(g() % 6);
    for (int k = 0; k < nh; ++k) h += (k ? " " : "") + ids[g() % pool_h];
    if (row % 5 == 0) h += " " + ids[0];  // an id shared by many chunks
    std::string imp;
    const int nc = 1 + (int)(g() % 5);
    for (int k = 0; k < nc; ++k) {
      imp += (k ? "  " : "") + ids[g() % pool_c];
      if (labels) imp += (g() % 3 == 0) ? "-1" : "-0";
    }
    if (malformed_late && row == n_rows - 3) imp += labels ? " N5-x" : "";
    const bool none = (nh == 0 && row % 5 != 0) && (row % 3 != 0);
    r.add(imp, none ? "" : h, none);
  }
  return r;
}

int main() {
  std::mt19937_64 g(1234);
  int failures = 0, cases = 0;
  const char* threads[] = {"2", "5", "16"};
  for (int rep = 0; rep < 3; ++rep) {
    for (int labels = 0; labels < 2; ++labels) {
      for (int n_rows : {97, 2000}) {
        const bool bad = rep == 2 && labels;
        Rows r = make_rows(g, n_rows, 300 + 50 * rep, labels, bad);
        const Result ref = parse(r, labels, "1", nullptr);
        if (bad != (ref.rc == NRH_ERR_UNSUPPORTED)) {
          std::fprintf(stderr, "case rep=%d labels=%d rows=%d: sequential rc %d\n", rep, labels, n_rows, ref.rc);
          ++failures;
        }
        for (const char* t : threads) {
          ++cases;
          const Result got = parse(r, labels, t, "1");
          if (!(got == ref)) {
            std::fprintf(stderr, "mismatch rep=%d labels=%d rows=%d threads=%s rc=%d/%d\n", rep, labels, n_rows, t,
                         got.rc, ref.rc);
            ++failures;
          }
        }
      }
    }
  }
  // no history at all: a valid parse with zero history rows
  Rows none;
  for (int i = 0; i < 40; ++i) none.add("N1-1 N2-0", "", true);
  const Result a = parse(none, 1, "1", nullptr), b = parse(none, 1, "5", "1");
  if (!(a == b) || a.rc != NRH_OK || a.sizes[4] != 0) ++failures;
  std::printf("behaviors sanitizer driver: %d parallel cases, %d failures\n", cases, failures);
  return failures ? 1 : 0;
}
