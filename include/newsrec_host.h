/*
 * newsrec_host.h — C-ABI of libnewsrec_host.so, the native host-side data path
 * (SURVEY §8(f) #2): MIND behaviours -> first-appearance news ids + int32 CSR
 * index arrays, bit-identical to the reference's pure-Python loop
 * split_impressions_and_history (src/news_rec_utils/data_utils.py:168-232).
 *
 * Bound with ctypes by news_recommendation_project_v2_amd/native.py, which
 * falls back to the Python restatement (same outputs) for inputs the native
 * parser declines (non-ASCII bytes, malformed labels): it returns
 * NRH_ERR_UNSUPPORTED for those instead of guessing Python's str semantics.
 *
 * Conventions: plain pointers and sizes; the parser owns its result until
 * nrh_split_free; errors are negative return codes with a message from
 * nrh_last_error() (thread-local).
 */
#ifndef NEWSREC_HOST_H
#define NEWSREC_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NRH_OK 0
#define NRH_ERR_INVALID -1
#define NRH_ERR_UNSUPPORTED -3

typedef struct nrh_split nrh_split;

/* Hash of the sources the library was built from (16 hex digits: sha256 of
 * csrc/host/behaviors.cpp + this header); native.py refuses a stale library. */
const char* nrh_build_hash(void);

/*
 * Parse n_rows behaviours rows.  imps / hist are the concatenated ASCII bytes
 * of the Impressions / History columns with row offsets imp_off / hist_off
 * [n_rows + 1]; hist_skip[i] != 0 marks a falsy history (None / "": no history
 * row, data_utils.py:183).  Tokens are split on ASCII whitespace like
 * str.split(); with label_present (the reference tests "-" in the first
 * impression row) each impression token is "<news>-<digits>".
 * On success *out receives a handle for nrh_split_sizes / nrh_split_copy.
 */
int nrh_split_behaviors(const char* imps, const int64_t* imp_off, const char* hist, const int64_t* hist_off,
                        const uint8_t* hist_skip, int64_t n_rows, int label_present, nrh_split** out);

/* sizes[0..5] = n_news, news id bytes, C (impression tokens), H (history
 * tokens), history rows, label count (== C if labels present else 0). */
int nrh_split_sizes(const nrh_split* s, int64_t sizes[6]);

/* Copy the results out (every pointer sized by nrh_split_sizes):
 * news_bytes/news_off [n_news + 1]: ids in first-appearance order;
 * imp_idx [C], imp_len [n_rows]; hist_idx [H], hist_len [history rows];
 * labels [C] (int8, nullable when absent). */
int nrh_split_copy(const nrh_split* s, char* news_bytes, int64_t* news_off, int32_t* imp_idx, int32_t* imp_len,
                   int32_t* hist_idx, int32_t* hist_len, int8_t* labels);

void nrh_split_free(nrh_split* s);

const char* nrh_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* NEWSREC_HOST_H */
