// Dense descending rank per impression (integer, bit-exact given the scores).
//
// Restates rank_group_preds (data_utils.py:414-415):
//   group_items(scores, imp_counts, lambda x: rankdata(-x, method="dense"))
// rank_i = 1 + |{distinct s_j : s_j > s_i}| over the impression's candidates.
//
// One wave per impression; the impression's scores are staged in LDS and two
// O(c^2 / 64) passes run with every lane owning one candidate: pass 1 marks
// the first occurrence of each value, pass 2 counts the marked values that are
// strictly greater.  MIND impressions have at most ~300 candidates; up to
// RANK_MAXC are supported, larger ones set *status = NR_ERR_UNSUPPORTED.
#include "nr_common.h"

namespace nr {

constexpr int RANK_MAXC = 2048;

__global__ __launch_bounds__(256) void dense_rank_kernel(const float* __restrict__ scores,
                                                         const int64_t* __restrict__ coff,
                                                         int64_t n_imp, int32_t* __restrict__ ranks,
                                                         int32_t* __restrict__ status) {
  __shared__ float s_val[4][RANK_MAXC];
  __shared__ unsigned char s_first[4][RANK_MAXC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t imp = (int64_t)blockIdx.x * 4 + w;
  int64_t c0 = 0;
  int c = 0;
  if (imp < n_imp) {
    c0 = coff[imp];
    const int64_t cc = coff[imp + 1] - c0;
    if (cc > RANK_MAXC) {
      if (lane == 0) atomicExch(status, NR_ERR_UNSUPPORTED);
      c = 0;
    } else {
      c = (int)cc;
    }
  }
  float* sv = s_val[w];
  unsigned char* sf = s_first[w];
  for (int i = lane; i < c; i += 64) sv[i] = scores[c0 + i];
  __syncthreads();
  for (int i0 = 0; i0 < c; i0 += 64) {
    const int i = i0 + lane;
    const float si = i < c ? sv[i] : 0.f;
    int first = 1;
    const int kend = min(i0 + 64, c);
    for (int k = 0; k < kend; ++k) {
      const float sk = sv[k];
      if (k < i && sk == si) first = 0;
    }
    if (i < c) sf[i] = (unsigned char)first;
  }
  __syncthreads();
  for (int i0 = 0; i0 < c; i0 += 64) {
    const int i = i0 + lane;
    const float si = i < c ? sv[i] : 0.f;
    int r = 1;
    for (int k = 0; k < c; ++k) r += (sf[k] && sv[k] > si) ? 1 : 0;
    if (i < c) ranks[c0 + i] = r;
  }
}

}  // namespace nr

extern "C" int nr_dense_rank(const float* scores, const int64_t* cand_off, int64_t n_imp,
                             int32_t* ranks, int32_t* status, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(n_imp >= 0, "nr_dense_rank: n_imp < 0");
  if (n_imp == 0) return NR_OK;
  NR_CHECK_ARG(scores && cand_off && ranks && status, "nr_dense_rank: null pointer");
  hipLaunchKernelGGL(nr::dense_rank_kernel, dim3((unsigned)((n_imp + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, scores, cand_off, n_imp, ranks, status);
  NR_CHECK_LAUNCH("nr_dense_rank");
  return NR_OK;
}
