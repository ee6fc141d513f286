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

// Impressions of up to RANK_REG_BLOCKS x 64 candidates (every MIND impression:
// at most ~300): the values stay in registers, lane l owning candidates
// 64 b + l, and every other value is broadcast with v_readlane (no LDS, so
// the kernel runs at full occupancy).  Larger ones are left to the LDS kernel.
constexpr int RANK_REG_BLOCKS = 5;

// NB = number of 64-candidate register blocks (compile time: no guarded work
// for the blocks an impression does not have; most have one).
template <int NB>
__device__ __forceinline__ void dense_rank_reg(const float* __restrict__ sc, int c, int lane, int32_t* __restrict__ rk) {
  float v[NB];
  int first[NB], r[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    v[b] = b * 64 + lane < c ? sc[b * 64 + lane] : 0.f;
    first[b] = 1;
    r[b] = 1;
  }
  // pass 1: candidate i is the first occurrence of its value
#pragma unroll
  for (int bk = 0; bk < NB; ++bk) {
    const int kend = min(64, c - bk * 64);
    for (int k = 0; k < kend; ++k) {
      const float sk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[bk]), k));
#pragma unroll
      for (int bi = bk; bi < NB; ++bi)
        if (bk * 64 + k < bi * 64 + lane && sk == v[bi]) first[bi] = 0;
    }
  }
  // pass 2: rank = 1 + distinct values strictly greater
#pragma unroll
  for (int bk = 0; bk < NB; ++bk) {
    const int kend = min(64, c - bk * 64);
    for (int k = 0; k < kend; ++k) {
      if (!__builtin_amdgcn_readlane(first[bk], k)) continue;  // uniform
      const float sk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[bk]), k));
#pragma unroll
      for (int bi = 0; bi < NB; ++bi) r[bi] += sk > v[bi] ? 1 : 0;
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b)
    if (b * 64 + lane < c) rk[b * 64 + lane] = r[b];
}

__global__ __launch_bounds__(256) void dense_rank_reg_kernel(const float* __restrict__ scores,
                                                             const int64_t* __restrict__ coff, int64_t n_imp,
                                                             int32_t* __restrict__ ranks) {
  const int lane = threadIdx.x & 63;
  const int64_t imp = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (imp >= n_imp) return;  // wave-uniform
  const int64_t c0 = coff[imp];
  const int64_t cc = coff[imp + 1] - c0;
  if (cc > 64 * RANK_REG_BLOCKS || cc <= 0) return;
  const int c = (int)cc;
  switch ((c + 63) / 64) {
    case 1: dense_rank_reg<1>(scores + c0, c, lane, ranks + c0); break;
    case 2: dense_rank_reg<2>(scores + c0, c, lane, ranks + c0); break;
    case 3: dense_rank_reg<3>(scores + c0, c, lane, ranks + c0); break;
    case 4: dense_rank_reg<4>(scores + c0, c, lane, ranks + c0); break;
    default: dense_rank_reg<5>(scores + c0, c, lane, ranks + c0); break;
  }
}

// The rest (RANK_REG_BLOCKS x 64 < c <= RANK_MAXC) through LDS.  A grid-stride
// loop over groups of 4 impressions (uniform trip count per workgroup, so the
// barriers line up): its LDS footprint holds few workgroups per CU and it
// skips the impressions the register kernel took.
__global__ __launch_bounds__(256) void dense_rank_kernel(const float* __restrict__ scores,
                                                         const int64_t* __restrict__ coff,
                                                         int64_t n_imp, int32_t* __restrict__ ranks,
                                                         int32_t* __restrict__ status) {
  __shared__ float s_val[4][RANK_MAXC];
  __shared__ unsigned char s_first[4][RANK_MAXC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t n_groups = (n_imp + 3) / 4;
  for (int64_t g = blockIdx.x; g < n_groups; g += gridDim.x) {
  const int64_t imp = g * 4 + w;
  int64_t c0 = 0;
  int c = 0;
  if (imp < n_imp) {
    c0 = coff[imp];
    const int64_t cc = coff[imp + 1] - c0;
    if (cc > RANK_MAXC) {
      if (lane == 0) atomicExch(status, NR_ERR_UNSUPPORTED);
      c = 0;
    } else {
      c = cc > 64 * RANK_REG_BLOCKS ? (int)cc : 0;  // smaller ones: dense_rank_reg_kernel
    }
  }
  float* sv = s_val[w];
  unsigned char* sf = s_first[w];
  __syncthreads();  // the previous group's reads of this wave's slots are done
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
  }  // group loop
}

}  // namespace nr

extern "C" int nr_dense_rank(const float* scores, const int64_t* cand_off, int64_t n_imp,
                             int32_t* ranks, int32_t* status, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(n_imp >= 0, "nr_dense_rank: n_imp < 0");
  if (n_imp == 0) return NR_OK;
  NR_CHECK_ARG(scores && cand_off && ranks && status, "nr_dense_rank: null pointer");
  NR_CHECK_DEVICE("nr_dense_rank", scores, cand_off, ranks, status);
  const int64_t groups = (n_imp + 3) / 4;
  hipLaunchKernelGGL(nr::dense_rank_reg_kernel, dim3((unsigned)groups), dim3(256), 0, (hipStream_t)stream, scores,
                     cand_off, n_imp, ranks);
  hipLaunchKernelGGL(nr::dense_rank_kernel, dim3((unsigned)(groups < 1024 ? groups : 1024)), dim3(256), 0,
                     (hipStream_t)stream, scores, cand_off, n_imp, ranks, status);
  NR_CHECK_LAUNCH("nr_dense_rank");
  return NR_OK;
}
