// MIND metrics per impression on the device, from the dense
// ranks of nr_dense_rank and 0/1 labels.  Replaces evaluation.score_row
// (evaluation.py:34-54: roc_auc_score(labels, 1 / rank), mrr_score,
// ndcg_score @5 / @10) run per impression in a ProcessPoolExecutor.
//
// One wave per impression; ranks in registers up to 320 candidates, beyond
// that a 2048-bin LDS histogram of the dense ranks:
//   AUC  = (sum over positives of the tie-averaged ascending rank - P(P+1)/2) / (P N)
//          (Mann-Whitney U == sklearn's trapezoidal ROC AUC on 1/rank; NaN when
//          P == 0 or N == 0, like sklearn 1.7's undefined-AUC result)
//   MRR  = sum_pos 1 / rank / P ;  nDCG@k = sum_{pos, rank <= k} 1 / log2(rank + 1)
//          / sum_{j < min(P, k)} 1 / log2(j + 2)
// MRR / nDCG use np.argsort(1 / rank)[::-1] positions in the reference, which
// equal rank - 1 only when no two candidates tie; impressions with ties are
// flagged (tie_flag = 1) for the host to evaluate with numpy's own tie order.
#include "nr_common.h"

namespace nr {

constexpr int kMaxCand = 2048;
// the rank-bin rewrite below packs (run << 12) | k with run, k <= kMaxCand in
// 12-bit fields: raising kMaxCand past 4095 needs a wider packing
static_assert(kMaxCand < 4096, "metrics_kernel packs counts in 12 bits");

// nDCG discounts 1 / log2(j + 2), j < 10, as numpy computes them (host libm,
// float64): only positions <= 10 enter nDCG@5 / @10, so no device log2 runs.
__constant__ double kDisc[10] = {1.0, 0.6309297535714575, 0.5, 0.43067655807339306, 0.38685280723454163,
                                 0.3562071871080222, 0.3333333333333333, 0.31546487678572877, 0.3010299956639812,
                                 0.2890648263178879};

// The per-impression outputs from the AUC / MRR / nDCG partial sums (lane 0).
__device__ __forceinline__ void write_metrics(double* o, int P, int N, double S, double rr, double d5, double d10) {
  const double nan = __builtin_nan("");
  o[0] = (P == 0 || N == 0) ? nan : (S - 0.5 * (double)P * (double)(P + 1)) / ((double)P * (double)N);
  double i5 = 0.0, i10 = 0.0;
  for (int j = 0; j < min(P, 10); ++j) {
    const double disc = kDisc[j];
    if (j < 5) i5 += disc;
    i10 += disc;
  }
  o[1] = rr / (double)P;  // P == 0 -> NaN like 0 / 0 in numpy
  o[2] = d5 / i5;
  o[3] = d10 / i10;
}

// Impressions of up to 5 x 64 candidates (every MIND impression): ranks and
// labels in registers (lane l owns candidates 64 b + l), each positive's
// count of lower-ranked and tied candidates from v_readlane broadcasts -- no
// LDS histogram.  NB = number of 64-candidate blocks.
constexpr int kRegBlocks = 5;

template <int NB>
__device__ __forceinline__ void metrics_reg(const int32_t* __restrict__ rk, const float* __restrict__ lb, int c,
                                            int lane, double* o, int32_t* tie, int32_t* status) {
  int r[NB];
  float y[NB];
  int P = 0, maxr = 0, bad = 0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const bool in = b * 64 + lane < c;
    r[b] = in ? rk[b * 64 + lane] : 0;
    y[b] = in ? lb[b * 64 + lane] : 0.f;
    if (in && (r[b] < 1 || r[b] > c)) bad = 1;
    if (y[b] != 0.f && y[b] != 1.f) bad = 1;
    P += y[b] != 0.f;
    maxr = max(maxr, r[b]);
  }
  for (int m = 32; m >= 1; m >>= 1) {
    P += __shfl_xor(P, m, 64);
    maxr = max(maxr, __shfl_xor(maxr, m, 64));
    bad |= __shfl_xor(bad, m, 64);
  }
  if (bad) {
    if (lane == 0) { atomicOr(status, 2); o[0] = o[1] = o[2] = o[3] = __builtin_nan(""); *tie = 1; }
    return;
  }
  // per positive (uniform loop over the ballot of label 1): candidates ranked
  // strictly below it (larger dense rank) and tied with it, summed over the wave
  // (lanes past c hold rank 0: neither)
  double S = 0.0, rr = 0.0, d5 = 0.0, d10 = 0.0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    uint64_t pm = __ballot(y[b] != 0.f);
    while (pm) {
      const int k = __builtin_ctzll(pm);
      pm &= pm - 1;
      const int rp = __builtin_amdgcn_readlane(r[b], k);
      int below = 0, eq = 0;
#pragma unroll
      for (int bb = 0; bb < NB; ++bb) {
        below += r[bb] > rp ? 1 : 0;
        eq += r[bb] == rp ? 1 : 0;
      }
      for (int m = 32; m >= 1; m >>= 1) {
        below += __shfl_xor(below, m, 64);
        eq += __shfl_xor(eq, m, 64);
      }
      S += (double)below + 0.5 * (double)(eq + 1);
      rr += 1.0 / (double)rp;
      if (rp <= 10) {
        d10 += kDisc[rp - 1];
        if (rp <= 5) d5 += kDisc[rp - 1];
      }
    }
  }
  if (lane == 0) {
    write_metrics(o, P, c - P, S, rr, d5, d10);
    *tie = maxr < c ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void metrics_reg_kernel(const int32_t* __restrict__ ranks,
                                                          const float* __restrict__ labels,
                                                          const int64_t* __restrict__ off, int64_t n_imp,
                                                          double* __restrict__ out, int32_t* __restrict__ tie_flag,
                                                          int32_t* __restrict__ status) {
  const int lane = threadIdx.x & 63;
  const int64_t imp = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (imp >= n_imp) return;  // wave-uniform
  const int64_t a = off[imp];
  const int c = (int)(off[imp + 1] - a);
  if (c > 64 * kRegBlocks) return;  // the LDS kernel
  double* o = out + imp * 4;
  switch (c <= 0 ? 1 : (c + 63) / 64) {
    case 1: metrics_reg<1>(ranks + a, labels + a, c, lane, o, tie_flag + imp, status); break;
    case 2: metrics_reg<2>(ranks + a, labels + a, c, lane, o, tie_flag + imp, status); break;
    case 3: metrics_reg<3>(ranks + a, labels + a, c, lane, o, tie_flag + imp, status); break;
    case 4: metrics_reg<4>(ranks + a, labels + a, c, lane, o, tie_flag + imp, status); break;
    default: metrics_reg<5>(ranks + a, labels + a, c, lane, o, tie_flag + imp, status); break;
  }
}

// Impressions of more than 5 x 64 candidates: a histogram of the dense ranks in
// LDS (one wave per impression; waves of smaller impressions return at once).
__global__ __launch_bounds__(256) void metrics_kernel(const int32_t* __restrict__ ranks, const float* __restrict__ labels,
                                                      const int64_t* __restrict__ off, int64_t n_imp,
                                                      double* __restrict__ out, int32_t* __restrict__ tie_flag,
                                                      int32_t* __restrict__ status) {
  __shared__ int cnt[4][kMaxCand + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // grid-stride over impressions (wave-private LDS slots, no workgroup barrier)
  for (int64_t imp = (int64_t)blockIdx.x * 4 + w; imp < n_imp; imp += (int64_t)gridDim.x * 4) {
  const int64_t a = off[imp];
  const int c = (int)(off[imp + 1] - a);
  if (c <= 64 * kRegBlocks) continue;  // metrics_reg_kernel
  double* o = out + imp * 4;
  if (c > kMaxCand) {
    if (lane == 0) { atomicOr(status, 1); o[0] = o[1] = o[2] = o[3] = __builtin_nan(""); tie_flag[imp] = 1; }
    continue;
  }
  int* h = cnt[w];
  for (int v = lane; v <= c; v += 64) h[v] = 0;
  __builtin_amdgcn_wave_barrier();
  // histogram of dense ranks (1..c), label sums, binary-label check
  int P = 0, maxr = 0, bad = 0;
  for (int i = lane; i < c; i += 64) {
    const int r = ranks[a + i];
    const float y = labels[a + i];
    if (r < 1 || r > c) bad = 1;
    else atomicAdd(&h[r], 1);
    if (y != 0.f && y != 1.f) bad = 1;
    P += y != 0.f;
    maxr = max(maxr, r);
  }
  __builtin_amdgcn_wave_barrier();
  for (int m = 32; m >= 1; m >>= 1) {
    P += __shfl_xor(P, m, 64);
    maxr = max(maxr, __shfl_xor(maxr, m, 64));
    bad |= __shfl_xor(bad, m, 64);
  }
  if (bad) {
    if (lane == 0) { atomicOr(status, 2); o[0] = o[1] = o[2] = o[3] = __builtin_nan(""); tie_flag[imp] = 1; }
    continue;
  }
  // h[v] <- number of candidates with dense rank > v (lower score): suffix sum
  // over 1..c, ceil(c / 64) consecutive bins per lane, then a wave scan of the
  // lane totals.
  const int per = (c + 63) / 64;
  const int lo = 1 + lane * per, hi = min(c, lo + per - 1);
  int tot = 0;
  for (int v = lo; v <= hi; ++v) tot += h[v];
  int suf = tot;  // inclusive suffix over lanes >= lane
  for (int m = 1; m < 64; m <<= 1) {
    const int t = __shfl_down(suf, m, 64);
    if (lane + m < 64) suf += t;
  }
  int run = suf - tot;  // candidates in bins above this lane's range
  // rewrite bins high -> low: bits 12+ = candidates ranked strictly below the
  // bin (run), bits 0-11 = the bin's own count (k)
  for (int v = hi; v >= lo; --v) {
    const int k = h[v];
    h[v] = (run << 12) | k;  // run, k <= kMaxCand < 4096
    run += k;
  }
  __builtin_amdgcn_wave_barrier();
  const int N = c - P;
  double S = 0.0, rr = 0.0, d5 = 0.0, d10 = 0.0;
  for (int i = lane; i < c; i += 64) {
    if (labels[a + i] == 0.f) continue;
    const int r = ranks[a + i];
    const int e = h[r];
    const int below = e >> 12, k = e & 4095;
    S += (double)below + 0.5 * (double)(k + 1);
    rr += 1.0 / (double)r;
    if (r <= 10) {
      d10 += kDisc[r - 1];
      if (r <= 5) d5 += kDisc[r - 1];
    }
  }
  for (int m = 32; m >= 1; m >>= 1) {
    S += __shfl_xor(S, m, 64);
    rr += __shfl_xor(rr, m, 64);
    d5 += __shfl_xor(d5, m, 64);
    d10 += __shfl_xor(d10, m, 64);
  }
  if (lane == 0) {
    write_metrics(o, P, N, S, rr, d5, d10);
    tie_flag[imp] = maxr < c ? 1 : 0;
  }
  __builtin_amdgcn_wave_barrier();  // this wave's histogram reads are done before the next impression
  }  // impression loop
}

}  // namespace nr

extern "C" int nr_impression_metrics(const int32_t* ranks, const float* labels, const int64_t* cand_off, int64_t n_imp,
                                     double* metrics, int32_t* tie_flag, int32_t* status, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(n_imp >= 0, "nr_impression_metrics: n_imp < 0");
  if (n_imp == 0) return NR_OK;
  NR_CHECK_ARG(ranks && labels && cand_off && metrics && tie_flag && status, "nr_impression_metrics: null pointer");
  NR_CHECK_DEVICE("nr_impression_metrics", ranks, labels, cand_off, metrics, tie_flag, status);
  const dim3 grid((unsigned)((n_imp + 3) / 4));
  hipLaunchKernelGGL(nr::metrics_reg_kernel, grid, dim3(256), 0, (hipStream_t)stream, ranks, labels, cand_off, n_imp,
                     metrics, tie_flag, status);
  hipLaunchKernelGGL(nr::metrics_kernel, dim3(grid.x < 1024 ? grid.x : 1024), dim3(256), 0, (hipStream_t)stream,
                     ranks, labels, cand_off, n_imp, metrics, tie_flag, status);
  NR_CHECK_LAUNCH("nr_impression_metrics");
  return NR_OK;
}
