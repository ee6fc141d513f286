// Title encoder (XLM-R-large architecture, e5-large-instruct) on gfx950.
//
// Replaces the transformers XLMRobertaModel forward that get_embed_from_model /
// get_text_embed_eval run per padded batch (modeling_utils.py:282-323) and the
// average_pool + F.normalize that follow (modeling_utils.py:55-59,
// data_model_helper.py:65-78).  Post-LN BERT layer:
//   x   = LN_emb(word[id] + pos[p] + type[0])
//   per layer:  qkv = x Wqkvᵀ + b ; ctx = softmax(q kᵀ / 8) v  (16 heads x 64)
//               x = LN1(ctx Woᵀ + bo + x) ; x = LN2(gelu(x W1ᵀ + b1) W2ᵀ + b2 + x)
// Sequences are packed varlen (no padding): cu_seqlens offsets, attention
// stays inside a sequence, which equals the reference's key-padding mask
// ((1 - m) * finfo.min -> exp() == 0).  GEMMs reuse gemm.hip; this file holds
// the embedding+LN kernel and the MFMA attention kernel.
#include "nr_common.h"

namespace nr {

// ------------------------------------------------------------------ embeddings
template <typename TO>
__global__ __launch_bounds__(256) void embed_ln_kernel(int64_t T, const int32_t* __restrict__ ids,
                                                       const int32_t* __restrict__ pos,
                                                       const TO* __restrict__ word, const TO* __restrict__ pemb,
                                                       const TO* __restrict__ temb, const float* __restrict__ g,
                                                       const float* __restrict__ b, float eps,
                                                       TO* __restrict__ out) {
  constexpr int D = 1024, NJ = D / 256;
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const TO* wr = word + (int64_t)ids[t] * D;
  const TO* pr = pemb + (int64_t)pos[t] * D;
  float v[NJ][4];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = j * 256 + lane * 4 + q;
      // reference order: (word + type) + position  (XLMRobertaEmbeddings.forward)
      v[j][q] = ((float)wr[e] + (float)temb[e]) + (float)pr[e];
      s += v[j][q];
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float qv = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float d = v[j][q] - mean;
      qv = fmaf(d, d, qv);
    }
  const float rstd = 1.0f / sqrtf(wave_sum(qv) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = j * 256 + lane * 4 + q;
      out[t * D + e] = (TO)((v[j][q] - mean) * rstd * g[e] + b[e]);
    }
}

// ------------------------------------------------------------------ attention
// One wave per (query block of 32 rows, head); 4 heads per 256-thread block.
// Sᵀ = K·Qᵀ for a 32-key block lands with the query on the lane and the key
// in the 16 accumulator registers (+4 per lane half), so the per-query online
// softmax reduces over registers and one lane^32 exchange, and the same
// registers are directly the A operand of O = P·V (sum over the key = the
// accumulator's row index, no LDS round trip).  V fragments come straight from
// L2 in B-operand order (32 consecutive d of one key row per half-wave).  The
// output tile (query rows in registers, d on the lane) stores 128-B row
// segments.  Scale 1/8 is folded into Q exactly (power of two).
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Bijection of [0, n): dispatch slot s (XCD s % 8) -> a contiguous run of ids per XCD.
__device__ __forceinline__ int xcd_contiguous(int s, int n) {
  const int xcd = s & 7, q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (s >> 3);
}

template <typename T>
__device__ __forceinline__ void attention_body(const T* __restrict__ qkv, const int32_t* __restrict__ cu,
                                               const int32_t* __restrict__ qoff, int32_t n_seq,
                                               T* __restrict__ ctx) {
  constexpr int D = 1024, LD = 3 * D, HD = 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // 1-D grid of 4 x (an upper bound of) the query blocks; nr_encoder_forward
  // launches the bound, the exact count lives on the device.  Dispatch slots
  // past the 4 x total work items exit (block-uniform); the others are remapped
  // XCD-contiguous (slot s runs on XCD s % 8), so the query blocks of one
  // sequence, which re-read its K/V rows, share one XCD's L2.
  const int total = qoff[n_seq];
  const int slot = blockIdx.x;
  if (slot >= 4 * total) return;
  const int item = xcd_contiguous(slot, 4 * total);
  const int h = (item / total) * 4 + wave;  // head
  const int qb_global = item % total;       // global query-block index
  // 64-ary search for the sequence owning this query block (qoff: prefix of
  // ceil(L/32), qoff[n_seq] = total): each step probes 64 boundaries with one
  // wave load + ballot, so 20k sequences take 3 dependent loads, not 15.
  int lo = 0, hi = n_seq;  // invariant: qoff[lo] <= qb_global < qoff[hi]
  while (hi - lo > 1) {
    const int step = (hi - lo + 63) >> 6;
    const int idx = lo + lane * step;
    const bool le = idx < hi && qoff[idx] <= qb_global;
    const unsigned long long b = __ballot(le);
    const int last = 63 - __builtin_clzll(b);  // lane 0 (idx = lo) is always set
    lo = lo + last * step;
    hi = min(hi, lo + step);
  }
  const int seq = lo;
  const int64_t s0 = cu[seq];
  const int L = cu[seq + 1] - cu[seq];
  const int q0 = (qb_global - qoff[seq]) * 32;
  const int li = lane & 31, lh = lane >> 5;

  // Q fragment (B operand of Sᵀ = K Qᵀ): lane (q = li, half lh)
  const int qrow = min(q0 + li, L - 1);
  const T* qp = qkv + (s0 + qrow) * LD + h * HD;
  const int64_t vcol = 2 * D + h * HD;

  f32x16 o[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;  // per query (lane column li)

  if constexpr (sizeof(T) == 4) {
    float qf[32];  // d = 32*lh + s
#pragma unroll
    for (int s4 = 0; s4 < 8; ++s4) {
      const float4 f = *reinterpret_cast<const float4*>(qp + 32 * lh + 4 * s4);
      qf[4 * s4] = f.x * 0.125f; qf[4 * s4 + 1] = f.y * 0.125f; qf[4 * s4 + 2] = f.z * 0.125f; qf[4 * s4 + 3] = f.w * 0.125f;
    }
    for (int kb = 0; kb < L; kb += 32) {
      const int krow = min(kb + li, L - 1);
      const float* kp = reinterpret_cast<const float*>(qkv) + (s0 + krow) * LD + D + h * HD + 32 * lh;
      f32x16 sacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
#pragma unroll
      for (int s4 = 0; s4 < 8; ++s4) {
        const float4 kf = *reinterpret_cast<const float4*>(kp + 4 * s4);
        sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.x, qf[4 * s4 + 0], sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.y, qf[4 * s4 + 1], sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.z, qf[4 * s4 + 2], sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.w, qf[4 * s4 + 3], sacc, 0, 0, 0);
      }
      // mask keys past L, online softmax per query column
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (kb + acc_row(r, lh) >= L) sacc[r] = -INFINITY;
        mx = fmaxf(mx, sacc[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float alpha = expf(m_run - m_new);
      float ps = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) { sacc[r] = expf(sacc[r] - m_new); ps += sacc[r]; }
      ps += __shfl_xor(ps, 32, 64);
      l_run = l_run * alpha + ps;
      m_run = m_new;
      // rescale O (query rows live in registers: q = acc_row(r, lh)) by alpha[q]
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float a = __shfl(alpha, acc_row(r, lh), 64);
        o[0][r] *= a;
        o[1][r] *= a;
      }
      // O += P V : step r uses keys acc_row(r, 0/1); A = P regs, B = V rows
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kr = min(kb + acc_row(r, lh), L - 1);
        const float* vp = reinterpret_cast<const float*>(qkv) + (s0 + kr) * LD + vcol + li;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) o[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(sacc[r], vp[32 * dt], o[dt], 0, 0, 0);
      }
    }
  } else {
    // Per-wave LDS: the 32-key V tile (rows of 192 B: conflict-free for the
    // transposed reads below, MI355X guide T10 bank rule), reused for the O tile.
    __shared__ __attribute__((aligned(16))) unsigned char lds_all[4][32 * 192];
    unsigned char* lds = lds_all[wave];
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    bf16x8 qf[4];  // step s: d = 16s + 8lh + j
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 raw = *reinterpret_cast<const bf16x8*>(qp + 16 * s + 8 * lh);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[s][j] = (__bf16)((float)raw[j] * 0.125f);
    }
    // transposed-read lane roles (T10): group g = lane >> 4 reads a 4-key x 16-d
    // block; lane 4q + p of the group addresses key row q, d columns 4p..4p+3
    const int tg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
    const int tr_off = tq * 192 + 2 * (16 * (tg & 1) + 4 * tp);
    for (int kb = 0; kb < L; kb += 32) {
      const int krow = min(kb + li, L - 1);
      const T* kp = qkv + (s0 + krow) * LD + D + h * HD;
      bf16x8 kf[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) kf[s] = *reinterpret_cast<const bf16x8*>(kp + 16 * s + 8 * lh);
      // V tile rows kb + 8i + lane/8 (clamped: those keys get P = 0), 16-B chunk lane % 8
      uint4 vt[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int vr = min(kb + 8 * i + (lane >> 3), L - 1);
        vt[i] = *reinterpret_cast<const uint4*>(qkv + (s0 + vr) * LD + vcol + 8 * (lane & 7));
      }
      if (kb > 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // last block's V reads are done
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<uint4*>(lds + (8 * i + (lane >> 3)) * 192 + 16 * (lane & 7)) = vt[i];
      f32x16 sacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[s], qf[s], sacc, 0, 0, 0);
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (kb + acc_row(r, lh) >= L) sacc[r] = -INFINITY;
        mx = fmaxf(mx, sacc[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float alpha = expf(m_run - m_new);
      float ps = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) { sacc[r] = expf(sacc[r] - m_new); ps += sacc[r]; }
      ps += __shfl_xor(ps, 32, 64);
      l_run = l_run * alpha + ps;
      m_run = m_new;
      if (kb > 0) {  // wave-uniform; O is still zero after the first key block
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float a = __shfl(alpha, acc_row(r, lh), 64);
          o[0][r] *= a;
          o[1][r] *= a;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's V tile is in LDS
      // O += P V: A = P from the accumulator (k-step s: registers 8s..8s+7,
      // element j <-> key 16s + 8(j>>2) + 4lh + (j&3)); B = V read transposed,
      // two 4-key blocks per fragment (j = 0..3 and 4..7), lane column d = 32dt + li
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pa;
#pragma unroll
        for (int j = 0; j < 8; ++j) pa[j] = (__bf16)sacc[8 * s + j];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const unsigned char* b0 = lds + (16 * s + 4 * lh) * 192 + 64 * dt + tr_off;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(b0));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(b0 + 8 * 192));
          // whole-vector bit cast (per-element bf16 inserts miscompile to a
          // duplicated dword here: hipcc 7.2, seen in the ISA)
          const bf16x8 vb = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, vb, o[dt], 0, 0, 0);
        }
      }
    }
    // O tile -> LDS (rows q, 144-B pitch) -> 16-B row stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = acc_row(r, lh);
      const float inv = 1.0f / __shfl(l_run, q, 64);
      __bf16* orow = reinterpret_cast<__bf16*>(lds + q * 144);
      orow[li] = (__bf16)(o[0][r] * inv);
      orow[32 + li] = (__bf16)(o[1][r] * inv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = 8 * i + (lane >> 3);
      const uint4 v = *reinterpret_cast<const uint4*>(lds + q * 144 + 16 * (lane & 7));
      if (q0 + q < L) *reinterpret_cast<uint4*>(ctx + (s0 + q0 + q) * D + h * HD + 8 * (lane & 7)) = v;
    }
    return;
  }
  // normalise by l[q] and store rows q0 + acc_row(r, lh), d = 32 dt + li
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int q = acc_row(r, lh);
    const float inv = 1.0f / __shfl(l_run, q, 64);
    if (q0 + q < L) {
      T* op = ctx + (s0 + q0 + q) * D + h * HD + li;
      op[0] = (T)(o[0][r] * inv);
      op[32] = (T)(o[1][r] * inv);
    }
  }
}

// f32 (config 2) keeps the compiler's register budget.  bf16: one wave per
// (query block, head) is a single dependent load -> MFMA -> softmax -> store
// chain for the short titles, so occupancy hides the latency; the V tile goes
// to LDS right after its load (its registers die before the S MFMA) and the
// kernel is held to 128 VGPRs = 4 waves per SIMD with no spill (3 at the
// compiler's choice of 146): 0.84x the time at 1 M tokens of length 20 / 66 /
// 200, bit-identical (tools/attn_ab.py, profiles/round3/s6/attn_ab_occupancy.jsonl).
__global__ __launch_bounds__(256) void attention_kernel_f32(const float* __restrict__ qkv,
                                                            const int32_t* __restrict__ cu,
                                                            const int32_t* __restrict__ qoff, int32_t n_seq,
                                                            float* __restrict__ ctx) {
  attention_body<float>(qkv, cu, qoff, n_seq, ctx);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void attention_kernel_bf16(
    const __bf16* __restrict__ qkv, const int32_t* __restrict__ cu, const int32_t* __restrict__ qoff, int32_t n_seq,
    __bf16* __restrict__ ctx) {
  attention_body<__bf16>(qkv, cu, qoff, n_seq, ctx);
}

// ------------------------------------------------------------ whole forward
constexpr int kPadId = 1;  // XLM-R <pad>; positions start at kPadId + 1

// cu32/cu64 = prefix sums of seq_lens, qoff = prefix sum of ceil(len / 32):
// one 1024-thread workgroup walks the sequences 1024 at a time (wave scans +
// one LDS pass), carrying the running totals.
__global__ __launch_bounds__(1024) void encoder_offsets_kernel(int64_t n_seq, const int32_t* __restrict__ lens,
                                                               int32_t* __restrict__ cu32, int64_t* __restrict__ cu64,
                                                               int32_t* __restrict__ qoff) {
  __shared__ int64_t wtok[16];
  __shared__ int32_t wqb[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int64_t carry_t = 0;
  int32_t carry_q = 0;
  if (tid == 0) {
    cu32[0] = 0;
    cu64[0] = 0;
    qoff[0] = 0;
  }
  for (int64_t base = 0; base < n_seq; base += 1024) {
    const int64_t i = base + tid;
    const int32_t L = i < n_seq ? lens[i] : 0;
    int64_t t = L;
    int32_t q = (L + 31) / 32;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // inclusive wave scans
      const int64_t tt = __shfl_up(t, o, 64);
      const int32_t qq = __shfl_up(q, o, 64);
      if (lane >= o) {
        t += tt;
        q += qq;
      }
    }
    if (lane == 63) {
      wtok[wave] = t;
      wqb[wave] = q;
    }
    __syncthreads();
    int64_t pt = carry_t;
    int32_t pq = carry_q;
    for (int w = 0; w < wave; ++w) {
      pt += wtok[w];
      pq += wqb[w];
    }
    if (i < n_seq) {
      cu64[i + 1] = pt + t;
      cu32[i + 1] = (int32_t)(pt + t);
      qoff[i + 1] = pq + q;
    }
    for (int w = 0; w < 16; ++w) {
      carry_t += wtok[w];
      carry_q += wqb[w];
    }
    __syncthreads();
  }
}

// transformers create_position_ids_from_input_ids per packed sequence:
// pos = pad + cumsum(id != pad) * (id != pad).  One wave per sequence.  Out-of-
// range ids / positions are clamped (so no row outside the tables is read) and
// flagged in *status.
__global__ __launch_bounds__(256) void encoder_positions_kernel(int64_t n_seq, const int32_t* __restrict__ cu,
                                                                int32_t* __restrict__ ids, int32_t* __restrict__ pos,
                                                                int64_t vocab, int64_t n_positions,
                                                                int32_t* __restrict__ status) {
  const int lane = threadIdx.x & 63;
  const int64_t seq = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seq >= n_seq) return;
  const int64_t s0 = cu[seq];
  const int L = cu[seq + 1] - cu[seq];
  int carry = 0, flag = 0;
  for (int b = 0; b < L; b += 64) {
    const int t = b + lane;
    int id = kPadId;
    if (t < L) {
      id = ids[s0 + t];
      if (id < 0 || id >= vocab) {
        flag |= 2;
        id = id < 0 ? 0 : (int)(vocab - 1);
        ids[s0 + t] = id;
      }
    }
    const bool m = t < L && id != kPadId;
    const unsigned long long bal = __ballot(m);
    const int incl = __popcll(bal & ((2ull << lane) - 1));
    int p = m ? kPadId + carry + incl : kPadId;
    if (p >= n_positions) {
      flag |= 1;
      p = (int)(n_positions - 1);
    }
    if (t < L) pos[s0 + t] = p;
    carry += __popcll(bal);
  }
  if (flag && status) atomicOr(status, flag);
}

static int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

struct EncWs {  // workspace carve-up of nr_encoder_forward
  int64_t x, big, ctx, tmp, pos, cu32, qoff, cu64, total;
};
static EncWs enc_ws(int dtype, int64_t T, int64_t n, bool own_x) {
  const int64_t es = dtype == NR_F32 ? 4 : 2;
  EncWs w{};
  int64_t o = 0;
  w.x = o;   o += own_x ? align256(T * 1024 * es) : 0;
  w.big = o; o += align256(T * 4096 * es);  // qkv [T][3072], later the FFN hidden [T][4096]
  w.ctx = o; o += align256(T * 1024 * es);
  w.tmp = o; o += align256(T * 1024 * es);
  w.pos = o; o += align256(T * 4);
  w.cu32 = o; o += align256((n + 1) * 4);
  w.qoff = o; o += align256((n + 1) * 4);
  w.cu64 = o; o += align256((n + 1) * 8);
  w.total = o;
  return w;
}

}  // namespace nr

extern "C" int64_t nr_encoder_workspace_bytes(int dtype, int64_t n_tokens, int64_t n_seq) {
  // sized for hidden == NULL (the library keeps x); a caller-provided hidden needs less
  return nr::enc_ws(dtype, n_tokens, n_seq, true).total;
}

extern "C" int nr_encoder_forward(int dtype, int n_layers, const nr_encoder_layer* layers, const void* word_emb,
                                  int64_t vocab, const void* pos_emb, int64_t n_positions, const void* type_emb,
                                  const float* emb_ln_g, const float* emb_ln_b, float eps, int64_t n_seq,
                                  int64_t n_tokens, const int32_t* seq_lens, const int32_t* ids, int pool,
                                  float* pooled, void* hidden, int32_t* status, void* ws, int64_t ws_bytes,
                                  void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(dtype == NR_F32 || dtype == NR_BF16, "nr_encoder_forward: bad dtype %d", dtype);
  NR_CHECK_ARG(n_layers >= 0 && (n_layers == 0 || layers), "nr_encoder_forward: bad layers");
  NR_CHECK_ARG(pool == NR_POOL_MEAN || pool == NR_POOL_LATENT || pool == NR_POOL_NONE,
               "nr_encoder_forward: bad pool %d", pool);
  NR_CHECK_ARG(n_seq >= 0 && n_tokens >= 0, "nr_encoder_forward: negative sizes");
  if (n_seq == 0) return NR_OK;
  NR_CHECK_ARG(n_tokens <= 0x7fffffff && n_seq <= 0x7fffffff, "nr_encoder_forward: too many tokens / sequences");
  NR_CHECK_ARG(word_emb && pos_emb && type_emb && emb_ln_g && emb_ln_b && seq_lens && ids && ws,
               "nr_encoder_forward: null pointer");
  NR_CHECK_ARG(vocab > 0 && n_positions > nr::kPadId + 1, "nr_encoder_forward: bad vocab / n_positions");
  NR_CHECK_ARG(pool == NR_POOL_NONE || pooled, "nr_encoder_forward: pooled is NULL");
  NR_CHECK_ARG(pool != NR_POOL_NONE || hidden, "nr_encoder_forward: nothing to output");
  for (int l = 0; l < n_layers; ++l) {
    const nr_encoder_layer& L = layers[l];
    NR_CHECK_ARG(L.wqkv && L.bqkv && L.wo && L.bo && L.ln1_g && L.ln1_b && L.w1 && L.b1 && L.w2 && L.b2 &&
                     L.ln2_g && L.ln2_b, "nr_encoder_forward: layer %d has a null pointer", l);
    NR_CHECK_DEVICE("nr_encoder_forward(layer)", L.wqkv, L.bqkv, L.wo, L.bo, L.ln1_g, L.ln1_b, L.w1, L.b1, L.w2,
                    L.b2, L.ln2_g, L.ln2_b);
  }
  NR_CHECK_DEVICE("nr_encoder_forward", word_emb, pos_emb, type_emb, emb_ln_g, emb_ln_b, seq_lens, ids, pooled,
                  hidden, status, ws);
  const nr::EncWs w = nr::enc_ws(dtype, n_tokens, n_seq, hidden == nullptr);
  NR_CHECK_ARG(ws_bytes >= w.total, "nr_encoder_forward: workspace too small (%lld < %lld)", (long long)ws_bytes,
               (long long)w.total);
  NR_CHECK_ARG(((uintptr_t)ws & 255) == 0 && (!hidden || ((uintptr_t)hidden & 15) == 0),
               "nr_encoder_forward: ws must be 256-byte aligned, hidden 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  char* b = (char*)ws;
  void* x = hidden ? hidden : (void*)(b + w.x);
  void* big = b + w.big;
  void* ctx = b + w.ctx;
  void* tmp = b + w.tmp;
  int32_t* pos = (int32_t*)(b + w.pos);
  int32_t* cu32 = (int32_t*)(b + w.cu32);
  int32_t* qoff = (int32_t*)(b + w.qoff);
  int64_t* cu64 = (int64_t*)(b + w.cu64);
  const int64_t T = n_tokens, D = 1024, F = 4096;
  // the ids are clamped in place when out of range: work on a copy in the workspace
  int32_t* ids_ws = (int32_t*)tmp;  // tmp is first written by layer 0's O-projection
  if (hipMemcpyAsync(ids_ws, ids, T * 4, hipMemcpyDeviceToDevice, s) != hipSuccess) {
    nr::set_error("nr_encoder_forward: copy of ids failed");
    return NR_ERR_HIP;
  }
  hipLaunchKernelGGL(nr::encoder_offsets_kernel, dim3(1), dim3(1024), 0, s, n_seq, seq_lens, cu32, cu64, qoff);
  NR_CHECK_LAUNCH("nr_encoder_forward(offsets)");
  hipLaunchKernelGGL(nr::encoder_positions_kernel, dim3((unsigned)((n_seq + 3) / 4)), dim3(256), 0, s, n_seq, cu32,
                     ids_ws, pos, vocab, n_positions, status);
  NR_CHECK_LAUNCH("nr_encoder_forward(positions)");
  int rc;
  if ((rc = nr_embed_ln(dtype, T, ids_ws, pos, word_emb, pos_emb, type_emb, emb_ln_g, emb_ln_b, eps, x, stream)))
    return rc;
  // upper bound of the query-block count (exact count sits in qoff[n_seq] on the device)
  const int64_t qb_bound = (T + 31) / 32 + n_seq;
  for (int l = 0; l < n_layers; ++l) {
    const nr_encoder_layer& L = layers[l];
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_NONE, T, 3 * D, D, x, D, L.wqkv, D, L.bqkv, nullptr, 0, big, 3 * D, s)))
      return rc;
    if ((rc = nr_attention_varlen(dtype, (int32_t)n_seq, qb_bound, big, cu32, qoff, ctx, stream))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_RESADD, T, D, D, ctx, D, L.wo, D, L.bo, x, D, tmp, D, s))) return rc;
    if ((rc = nr::layernorm_dispatch(dtype, dtype, T, D, tmp, D, L.ln1_g, L.ln1_b, eps, x, D, s))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_GELU, T, F, D, x, D, L.w1, D, L.b1, nullptr, 0, big, F, s))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_RESADD, T, D, F, big, F, L.w2, F, L.b2, x, D, tmp, D, s))) return rc;
    if ((rc = nr::layernorm_dispatch(dtype, dtype, T, D, tmp, D, L.ln2_g, L.ln2_b, eps, x, D, s))) return rc;
  }
  if (pool != NR_POOL_NONE)
    if ((rc = nr::pool_rows_dispatch(pool, dtype, x, D, cu64, n_seq, pooled, s))) return rc;
  return NR_OK;
}

extern "C" int nr_embed_ln(int dtype, int64_t n_tokens, const int32_t* ids, const int32_t* pos,
                           const void* word, const void* pos_emb, const void* type_emb, const float* gamma,
                           const float* beta, float eps, void* out, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(dtype == NR_F32 || dtype == NR_BF16, "nr_embed_ln: bad dtype");
  if (n_tokens <= 0) return NR_OK;
  NR_CHECK_ARG(ids && pos && word && pos_emb && type_emb && gamma && beta && out, "nr_embed_ln: null pointer");
  NR_CHECK_DEVICE("nr_embed_ln", ids, pos, word, pos_emb, type_emb, gamma, beta, out);
  const dim3 grid((unsigned)((n_tokens + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == NR_F32)
    hipLaunchKernelGGL(nr::embed_ln_kernel<float>, grid, dim3(256), 0, s, n_tokens, ids, pos, (const float*)word,
                       (const float*)pos_emb, (const float*)type_emb, gamma, beta, eps, (float*)out);
  else
    hipLaunchKernelGGL(nr::embed_ln_kernel<__bf16>, grid, dim3(256), 0, s, n_tokens, ids, pos, (const __bf16*)word,
                       (const __bf16*)pos_emb, (const __bf16*)type_emb, gamma, beta, eps, (__bf16*)out);
  NR_CHECK_LAUNCH("nr_embed_ln");
  return NR_OK;
}

extern "C" int nr_attention_varlen(int dtype, int32_t n_seq, int64_t n_qblocks, const void* qkv,
                                   const int32_t* cu_seqlens, const int32_t* qblock_off, void* ctx, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(dtype == NR_F32 || dtype == NR_BF16, "nr_attention_varlen: bad dtype");
  if (n_seq <= 0 || n_qblocks <= 0) return NR_OK;
  NR_CHECK_ARG(qkv && cu_seqlens && qblock_off && ctx, "nr_attention_varlen: null pointer");
  NR_CHECK_DEVICE("nr_attention_varlen", qkv, cu_seqlens, qblock_off, ctx);
  // 4 workgroups x 4 waves = 16 heads per query block; 256 x grid fits in 32 bits
  NR_CHECK_ARG(n_qblocks <= (1 << 22) - 1, "nr_attention_varlen: too many query blocks");
  const dim3 grid((unsigned)(4 * n_qblocks));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == NR_F32)
    hipLaunchKernelGGL(nr::attention_kernel_f32, grid, dim3(256), 0, s, (const float*)qkv, cu_seqlens,
                       qblock_off, n_seq, (float*)ctx);
  else
    hipLaunchKernelGGL(nr::attention_kernel_bf16, grid, dim3(256), 0, s, (const __bf16*)qkv, cu_seqlens,
                       qblock_off, n_seq, (__bf16*)ctx);
  NR_CHECK_LAUNCH("nr_attention_varlen");
  return NR_OK;
}
