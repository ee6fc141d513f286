// C-ABI plumbing (errors, init, version) and the per-news pooler transforms,
// which chain the GEMM / row kernels over row chunks with a caller workspace.
#include "nr_common.h"

#include <atomic>
#include <mutex>
#include <string.h>

namespace nr {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
void clear_error() { g_err[0] = 0; }

// ---------------------------------------------------------------- residency
// Every pointer a public entry hands to a kernel must be device (or managed)
// memory: a host pointer reaching an async launch faults the GPU instead of
// failing the call.  hipPointerGetAttributes costs ~µs, so
// verified allocations are remembered as [base, base + size) ranges in a small
// per-thread table (torch's caching allocator hands out sub-ranges of a few
// large segments, so the table hits on almost every call).  A freed range may
// later hold other memory, so the tables are dropped whenever the process-wide
// generation moves (nr_residency_flush, called by the Python side after it
// returns cached segments to the driver).
namespace {
struct Range {
  uintptr_t lo, hi;
};
constexpr int kRanges = 64;
thread_local Range t_ranges[kRanges];
thread_local int t_next = 0;
thread_local uint64_t t_gen = 0;
std::atomic<uint64_t> g_res_gen{0};
}  // namespace

void residency_flush() { g_res_gen.fetch_add(1, std::memory_order_release); }

bool device_accessible(const void* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint64_t gen = g_res_gen.load(std::memory_order_acquire);
  if (gen != t_gen) {
    for (int i = 0; i < kRanges; ++i) t_ranges[i] = Range{0, 0};
    t_next = 0;
    t_gen = gen;
  }
  for (int i = 0; i < kRanges; ++i)
    if (a >= t_ranges[i].lo && a < t_ranges[i].hi) return true;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // unregistered host memory: do not leave the error for torch's launch checks
    return false;
  }
  if (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeManaged) return false;
  void* base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (void*)p) == hipSuccess && size) {
    t_ranges[t_next] = Range{(uintptr_t)base, (uintptr_t)base + size};
    t_next = (t_next + 1) % kRanges;
  } else {
    (void)hipGetLastError();
  }
  return true;
}

int check_device_ptrs(const char* fn, const char* names, std::initializer_list<const void*> ptrs) {
  int i = 0;
  for (const void* p : ptrs) {
    if (p && !device_accessible(p)) {
      // the i-th name of the stringified argument list
      const char* s = names;
      for (int k = 0; k < i && s; ++k) {
        s = strchr(s, ',');
        if (s) ++s;
      }
      while (s && *s == ' ') ++s;
      const char* e = s ? strchr(s, ',') : nullptr;
      const int len = s ? (e ? (int)(e - s) : (int)strlen(s)) : 1;
      set_error("%s: `%.*s` (%p) is not device memory (host pointer? pass tensors on the GPU)", fn, len,
                s ? s : "?", p);
      return NR_ERR_INVALID;
    }
    ++i;
  }
  return NR_OK;
}

static int esize(int dtype) { return dtype == NR_F32 ? 4 : 2; }

// Rows per chunk of the transforms: one chunk covers every MIND split's news
// table (<= 161k), so each GEMM runs once over all rows; the workspace stays
// bounded (f32 FinalAttention: 2 x 262144 x 4096 x 4 B = 8 GiB of 288 GB).
constexpr int64_t kChunk = 262144;

}  // namespace nr

extern "C" int nr_version(void) { return 100; }

// Hash of the sources this library was compiled from (_lib.source_hash over
// csrc/*.hip + nr_common.h + include/newsrec.h, passed by the build as
// -DNR_BUILD_HASH).  The tag is kept in the binary so the build can read it
// without loading the library; _lib.load() refuses a mismatching library.
#ifndef NR_BUILD_HASH
#define NR_BUILD_HASH "unknown"
#endif
static const char kBuildTag[] __attribute__((used)) = "nr-build-hash:" NR_BUILD_HASH;

extern "C" const char* nr_build_hash(void) { return kBuildTag + 14; }

extern "C" const char* nr_last_error(void) { return nr::g_err; }

extern "C" int nr_residency_flush(void) {
  nr::residency_flush();
  return NR_OK;
}

extern "C" int nr_is_device_pointer(const void* p) { return p && nr::device_accessible(p) ? 1 : 0; }

extern "C" int nr_init(int device) {
  nr::clear_error();
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    nr::set_error("nr_init: hipSetDevice(%d): %s", device, hipGetErrorString(e));
    return NR_ERR_HIP;
  }
  return NR_OK;
}

// ---------------------------------------------------------------- FinalAttention
extern "C" int64_t nr_final_attn_workspace_bytes(int dtype, int64_t n) {
  const int64_t m = n < nr::kChunk ? n : nr::kChunk;
  return 2 * m * 4096 * (int64_t)nr::esize(dtype);
}

// modeling_utils.py:218-224 on unique news rows (dropout inactive in eval):
//   X1 = relu(E W1ᵀ + b1); X2 = relu(X1 W2ᵀ + b2); x = X2 W3ᵀ + b3;
//   Y = relu(x W4ᵀ + b4); p = exp(Y W5ᵀ)  -> table[n][2][1024] = (x, p)
extern "C" int nr_final_attn_transform(int dtype, int64_t n, const void* emb, int64_t emb_ld,
                                       const void* W1, const float* b1, const void* W2,
                                       const float* b2, const void* W3, const float* b3,
                                       const void* W4, const float* b4, const void* W5,
                                       void* table, void* ws, int64_t ws_bytes, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(dtype == NR_F32 || dtype == NR_BF16, "nr_final_attn_transform: bad dtype");
  NR_CHECK_ARG(n >= 0, "nr_final_attn_transform: n < 0");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(emb && W1 && b1 && W2 && b2 && W3 && b3 && W4 && b4 && W5 && table && ws,
               "nr_final_attn_transform: null pointer");
  NR_CHECK_DEVICE("nr_final_attn_transform", emb, W1, b1, W2, b2, W3, b3, W4, b4, W5, table, ws);
  NR_CHECK_ARG(ws_bytes >= nr_final_attn_workspace_bytes(dtype, n),
               "nr_final_attn_transform: workspace too small (%lld < %lld)", (long long)ws_bytes,
               (long long)nr_final_attn_workspace_bytes(dtype, n));
  const int es = nr::esize(dtype);
  const int64_t D = 1024, H = 4096;
  hipStream_t s = (hipStream_t)stream;
  char* w0 = (char*)ws;
  char* w1 = w0 + (int64_t)(n < nr::kChunk ? n : nr::kChunk) * H * es;
  for (int64_t r0 = 0; r0 < n; r0 += nr::kChunk) {
    const int64_t m = (n - r0) < nr::kChunk ? (n - r0) : nr::kChunk;
    const char* e = (const char*)emb + r0 * emb_ld * es;
    char* x = (char*)table + r0 * 2 * D * es;
    char* p = x + D * es;
    int rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_RELU, m, H, D, e, emb_ld, W1, D, b1, nullptr, 0, w0, H, s))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_RELU, m, H, H, w0, H, W2, H, b2, nullptr, 0, w1, H, s))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_NONE, m, D, H, w1, H, W3, H, b3, nullptr, 0, x, 2 * D, s))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_RELU, m, H, D, x, 2 * D, W4, D, b4, nullptr, 0, w0, H, s))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_EXP, m, D, H, w0, H, W5, H, nullptr, nullptr, 0, p, 2 * D, s))) return rc;
  }
  return NR_OK;
}

// ---------------------------------------------------------------- Latent
extern "C" int64_t nr_latent_workspace_bytes(int dtype, int64_t n) {
  const int64_t m = n < nr::kChunk ? n : nr::kChunk;
  const int64_t es = nr::esize(dtype);
  // y [m,1024] dtype | s [m,512] f32 | p [m,512] dtype | f [m,4096] dtype
  return m * (1024 * es + 512 * 4 + 512 * es + 4096 * es);
}

// latent_attention.py:157-163 with the 64 latents' K/V folded into A and Bt:
//   y = LN_q(e); P = softmax64(y Aᵀ) (fused epilogue); h1 = e + P Btᵀ;
//   h = h1 + GEGLU(LN_f(h1) W1iᵀ + b1i) W2ᵀ + b2     -> table[n][1024]
extern "C" int nr_latent_transform(int dtype, int64_t n, const void* emb, int64_t emb_ld,
                                   const float* lnq_g, const float* lnq_b, const void* A,
                                   const void* Bt, const float* lnf_g, const float* lnf_b,
                                   const void* W1i, const float* b1i, const void* W2,
                                   const float* b2, void* table, void* ws, int64_t ws_bytes,
                                   void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(dtype == NR_F32 || dtype == NR_BF16, "nr_latent_transform: bad dtype");
  NR_CHECK_ARG(n >= 0, "nr_latent_transform: n < 0");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(emb && A && Bt && W1i && b1i && W2 && b2 && table && ws,
               "nr_latent_transform: null pointer");
  NR_CHECK_DEVICE("nr_latent_transform", emb, lnq_g, lnq_b, A, Bt, lnf_g, lnf_b, W1i, b1i, W2, b2, table, ws);
  NR_CHECK_ARG(ws_bytes >= nr_latent_workspace_bytes(dtype, n),
               "nr_latent_transform: workspace too small");
  const int es = nr::esize(dtype);
  const int64_t D = 1024, S = 512, F = 4096;
  const int64_t mc = n < nr::kChunk ? n : nr::kChunk;
  hipStream_t st = (hipStream_t)stream;
  char* wy = (char*)ws;
  char* wsc = wy + mc * D * es;
  char* wp = wsc + mc * S * 4;  // (wsc: f32 scores of the unfused path, kept for the ABI's workspace size)
  char* wf = wp + mc * S * es;
  for (int64_t r0 = 0; r0 < n; r0 += nr::kChunk) {
    const int64_t m = (n - r0) < nr::kChunk ? (n - r0) : nr::kChunk;
    const char* e = (const char*)emb + r0 * emb_ld * es;
    char* h = (char*)table + r0 * D * es;
    int rc;
    if ((rc = nr::layernorm_dispatch(dtype, dtype, m, D, e, emb_ld, lnq_g, lnq_b, 1e-5f, wy, D, st))) return rc;
    // scores + the per-head 64-latent softmax fused in the GEMM epilogue
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_SOFTMAX64, m, S, D, wy, D, A, D, nullptr, nullptr, 0, wp, S, st))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_RESADD, m, D, S, wp, S, Bt, S, nullptr, e, emb_ld, h, D, st))) return rc;
    if ((rc = nr::layernorm_dispatch(dtype, dtype, m, D, h, D, lnf_g, lnf_b, 1e-5f, wy, D, st))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_GEGLU, m, 2 * F, D, wy, D, W1i, D, b1i, nullptr, 0, wf, F, st))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_RESADD, m, D, F, wf, F, W2, F, b2, h, D, h, D, st))) return rc;
  }
  return NR_OK;
}

// bf16: both LayerNorms applied inside the GEMM that consumes them
// (gemm_lnfold_dispatch); only per-row (mean, rstd) pairs are written.
//   sq = stats(e); P = softmax64(LN_q(e) Aᵀ) via (e, Aq, ucq, sq); h1 = e + P Btᵀ
//   sf = stats(h1); f = GEGLU(LN_f(h1) W1iᵀ + b1i) via (h1, W1f, ucf, sf); h = h1 + f W2ᵀ + b2
extern "C" int nr_latent_transform_lnfold(int dtype, int64_t n, const void* emb, int64_t emb_ld, const void* Aq,
                                          const float* ucq, const void* Bt, const void* W1f, const float* ucf,
                                          const void* W2, const float* b2, void* table, void* ws, int64_t ws_bytes,
                                          void* stream) {
  nr::clear_error();
  if (dtype != NR_BF16) {
    nr::set_error("nr_latent_transform_lnfold: bf16 only (f32 uses nr_latent_transform)");
    return NR_ERR_UNSUPPORTED;
  }
  NR_CHECK_ARG(n >= 0, "nr_latent_transform_lnfold: n < 0");
  if (n == 0) return NR_OK;
  NR_CHECK_ARG(emb && Aq && ucq && Bt && W1f && ucf && W2 && b2 && table && ws,
               "nr_latent_transform_lnfold: null pointer");
  NR_CHECK_DEVICE("nr_latent_transform_lnfold", emb, Aq, ucq, Bt, W1f, ucf, W2, b2, table, ws);
  NR_CHECK_ARG(ws_bytes >= nr_latent_workspace_bytes(dtype, n), "nr_latent_transform_lnfold: workspace too small");
  NR_CHECK_ARG(((uintptr_t)ws & 15) == 0, "nr_latent_transform_lnfold: workspace must be 16-byte aligned");
  const int es = 2;
  const int64_t D = 1024, S = 512, F = 4096;
  const int64_t mc = n < nr::kChunk ? n : nr::kChunk;
  hipStream_t st = (hipStream_t)stream;
  // workspace: [stats_q | stats_f] in the unfused path's LN-output region
  float* sq = (float*)ws;
  float* sf = sq + 2 * mc;
  char* wp = (char*)ws + mc * (D * es + S * 4);
  char* wf = wp + mc * S * es;
  for (int64_t r0 = 0; r0 < n; r0 += nr::kChunk) {
    const int64_t m = (n - r0) < nr::kChunk ? (n - r0) : nr::kChunk;
    const char* e = (const char*)emb + r0 * emb_ld * es;
    char* h = (char*)table + r0 * D * es;
    int rc;
    if ((rc = nr::row_stats_dispatch(dtype, m, D, e, emb_ld, 1e-5f, sq, st))) return rc;
    if ((rc = nr::gemm_lnfold_dispatch(NR_EPI_SOFTMAX64, m, S, D, e, emb_ld, Aq, D, sq, ucq, wp, S, st))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_RESADD, m, D, S, wp, S, Bt, S, nullptr, e, emb_ld, h, D, st))) return rc;
    if ((rc = nr::row_stats_dispatch(dtype, m, D, h, D, 1e-5f, sf, st))) return rc;
    if ((rc = nr::gemm_lnfold_dispatch(NR_EPI_GEGLU, m, 2 * F, D, h, D, W1f, D, sf, ucf, wf, F, st))) return rc;
    if ((rc = nr::gemm_dispatch(dtype, dtype, NR_EPI_RESADD, m, D, F, wf, F, W2, F, b2, h, D, h, D, st))) return rc;
  }
  return NR_OK;
}
