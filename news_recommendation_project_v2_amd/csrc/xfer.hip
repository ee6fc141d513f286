// Host <-> device transfers of the drop-in API: the CSR index
// arrays and the news table go up, the scores and ranks come down.  The
// reference moves them with torch's pageable copies (`.to(DEVICE)`,
// `.cpu()`; data_model_helper.py:112-131, 199-230, 416-443), which HIP stages
// through its own small pinned buffer one piece at a time: 14 GB/s up and
// 6.3 GB/s down on the MI355X box (bench `pcie_ms`, round 5).
//
// Here a transfer runs through a ring of pinned chunks, pipelined: worker
// threads copy chunk i between the caller's pageable memory and pinned chunk
// i % kRing while the DMA engine moves chunk i - 1, so the leg runs at the
// slower of the PCIe DMA rate and the threads' memcpy rate instead of at the
// sum of their times.  Host code only (no kernel): the DMAs are
// hipMemcpyAsync on the caller's stream, events recycle the chunks.
//
//   nr_copy_h2d(dst_dev, src_host, bytes, stream): returns once every byte of
//     src has been read (the caller may reuse it); the data lands in stream order.
//   nr_copy_d2h(dst_host, src_dev, bytes, stream): returns with dst complete
//     (in stream order after the work queued before it).
// Calls are serialised on one process-wide ring (a mutex); the ring (2 x kRing
// x kChunk pinned bytes) is allocated on first use.
#include "nr_common.h"

#include <string.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

namespace nr {
namespace {

constexpr int kRing = 4;
constexpr int64_t kChunk = 8ll << 20;   // 8 MiB per chunk
constexpr int64_t kDirect = 1ll << 20;  // below this: one pinned bounce, no threads

struct Ring {
  char* buf[kRing] = {};
  hipEvent_t ev[kRing] = {};
  int device = -1;
  bool ok = false;
};

std::mutex g_mu;
Ring g_ring[2];  // [0] up, [1] down

int ring_for(int dir, Ring** out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    set_error("nr_copy: hipGetDevice failed");
    return NR_ERR_HIP;
  }
  Ring& r = g_ring[dir];
  if (r.ok && r.device != dev) {  // the ring's events belong to another device: rebuild
    for (int i = 0; i < kRing; ++i) {
      (void)hipEventDestroy(r.ev[i]);
      (void)hipHostFree(r.buf[i]);
    }
    r = Ring{};
  }
  if (!r.ok) {
    for (int i = 0; i < kRing; ++i) {
      if (hipHostMalloc((void**)&r.buf[i], kChunk, hipHostMallocDefault) != hipSuccess ||
          hipEventCreateWithFlags(&r.ev[i], hipEventDisableTiming) != hipSuccess) {
        set_error("nr_copy: pinned staging allocation failed (%d x %lld bytes)", kRing, (long long)kChunk);
        return NR_ERR_HIP;
      }
    }
    r.device = dev;
    r.ok = true;
  }
  *out = &r;
  return NR_OK;
}

int n_threads() {
  static const int n = [] {
    int t = 8;
    if (const char* e = getenv("NR_COPY_THREADS")) t = atoi(e);
    const int hw = (int)std::thread::hardware_concurrency();
    if (hw > 0) t = std::min(t, hw);
    return std::max(1, std::min(t, 32));
  }();
  return n;
}

// Pipeline over chunks 0..n-1 with `nt` copy threads.  h2d: the threads fill
// chunk i (after the DMA that last used its slot completed), then the
// coordinator issues its DMA.  d2h: the coordinator issues chunk i's DMA (once
// the threads have drained the slot's previous chunk), waits for it, then the
// threads drain it.  Slices of a chunk are copied by all threads in parallel.
struct Pipe {
  std::atomic<int64_t> ready{-1};   // h2d: slots free through chunk `ready`; d2h: landed through `ready`
  std::atomic<int64_t> done[kRing];  // threads finished with the chunk in this slot (count)
  std::atomic<bool> abort{false};
};

void spin_until(const std::atomic<int64_t>& a, int64_t v, const std::atomic<bool>& abort) {
  int k = 0;
  while (a.load(std::memory_order_acquire) < v && !abort.load(std::memory_order_relaxed)) {
    if (++k > 64) std::this_thread::yield();
  }
}

int run(bool up, char* host, char* dev, int64_t bytes, hipStream_t s) {
  Ring* r = nullptr;
  const int rc = ring_for(up ? 0 : 1, &r);
  if (rc != NR_OK) return rc;
  const hipMemcpyKind kind = up ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
  if (bytes <= kDirect) {  // one bounce through slot 0
    if (hipEventSynchronize(r->ev[0]) != hipSuccess) goto fail;
    if (up) memcpy(r->buf[0], host, (size_t)bytes);
    if (hipMemcpyAsync(up ? (void*)dev : (void*)r->buf[0], up ? (const void*)r->buf[0] : (const void*)dev,
                       (size_t)bytes, kind, s) != hipSuccess ||
        hipEventRecord(r->ev[0], s) != hipSuccess)
      goto fail;
    if (!up) {
      if (hipEventSynchronize(r->ev[0]) != hipSuccess) goto fail;
      memcpy(host, r->buf[0], (size_t)bytes);
    }
    return NR_OK;
  }
  {
    const int64_t n = (bytes + kChunk - 1) / kChunk;
    const int nt = n_threads();
    Pipe p;
    for (int i = 0; i < kRing; ++i) p.done[i].store(0);
    auto chunk_len = [&](int64_t c) { return std::min(kChunk, bytes - c * kChunk); };
    // worker t copies slice t of every chunk
    auto worker = [&](int t) {
      for (int64_t c = 0; c < n; ++c) {
        spin_until(p.ready, c, p.abort);
        if (p.abort.load()) return;
        const int64_t len = chunk_len(c), per = ((len + nt - 1) / nt + 63) / 64 * 64;  // nt slices cover len
        const int64_t a = std::min(len, t * per), b = std::min(len, a + per);
        char* pin = r->buf[c % kRing];
        if (b > a) {
          if (up) memcpy(pin + a, host + c * kChunk + a, (size_t)(b - a));
          else memcpy(host + c * kChunk + a, pin + a, (size_t)(b - a));
        }
        p.done[c % kRing].fetch_add(1, std::memory_order_acq_rel);
      }
    };
    std::vector<std::thread> th;
    th.reserve(nt);
    for (int t = 0; t < nt; ++t) th.emplace_back(worker, t);
    bool ok = true;
    auto wait_slot_drained = [&](int64_t c) {  // the threads are done with chunk c (all nt slices)
      const int slot = (int)(c % kRing);
      const int64_t want = (c / kRing + 1) * nt;
      int k = 0;
      while (p.done[slot].load(std::memory_order_acquire) < want) {
        if (++k > 64) std::this_thread::yield();
      }
    };
    if (up) {
      for (int64_t c = 0; c < n && ok; ++c) {
        const int slot = (int)(c % kRing);
        // the slot's previous DMA (chunk c - kRing) must have read it before the threads refill it
        ok = hipEventSynchronize(r->ev[slot]) == hipSuccess;
        if (!ok) break;
        p.ready.store(c, std::memory_order_release);
        wait_slot_drained(c);
        ok = hipMemcpyAsync(dev + c * kChunk, r->buf[slot], (size_t)chunk_len(c), kind, s) == hipSuccess &&
             hipEventRecord(r->ev[slot], s) == hipSuccess;
      }
    } else {
      int64_t issued = 0;  // up to kRing DMAs in flight ahead of the threads
      for (int64_t c = 0; c < n && ok; ++c) {
        while (ok && issued < n && issued < c + kRing) {
          if (issued >= kRing) wait_slot_drained(issued - kRing);  // the threads have copied that slot out
          const int slot = (int)(issued % kRing);
          ok = hipMemcpyAsync(r->buf[slot], dev + issued * kChunk, (size_t)chunk_len(issued), kind, s) == hipSuccess &&
               hipEventRecord(r->ev[slot], s) == hipSuccess;
          ++issued;
        }
        ok = ok && hipEventSynchronize(r->ev[c % kRing]) == hipSuccess;
        if (ok) p.ready.store(c, std::memory_order_release);  // chunk c landed: the threads copy it out
      }
    }
    if (!ok) p.abort.store(true);
    for (auto& x : th) x.join();  // h2d: every byte of the caller's memory read; d2h: every byte written
    if (!ok) goto fail;
    return NR_OK;
  }
fail:
  set_error("nr_copy_%s: HIP copy or event call failed (%s)", up ? "h2d" : "d2h", hipGetErrorString(hipGetLastError()));
  return NR_ERR_HIP;
}

}  // namespace
}  // namespace nr

extern "C" int nr_copy_h2d(void* dst, const void* src, int64_t bytes, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(bytes >= 0, "nr_copy_h2d: bytes < 0");
  if (bytes == 0) return NR_OK;
  NR_CHECK_ARG(dst && src, "nr_copy_h2d: null pointer");
  NR_CHECK_DEVICE("nr_copy_h2d", dst);
  std::lock_guard<std::mutex> g(nr::g_mu);
  return nr::run(true, (char*)src, (char*)dst, bytes, (hipStream_t)stream);
}

extern "C" int nr_copy_d2h(void* dst, const void* src, int64_t bytes, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(bytes >= 0, "nr_copy_d2h: bytes < 0");
  if (bytes == 0) return NR_OK;
  NR_CHECK_ARG(dst && src, "nr_copy_d2h: null pointer");
  NR_CHECK_DEVICE("nr_copy_d2h", src);
  std::lock_guard<std::mutex> g(nr::g_mu);
  return nr::run(false, (char*)dst, (char*)src, bytes, (hipStream_t)stream);
}
