// RCCL communicator of the multi-GPU eval (SURVEY §8(b) nr_allgather, §8(e)):
// one process per GPU, the per-news table transformed in row shards and
// all-gathered once over xGMI.  The reference has no distributed code; this is
// the exchange step the north star adds.
//
// RCCL is resolved at run time (dlopen of librccl.so.1, reusing the copy the
// process already mapped, e.g. torch's) so the library has no link-time RCCL
// dependency and a host without RCCL still loads it (the entries then return
// NR_ERR_UNSUPPORTED).  Only host code here: the collective runs RCCL's own
// kernels on the caller's stream.
#include "nr_common.h"

#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include <chrono>
#include <mutex>
#include <thread>

namespace nr {
namespace {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*get_version)(int*) = nullptr;
  // non-blocking init with a deadline (optional: the blocking entries above suffice)
  ncclResult_t (*comm_init_rank_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*get_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  bool ok = false;
};

const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so"}) {
      h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);  // the process's RCCL (torch's) if mapped
      if (!h) h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) return;
    api.get_unique_id = (decltype(api.get_unique_id))dlsym(h, "ncclGetUniqueId");
    api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(h, "ncclCommInitRank");
    api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
    api.all_gather = (decltype(api.all_gather))dlsym(h, "ncclAllGather");
    api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
    api.get_version = (decltype(api.get_version))dlsym(h, "ncclGetVersion");
    api.comm_init_rank_config = (decltype(api.comm_init_rank_config))dlsym(h, "ncclCommInitRankConfig");
    api.get_async_error = (decltype(api.get_async_error))dlsym(h, "ncclCommGetAsyncError");
    api.comm_abort = (decltype(api.comm_abort))dlsym(h, "ncclCommAbort");
    api.ok = api.get_unique_id && api.comm_init_rank && api.comm_destroy && api.all_gather && api.error_string;
  });
  return api;
}

int rccl_missing(const char* fn) {
  set_error("%s: RCCL (librccl.so.1) is not available in this process", fn);
  return NR_ERR_UNSUPPORTED;
}

int rccl_fail(const char* fn, ncclResult_t r) {
  set_error("%s: %s (ncclResult %d)", fn, rccl().error_string ? rccl().error_string(r) : "?", (int)r);
  return NR_ERR_HIP;
}

// A non-blocking communicator's calls may return ncclInProgress: poll its state
// until it settles, up to `deadline_ms` (<= 0: no deadline).  Returns the
// settled state, or ncclInProgress when the deadline passed first.
ncclResult_t settle(ncclComm_t c, ncclResult_t r, int64_t deadline_ms) {
  const RcclApi& a = rccl();
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress) {
    if (deadline_ms > 0 && std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0)
                                   .count() >= deadline_ms)
      return ncclInProgress;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (a.get_async_error(c, &r) != ncclSuccess) return ncclInternalError;
  }
  return r;
}

}  // namespace
}  // namespace nr

struct nr_comm {
  ncclComm_t comm;
  int nranks, rank;
  bool nonblocking;
};

extern "C" int nr_rccl_version(void) {
  const nr::RcclApi& a = nr::rccl();
  int v = 0;
  if (!a.ok || !a.get_version || a.get_version(&v) != ncclSuccess) return 0;
  return v;
}

extern "C" int nr_comm_unique_id(unsigned char* id) {
  nr::clear_error();
  NR_CHECK_ARG(id, "nr_comm_unique_id: null id buffer");
  const nr::RcclApi& a = nr::rccl();
  if (!a.ok) return nr::rccl_missing("nr_comm_unique_id");
  ncclUniqueId u;
  const ncclResult_t r = a.get_unique_id(&u);
  if (r != ncclSuccess) return nr::rccl_fail("nr_comm_unique_id", r);
  memcpy(id, u.internal, NR_COMM_ID_BYTES);
  return NR_OK;
}

extern "C" int nr_comm_init_timeout(nr_comm_t* comm, const unsigned char* id, int nranks, int rank, int64_t timeout_ms) {
  nr::clear_error();
  NR_CHECK_ARG(comm && id, "nr_comm_init: null argument");
  NR_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "nr_comm_init: rank %d of %d", rank, nranks);
  *comm = nullptr;
  const nr::RcclApi& a = nr::rccl();
  if (!a.ok) return nr::rccl_missing("nr_comm_init");
  ncclUniqueId u;
  memcpy(u.internal, id, NR_COMM_ID_BYTES);
  ncclComm_t c = nullptr;
  const bool nonblocking = timeout_ms > 0 && a.comm_init_rank_config && a.get_async_error && a.comm_abort;
  if (!nonblocking) {
    const ncclResult_t r = a.comm_init_rank(&c, nranks, u, rank);  // collective over the nranks processes
    if (r != ncclSuccess) return nr::rccl_fail("nr_comm_init", r);
    *comm = new nr_comm{c, nranks, rank, false};
    return NR_OK;
  }
  // non-blocking init (config.blocking = 0): the call returns at once and the
  // communicator settles in the background; a peer that never joins leaves it
  // in progress, and at the deadline it is aborted instead of blocking forever
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = a.comm_init_rank_config(&c, nranks, u, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) return nr::rccl_fail("nr_comm_init", r);
  r = nr::settle(c, r, timeout_ms);
  if (r == ncclInProgress) {
    a.comm_abort(c);
    nr::set_error("nr_comm_init: rank %d of %d: the communicator did not form within %lld ms (a peer did not join); "
                  "aborted", rank, nranks, (long long)timeout_ms);
    return NR_ERR_TIMEOUT;
  }
  if (r != ncclSuccess) {
    a.comm_abort(c);
    return nr::rccl_fail("nr_comm_init", r);
  }
  *comm = new nr_comm{c, nranks, rank, true};
  return NR_OK;
}

extern "C" int nr_comm_init(nr_comm_t* comm, const unsigned char* id, int nranks, int rank) {
  return nr_comm_init_timeout(comm, id, nranks, rank, 0);
}

extern "C" int nr_comm_destroy(nr_comm_t comm) {
  nr::clear_error();
  if (!comm) return NR_OK;
  const nr::RcclApi& a = nr::rccl();
  ncclResult_t r = a.ok ? a.comm_destroy(comm->comm) : ncclSuccess;
  if (a.ok && comm->nonblocking) r = nr::settle(comm->comm, r, 0);
  delete comm;
  return r == ncclSuccess ? NR_OK : nr::rccl_fail("nr_comm_destroy", r);
}

extern "C" int nr_allgather(nr_comm_t comm, const void* send, void* recv, int64_t bytes_per_rank, void* stream) {
  nr::clear_error();
  NR_CHECK_ARG(comm, "nr_allgather: null communicator");
  NR_CHECK_ARG(bytes_per_rank >= 0, "nr_allgather: bytes_per_rank < 0");
  if (bytes_per_rank == 0) return NR_OK;
  NR_CHECK_ARG(send && recv, "nr_allgather: null buffer");
  NR_CHECK_DEVICE("nr_allgather", send, recv);
  const nr::RcclApi& a = nr::rccl();
  if (!a.ok) return nr::rccl_missing("nr_allgather");
  // in place when send == recv + rank * bytes_per_rank (RCCL's in-place rule)
  ncclResult_t r = a.all_gather(send, recv, (size_t)bytes_per_rank, ncclUint8, comm->comm, (hipStream_t)stream);
  if (comm->nonblocking) r = nr::settle(comm->comm, r, 0);  // enqueued once it settles
  if (r != ncclSuccess) return nr::rccl_fail("nr_allgather", r);
  return NR_OK;
}
