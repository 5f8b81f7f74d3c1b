// RCCL over xGMI: the exchange step of the sharded evaluation.
//
// Reference: segments are spread over worker pods by Math.floorMod(segmentId.hashCode, pods)
// (core/.../discovery/WorkerManager.scala:150-156) and the per-pod partial aggregates are merged by the
// query-api (TimeGroupedSketchAggregator.scala:57-114).  Here each GPU scans its shard into a partial
// table in a key space every rank derives identically from the request, then one reduce lands the
// merged table on rank 0, which alone finalizes and emits.  Tables are small (KB-MB): the reduce is
// latency-bound, a single collective per array.
#include "comm.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "../../include/lakeside_gpu.h"
#include "kernels.hpp"
#include "plan.hpp"

namespace lk {

struct Comm {
  ncclComm_t comm = nullptr;
  int world = 1;
  int rank = 0;
};

#define NCCL_TRY(x)                                                                            \
  do {                                                                                         \
    ncclResult_t _r = (x);                                                                     \
    if (_r != ncclSuccess)                                                                     \
      throw PlanError(LK_ERR_DEVICE, std::string("RCCL: ") + #x + ": " + ncclGetErrorString(_r)); \
  } while (0)

#define HIP_TRY2(x)                                                                             \
  do {                                                                                          \
    hipError_t _e = (x);                                                                        \
    if (_e != hipSuccess)                                                                       \
      throw PlanError(LK_ERR_DEVICE, std::string("HIP: ") + #x + ": " + hipGetErrorString(_e)); \
  } while (0)

int comm_world(const Engine& E) { return E.comm ? E.comm->world : 1; }
int comm_rank(const Engine& E) { return E.comm ? E.comm->rank : 0; }

void Engine::comm_destroy() {
  if (comm) {
    if (comm->comm) ncclCommDestroy(comm->comm);
    delete comm;
    comm = nullptr;
  }
}

void comm_allreduce_max_u8(Engine& E, uint8_t* host, size_t n) {
  if (!E.comm) throw PlanError(LK_ERR_ARG, "lk_comm_init has not been called");
  uint8_t* d = static_cast<uint8_t*>(E.workspace("comm_u8", n));
  HIP_TRY2(hipSetDevice(E.device));
  HIP_TRY2(hipMemcpyAsync(d, host, n, hipMemcpyHostToDevice, E.stream));
  NCCL_TRY(ncclAllReduce(d, d, n, ncclUint8, ncclMax, E.comm->comm, E.stream));
  HIP_TRY2(hipMemcpyAsync(host, d, n, hipMemcpyDeviceToHost, E.stream));
  HIP_TRY2(hipStreamSynchronize(E.stream));
}

void comm_reduce_table(Engine& E, const QParams& P, int agg, size_t nc) {
  if (!E.comm) throw PlanError(LK_ERR_ARG, "lk_comm_init has not been called");
  Comm& C = *E.comm;
  if (C.world == 1) return;
  ncclComm_t cm = C.comm;
  hipStream_t st = E.stream;
  NCCL_TRY(ncclReduce(P.rows, P.rows, nc, ncclUint64, ncclSum, 0, cm, st));
  NCCL_TRY(ncclReduce(P.cnt, P.cnt, nc, ncclUint64, ncclSum, 0, cm, st));
  if (agg == AGG_MIN) NCCL_TRY(ncclReduce(P.ext, P.ext, nc, ncclUint64, ncclMin, 0, cm, st));
  if (agg == AGG_MAX) NCCL_TRY(ncclReduce(P.ext, P.ext, nc, ncclUint64, ncclMax, 0, cm, st));
  if (agg == AGG_SUM) {
    // hi and lo are adjacent in the table: one 2*nc-double message per rank, merged in rank order
    double* parts = C.rank == 0 ? static_cast<double*>(E.workspace("comm_parts", size_t(C.world) * nc * 16)) : nullptr;
    NCCL_TRY(ncclGroupStart());
    if (C.rank == 0) {
      for (int r = 1; r < C.world; r++) NCCL_TRY(ncclRecv(parts + size_t(r) * nc * 2, nc * 2, ncclFloat64, r, cm, st));
    } else {
      NCCL_TRY(ncclSend(P.hi, nc * 2, ncclFloat64, 0, cm, st));
    }
    NCCL_TRY(ncclGroupEnd());
    if (C.rank == 0) HIP_TRY2(launch_merge_dd(P.hi, P.lo, parts, C.world, nc, st));
  }
}

}  // namespace lk

extern "C" {

int lk_comm_unique_id(uint8_t* id) {
  if (!id) return LK_ERR_ARG;
  static_assert(sizeof(ncclUniqueId) == LK_UNIQUE_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) {
    lk::set_error(std::string("RCCL: ncclGetUniqueId: ") + ncclGetErrorString(r));
    return LK_ERR_DEVICE;
  }
  memcpy(id, &u, sizeof(u));
  return LK_OK;
}

int lk_comm_init(lk_engine* e, const uint8_t* id, int world, int rank) {
  if (!e || !id || world < 1 || rank < 0 || rank >= world) return LK_ERR_ARG;
  lk::Engine& E = *e->e;
  if (E.comm) {
    lk::set_error("communicator already initialised");
    return LK_ERR_ARG;
  }
  if (hipSetDevice(E.device) != hipSuccess) return LK_ERR_DEVICE;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  auto* C = new lk::Comm();
  C->world = world;
  C->rank = rank;
  ncclResult_t r = ncclCommInitRank(&C->comm, world, u, rank);
  if (r != ncclSuccess) {
    lk::set_error(std::string("RCCL: ncclCommInitRank: ") + ncclGetErrorString(r));
    delete C;
    return LK_ERR_DEVICE;
  }
  E.comm = C;
  return LK_OK;
}

}  // extern "C"
