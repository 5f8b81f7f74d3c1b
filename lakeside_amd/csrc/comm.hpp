// Multi-GPU: one process per GPU, segments sharded across ranks, partial group tables merged over RCCL.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/lakeside_gpu.h"
#include "engine.hpp"
#include "layout.hpp"
#include "plan.hpp"

namespace lk {

int comm_world(const Engine& E);
// JSON object describing the communicator as its transport sees it ("null" without one): lk_engine_stats' "comm".
std::string comm_describe(const Engine& E);
// Collectives this rank has issued on the communicator (cumulative; a call's stats report the difference).  RCCL: one
// ncclAllGather per all-gather, one grouped ncclSend/ncclRecv set per point-to-point group; host transport: one
// callback all-gather each.
struct CommCounters {
  uint64_t allgathers = 0, allgather_bytes = 0, p2p_groups = 0, p2p_bytes = 0;
};
CommCounters comm_counters(const Engine& E);
int comm_rank(const Engine& E);
// RCCL loopback test mode at world 1 (LK_COMM_LOOPBACK=1): collectives and point-to-point transfers run anyway.
bool comm_loopback(const Engine& E);
// Concatenation, in rank order, of every rank's byte blob (variable length): one all-gather of the sizes,
// one of the blobs padded to the largest.
std::vector<std::string> comm_allgather_bytes(Engine& E, CallCtx& X, const std::string& mine);
// The agreement point: every rank contributes (status, payload) to one all-gather; when any rank's status is set
// (its `code`, or else its pending X.pend_code), every rank throws the lowest failing rank's PlanError -- no rank is
// left waiting in a later collective.  Returns every rank's payload, rank order.
std::vector<std::string> comm_allgather_status(Engine& E, CallCtx& X, int code, const std::string& msg,
                                               const std::string& payload);
// Every rank reports its local status (0 = ok); if any rank failed, every rank throws the first failure
// (PlanError with that rank's code), so no rank is left waiting in a later collective.
void comm_agree(Engine& E, CallCtx& X, int code, const std::string& msg);
// Run a rank-local stage that precedes a collective: a PlanError (or any std::exception) is kept as the call's
// pending status instead of unwinding this rank alone; the next agreement point fails every rank with it.
template <class F>
bool comm_local(CallCtx& X, F&& f) {
  if (X.pend_code) return false;
  try {
    f();
    return true;
  } catch (const PlanError& e) {
    X.pend_code = e.code;
    X.pend_msg = e.what();
  } catch (const std::exception& e) {
    X.pend_code = LK_ERR_DEVICE;
    X.pend_msg = e.what();
  }
  return false;
}
// After the last collective of a distributed call: a pending rank-local failure is thrown on this rank.
void comm_throw_pending(CallCtx& X);
// Tests only (env LK_FAULT=<stage>[@rank]): throws an injected LK_ERR_DEVICE at that stage on that rank (any rank
// without @rank), so the multi-rank failure paths can be exercised on hardware that does not fail.
void fault_point(const Engine& E, const char* stage);
// The same test as fault_point without throwing (a stage whose failure is a result, not an exception).
bool fault_hit(const Engine& E, const char* stage);
// comm_agree and an element-wise max of a small host byte array (glob column unions, NULL flags) in one all-gather.
void comm_agree_max_u8(Engine& E, CallCtx& X, int code, const std::string& msg, uint8_t* host, size_t n);
// Dense mode: reduce the partial aggregation table (P.rows/cnt/hi/lo/ext, nc cells) onto rank 0: counts by
// sum, min/max by min/max on order-preserving bits (exact), compensated sums gathered and added in rank order.
// Rank 0's receive buffer (world x the table) is placed by comm_reduce_prepare before the scan's agreement point.
void comm_reduce_prepare(Engine& E, CallCtx& X, size_t nc);
void comm_reduce_table(Engine& E, CallCtx& X, const QParams& P, int agg, size_t nc);
// Hash mode: every rank compacts its occupied slots into records; rank 0 gathers them and inserts every rank's
// records, in rank order, into a fresh table sized for their union (launch_merge_records).  On rank 0, P's table
// pointers and `cap` (slots) are replaced by the merged table's.
void comm_reduce_hash(Engine& E, CallCtx& X, QParams& P, int agg, unsigned long long& cap);

// Point-to-point exchange of device buffers (all-to-all / gather building block): `sends` and `recvs` list pieces
// (peer, device pointer, bytes); the pieces between one pair of ranks are matched in list order.  Pieces with
// peer == this rank are copied on the device.  RCCL: one grouped ncclSend/ncclRecv set (every peer on its own xGMI
// link at once).  Host transport: one all-gather round per destination rank.
struct Piece {
  int peer;
  void* ptr;
  size_t bytes;
};
void comm_exchange(Engine& E, CallCtx& X, const std::vector<Piece>& sends, const std::vector<Piece>& recvs);

// Shared host result block of a key-range reduce (one node): rank 0 offers a block of >= `bytes` from its pool of
// POSIX shared-memory blocks (pinned by every rank once per block generation), every rank maps it, and each rank's
// GPU writes its range's rows into it at the range's row offset -- the result rows cross all the node's PCIe links
// at once instead of funnelling through rank 0's.  Collective.  ok == false on every rank when rank 0 has no block
// (the caller gathers the rows into rank 0 instead); `mapped` == false on a rank that could not map it (the caller
// reports that in its completion status, which fails the call everywhere).  Rank 0's `lease` keeps the block out of
// the pool while its result lives.
struct EmitTarget {
  bool ok = false, mapped = false;
  uint8_t* host = nullptr;
  uint8_t* dev = nullptr;
  size_t cap = 0;
  std::shared_ptr<void> lease;
  int block = -1;      // rank 0's pool index and generation of the offered block
  uint64_t gen = 0;
};
EmitTarget comm_emit_begin(Engine& E, CallCtx& X, size_t bytes);
// After the agreement that follows every rank's writes.  agreed: every rank holds its mapping, so rank 0 unlinks this
// call's block name (a crash then leaves nothing in /dev/shm).  Not agreed (some rank failed to map or write): rank 0
// drops the block from its pool, so a later call creates a new generation rather than re-offering this one.
void comm_emit_end(Engine& E, const EmitTarget& T, bool agreed);

// Agreed dim space of an unrestricted group dimension over the ranks (dims.cpp; collective: every rank calls it in
// the same order).  The cached union is reused while no rank's dictionary changed (one all-gather); `rebuilt` says a
// new one was built; `ms` is the agreement's wall time on this rank.
std::shared_ptr<DimUnion> agree_dim_union(Engine& E, CallCtx& X, const std::string& col, uint32_t dict_n, double& ms,
                                          bool& rebuilt);

}  // namespace lk
