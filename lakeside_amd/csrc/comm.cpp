// The exchange step of the sharded evaluation: RCCL over xGMI (default), or a caller-supplied host all-gather.
//
// Reference: segments are spread over worker pods by Math.floorMod(segmentId.hashCode, pods)
// (core/.../discovery/WorkerManager.scala:150-156) and the per-pod partial aggregates are merged by the
// query-api (TimeGroupedSketchAggregator.scala:57-114).  Here each GPU scans its shard into a partial
// table in a key space every rank derives identically from the request (bucket space from the window;
// group dims from the filter, or from the sorted union of every rank's dictionary), then rank 0 gathers the
// partial tables, folds them in rank order (merge_tables) and alone finalizes and emits.
//
// Two primitives carry everything:
//   allgather_bytes: every rank's host blob (variable length) -> all ranks, in rank order
//     (glob column unions, dictionaries);
//   gather_table: every rank's device table block -> rank 0's device buffer, in rank order.
// RCCL: all-gather of sizes + padded blobs; grouped ncclSend/ncclRecv into rank 0 (each peer on its own xGMI
// link, the tables are KB-MB so this is latency-bound).  Host transport (lk_comm_init_host): the caller's
// fixed-size all-gather callback (e.g. torch.distributed/gloo, MPI) over host copies of the same buffers;
// it lets several ranks share one GPU (RCCL refuses two ranks on one device), and feeds the same merge.
#include "comm.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>

#include "../../include/lakeside_gpu.h"
#include "kernels.hpp"
#include "plan.hpp"

namespace lk {

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

// Shared host result blocks (one node; comm_emit_begin): rank 0 owns a small pool of POSIX shared-memory blocks,
// every rank maps and registers them with HIP once per block generation, and each rank's GPU writes its key range's
// result rows straight into rank 0's result over its own PCIe link.  A mapping is its own reference-counted object:
// the pool entry holds one reference and a result whose rows live in the block holds another (through its lease),
// so a result outlives the engine and communicator that produced it.  The name is unlinked as soon as
// every rank has mapped the generation, so a crashed process leaves nothing behind in /dev/shm.
struct ShmBlock {
  std::string name;
  void* host = nullptr;
  void* dev = nullptr;
  size_t cap = 0;
  bool linked = false;          // rank 0: the name still exists in /dev/shm
  ~ShmBlock() {
    if (host) {
      (void)hipHostUnregister(host);
      (void)hipGetLastError();
      munmap(host, cap);
    }
    if (linked) shm_unlink(name.c_str());
  }
  void unlink() {
    if (linked) shm_unlink(name.c_str());
    linked = false;
  }
};
struct ShmMap {
  std::shared_ptr<ShmBlock> blk;
  uint64_t gen = 0;
  std::weak_ptr<void> lease;    // rank 0: the result currently holding the block
  size_t cap() const { return blk ? blk->cap : 0; }
  void release() { blk.reset(); }
};
// A result's hold on a block: keeps the mapping alive and marks the pool entry busy.
struct ShmLease {
  std::shared_ptr<ShmBlock> blk;
};

struct Comm {
  int world = 1;
  int rank = 0;
  std::map<int, ShmMap> shm;    // by block index (rank 0's pool / this rank's mappings of it)
  uint64_t shm_gen = 0;
  // Loopback (RCCL only, env LK_COMM_LOOPBACK=1 at lk_comm_init; tests): at world 1 every collective still runs --
  // all-gathers through ncclAllGather, the table / record gathers and the key-range pieces through grouped
  // ncclSend/ncclRecv to self -- and the merge reads what came back through RCCL, so the single-GPU box executes
  // (and checks) every RCCL data-path call the 8-GPU run makes.
  bool loopback = false;
  CommCounters cnt;             // collectives issued by this rank (stats)
  bool active() const { return world > 1 || loopback; }
  virtual ~Comm() = default;   // mappings go with their last reference (pool entry or a live result)
  // host blobs of every rank, rank order
  virtual std::vector<std::string> allgather_bytes(Engine& E, CallCtx& X, const std::string& mine) = 0;
  // `bytes[r]` of device memory from every rank r into rank 0's `recv` at offsets `off[r]` (slot 0 is left
  // untouched), ordered on X.stream
  virtual void gather_to_root(Engine& E, CallCtx& X, const void* send, void* recv, const std::vector<size_t>& bytes,
                              const std::vector<size_t>& off) = 0;
  // pieces to / from other ranks (comm_exchange)
  virtual void exchange(Engine& E, CallCtx& X, const std::vector<Piece>& sends, const std::vector<Piece>& recvs) = 0;
  // the transport's own view of the communicator (lk_engine_stats): RCCL reports what ncclCommCount /
  // ncclCommUserRank / ncclCommCuDevice return, not what the caller passed to lk_comm_init
  virtual std::string describe() const = 0;
};

namespace {

constexpr size_t kCommPinBytes = size_t(64) << 10;

struct RcclComm final : Comm {
  ncclComm_t comm = nullptr;
  ~RcclComm() override {
    if (comm) ncclCommDestroy(comm);
  }

  std::string describe() const override {
    int n = -1, r = -1, dev = -1;
    if (comm) {
      if (ncclCommCount(comm, &n) != ncclSuccess) n = -1;
      if (ncclCommUserRank(comm, &r) != ncclSuccess) r = -1;
      if (ncclCommCuDevice(comm, &dev) != ncclSuccess) dev = -1;
    }
    return "{\"transport\":\"rccl\",\"world\":" + std::to_string(n) + ",\"rank\":" + std::to_string(r) +
           ",\"device\":" + std::to_string(dev) + ",\"loopback\":" + (loopback ? "true" : "false") + "}";
  }

  std::vector<std::string> allgather_bytes(Engine& E, CallCtx& X, const std::string& mine) override {
    if (!active()) return {mine};
    HIP_TRY2(hipSetDevice(E.device));
    hipStream_t st = X.stream;
    std::vector<uint64_t> sz(size_t(world), 0);
    // One all-gather of fixed slots ([length | bytes], through pinned host memory) carries every rank's blob when
    // each fits its slot -- the agreement points' status blobs always do; a larger blob takes a second all-gather
    // sized by the lengths the first one delivered.
    constexpr size_t SLOT = 512;
    if (size_t(world + 1) * SLOT <= kCommPinBytes) {
      if (!X.comm_pin) HIP_TRY2(hipHostMalloc(&X.comm_pin, kCommPinBytes));
      uint8_t* h = static_cast<uint8_t*>(X.comm_pin);
      uint8_t* d = static_cast<uint8_t*>(X.workspace("comm_slots", size_t(world) * SLOT));
      const uint64_t n = mine.size();
      memcpy(h, &n, 8);
      if (n <= SLOT - 8 && n) memcpy(h + 8, mine.data(), n);
      HIP_TRY2(hipMemcpyAsync(d + size_t(rank) * SLOT, h, SLOT, hipMemcpyHostToDevice, st));
      NCCL_TRY(ncclAllGather(d + size_t(rank) * SLOT, d, SLOT, ncclUint8, comm, st));
      cnt.allgathers++;
      cnt.allgather_bytes += uint64_t(world) * SLOT;
      HIP_TRY2(hipMemcpyAsync(h + SLOT, d, size_t(world) * SLOT, hipMemcpyDeviceToHost, st));
      HIP_TRY2(hipStreamSynchronize(st));
      bool fits = true;
      for (int r = 0; r < world; r++) {
        memcpy(&sz[size_t(r)], h + SLOT * size_t(r + 1), 8);
        fits = fits && sz[size_t(r)] <= SLOT - 8;
      }
      if (fits) {
        std::vector<std::string> out(static_cast<size_t>(world));
        for (int r = 0; r < world; r++)
          out[size_t(r)].assign(reinterpret_cast<const char*>(h + SLOT * size_t(r + 1) + 8), size_t(sz[size_t(r)]));
        return out;
      }
    } else {
      uint64_t* dsz = static_cast<uint64_t*>(X.workspace("comm_sizes", size_t(world) * 8));
      sz[size_t(rank)] = mine.size();
      HIP_TRY2(hipMemcpyAsync(dsz + rank, &sz[size_t(rank)], 8, hipMemcpyHostToDevice, st));
      NCCL_TRY(ncclAllGather(dsz + rank, dsz, 1, ncclUint64, comm, st));
      cnt.allgathers++;
      HIP_TRY2(hipMemcpyAsync(sz.data(), dsz, size_t(world) * 8, hipMemcpyDeviceToHost, st));
      HIP_TRY2(hipStreamSynchronize(st));
    }
    uint64_t mx = 1;
    for (uint64_t x : sz) mx = std::max(mx, x);
    uint8_t* d = static_cast<uint8_t*>(X.workspace("comm_blobs", size_t(world) * mx));
    if (!mine.empty())
      HIP_TRY2(hipMemcpyAsync(d + size_t(rank) * mx, mine.data(), mine.size(), hipMemcpyHostToDevice, st));
    NCCL_TRY(ncclAllGather(d + size_t(rank) * mx, d, mx, ncclUint8, comm, st));
    cnt.allgathers++;
    cnt.allgather_bytes += uint64_t(world) * mx;
    std::string all(size_t(world) * mx, '\0');
    HIP_TRY2(hipMemcpyAsync(&all[0], d, all.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY2(hipStreamSynchronize(st));
    std::vector<std::string> out(static_cast<size_t>(world));
    for (int r = 0; r < world; r++) out[size_t(r)] = all.substr(size_t(r) * mx, sz[size_t(r)]);
    return out;
  }

  void gather_to_root(Engine& E, CallCtx& X, const void* send, void* recv, const std::vector<size_t>& bytes,
                      const std::vector<size_t>& off) override {
    if (!active()) return;
    // grouped point-to-point: every peer streams into rank 0 over its own xGMI link at once (loopback: rank 0's own
    // block too, into slot 0)
    cnt.p2p_groups++;
    for (int r = 0; r < world; r++)
      if (r != 0 || loopback) cnt.p2p_bytes += bytes[size_t(r)];
    NCCL_TRY(ncclGroupStart());
    if (rank == 0) {
      for (int r = loopback ? 0 : 1; r < world; r++)
        if (bytes[size_t(r)])
          NCCL_TRY(ncclRecv(static_cast<uint8_t*>(recv) + off[size_t(r)], bytes[size_t(r)], ncclUint8, r, comm, X.stream));
    }
    if ((rank != 0 || loopback) && bytes[size_t(rank)]) NCCL_TRY(ncclSend(send, bytes[size_t(rank)], ncclUint8, 0, comm, X.stream));
    NCCL_TRY(ncclGroupEnd());
  }

  void exchange(Engine& E, CallCtx& X, const std::vector<Piece>& sends, const std::vector<Piece>& recvs) override {
    // loopback: own pieces go through RCCL as well (send / recv to self, matched in list order)
    cnt.p2p_groups++;
    for (const Piece& p : sends)
      if (p.peer != rank || loopback) cnt.p2p_bytes += p.bytes;
    NCCL_TRY(ncclGroupStart());
    for (const Piece& p : sends)
      if ((p.peer != rank || loopback) && p.bytes) NCCL_TRY(ncclSend(p.ptr, p.bytes, ncclUint8, p.peer, comm, X.stream));
    for (const Piece& p : recvs)
      if ((p.peer != rank || loopback) && p.bytes) NCCL_TRY(ncclRecv(p.ptr, p.bytes, ncclUint8, p.peer, comm, X.stream));
    NCCL_TRY(ncclGroupEnd());
  }
};

struct HostComm final : Comm {
  lk_allgather_fn fn = nullptr;
  void* user = nullptr;

  std::string describe() const override {
    return "{\"transport\":\"host\",\"world\":" + std::to_string(world) + ",\"rank\":" + std::to_string(rank) +
           ",\"loopback\":false}";
  }

  void allgather(const void* send, size_t bytes, void* recv) {
    cnt.allgathers++;
    cnt.allgather_bytes += uint64_t(world) * bytes;
    if (fn(user, send, bytes, recv) != 0) throw PlanError(LK_ERR_DEVICE, "host transport: all-gather callback failed");
  }

  std::vector<std::string> allgather_bytes(Engine& E, CallCtx& X, const std::string& mine) override {
    if (world == 1) return {mine};
    const uint64_t n = mine.size();
    std::vector<uint64_t> sz(static_cast<size_t>(world));
    allgather(&n, 8, sz.data());
    uint64_t mx = 1;
    for (uint64_t x : sz) mx = std::max(mx, x);
    std::string pad(mine);
    pad.resize(mx, '\0');
    std::string all(size_t(world) * mx, '\0');
    allgather(pad.data(), mx, &all[0]);
    std::vector<std::string> out(static_cast<size_t>(world));
    for (int r = 0; r < world; r++) out[size_t(r)] = all.substr(size_t(r) * mx, sz[size_t(r)]);
    return out;
  }

  void gather_to_root(Engine& E, CallCtx& X, const void* send, void* recv, const std::vector<size_t>& bytes,
                      const std::vector<size_t>& off) override {
    if (world == 1) return;
    // each rank's block travels behind a fixed header -- 8-byte status + the first bytes of its message: a rank whose
    // device copy failed still takes part in the all-gather, and every rank then throws that failure (none is left
    // inside the collective)
    constexpr size_t H = 128;
    size_t mx = 1;
    for (size_t b : bytes) mx = std::max(mx, b);
    std::vector<uint8_t> mine(H + mx, 0), all(size_t(world) * (H + mx));
    uint64_t status = 0;
    comm_local(X, [&] {
      fault_point(E, "gather");
      HIP_TRY2(hipSetDevice(E.device));
      if (bytes[size_t(rank)]) {
        HIP_TRY2(hipMemcpyAsync(mine.data() + H, send, bytes[size_t(rank)], hipMemcpyDeviceToHost, X.stream));
        HIP_TRY2(hipStreamSynchronize(X.stream));
      }
    });
    if (X.pend_code) {
      status = uint64_t(uint32_t(X.pend_code));
      memcpy(mine.data() + 8, X.pend_msg.data(), std::min(X.pend_msg.size(), H - 9));
    }
    memcpy(mine.data(), &status, 8);
    allgather(mine.data(), H + mx, all.data());
    for (int r = 0; r < world; r++) {
      uint64_t st;
      const uint8_t* blk = all.data() + size_t(r) * (H + mx);
      memcpy(&st, blk, 8);
      if (st) {
        const std::string m = r == rank ? X.pend_msg
                                        : "rank " + std::to_string(r) + ": " + reinterpret_cast<const char*>(blk + 8);
        X.pend_code = 0;
        X.pend_msg.clear();
        throw PlanError(int(st), m);
      }
    }
    if (rank == 0) {   // the last step of the gather: rank 0 alone
      for (int r = 1; r < world; r++)
        if (bytes[size_t(r)])
          HIP_TRY2(hipMemcpyAsync(static_cast<uint8_t*>(recv) + off[size_t(r)], all.data() + size_t(r) * (H + mx) + H,
                                  bytes[size_t(r)], hipMemcpyHostToDevice, X.stream));
      HIP_TRY2(hipStreamSynchronize(X.stream));   // `all` is freed on return
    }
  }

  void exchange(Engine& E, CallCtx& X, const std::vector<Piece>& sends, const std::vector<Piece>& recvs) override {
    // one all-gather round per destination d: every rank contributes its pieces for d, concatenated (padded to
    // the largest contribution); d unpacks each source's bytes into its receive pieces from that source, in order.
    // Each round's size all-gather carries every rank's status (a failed device copy -- of this round, or the
    // previous round's unpacking -- fails every rank there); the last round's unpacking failure stays pending for
    // the caller's next agreement point.
    for (int d = 0; d < world; d++) {
      size_t mine_n = 0;
      for (const Piece& p : sends)
        if (p.peer == d && d != rank) mine_n += p.bytes;
      std::vector<uint8_t> buf(std::max<size_t>(mine_n, 1), 0);
      comm_local(X, [&] {
        HIP_TRY2(hipSetDevice(E.device));
        size_t o = 0;
        for (const Piece& p : sends)
          if (p.peer == d && d != rank && p.bytes) {
            HIP_TRY2(hipMemcpyAsync(buf.data() + o, p.ptr, p.bytes, hipMemcpyDeviceToHost, X.stream));
            o += p.bytes;
          }
        HIP_TRY2(hipStreamSynchronize(X.stream));
      });
      uint64_t hdr[2] = {mine_n, uint64_t(uint32_t(X.pend_code))};
      std::vector<uint64_t> sz2(size_t(world) * 2);
      allgather(hdr, 16, sz2.data());
      for (int r = 0; r < world; r++)
        if (sz2[size_t(r) * 2 + 1]) {
          const std::string m = r == rank ? X.pend_msg : "rank " + std::to_string(r) + ": device copy of its exchange pieces failed";
          X.pend_code = 0;
          X.pend_msg.clear();
          throw PlanError(int(sz2[size_t(r) * 2 + 1]), m);
        }
      size_t mx = 1;
      for (int r = 0; r < world; r++) mx = std::max(mx, size_t(sz2[size_t(r) * 2]));
      buf.resize(mx, 0);
      std::vector<uint8_t> all(size_t(world) * mx);
      allgather(buf.data(), mx, all.data());
      if (d != rank) continue;
      comm_local(X, [&] {
        std::vector<size_t> cur(size_t(world), 0);
        for (const Piece& p : recvs) {
          if (p.peer == rank || !p.bytes) continue;
          size_t& c = cur[size_t(p.peer)];
          if (c + p.bytes > sz2[size_t(p.peer) * 2]) throw PlanError(LK_ERR_DEVICE, "host transport: exchange size mismatch");
          HIP_TRY2(hipMemcpyAsync(p.ptr, all.data() + size_t(p.peer) * mx + c, p.bytes, hipMemcpyHostToDevice, X.stream));
          c += p.bytes;
        }
        HIP_TRY2(hipStreamSynchronize(X.stream));   // `all` is freed at the end of the round
      });
    }
  }
};

}  // namespace

int comm_world(const Engine& E) { return E.comm ? E.comm->world : 1; }
// The communicator's description, cached when lk_comm_init* installed it: a stats call never touches the
// communicator itself, so it cannot race with its creation.
std::string comm_describe(const Engine& E) {
  std::lock_guard<std::mutex> g(const_cast<Engine&>(E).comm_init_mu);
  return E.comm_desc;
}
CommCounters comm_counters(const Engine& E) { return E.comm ? E.comm->cnt : CommCounters{}; }
bool comm_loopback(const Engine& E) { return E.comm && E.comm->loopback; }
int comm_rank(const Engine& E) { return E.comm ? E.comm->rank : 0; }

void Engine::comm_destroy() {
  delete comm;
  comm = nullptr;
}

static Comm& need_comm(Engine& E) {
  if (!E.comm) throw PlanError(LK_ERR_ARG, "lk_comm_init has not been called");
  return *E.comm;
}

std::vector<std::string> comm_allgather_status(Engine& E, CallCtx& X, int code, const std::string& msg,
                                               const std::string& payload) {
  Comm& C = need_comm(E);
  std::string m = msg;
  if (!code && X.pend_code) {   // a failure met after an earlier collective step travels with this agreement
    code = X.pend_code;
    m = X.pend_msg;
  }
  X.pend_code = 0;
  X.pend_msg.clear();
  if (!C.active()) {
    if (code) throw PlanError(code, m);
    return {payload};
  }
  // blob: status (4 B) | message length (4 B) | message | payload
  std::string mine(8, '\0');
  const uint32_t ml = code ? uint32_t(m.size()) : 0u;
  memcpy(&mine[0], &code, 4);
  memcpy(&mine[4], &ml, 4);
  if (code) mine += m;
  mine += payload;
  std::vector<std::string> all = C.allgather_bytes(E, X, mine);
  for (int r = 0; r < C.world; r++) {
    const std::string& b = all[size_t(r)];
    int c = 0;
    uint32_t l = 0;
    if (b.size() < 8) throw PlanError(LK_ERR_DEVICE, "internal: short status blob from rank " + std::to_string(r));
    memcpy(&c, b.data(), 4);
    memcpy(&l, b.data() + 4, 4);
    if (c) throw PlanError(c, (r == C.rank ? std::string() : "rank " + std::to_string(r) + ": ") + b.substr(8, l));
  }
  for (auto& b : all) {
    uint32_t l = 0;
    memcpy(&l, b.data() + 4, 4);
    b.erase(0, 8 + size_t(l));
  }
  return all;
}

void comm_agree_max_u8(Engine& E, CallCtx& X, int code, const std::string& msg, uint8_t* host, size_t n) {
  const std::vector<std::string> all =
      comm_allgather_status(E, X, code, msg, std::string(reinterpret_cast<const char*>(host), n));
  for (auto& b : all) {
    if (b.size() != n) throw PlanError(LK_ERR_ARG, "ranks disagree on the request (glob column union size)");
    for (size_t i = 0; i < n; i++) host[i] = std::max(host[i], uint8_t(b[i]));
  }
}

std::vector<std::string> comm_allgather_bytes(Engine& E, CallCtx& X, const std::string& mine) {
  return need_comm(E).allgather_bytes(E, X, mine);
}

void comm_agree(Engine& E, CallCtx& X, int code, const std::string& msg) {
  (void)comm_allgather_status(E, X, code, msg, std::string());
}

void comm_throw_pending(CallCtx& X) {
  if (!X.pend_code) return;
  const int c = X.pend_code;
  const std::string m = X.pend_msg;
  X.pend_code = 0;
  X.pend_msg.clear();
  throw PlanError(c, m);
}

bool fault_hit(const Engine& E, const char* stage) {
  const char* f = getenv("LK_FAULT");
  if (!f || !*f) return false;
  const std::string spec(f);
  const size_t at = spec.find('@');
  const bool hit = spec.substr(0, at) == stage &&
                   (at == std::string::npos || atoi(spec.c_str() + at + 1) == comm_rank(E));
  if (getenv("LK_FAULT_TRACE"))
    fprintf(stderr, "[lk fault] rank %d stage %s spec %s -> %s\n", comm_rank(E), stage, f, hit ? "inject" : "pass");
  return hit;
}

void fault_point(const Engine& E, const char* stage) {
  if (fault_hit(E, stage)) throw PlanError(LK_ERR_DEVICE, std::string("injected fault at stage '") + stage + "' (LK_FAULT)");
}

void comm_exchange(Engine& E, CallCtx& X, const std::vector<Piece>& sends, const std::vector<Piece>& recvs) {
  Comm& C = need_comm(E);
  HIP_TRY2(hipSetDevice(E.device));
  // own pieces: device copies, matched in list order
  std::vector<const Piece*> os, orv;
  for (const Piece& p : sends)
    if (p.peer == C.rank) os.push_back(&p);
  for (const Piece& p : recvs)
    if (p.peer == C.rank) orv.push_back(&p);
  if (os.size() != orv.size()) throw PlanError(LK_ERR_DEVICE, "internal: own exchange pieces do not pair up");
  for (size_t i = 0; i < os.size(); i++) {
    if (os[i]->bytes != orv[i]->bytes) throw PlanError(LK_ERR_DEVICE, "internal: own exchange piece sizes differ");
    if (os[i]->bytes && !C.loopback)
      HIP_TRY2(hipMemcpyAsync(orv[i]->ptr, os[i]->ptr, os[i]->bytes, hipMemcpyDeviceToDevice, X.stream));
  }
  if (C.active()) C.exchange(E, X, sends, recvs);
}

void comm_reduce_prepare(Engine& E, CallCtx& X, size_t nc) {
  Comm& C = need_comm(E);
  if (!C.active() || C.rank != 0) return;
  const size_t bytes = nc * 8 * 5;
  void* parts = X.workspace("comm_parts", size_t(C.world) * bytes);
  // loopback: rank 0's own table makes the round trip into slot 0 (poisoned first, so a transfer that did not
  // happen cannot pass), and the table is rebuilt from what arrived
  if (C.loopback) HIP_TRY2(hipMemsetAsync(parts, 0xA5, bytes, X.stream));
}

void comm_reduce_table(Engine& E, CallCtx& X, const QParams& P, int agg, size_t nc) {
  Comm& C = need_comm(E);
  if (!C.active()) return;
  // The table is one contiguous block [rows | cnt | hi | lo | ext] (eval.cpp).  Rank 0's receive buffer was placed
  // by comm_reduce_prepare before the scan's agreement point, so nothing between that agreement and the gather can
  // fail on one rank alone.
  const size_t bytes = nc * 8 * 5;
  unsigned long long* parts = nullptr;
  if (C.rank == 0) {
    auto it = X.ws.find("comm_parts");
    if (it == X.ws.end() || it->second.cap < size_t(C.world) * bytes)
      throw PlanError(LK_ERR_DEVICE, "internal: comm_reduce_prepare was not called");
    parts = static_cast<unsigned long long*>(it->second.p);
  }
  std::vector<size_t> sz(size_t(C.world), bytes), off(size_t(C.world));
  for (int r = 0; r < C.world; r++) off[size_t(r)] = size_t(r) * bytes;
  C.gather_to_root(E, X, P.rows, parts, sz, off);
  if (C.rank == 0) {   // after the last collective: rank 0 alone
    fault_point(E, "merge");
    if (C.loopback) HIP_TRY2(hipMemcpyAsync(P.rows, parts, bytes, hipMemcpyDeviceToDevice, X.stream));
    TableRef T{P.rows, P.cnt, P.hi, P.lo, P.ext};
    HIP_TRY2(launch_merge_tables(T, parts, C.world, nc, agg, X.stream));
  }
}

void comm_reduce_hash(Engine& E, CallCtx& X, QParams& P, int agg, unsigned long long& cap) {
  Comm& C = need_comm(E);
  if (!C.active()) return;
  // this rank's occupied slots -> compact records [key | rows | cnt | hi | lo | ext]; a failure here travels with
  // the record-count all-gather
  uint32_t n = 0;
  unsigned long long* recs = nullptr;
  comm_local(X, [&] {
    fault_point(E, "records");
    SParams S{};
    S.keys = P.hkeys;
    S.rows = P.rows;
    S.cnt = P.cnt;
    S.hi = P.hi;
    S.lo = P.lo;
    S.ext = P.ext;
    S.cap = cap;
    const uint32_t nb = sparse_blocks(cap);
    uint32_t* counts = static_cast<uint32_t*>(X.workspace("comm_rec_counts", (size_t(nb) + 2) * 4));
    HIP_TRY2(launch_sparse_count(S, counts, X.stream));
    HIP_TRY2(hipMemcpyAsync(&n, counts + nb, 4, hipMemcpyDeviceToHost, X.stream));
    HIP_TRY2(hipStreamSynchronize(X.stream));
    recs = static_cast<unsigned long long*>(X.workspace("comm_recs", size_t(n) * 48 + 64));
    HIP_TRY2(launch_table_records(P, cap, counts, recs, n, X.stream));
    HIP_TRY2(hipStreamSynchronize(X.stream));   // records complete before they are sent
  });
  // record counts of every rank, then the records into rank 0 (rank order)
  const uint64_t n64 = n;
  const std::vector<std::string> all =
      comm_allgather_status(E, X, 0, std::string(), std::string(reinterpret_cast<const char*>(&n64), 8));
  std::vector<size_t> sz(size_t(C.world)), off(size_t(C.world));
  size_t total = 0, nrec = 0;
  for (int r = 0; r < C.world; r++) {
    uint64_t x;
    memcpy(&x, all[size_t(r)].data(), 8);
    sz[size_t(r)] = size_t(x) * 48;
    off[size_t(r)] = total;
    total += sz[size_t(r)];
    nrec += size_t(x);
  }
  // rank 0's receive buffer (sized only now): placed, then agreed on before the point-to-point gather
  unsigned long long* parts = nullptr;
  comm_local(X, [&] {
    if (C.rank != 0) return;
    parts = static_cast<unsigned long long*>(X.workspace("comm_rec_parts", total + 64));
    if (C.loopback && sz[0]) HIP_TRY2(hipMemsetAsync(parts, 0xA5, sz[0], X.stream));
  });
  comm_agree(E, X, 0, std::string());
  C.gather_to_root(E, X, recs, parts, sz, off);
  if (C.rank != 0) return;
  // rank 0 (after the last collective): a fresh table for the union (at most nrec distinct keys, load factor <= 1/2)
  unsigned long long cap0 = 1 << 16;
  while (cap0 < 2 * nrec) cap0 <<= 1;
  uint8_t* tb = static_cast<uint8_t*>(X.workspace("table_merged", size_t(cap0) * 48 + 1024));
  P.rows = reinterpret_cast<unsigned long long*>(tb);
  P.cnt = reinterpret_cast<unsigned long long*>(tb + cap0 * 8);
  P.hi = reinterpret_cast<double*>(tb + cap0 * 16);
  P.lo = reinterpret_cast<double*>(tb + cap0 * 24);
  P.ext = reinterpret_cast<unsigned long long*>(tb + cap0 * 32);
  P.hkeys = reinterpret_cast<unsigned long long*>(tb + cap0 * 40);
  P.hmask = cap0 - 1;
  HIP_TRY2(hipMemsetAsync(tb, 0, size_t(cap0) * 32, X.stream));
  HIP_TRY2(hipMemsetAsync(P.ext, agg == AGG_MIN ? 0xff : 0, size_t(cap0) * 8, X.stream));
  HIP_TRY2(hipMemsetAsync(P.hkeys, 0xff, size_t(cap0) * 8, X.stream));
  // rank 0's own records: as gathered through RCCL in loopback mode, else the local copy
  HIP_TRY2(launch_merge_records(P, C.loopback ? parts : recs, n, agg, X.stream));
  for (int r = 1; r < C.world; r++)
    HIP_TRY2(launch_merge_records(P, parts + off[size_t(r)] / 8, sz[size_t(r)] / 48, agg, X.stream));
  cap = cap0;
}

// ---- shared host result blocks ----
namespace {
std::shared_ptr<ShmBlock> map_block(const std::string& name, size_t cap, bool create) {
  const int fd = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) return nullptr;
  auto b = std::make_shared<ShmBlock>();
  b->name = name;
  b->linked = create;
  if (create && ftruncate(fd, off_t(cap)) != 0) {
    close(fd);
    return nullptr;   // ~ShmBlock unlinks
  }
  void* p = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  void* d = nullptr;
  if (hipHostRegister(p, cap, hipHostRegisterMapped) != hipSuccess || hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipHostUnregister(p);
    (void)hipGetLastError();
    munmap(p, cap);
    return nullptr;
  }
  b->host = p;
  b->dev = d;
  b->cap = cap;
  return b;
}
}  // namespace

EmitTarget comm_emit_begin(Engine& E, CallCtx& X, size_t bytes) {
  Comm& C = need_comm(E);
  EmitTarget T;
  // rank 0 picks a free block of >= bytes (growing or adding one) and announces (pid, block, generation, size); a
  // pending failure of any rank travels with the announcement
  uint64_t hdr[5] = {0, 0, 0, 0, 0};   // ok, pid, block, gen, cap
  std::shared_ptr<void> lease;
  if (C.rank == 0) {
    comm_local(X, [&] {
      int pick = -1;
      for (auto& kv : C.shm)
        if (kv.second.lease.expired() && kv.second.cap() >= bytes) { pick = kv.first; break; }
      if (pick < 0)
        for (auto& kv : C.shm)
          if (kv.second.lease.expired()) { pick = kv.first; break; }
      if (pick < 0 && C.shm.size() < 8) pick = int(C.shm.size());
      if (pick < 0) return;
      ShmMap& m = C.shm[pick];
      if (!m.blk || m.cap() < bytes) {
        const size_t cap = std::max<size_t>((std::max(bytes, m.cap() * 3 / 2) + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1),
                                            size_t(2) << 20);
        m.release();
        const uint64_t gen = ++C.shm_gen;
        const std::string name = "/lakeside-" + std::to_string(getpid()) + "-" + std::to_string(pick) + "-" +
                                 std::to_string(gen);
        m.blk = map_block(name, cap, true);
        m.gen = gen;
      }
      if (!m.blk) return;
      auto l = std::make_shared<ShmLease>();
      l->blk = m.blk;
      lease = l;
      m.lease = lease;
      hdr[0] = 1;
      hdr[1] = uint64_t(getpid());
      hdr[2] = uint64_t(pick);
      hdr[3] = m.gen;
      hdr[4] = m.blk->cap;
    });
  }
  const std::vector<std::string> all =
      comm_allgather_status(E, X, 0, std::string(), std::string(reinterpret_cast<const char*>(hdr), sizeof(hdr)));
  if (all.empty() || all[0].size() < sizeof(hdr)) return T;
  memcpy(hdr, all[0].data(), sizeof(hdr));
  if (!hdr[0]) return T;   // no block on rank 0: every rank takes the gather path
  const int b = int(hdr[2]);
  ShmMap& m = C.shm[b];
  if (C.rank != 0 && fault_hit(E, "emit_map")) {   // tests only (LK_FAULT=emit_map@rank): the mapping fails
    m.release();
    m.gen = hdr[3];
  } else if (C.rank != 0 && (!m.blk || m.gen != hdr[3])) {
    m.release();
    const std::string name = "/lakeside-" + std::to_string(hdr[1]) + "-" + std::to_string(b) + "-" + std::to_string(hdr[3]);
    m.blk = map_block(name, size_t(hdr[4]), false);
    m.gen = hdr[3];
  }
  // a rank that could not map the block reports it with its rows (the caller's agreement fails the call everywhere)
  T.ok = true;   // uniform over the ranks: rank 0 offered a block
  T.mapped = m.blk != nullptr;
  T.host = m.blk ? static_cast<uint8_t*>(m.blk->host) : nullptr;
  T.dev = m.blk ? static_cast<uint8_t*>(m.blk->dev) : nullptr;
  T.cap = m.cap();
  T.lease = lease;
  T.block = b;
  T.gen = hdr[3];
  return T;
}

void comm_emit_end(Engine& E, const EmitTarget& T, bool agreed) {
  Comm& C = need_comm(E);
  if (C.rank != 0 || !T.ok) return;
  auto it = C.shm.find(T.block);
  if (it == C.shm.end() || !it->second.blk || it->second.gen != T.gen) return;
  if (agreed) {
    // every rank has mapped this call's block generation (the agreement follows their writes): its name can go.
    // Only this block: another block's generation may not have been mapped by every rank yet.
    it->second.blk->unlink();
  } else {
    // the emit agreement failed -- possibly because a rank could not map this generation: drop the block from the
    // pool, so the next call that needs one creates a new generation that every rank maps afresh, instead of
    // re-offering a name that may already be gone (the mapping itself lives on while a lease holds it)
    it->second.release();
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
  std::lock_guard<std::mutex> g(E.comm_init_mu);   // set once: concurrent inits cannot both pass the check
  if (E.comm) {
    lk::set_error("communicator already initialised");
    return LK_ERR_ARG;
  }
  if (hipSetDevice(E.device) != hipSuccess) return LK_ERR_DEVICE;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  auto* C = new lk::RcclComm();
  C->world = world;
  C->rank = rank;
  const char* lb = getenv("LK_COMM_LOOPBACK");
  C->loopback = world == 1 && lb && *lb == '1';
  ncclResult_t r = ncclCommInitRank(&C->comm, world, u, rank);
  if (r != ncclSuccess) {
    lk::set_error(std::string("RCCL: ncclCommInitRank: ") + ncclGetErrorString(r));
    delete C;
    return LK_ERR_DEVICE;
  }
  E.comm_desc = C->describe();
  E.comm = C;
  return LK_OK;
}

int lk_comm_init_host(lk_engine* e, int world, int rank, lk_allgather_fn fn, void* user) {
  if (!e || !fn || world < 1 || rank < 0 || rank >= world) return LK_ERR_ARG;
  lk::Engine& E = *e->e;
  std::lock_guard<std::mutex> g(E.comm_init_mu);
  if (E.comm) {
    lk::set_error("communicator already initialised");
    return LK_ERR_ARG;
  }
  auto* C = new lk::HostComm();
  C->world = world;
  C->rank = rank;
  C->fn = fn;
  C->user = user;
  E.comm_desc = C->describe();
  E.comm = C;
  return LK_OK;
}

}  // extern "C"
