// scan_lean<AGG, HASH>: the single-string-column scan (C2's shape: filter and group dim on `name` only) over the
// tiles where that column needs no general machinery.  Included by scan_inst.hpp; the general scan_tiles kernel
// skips these tiles (QParams.lean_split).
//
// A tile is "lean" when, over it, the timestamp, value and name columns hold no NULL (value index = row) and
// the name column's chunk dictionary has at most 64 entries packed in at most 6 bits.  Then the filter outcome is a
// function of the 6-bit code alone: a 64-bit mask of passing codes (one ballot over the chunk dictionary).
//
// Work unit: a 16-value chunk of one hybrid run (bit-packed chunks start on a byte boundary: 16 codes = 2*BW bytes),
// one chunk per thread per round, chunks of every useful run of the tile flattened into one index space (an RLE
// run of a failing code contributes no chunk at all).  Per chunk:
//   one 16-B buffer load of the packed codes -> a pass mask:  SWAR (BW = 1, 2, 4, at most 4 passing codes: per
//   32-bit word, xor with the code repeated, zero-field detect) or per code (a bit test of the pass mask);
//   the wave's passing rows are compacted into its LDS list and processed 128 per trip with every lane busy
//   (late-column lookups, late filter, value gather; NL = 0 COUNT and dense-code tiles keep a per-lane loop, two rows
//   per round trip) and accumulate into a per-thread register cell, spilling to an LDS table; the timestamp is
//   gathered only when neither the tile's zone map (one bucket) nor a split (sorted timestamps, bucket boundaries
//   found by search) gives the row's bucket; dense blocks (most rows pass) are read row-major with coalesced loads.
// No workgroup barrier in the main loop.  VALU per row is a fraction of scan_tiles' (which decodes every column
// generally and compacts rows through LDS).
#pragma once
#include <type_traits>

#include "device_common.hpp"

namespace lk {

constexpr int LEAN_H = HCAP / 2;                                 // LDS hash cells (hash mode)
constexpr uint32_t LEAN_CHUNKS = (TILE_ROWS / 16 + RUN_CAP + 1 + 7) & ~7u;   // chunks of a tile, upper bound (x4 B writes)
constexpr uint32_t LEAN_LINES = (TILE_ROWS * 8 / 128 + 2 + 31) / 32;   // plan bytes: line bitmap words
constexpr uint32_t LEAN_LLINES = (TILE_ROWS * 4 / 128 + 2 + 31) / 32;  // plan bytes: late stream lines (bw <= 32)
constexpr uint32_t LEAN_SPLIT_MAX = 4;   // split tiles: class boundaries (the tile's bucket span + 1) at most

#ifndef LK_LEAN_LIST
#define LK_LEAN_LIST 512
#endif
constexpr uint32_t LEAN_LIST = LK_LEAN_LIST;                           // per-wave list of passing rows (late columns)
#ifndef LK_LEAN_ROWS
#define LK_LEAN_ROWS 2
#endif
#ifndef LK_LEAN_WAVES2
#define LK_LEAN_WAVES2 4
#endif
#ifndef LK_LEAN_WAVES1
#define LK_LEAN_WAVES1 5
#endif
// NL = 0 with a value gather (C2): passing rows through the wave's LDS list too -- a trip of 128 rows with every lane
// busy per round trip -- instead of each lane looping over its own chunk's passing rows two at a time (a round then
// lasts as many round trips as its busiest lane); built for 4 waves per SIMD with 2 chunk rounds in flight: C2 1.27 ->
// 1.08 ms, C2 at a 10 s step 1.40 -> 1.18 ms (A/B: -DLK_LEAN_LIST0=0).  Dense-code tiles (a quarter or more of the
// codes pass: the dense query) keep the per-lane loop and its row-major dense blocks.
#ifndef LK_LEAN_LIST0
#define LK_LEAN_LIST0 1
#endif
#ifndef LK_LEAN_WAVES0V
#define LK_LEAN_WAVES0V 4
#endif
// one late column with a value gather (C4 / C5: SUM / MIN / MAX): 4 waves per SIMD and 3 chunk loads in flight measured
// faster than 5 waves with one (C4 1.59 -> 1.47 ms); COUNT(*) (tag queries, no gather) keeps 5 waves (A/B: -DLK_LEAN_WAVES1V)
#ifndef LK_LEAN_WAVES1V
#define LK_LEAN_WAVES1V 4
#endif
#ifndef LK_LEAN_PF1V
#define LK_LEAN_PF1V 3
#endif
// chunk loads in flight ahead of the round, by late-column count (A/B: -DLK_LEAN_PF0 / 1 / 2); the 5-wave shapes
// (NL <= 1, 96 VGPRs) keep their register budget, the 4-wave NL = 2 shape has room for a deeper ring
#ifndef LK_LEAN_PF0
#define LK_LEAN_PF0 (LK_LEAN_LIST0 ? 2 : 0)
#endif
#ifndef LK_LEAN_PF0E
#define LK_LEAN_PF0E 0   // NL = 0 dense-code shape (EARLY): chunk loads in the round itself
#endif
#ifndef LK_LEAN_PF0C
#define LK_LEAN_PF0C 2   // NL = 0 COUNT (no value gather): 0.857 -> 0.754 ms on `count` with 2 rounds in flight
#endif
#ifndef LK_LEAN_PF1
#define LK_LEAN_PF1 1
#endif
// unrotated chunk ring (A/B: -DLK_LEAN_SLOTS=0, the rotated ring of r02-r06): see the main loop
#ifndef LK_LEAN_SLOTS
#define LK_LEAN_SLOTS 1
#endif
// deferred trips of the late-column shapes (opt-in A/B: -DLK_LEAN_DEFER=1): see list_trip.  The pending trip's
// registers (rows, group terms, late words) live across the chunk rounds, so these shapes run a shallower chunk ring
// (LK_LEAN_PF1D / LK_LEAN_PF2D) and the COUNT(*) one 4 waves per SIMD (LK_LEAN_WAVES1D).  Measured (r06, validated):
// tag 0.970 -> 1.161 ms, C4 1.352 -> 1.357, C3 1.786 -> 1.784, with a 2-deep ring C4 1.409, C3 1.820 -- the other
// waves on the SIMD already hide the trip's first round trip, and the shallower ring / fewer waves cost more than
// the overlap buys (profiles/r06_ab_defer_*.json)
#ifndef LK_LEAN_DEFER
#define LK_LEAN_DEFER 0
#endif
#define LEAN_DEFER(NL, AGG) (LK_LEAN_DEFER && (NL) > 0)
#ifndef LK_LEAN_PF1D
#define LK_LEAN_PF1D 1
#endif
#ifndef LK_LEAN_PF2D
#define LK_LEAN_PF2D 1
#endif
#ifndef LK_LEAN_WAVES1D
#define LK_LEAN_WAVES1D 4
#endif
#ifndef LK_LEAN_PF2
#define LK_LEAN_PF2 3
#endif
// waves per SIMD the kernel is built for (A/B: -DLK_LEAN_WAVES1 / -DLK_LEAN_WAVES2)
#define LEAN_WAVES(NL, AGG) ((NL) == 0 ? ((AGG) == AGG_COUNT || !LK_LEAN_LIST0 ? LK_LEAN_WAVES1 : LK_LEAN_WAVES0V) \
                                      : (NL) == 1 ? ((AGG) == AGG_COUNT ? (LEAN_DEFER(NL, AGG) ? LK_LEAN_WAVES1D : LK_LEAN_WAVES1) \
                                                                        : LK_LEAN_WAVES1V) : LK_LEAN_WAVES2)
constexpr int LEAN_ROWS = LK_LEAN_ROWS;                                // listed rows per lane per trip (A/B: -DLK_LEAN_ROWS)
constexpr uint32_t LEAN_TRIP = 64u * LEAN_ROWS;                        // listed rows per trip
// the per-wave list is a ring indexed with & (LEAN_LIST - 1) and drained LEAN_TRIP rows at a time
static_assert((LEAN_LIST & (LEAN_LIST - 1u)) == 0u && LEAN_TRIP <= LEAN_LIST, "LK_LEAN_LIST / LK_LEAN_ROWS");

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

struct LeanRun {            // one run of the name column over the tile (24 B)
  uint32_t start;           // first value index (page-relative)
  uint32_t off_lit;         // bit 31: bit-packed; bits 0..30: byte offset in the value stream
  uint32_t value;           // RLE: the code
  uint32_t lo, hi;          // value range of the run inside the tile
  uint32_t cbk;             // chunk index of the run's chunk k = 0 (so k = q - cbk)
};

struct LeanHash {           // hash mode: the LDS hash table (lds_merge's layout)
  static constexpr int H = LEAN_H;
  unsigned long long hkey[H];
  uint32_t hrows[H];
  uint32_t hcnt[H];
  double hhi[H];
  double hlo[H];
  unsigned long long hval[1];
  uint32_t hfull;
};

template <int NL, bool LISTED_>
struct LeanLds {
  static constexpr int NLA = NL > 0 ? NL : 1;
  static constexpr uint32_t RW = lean_dir_words(NL);
  // per-wave list ring (a power of two >= LEAN_TRIP): half size with two late columns, whose direct table is larger
  static constexpr uint32_t LIST = NL >= 2 ? LEAN_LIST / 2 : LEAN_LIST;
  static_assert((LIST & (LIST - 1u)) == 0u && LEAN_TRIP <= LIST, "LeanLds::LIST");
  LeanRun runs[RUN_CAP];
  uint32_t cb[RUN_CAP + 1];               // first flattened chunk of each run (cb[nr] = chunks of the tile)
  alignas(4) uint8_t ctab[LEAN_CHUNKS];   // flattened chunk -> run (written 4 entries at a time)
  uint32_t lut[64];                       // code -> (leaf bits << 24) | dim id
  uint32_t etruth[(1u << (2 * TT_MAX_LEAVES)) / 32];   // the early conjuncts' truth table (staged with the lookups)
  // The tile's aggregation table: the hash table, or the direct table (the tile's buckets x ngroups cells, P.dir_planes
  // u64 planes: value (SUM: hi), SUM: lo, rows when the table keeps them)
  union {
    LeanHash hs;
    unsigned long long dir[RW];
  } agg;
  uint32_t lines_t[LEAN_LINES], lines_v[LEAN_LINES];   // plan bytes only: 128-B lines gathered
  uint32_t scnt[LEAN_SPLIT_MAX], sbnd[LEAN_SPLIT_MAX];  // split tiles: samples below each class, boundary rows
  // late columns (NL > 0): value runs (+ sentinel), run-block tables, lookup values, the late conjuncts' table
  LRun lruns[NLA][NL > 0 ? RUN_CAP + 1 : 1];
  alignas(4) uint8_t lrblk[NLA][NL > 0 ? TILE_ROWS / 64 + 8 : 1];
  uint32_t llut[NLA][NL > 0 ? LUT_CAP : 1];
  uint32_t ltruth[NL > 0 ? (1u << (2 * TT_MAX_LEAVES)) / 32 : 1];
  uint32_t lines_l[NLA][NL > 0 ? LEAN_LLINES : 1];     // plan bytes only: late stream lines gathered
  // the shapes that list their passing rows (NL > 0, and NL = 0 with a value gather outside the dense shape) hold a
  // per-wave ring; the COUNT and dense-code NL = 0 shapes, which never list, keep its 8 KB of LDS
  static constexpr bool LISTED = LISTED_;
  uint32_t wlist[LISTED ? BLOCK / 64 : 1][LISTED ? LIST : 1];   // each wave's passing rows
};

// (lean_tile, the test of a tile scan_lean takes, is in device_common.hpp: scan_tiles applies it too)

// Run of value v among `n` staged runs (+ sentinel) through a 64-value-block table (blk[b]: run holding vbase + 64b).
__device__ __forceinline__ int lean_find_run(const LRun* runs, const uint8_t* blk, uint32_t nb, uint32_t vbase,
                                             uint32_t v) {
  uint32_t b = (v - vbase) >> 6;
  b = b < nb ? b : nb - 1u;
  int lo = blk[b], hi = blk[b + 1];
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (runs[m].start <= v) lo = m;
    else hi = m - 1;
  }
  return lo;
}

// Code e (0..15) of a 16-code window of BW-bit fields held in w0..w2 (by value: no address-taken selects).
template <uint32_t BW>
__device__ __forceinline__ uint32_t lean_code(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t e) {
  const uint32_t bit = e * BW, wi = bit >> 5, off = bit & 31u;
  const uint32_t lo = wi == 0 ? w0 : (wi == 1 ? w1 : w2);
  const uint32_t hi = wi == 0 ? w1 : (wi == 1 ? w2 : 0u);
  return __builtin_amdgcn_alignbit(hi, lo, off) & ((1u << BW) - 1u);
}

// An RLE chunk's code v as 16 BW-bit fields in (w0, w1, w2) (the layout lean_code reads).
template <uint32_t BW>
__device__ __forceinline__ void lean_rep(uint32_t v, uint32_t& w0, uint32_t& w1, uint32_t& w2) {
  uint32_t w[3] = {0u, 0u, 0u};
#pragma unroll
  for (uint32_t e = 0; e < 16; e++) {
    const uint32_t bit = e * BW, wi = bit >> 5, off = bit & 31u;
    w[wi] |= v << off;
    if (off + BW > 32u) w[wi + 1] |= v >> (32u - off);
  }
  w0 = w[0];
  w1 = w[1];
  w2 = w[2];
}

// EARLY (NL > 0, a late filter leaf: P.late_chunk): tiles that allow it decode the late columns per chunk (early_late
// below); its own kernel, built for 4 waves per SIMD, so the other shapes keep their occupancy.
template <int AGG, bool HASH, int NL, bool EARLY = false>
// NL = 0 with EARLY (P.late_chunk set by the host when the filter passes a quarter or more of the name values: the
// dense query): the per-lane loop and row-major dense blocks at 5 waves per SIMD, the shape those tiles measured best in
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(EARLY ? (NL == 0 ? LK_LEAN_WAVES1 : 4) : LEAN_WAVES(NL, AGG)))) void scan_lean(QParams P) {
  using LT = LeanLds<NL, (NL > 0 || (LK_LEAN_LIST0 && AGG != AGG_COUNT && !EARLY))>;
  __shared__ LT L;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const QSeg* Sp = P.segs + blockIdx.y;
  const uint32_t t = blockIdx.x;
  if (t >= Sp->ntiles) return;
  const TileDesc* tdp = Sp->tiles + t;
  const int64_t win_lo = Sp->win_lo, win_hi = Sp->win_hi;
  if (tdp->ts_max < win_lo || tdp->ts_min >= win_hi) return;    // zone map: outside the glob window
  if (!lean_tile(Sp, t, NL, P.rows_only)) return;
  const TileCol* tc0 = Sp->cols[0].tcols + t;
  const TileCol* tc1 = Sp->cols[1].present ? Sp->cols[1].tcols + t : tc0;   // COUNT(*): never read
  const TileCol* tc2 = Sp->cols[2].tcols + t;
  const uint32_t nrows = tdp->nrows;
  const uint32_t nr = tc2->nruns, dict_n = tc2->dict_n, bw = tc2->bw;
  const uint32_t vb2 = tc2->vbase, vend = vb2 + nrows;
  const bool count_plan = P.plan_bytes != nullptr;
  const unsigned long long glob_base = (unsigned long long)Sp->glob_slot * P.nbuckets;
  uint64_t pbytes = 0;

  // ---- the tile's aggregation table ----
  // Direct table (P.dir_span > 0: a dense table whose group space fits LDS, and the tile's buckets -- zone map clipped
  // to the window -- number at most dir_span): cell (bucket - tbl) * ngroups + group, indexed without key or probe.
  // Otherwise the LDS hash table (lds_merge).
  int64_t tbl = 0;
  uint32_t tspan = 0;   // buckets of the direct table (0: hash table)
  if (!HASH && P.dir_span) {
    auto bucket_of = [&](int64_t ts) __attribute__((always_inline)) -> int64_t {   // monotone in ts
      if (P.metrics) return (ts - P.bucket_base) / P.step;
      return ((ts - ts % P.step) - P.bucket_base) / P.step;
    };
    const int64_t lo_ts = tdp->ts_min > win_lo ? tdp->ts_min : win_lo;
    const int64_t hi_ts = tdp->ts_max < win_hi - 1 ? tdp->ts_max : win_hi - 1;
    int64_t bl = bucket_of(lo_ts), bh = bucket_of(hi_ts);
    bl = bl < 0 ? 0 : bl;
    bh = bh >= int64_t(P.nbuckets) ? int64_t(P.nbuckets) - 1 : bh;
    if (bl <= bh && bh - bl < int64_t(P.dir_span)) {
      tbl = bl;
      tspan = uint32_t(bh - bl + 1);
    }
  }
  const uint32_t ngr = tspan ? uint32_t(P.ngroups) : 0u;
  // P.dir_rep replicas of every cell (a lane adds into replica lane % rep): lanes adding into the same few cells (the
  // dense query: 64 rows over 16 names) spread over rep times as many LDS addresses; combined at the flush
  const uint32_t rep = P.dir_rep ? P.dir_rep : 1u;
  const uint32_t myrep = uint32_t(lane) & (rep - 1u);
  const uint32_t ndir = tspan * ngr * rep;                          // direct cells (replicas included)
  unsigned long long* const rv = L.agg.dir;                         // value plane (SUM: hi)
  unsigned long long* const rlo = L.agg.dir + ndir;                 // SUM: lo plane
  const bool rrows_on = P.dir_planes > (AGG == AGG_SUM ? 2u : 1u);      // the table keeps rows: a rows plane
  unsigned long long* const rrows = L.agg.dir + (P.dir_planes - 1u) * ndir;
  // empty value: SUM's -0.0 marker (no rows plane: LEAN_SUM_EXISTS), the MIN / MAX identity, COUNT 0
  const unsigned long long rident = AGG == AGG_SUM ? (rrows_on ? 0ull : NEG_ZERO_BITS) : (AGG == AGG_MIN ? ~0ull : 0ull);
  constexpr unsigned long long GBIT = 1ull << 63;                   // register-cell key: a global cell, not a direct one
  if (tspan) {
    for (uint32_t x = tid; x < ndir; x += BLOCK) {
      rv[x] = rident;
      if (AGG == AGG_SUM) rlo[x] = 0ull;
      if (rrows_on) rrows[x] = 0ull;
    }
  } else {
    for (int i = tid; i < LeanHash::H; i += BLOCK) {
      L.agg.hs.hkey[i] = EMPTY;
      L.agg.hs.hrows[i] = 0;
      L.agg.hs.hcnt[i] = 0;
      L.agg.hs.hlo[i] = 0.0;
      if (AGG == AGG_MIN) reinterpret_cast<unsigned long long*>(L.agg.hs.hhi)[i] = ~0ull;
      else L.agg.hs.hhi[i] = 0.0;
    }
    if (tid == 0) L.agg.hs.hfull = 0u;
  }

  // ---- prologue: code lookup values ----
  {
    const uint32_t* remap = Sp->cols[2].remap + tc2->remap;
    const uint32_t* tab = P.strp[0].strtab;
    if (uint32_t(tid) < dict_n) {
      const uint32_t g = remap[tid];
      L.lut[tid] = tab ? tab[g] : g;
    }
  }
  if (tid < int(LEAN_SPLIT_MAX)) {
    L.scnt[tid] = 0u;
    L.sbnd[tid] = ~0u;
  }
  {   // staged beside the code lookups, so the pass ballot after the barrier waits on no global load
    const uint32_t* tt = NL > 0 ? P.truth_early : P.truth;
    const uint32_t words = ((1u << (2 * P.nleaves)) + 31) / 32;
    for (uint32_t i = tid; i < words; i += BLOCK) L.etruth[i] = tt[i];
  }
  if (count_plan) {
    for (uint32_t i = tid; i < LEAN_LINES; i += BLOCK) L.lines_t[i] = L.lines_v[i] = 0u;
#pragma unroll
    for (int k = 0; k < NL; k++)
      for (uint32_t i = tid; i < LEAN_LLINES; i += BLOCK) L.lines_l[k][i] = 0u;
  }
  __syncthreads();

  // passing codes: one ballot per wave over the chunk dictionary (Kleene: the leaves' T/F bits of the code)
  unsigned long long emask;
  {
    bool pass = false;
    if (uint32_t(lane) < dict_n) {
      const uint32_t lf = Sp->leaf_false;
      const uint32_t bits = (L.lut[lane] >> 24) << P.strp[0].lbase;
      const uint32_t lmask = P.strp[0].lmask;
      const uint32_t T = bits & lmask & ~lf, F = (~bits & lmask) | lf;
      const uint32_t ix = T | (F << P.nleaves);
      pass = (L.etruth[ix >> 5] >> (ix & 31)) & 1u;
    }
    emask = __ballot(pass);
  }
  if (!emask) return;   // no row of the tile passes (uniform: every thread leaves; nothing staged to flush)

  // late columns: runs, lookup values, the late conjuncts' truth table (run-block tables after the next barrier)
  const uint32_t nblk = (nrows + 63u) / 64u;
  uint32_t lpres = 0, llut_on = 0;          // bit k: late column k present / its lookup values in LDS
  uint32_t lnr[LT::NLA], lvb[LT::NLA], lbw[LT::NLA];
  __amdgpu_buffer_rsrc_t lrs[LT::NLA];
  const uint32_t* lremap[LT::NLA];
#pragma unroll
  for (int k = 0; k < NL; k++) {
    lnr[k] = lvb[k] = lbw[k] = 0;
    lremap[k] = nullptr;
    lrs[k] = make_rsrc(Sp->base, 0u);
    if (!Sp->cols[3 + k].present) continue;
    const TileCol* tl = Sp->cols[3 + k].tcols + t;
    lpres |= 1u << k;
    lnr[k] = tl->nruns;
    lvb[k] = tl->vbase;
    lbw[k] = tl->bw;
    lrs[k] = make_rsrc(Sp->base + tl->vals, tl->vals_len + 8u);
    lremap[k] = Sp->cols[3 + k].remap + tl->remap;
    const RunDesc* rr = Sp->cols[3 + k].runs + tl->run_lo;
    for (uint32_t i = tid; i < lnr[k]; i += BLOCK) {
      const RunDesc r = rr[i];
      L.lruns[k][i] = LRun{r.start, r.off_lit, r.value};
      if (i == lnr[k] - 1) L.lruns[k][lnr[k]] = LRun{r.start + r.count, 0u, 0u};
    }
    const uint32_t dn = tl->dict_n;
    if (dn <= LUT_CAP) {
      llut_on |= 1u << k;
      const uint32_t* tab = P.strp[1 + k].strtab;
      for (uint32_t i = tid; i < dn; i += BLOCK) {
        const uint32_t g = lremap[k][i];
        L.llut[k][i] = tab ? tab[g] : g;
      }
    }
    if (count_plan && tid == 0)
      pbytes += sizeof(TileCol) + uint64_t(lnr[k]) * sizeof(RunDesc) + ((llut_on >> k) & 1u ? uint64_t(dn) * 8u : 0u);
  }
  if (NL > 0) {
    const uint32_t words = ((1u << (2 * P.nleaves)) + 31) / 32;
    for (uint32_t i = tid; i < words; i += BLOCK) L.ltruth[i] = P.truth_late[i];
  }

  // runs of the tile: value range inside the tile, chunk counts (useful runs only)
  if (uint32_t(tid) < nr) {
    const RunDesc r = Sp->cols[2].runs[tc2->run_lo + tid];
    const uint32_t lo = r.start > vb2 ? r.start : vb2;
    const uint32_t hi = (r.start + r.count) < vend ? (r.start + r.count) : vend;
    const bool lit = (r.off_lit & 0x80000000u) != 0u;
    const bool useful = lo < hi && (lit || ((emask >> (r.value & 63u)) & 1ull));
    const uint32_t k0 = useful ? (lo - r.start) >> 4 : 0u, k1 = useful ? (hi - r.start + 15u) >> 4 : 0u;
    L.runs[tid] = LeanRun{r.start, r.off_lit, r.value, lo, hi, k0};
    L.cb[tid] = k1 - k0;
    if (count_plan && lit && lo < hi) pbytes += (uint64_t(hi - lo) * bw + 7u) / 8u;   // codes decoded in full
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NL; k++)   // run-block tables of the late columns (runs staged above)
    if ((lpres >> k) & 1u)
      for (uint32_t b0 = 4u * uint32_t(tid); b0 <= nblk; b0 += 4u * BLOCK) {   // 4 blocks per thread: one search
        uint32_t lo = 0;
        const uint32_t v = lvb[k] + 64u * b0;
#pragma unroll
        for (uint32_t st = RUN_CAP / 2; st >= 1; st >>= 1) {
          const uint32_t m = lo + st;
          lo = (m < lnr[k] && L.lruns[k][m].start <= v) ? m : lo;
        }
        uint32_t word = lo;
#pragma unroll
        for (uint32_t i = 1; i < 4; i++) {
          while (lo + 1u < lnr[k] && L.lruns[k][lo + 1u].start <= v + 64u * i) lo++;
          word |= lo << (8u * i);
        }
        *reinterpret_cast<uint32_t*>(&L.lrblk[k][b0]) = word;
      }
  if (tid < 64) {   // exclusive prefix of the chunk counts (<= 128 runs: two per lane)
    const uint32_t i0 = 2u * uint32_t(lane), i1 = i0 + 1u;
    const uint32_t n0 = i0 < nr ? L.cb[i0] : 0u, n1 = i1 < nr ? L.cb[i1] : 0u;
    uint32_t s = n0 + n1, inc = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d, 64);
      if (lane >= d) inc += o;
    }
    const uint32_t ex = inc - s;
    const uint32_t tot = __shfl(inc, 63, 64);
    if (i0 < nr) {
      L.runs[i0].cbk = ex - L.runs[i0].cbk;
      L.cb[i0] = ex;
    }
    if (i1 < nr) {
      L.runs[i1].cbk = ex + n0 - L.runs[i1].cbk;
      L.cb[i1] = ex + n0;
    }
    if (lane == 0) L.cb[nr] = tot;
  }
  __syncthreads();
  const uint32_t total = L.cb[nr];   // chunks of the tile
  // chunk -> run: the last run whose first chunk <= q; 4 chunks per thread (one search, then runs advanced in order)
  for (uint32_t q = 4u * uint32_t(tid); q < total; q += 4u * BLOCK) {
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t st = RUN_CAP / 2; st >= 1; st >>= 1) {
      const uint32_t m = lo + st;
      lo = (m < nr && L.cb[m] <= q) ? m : lo;
    }
    uint32_t word = lo;
#pragma unroll
    for (uint32_t i = 1; i < 4; i++) {
      while (lo + 1u < nr && L.cb[lo + 1u] <= q + i) lo++;
      word |= lo << (8u * i);
    }
    *reinterpret_cast<uint32_t*>(&L.ctab[q]) = word;
  }
  __syncthreads();

  if (P.ablate & 0x80000u) return;   // diagnostics only: the tile prologue alone (uniform)

  // ---- per-row state ----
  const uint32_t vb0 = tc0->vbase, vb1 = tc1->vbase;
  const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(Sp->base + tc0->vals, tc0->vals_len);
  const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(Sp->base + tc1->vals, tc1->vals_len);
  const __amdgpu_buffer_rsrc_t rs2 = make_rsrc(Sp->base + tc2->vals, tc2->vals_len + 16u);
  const uint32_t line_t0 = (vb0 * 8u) >> 7, line_v0 = (vb1 * 8u) >> 7;
  const uint32_t stride = P.strp[0].dim_stride;
  const uint32_t npass = uint32_t(__popcll(emask));
  const uint32_t code0 = uint32_t(__builtin_ctzll(emask));
  const uint32_t dim_u = (L.lut[code0] & DIM_MASK) * stride;   // the only passing code's group term
  int64_t tile_b = -1;                                         // zone map: every row in one bucket
  {
    const int64_t tmin = tdp->ts_min, tmax = tdp->ts_max;
    if (tmin >= win_lo && tmax < win_hi) {
      if (P.metrics) {
        if (tmin == tmax && (tmin - P.bucket_base) % P.step == 0) tile_b = (tmin - P.bucket_base) / P.step;
      } else {
        const int64_t b0 = ((tmin - tmin % P.step) - P.bucket_base) / P.step;
        const int64_t b1 = ((tmax - tmax % P.step) - P.bucket_base) / P.step;
        if (b0 == b1) tile_b = b0;
      }
      if (tile_b >= int64_t(P.nbuckets)) tile_b = -1;
    }
  }
  const bool one_bucket = tile_b >= 0;
  const uint32_t step32 = uint32_t(P.step);
  // Split tiles (TILE_TS_SORTED: the tile's timestamps never decrease; not metrics, whose rows must be checked on the
  // step grid): a tile the zone map cannot pin to one bucket has its rows' classes -- 0 before the window, 1 .. span
  // its buckets split_bl .. split_bl + span - 1, span + 1 after the window, non-decreasing with the row -- split by
  // boundary rows found with two rounds of timestamp loads (256 samples, then the sample gap holding each boundary),
  // so a passing row's bucket follows from its row index and no timestamp is gathered per row.
  uint32_t nsb = 0;        // boundaries (span + 1; 0: not a split tile) -- uniform
  int64_t split_bl = 0;
  uint32_t sb[LEAN_SPLIT_MAX];
#pragma unroll
  for (uint32_t k = 0; k < LEAN_SPLIT_MAX; k++) sb[k] = 0u;
  // (not built into the COUNT(*) late-column shape: tag queries have one bucket, and its 5-wave budget has no room)
  constexpr bool SPLIT = !(AGG == AGG_COUNT && NL >= 1);
  if (SPLIT && !one_bucket && !P.metrics && (tdp->pad & TILE_TS_SORTED) && P.split_ok) {
    auto bucket_of = [&](int64_t ts) __attribute__((always_inline)) -> int64_t {
      return ((ts - ts % P.step) - P.bucket_base) / P.step;
    };
    const int64_t lo_ts = tdp->ts_min > win_lo ? tdp->ts_min : win_lo;
    const int64_t hi_ts = tdp->ts_max < win_hi - 1 ? tdp->ts_max : win_hi - 1;
    const int64_t bl = bucket_of(lo_ts), bh = bucket_of(hi_ts);
    if (lo_ts <= hi_ts && bl >= 0 && bh < int64_t(P.nbuckets) && bh - bl + 2 <= int64_t(LEAN_SPLIT_MAX)) {
      nsb = uint32_t(bh - bl + 2);
      split_bl = bl;
    }
  }
  if (nsb) {   // uniform
    const __amdgpu_buffer_rsrc_t rst = make_rsrc(Sp->base + tc0->vals, tc0->vals_len);
    const uint32_t vbt = tc0->vbase;
    auto cls_of = [&](int64_t ts) __attribute__((always_inline)) -> uint32_t {
      if (ts < win_lo) return 0u;
      if (ts >= win_hi) return nsb;
      return uint32_t(((ts - ts % P.step) - P.bucket_base) / P.step - split_bl) + 1u;
    };
    auto sample = [&](uint32_t t) __attribute__((always_inline)) -> uint32_t {   // row of sample t (t = 256: nrows)
      return uint32_t((uint64_t(t) * nrows) >> 8);
    };
    {   // round 1: samples; per class c, the samples below it
      const v2u x = __builtin_amdgcn_raw_buffer_load_b64(rst, (vbt + sample(uint32_t(tid))) * 8u, 0, 0);
      const uint32_t c = cls_of(int64_t(((uint64_t)x.y << 32) | x.x));
#pragma unroll
      for (uint32_t k = 0; k < LEAN_SPLIT_MAX; k++) {
        if (k >= nsb) break;
        const unsigned long long bl = __ballot(c < k + 1u);
        if (lane == 0 && bl) atomicAdd(&L.scnt[k], uint32_t(__popcll(bl)));
      }
    }
    __syncthreads();
    // round 2: boundary k + 1 lies in the sample gap (sample(n - 1), sample(n)] (n samples below it; none: row 0)
#pragma unroll
    for (uint32_t k = 0; k < LEAN_SPLIT_MAX; k++) {
      if (k >= nsb) break;
      const uint32_t n = L.scnt[k];
      if (n == 0u) continue;   // uniform
      const uint32_t lo = sample(n - 1u) + 1u, hi = sample(n);
      const uint32_t r = lo + uint32_t(tid);
      bool f = false;
      if (r < hi) {
        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(rst, (vbt + r) * 8u, 0, 0);
        f = cls_of(int64_t(((uint64_t)x.y << 32) | x.x)) >= k + 1u;
      }
      const unsigned long long bl = __ballot(f);
      if (lane == 0 && bl) atomicMin(&L.sbnd[k], r - uint32_t(lane) + uint32_t(__builtin_ctzll(bl)));
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < LEAN_SPLIT_MAX; k++) {
      const uint32_t n = L.scnt[k];
      const uint32_t hi = sample(n);   // the first sample at or above the class (n = 256: nrows, no such row)
      const uint32_t b = n == 0u ? 0u : (L.sbnd[k] < hi ? L.sbnd[k] : hi);
      sb[k] = k < nsb ? uint32_t(__builtin_amdgcn_readfirstlane(int(b))) : 0xffffffffu;
    }
    if (count_plan && tid == 0) pbytes += 128u * (256u / 16u + nsb * 2u);   // sample and gap lines (approx.)
  }
  const bool split = nsb != 0u;
  const bool ts_gather = !one_bucket && !split;   // rows gather their timestamp (uniform)
  auto split_class = [&](uint32_t r) __attribute__((always_inline)) -> uint32_t {
    uint32_t c = 0;
#pragma unroll
    for (uint32_t k = 0; k < LEAN_SPLIT_MAX; k++) c += r >= sb[k] ? 1u : 0u;
    return c;
  };
  // dense-block test only where a quarter or more of the chunk dictionary's codes pass (uniform; C2's 1 of 16 skips it)
  const bool dense_codes = NL == 0 && 4u * npass >= dict_n;
  // dense blocks over several passing codes: rows straight into the direct table (`row`'s `direct`)
  const bool dense_direct = dense_codes && npass > 1 && !(P.lean & LEAN_NO_DENSE_DIRECT);
  bool late_trivial = true;   // no filter leaf on a late column: the late stage only adds group terms (uniform)
#pragma unroll
  for (int k = 0; k < NL; k++) late_trivial = late_trivial && P.strp[1 + k].lmask == 0u;
  // Late columns decoded per chunk (uniform): every present late column has its lookup values in LDS and <= 7-bit
  // codes (16 codes + the window's bit offset fit one 20-B load), and the group space fits the list entry's high 16
  // bits.  The chunk's late codes are then loaded one round ahead with its name codes, the late filter runs before
  // the list, and a listed row waits only on its value gather -- one memory round trip per trip instead of two.
  bool early_late = false;
  if constexpr (NL > 0 && EARLY) {
    early_late = P.ngroups <= 65536u;
#pragma unroll
    for (int k = 0; k < NL; k++)
      if ((lpres >> k) & 1u) early_late = early_late && ((llut_on >> k) & 1u) && lbw[k] <= 7u;
  }
  // early_late COUNT(*) tiles inside one bucket of the direct table (tag queries): rows counted in the chunk loop
  const bool direct_count = early_late && AGG == AGG_COUNT && P.rows_only && one_bucket && tspan && !P.nvl &&
                            uint64_t(tile_b - tbl) < uint64_t(tspan);

  Acc acc;
  acc_reset<AGG>(acc, EMPTY);
  // a register cell into the tile's table: its direct cell (LDS atomics), HBM (a bucket beyond the direct table's
  // span), or the LDS hash table
  auto flush = [&]() __attribute__((always_inline)) {
    if (acc.rows == 0) return;
    if (!tspan && P.global_cells) {   // (uniform) a group space far beyond the LDS table: straight to HBM
      global_merge<AGG, HASH>(P, acc.key, acc.rows, acc.cnt, acc.hi, acc.lo, acc.ext);
    } else if (!tspan) {
      lds_merge<AGG, HASH, false>(L.agg.hs, P, acc);
    } else if (acc.key & GBIT) {
      global_merge<AGG, HASH>(P, acc.key & ~GBIT, acc.rows, acc.cnt, acc.hi, acc.lo, acc.ext);
    } else {
      const uint32_t x = uint32_t(acc.key);
      if (AGG == AGG_SUM) {
        const double h = acc.hi + 0.0;   // never -0.0 (the empty marker)
        if (P.exact_sum) {   // exact adds: nothing to compensate
          __hip_atomic_fetch_add(reinterpret_cast<double*>(rv + x), h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          const double old = atomicAdd(reinterpret_cast<double*>(rv + x), h);
          double s, e;
          two_sum(old, h, s, e);
          const double c = acc.lo + e;
          if (c != 0.0) atomicAdd(reinterpret_cast<double*>(rlo + x), c);
        }
      } else if (AGG == AGG_MIN) {
        atomicMin(rv + x, acc.ext);
      } else if (AGG == AGG_MAX) {
        atomicMax(rv + x, acc.ext);
      } else {
        atomicAdd(rv + x, (unsigned long long)acc.rows);
      }
      if (rrows_on) atomicAdd(rrows + x, (unsigned long long)acc.rows);
    }
  };
  // one passing row: bucket (BaseExpr.scala:159-165 window, 163-165 / 376-394 bucket), cell, register cell
  auto row = [&](int64_t ts, double v, uint32_t dim, uint32_t r) __attribute__((always_inline)) {
    if (P.nvl) {   // numeric leaves on the value column (uniform)
      uint32_t bits = 0;
      // read through the kernarg segment pointer (P is the kernel's only argument): a runtime index into the by-value
      // argument would copy it to scratch, and an unrolled loop holds every leaf's bounds in SGPRs
      const VLeaf* vls = static_cast<const QParams*>((const void*)__builtin_amdgcn_kernarg_segment_ptr())->vl;
#pragma unroll 1
      for (uint32_t k = 0; k < P.nvl; k++) {
        const VLeaf vl = vls[k];
        const bool pass = v != v ? vl.nan_pass != 0u
                                 : ((v > vl.lo || (vl.lo_incl && v == vl.lo)) && (v < vl.hi || (vl.hi_incl && v == vl.hi)));
        bits |= uint32_t(pass) << k;
      }
      if (!((P.vtab >> bits) & 1u)) return;
    }
    bool ok = true;
    int64_t b = tile_b;
    if (split) {   // uniform: the row's class from its index
      const uint32_t c = split_class(r);
      if (c == 0u || c >= nsb) return;   // outside the window
      b = split_bl + int64_t(c) - 1;
    } else if (!one_bucket) {
      ok = ts >= win_lo && ts < win_hi;
      if (P.fast_div) {
        const uint32_t d = uint32_t(ts - P.bucket_base);
        uint32_t qd = uint32_t(double(d) * P.inv_step);
        int64_t rm = int64_t(d) - int64_t(qd) * step32;
        qd = rm < 0 ? qd - 1 : (rm >= int64_t(step32) ? qd + 1 : qd);
        rm = int64_t(d) - int64_t(qd) * step32;
        if (P.metrics && rm != 0 && ok) {
          atomicOr(P.flags, FLAG_METRICS_UNALIGNED);
          ok = false;
        }
        b = qd;
      } else if (ok) {
        if (P.metrics) {
          const int64_t d = ts - P.bucket_base;
          b = d / P.step;
          if (d - b * P.step != 0) {
            atomicOr(P.flags, FLAG_METRICS_UNALIGNED);
            ok = false;
          }
        } else {
          b = ((ts - ts % P.step) - P.bucket_base) / P.step;
        }
      }
      if (!ok) return;
      if (b < 0 || (uint64_t)b >= P.nbuckets) {
        atomicOr(P.flags, FLAG_CELL_RANGE);
        return;
      }
    }
    unsigned long long cell;
    const uint64_t j = uint64_t(b - tbl);
    if (tspan && j < tspan) {
      cell = (uint32_t(j) * ngr + dim) * rep + myrep;
    } else {
      cell = (glob_base + (unsigned long long)b) * P.ngroups + dim;
      if (tspan) cell |= GBIT;
    }
    if (cell != acc.key) {
      flush();
      acc_reset<AGG>(acc, cell);
    }
    min_nan_check<AGG>(P, true, v);
    acc_add<AGG>(acc, true, v);
  };

  // The late-column loads of N rows per lane (rr[u] live when aa[u]): run lookup + packed word lw[u][k], its bit
  // offset / RLE code lm[u][k]; all N rows' loads in flight together
  auto late_issue = [&](auto ncst, const uint32_t* rr, const bool* aa, auto& lw, auto& lm) __attribute__((always_inline)) {
    constexpr int N = decltype(ncst)::value;
#pragma unroll
    for (int k = 0; k < NL; k++) {
#pragma unroll
      for (int u = 0; u < N; u++) {
        lw[u][k] = v2u{0u, 0u};
        lm[u][k] = 0u;
      }
      if (!((lpres >> k) & 1u)) continue;   // uniform
#pragma unroll
      for (int u = 0; u < N; u++) {
        const uint32_t v = lvb[k] + rr[u];
        const int ri = lnr[k] == 1u ? 0 : lean_find_run(L.lruns[k], L.lrblk[k], nblk, lvb[k], v);
        const LRun lr = L.lruns[k][ri];
        const bool lt = (lr.off_lit & 0x80000000u) != 0u;
        const uint32_t bit = (v - lr.start) * lbw[k];
        const uint32_t byte = (lr.off_lit & 0x7fffffffu) + (bit >> 3);
        lw[u][k] = __builtin_amdgcn_raw_buffer_load_b64(lrs[k], (aa[u] && lt) ? (byte & ~3u) : OOB, 0, 0);
        lm[u][k] = lt ? (0x80000000u | ((byte & 3u) * 8u + (bit & 7u))) : lr.value;
        if (count_plan && aa[u] && lt) {   // distinct 128-B lines of the late stream gathered
          const uint32_t l = ((byte & ~3u) >> 7) - ((L.lruns[k][0].off_lit & 0x7fffffffu) >> 7);
          if (l < LEAN_LLINES * 32u) atomicOr(&L.lines_l[k][l >> 5], 1u << (l & 31u));
        }
      }
    }
  };
  // N rows per lane (rr[u] live when aa[u]) with group terms dd[u] and their late-column words lw / lm (late_issue,
  // issued by the caller): late filter, timestamp / value gather, accumulate
  auto rowsN = [&](auto ncst, auto ldc, const uint32_t* rr, const bool* aa, uint32_t* dd, auto& lw, auto& lm) __attribute__((always_inline)) {
    constexpr int N = decltype(ncst)::value;
    constexpr bool LATE_DONE = decltype(ldc)::value;   // late columns decoded already (dd complete): values only
    bool p[N], ld[N];   // ld: rows whose timestamp / value loads were issued (plan bytes)
    v2u tt[N], xx[N];
#pragma unroll
    for (int u = 0; u < N; u++) {
      p[u] = aa[u];
      ld[u] = aa[u];
      tt[u] = xx[u] = v2u{0u, 0u};
    }
    auto gather = [&]() __attribute__((always_inline)) {   // timestamps / values of the passing rows
#pragma unroll
      for (int u = 0; u < N; u++) {
        if (ts_gather) tt[u] = __builtin_amdgcn_raw_buffer_load_b64(rs0, p[u] ? (vb0 + rr[u]) * 8u : OOB, 0, 0);
        if (AGG != AGG_COUNT || P.nvl) xx[u] = __builtin_amdgcn_raw_buffer_load_b64(rs1, p[u] ? (vb1 + rr[u]) * 8u : OOB, 0, 0);
      }
    };
    if constexpr (NL > 0 && !LATE_DONE) {
      // with no late filter leaf every row passes, so the timestamp / value loads go out with the late-column words
      // speculative gather (P.spec_gather): with a late filter, every listed row's timestamp / value loads go out now,
      // with its late-column loads, instead of after the late filter -- one dependent memory round trip less per trip
      // for the loads of the rows the filter then drops
      const bool spec = !late_trivial && P.spec_gather;
      if (late_trivial || spec) gather();
      uint32_t T[N], F[N];
#pragma unroll
      for (int u = 0; u < N; u++) T[u] = F[u] = 0u;
#pragma unroll
      for (int k = 0; k < NL; k++) {
        const StrParam sp = P.strp[1 + k];
        if (!((lpres >> k) & 1u)) {   // absent column: NULL in every row
#pragma unroll
          for (int u = 0; u < N; u++) {
            dd[u] += sp.dim_null * sp.dim_stride;
            F[u] |= sp.hmask;
          }
          continue;
        }
        const uint32_t bwk = lbw[k];
        const uint32_t msk = bwk >= 32u ? ~0u : ((1u << bwk) - 1u);
#pragma unroll
        for (int u = 0; u < N; u++) {
          const uint64_t x = ((uint64_t)lw[u][k].y << 32) | lw[u][k].x;
          const uint32_t meta = lm[u][k];
          const uint32_t idx = (meta >> 31) ? uint32_t(x >> (meta & 63u)) & msk : meta;
          uint32_t packed;
          if ((llut_on >> k) & 1u) {
            packed = L.llut[k][idx < LUT_CAP ? idx : 0u];
          } else {
            const uint32_t g = aa[u] ? lremap[k][idx] : 0u;
            packed = sp.strtab ? sp.strtab[g] : g;
          }
          const uint32_t bits = (packed >> 24) << sp.lbase;
          dd[u] += (packed & DIM_MASK) * sp.dim_stride;
          T[u] |= bits & sp.lmask;
          F[u] |= ~bits & sp.lmask;
        }
      }
      if (!late_trivial) {
        const uint32_t lf = Sp->leaf_false;
#pragma unroll
        for (int u = 0; u < N; u++) {
          const uint32_t ix = (T[u] & ~lf) | ((F[u] | lf) << P.nleaves);
          p[u] = aa[u] && ((L.ltruth[ix >> 5] >> (ix & 31)) & 1u);
          if (!spec) ld[u] = p[u];
        }
        if (!spec) gather();
      }
    } else {
      gather();
    }
    if (count_plan) {
      auto mark = [&](uint32_t* bm, uint32_t off, uint32_t line0) __attribute__((always_inline)) {
        const uint32_t l = (off >> 7) - line0;
        atomicOr(&bm[l >> 5], 1u << (l & 31u));
      };
#pragma unroll
      for (int u = 0; u < N; u++) {
        if (!ld[u]) continue;
        if (ts_gather) mark(L.lines_t, (vb0 + rr[u]) * 8u, line_t0);
        if (AGG != AGG_COUNT || P.nvl) mark(L.lines_v, (vb1 + rr[u]) * 8u, line_v0);
      }
    }
    if (P.ablate & 0x40000u) {   // diagnostics only: nothing accumulated (the loads' cost without the table updates)
#pragma unroll
      for (int u = 0; u < N; u++) p[u] = p[u] && (tt[u].x ^ xx[u].x ^ dd[u]) == 0x9e3779b9u;
    }
#pragma unroll
    for (int u = 0; u < N; u++)
      if (p[u])
        row((int64_t)(((uint64_t)tt[u].y << 32) | tt[u].x), __longlong_as_double((long long)(((uint64_t)xx[u].y << 32) | xx[u].x)), dd[u], rr[u]);
  };
  // Late columns: each wave's passing rows wait in its LDS list (a ring of LEAN_LIST entries, tile row | code << 16)
  // until a full trip of LEAN_TRIP rows -- LEAN_ROWS per lane, every lane busy, all their late-column loads and then
  // all their value loads in flight together -- is ready, across the tile's rounds; the rest drains at the tile's end.
  uint32_t lhead = 0, ltail = 0;   // wave-uniform list positions (mod LEAN_LIST)
  uint32_t* const wl = L.wlist[LT::LISTED ? (tid >> 6) : 0];
  // Deferred trips (LK_LEAN_DEFER, the late-column shapes outside early_late): a trip's late-column words are issued
  // and the trip is finished (decode, late filter, value gather, accumulate) only at the next trip or the tile's end,
  // so its first memory round trip overlaps the chunk rounds in between instead of being waited for on the spot.
  // Needs the unrotated chunk ring (a rotated ring's latch waits for every load in flight, the trip's included).
  uint32_t prr[LEAN_ROWS], pdd[LEAN_ROWS];
  bool paa[LEAN_ROWS];
  v2u plw[LEAN_ROWS][LT::NLA];
  uint32_t plm[LEAN_ROWS][LT::NLA];
  bool pend = false;   // (uniform) a deferred trip is in flight
  auto list_trip = [&](auto ec, uint32_t n) __attribute__((always_inline)) {   // the n (<= LEAN_TRIP) rows at lhead
    constexpr bool ELIST = decltype(ec)::value;   // entries carry complete group terms (early_late)
    constexpr bool DEFER = LEAN_DEFER(NL, AGG) && !ELIST;
    if (P.ablate & 0x20000u) {   // diagnostics only: listed rows dropped unprocessed (the trips' cost)
      lhead += n;
      return;
    }
    uint32_t rr[LEAN_ROWS], dd[LEAN_ROWS];
    bool aa[LEAN_ROWS];
    if constexpr (DEFER) {
      if (pend) rowsN(std::integral_constant<int, LEAN_ROWS>{}, ec, prr, paa, pdd, plw, plm);   // the previous trip
    }
#pragma unroll
    for (int u = 0; u < LEAN_ROWS; u++) {
      const uint32_t i = uint32_t(lane) + 64u * uint32_t(u);
      aa[u] = i < n;
      const uint32_t x = aa[u] ? wl[(lhead + i) & (LT::LIST - 1u)] : 0u;
      rr[u] = x & 0xffffu;
      dd[u] = ELIST ? (x >> 16) : (npass > 1 ? (L.lut[x >> 16] & DIM_MASK) * stride : dim_u);
    }
    if constexpr (DEFER) {
      late_issue(std::integral_constant<int, LEAN_ROWS>{}, rr, aa, plw, plm);
#pragma unroll
      for (int u = 0; u < LEAN_ROWS; u++) {
        prr[u] = rr[u];
        paa[u] = aa[u];
        pdd[u] = dd[u];
      }
      pend = true;
    } else {
      v2u lw[LEAN_ROWS][LT::NLA];
      uint32_t lm[LEAN_ROWS][LT::NLA];
      if constexpr (NL > 0 && !ELIST) late_issue(std::integral_constant<int, LEAN_ROWS>{}, rr, aa, lw, lm);
      rowsN(std::integral_constant<int, LEAN_ROWS>{}, ec, rr, aa, dd, lw, lm);
    }
    lhead += n;
  };
  auto wave_sync = [&]() __attribute__((always_inline)) {   // the wave's list writes / reads are ordered
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  auto body = [&](auto bwc, auto ec) __attribute__((always_inline)) {
    constexpr uint32_t BW = decltype(bwc)::value;
    constexpr bool ECH = NL > 0 && decltype(ec)::value;   // early_late tile (its own body instantiation)
    constexpr bool POW2 = BW == 1 || BW == 2 || BW == 4;
    // SWAR filter: BW | 32, at most 4 passing codes (uniform)
    const bool swar = POW2 && npass <= 4;
    constexpr uint32_t REP = BW == 1 ? 0xffffffffu : BW == 2 ? 0x55555555u : 0x11111111u;   // 1 per field
    constexpr uint32_t HI = BW == 1 ? 0xffffffffu : BW == 2 ? 0xaaaaaaaau : 0x88888888u;    // field high bits
    uint32_t pc[4];
    {
      unsigned long long em = emask;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        pc[j] = em ? uint32_t(__builtin_ctzll(em)) : 0xffffffffu;
        em &= em ? em - 1 : 0ull;
      }
    }
    // The packed codes of the next PF rounds are in flight while a round runs (a register ring; loads return in issue
    // order, so a round waits only for its own chunk): a round's own work is far shorter than a memory round trip, and
    // one load per lane in flight would leave the tile's stream latency-bound (PF = 0: loaded in the round itself).
    constexpr int PF = NL == 0 ? (EARLY ? LK_LEAN_PF0E : AGG == AGG_COUNT ? LK_LEAN_PF0C : LK_LEAN_PF0)
                               : (NL == 1 ? (AGG == AGG_COUNT ? LK_LEAN_PF1 : (LEAN_DEFER(NL, AGG) ? LK_LEAN_PF1D : LK_LEAN_PF1V))
                                          : (LEAN_DEFER(NL, AGG) ? LK_LEAN_PF2D : LK_LEAN_PF2));
    auto chunk_load = [&](uint32_t qq) __attribute__((always_inline)) {
      const bool lv = qq < total;
      const LeanRun Rn = L.runs[lv ? L.ctab[qq] : 0u];
      const uint32_t bn = (Rn.off_lit & 0x7fffffffu) + 2u * BW * (qq - Rn.cbk);
      return __builtin_amdgcn_raw_buffer_load_b128(rs2, (lv && (Rn.off_lit & 0x80000000u)) ? (bn & ~3u) : OOB, 0, 0);
    };
    v4u xr[PF > 0 ? PF : 1];
#pragma unroll
    for (int i = 0; i < PF; i++) xr[i] = chunk_load(uint32_t(tid) + uint32_t(i) * BLOCK);
    // early_late: chunk qq's late codes -- one 20-B window per late column over the late values of its valid rows
    // (meta: bit 31 a bit-packed window, bits 0..7 its bit offset; bit 30 the rows straddle a run boundary: decoded
    // row by row; else the RLE run's code)
    struct LWin {
      v4u x;
      uint32_t x4, meta;
    };
    LWin lpre[LT::NLA];
    auto late_load = [&](uint32_t qq) __attribute__((always_inline)) {
      const bool lv = qq < total;
      const LeanRun Rn = L.runs[lv ? L.ctab[qq] : 0u];
      const uint32_t v0n = Rn.start + 16u * (qq - Rn.cbk);
      const uint32_t an = (Rn.lo > v0n ? Rn.lo : v0n) - v0n;
      const uint32_t bn = ((Rn.hi < v0n + 16u) ? Rn.hi : v0n + 16u) - v0n;
#pragma unroll
      for (int k = 0; k < NL; k++) {
        lpre[k] = LWin{v4u{0u, 0u, 0u, 0u}, 0u, 0x40000000u};
        if (!((lpres >> k) & 1u) || !lv || an >= bn) continue;
        const uint32_t v = lvb[k] + (v0n + an - vb2);   // late value of the chunk's first valid row (no NULLs)
        const int ri = lnr[k] == 1u ? 0 : lean_find_run(L.lruns[k], L.lrblk[k], nblk, lvb[k], v);
        const LRun lr = L.lruns[k][ri];
        if (v + (bn - an) > L.lruns[k][ri + 1].start) continue;   // straddles a run boundary (sentinel at lnr)
        if (!(lr.off_lit & 0x80000000u)) {
          lpre[k].meta = lr.value;
          continue;
        }
        const uint32_t bit = (v - lr.start) * lbw[k];
        const uint32_t byte = (lr.off_lit & 0x7fffffffu) + (bit >> 3);
        lpre[k].x = __builtin_amdgcn_raw_buffer_load_b128(lrs[k], byte & ~3u, 0, 0);
        lpre[k].x4 = __builtin_amdgcn_raw_buffer_load_b32(lrs[k], (byte & ~3u) + 16u, 0, 0);
        lpre[k].meta = 0x80000000u | ((byte & 3u) * 8u + (bit & 7u));
        if (count_plan) {   // distinct 128-B lines of the late stream read
          const uint32_t l0 = ((L.lruns[k][0].off_lit & 0x7fffffffu) >> 7);
          const uint32_t la = ((byte & ~3u) >> 7) - l0, lb = (((byte & ~3u) + 19u) >> 7) - l0;
          if (la < LEAN_LLINES * 32u) atomicOr(&L.lines_l[k][la >> 5], 1u << (la & 31u));
          if (lb != la && lb < LEAN_LLINES * 32u) atomicOr(&L.lines_l[k][lb >> 5], 1u << (lb & 31u));
        }
      }
    };
    if constexpr (ECH) late_load(uint32_t(tid));
    // Ring slots (LK_LEAN_SLOTS, r06): outside the early_late bodies round j consumes slot j % PF and refills it right
    // after the slot's last use, and the rounds run PF at a time (the loop below), so each slot keeps its registers.  A
    // rotated ring (x = xr[0]; xr[i] = xr[i + 1]) copies the newest load's registers at the loop latch, and that copy
    // waits for the load (s_waitcnt vmcnt(0): the counter retires in order) -- one exposed memory round trip per round
    // however deep the ring, which is what left the COUNT shapes latency-bound (`count` 0.733 -> 0.476 ms with the
    // load-free COUNT rows below).  The late-column shapes keep the rotated ring: their list trips wait on their own
    // loads, which drains the ring either way (tag 0.969 / 0.973 ms, C4 1.351 / 1.351), and C3's three unrolled rounds
    // spill (1.80 -> 1.86 ms); C2 measured the same both ways (1.105 ms) and keeps the slots.
    constexpr bool ROT = PF > 0 && (ECH || (NL > 0 && !LEAN_DEFER(NL, AGG)) || !LK_LEAN_SLOTS);
    auto round = [&](uint32_t q0, auto slc) __attribute__((always_inline)) {
      constexpr int S = decltype(slc)::value;   // the ring slot this round consumes (unrotated ring)
      const uint32_t q = q0 + uint32_t(tid);
      const bool live = q < total;
      const LeanRun R = L.runs[live ? L.ctab[q] : 0u];
      const uint32_t k = q - R.cbk;
      const uint32_t v0 = R.start + 16u * k;
      const uint32_t a = (R.lo > v0 ? R.lo : v0) - v0;
      const uint32_t bnd = ((R.hi < v0 + 16u) ? R.hi : v0 + 16u) - v0;
      const uint32_t valid = (live && a < bnd) ? (((1u << bnd) - 1u) & ~((1u << a) - 1u)) : 0u;   // bit e
      const bool lit = (R.off_lit & 0x80000000u) != 0u;
      const uint32_t rval = R.value & 63u;
      const uint32_t byte = (R.off_lit & 0x7fffffffu) + 2u * BW * k;
      v4u x;
      LWin lcur[LT::NLA];
      if constexpr (ROT) {
        x = xr[0];
#pragma unroll
        for (int i = 0; i + 1 < PF; i++) xr[i] = xr[i + 1];
        xr[PF - 1] = chunk_load(q + uint32_t(PF) * BLOCK);
      } else if constexpr (PF > 0) {
        x = xr[S];   // refilled below, after its last use
      } else {
        x = __builtin_amdgcn_raw_buffer_load_b128(rs2, (live && lit) ? (byte & ~3u) : OOB, 0, 0);
      }
      if constexpr (ECH) {
#pragma unroll
        for (int k = 0; k < NL; k++) lcur[k] = lpre[k];
        late_load(q + BLOCK);
      }
      const uint32_t sh = (byte & 3u) * 8u;
      uint32_t w0 = __builtin_amdgcn_alignbit(x.y, x.x, sh);
      uint32_t w1 = __builtin_amdgcn_alignbit(x.z, x.y, sh);
      uint32_t w2 = __builtin_amdgcn_alignbit(x.w, x.z, sh);
      if constexpr (PF > 0 && !ROT) xr[S] = chunk_load(q + uint32_t(PF) * BLOCK);   // x is dead: the slot's next chunk
      if (!lit) {   // RLE run: every field holds the run's code
        if constexpr (POW2) {
          w0 = w1 = rval * REP;
        }
      }
      // pass flags: bit e * S + S - 1 (S = BW for SWAR, 1 per code)
      unsigned long long m = 0;
      uint32_t shs = 0;
      if (swar) {
        if constexpr (POW2) {
          constexpr uint32_t LO = ~HI;
          auto zf = [&](uint32_t y) __attribute__((always_inline)) { return ~(((y & LO) + LO) | y | LO); };   // high bit set <=> field == 0
          uint32_t z0 = 0, z1 = 0;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            if (pc[j] == 0xffffffffu) break;   // uniform
            const uint32_t rp = pc[j] * REP;
            z0 |= zf(w0 ^ rp);
            if (BW == 4) z1 |= zf(w1 ^ rp);
          }
          // valid rows [a, bnd) in field-high-bit form: fields a*BW .. bnd*BW - 1 of the high-bit pattern
          constexpr unsigned long long HI64 = ((unsigned long long)HI << 32) | HI;
          const uint32_t hb = bnd * BW;   // <= 64
          const unsigned long long vm = valid ? (hb >= 64u ? ~0ull : (1ull << hb) - 1ull) & ~((1ull << (a * BW)) - 1ull) & HI64 : 0ull;
          m = (((unsigned long long)z1 << 32) | z0) & vm;
          shs = BW == 1 ? 0u : BW == 2 ? 1u : 2u;
        }
      } else {
        uint32_t f = 0;
#pragma unroll
        for (int e = 0; e < 16; e++) {
          const uint32_t c = lit ? lean_code<BW>(w0, w1, w2, uint32_t(e)) : rval;
          f |= uint32_t((emask >> c) & 1ull) << e;
        }
        m = f & valid;
      }
      const uint32_t rbase = v0 - vb2;   // tile row of value v0
      // (not built into the unrotated-ring COUNT(*) shape: its rows gather nothing to coalesce unless the timestamps are
      // unsorted, and the block's registers would spill inside the round -- a spill reload waits like any load; the
      // host sends dense filters to the EARLY shape, which keeps the block)
      constexpr bool DENSE_BLK = NL == 0 && !(AGG == AGG_COUNT && !EARLY && LK_LEAN_SLOTS);
      if (DENSE_BLK && dense_codes) {   // uniform
        // Dense block: the wave's 64 chunks are 1024 row-contiguous rows and most chunks pass several rows.  The
        // per-lane loop below would have each load instruction touch 64 different 128-B lines (8 B used of each,
        // the other 120 B re-fetched by later trips -- evicted from L2 in between when every row passes), so the
        // block is read row-major instead: trip j, lane L takes row 64j + L (one 512-B coalesced load per column);
        // its pass bit and code come from the chunk's owner lane 4j + L/16 by cross-lane reads.
        uint32_t f16 = uint32_t(m);
        if (swar) {
          f16 = 0;
#pragma unroll
          for (int e = 0; e < 16; e++) f16 |= uint32_t((m >> (e * BW + BW - 1)) & 1ull) << e;
        }
        const uint32_t v0l = uint32_t(__shfl(int(v0), 0));
        const bool contig = live && valid == 0xffffu && v0 == v0l + 16u * uint32_t(lane);
        if (__ballot(contig) == ~0ull && __popcll(__ballot(__popc(f16) >= 2u)) >= 48) {
          const uint32_t rb0 = uni(rbase);
          // several passing codes over one bucket's direct table: rows go straight to their cell (uniform)
          const uint64_t jt = uint64_t(tile_b - tbl);
          const bool ddir = dense_direct && one_bucket && !P.nvl && tspan && jt < tspan;
          const uint32_t dbase = ddir ? uint32_t(jt) * ngr * rep + myrep : 0u;
          // The owner lane's 16 codes as 16 BW-bit fields in (c0, c1, c2) -- an RLE chunk's code replicated -- with
          // the pass bits in the spare high bits (BW <= 5), so a reader takes its code and pass bit with 1-3 cross-lane
          // reads instead of six.
          uint32_t c0 = w0, c1 = w1, c2 = w2;
          if (!lit) lean_rep<BW>(rval, c0, c1, c2);
          constexpr uint32_t FSH = BW <= 4 ? 0u : 16u;   // f16's place in c2 (BW == 6: no room, its own read)
          if constexpr (BW <= 5) c2 = (BW <= 4 ? 0u : (c2 & 0xffffu)) | (f16 << FSH);
#pragma unroll 1
          for (int j0 = 0; j0 < 16; j0 += 4) {
            v2u tt[4], xx[4];
            bool pp[4];
            uint32_t dd[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {   // issue the 4 trips' loads before any use
              const int src = 4 * (j0 + u) + (lane >> 4);
              const uint32_t e = uint32_t(lane) & 15u;
              const uint32_t a2 = BW <= 5 ? uint32_t(__shfl(int(c2), src)) : 0u;
              pp[u] = ((BW <= 5 ? a2 >> FSH : uint32_t(__shfl(int(f16), src))) >> e) & 1u;
              const uint32_t r = rb0 + 64u * uint32_t(j0 + u) + uint32_t(lane);
              tt[u] = v2u{0u, 0u};
              xx[u] = v2u{0u, 0u};
              if (ts_gather) tt[u] = __builtin_amdgcn_raw_buffer_load_b64(rs0, pp[u] ? (vb0 + r) * 8u : OOB, 0, 0);
              if (AGG != AGG_COUNT || P.nvl) xx[u] = __builtin_amdgcn_raw_buffer_load_b64(rs1, pp[u] ? (vb1 + r) * 8u : OOB, 0, 0);
              dd[u] = dim_u;
              if (npass > 1) {   // uniform
                const uint32_t a0 = uint32_t(__shfl(int(c0), src));
                const uint32_t a1 = BW > 2 ? uint32_t(__shfl(int(c1), src)) : 0u;
                const uint32_t a2c = BW == 6 ? uint32_t(__shfl(int(c2), src)) : a2;
                dd[u] = (L.lut[lean_code<BW>(a0, a1, a2c, e)] & DIM_MASK) * stride;
              }
              if (count_plan && pp[u]) {
                if (ts_gather) {
                  const uint32_t l = (((vb0 + r) * 8u) >> 7) - line_t0;
                  atomicOr(&L.lines_t[l >> 5], 1u << (l & 31u));
                }
                if (AGG != AGG_COUNT || P.nvl) {
                  const uint32_t l = (((vb1 + r) * 8u) >> 7) - line_v0;
                  atomicOr(&L.lines_v[l >> 5], 1u << (l & 31u));
                }
              }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
              if (!pp[u]) continue;
              const double v = __longlong_as_double((long long)(((uint64_t)xx[u].y << 32) | xx[u].x));
              if (ddir) {   // uniform: straight into the direct-table cell (neighbouring rows rarely share it)
                const uint32_t x = dbase + dd[u] * rep;
                min_nan_check<AGG>(P, true, v);
                if (AGG == AGG_SUM) {
                  const double h = v + 0.0;   // never -0.0 (the empty marker)
                  if (P.exact_sum) {
                    __hip_atomic_fetch_add(reinterpret_cast<double*>(rv + x), h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                  } else {
                    const double old = atomicAdd(reinterpret_cast<double*>(rv + x), h);
                    double s, e;
                    two_sum(old, h, s, e);
                    if (e != 0.0) atomicAdd(reinterpret_cast<double*>(rlo + x), e);
                  }
                } else if (AGG == AGG_MIN) {
                  atomicMin(rv + x, dbl_order(v));
                } else if (AGG == AGG_MAX) {
                  atomicMax(rv + x, dbl_order(v));
                } else {
                  atomicAdd(rv + x, 1ull);
                }
                if (rrows_on) atomicAdd(rrows + x, 1ull);
              } else {
                row((int64_t)(((uint64_t)tt[u].y << 32) | tt[u].x), v, dd[u], rb0 + 64u * uint32_t(j0 + u) + uint32_t(lane));
              }
            }
          }
          m = 0;
        }
      }
      constexpr bool LIST0 = NL == 0 && LK_LEAN_LIST0 && AGG != AGG_COUNT && !EARLY;
      if (AGG == AGG_COUNT && NL == 0 && LK_LEAN_SLOTS && !ts_gather && !P.nvl) {   // uniform
        // COUNT(*) with every row's bucket from the zone map or the split: no per-row load, so no loop here carries
        // one (a wait at its head would drain the chunk ring too).  One passing code and no split boundary inside the
        // chunk: the chunk's rows are one register-cell add of their popcount.
        const uint32_t n = uint32_t(__popcll(m));
        const uint32_t c0 = split ? split_class(rbase) : 1u, c15 = split ? split_class(rbase + 15u) : 1u;
        if (n && npass == 1 && c0 == c15) {
          if (c0 != 0u && (!split || c0 < nsb)) {   // inside the window
            row(0, 0.0, dim_u, rbase + (uint32_t(__builtin_ctzll(m)) >> shs));
            acc.rows += n - 1u;
            acc.cnt += n - 1u;
          }
        } else {
          while (m) {
            const uint32_t e = uint32_t(__builtin_ctzll(m)) >> shs;
            m &= m - 1ull;
            const uint32_t d = npass > 1 ? (L.lut[lit ? lean_code<BW>(w0, w1, w2, e) : rval] & DIM_MASK) * stride : dim_u;
            row(0, 0.0, d, rbase + e);
          }
        }
      } else if (!LT::LISTED || (NL == 0 && (!LIST0 || dense_codes))) {   // uniform
        // passing rows: two per trip (their loads in flight together)
        while (m) {
          const uint32_t e1 = uint32_t(__builtin_ctzll(m)) >> shs;
          m &= m - 1ull;
          const bool two = m != 0ull;
          const uint32_t e2 = two ? (uint32_t(__builtin_ctzll(m)) >> shs) : e1;
          if (two) m &= m - 1ull;
          uint32_t d1 = dim_u, d2 = dim_u;
          if (npass > 1) {   // uniform: the rows' codes -> group terms
            d1 = (L.lut[lit ? lean_code<BW>(w0, w1, w2, e1) : rval] & DIM_MASK) * stride;
            d2 = (L.lut[lit ? lean_code<BW>(w0, w1, w2, e2) : rval] & DIM_MASK) * stride;
          }
          const uint32_t rr[2] = {rbase + e1, rbase + e2};
          const bool aa[2] = {true, two};
          uint32_t dd[2] = {d1, d2};
          v2u lw[2][LT::NLA];   // (NL = 0 here: no late columns)
          uint32_t lm[2][LT::NLA];
          rowsN(std::integral_constant<int, 2>{}, std::false_type{}, rr, aa, dd, lw, lm);
        }
      } else if constexpr (LT::LISTED) {
        // Late columns: the wave's passing rows are appended to its LDS list (lane-major) and processed LEAN_TRIP at
        // a time (list_trip) -- a per-lane loop would run as many trips as the lane with the most passing rows, each
        // a chain of dependent late-column and value loads.
        // passing rows: row e at bit (e << fs) + (1 << fs) - 1 of fm (SWAR: the field's high bit; else one bit per row)
        unsigned long long fm = m;
        uint32_t fs = shs;
        uint32_t f16 = 0;
        if constexpr (ECH) {   // early_late: one bit per row
          f16 = uint32_t(m);
          if (swar) {
            f16 = 0;
#pragma unroll
            for (int e = 0; e < 16; e++) f16 |= uint32_t((m >> (e * BW + BW - 1)) & 1ull) << e;
          }
        }
        // early_late: row e's late code k from the chunk's window (chunk-relative index e - a), its lookup value
        auto late_code = [&](int k, uint32_t e) __attribute__((always_inline)) -> uint32_t {
          const LWin& w = lcur[k];
          if (w.meta >> 31) {
            const uint32_t sh = (w.meta & 0xffu) + (e - a) * lbw[k], wi = sh >> 5, off = sh & 31u;
            const uint32_t lo = wi == 0 ? w.x.x : wi == 1 ? w.x.y : wi == 2 ? w.x.z : wi == 3 ? w.x.w : w.x4;
            const uint32_t hi = wi == 0 ? w.x.y : wi == 1 ? w.x.z : wi == 2 ? w.x.w : wi == 3 ? w.x4 : 0u;
            return __builtin_amdgcn_alignbit(hi, lo, off) & ((1u << lbw[k]) - 1u);
          }
          if (!(w.meta >> 30)) return w.meta;
          // the chunk straddles a late run boundary: this row's run and packed word (synchronous; rare)
          const uint32_t v = lvb[k] + rbase + e;
          const int ri = lnr[k] == 1u ? 0 : lean_find_run(L.lruns[k], L.lrblk[k], nblk, lvb[k], v);
          const LRun lr = L.lruns[k][ri];
          if (!(lr.off_lit & 0x80000000u)) return lr.value;
          const uint32_t bit = (v - lr.start) * lbw[k];
          const uint32_t byte = (lr.off_lit & 0x7fffffffu) + (bit >> 3);
          const v2u ww = __builtin_amdgcn_raw_buffer_load_b64(lrs[k], byte & ~3u, 0, 0);
          const uint64_t xx = ((uint64_t)ww.y << 32) | ww.x;
          return uint32_t(xx >> ((byte & 3u) * 8u + (bit & 7u))) & ((1u << lbw[k]) - 1u);
        };
        if constexpr (ECH) {   // the late filter before the list
          if (!late_trivial) {
            uint32_t keep = 0u, f = f16;
            const uint32_t lf = Sp->leaf_false;
            while (f) {
              const uint32_t e = uint32_t(__builtin_ctz(f));
              f &= f - 1u;
              uint32_t T = 0u, F = 0u;
#pragma unroll
              for (int k = 0; k < NL; k++) {
                const StrParam& sp = P.strp[1 + k];
                if (!((lpres >> k) & 1u)) {
                  F |= sp.hmask;
                  continue;
                }
                const uint32_t bits = (L.llut[k][late_code(k, e)] >> 24) << sp.lbase;
                T |= bits & sp.lmask;
                F |= ~bits & sp.lmask;
              }
              const uint32_t ix = (T & ~lf) | ((F | lf) << P.nleaves);
              keep |= ((L.ltruth[ix >> 5] >> (ix & 31)) & 1u) << e;
            }
            f16 = keep;
          }
          fm = f16;
          fs = 0;
        }
        if constexpr (ECH) {
          // COUNT(*) into a one-bucket direct table (tag queries): the chunk's late codes are in
          // its window already, so a passing row is counted right here -- no list, no per-row late-column load
          if (direct_count) {   // uniform
            const uint32_t base = uint32_t(tile_b - tbl) * ngr;
            uint32_t f = f16;
            while (f) {
              const uint32_t e = uint32_t(__builtin_ctz(f));
              f &= f - 1u;
              const uint32_t code = lit ? lean_code<BW>(w0, w1, w2, e) : rval;
              uint32_t term = npass > 1 ? (L.lut[code] & DIM_MASK) * stride : dim_u;
#pragma unroll
              for (int k = 0; k < NL; k++) {
                const StrParam& sp = P.strp[1 + k];
                term += ((lpres >> k) & 1u) ? (L.llut[k][late_code(k, e)] & DIM_MASK) * sp.dim_stride
                                            : sp.dim_null * sp.dim_stride;
              }
              const uint32_t x = (base + term) * rep + myrep;
              atomicAdd(rv + x, 1ull);
              if (rrows_on) atomicAdd(rrows + x, 1ull);
            }
            return;   // (uniform) the next round of chunks
          }
        }
        if (P.ablate & 0x10000u) fm = 0;   // diagnostics only: no row listed (the chunk filter's cost alone)
        const uint32_t cnt = uint32_t(__popcll(fm));
        uint32_t inc = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t o = uint32_t(__shfl_up(int(inc), d, 64));
          if (lane >= d) inc += o;
        }
        const uint32_t wtotal = uni(uint32_t(__shfl(int(inc), 63)));
        const uint32_t pos0 = inc - cnt;
        for (uint32_t done = 0; done < wtotal;) {   // uniform
          const uint32_t take = min(LT::LIST - (ltail - lhead), wtotal - done);
          unsigned long long f = fm;
          uint32_t pos = pos0;
          while (f) {
            const uint32_t e = uint32_t(__builtin_ctzll(f)) >> fs;
            f &= f - 1ull;
            if (pos >= done && pos < done + take) {
              const uint32_t code = lit ? lean_code<BW>(w0, w1, w2, e) : rval;
              uint32_t hi16 = code;
              if constexpr (ECH) {   // the row's complete group term
                hi16 = npass > 1 ? (L.lut[code] & DIM_MASK) * stride : dim_u;
#pragma unroll
                for (int k = 0; k < NL; k++) {
                  const StrParam& sp = P.strp[1 + k];
                  hi16 += ((lpres >> k) & 1u) ? (L.llut[k][late_code(k, e)] & DIM_MASK) * sp.dim_stride
                                              : sp.dim_null * sp.dim_stride;
                }
              }
              wl[(ltail + pos - done) & (LT::LIST - 1u)] = (rbase + e) | (hi16 << 16);
            }
            pos++;
          }
          ltail += take;
          done += take;
          wave_sync();
          while (ltail - lhead >= LEAN_TRIP) list_trip(ec, LEAN_TRIP);   // uniform
          wave_sync();   // the trips' entries are rewritten by later appends
        }
      }
    };
    if constexpr (ROT || PF <= 1) {
      for (uint32_t q0 = 0; q0 < total; q0 += BLOCK) round(q0, std::integral_constant<int, 0>{});   // uniform trip count
    } else {
      for (uint32_t q0 = 0; q0 < total; q0 += uint32_t(PF) * BLOCK) {   // uniform: PF rounds, slots 0 .. PF - 1
        round(q0, std::integral_constant<int, 0>{});
        if (q0 + BLOCK < total) round(q0 + BLOCK, std::integral_constant<int, 1>{});
        if constexpr (PF > 2) {
          if (q0 + 2u * BLOCK < total) round(q0 + 2u * BLOCK, std::integral_constant<int, 2>{});
        }
        static_assert(PF <= 3, "ring slots: rounds unrolled up to 3");
      }
    }
    if constexpr (LT::LISTED) {
      while (ltail != lhead) list_trip(ec, min(LEAN_TRIP, ltail - lhead));   // the tile's last rows
      if constexpr (LEAN_DEFER(NL, AGG) && !ECH) {
        if (pend) rowsN(std::integral_constant<int, LEAN_ROWS>{}, ec, prr, paa, pdd, plw, plm);   // the last trip
        pend = false;
      }
      wave_sync();
    }
  };
  auto body2 = [&](auto bwc) __attribute__((always_inline)) {
    if constexpr (NL > 0 && EARLY) {
      if (early_late) body(bwc, std::true_type{});   // uniform
      else body(bwc, std::false_type{});
    } else {
      body(bwc, std::false_type{});
    }
  };
  switch (bw) {   // uniform
    case 1: body2(std::integral_constant<uint32_t, 1>{}); break;
    case 2: body2(std::integral_constant<uint32_t, 2>{}); break;
    case 3: body2(std::integral_constant<uint32_t, 3>{}); break;
    case 4: body2(std::integral_constant<uint32_t, 4>{}); break;
    case 5: body2(std::integral_constant<uint32_t, 5>{}); break;
    default: body2(std::integral_constant<uint32_t, 6>{}); break;
  }

  flush();
  __syncthreads();
  if (count_plan) {
    if (tid == 0) {
      pbytes += sizeof(TileDesc) + 3 * sizeof(TileCol) + uint64_t(nr) * sizeof(RunDesc) + uint64_t(dict_n) * 8u;
    }
    // diagnostics only (LK_ABLATE bits 8..11): leave a category out of the count -- bit 8 timestamp lines, 9 value
    // lines, 10 late-stream lines, 11 the name stream and metadata
    const uint32_t pm = P.ablate >> 8;
    if (pm & 8u) pbytes = 0;
    for (uint32_t i = tid; i < LEAN_LINES; i += BLOCK)
      pbytes += 128u * uint64_t((pm & 1u ? 0 : __popc(L.lines_t[i])) + (pm & 2u ? 0 : __popc(L.lines_v[i])));
#pragma unroll
    for (int k = 0; k < NL; k++)
      for (uint32_t i = tid; i < LEAN_LLINES && !(pm & 4u); i += BLOCK) pbytes += 128u * uint64_t(__popc(L.lines_l[k][i]));
    if (pbytes) atomicAdd(P.plan_bytes, (unsigned long long)pbytes);
  }
  // ---- the table's cells -> the global table (device atomics) ----
  if (tspan) {
    for (uint32_t c = tid; c < tspan * ngr; c += BLOCK) {   // a cell's replicas, combined
      unsigned long long v = rident, r = 0;
      double hi = 0.0, lo = 0.0;
      for (uint32_t k = 0; k < rep; k++) {
        const uint32_t x = c * rep + k;
        const unsigned long long vk = rv[x];
        const unsigned long long rk = rrows_on ? rrows[x] : (AGG == AGG_COUNT ? vk : (vk != rident ? 1ull : 0ull));
        if (rk == 0ull) continue;
        r += rk;
        if (AGG == AGG_SUM) {
          double s2, e;
          two_sum(hi, __longlong_as_double((long long)vk), s2, e);
          hi = s2;
          lo += e + __longlong_as_double((long long)rlo[x]);
        } else if (AGG == AGG_MIN) {
          v = vk < v ? vk : v;
        } else if (AGG == AGG_MAX) {
          v = vk > v ? vk : v;
        } else {
          v = (v == rident ? 0ull : v) + vk;
        }
      }
      if (r == 0ull) continue;
      const uint32_t j = c / ngr, g = c - j * ngr;
      if (AGG == AGG_SUM) v = (unsigned long long)__double_as_longlong(hi);
      global_merge<AGG, HASH>(P, (glob_base + (unsigned long long)(tbl + j)) * P.ngroups + g, uint32_t(r), uint32_t(r),
                              hi, lo, v);
    }
  } else {
    for (int i = tid; i < LeanHash::H; i += BLOCK) {
      if (L.agg.hs.hkey[i] == EMPTY) continue;
      global_merge<AGG, HASH>(P, L.agg.hs.hkey[i], L.agg.hs.hrows[i], L.agg.hs.hcnt[i], L.agg.hs.hhi[i], L.agg.hs.hlo[i],
                              reinterpret_cast<unsigned long long*>(L.agg.hs.hhi)[i]);
    }
  }
}

}  // namespace lk
