// Calibration microbenchmark for the scan kernel's access patterns on MI355X (gfx950), over a 4 GiB buffer
// (16x the 256 MB Infinity Cache), each pattern timed with HIP events and, under `rocprofv3 --pmc FETCH_SIZE`,
// counted, so that FETCH_SIZE of the scan kernel can be converted to HBM bytes for ITS access widths:
//
//   stream16     every byte read once, 16 B per lane, coalesced (the guide's calibrated case)
//   gather8_s<S> one 8-B load per lane at stride S bytes (S = 64, 128, 256): 8-B per-lane gathers
//   sel8_p<k>    the scan kernel's pattern: rows of a PLAIN double column selected with probability 1/k (sorted
//                row lists, 64 rows per wave-instruction, 8 B per lane) -- k = 16 is C2's selectivity
//   line16_p<k>  the same selected rows, read line-granular: every 128-B line holding a selected row loaded whole
//                with 16 B per lane (8 lanes per line), the rows' values then taken from registers
//
// Prints one JSON line per pattern: bytes touched (distinct 128-B lines x 128, or stream bytes), time, GB/s.
//   hipcc -O3 --offload-arch=gfx950 -o tools/gather_bench tools/gather_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, int(bytes), 0x00020000);
}

// every 16-B chunk once; grid-stride
__global__ __launch_bounds__(256) void stream16(const v4u* a, size_t n16, unsigned long long* sink) {
  unsigned acc = 0;
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += size_t(gridDim.x) * 256) {
    const v4u v = __builtin_nontemporal_load(a + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// one 8-B load per lane at stride S
__global__ __launch_bounds__(256) void gather8(const unsigned char* a, size_t nelem, unsigned stride,
                                               unsigned long long* sink) {
  unsigned long long acc = 0;
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < nelem; i += size_t(gridDim.x) * 256)
    acc ^= *reinterpret_cast<const unsigned long long*>(a + i * stride);
  if (acc == 0x12345678ull) sink[0] = acc;
}

// the scan kernel's gather: sorted selected row indices (u32, relative to a 2^20-row page), 8 B per lane
__global__ __launch_bounds__(256) void sel8(const double* vals, const unsigned* rows, size_t nsel,
                                            unsigned long long* sink) {
  double acc = 0;
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < nsel; i += size_t(gridDim.x) * 256) acc += vals[rows[i]];
  if (acc == -1.2345) sink[0] = 1;
}

// line-granular: per wave, the 64 selected rows' distinct lines are loaded whole (8 lanes x 16 B per line, 8 lines
// per instruction), then each row's value is taken from the lane holding it (ds_bpermute)
__global__ __launch_bounds__(256) void line16(const double* vals, const unsigned* rows, size_t nsel,
                                              unsigned long long* sink) {
  __shared__ unsigned slot_line[4][64];
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double acc = 0;
  const size_t nw = (nsel + 63) / 64;
  for (size_t wi = size_t(blockIdx.x) * 4 + w; wi < nw; wi += size_t(gridDim.x) * 4) {
    const size_t i = wi * 64 + lane;
    const bool live = i < nsel;
    const unsigned row = live ? rows[i] : 0u;
    const unsigned line = row >> 4;                      // 16 doubles per 128-B line
    const unsigned prev = __shfl_up(line, 1, 64);
    const bool fresh = live && (lane == 0 || line != prev);
    const unsigned long long fm = __ballot(fresh);
    const unsigned slot = __builtin_amdgcn_mbcnt_hi(unsigned(fm >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(fm), 0u)) -
                          (fresh ? 0u : 1u);           // slot of this row's line (fresh lanes count themselves)
    if (fresh) slot_line[w][slot] = line;
    __builtin_amdgcn_wave_barrier();
    const unsigned nl = unsigned(__popcll(fm));
    double v = 0;
    for (unsigned k = 0; k * 8 < nl; k++) {             // 8 lines per wave-instruction
      const unsigned s = k * 8 + (lane >> 3);
      const unsigned ln = s < nl ? slot_line[w][s] : slot_line[w][0];
      const v4u x = *reinterpret_cast<const v4u*>(reinterpret_cast<const unsigned char*>(vals) + size_t(ln) * 128 +
                                                  (lane & 7) * 16);
      // row's value: line slot s' = slot, piece (row & 15) / 2 of lane 8 * (slot % 8) + piece
      const unsigned src = (8u * (slot & 7u) + ((row & 15u) >> 1)) * 4u;
      const unsigned lo = __builtin_amdgcn_ds_bpermute(src, (row & 1u) ? x.z : x.x);
      const unsigned hi = __builtin_amdgcn_ds_bpermute(src, (row & 1u) ? x.w : x.y);
      if ((slot >> 3) == k) v = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    }
    if (live) acc += v;
    __builtin_amdgcn_wave_barrier();
  }
  if (acc == -1.2345) sink[0] = 1;
}

int main(int argc, char** argv) {
  const size_t bytes = size_t(4) << 30;
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  unsigned char* a;
  unsigned long long* sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 1, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 256 * 8 * 4;
  auto timeit = [&](const char* name, double touched, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("{\"pattern\": \"%s\", \"touched_bytes\": %.0f, \"ms\": %.4f, \"touched_gbs\": %.1f}\n", name, touched, ms,
           touched / (ms / 1e3) / 1e9);
    fflush(stdout);
  };
  timeit("stream16", double(bytes), [&] { stream16<<<grid, 256>>>(reinterpret_cast<const v4u*>(a), bytes / 16, sink); });
  for (unsigned s : {64u, 128u, 256u}) {
    const size_t n = bytes / s;
    const double lines = s >= 128 ? double(n) : double(bytes / 128);
    timeit(("gather8_s" + std::to_string(s)).c_str(), lines * 128, [&] { gather8<<<grid, 256>>>(a, n, s, sink); });
  }
  // selected rows of the buffer viewed as doubles, probability 1/k
  const size_t nrows = bytes / 8;
  std::mt19937_64 rng(7);
  for (unsigned k : {4u, 16u, 64u}) {
    std::vector<unsigned> sel;
    sel.reserve(nrows / k + 1024);
    // rows addressed as u32 indices: use the first 2^32 / 8 ... keep indices < 2^29 (4 GiB / 8)
    for (size_t r = 0; r < nrows; r++)
      if ((rng() % k) == 0) sel.push_back(unsigned(r));
    size_t lines = 0;
    for (size_t i = 0; i < sel.size(); i++)
      if (i == 0 || (sel[i] >> 4) != (sel[i - 1] >> 4)) lines++;
    unsigned* d_sel;
    CK(hipMalloc(&d_sel, sel.size() * 4));
    CK(hipMemcpy(d_sel, sel.data(), sel.size() * 4, hipMemcpyHostToDevice));
    const double touched = double(lines) * 128 + double(sel.size()) * 4;
    timeit(("sel8_p" + std::to_string(k)).c_str(), touched,
           [&] { sel8<<<grid, 256>>>(reinterpret_cast<const double*>(a), d_sel, sel.size(), sink); });
    timeit(("line16_p" + std::to_string(k)).c_str(), touched,
           [&] { line16<<<grid, 256>>>(reinterpret_cast<const double*>(a), d_sel, sel.size(), sink); });
    CK(hipFree(d_sel));
  }
  CK(hipFree(a));
  return 0;
}
