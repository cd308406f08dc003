// stream_probe.hip — achievable HBM read rate on this box for a 1 GiB fp64 buffer (the size of
// A at the north-star shape), to price how far the A@X and A^T R passes sit from it.
// Forms: 16-B register loads (default policy / nontemporal), grid-stride or one contiguous
// chunk per workgroup, and LDS-DMA (global_load_lds_dwordx4, aux 0 or 2 = nt) into a 4-slot ring
// with no consumer. Prints one line per form: best and median of 10 timed launches.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/stream_probe scripts/stream_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <vector>

typedef double v2d __attribute__((ext_vector_type(2)));

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

template <int UNR, bool NT>
__global__ __launch_bounds__(256) void k_stride(const v2d* __restrict__ a, size_t n2, double* out) {
  v2d acc = {0.0, 0.0};
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i + (UNR - 1) * stride < n2; i += UNR * stride) {
    v2d v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = NT ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc += v[u];
  }
  if (acc.x == 1234.5) out[0] = acc.y;   // never: keeps the loads
}

// one contiguous chunk per workgroup, UNR 4-KiB steps in flight per block
template <int UNR, bool NT>
__global__ __launch_bounds__(256) void k_chunk(const v2d* __restrict__ a, size_t n2, double* out) {
  v2d acc = {0.0, 0.0};
  const size_t per = n2 / gridDim.x;
  const v2d* p = a + (size_t)blockIdx.x * per;
  for (size_t i = threadIdx.x; i + (UNR - 1) * 256 < per; i += UNR * 256) {
    v2d v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = NT ? __builtin_nontemporal_load(p + i + u * 256) : p[i + u * 256];
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc += v[u];
  }
  if (acc.x == 1234.5) out[0] = acc.y;
}

// LDS-DMA: each wave moves 1 KiB per instruction into its own quarter of a 16-KiB ring slot;
// 4 instructions per slot per wave, DEPTH slots in flight, nobody reads the LDS
template <int AUX, int DEPTH>
__global__ __launch_bounds__(256) void k_glds(const double* __restrict__ a, size_t nbytes, double* out) {
  __shared__ __attribute__((aligned(16))) char ring[DEPTH][16384];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t per = nbytes / gridDim.x;
  const char* base = reinterpret_cast<const char*>(a) + (size_t)blockIdx.x * per;
  const size_t steps = per / 16384;
  for (size_t s = 0; s < steps; ++s) {
    const int slot = (int)(s % DEPTH);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const char* g = base + s * 16384 + (size_t)(wave * 4 + k) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g),
                                       (__attribute__((address_space(3))) void*)(
                                           &ring[slot][(wave * 4 + k) * 1024]),
                                       16, 0, AUX);
    }
    if (DEPTH == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0 && ring[0][wave] == 123) out[0] = 1.0;
}


// Access patterns of the two passes over A (m = 8192 rows of n = 16384 fp64), loads only.
// ax_rows: k_ax_lds's single-RHS tile as it reads A today: 8 waves, wave w owns 16 rows, lane
// (i, q) reads 32 B of row i at k = 16 c + 4 q per 16-wide chunk c; K split S over blockIdx.
// ax_blk: the same tile over a blocked copy (16 x 16 blocks of 2 KiB, the blocks of one 16-row
// tile consecutive along k): a wave's chunk is 2 KiB contiguous.
template <bool NT, bool BLK>
__global__ __launch_bounds__(512) void k_ax_pat(const v2d* __restrict__ a, int m, int n, int S, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int gx = m / 128;
  const int bx = blockIdx.x % gx, by = blockIdx.x / gx;
  const int rt = bx * 8 + wave;            // 16-row tile
  const int nch = n / 16;
  const int c0 = nch * by / S, c1 = nch * (by + 1) / S;
  v2d acc = {0.0, 0.0};
  for (int c = c0; c + 3 < c1; c += 4) {
    v2d v[8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t off = BLK ? ((size_t)rt * nch + c + u) * 256 + i * 16 + q * 4
                             : (size_t)(rt * 16 + i) * n + (size_t)(c + u) * 16 + q * 4;
      const v2d* p = a + off / 2;
      v[2 * u] = NT ? __builtin_nontemporal_load(p) : p[0];
      v[2 * u + 1] = NT ? __builtin_nontemporal_load(p + 1) : p[1];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  if (acc.x == 1234.5) out[0] = acc.y;
}

// atr_rows: A^T R's panel as it reads A today (approximately): 4 waves on one 64-column panel,
// wave w walks rows w, w + 4, ...; one wave-instruction = 512 B of each of two rows.
// atr_blk: the same panel over the blocked copy: per 16-row tile the panel is 4 consecutive
// 2-KiB blocks (8 KiB contiguous); wave w walks tiles w, w + 4, ...
template <bool NT, bool BLK>
__global__ __launch_bounds__(256) void k_atr_pat(const v2d* __restrict__ a, int m, int n, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int panel = blockIdx.x;
  const int nch = n / 16;
  v2d acc = {0.0, 0.0};
  if (BLK) {
    for (int rt = wave; rt + 4 < m / 16; rt += 8) {
      v2d v[16];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const size_t off = ((size_t)(rt + 4 * u) * nch + panel * 4) * 256 + j * 128 + lane * 2;
          const v2d* p = a + off / 2;
          v[u * 8 + j] = NT ? __builtin_nontemporal_load(p) : p[0];
        }
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[u];
    }
  } else {
    // row pairs rp = wave + 4 (16 t + j): 16 wave-instructions (1 KiB each) in flight per trip
    for (int t = 0; t < m / 2 / 64; ++t) {
      v2d v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int row = 2 * (wave + 4 * (16 * t + j)) + (lane >> 5);
        const v2d* p = a + ((size_t)row * n + (size_t)panel * 64 + (lane & 31) * 2) / 2;
        v[j] = NT ? __builtin_nontemporal_load(p) : p[0];
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[u];
    }
  }
  if (acc.x == 1234.5) out[0] = acc.y;
}


// A^T R as k_atr_prox reads A: one 64-column panel per 4-wave block, 4 rows per step (lane
// (i, q): row q, columns 4i..4i+3 as two 16-B loads), PF = 8 steps in flight per wave.
// ILV = 0: wave w walks its own quarter of the rows (today); ILV = 1: the waves interleave
// (step s of wave w = rows 4 (4 s + w) .. +3), so the block walks consecutive rows together.
template <bool NT, bool ILV>
__global__ __launch_bounds__(256) void k_atr_real(const double* __restrict__ a, int m, int n, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int steps = m / 4, per = steps / 4;
  const int64_t col0 = (int64_t)blockIdx.x * 64 + 4 * i;
  v2d acc = {0.0, 0.0};
  for (int s0 = 0; s0 < per; s0 += 8) {
    v2d v[16];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int step = ILV ? 4 * (s0 + p) + wave : wave * per + s0 + p;
      const double* ptr = a + (int64_t)(4 * step + q) * n + col0;
      v[2 * p] = NT ? __builtin_nontemporal_load(reinterpret_cast<const v2d*>(ptr)) : *reinterpret_cast<const v2d*>(ptr);
      v[2 * p + 1] = NT ? __builtin_nontemporal_load(reinterpret_cast<const v2d*>(ptr + 2)) : *reinterpret_cast<const v2d*>(ptr + 2);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += v[u];
  }
  if (acc.x == 1234.5) out[0] = acc.y;
}

// A@X single RHS over the blocked copy with the waves of a block splitting K instead of rows:
// 8 waves, MT row tiles shared by the block, super-chunk j = 8 chunks of 16 k, wave w takes
// chunk 8 j + w of every row tile (2 KiB per tile, the 8 waves' blocks adjacent: 16 KiB
// contiguous per tile per super-chunk); PF super-chunks in flight.
template <bool NT, int MT>
__global__ __launch_bounds__(512) void k_ax_ksplit(const v2d* __restrict__ a, int m, int n, int S, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = n / 16, nsc = nch / 8;
  const int gx = m / (16 * MT);
  const int bx = blockIdx.x % gx, by = blockIdx.x / gx;
  const int j0 = nsc * by / S, j1 = nsc * (by + 1) / S;
  v2d acc = {0.0, 0.0};
  for (int j = j0; j + 1 < j1; j += 2) {
    v2d v[2][MT][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const size_t rt = (size_t)bx * MT + t;
        const size_t off = (rt * nch + (size_t)(8 * (j + u) + wave)) * 256 + lane * 4;
        const v2d* p = a + off / 2;
        v[u][t][0] = NT ? __builtin_nontemporal_load(p) : p[0];
        v[u][t][1] = NT ? __builtin_nontemporal_load(p + 1) : p[1];
      }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t) acc += v[u][t][0] + v[u][t][1];
  }
  if (acc.x == 1234.5) out[0] = acc.y;
}


// A@X single-RHS row tile with the k of a chunk remapped so that each 16-B load instruction
// reads 64 contiguous bytes of each of its 16 rows (lane (i, q): k = 16 c + 8 v + 2 q), and a
// form with 8 rows x 128 B per instruction (lane l: row l / 8, k = 16 c + 2 (l % 8)).
template <bool NT, int FORM>
__global__ __launch_bounds__(512) void k_ax_pat2(const v2d* __restrict__ a, int m, int n, int S, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int gx = m / 128;
  const int bx = blockIdx.x % gx, by = blockIdx.x / gx;
  const int rt = bx * 8 + wave;
  const int nch = n / 16;
  const int c0 = nch * by / S, c1 = nch * (by + 1) / S;
  v2d acc = {0.0, 0.0};
  for (int c = c0; c + 3 < c1; c += 4) {
    v2d v[8];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        size_t off;
        if (FORM == 0) off = (size_t)(rt * 16 + i) * n + (size_t)(c + u) * 16 + w * 8 + q * 2;
        else off = (size_t)(rt * 16 + w * 8 + lane / 8) * n + (size_t)(c + u) * 16 + (lane % 8) * 2;
        const v2d* p = a + off / 2;
        v[2 * u + w] = NT ? __builtin_nontemporal_load(p) : p[0];
      }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  if (acc.x == 1234.5) out[0] = acc.y;
}

template <typename F>
static int timeit(const char* name, double bytes, F launch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < 10; ++r) {
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  std::printf("%-34s best %7.1f us %5.2f TB/s   median %7.1f us %5.2f TB/s\n", name, ts[0] * 1e3,
              bytes / (ts[0] * 1e-3) / 1e12, ts[5] * 1e3, bytes / (ts[5] * 1e-3) / 1e12);
  std::fflush(stdout);
  return 0;
}

int main() {
  const size_t nbytes = (size_t)8192 * 16384 * 8;   // 8192 x 16384 fp64 = 1 GiB
  double* a = nullptr;
  double* out = nullptr;
  CK(hipMalloc(&a, nbytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, nbytes));
  const size_t n2 = nbytes / 16;
  const v2d* a2 = reinterpret_cast<const v2d*>(a);
  const double B = (double)nbytes;
  const bool all = std::getenv("PROBE_ALL") != nullptr;
  for (int g : {1024, 2048, 4096, 8192}) {
    if (!all) break;
    char nm[64];
    std::snprintf(nm, sizeof nm, "stride u4 g%d", g);
    if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_stride<4, false>), dim3(g), dim3(256), 0, 0, a2, n2, out); })) return 1;
    std::snprintf(nm, sizeof nm, "stride u4 nt g%d", g);
    if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_stride<4, true>), dim3(g), dim3(256), 0, 0, a2, n2, out); })) return 1;
    std::snprintf(nm, sizeof nm, "stride u8 g%d", g);
    if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_stride<8, false>), dim3(g), dim3(256), 0, 0, a2, n2, out); })) return 1;
  }
  for (int g : {512, 1024, 2048}) {
    if (!all) break;
    char nm[64];
    std::snprintf(nm, sizeof nm, "chunk u8 g%d", g);
    if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_chunk<8, false>), dim3(g), dim3(256), 0, 0, a2, n2, out); })) return 1;
    std::snprintf(nm, sizeof nm, "chunk u8 nt g%d", g);
    if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_chunk<8, true>), dim3(g), dim3(256), 0, 0, a2, n2, out); })) return 1;
  }
  for (int g : {256, 512, 1024}) {
    if (!all) break;
    char nm[64];
    std::snprintf(nm, sizeof nm, "glds d4 g%d", g);
    if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_glds<0, 4>), dim3(g), dim3(256), 0, 0, a, nbytes, out); })) return 1;
    std::snprintf(nm, sizeof nm, "glds d4 nt g%d", g);
    if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_glds<2, 4>), dim3(g), dim3(256), 0, 0, a, nbytes, out); })) return 1;
    std::snprintf(nm, sizeof nm, "glds d2 nt g%d", g);
    if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_glds<2, 2>), dim3(g), dim3(256), 0, 0, a, nbytes, out); })) return 1;
  }
  {
    const int m = 8192, n = 16384;
    for (int S : {4, 8, 16}) {
      char nm[64];
      const int g = (m / 128) * S;
      std::snprintf(nm, sizeof nm, "ax rows S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_pat<false, false>), dim3(g), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
      std::snprintf(nm, sizeof nm, "ax rows nt S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_pat<true, false>), dim3(g), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
      std::snprintf(nm, sizeof nm, "ax blk S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_pat<false, true>), dim3(g), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
      std::snprintf(nm, sizeof nm, "ax blk nt S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_pat<true, true>), dim3(g), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
    }
    if (timeit("atr rows", B, [&] { hipLaunchKernelGGL((k_atr_pat<false, false>), dim3(n / 64), dim3(256), 0, 0, a2, m, n, out); })) return 1;
    if (timeit("atr rows nt", B, [&] { hipLaunchKernelGGL((k_atr_pat<true, false>), dim3(n / 64), dim3(256), 0, 0, a2, m, n, out); })) return 1;
    if (timeit("atr blk", B, [&] { hipLaunchKernelGGL((k_atr_pat<false, true>), dim3(n / 64), dim3(256), 0, 0, a2, m, n, out); })) return 1;
    if (timeit("atr blk nt", B, [&] { hipLaunchKernelGGL((k_atr_pat<true, true>), dim3(n / 64), dim3(256), 0, 0, a2, m, n, out); })) return 1;
    if (timeit("atr real", B, [&] { hipLaunchKernelGGL((k_atr_real<false, false>), dim3(n / 64), dim3(256), 0, 0, a, m, n, out); })) return 1;
    if (timeit("atr real nt", B, [&] { hipLaunchKernelGGL((k_atr_real<true, false>), dim3(n / 64), dim3(256), 0, 0, a, m, n, out); })) return 1;
    if (timeit("atr ilv", B, [&] { hipLaunchKernelGGL((k_atr_real<false, true>), dim3(n / 64), dim3(256), 0, 0, a, m, n, out); })) return 1;
    if (timeit("atr ilv nt", B, [&] { hipLaunchKernelGGL((k_atr_real<true, true>), dim3(n / 64), dim3(256), 0, 0, a, m, n, out); })) return 1;
    for (int S : {2, 4, 8}) {
      char nm[64];
      std::snprintf(nm, sizeof nm, "ax ksplit mt4 S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_ksplit<false, 4>), dim3(m / 64 * S), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
      std::snprintf(nm, sizeof nm, "ax ksplit mt4 nt S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_ksplit<true, 4>), dim3(m / 64 * S), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
      std::snprintf(nm, sizeof nm, "ax ksplit mt2 nt S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_ksplit<true, 2>), dim3(m / 32 * S), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
      std::snprintf(nm, sizeof nm, "ax ksplit mt1 nt S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_ksplit<true, 1>), dim3(m / 16 * S), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
    }
    for (int S : {4, 8}) {
      char nm[64];
      const int g = (m / 128) * S;
      std::snprintf(nm, sizeof nm, "ax rows64 S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_pat2<false, 0>), dim3(g), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
      std::snprintf(nm, sizeof nm, "ax rows64 nt S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_pat2<true, 0>), dim3(g), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
      std::snprintf(nm, sizeof nm, "ax rows128 S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_pat2<false, 1>), dim3(g), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
      std::snprintf(nm, sizeof nm, "ax rows128 nt S%d", S);
      if (timeit(nm, B, [&] { hipLaunchKernelGGL((k_ax_pat2<true, 1>), dim3(g), dim3(512), 0, 0, a2, m, n, S, out); })) return 1;
    }
  }
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
