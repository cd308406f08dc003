// kernels_gather.hip — the thresholded part of ProxGD's line-search candidate, A e, read from a
// transposed copy of A (split-candidate mode, solver.cpp iter_proxgd).
//
// The candidate p of a ProxGD trial is recorded (objective, gl_ProxGD_primal.py:112) before the
// hard threshold (:127) turns it into the next iterate p_thr, so one trial needs A p and A p_thr.
// Here A p = A p_thr + A e with e = p - p_thr: e is exactly p in the entries |p| < thres and 0
// elsewhere, and only a fraction of the rows of x have such entries (≈ 3 000 of 16 384 at the
// north-star size, ≈ 560 in the first iterations). A p_thr streams A once (the dense A@X tile
// with one right-hand side, HBM-bound); A e needs column k of A for every flagged row k of e,
// which is row k of At = A^T (n x m, one contiguous m-vector), built once per session:
//
//   P[s][r][c] = sum over the flagged rows k of split s (ascending):  At[k][r] * e[k][c]
//
// Every workgroup compacts the n row flags (zf[k] != 0, written by the trial kernel) into an
// ascending index list in LDS (a 256-thread scan; the order is fixed, so the sums are
// deterministic), takes its share s of the list, and runs a 16x16x4 MFMA loop whose K index
// walks the list: lane (i, q) loads At[k_q][r0 + 16 mt + i] (16 lanes = 128 contiguous bytes of
// one At row) and e[k_q][16 nt + i]. Reads |flagged| * m * s bytes of At: ≈ 190 MiB at 3 000
// rows instead of a second dense pass (1 GiB of MFMA-bound work). Partial slabs go to the
// finalize kernel, which forms A p - b = (A p_thr - b) + sum_s P[s].
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "glx.h"
#include "glx_device.h"

namespace glx {

namespace {
typedef double gd4 __attribute__((ext_vector_type(4)));
typedef float gf4 __attribute__((ext_vector_type(4)));
template <typename T> struct GM;
template <> struct GM<double> {
  typedef gd4 acc_t;
  __device__ static inline acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __device__ static inline int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <> struct GM<float> {
  typedef gf4 acc_t;
  __device__ static inline acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static inline int row(int lane, int r) { return ((lane >> 4) << 2) + r; }
};

constexpr int kGW = 4;                  // waves per workgroup
constexpr int kGThreads = 64 * kGW;
constexpr int kGMT = 4;                 // 16-row tiles per wave (64 output rows)
constexpr int kGRows = 16 * kGMT * kGW; // output rows per workgroup
}  // namespace

// At = A^T through 64 x 64 LDS tiles (padded rows: conflict-free transposed reads)
template <typename T>
__global__ __launch_bounds__(256) void k_transpose(const T* __restrict__ A, T* __restrict__ At,
                                                   int64_t m, int64_t n) {
  __shared__ T tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int rr = ty + 4 * k;
    const int64_t r = r0 + rr, c = c0 + tx;
    tile[rr][tx] = (r < m && c < n) ? A[r * n + c] : T(0);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int cc = ty + 4 * k;
    const int64_t c = c0 + cc, r = r0 + tx;
    if (c < n && r < m) At[c * m + r] = tile[tx][cc];
  }
}

// grid: gx row blocks x S splits of the flagged-row list (blockIdx.x = split * gx + row block)
// PF k-steps in flight per wave (2 KiB of At each at l = 32, f64)
template <typename T, int NT, int kGPF>
__global__ __launch_bounds__(kGThreads) void k_at_gather(const T* __restrict__ At,
                                                         const T* __restrict__ E,
                                                         const uint8_t* __restrict__ zf,
                                                         int64_t m, int64_t n, T* __restrict__ P,
                                                         int S, int gx) {
  typedef GM<T> M;
  typedef typename M::acc_t C;
  constexpr int L = 16 * NT;
  extern __shared__ unsigned short lst[];            // n entries (worst case: every row flagged)
  __shared__ unsigned wsum[kGW];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int bx = (int)blockIdx.x % gx, split = (int)blockIdx.x / gx;

  // ---- compaction: thread t owns flags [t * per, (t + 1) * per), per a multiple of 16, read
  // as 16-B vectors (the flag buffer is padded to 256 B; bytes at k >= n are ignored)
  const int64_t per = (((n + kGThreads - 1) / kGThreads) + 15) & ~int64_t(15);
  const int64_t f0 = tid * per;
  const int64_t f1 = (f0 + per < n) ? f0 + per : (f0 < n ? n : f0);
  auto flagged = [&](int64_t k) -> bool { return zf[k] != 0; };
  unsigned cntl = 0;
  for (int64_t k = f0; k < f1; k += 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(zf + k);
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (k + j < f1 && ((w[j >> 2] >> (8 * (j & 3))) & 0xffu) != 0) ++cntl;
  }
  // inclusive scan over the wave, then over the waves
  unsigned inc = cntl;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned v = __shfl_up(inc, off);
    if (lane >= off) inc += v;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  unsigned wbase = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kGW; ++w) {
    if (w < wave) wbase += wsum[w];
    total += wsum[w];
  }
  unsigned pos = wbase + inc - cntl;
  if (cntl != 0)
    for (int64_t k = f0; k < f1; ++k)
      if (flagged(k)) lst[pos++] = (unsigned short)k;
  __syncthreads();

  const int64_t beg = (int64_t)total * split / S, end = (int64_t)total * (split + 1) / S;
  const int64_t row0 = (int64_t)bx * kGRows + (int64_t)wave * (16 * kGMT);
  C acc[kGMT][NT];
#pragma unroll
  for (int mt = 0; mt < kGMT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = C{};

  if (end > beg) {
    int64_t rr[kGMT];
#pragma unroll
    for (int mt = 0; mt < kGMT; ++mt) {
      const int64_t r = row0 + 16 * mt + i;
      rr[mt] = r < m ? r : m - 1;
    }
    const int64_t nsteps = (end - beg + 3) / 4;
    T a[kGPF][kGMT], e[kGPF][NT];
    // step s, lane group q: list position beg + 4 s + q (past the end: a zero e row)
    auto ld = [&](int p, int64_t s) {
      s = s < nsteps ? s : nsteps - 1;
      const int64_t ps = beg + 4 * s + q;
      const bool ok = ps < end;
      const int64_t k = lst[ok ? ps : beg];
#pragma unroll
      for (int mt = 0; mt < kGMT; ++mt) a[p][mt] = At[k * m + rr[mt]];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) e[p][nt] = ok ? E[k * L + 16 * nt + i] : T(0);
    };
#pragma unroll
    for (int p = 0; p < kGPF; ++p) ld(p, p);
    int64_t s0 = 0;
    for (; s0 + kGPF <= nsteps; s0 += kGPF) {
#pragma unroll
      for (int p = 0; p < kGPF; ++p) {
#pragma unroll
        for (int mt = 0; mt < kGMT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = M::mma(a[p][mt], e[p][nt], acc[mt][nt]);
        ld(p, s0 + p + kGPF);
      }
    }
#pragma unroll
    for (int p = 0; p < kGPF - 1; ++p)
      if (s0 + p < nsteps) {
#pragma unroll
        for (int mt = 0; mt < kGMT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = M::mma(a[p][mt], e[p][nt], acc[mt][nt]);
      }
  }
  T* out = P + (int64_t)split * m * L;
#pragma unroll
  for (int mt = 0; mt < kGMT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = row0 + 16 * mt + M::row(lane, r);
      if (row < m) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) out[row * L + 16 * nt + i] = acc[mt][nt][r];
      }
    }
}

static int genv(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

// K splits of the flagged-row list: about kGatherBlocks workgroups (GLX_GATHER_BLOCKS)
static constexpr int kGatherBlocks = 512;
int gather_split(int64_t m) {
  const int64_t gx = (m + kGRows - 1) / kGRows;
  int64_t s = genv("GLX_GATHER_BLOCKS", kGatherBlocks) / gx;
  if (s < 1) s = 1;
  if (s > 32) s = 32;
  return (int)s;
}

bool gather_ok(int64_t n, int64_t l) { return (l == 16 || l == 32) && n <= 65535; }

template <typename T>
void launch_transpose(const T* A, T* At, int64_t m, int64_t n, hipStream_t st) {
  const dim3 grid((unsigned)((n + 63) / 64), (unsigned)((m + 63) / 64));
  hipLaunchKernelGGL(k_transpose<T>, grid, dim3(256), 0, st, A, At, m, n);
}

template <typename T>
void launch_at_gather(const T* At, const T* E, const uint8_t* zf, int64_t m, int64_t n, int64_t l,
                      T* P, int S, hipStream_t st) {
  if (!gather_ok(n, l)) throw Error{GLX_E_INVALID, "A e gather: needs l in {16, 32} and n < 65536"};
  const int gx = (int)((m + kGRows - 1) / kGRows);
  const size_t lds = sizeof(unsigned short) * (size_t)n;
  static const int pf = genv("GLX_GATHER_PF", 8);
  auto go = [&](auto kern) {
    static bool attr = false;
    if (!attr) {   // the list exceeds the default 64 KiB dynamic LDS limit only past n = 32768
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 64);
      attr = true;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)(gx * S)), dim3(kGThreads), lds, st, At, E, zf, m, n, P,
                       S, gx);
  };
  if (l == 32) {
    if (pf == 4) go(k_at_gather<T, 2, 4>);
    else go(k_at_gather<T, 2, 8>);
  } else {
    if (pf == 4) go(k_at_gather<T, 1, 4>);
    else go(k_at_gather<T, 1, 8>);
  }
}

template void launch_transpose<double>(const double*, double*, int64_t, int64_t, hipStream_t);
template void launch_transpose<float>(const float*, float*, int64_t, int64_t, hipStream_t);
template void launch_at_gather<double>(const double*, const double*, const uint8_t*, int64_t, int64_t,
                                       int64_t, double*, int, hipStream_t);
template void launch_at_gather<float>(const float*, const float*, const uint8_t*, int64_t, int64_t,
                                      int64_t, float*, int, hipStream_t);

}  // namespace glx
