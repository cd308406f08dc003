// kernels_gemv.hip — the l = 1 descent iteration (SGD / GD, config C4) in ONE pass over A.
//
// Reference (gl_SGD_primal.py:51-57, gl_GD_primal.py:59-63): every iteration needs
//   r1 = A x - b          (the objective of x, recorded before the step)
//   r2 = A thr(x) - b     (the subgradient's residual, :93 thresholds x first)
//   G  = A^T r2
// which the two-kernel path streams A twice for (A @ [x | thr(x)], then A^T r2). With l = 1 each
// row of A is a dot product away from its residual: a workgroup that owns a range of rows keeps
// a few whole rows in registers, reduces their dot products with x and thr(x) over the
// workgroup, and immediately adds row * r2 into its private copy of G — the second use of the
// row costs no HBM traffic. A is read once per iteration, halving the iteration's bytes.
//
// Layout: 512 threads (8 waves), thread t holds the 16-B column vectors t, t + 512, ... of x,
// thr(x), its G partial and of every row in flight (VPT vectors). Rows are processed RB at a
// time and double-buffered: the loads of rows i + RB .. i + 2RB - 1 are issued before the dot
// products of rows i .. i + RB - 1. Every sum has a fixed order (lane order, wave shuffle tree,
// waves 0..7, rows in order, workgroups in order), so results are deterministic.
// Outputs: Gp[workgroup][n] (summed by k_sum_cols), out[0] = sum r1^2, out[1] = sum r2^2, and
// (optionally) fh[0] = 0.5 out[0] + mu * (*rn) — the device-side objective record.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "glx_device.h"

namespace glx {

namespace {
typedef double gd2 __attribute__((ext_vector_type(2)));
typedef float gf4 __attribute__((ext_vector_type(4)));
template <typename T> struct GV;
template <> struct GV<double> { typedef gd2 v; static constexpr int E = 2; };
template <> struct GV<float> { typedef gf4 v; static constexpr int E = 4; };

constexpr int kGemvThreads = 512;
constexpr int kGemvWaves = kGemvThreads / 64;
constexpr int kGemvMaxBlocks = 256;    // one 8-wave workgroup per CU
}  // namespace

// RB rows per batch (two batches in flight): 2 for VPT <= 4, 1 for VPT = 8 (register budget of
// two waves per SIMD: 2 x RB x VPT row vectors + x, thr(x) and G).
// NT: A read with the non-temporal policy. A workgroup streams one contiguous range of rows in
// whole 1-KiB wave-instructions, the shape the streaming probe reads at 7.1-7.2 TB/s
// non-temporal against 6.1-6.2 TB/s default (scripts/stream_probe.hip, "chunk"); used when A
// cannot stay in the Infinity Cache anyway (kGemvNtBytes).
template <typename T, int VPT, int RB, bool NT>
__global__ __launch_bounds__(kGemvThreads) void k_gemv_pair_fused(
    const T* __restrict__ A, const T* __restrict__ x, const T* __restrict__ xt,
    const T* __restrict__ b, T* __restrict__ Gp, int64_t m, int64_t n, double* fh, double fh_mu,
    const double* rn, Red red) {
  typedef typename GV<T>::v V;
  constexpr int E = GV<T>::E;
  constexpr int NW = kGemvWaves;
  __shared__ double part[2][RB][2][NW];   // [batch parity][row][x | thr(x)][wave]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int64_t nv = n / E;
  const int64_t r0 = m * blockIdx.x / gridDim.x, r1 = m * (blockIdx.x + 1) / gridDim.x;
  const int64_t nrows = r1 - r0;

  V xv[VPT], xtv[VPT], g[VPT];
  int64_t col[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t v = tid + (int64_t)kGemvThreads * k;
    const bool on = v < nv;
    col[k] = (on ? v : nv - 1) * E;   // clamped: loads stay in bounds and unpredicated
    xv[k] = on ? *reinterpret_cast<const V*>(x + col[k]) : V{};
    xtv[k] = on ? *reinterpret_cast<const V*>(xt + col[k]) : V{};
    g[k] = V{};
  }

  V a[2][RB][VPT];
  auto load_batch = [&](V (&dst)[RB][VPT], int64_t i0) {
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      int64_t i = i0 + r;
      i = i < nrows ? i : nrows - 1;
      const T* rowp = A + (r0 + i) * n;
#pragma unroll
      for (int k = 0; k < VPT; ++k)
        dst[r][k] = NT ? __builtin_nontemporal_load(reinterpret_cast<const V*>(rowp + col[k]))
                       : *reinterpret_cast<const V*>(rowp + col[k]);
    }
  };

  double s1 = 0.0, s2 = 0.0;   // thread 0: sums of r1^2, r2^2 in row order
  // one batch: dot products, workgroup reduction, residuals, G += row * r2
  auto step = [&](V (&rows)[RB][VPT], int par, int64_t i0) {
    double d1[RB], d2[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      T p1 = T(0), p2 = T(0);
#pragma unroll
      for (int k = 0; k < VPT; ++k)
#pragma unroll
        for (int e = 0; e < E; ++e) {
          p1 = p1 + rows[r][k][e] * xv[k][e];
          p2 = p2 + rows[r][k][e] * xtv[k][e];
        }
      d1[r] = (double)p1;
      d2[r] = (double)p2;
    }
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        d1[r] += __shfl_xor(d1[r], off);
        d2[r] += __shfl_xor(d2[r], off);
      }
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        part[par][r][0][wave] = d1[r];
        part[par][r][1][wave] = d2[r];
      }
    }
    __syncthreads();   // part[par] is rewritten two batches later, after the next barrier
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (i0 + r >= nrows) break;   // workgroup-uniform
      const double q1 = waves_combine<NW>(OP_SUM, part[par][r][0]);
      const double q2 = waves_combine<NW>(OP_SUM, part[par][r][1]);
      const T bi = b[r0 + i0 + r];
      // the residual in the dtype of A, as NumPy forms (A @ x) - b
      const T e1 = (T)q1 - bi, e2 = (T)q2 - bi;
      if (tid == 0) {
        s1 += (double)e1 * (double)e1;
        s2 += (double)e2 * (double)e2;
      }
#pragma unroll
      for (int k = 0; k < VPT; ++k)
#pragma unroll
        for (int e = 0; e < E; ++e) g[k][e] = g[k][e] + rows[r][k][e] * e2;
    }
  };

  if (nrows > 0) {
    load_batch(a[0], 0);
    int64_t i0 = 0;
    for (; i0 < nrows; i0 += 2 * RB) {
      load_batch(a[1], i0 + RB);
      step(a[0], 0, i0);
      load_batch(a[0], i0 + 2 * RB);
      step(a[1], 1, i0 + RB);
    }
  }
  // this workgroup's slab of G
  T* gout = Gp + (int64_t)blockIdx.x * n;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t v = tid + (int64_t)kGemvThreads * k;
    if (v < nv) *reinterpret_cast<V*>(gout + v * E) = g[k];
  }
  double acc[2] = {s1, s2};
  if (grid_reduce<2, 0x0u, NW>(acc, red) && fh != nullptr && tid == 0)
    fh[0] = 0.5 * red.out[0] + fh_mu * rn[0];
}

// G[j] = sum_{s < S} Gp[s][j] in slab order: a workgroup owns 64 columns, its 4 waves sum a
// quarter of the slabs each (loads issued 8 at a time), then ((w0 + w1) + w2) + w3 through LDS.
// Deterministic. For the S = number of fused workgroups slabs of k_gemv_pair_fused.
template <typename T>
__global__ __launch_bounds__(256) void k_sum_cols(const T* __restrict__ Gp, int S, T* __restrict__ G,
                                                  int64_t n) {
  __shared__ T sh[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + lane;
  const int64_t jc = j < n ? j : n - 1;
  const int sb = S * wave / 4, se = S * (wave + 1) / 4;
  T acc = T(0);
  int s = sb;
  for (; s + 8 <= se; s += 8) {
    T v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = Gp[(int64_t)(s + u) * n + jc];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = acc + v[u];
  }
  for (; s < se; ++s) acc = acc + Gp[(int64_t)s * n + jc];
  sh[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && j < n) G[j] = ((sh[0][lane] + sh[1][lane]) + sh[2][lane]) + sh[3][lane];
}

int gemv_fused_blocks(int esize, int64_t m, int64_t n, int64_t l) {
  const int E = 16 / esize;
  if (l != 1 || n % E != 0) return 0;
  const int64_t vpt = (n / E + kGemvThreads - 1) / kGemvThreads;
  if (vpt > 8) return 0;   // register budget of the 2 x RB row buffers
  int64_t blocks = (m + 7) / 8;   // >= 8 rows per workgroup
  if (blocks > kGemvMaxBlocks) blocks = kGemvMaxBlocks;
  return (int)std::max<int64_t>(1, blocks);
}

constexpr double kGemvNtBytes = 384.0 * 1024 * 1024;
template <typename T, int VPT, int RB>
static void gemv_go(int blocks, const T* A, const T* x, const T* xt, const T* b, T* Gp, int64_t m,
                    int64_t n, double* fh, double fh_mu, const double* rn, Red red, hipStream_t st) {
  static const int nt_env = [] {
    const char* e = std::getenv("GLX_GEMV_NT");
    return e ? std::atoi(e) : -1;
  }();
  const bool nt = nt_env >= 0 ? nt_env != 0 : (double)m * n * sizeof(T) > kGemvNtBytes;
  if (nt)
    glx_launch((k_gemv_pair_fused<T, VPT, RB, true>), dim3((unsigned)blocks),
                       dim3(kGemvThreads), 0, st, A, x, xt, b, Gp, m, n, fh, fh_mu, rn, red);
  else
    glx_launch((k_gemv_pair_fused<T, VPT, RB, false>), dim3((unsigned)blocks),
                       dim3(kGemvThreads), 0, st, A, x, xt, b, Gp, m, n, fh, fh_mu, rn, red);
}

template <typename T>
void launch_gemv_fused(int blocks, const T* A, const T* x, const T* xt, const T* b, T* Gp, int64_t m,
                       int64_t n, double* fh, double fh_mu, const double* rn, Red red,
                       hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int64_t vpt = (n / E + kGemvThreads - 1) / kGemvThreads;
  if (vpt <= 1) gemv_go<T, 1, 2>(blocks, A, x, xt, b, Gp, m, n, fh, fh_mu, rn, red, st);
  else if (vpt <= 2) gemv_go<T, 2, 2>(blocks, A, x, xt, b, Gp, m, n, fh, fh_mu, rn, red, st);
  else if (vpt <= 4) gemv_go<T, 4, 2>(blocks, A, x, xt, b, Gp, m, n, fh, fh_mu, rn, red, st);
  else gemv_go<T, 8, 1>(blocks, A, x, xt, b, Gp, m, n, fh, fh_mu, rn, red, st);
}

template <typename T>
void launch_sum_cols(const T* Gp, int S, T* G, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_sum_cols<T>, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, Gp, S, G, n);
}

#define GLX_GEMV_INST(T)                                                                           \
  template void launch_gemv_fused<T>(int, const T*, const T*, const T*, const T*, T*, int64_t,     \
                                     int64_t, double*, double, const double*, Red, hipStream_t); \
  template void launch_sum_cols<T>(const T*, int, T*, int64_t, hipStream_t);
GLX_GEMV_INST(double)
GLX_GEMV_INST(float)

}  // namespace glx
