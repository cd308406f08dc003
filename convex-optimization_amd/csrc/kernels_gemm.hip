// kernels_gemm.hip — the two dense contractions of the prox-grad iteration on CDNA4 (gfx950).
//
//   A @ X   (reference: gl_ProxGD_primal.py:25,61,129 — `A @ x`):   M = m, K = n, N = l
//   A^T R   (reference: gl_ProxGD_primal.py:129 — `A.T @ (...)`):  M = n, K = m, N = l
//
// Both stream A (m x n, row-major, 1 GiB at the north-star size) once per launch. At
// l = 16/32 their arithmetic intensity (l/4 flop/B fp64, l/2 fp32) is below the MI355X ridge,
// so the kernels are built to keep HBM busy: 16-byte loads, many bytes in flight per CU, and
// v_mfma_f64_16x16x4f64 / v_mfma_f32_16x16x4f32 so the multiply-adds never become the limit.
//
// MFMA 16x16x4 operand maps (cdna_hip_programming.md §3): lane l supplies A_op[l&15][l>>4] and
// B_op[l>>4][l&15]; the C/D map is row=(l>>4)+4r (f64) or 4(l>>4)+r (f32), col=l&15.
//
// A @ X: the K index sits on l>>4, i.e. the 16 lanes of a k-slice live in 16 different rows of
// A. Each lane therefore loads 16 contiguous bytes (E = 2 f64 / 4 f32 consecutive k) of its
// row and feeds them to E consecutive MFMAs: MFMA e covers k = k0 + 4*E*... (k permuted inside a
// 4E-wide chunk; X is gathered with the same permutation, so the sum is unchanged).
//   kind 1 — each lane loads its own row (lane -> row l&15, chunk l>>4);
//   kind 2 — quad-coalesced loads (lane -> row L>>2, chunk L&3: 64 contiguous bytes per quad)
//            and a ds_bpermute to the MFMA layout (no LDS storage, no barriers).
// A^T R: the K index (rows of A) is on l>>4 and the 16-wide M index (columns of A) on l&15,
// so lanes 0..15 read consecutive columns: a lane loads 4 consecutive columns (32 B f64 /
// 16 B f32) of one row and feeds 4 MFMAs whose output rows are columns c0+4i+e.
//
// Split-K: each workgroup is 4 waves; the waves of a workgroup split the K range and are
// summed through LDS in a fixed order, and workgroups along gridDim.y write partial slabs that
// the consumer sums in slab order — the result is deterministic run to run.
#include "glx_internal.h"

namespace glx {

typedef double d2_t __attribute__((ext_vector_type(2)));
typedef double d4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));

template <typename T> struct MF;
template <> struct MF<double> {
  typedef d4_t acc_t;
  typedef d2_t vec_t;
  static constexpr int E = 2;
  __device__ static inline acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __device__ static inline int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <> struct MF<float> {
  typedef f4_t acc_t;
  typedef f4_t vec_t;
  static constexpr int E = 4;
  __device__ static inline acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static inline int row(int lane, int r) { return ((lane >> 4) << 2) + r; }
};

template <typename V>
__device__ inline V bpermute_vec(V v, int src_lane) {
  constexpr int ND = sizeof(V) / 4;
  union U { V v; int d[ND]; };
  U in, out;
  in.v = v;
#pragma unroll
  for (int j = 0; j < ND; ++j) out.d[j] = __builtin_amdgcn_ds_bpermute(src_lane << 2, in.d[j]);
  return out.v;
}

// ------------------------------------------------------------------------------------------
// A @ X on MFMA: block = 4 waves; a wave owns MT 16-row tiles x NT 16-col tiles over its share
// of the K chunks; the block's 4 waves split the block's chunks; blockIdx.y = K split.
// P[blockIdx.y][m][16*NT] receives the block's partial.
// ------------------------------------------------------------------------------------------
template <typename T, int MT, int NT, bool QUAD>
__global__ __launch_bounds__(256) void k_ax_mfma(const T* __restrict__ A, const T* __restrict__ X,
                                                 T* __restrict__ P, int64_t m, int64_t n,
                                                 int64_t chunks, int S,
                                                 const int* __restrict__ gate) {
  typedef MF<T> M;
  typedef typename M::vec_t V;
  typedef typename M::acc_t C;
  constexpr int E = M::E;
  constexpr int CK = 4 * E;   // k per chunk
  constexpr int L = 16 * NT;  // == l
  if (gate != nullptr && *gate == 0) return;
  __shared__ C red[MT * NT][64];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * (16 * MT);
  const int64_t W = (int64_t)S * 4;
  const int64_t w = (int64_t)blockIdx.y * 4 + wave;
  const int64_t cb = chunks * w / W, ce = chunks * (w + 1) / W;

  const int lrow = QUAD ? (lane >> 2) : i;
  const int lchk = QUAD ? (lane & 3) : q;
  const int src = i * 4 + q;  // QUAD: lane holding (row i, chunk q)
  const T* ap[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int64_t r = row0 + mt * 16 + lrow;
    r = r < m ? r : m - 1;
    ap[mt] = A + r * n + cb * CK + (int64_t)lchk * E;
  }
  const T* xp = X + (cb * CK + (int64_t)q * E) * L + i;

  C acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = C{};

  V a[MT];
  T xb[E][NT];
  if (cb < ce) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[mt] = *reinterpret_cast<const V*>(ap[mt]);
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) xb[e][nt] = xp[e * L + nt * 16];
  }
  for (int64_t c = cb; c < ce; ++c) {
    // prefetch chunk c+1 (re-read chunk c on the last trip: harmless, keeps the loop branch-free)
    const int64_t adv = (c + 1 < ce) ? CK : 0;
    V an[MT];
    T xn[E][NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      ap[mt] += adv;
      an[mt] = *reinterpret_cast<const V*>(ap[mt]);
    }
    xp += adv * L;
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) xn[e][nt] = xp[e * L + nt * 16];

    V av[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) av[mt] = QUAD ? bpermute_vec(a[mt], src) : a[mt];
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = M::mma(av[mt][e], xb[e][nt], acc[mt][nt]);

#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[mt] = an[mt];
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) xb[e][nt] = xn[e][nt];
  }

  // fixed-order reduction of the 4 waves: ((w0 + w1) + w2) + w3
#pragma unroll
  for (int s = 1; s < 4; ++s) {
    __syncthreads();
    if (wave == s) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) red[mt * NT + nt][lane] = acc[mt][nt];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] += red[mt * NT + nt][lane];
    }
  }
  if (wave != 0) return;
  T* pout = P + (int64_t)blockIdx.y * m * L;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = row0 + mt * 16 + M::row(lane, r);
      if (row < m) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) pout[row * L + nt * 16 + i] = acc[mt][nt][r];
      }
    }
}

// ------------------------------------------------------------------------------------------
// A^T R on MFMA: a wave owns 64 columns of A (= 64 rows of G) x NT 16-col tiles of G; the
// 4 waves of a block split the block's row range; blockIdx.y = row split. Needs n % 64 == 0,
// m % 4 == 0. Gp[blockIdx.y][n][16*NT].
// ------------------------------------------------------------------------------------------
template <typename T> struct Load4;
template <> struct Load4<double> {
  __device__ static inline void go(const double* p, double (&a)[4]) {
    const d2_t v0 = *reinterpret_cast<const d2_t*>(p);
    const d2_t v1 = *reinterpret_cast<const d2_t*>(p + 2);
    a[0] = v0[0]; a[1] = v0[1]; a[2] = v1[0]; a[3] = v1[1];
  }
};
template <> struct Load4<float> {
  __device__ static inline void go(const float* p, float (&a)[4]) {
    const f4_t v = *reinterpret_cast<const f4_t*>(p);
    a[0] = v[0]; a[1] = v[1]; a[2] = v[2]; a[3] = v[3];
  }
};

template <typename T, int NT>
__global__ __launch_bounds__(256) void k_atr_mfma(const T* __restrict__ A, const T* __restrict__ R,
                                                  T* __restrict__ Gp, int64_t m, int64_t n, int S) {
  typedef MF<T> M;
  typedef typename M::acc_t C;
  constexpr int L = 16 * NT;
  __shared__ C red[4 * NT][64];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int64_t col0 = (int64_t)blockIdx.x * 64;
  const int64_t steps = m / 4;
  const int64_t W = (int64_t)S * 4;
  const int64_t w = (int64_t)blockIdx.y * 4 + wave;
  const int64_t sb = steps * w / W, se = steps * (w + 1) / W;

  const T* ap = A + (sb * 4 + q) * n + col0 + 4 * i;
  const T* rp = R + (sb * 4 + q) * L + i;

  C acc[4][NT];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[e][nt] = C{};

  T a[4], rb[NT];
  if (sb < se) {
    Load4<T>::go(ap, a);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) rb[nt] = rp[nt * 16];
  }
  for (int64_t s = sb; s < se; ++s) {
    const int64_t adv = (s + 1 < se) ? 4 : 0;
    ap += adv * n;
    rp += adv * L;
    T an[4], rn[NT];
    Load4<T>::go(ap, an);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) rn[nt] = rp[nt * 16];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[e][nt] = M::mma(a[e], rb[nt], acc[e][nt]);
#pragma unroll
    for (int e = 0; e < 4; ++e) a[e] = an[e];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) rb[nt] = rn[nt];
  }

#pragma unroll
  for (int s = 1; s < 4; ++s) {
    __syncthreads();
    if (wave == s) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) red[e * NT + nt][lane] = acc[e][nt];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[e][nt] += red[e * NT + nt][lane];
    }
  }
  if (wave != 0) return;
  T* gout = Gp + (int64_t)blockIdx.y * n * L;
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t grow = col0 + 4 * M::row(lane, r) + e;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) gout[grow * L + nt * 16 + i] = acc[e][nt][r];
    }
}

// ------------------------------------------------------------------------------------------
// VALU fallback for small l (GEMV-like, l <= 8 per pass) and ragged shapes.
// A @ X: a wave owns RW rows and one K split; lanes stride the row with (16-byte) loads,
// each X element is reused across the RW rows; columns [c0, c0+LB) of the output.
// ------------------------------------------------------------------------------------------
__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

template <typename T, int LB, int RW, bool VEC>
__global__ __launch_bounds__(256) void k_ax_valu(const T* __restrict__ A, const T* __restrict__ X,
                                                 T* __restrict__ P, int64_t m, int64_t n,
                                                 int64_t l, int c0, int S,
                                                 const int* __restrict__ gate) {
  constexpr int E = VEC ? (16 / (int)sizeof(T)) : 1;
  if (gate != nullptr && *gate == 0) return;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * RW;
  if (row0 >= m) return;  // wave-uniform; no barriers below
  const int s = blockIdx.y;
  const int64_t nv = n / E;
  const int64_t kb = E * (nv * s / S);
  const int64_t ke = (s == S - 1) ? n : E * (nv * (s + 1) / S);
  const int nc = (int)((l - c0) < LB ? (l - c0) : LB);

  const T* arow[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    int64_t rr = row0 + r;
    rr = rr < m ? rr : m - 1;
    arow[r] = A + rr * n;
  }
  T acc[RW][LB];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int c = 0; c < LB; ++c) acc[r][c] = T(0);

  for (int64_t k = kb + (int64_t)lane * E; k < ke; k += 64 * E) {
    T a[RW][E];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      if constexpr (VEC) {
        typedef typename MF<T>::vec_t V;
        const V v = *reinterpret_cast<const V*>(arow[r] + k);
#pragma unroll
        for (int e = 0; e < E; ++e) a[r][e] = v[e];
      } else {
        a[r][0] = arow[r][k];
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      T xv[LB];
#pragma unroll
      for (int c = 0; c < LB; ++c) xv[c] = (c < nc) ? X[(k + e) * l + c0 + c] : T(0);
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int c = 0; c < LB; ++c) acc[r][c] = __builtin_fma(a[r][e], xv[c], acc[r][c]);
    }
  }
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int c = 0; c < LB; ++c) acc[r][c] = wave_sum(acc[r][c]);
  if (lane == 0) {
    T* pout = P + (int64_t)s * m * l;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int64_t row = row0 + r;
      if (row < m) {
#pragma unroll
        for (int c = 0; c < LB; ++c)
          if (c < nc) pout[row * l + c0 + c] = acc[r][c];
      }
    }
  }
}

// A^T R on VALU: a thread owns E consecutive columns of A over a row range; R[row][c0..c0+LB)
// is wave-uniform (scalar loads). Gp[blockIdx.y][n][l].
template <typename T, int LB, bool VEC>
__global__ __launch_bounds__(256) void k_atr_valu(const T* __restrict__ A, const T* __restrict__ R,
                                                  T* __restrict__ Gp, int64_t m, int64_t n,
                                                  int64_t l, int c0, int S) {
  constexpr int E = VEC ? (16 / (int)sizeof(T)) : 1;
  const int64_t col = ((int64_t)blockIdx.x * 256 + threadIdx.x) * E;
  const int s = blockIdx.y;
  const int64_t rb = m * s / S, re = m * (s + 1) / S;
  const int nc = (int)((l - c0) < LB ? (l - c0) : LB);
  const bool active = col < n;
  const int64_t ccol = active ? col : 0;

  T acc[E][LB];
#pragma unroll
  for (int e = 0; e < E; ++e)
#pragma unroll
    for (int c = 0; c < LB; ++c) acc[e][c] = T(0);

  const T* ap = A + rb * n + ccol;
  const T* rp = R + rb * l + c0;
#pragma unroll 4
  for (int64_t row = rb; row < re; ++row) {
    T a[E];
    if constexpr (VEC) {
      typedef typename MF<T>::vec_t V;
      const V v = *reinterpret_cast<const V*>(ap);
#pragma unroll
      for (int e = 0; e < E; ++e) a[e] = v[e];
    } else {
      a[0] = *ap;
    }
    T rv[LB];
#pragma unroll
    for (int c = 0; c < LB; ++c) rv[c] = (c < nc) ? rp[c] : T(0);
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int c = 0; c < LB; ++c) acc[e][c] = __builtin_fma(a[e], rv[c], acc[e][c]);
    ap += n;
    rp += l;
  }
  if (!active) return;
  T* gout = Gp + (int64_t)s * n * l;
#pragma unroll
  for (int e = 0; e < E; ++e)
#pragma unroll
    for (int c = 0; c < LB; ++c)
      if (c < nc) gout[(col + e) * l + c0 + c] = acc[e][c];
}

// ------------------------------------------------------------------------------------------
// planning + launch
// ------------------------------------------------------------------------------------------
static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
static inline int64_t clampi(int64_t v, int64_t lo, int64_t hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}
static constexpr int64_t kTargetWaves = 2048;   // 8 waves per CU on 256 CUs
static constexpr int kMaxSplit = 64;

GemmPlan make_plan(int esize, int64_t m, int64_t n, int64_t l, int ax_variant) {
  GemmPlan p{};
  p.esize = esize;
  p.m = m; p.n = n; p.l = l;
  const int E = 16 / esize;
  const bool mfma_l = (l == 16 || l == 32);
  // ---- A @ X ----
  const bool ax_mfma_ok = mfma_l && (n % (4 * E) == 0);
  if (ax_variant == 3 || !ax_mfma_ok) {
    p.ax_kind = 3;
    p.ax_lb = l >= 8 ? 8 : (l >= 4 ? 4 : (l >= 2 ? 2 : 1));
    if (l == 3) p.ax_lb = 4;
    if (l > 4 && l < 8) p.ax_lb = 8;
    p.ax_vec = (n % E == 0) ? 1 : 0;
    const int64_t waves = cdiv(m, 4);                    // RW = 4 rows per wave
    const int64_t kunits = n / (64 * (p.ax_vec ? E : 1)); // 64-lane strides per row
    p.ax_S = (int)clampi(cdiv(kTargetWaves, waves), 1, std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, kunits / 4)));
  } else {
    p.ax_kind = (ax_variant == 2) ? 2 : 1;
    const int64_t blocks = cdiv(m, 64);                   // MT = 4 -> 64 rows per block
    const int64_t chunks = n / (4 * E);
    p.ax_S = (int)clampi(cdiv(kTargetWaves, blocks * 4), 1,
                         std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, chunks / 16)));
  }
  // ---- A^T R ----
  const bool atr_mfma_ok = mfma_l && (n % 64 == 0) && (m % 4 == 0);
  if (ax_variant == 3 || !atr_mfma_ok) {
    p.atr_kind = 3;
    p.atr_lb = l >= 8 ? 8 : (l >= 4 ? 4 : (l >= 2 ? 2 : 1));
    if (l == 3) p.atr_lb = 4;
    if (l > 4 && l < 8) p.atr_lb = 8;
    p.atr_vec = (n % E == 0) ? 1 : 0;
    const int64_t cols_per_block = 256 * (p.atr_vec ? E : 1);
    const int64_t blocks = cdiv(n, cols_per_block);
    p.atr_S = (int)clampi(cdiv(kTargetWaves / 4, blocks), 1, std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, m / 16)));
  } else {
    p.atr_kind = 1;
    const int64_t blocks = n / 64;
    const int64_t steps = m / 4;
    p.atr_S = (int)clampi(cdiv(kTargetWaves, blocks * 4), 1,
                          std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, steps / 16)));
  }
  return p;
}

template <typename T, int LB>
static void ax_valu_lb(const GemmPlan& p, const T* A, const T* X, T* P, const int* gate,
                       hipStream_t st) {
  const dim3 grid((unsigned)cdiv(cdiv(p.m, 4), 4), (unsigned)p.ax_S);
  for (int64_t c0 = 0; c0 < p.l; c0 += LB) {
    if (p.ax_vec)
      hipLaunchKernelGGL((k_ax_valu<T, LB, 4, true>), grid, dim3(256), 0, st, A, X, P, p.m, p.n,
                         p.l, (int)c0, p.ax_S, gate);
    else
      hipLaunchKernelGGL((k_ax_valu<T, LB, 4, false>), grid, dim3(256), 0, st, A, X, P, p.m, p.n,
                         p.l, (int)c0, p.ax_S, gate);
  }
}

template <typename T>
void launch_ax(const GemmPlan& p, const T* A, const T* X, T* P, const int* gate, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  if (p.ax_kind == 3) {
    switch (p.ax_lb) {
      case 1: ax_valu_lb<T, 1>(p, A, X, P, gate, st); break;
      case 2: ax_valu_lb<T, 2>(p, A, X, P, gate, st); break;
      case 4: ax_valu_lb<T, 4>(p, A, X, P, gate, st); break;
      default: ax_valu_lb<T, 8>(p, A, X, P, gate, st); break;
    }
    return;
  }
  const dim3 grid((unsigned)cdiv(p.m, 64), (unsigned)p.ax_S);
  const int64_t chunks = p.n / (4 * E);
  if (p.l == 16) {
    if (p.ax_kind == 2)
      hipLaunchKernelGGL((k_ax_mfma<T, 4, 1, true>), grid, dim3(256), 0, st, A, X, P, p.m, p.n, chunks, p.ax_S, gate);
    else
      hipLaunchKernelGGL((k_ax_mfma<T, 4, 1, false>), grid, dim3(256), 0, st, A, X, P, p.m, p.n, chunks, p.ax_S, gate);
  } else {
    if (p.ax_kind == 2)
      hipLaunchKernelGGL((k_ax_mfma<T, 4, 2, true>), grid, dim3(256), 0, st, A, X, P, p.m, p.n, chunks, p.ax_S, gate);
    else
      hipLaunchKernelGGL((k_ax_mfma<T, 4, 2, false>), grid, dim3(256), 0, st, A, X, P, p.m, p.n, chunks, p.ax_S, gate);
  }
}

template <typename T, int LB>
static void atr_valu_lb(const GemmPlan& p, const T* A, const T* R, T* Gp, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int64_t cols_per_block = 256 * (p.atr_vec ? E : 1);
  const dim3 grid((unsigned)cdiv(p.n, cols_per_block), (unsigned)p.atr_S);
  for (int64_t c0 = 0; c0 < p.l; c0 += LB) {
    if (p.atr_vec)
      hipLaunchKernelGGL((k_atr_valu<T, LB, true>), grid, dim3(256), 0, st, A, R, Gp, p.m, p.n,
                         p.l, (int)c0, p.atr_S);
    else
      hipLaunchKernelGGL((k_atr_valu<T, LB, false>), grid, dim3(256), 0, st, A, R, Gp, p.m, p.n,
                         p.l, (int)c0, p.atr_S);
  }
}

template <typename T>
void launch_atr(const GemmPlan& p, const T* A, const T* R, T* Gp, hipStream_t st) {
  if (p.atr_kind == 3) {
    switch (p.atr_lb) {
      case 1: atr_valu_lb<T, 1>(p, A, R, Gp, st); break;
      case 2: atr_valu_lb<T, 2>(p, A, R, Gp, st); break;
      case 4: atr_valu_lb<T, 4>(p, A, R, Gp, st); break;
      default: atr_valu_lb<T, 8>(p, A, R, Gp, st); break;
    }
    return;
  }
  const dim3 grid((unsigned)(p.n / 64), (unsigned)p.atr_S);
  if (p.l == 16)
    hipLaunchKernelGGL((k_atr_mfma<T, 1>), grid, dim3(256), 0, st, A, R, Gp, p.m, p.n, p.atr_S);
  else
    hipLaunchKernelGGL((k_atr_mfma<T, 2>), grid, dim3(256), 0, st, A, R, Gp, p.m, p.n, p.atr_S);
}

template void launch_ax<double>(const GemmPlan&, const double*, const double*, double*, const int*, hipStream_t);
template void launch_ax<float>(const GemmPlan&, const float*, const float*, float*, const int*, hipStream_t);
template void launch_atr<double>(const GemmPlan&, const double*, const double*, double*, hipStream_t);
template void launch_atr<float>(const GemmPlan&, const float*, const float*, float*, hipStream_t);

}  // namespace glx
