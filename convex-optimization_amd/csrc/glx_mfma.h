// glx_mfma.h — pieces shared by the dense-product kernels (kernels_gemm.hip: A @ X,
// kernels_axdma.hip: the LDS-DMA A @ X tile, kernels_atr.hip: A^T R): MFMA operand types and
// maps, load helpers, the (row block, K split) decode of a 1-D A @ X grid, and host-side plan
// helpers.
#pragma once

#include <cstdlib>

#include "glx.h"
#include "glx_device.h"

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
// of the K chunks (CK = 4E values of k per chunk); the block's 4 waves split the block's chunks;
// blockIdx.y = K split. PF chunks are kept in flight per wave (a register ring, statically
// indexed). P[blockIdx.y][m][16*NT] receives the block's partial.
// ------------------------------------------------------------------------------------------
__device__ inline bool gate_live(const int* gate, int epoch) { return gate == nullptr || *gate == epoch; }

template <typename T, bool NTL>
__device__ inline typename MF<T>::vec_t load_vec(const T* p) {
  typedef typename MF<T>::vec_t V;
  if constexpr (NTL) return __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
  else return *reinterpret_cast<const V*>(p);
}

// NSRC right-hand sides X0..X2 (each n x 16NT) share every loaded A fragment: the batched
// products of the next iteration (e.g. A @ [z | p_thr]) cost one pass over A.
// P[src][S][m][16NT]. NTL: A streamed with non-temporal loads (keeps X resident in L2).
// Logical (row block, K split) of a 1-D launch. xmap = 1 groups K splits by XCD: blocks are
// observed to be dealt round-robin over the 8 XCDs (lin % 8 shares an L2), so split s is
// given to XCD group s (S | 8: 8/S XCDs per split; 8 | S: S/8 splits per XCD). Each XCD's L2
// then holds only its own slice of X instead of all of it. Placement is a speed matter only:
// any other placement computes the same result.
__device__ inline bool ax_block(int xmap, int gx, int S, int& bx, int& by, int shift = 0) {
  const int lin = (int)blockIdx.x - shift;   // shift 1: workgroup 0 carries the scalar packet
  if (xmap & 1) {
    const int xcd = lin & 7, slot = lin >> 3;
    if (S <= 8) {
      const int G = 8 / S;
      by = xcd / G;
      bx = slot * G + (xcd % G);
    } else {
      by = xcd + 8 * (slot / gx);
      bx = slot % gx;
    }
    return bx < gx && by < S;
  }
  bx = lin % gx;
  by = lin / gx;
  return true;
}
static inline int ax_grid(int xmap, int gx, int S) {
  if ((xmap & 1) && S <= 8) {
    const int G = 8 / S;
    return ((gx + G - 1) / G) * G * S;
  }
  return gx * S;
}
static inline int ax_xmap_ok(int S) { return (S <= 8) ? (8 % S == 0) : (S % 8 == 0); }
// bit 1 of xmap (the LDS tiles, kinds 5 and 8): row block bx walks its K chunks starting at
// chunk bx * nch / gx (mod nch) instead of 0. Blocks advance in near lockstep, so without it
// every workgroup reads the same few column offsets of its rows at any moment (rows are
// 128 KiB apart at NS); rotated, the chip's reads spread over the whole row width. Changes the
// summation order of a block's partial, not its determinism (GLX_AX_ROT=0: off).
__device__ inline int64_t ax_rot(int xmap, int bx, int gx, int64_t nch) {
  return (xmap & 2) ? ((int64_t)bx * nch) / gx : 0;
}
static inline int ax_xmap_flags(const GemmPlan& p, int S) {
  return ((p.ax_xmap & 1) && ax_xmap_ok(S) ? 1 : 0) | (p.ax_xmap & 2);
}

// A lane (i, q) of a row step feeds the four MFMAs e = 0..3 with row q of A at panel columns
// atr_col(i, e); MFMA e's output row i is then G row col0 + atr_col(i, e). f64: columns
// {2i, 2i+1} and {32 + 2i, 33 + 2i}, so each of the two 16-B loads of a wave-instruction covers
// 256 contiguous bytes of each of its four rows (the streaming probe, scripts/stream_probe.hip:
// 6.1 TB/s for the 4i..4i+3 form, whose loads leave every other 16 B of a 512-B span to the
// next instruction, against 6.3-7.1 TB/s for contiguous 256/512-B pieces). f32: one 16-B load
// already covers columns 4i..4i+3.
template <typename T>
__device__ inline int atr_col(int i, int e) {
  if constexpr (sizeof(T) == 8) return (e >> 1) * 32 + 2 * i + (e & 1);
  else return 4 * i + e;
}
template <typename T, bool NTL> struct Load4;
template <bool NTL> struct Load4<double, NTL> {
  __device__ static inline void go(const double* p, double (&a)[4]) {   // p = row + col0 + 2i
    const d2_t v0 = load_vec<double, NTL>(p);
    const d2_t v1 = load_vec<double, NTL>(p + 32);
    a[0] = v0[0]; a[1] = v0[1]; a[2] = v1[0]; a[3] = v1[1];
  }
};
template <bool NTL> struct Load4<float, NTL> {
  __device__ static inline void go(const float* p, float (&a)[4]) {
    const f4_t v = load_vec<float, NTL>(p);
    a[0] = v[0]; a[1] = v[1]; a[2] = v[2]; a[3] = v[3];
  }
};

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

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
static inline int64_t clampi(int64_t v, int64_t lo, int64_t hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}
static constexpr int64_t kTargetWaves = 2048;   // 8 waves per CU on 256 CUs
static constexpr int kMaxSplit = 64;

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

// Occupancy pad (tuning experiment, GLX_AX_LDS_PAD / GLX_ATR_LDS_PAD bytes): unused dynamic
// LDS added to a launch so that at most one workgroup fits per CU — a 256-workgroup grid can
// then not double up on some CUs while others idle. 0 = off (the default).
template <typename K>
static size_t lds_pad(K kernel, const char* env) {
  const int pad = env_int(env, 0);
  if (pad <= 0) return 0;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, pad);
  return (size_t)pad;
}

// Defaults chosen by the sweep in scripts/kbench.py on MI355X.
// ax code: kind*1000 + MT*100 + PF*10 + NTL (kind 1 = direct row loads, 2 = quad + bpermute).
// kind 5 (X staged in LDS) code: 5 MT PF VPL WAVES. Kind-5 defaults fall back to the register

}  // namespace glx
// In-kernel clock probe (diagnostic builds only: scripts/clock_probe.sh compiles the library with
// -DGLX_CLOCK_PROBE; the shipped library has no stamps). Thread 0 of every workgroup stamps the
// shader clock (s_memtime) and the 100 MHz constant clock (s_memrealtime) at kernel entry (k 0),
// main-loop start (1) and end (2), kernel end (3), and in A^T R the end of the block's LDS
// reduction (4) and of the fused epilogue's row work (5), of the two passes over A, into a buffer of the code object (one per translation unit) that no
// kernel reads; the last launch's stamps are read back by glx_probe_clock_ax / _atr
// (kernels_axdma.hip, kernels_atr.hip). MI355X_MICROARCH.md "DVFS give-back" (6).
#ifdef GLX_CLOCK_PROBE
namespace glx {
static __device__ unsigned long long g_clk[2048][12];   // [block][stamp pair k: 2k, 2k+1]
}
#define GLX_CLK(k)                                                                          \
  do {                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < 2048) {                                            \
      glx::g_clk[blockIdx.x][2 * (k)] = __builtin_amdgcn_s_memtime();                       \
      glx::g_clk[blockIdx.x][2 * (k) + 1] = __builtin_amdgcn_s_memrealtime();               \
    }                                                                                       \
  } while (0)
#define GLX_CLK_READER(fn)                                                                  \
  extern "C" int fn(unsigned long long* out) {                                              \
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(glx::g_clk), sizeof(glx::g_clk), 0,          \
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;                \
  }
#else
#define GLX_CLK(k) do {} while (0)
#define GLX_CLK_READER(fn)
#endif


