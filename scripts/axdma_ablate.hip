// axdma_ablate.hip — where k_ax_dma's time goes at the north-star shape (timing only, the
// results are not checked): the tile's LDS-DMA loop (8 waves x 16 rows, KC = 32, 3-slot ring,
// non-temporal A) with its parts switched on one at a time: the DMA alone, + the per-chunk
// barrier, + the LDS operand reads, + the MFMAs. Best / median of 10 launches each.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/axdma_ablate scripts/axdma_ablate.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);  \
      return 1;                                                              \
    }                                                                        \
  } while (0)

typedef __attribute__((address_space(1))) void gv_t;
typedef __attribute__((address_space(3))) void lv_t;
typedef double d2_t __attribute__((ext_vector_type(2)));
typedef double d4_t __attribute__((ext_vector_type(4)));

constexpr int KC = 32, W = 8, NS = 3, L = 32;
constexpr int SLR = KC / 2, AW = 16 * KC * 8, NIA = AW / 1024, XS = KC * L * 8, SLOT = W * AW + XS;

// MODE bits: 1 barrier per chunk, 2 LDS reads, 4 MFMAs (on the read values, or on registers),
// 8 register operands change every chunk (random bits, as the loaded data would), 16 waits for
// the LDS reads but feeds the MFMAs from registers. clk[block] = in-kernel shader clock (MHz).
template <int MODE>
__global__ __launch_bounds__(512) void k_abl(const double* __restrict__ A, const double* __restrict__ X,
                                             double* __restrict__ P, int64_t m, int64_t n, int S,
                                             double* __restrict__ clk) {
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  __shared__ __attribute__((aligned(1024))) char lds[NS * SLOT];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int64_t gx = m / (16 * W), chunks = n / KC;
  const int64_t bx = blockIdx.x % gx, by = blockIdx.x / gx;
  const int64_t row0 = bx * 16 * W + wave * 16;
  const int64_t cb = chunks * by / S, nch = chunks * (by + 1) / S - cb;
  const double* asrc[NIA];
#pragma unroll
  for (int t = 0; t < NIA; ++t) {
    const int ls = 64 * t + lane, ri = ls / SLR, p = ls % SLR;
    asrc[t] = A + (row0 + ri) * n + cb * KC + 2 * (p ^ (ri & 15));
  }
  const double* xsrc = X + (cb * KC + (wave * 8 + (lane >> 3)) / 2) * L + ((wave * 8 + (lane >> 3)) % 2) * 16 + (lane & 7) * 2;
  auto issue = [&](int64_t c, int slot) {
    c = c < nch ? c : nch - 1;
    char* sb = lds + slot * SLOT;
#pragma unroll
    for (int t = 0; t < NIA; ++t)
      __builtin_amdgcn_global_load_lds((gv_t*)(asrc[t] + c * KC), (lv_t*)(sb + wave * AW + t * 1024), 16, 0, 2);
    __builtin_amdgcn_global_load_lds((gv_t*)(xsrc + c * KC * L), (lv_t*)(sb + W * AW + wave * 1024), 16, 0, 0);
  };
  d4_t acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
  const int aoff = wave * AW + i * (SLR * 16);
  double ra = 1.0 + lane * 0.0123, rb = 1.5 - lane * 0.0071;
#pragma unroll
  for (int d = 0; d < NS - 1; ++d) issue(d, d);
  int cs = 0;
  for (int64_t c = 0; c < nch; ++c) {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NS - 2) * (NIA + 1)) : "memory");
    if (MODE & 1) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int is = cs == 0 ? NS - 1 : cs - 1;
    issue(c + NS - 1, is);
    const char* sb = lds + cs * SLOT;
#pragma unroll
    for (int j = 0; j < KC / 8; ++j) {
      d2_t av = {ra, rb};
      if (MODE & 2) av = *reinterpret_cast<const d2_t*>(sb + aoff + 16 * ((q + 4 * j) ^ i));
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int k = 2 * (q + 4 * j) + e;
        double x0 = rb, x1 = ra;
        if (MODE & 2) {
          x0 = *reinterpret_cast<const double*>(sb + W * AW + ((k * 2) ^ (q & 1)) * 128 + 8 * i);
          x1 = *reinterpret_cast<const double*>(sb + W * AW + ((k * 2 + 1) ^ (q & 1)) * 128 + 8 * i);
        }
        if (MODE & 16) {   // reads waited for, MFMAs fed from registers
          asm volatile("" ::"v"(x0), "v"(x1), "v"(av[e]));
          x0 = rb; x1 = ra;
          av[e] = e ? rb : ra;
        }
        if (MODE & 4) {
          acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[e], x0, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[e], x1, acc1, 0, 0, 0);
        } else {
          acc0[0] += av[e] * x0;
          acc1[0] += av[e] * x1;
        }
      }
    }
    cs = cs + 1 == NS ? 0 : cs + 1;
    if (MODE & 8) {   // new random operand bits every chunk
      unsigned long long u = __double_as_longlong(ra) * 6364136223846793005ull + 1442695040888963407ull;
      ra = __longlong_as_double((long long)((u >> 12) | 0x3ff0000000000000ull));
      u = __double_as_longlong(rb) * 6364136223846793005ull + 1442695040888963407ull;
      rb = __longlong_as_double((long long)((u >> 12) | 0x3ff0000000000000ull));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[blockIdx.x] = (double)(t1 - t0) / (double)(r1 - r0) * 100.0;
  }
  P[(by * m + row0) * 64 + lane] = acc0[0] + acc0[1] + acc0[2] + acc0[3] + acc1[0] + acc1[1] + acc1[2] + acc1[3];
}

__global__ void k_fill(double* a, int64_t n, unsigned seed) {   // random operands (DVFS reads zeros high)
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    a[i] = (double)(int)h * 4.656612873077393e-10;
  }
}

template <int MODE>
int run(const char* name, const double* A, const double* X, double* P, int64_t m, int64_t n, int S,
        double* clk) {
  const int64_t grid = m / (16 * W) * S;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(k_abl<MODE>, dim3(grid), dim3(512), 0, 0, A, X, P, m, n, S, clk);
  for (int it = 0; it < 10; ++it) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_abl<MODE>, dim3(grid), dim3(512), 0, 0, A, X, P, m, n, S, clk);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ts.push_back(t);
  }
  std::sort(ts.begin(), ts.end());
  std::vector<double> c(grid);
  CK(hipMemcpy(c.data(), clk, sizeof(double) * grid, hipMemcpyDeviceToHost));
  std::sort(c.begin(), c.end());
  const double bytes = 8.0 * m * n;
  std::printf("%-40s best %7.1f us %5.2f TB/s  median %7.1f us %5.2f TB/s  clock %4.0f MHz\n", name, ts[0] * 1e3,
              bytes / (ts[0] * 1e-3) / 1e12, ts[5] * 1e3, bytes / (ts[5] * 1e-3) / 1e12, c[grid / 2]);
  return 0;
}

int main() {
  const int64_t m = 8192, n = 16384;
  double *A, *X, *P, *clk;
  CK(hipMalloc(&clk, 8 * 4096));
  CK(hipMalloc(&A, 8 * m * n));
  CK(hipMalloc(&X, 8 * n * L));
  CK(hipMalloc(&P, 8 * 8 * m * 64));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, A, m * n, 1u);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, X, n * L, 2u);
  CK(hipDeviceSynchronize());
  for (int w = 0; w < 10; ++w) run<7>("warm", A, X, P, m, n, 4, clk);
  for (int rep = 0; rep < 3; ++rep) {
    run<1>("dma + barrier", A, X, P, m, n, 4, clk);
    run<5>("dma + barrier + mfma (const regs)", A, X, P, m, n, 4, clk);
    run<13>("dma + barrier + mfma (random regs)", A, X, P, m, n, 4, clk);
    run<7>("full (reads + mfma)", A, X, P, m, n, 4, clk);
    run<23>("reads waited, mfma on const regs", A, X, P, m, n, 4, clk);
    run<31>("reads waited, mfma on random regs", A, X, P, m, n, 4, clk);
  }
  return 0;
}
