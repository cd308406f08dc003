// Round 6 probe (not part of libglx): C3's fp32 A^T R (8192 x 16384 x 32)
// with A staged by LDS-DMA instead of loaded into the MFMA operand registers.
//
// Block = one 64-column panel of A, 8 waves; wave w walks rows [w m/8, (w+1) m/8) in chunks of 16
// rows. Per chunk a wave issues 4 LDS-DMA instructions for its A rows (4 rows x 256 B each: the
// panel's 64 f32 columns) and 2 for its R rows (16 x 32 f32), into a private ring of NS slots, so
// no barrier is needed: the wave waits for its own DMAs with a counted vmcnt and, before reusing
// a slot, for its own LDS reads (lgkmcnt). Lane (i, q) of a 4-row step reads columns 4i..4i+3 of
// row q with one ds_read_b128 and feeds 4 x 2 MFMAs v_mfma_f32_16x16x4f32 (output rows 4i + e,
// e < 4, as kernels_atr.hip's f32 panel). After the walk the 8 waves' accumulators are summed
// through LDS in wave order and stored. Checked against a VALU kernel (relative 1e-5), timed with
// HIP events over 20 launches; prints one line.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/atr_dma_probe scripts/atr_dma_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) void g_void_t;
typedef __attribute__((address_space(3))) void l_void_t;

// CR rows of A per chunk (8 or 16), NS ring slots per wave, WAVES waves splitting the rows
template <int CR, int NS, bool NTL, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_atr_dma(const float* __restrict__ A, const float* __restrict__ R,
                                                       float* __restrict__ G, int m, int n) {
  constexpr int ABYTES = CR * 64 * 4;          // A per wave and chunk
  constexpr int RBYTES = CR * 32 * 4;          // R
  constexpr int SLOTB = ABYTES + RBYTES;
  constexpr int NST = CR / 4;                  // 4-row MFMA steps per chunk
  constexpr int NI = ABYTES / 1024 + RBYTES / 1024;   // DMA instructions per chunk
  constexpr int WAITN = (NS - 2) * NI;                // chunks in flight beyond the next one
  constexpr int kWait = (WAITN & 15) | (7 << 4) | (15 << 8) | ((WAITN >> 4) << 14);   // vmcnt(WAITN)
  constexpr int kWaitL = 63 | (7 << 4) | (0 << 8) | (3 << 14);                         // lgkmcnt(0)
  __shared__ __attribute__((aligned(1024))) char lds[WAVES * NS * SLOTB];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int col0 = blockIdx.x * 64;
  const int rows = m / WAVES, r0 = wave * rows, nch = rows / CR;
  char* mine = lds + wave * NS * SLOTB;
  // DMA sources: A instruction t covers rows 4t..4t+3 of the chunk (lane: row 4t + lane/16,
  // 16 B at column 4 (lane%16)); R instruction t covers rows 8t..8t+7 (lane: row 8t + lane/8,
  // 16 B at column 4 (lane%8))
  auto issue = [&](int c, int slot) {
    c = c < nch ? c : nch - 1;
    char* sb = mine + slot * SLOTB;
    const int rb = r0 + c * CR;
#pragma unroll
    for (int t = 0; t < CR / 4; ++t) {
      const float* src = A + (size_t)(rb + 4 * t + lane / 16) * n + col0 + 4 * (lane % 16);
      __builtin_amdgcn_global_load_lds((g_void_t*)src, (l_void_t*)(sb + t * 1024), 16, 0, NTL ? 2 : 0);
    }
#pragma unroll
    for (int t = 0; t < CR / 8; ++t) {
      const float* src = R + (size_t)(rb + 8 * t + lane / 8) * 32 + 4 * (lane % 8);
      __builtin_amdgcn_global_load_lds((g_void_t*)src, (l_void_t*)(sb + ABYTES + t * 1024), 16, 0, 0);
    }
  };
  typedef float c4 __attribute__((ext_vector_type(4)));
  c4 acc[4][2];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[e][nt] = c4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(s, s);
  for (int c = 0; c < nch; ++c) {
    const int slot = c % NS;
    __builtin_amdgcn_s_waitcnt(kWait);   // this wave's DMAs of chunk c have landed
    const char* sb = mine + slot * SLOTB;
    f4 av[NST];
    float rv[NST][2];
#pragma unroll
    for (int st = 0; st < NST; ++st) {   // 4-row steps: lane (i, q) row 4 st + q
      av[st] = *reinterpret_cast<const f4*>(sb + (4 * st + q) * 256 + 16 * i);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        rv[st][nt] = *reinterpret_cast<const float*>(sb + ABYTES + (4 * st + q) * 128 + 4 * (nt * 16 + i));
    }
#pragma unroll
    for (int st = 0; st < NST; ++st)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[e][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[st][e], rv[st][nt], acc[e][nt], 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(kWaitL);   // the reads of this slot are done before it is refilled
    issue(c + NS - 1, (c + NS - 1) % NS);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  // waves in order through LDS: red[w][e][nt][lane] (reuses the ring)
  float* red = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((wave * 8 + e * 2 + nt) * 4 + r) * 64 + lane] = acc[e][nt][r];
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = red[((0 * 8 + e * 2 + nt) * 4 + r) * 64 + lane];
        for (int w = 1; w < WAVES; ++w) v += red[((w * 8 + e * 2 + nt) * 4 + r) * 64 + lane];
        // MFMA e: D[M][N] with M = 4 (lane >> 4) + r, N = lane & 15 (the 16x16 C/D layout);
        // M indexes A columns 4 M + e, N the columns of the 16-wide tile nt of R
        const int grow = col0 + 4 * (4 * (lane >> 4) + r) + e;
        const int gcol = nt * 16 + (lane & 15);
        G[(size_t)grow * 32 + gcol] = v;
      }
}

__global__ void k_ref(const float* A, const float* R, float* G, int m, int n) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;   // G row (column of A)
  if (j >= n) return;
  double acc[32] = {0};
  for (int k = 0; k < m; ++k) {
    const double a = A[(size_t)k * n + j];
    for (int c = 0; c < 32; ++c) acc[c] += a * R[(size_t)k * 32 + c];
  }
  for (int c = 0; c < 32; ++c) G[(size_t)j * 32 + c] = (float)acc[c];
}

template <int CR, int NS, bool NTL, int WAVES = 8>
static double run(const float* A, const float* R, float* G, int m, int n, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_atr_dma<CR, NS, NTL, WAVES>), dim3(n / 64), dim3(64 * WAVES), 0, 0, A, R, G, m, n);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_atr_dma<CR, NS, NTL, WAVES>), dim3(n / 64), dim3(64 * WAVES), 0, 0, A, R, G, m, n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3 * ms / reps;
}

int main() {
  const int m = 8192, n = 16384, reps = 20;
  std::vector<float> hA((size_t)m * n), hR((size_t)m * 32);
  unsigned s = 12345u;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 8) & 0xFFFF) / 65536.f - 0.5f; };
  for (auto& v : hA) v = rnd();
  for (auto& v : hR) v = rnd();
  float *A, *R, *G, *Gr;
  CK(hipMalloc(&A, hA.size() * 4));
  CK(hipMalloc(&R, hR.size() * 4));
  CK(hipMalloc(&G, (size_t)n * 32 * 4));
  CK(hipMalloc(&Gr, (size_t)n * 32 * 4));
  CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(R, hR.data(), hR.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_ref, dim3(n / 256), dim3(256), 0, 0, A, R, Gr, m, n);
  CK(hipDeviceSynchronize());
  std::vector<float> g((size_t)n * 32), gr((size_t)n * 32);
  CK(hipMemcpy(gr.data(), Gr, gr.size() * 4, hipMemcpyDeviceToHost));
  const double bytes = (double)m * n * 4 + (double)m * 32 * 4 + (double)n * 32 * 4;
  auto check = [&](const char* name, double us) {
    CK(hipMemcpy(g.data(), G, g.size() * 4, hipMemcpyDeviceToHost));
    double err = 0, scale = 0;
    for (size_t k = 0; k < g.size(); ++k) {
      err = std::fmax(err, std::fabs((double)g[k] - gr[k]));
      scale = std::fmax(scale, std::fabs((double)gr[k]));
    }
    std::printf("%s: %.1f us  %.2f TB/s  %.1f TF  max rel err %.2e\n", name, us, bytes / us / 1e6,
                2.0 * m * n * 32 / us / 1e6, err / scale);
  };
  check("W8 CR16 NS3 NTL", run<16, 3, true>(A, R, G, m, n, reps));
  check("W8 CR8 NS5 NTL", run<8, 5, true>(A, R, G, m, n, reps));
  check("W4 CR16 NS3 NTL (2 blocks/CU)", run<16, 3, true, 4>(A, R, G, m, n, reps));
  check("W4 CR8 NS5 NTL (2 blocks/CU)", run<8, 5, true, 4>(A, R, G, m, n, reps));
  check("W4 CR8 NS6 NTL (2 blocks/CU)", run<8, 6, true, 4>(A, R, G, m, n, reps));
  check("W4 CR16 NS3 (2 blocks/CU)", run<16, 3, false, 4>(A, R, G, m, n, reps));
  return 0;
}
