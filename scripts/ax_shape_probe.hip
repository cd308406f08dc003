// ax_shape_probe.hip — HBM read rate of A (8192 x 16384 fp64, 1 GiB, row-major) in the access
// shapes an A@X tile can take, with nothing consuming the data: a workgroup owns ROWS rows x one
// K split of the columns and walks its K range in chunks; per chunk every row contributes one
// contiguous PIECE-byte run, fetched by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction; runs of < 1 KiB: several rows per instruction) into a DEPTH-slot ring with a
// counted vmcnt, as k_ax_dma does. Prints best / median of 10 launches per shape.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/ax_shape_probe scripts/ax_shape_probe.hip
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

// block = 8 waves; chunk = ROWS x PIECE bytes = CH bytes; instruction i of the chunk covers bytes
// [1024 i, 1024 i + 1024) of the chunk image (row-major [ROWS][PIECE]); wave w issues i = w, w+8..
template <int ROWS, int PIECE, int DEPTH, int AUX>
__global__ __launch_bounds__(512) void k_probe(const char* __restrict__ A, int64_t m, int64_t nbytes_row,
                                               int S, double* out) {
  constexpr int CH = ROWS * PIECE;
  constexpr int NI = CH / 1024;          // instructions per chunk
  static_assert(NI % 8 == 0, "whole instructions per wave");
  constexpr int NIW = NI / 8;
  static_assert(DEPTH * CH <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char ring[DEPTH * CH];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t gx = m / ROWS;
  const int64_t bx = blockIdx.x % gx, by = blockIdx.x / gx;
  const int64_t kb = nbytes_row / S * by, ke = nbytes_row / S * (by + 1);
  const int64_t nch = (ke - kb) / PIECE;
  const char* src[NIW];
#pragma unroll
  for (int j = 0; j < NIW; ++j) {
    const int64_t off = (int64_t)(wave + 8 * j) * 1024 + lane * 16;   // byte in the chunk image
    const int64_t r = off / PIECE, p = off % PIECE;
    src[j] = A + (bx * ROWS + r) * nbytes_row + kb + p;
  }
  auto issue = [&](int64_t c, int slot) {
    c = c < nch ? c : nch - 1;
#pragma unroll
    for (int j = 0; j < NIW; ++j)
      __builtin_amdgcn_global_load_lds((gv_t*)(src[j] + c * PIECE),
                                       (lv_t*)(ring + slot * CH + (wave + 8 * j) * 1024), 16, 0, AUX);
  };
#pragma unroll
  for (int d = 0; d < DEPTH - 1; ++d) issue(d, d);
  int cs = 0;
  for (int64_t c = 0; c < nch; ++c) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DEPTH - 2) * NIW) : "memory");
    __builtin_amdgcn_s_barrier();
    const int is = cs == 0 ? DEPTH - 1 : cs - 1;
    issue(c + DEPTH - 1, is);
    cs = cs + 1 == DEPTH ? 0 : cs + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0 && ring[wave] == 123 && ring[CH - 1] == 45) out[0] = 1.0;
}

template <int ROWS, int PIECE, int DEPTH, int AUX>
int run(const char* A, int64_t m, int64_t rowb, int S, double* out) {
  const int64_t grid = (m / ROWS) * S;
  std::vector<float> ts;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_probe<ROWS, PIECE, DEPTH, AUX>), dim3(grid), dim3(512), 0, 0, A, m, rowb, S, out);
  for (int it = 0; it < 10; ++it) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_probe<ROWS, PIECE, DEPTH, AUX>), dim3(grid), dim3(512), 0, 0, A, m, rowb, S, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ts.push_back(t);
  }
  std::sort(ts.begin(), ts.end());
  const double bytes = (double)m * rowb;
  std::printf("rows %3d piece %5d depth %d %s S %2d grid %5lld  best %7.1f us %5.2f TB/s  median %7.1f us %5.2f TB/s\n",
              ROWS, PIECE, DEPTH, AUX ? "nt " : "def", S, (long long)grid, ts[0] * 1e3, bytes / (ts[0] * 1e-3) / 1e12,
              ts[5] * 1e3, bytes / (ts[5] * 1e-3) / 1e12);
  return 0;
}

int main() {
  const int64_t m = 8192, n = 16384, rowb = n * 8;
  char* A;
  double* out;
  CK(hipMalloc(&A, m * rowb));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(A, 1, m * rowb));
  // warm the clocks
  for (int i = 0; i < 20; ++i) run<128, 256, 4, 2>(A, m, rowb, 4, out);
  for (int rep = 0; rep < 2; ++rep) {
    run<128, 256, 4, 2>(A, m, rowb, 4, out);     // k_ax_dma 84218
    run<128, 256, 3, 2>(A, m, rowb, 4, out);
    run<128, 256, 4, 0>(A, m, rowb, 4, out);
    run<64, 512, 4, 2>(A, m, rowb, 4, out);
    run<64, 512, 4, 2>(A, m, rowb, 8, out);
    run<32, 1024, 4, 2>(A, m, rowb, 1, out);
    run<32, 1024, 4, 2>(A, m, rowb, 2, out);
    run<32, 1024, 4, 0>(A, m, rowb, 1, out);
    run<16, 2048, 4, 2>(A, m, rowb, 1, out);
    run<16, 2048, 4, 0>(A, m, rowb, 1, out);
    run<16, 4096, 2, 2>(A, m, rowb, 1, out);
    run<8, 4096, 4, 2>(A, m, rowb, 1, out);
    run<8, 8192, 2, 2>(A, m, rowb, 1, out);
  }
  return 0;
}
