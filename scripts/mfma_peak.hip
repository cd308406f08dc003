// Measured MFMA ceiling of the two instructions the dense products use (tuning tool).
//
//   hipcc -O3 --offload-arch=gfx950 -o scripts/mfma_peak scripts/mfma_peak.hip && scripts/mfma_peak
//
// Every wave issues back-to-back v_mfma_f64_16x16x4_f64 (or v_mfma_f32_16x16x4_f32) on CH
// independent accumulators; one or two waves per SIMD on every CU. Prints one JSON line per
// (dtype, waves per SIMD, chains) with TFLOP/s on random operands; the AMD spec peaks are
// 78.6 TF (fp64 matrix) and 157.3 TF (f32 matrix).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

// random operands: DVFS holds a lower clock on random data than on zeros
__global__ void k_fill(d2* buf, int64_t nvec) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u; h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    buf[i] = d2{(double)(h & 0xffff) / 65536.0 - 0.5, (double)(h >> 16) / 65536.0 - 0.5};
  }
}

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int CH>
__global__ __launch_bounds__(512) void k_f64(const double* in, double* out, int iters) {
  double a = in[threadIdx.x & 63], b = in[64 + (threadIdx.x & 63)];
  d4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = d4{0, 0, 0, 0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(512) void k_f32(const float* in, float* out, int iters) {
  float a = in[threadIdx.x & 63], b = in[64 + (threadIdx.x & 63)];
  f4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f4{0, 0, 0, 0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  }
  float s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// MFMA beside HBM streaming at the A@X mix: every MPL MFMAs one 16-B-per-lane load of a
// 2 GiB buffer (row-contiguous, 8 loads in flight per wave). Lane 0 of each wave stamps
// s_memtime / s_memrealtime (100 MHz) around the loop: clk[] = shader cycles, wall ticks.
// PAT 0: a wave-instruction reads 1 KiB contiguous. PAT 1: the A@X (kind 1/5, VPL 2) pattern —
// the buffer is a 16384 x 16384 f64 matrix, wave w owns 16 rows, lane reads row (lane & 15)
// at k = 16c + 4(lane >> 4) + 2v: one instruction = 16 rows x 4 x 16 B, two = 16 x 128 B.
template <int MPL, int PAT = 0>
__global__ __launch_bounds__(512) void k_mix(const double* in, const d2* __restrict__ buf,
                                              int64_t nvec, double* out,
                                              unsigned long long* clk, int iters) {
  double a = in[threadIdx.x & 63], b = in[64 + (threadIdx.x & 63)];
  d4 acc[4];
  for (int c = 0; c < 4; ++c) acc[c] = d4{0, 0, 0, 0};
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
  int64_t idx = gw * 64 + (threadIdx.x & 63);
  const int64_t step = nw * 64;
  // PAT 1 state: row base (in d2 units) and the k position (chunk c, half v)
  const int lane = threadIdx.x & 63;
  const int64_t rowb = ((gw % 1024) * 16 + (lane & 15)) * (16384 / 2);
  const int64_t kbase = ((gw / 1024) % 2) * (8192 / 2) + (lane >> 4) * 2;
  int64_t kc = 0;   // load counter: chunk = kc >> 1, v = kc & 1
  auto next = [&]() -> int64_t {
    if (PAT == 0) { const int64_t r = idx; idx += step; if (idx >= nvec) idx -= nvec; return r; }
    const int64_t r = rowb + kbase + (kc >> 1) * 8 + (kc & 1);
    kc = (kc + 1) & 1023;   // 512 chunks of 16 k within the half row
    return r;
  };
  d2 ring[8];
  for (int r = 0; r < 8; ++r) ring[r] = __builtin_nontemporal_load(buf + next());
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const d2 v = ring[r];
      ring[r] = __builtin_nontemporal_load(buf + next());
      a += v.x; b += v.y;
#pragma unroll
      for (int j = 0; j < MPL; ++j) acc[j & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j & 3], 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
  for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  for (int r = 0; r < 8; ++r) s += ring[r].x;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) { clk[2 * gw] = t1 - t0; clk[2 * gw + 1] = r1 - r0; }
}

template <int MPL, int PAT = 0>
static void run_mix(int wps, int cus, const d2* buf, int64_t nvec) {
  const int threads = 256 * wps, blocks = cus, iters = MPL ? 4000 / MPL + 50 : 600;
  const int nwaves = blocks * threads / 64;
  double* in; double* out; unsigned long long* clk;
  CHECK(hipMalloc(&in, 128 * sizeof(double)));
  CHECK(hipMemset(in, 0, 128 * sizeof(double)));
  CHECK(hipMalloc(&out, (size_t)blocks * threads * sizeof(double)));
  CHECK(hipMalloc(&clk, (size_t)nwaves * 2 * sizeof(unsigned long long)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 20; ++w)   // >= 2 s-class warm loop is too long here; 20 launches settle DVFS
    hipLaunchKernelGGL((k_mix<MPL, PAT>), dim3(blocks), dim3(threads), 0, 0, in, buf, nvec, out, clk, iters);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((k_mix<MPL, PAT>), dim3(blocks), dim3(threads), 0, 0, in, buf, nvec, out, clk, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long* h = (unsigned long long*)malloc(nwaves * 2 * sizeof(unsigned long long));
  CHECK(hipMemcpy(h, clk, nwaves * 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  double ghz = 0;
  for (int w = 0; w < nwaves; ++w) ghz += (double)h[2 * w] / (double)h[2 * w + 1] * 0.1;
  ghz /= nwaves;
  const double flops = 2.0 * 16 * 16 * 4 * (double)iters * 8 * MPL * nwaves;
  const double bytes = (double)iters * 8 * 1024 * nwaves;
  printf("{\"mix\": \"f64 mfma/load=%d pat=%d\", \"waves_per_simd\": %d, \"ms\": %.3f, \"TFs\": %.2f, \"GBs\": %.0f, \"clock_GHz\": %.3f}\n",
         MPL, PAT, wps, ms, flops / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 1e9, ghz);
  free(h);
  CHECK(hipFree(in)); CHECK(hipFree(out)); CHECK(hipFree(clk));
}

template <typename T, typename K>
static void run(const char* name, K kern, int ch, int wps, int cus) {
  const int threads = 256 * wps, blocks = cus, iters = 20000;
  T* in; T* out;
  CHECK(hipMalloc(&in, 128 * sizeof(T)));
  CHECK(hipMalloc(&out, (size_t)blocks * threads * sizeof(T)));
  T h[128];
  for (int i = 0; i < 128; ++i) h[i] = (T)((i * 2654435761u % 1000) / 1000.0 - 0.5);
  CHECK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, in, out, 200);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double flops = 2.0 * 16 * 16 * 4 * (double)iters * ch * (blocks * threads / 64);
  printf("{\"mfma\": \"%s\", \"waves_per_simd\": %d, \"chains\": %d, \"ms\": %.3f, \"TFs\": %.2f}\n",
         name, wps, ch, ms, flops / (ms * 1e-3) / 1e12);
  CHECK(hipFree(in)); CHECK(hipFree(out));
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  for (int wps = 1; wps <= 2; ++wps) {
    run<double>("f64_16x16x4", k_f64<4>, 4, wps, cus);
    run<double>("f64_16x16x4", k_f64<8>, 8, wps, cus);
    run<float>("f32_16x16x4", k_f32<4>, 4, wps, cus);
    run<float>("f32_16x16x4", k_f32<8>, 8, wps, cus);
  }
  const int64_t nvec = (int64_t)1 << 27;   // 2 GiB of 16-B vectors
  d2* buf;
  CHECK(hipMalloc(&buf, nvec * sizeof(d2)));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, buf, nvec);
  CHECK(hipDeviceSynchronize());
  for (int wps = 1; wps <= 2; ++wps) {
    run_mix<0>(wps, cus, buf, nvec);
    run_mix<4>(wps, cus, buf, nvec);
    run_mix<8>(wps, cus, buf, nvec);
    run_mix<16>(wps, cus, buf, nvec);
    run_mix<64>(wps, cus, buf, nvec);
    run_mix<0, 1>(wps, cus, buf, nvec);
    run_mix<4, 1>(wps, cus, buf, nvec);
    run_mix<8, 1>(wps, cus, buf, nvec);
  }
  CHECK(hipFree(buf));
  return 0;
}
