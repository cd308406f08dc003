// glx_internal.h — declarations shared by the HIP kernels and the host-side driver.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <string>

namespace glx {

// error carried to the C ABI boundary (never crosses it)
struct Error {
  int code;
  std::string msg;
};
extern thread_local std::string g_last_error;

constexpr int kMaxBlocks = 1024;   // grid cap of every reducing kernel (size of a partials row)
constexpr int kMaxRedVals = 6;     // max scalars one reducing kernel produces
constexpr int kMaxL = 128;         // largest l (columns of x) supported by the row kernels

// Deterministic grid-wide reduction target: each block writes its partial to
// part[v * kMaxBlocks + block]; the last block (arrival ticket) sums them in block order
// and writes out[v]. `ticket` must be zero before the first launch; the last block resets it.
struct Red {
  double* part;
  unsigned* ticket;
  double* out;     // kMaxRedVals consecutive doubles (caller picks the slots)
};

// Launch plan of the two dense products for one (dtype, m, n, l).
struct GemmPlan {
  int esize;        // 4 or 8
  int64_t m, n, l;
  // A @ X  ->  P[ax_S][m][l] partial slabs (summed by finalize_residual)
  int ax_kind;      // 1 = MFMA direct row loads, 2 = MFMA quad loads + bpermute, 3 = VALU
  int ax_S;         // K (= n) splits across workgroups
  int ax_lb;        // VALU: column block width (1,2,4,8); ax_ncb = ceil(l / ax_lb)
  int ax_vec;       // VALU: 16-byte loads
  // A^T R  ->  Gp[atr_S][n][l]
  int atr_kind;     // 1 = MFMA, 3 = VALU
  int atr_S;        // M (= m) splits across workgroups
  int atr_lb, atr_vec;
};

GemmPlan make_plan(int esize, int64_t m, int64_t n, int64_t l, int ax_variant);

// ---- dense products (kernels_gemm.hip) ----
template <typename T>
void launch_ax(const GemmPlan& p, const T* A, const T* X, T* P, const int* gate, hipStream_t st);
template <typename T>
void launch_atr(const GemmPlan& p, const T* A, const T* R, T* Gp, hipStream_t st);

// ---- row / elementwise kernels (kernels_elem.hip) ----
// R = sum_s P[s] - B (if gate == NULL or *gate); out[0] = sum R^2.
// gate_mode: what to do when *gate == 0: 0 = nothing, 1 = recompute sum R^2 from R.
template <typename T>
void launch_finalize_residual(const T* P, int S, const T* B, T* R, int64_t ml, const int* gate,
                              int gate_mode, Red red, hipStream_t st);
template <typename T>
void launch_sum_partials(const T* Gp, int S, T* G, int64_t nl, hipStream_t st);
// ProxGD trial: p = prox(x - t g, t), G_t = (x - p)/t, z = x - t G_t.
// out: [sum g*G_t, sum G_t^2, sum_i ||p_i||, max |p|]
template <typename T>
void launch_prox_pgd(const T* x, const T* g, T* p, T* z, int64_t n, int64_t l, double t,
                     double mu, double thres, Red red, hipStream_t st);
// FISTA trial: xc = prox(y - t g, t). out: [sum g*(xc-y), sum (xc-y)^2, sum ||xc_i||, max |xc|]
template <typename T>
void launch_prox_fista(const T* y, const T* g, T* xc, int64_t n, int64_t l, double t, double mu,
                       double thres, Red red, hipStream_t st);
// plain prox of W (glx_prox): out: [sum ||x_i||, max |x|]
template <typename T>
void launch_prox_plain(const T* w, T* x, int64_t n, int64_t l, double t, double mu, double thres,
                       Red red, hipStream_t st);
// out[0] = count(|x| > 1e-6 * (*maxv))
template <typename T>
void launch_count_above(const T* x, int64_t nl, const double* maxv, Red red, hipStream_t st);
// x[|x| < thres] = 0 in place; *flag |= any value changed (caller zeroes *flag)
template <typename T>
void launch_threshold(T* x, int64_t nl, double thres, int* flag, hipStream_t st);
// y = a*xk + b*vk
template <typename T>
void launch_axpby(const T* xk, const T* vk, T* y, int64_t nl, double a, double b, hipStream_t st);
// v = xk + (x - xk)/theta
template <typename T>
void launch_fista_v(const T* xk, const T* x, T* v, int64_t nl, double theta, hipStream_t st);
// SGD (mode 0) / GD (mode 1) step, in place. out: [sum ||x_new_i||]
template <typename T>
void launch_descent(T* x, const T* g, int64_t n, int64_t l, double alpha, double mu, double thres,
                    double delta, int mode, Red red, hipStream_t st);
// out: [sum ||x_i||, max |x|]
template <typename T>
void launch_rownorm_max(const T* x, int64_t n, int64_t l, Red red, hipStream_t st);
// FGD: g += mu * y / sqrt(||y_i||^2 + delta^2); out: [sum (sqrt(||y_i||^2+delta^2) - delta)]
template <typename T>
void launch_fgd_grad(const T* y, T* g, int64_t n, int64_t l, double mu, double delta, Red red,
                     hipStream_t st);
// FGD trial: xc = y - t g. out: [sum g*(xc-y), sum (xc-y)^2, smooth reg(xc), sum ||xc_i||, max |xc|]
template <typename T>
void launch_fgd_trial(const T* y, const T* g, T* xc, int64_t n, int64_t l, double t, double delta,
                      Red red, hipStream_t st);
// fh[idx] = 0.5 * s[i_sumsq] + mu * s[i_reg]
void launch_record_f(const double* s, int i_sumsq, int i_reg, double mu, double* fh, int64_t idx,
                     hipStream_t st);

}  // namespace glx
