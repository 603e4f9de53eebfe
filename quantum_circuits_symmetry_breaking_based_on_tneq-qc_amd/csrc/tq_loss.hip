// Fidelity loss of the symmetry-breaking fit (symmetry_breaking_quantum.py:220-229, the loss every
// pruning candidate minimises; also validate_target_tensor :159-166):
//
//     a = <t, o> = sum conj(t_i) o_i,  T = <t, t>,  N = <o, o>,  D = max(T N, 1e-12)
//     L = 1 - |a|^2 / D
//
// torch evaluates it as ~10 small launches forward and ~15 backward (three vdots, abs, pow,
// clamp, div, sub and their adjoints); here it is one launch each way:
//  * fidelity_forward — one workgroup sums a, T, N over the n elements (float64 accumulation)
//    and writes the four sums (the backward's input) and L;
//  * fidelity_backward — torch's gradient of a real loss w.r.t. a complex tensor, 2 dL/d(conj o):
//        grad_o_i = g * 2 * (-a t_i / D + [T N >= 1e-12] |a|^2 T o_i / D^2)
//    (the clamp passes no gradient to N when it is active), g = the upstream gradient of L.
// HBM-bound (2 or 3 complex n-vectors per launch); C5: n = 2^16, one workgroup suffices.
#include "tq_common.h"

namespace tq {

namespace {

constexpr int kLossNT = 1024;

template <typename T>
__global__ void __launch_bounds__(kLossNT) fidelity_fwd_kernel(int64_t n, const T* __restrict__ t,
                                                               const T* __restrict__ o,
                                                               double* __restrict__ stats,
                                                               typename Traits<T>::R* __restrict__ loss) {
  double ar = 0.0, ai = 0.0, tt = 0.0, oo = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kLossNT) {
    const double tr = (double)t[i].re, ti = (double)t[i].im;
    const double orr = (double)o[i].re, oi = (double)o[i].im;
    ar += tr * orr + ti * oi;   // conj(t) o
    ai += tr * oi - ti * orr;
    tt += tr * tr + ti * ti;
    oo += orr * orr + oi * oi;
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    ar += __shfl_xor(ar, s);
    ai += __shfl_xor(ai, s);
    tt += __shfl_xor(tt, s);
    oo += __shfl_xor(oo, s);
  }
  __shared__ double red[4][kLossNT / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = ar;
    red[1][w] = ai;
    red[2][w] = tt;
    red[3][w] = oo;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    double v = 0.0;
    for (int k = 0; k < kLossNT / 64; ++k) v += red[threadIdx.x][k];
    stats[threadIdx.x] = v;
    red[threadIdx.x][0] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double a2 = red[0][0] * red[0][0] + red[1][0] * red[1][0];
    const double d = fmax(red[2][0] * red[3][0], 1e-12);
    *loss = (typename Traits<T>::R)(1.0 - a2 / d);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) fidelity_bwd_kernel(int64_t n, const T* __restrict__ t,
                                                           const T* __restrict__ o,
                                                           const double* __restrict__ stats,
                                                           const typename Traits<T>::R* __restrict__ g,
                                                           T* __restrict__ grad) {
  using R = typename Traits<T>::R;
  const double ar = stats[0], ai = stats[1], tt = stats[2], oo = stats[3];
  const double tn = tt * oo;
  const double d = fmax(tn, 1e-12);
  const double gs = 2.0 * (double)(*g);
  // coefficient of t_i: -a / D; of o_i: |a|^2 T / D^2 (0 when the clamp is active)
  const double cr = -gs * ar / d, ci = -gs * ai / d;
  const double co = tn >= 1e-12 ? gs * (ar * ar + ai * ai) * tt / (d * d) : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double tr = (double)t[i].re, ti = (double)t[i].im;
    T v;
    v.re = (R)(cr * tr - ci * ti + co * (double)o[i].re);
    v.im = (R)(cr * ti + ci * tr + co * (double)o[i].im);
    grad[i] = v;
  }
}

template <typename T>
int fwd_t(int64_t n, const void* t, const void* o, double* stats, void* loss, hipStream_t s) {
  hipLaunchKernelGGL(fidelity_fwd_kernel<T>, dim3(1), dim3(kLossNT), 0, s, n, (const T*)t, (const T*)o, stats,
                     (typename Traits<T>::R*)loss);
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

template <typename T>
int bwd_t(int64_t n, const void* t, const void* o, const double* stats, const void* g, void* grad,
          hipStream_t s) {
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 2048);
  if (blocks <= 0) return TQ_OK;
  hipLaunchKernelGGL(fidelity_bwd_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, n, (const T*)t,
                     (const T*)o, stats, (const typename Traits<T>::R*)g, (T*)grad);
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

}  // namespace

int fidelity_forward_launch(int dtype, int64_t n, const void* t, const void* o, double* stats, void* loss,
                            hipStream_t s) {
  switch (dtype) {
    case TQ_C64: return fwd_t<c64>(n, t, o, stats, loss, s);
    case TQ_C128: return fwd_t<c128>(n, t, o, stats, loss, s);
  }
  set_error("fidelity loss: complex dtypes only (TQ_C64 / TQ_C128)");
  return TQ_ERR_INVALID;
}

int fidelity_backward_launch(int dtype, int64_t n, const void* t, const void* o, const double* stats,
                             const void* g, void* grad, hipStream_t s) {
  switch (dtype) {
    case TQ_C64: return bwd_t<c64>(n, t, o, stats, g, grad, s);
    case TQ_C128: return bwd_t<c128>(n, t, o, stats, g, grad, s);
  }
  set_error("fidelity loss: complex dtypes only (TQ_C64 / TQ_C128)");
  return TQ_ERR_INVALID;
}

}  // namespace tq
