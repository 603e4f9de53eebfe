// Small-operand contraction along a contiguous mode group, in one HBM pass.
//
// In the contraction trees of quantum circuits most pairwise steps absorb a tiny tensor
// (a (2,2,2,2) gate, a (2,) input state or output projector) into a large running tensor
// (reference: each such step is a tensordot inside the opt_einsum ContractExpression built at
// tneq_qc/contractor/einsum_strategy.py:639-643, i.e. transpose + GEMM with K <= 4).
// When the contracted modes of the big operand S form at most two runs in its layout,
// S = [O][K1][M][K2][I], the step is
//      C[o][n][m][i] = sum_{k1,k2} S[o][k1][m][k2][i] * G[k1 k2][n]
// (a strided batched GEMM with tiny K, N): no transpose is needed and the step is purely
// HBM-bound, so it is done as one streaming pass: read S once, write C once
// (algorithmic bytes = (numel(S) + numel(C)) * sizeof).  G lives in LDS.
#include <algorithm>

#include "tq_common.h"

namespace tq {

namespace {

constexpr int kThreads = 256;

template <typename T, int KMAX, int NMAX>
__global__ void __launch_bounds__(kThreads)
apply_kernel(const T* __restrict__ S, const T* __restrict__ G, const int32_t* __restrict__ gidx,
             T* __restrict__ C, int64_t O,
             int K1, int64_t M, int K2, int64_t I, int N, float beta_f, double beta_d,
             int use_beta) {
  __shared__ T g[KMAX * NMAX];
  __shared__ int64_t koff[KMAX];
  const int K = K1 * K2;
  const int64_t MI = M * I;
  const int64_t total = O * MI;
  const int64_t sK1 = M * K2 * I, sK2 = I;  // strides of the two contracted runs in S
  for (int t = threadIdx.x; t < K * N; t += kThreads) g[t] = G[gidx ? gidx[t] : t];
  for (int k = threadIdx.x; k < KMAX; k += kThreads) koff[k] = (k / K2) * sK1 + (k % K2) * sK2;
  __syncthreads();
  for (int64_t x = blockIdx.x * (int64_t)kThreads + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * kThreads) {
    int64_t o, r, m, i;
    if (M == 1) {  // one contracted run: skip the middle split
      o = x / I; i = x - o * I; m = 0; r = i;
    } else {
      o = x / MI; r = x - o * MI; m = r / I; i = r - m * I;
    }
    const T* s = S + o * K1 * sK1 + m * K2 * I + i;
    T v[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) v[k] = k < K ? s[koff[k]] : tzero<T>();
    T* c = C + o * N * MI + r;
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
      if (n < N) {
        T acc = tzero<T>();
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
          if (k < K) cmac(acc, v[k], g[k * N + n]);
        if (use_beta) {
          if constexpr (sizeof(typename Traits<T>::R) == 4) acc = acc + c[n * MI] * beta_f;
          else acc = acc + c[n * MI] * beta_d;
        }
        c[n * MI] = acc;
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
axpy_kernel(int64_t n, const T* __restrict__ x, T* __restrict__ y, float bf, double bd, int use_beta) {
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kThreads) {
    T v = x[i];
    if (use_beta) {
      if constexpr (sizeof(typename Traits<T>::R) == 4) v = v + y[i] * bf;
      else v = v + y[i] * bd;
    }
    y[i] = v;
  }
}

// y[i] = sum_{j < nl} y[i + j * stride]: the slice lanes' copies of a per-slice result summed
// into lane 0's (Plan::lanes; the real / complex parts are independent, so R words suffice)
template <typename R>
__global__ void __launch_bounds__(kThreads)
lane_sum_kernel(int64_t n, R* __restrict__ y, int64_t stride, int nl) {
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kThreads) {
    R v = y[i];
    for (int j = 1; j < nl; ++j) v += y[i + j * stride];
    y[i] = v;
  }
}

template <typename T>
int apply_t(int64_t O, int64_t K1, int64_t M, int64_t K2, int64_t I, int64_t N, const void* S,
            const void* G, const int32_t* gidx, void* C, double beta, hipStream_t stream) {
  const int64_t total = O * M * I;
  const int64_t K = K1 * K2;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + kThreads - 1) / kThreads, 8192));
  const int ub = beta != 0.0;
#define TQ_APPLY_CASE(KM, NM)                                                                 \
  if (K <= KM && N <= NM) {                                                                   \
    hipLaunchKernelGGL((apply_kernel<T, KM, NM>), dim3(blocks), dim3(kThreads), 0, stream,    \
                       (const T*)S, (const T*)G, gidx, (T*)C, O, (int)K1, M, (int)K2, I,     \
                       (int)N,                                                                \
                       (float)beta, beta, ub);                                                \
    TQ_HIP(hipGetLastError());                                                                \
    return TQ_OK;                                                                             \
  }
  TQ_APPLY_CASE(2, 1)
  TQ_APPLY_CASE(2, 2)
  TQ_APPLY_CASE(4, 4)
  TQ_APPLY_CASE(4, 16)
  TQ_APPLY_CASE(16, 4)
  TQ_APPLY_CASE(16, 16)
  TQ_APPLY_CASE(32, 32)
#undef TQ_APPLY_CASE
  set_error("apply: K or N too large");
  return TQ_ERR_UNSUPPORTED;
}

template <typename T>
int axpy_t(int64_t n, const void* x, void* y, double beta, hipStream_t stream) {
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, 4096));
  hipLaunchKernelGGL((axpy_kernel<T>), dim3(blocks), dim3(kThreads), 0, stream, n, (const T*)x,
                     (T*)y, (float)beta, beta, (int)(beta != 0.0));
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

}  // namespace

int apply_launch(int dtype, int64_t O, int64_t K1, int64_t M, int64_t K2, int64_t I, int64_t N,
                 const void* S, const void* G, const int32_t* gidx, void* C, double beta,
                 hipStream_t stream) {
  if (O * M * I == 0) return TQ_OK;
  switch (dtype) {
    case TQ_F32: return apply_t<float>(O, K1, M, K2, I, N, S, G, gidx, C, beta, stream);
    case TQ_F64: return apply_t<double>(O, K1, M, K2, I, N, S, G, gidx, C, beta, stream);
    case TQ_C64: return apply_t<c64>(O, K1, M, K2, I, N, S, G, gidx, C, beta, stream);
    case TQ_C128: return apply_t<c128>(O, K1, M, K2, I, N, S, G, gidx, C, beta, stream);
  }
  set_error("apply: bad dtype");
  return TQ_ERR_INVALID;
}

int lane_sum_launch(int dtype, int64_t n, void* y, int64_t stride, int nl, hipStream_t stream) {
  if (n == 0 || nl <= 1) return TQ_OK;
  const int w = (dtype == TQ_C64 || dtype == TQ_C128) ? 2 : 1;   // R words per element
  const int64_t nr = n * w;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((nr + kThreads - 1) / kThreads, 4096));
  if (dtype == TQ_F32 || dtype == TQ_C64)
    hipLaunchKernelGGL((lane_sum_kernel<float>), dim3(blocks), dim3(kThreads), 0, stream, nr, (float*)y, stride * w, nl);
  else if (dtype == TQ_F64 || dtype == TQ_C128)
    hipLaunchKernelGGL((lane_sum_kernel<double>), dim3(blocks), dim3(kThreads), 0, stream, nr, (double*)y, stride * w, nl);
  else {
    set_error("lane_sum: bad dtype");
    return TQ_ERR_INVALID;
  }
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

int axpy_launch(int dtype, int64_t n, const void* x, void* y, double beta, hipStream_t stream) {
  if (n == 0) return TQ_OK;
  switch (dtype) {
    case TQ_F32: return axpy_t<float>(n, x, y, beta, stream);
    case TQ_F64: return axpy_t<double>(n, x, y, beta, stream);
    case TQ_C64: return axpy_t<c64>(n, x, y, beta, stream);
    case TQ_C128: return axpy_t<c128>(n, x, y, beta, stream);
  }
  set_error("axpy: bad dtype");
  return TQ_ERR_INVALID;
}

}  // namespace tq
