// Small-operand contraction along a contiguous mode group, in one HBM pass.
//
// In the contraction trees of quantum circuits most pairwise steps absorb a tiny tensor
// (a (2,2,2,2) gate, a (2,) input state or output projector) into a large running tensor
// (reference: each such step is a tensordot inside the opt_einsum ContractExpression built at
// tneq_qc/contractor/einsum_strategy.py:639-643, i.e. transpose + GEMM with K <= 4).
// When the contracted modes of the big operand S are adjacent in its layout, the step is
//      C[o][n][i] = sum_k S[o][k][i] * G[k][n]
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
apply_kernel(const T* __restrict__ S, const T* __restrict__ G, T* __restrict__ C, int64_t O,
             int K, int N, int64_t I, float beta_f, double beta_d, int use_beta) {
  __shared__ T g[KMAX * NMAX];
  for (int t = threadIdx.x; t < K * N; t += kThreads) g[t] = G[t];
  __syncthreads();
  const int64_t total = O * I;
  for (int64_t x = blockIdx.x * (int64_t)kThreads + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * kThreads) {
    const int64_t o = x / I, i = x - o * I;
    const T* s = S + o * K * I + i;
    T v[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) v[k] = k < K ? s[k * I] : tzero<T>();
    T* c = C + o * N * I + i;
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
      if (n < N) {
        T acc = tzero<T>();
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
          if (k < K) cmac(acc, v[k], g[k * N + n]);
        if (use_beta) {
          if constexpr (sizeof(typename Traits<T>::R) == 4) acc = acc + c[n * I] * beta_f;
          else acc = acc + c[n * I] * beta_d;
        }
        c[n * I] = acc;
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

template <typename T>
int apply_t(int64_t O, int64_t K, int64_t N, int64_t I, const void* S, const void* G, void* C,
            double beta, hipStream_t stream) {
  const int64_t total = O * I;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + kThreads - 1) / kThreads, 4096));
  const int ub = beta != 0.0;
#define TQ_APPLY_CASE(KM, NM)                                                                 \
  if (K <= KM && N <= NM) {                                                                   \
    hipLaunchKernelGGL((apply_kernel<T, KM, NM>), dim3(blocks), dim3(kThreads), 0, stream,    \
                       (const T*)S, (const T*)G, (T*)C, O, (int)K, (int)N, I, (float)beta,   \
                       beta, ub);                                                             \
    TQ_HIP(hipGetLastError());                                                                \
    return TQ_OK;                                                                             \
  }
  TQ_APPLY_CASE(2, 1)
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

int apply_launch(int dtype, int64_t O, int64_t K, int64_t N, int64_t I, const void* S,
                 const void* G, void* C, double beta, hipStream_t stream) {
  if (O * I == 0) return TQ_OK;
  switch (dtype) {
    case TQ_F32: return apply_t<float>(O, K, N, I, S, G, C, beta, stream);
    case TQ_F64: return apply_t<double>(O, K, N, I, S, G, C, beta, stream);
    case TQ_C64: return apply_t<c64>(O, K, N, I, S, G, C, beta, stream);
    case TQ_C128: return apply_t<c128>(O, K, N, I, S, G, C, beta, stream);
  }
  set_error("apply: bad dtype");
  return TQ_ERR_INVALID;
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
