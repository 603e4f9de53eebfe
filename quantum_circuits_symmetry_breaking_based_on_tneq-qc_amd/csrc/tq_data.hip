// Measurement-data kernels of the EngineSiamese caller.
//
//  * hermite_kernel — EngineSiamese.generate_data (tneq_qc/core/engine_siamese.py:133-254):
//    for every scalar input x_p (one (batch, qubit) entry)
//        phi[p][k]   = (w_k * sqrt(exp(-x_p^2 / 2))) * He_k(x_p),   k < K
//        Mx[p][k][l] = conj(phi[p][k]) * phi[p][l]
//    with the probabilists' Hermite recurrence He_i = x He_{i-1} - (i-1) He_{i-2} (:82-131)
//    and w_k = exp(-(log(2 pi)/2 + lgamma(k+1))/2) (:59-80; computed on the host exactly as
//    the reference does and passed by value).  As in the reference a complex dtype computes in
//    float64 and rounds once (:165-207) and a real dtype computes in its own precision
//    (:212-254); FP contraction is off, so every value follows the reference's sequence of
//    roundings.  HBM-bound: algorithmic bytes = n * (8 + (K + K^2) * sizeof(T)).
//    A workgroup owns 32 points: the recurrences run one point per lane into LDS, then all 256
//    lanes stream phi and Mx out in linear (coalesced) order.
//  * icdf_kernel — one inverse-CDF draw per row (EngineSiamese.sample, :854-905): clamp the
//    density at 0, inclusive prefix sum, normalise by (total + 1e-10), count cdf < u, clamp the
//    index to G-2, interpolate linearly on the grid.  One workgroup per row; the row's CDF lives
//    in LDS.
#include <algorithm>

#include "tq_common.h"

namespace tq {

namespace {

constexpr int kHermNT = 256, kHermPts = 32;
constexpr int kCdfNT = 256;

struct HermW {
  double w[TQ_HERMITE_MAX_K];
};

template <typename T, typename R>
__device__ __forceinline__ T from_real(R v) {
  if constexpr (Traits<T>::cplx) {
    using E = typename Traits<T>::R;
    return T{(E)v, (E)0};
  } else {
    return (T)v;
  }
}

template <typename R>
__device__ __forceinline__ void hermite_point(double xd, int K, const HermW& W, R* __restrict__ f) {
#pragma clang fp contract(off)
  const R x = (R)xd;
  const R g = sqrt(exp(-(x * x) / (R)2));
  R h0 = (R)1, h1 = x;
  f[0] = ((R)W.w[0] * g) * h0;
  if (K > 1) f[1] = ((R)W.w[1] * g) * h1;
  for (int i = 2; i < K; ++i) {
    const R h = x * h1 - (R)(i - 1) * h0;
    f[i] = ((R)W.w[i] * g) * h;
    h0 = h1;
    h1 = h;
  }
}

template <typename T, typename R>
__global__ void __launch_bounds__(kHermNT)
hermite_kernel(int64_t npts, int K, const double* __restrict__ x, HermW W, T* __restrict__ phi,
               T* __restrict__ mx) {
#pragma clang fp contract(off)
  __shared__ R f[kHermPts * TQ_HERMITE_MAX_K];
  const int tid = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * kHermPts;
  const int np = (int)(npts - p0 < kHermPts ? npts - p0 : kHermPts);
  if (tid < np) hermite_point<R>(x[p0 + tid], K, W, f + tid * K);
  __syncthreads();
  if (phi) {
    T* __restrict__ o = phi + p0 * K;
    for (int i = tid; i < np * K; i += kHermNT) o[i] = from_real<T, R>(f[i]);
  }
  if (mx) {
    const int KK = K * K;
    T* __restrict__ o = mx + p0 * KK;
    if (KK >= kHermNT) {
      // one (k, l) per lane, points in turn: one division per lane and slice of KK
      for (int r0 = 0; r0 < KK; r0 += kHermNT) {
        const int r = r0 + tid;
        if (r < KK) {
          const int k = r / K, l = r - k * K;
          for (int p = 0; p < np; ++p)
            o[(int64_t)p * KK + r] = from_real<T, R>(f[p * K + k] * f[p * K + l]);
        }
      }
    } else {
      for (int i = tid; i < np * KK; i += kHermNT) {
        const int p = i / KK, r = i - p * KK, k = r / K, l = r - k * K;
        o[i] = from_real<T, R>(f[p * K + k] * f[p * K + l]);
      }
    }
  }
}

template <typename R>
__global__ void __launch_bounds__(kCdfNT)
icdf_kernel(int G, const R* __restrict__ dens, int64_t ldd, const R* __restrict__ grid,
            const float* __restrict__ u, R* __restrict__ out, int64_t ostride) {
#pragma clang fp contract(off)
  __shared__ R c[TQ_ICDF_MAX_GRID];
  __shared__ R part[kCdfNT];
  __shared__ int cnt[kCdfNT];
  const int tid = threadIdx.x;
  const int64_t s = blockIdx.x;
  const R* __restrict__ row = dens + s * ldd;
  for (int i = tid; i < G; i += kCdfNT) {
    const R v = row[i];
    c[i] = v < (R)0 ? (R)0 : v;   // clamp(min=0); NaN propagates as in torch.clamp
  }
  __syncthreads();
  // inclusive prefix sum: per-lane segment, then a scan of the segment totals
  const int seg = (G + kCdfNT - 1) / kCdfNT;
  const int b = min(tid * seg, G), e = min(b + seg, G);
  R acc = (R)0;
  for (int i = b; i < e; ++i) {
    acc += c[i];
    c[i] = acc;
  }
  part[tid] = acc;
  __syncthreads();
  for (int off = 1; off < kCdfNT; off <<= 1) {
    const R v = tid >= off ? part[tid - off] : (R)0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  const R base = tid > 0 ? part[tid - 1] : (R)0;
  for (int i = b; i < e; ++i) c[i] += base;
  __syncthreads();
  const R denom = c[G - 1] + (R)1e-10;
  const R uu = (R)u[s];
  int n = 0;
  for (int i = tid; i < G; i += kCdfNT) n += (c[i] / denom < uu) ? 1 : 0;
  cnt[tid] = n;
  __syncthreads();
  for (int off = kCdfNT / 2; off > 0; off >>= 1) {
    if (tid < off) cnt[tid] += cnt[tid + off];
    __syncthreads();
  }
  if (tid == 0) {
    const int idx = min(cnt[0], G - 2);
    const R cl = c[idx] / denom, cr = c[idx + 1] / denom;
    const R xl = grid[idx], xr = grid[idx + 1];
    const R fr = (uu - cl) / (cr - cl + (R)1e-10);
    out[s * ostride] = xl + fr * (xr - xl);
  }
}

template <typename T, typename R>
int herm_t(int64_t n, int K, const double* x, const HermW& W, void* phi, void* mx, hipStream_t st) {
  const int64_t blocks = (n + kHermPts - 1) / kHermPts;
  hipLaunchKernelGGL((hermite_kernel<T, R>), dim3((unsigned)blocks), dim3(kHermNT), 0, st, n, K, x,
                     W, reinterpret_cast<T*>(phi), reinterpret_cast<T*>(mx));
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

template <typename R>
int icdf_t(int64_t rows, int G, const void* dens, int64_t ldd, const void* grid, const float* u,
           void* out, int64_t ostride, hipStream_t st) {
  hipLaunchKernelGGL((icdf_kernel<R>), dim3((unsigned)rows), dim3(kCdfNT), 0, st, G,
                     reinterpret_cast<const R*>(dens), ldd, reinterpret_cast<const R*>(grid), u,
                     reinterpret_cast<R*>(out), ostride);
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

}  // namespace

int hermite_launch(int dtype, int64_t n, int K, const double* x, const double* w, void* phi,
                   void* mx, hipStream_t stream) {
  if (n == 0) return TQ_OK;
  if ((n + kHermPts - 1) / kHermPts > INT32_MAX) {
    set_error("hermite: too many points for one launch");
    return TQ_ERR_INVALID;
  }
  HermW W{};
  for (int k = 0; k < K; ++k) W.w[k] = w[k];
  switch (dtype) {
    case TQ_F32: return herm_t<float, float>(n, K, x, W, phi, mx, stream);
    case TQ_F64: return herm_t<double, double>(n, K, x, W, phi, mx, stream);
    case TQ_C64: return herm_t<c64, double>(n, K, x, W, phi, mx, stream);
    case TQ_C128: return herm_t<c128, double>(n, K, x, W, phi, mx, stream);
  }
  set_error("hermite: bad dtype");
  return TQ_ERR_INVALID;
}

int icdf_launch(int dtype, int64_t rows, int64_t grid_size, const void* density, int64_t ld,
                const void* grid_x, const float* u, void* out, int64_t out_stride,
                hipStream_t stream) {
  if (rows == 0) return TQ_OK;
  switch (dtype) {
    case TQ_F32: return icdf_t<float>(rows, (int)grid_size, density, ld, grid_x, u, out, out_stride, stream);
    case TQ_F64: return icdf_t<double>(rows, (int)grid_size, density, ld, grid_x, u, out, out_stride, stream);
  }
  set_error("inverse_cdf: density must be TQ_F32 or TQ_F64");
  return TQ_ERR_INVALID;
}

}  // namespace tq
