// One optimizer step of the reference's Stiefel SGD (SGDG) for every parameter of a group in ONE
// launch: tneq_qc/optim/stiefel_optimizer_complex.py:77-176 (SGDG.step) with its helpers
// tneq_qc/optim/gutils.py:7-9 (unit), :62-83 (qr_retraction), :133-137 (matrix_norm_one) and
// SGDG.compute_Y (:66-74, the Cayley transform).  The symmetry-breaking training loop
// (symmetry_breaking_quantum.py:216-230) runs this step on every core after every backward pass;
// in the reference each core costs ~20 small torch launches (norms, 6 matmuls, an inverse), here the
// whole group is one launch: one workgroup per parameter, every matrix in LDS (cols <= 32; larger
// parameters -- a 1-D parameter is 1 x len, a core of bond dimension >= 3 has cols >= 9 ... -- run on
// a global-memory scratch, `GM`: when 2 rows < cols in the low-rank Woodbury form, lowrank_step,
// O(cols^2 rows) work and O(cols rows) scratch; otherwise the dense code below, O(cols^3)).
//
// Per parameter (X = the core viewed as row_dim x col_dim = p x n, row-normalised):
//   Stiefel (p <= n):  V = momentum * buf - g^H;  MX = V X;  W^ = MX - 1/2 X^H X MX;
//                      W = W^ - W^H;  alpha = min(lr, 1 / (||W||_1 + 1e-8));
//                      X' = ((I - alpha/2 W)^-1 (I + alpha/2 W) X^H)^H;  buf = W X^H
//                      (optionally X <- qr_retraction(X) first: the reference's 1-in-101 draw)
//   otherwise:         SGD with weight decay / momentum / dampening / nesterov (:149-170).
// Everything is computed in the parameter's precision (complex64 -> f32), as torch does.
// The solve is Gauss-Jordan without pivoting: I - alpha/2 W has a positive definite Hermitian part
// (W is skew-Hermitian), so elimination needs no pivots.
#include <algorithm>
#include <string>

#include "tq_common.h"
#include "tq_optim.h"

namespace tq {

namespace {

constexpr int kThreads = 256;

template <typename R>
struct Cx {
  R re, im;
};
template <typename R> __device__ __forceinline__ Cx<R> cx(R a, R b = R(0)) { return {a, b}; }
template <typename R> __device__ __forceinline__ Cx<R> operator+(Cx<R> a, Cx<R> b) { return {a.re + b.re, a.im + b.im}; }
template <typename R> __device__ __forceinline__ Cx<R> operator-(Cx<R> a, Cx<R> b) { return {a.re - b.re, a.im - b.im}; }
template <typename R> __device__ __forceinline__ Cx<R> operator*(Cx<R> a, Cx<R> b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
template <typename R> __device__ __forceinline__ Cx<R> operator*(R s, Cx<R> a) { return {s * a.re, s * a.im}; }
template <typename R> __device__ __forceinline__ Cx<R> conj(Cx<R> a) { return {a.re, -a.im}; }
template <typename R> __device__ __forceinline__ R abs2(Cx<R> a) { return a.re * a.re + a.im * a.im; }
template <typename R> __device__ __forceinline__ R cabs(Cx<R> a) { return sqrt(abs2(a)); }
template <typename R> __device__ __forceinline__ Cx<R> cdiv(Cx<R> a, Cx<R> b) {
  const R d = abs2(b);
  return {(a.re * b.re + a.im * b.im) / d, (a.im * b.re - a.re * b.im) / d};
}

// element i of a stored parameter-like array (real or interleaved complex) as complex
template <typename T, typename R>
__device__ __forceinline__ Cx<R> ld(const T* p, int64_t i) {
  if constexpr (sizeof(T) == sizeof(R)) return cx<R>(reinterpret_cast<const R*>(p)[i]);
  else return cx<R>(reinterpret_cast<const R*>(p)[2 * i], reinterpret_cast<const R*>(p)[2 * i + 1]);
}
template <typename T, typename R>
__device__ __forceinline__ void st(T* p, int64_t i, Cx<R> v) {
  if constexpr (sizeof(T) == sizeof(R)) {
    reinterpret_cast<R*>(p)[i] = v.re;
  } else {
    reinterpret_cast<R*>(p)[2 * i] = v.re;
    reinterpret_cast<R*>(p)[2 * i + 1] = v.im;
  }
}

// C[M x N] = A[M x K] * B[K x N] (row-major LDS matrices; op conjugate-transposes as asked)
template <typename R, bool CA, bool CB>
__device__ void mm(Cx<R>* C, const Cx<R>* A, int lda, const Cx<R>* B, int ldb, int M, int N, int K) {
  // CA: A given as K x M (use A^H); CB: B given as N x K (use B^H)
  for (int e = threadIdx.x; e < M * N; e += kThreads) {
    const int i = e / N, j = e % N;
    Cx<R> s = cx<R>(0);
    for (int k = 0; k < K; ++k) {
      const Cx<R> a = CA ? conj(A[k * lda + i]) : A[i * lda + k];
      const Cx<R> b = CB ? conj(B[j * ldb + k]) : B[k * ldb + j];
      s = s + a * b;
    }
    C[i * N + j] = s;
  }
}

// Stiefel step for p x n parameters with 2p < n (1-D parameters, wide cores): W = W^ - W^^H has
// rank <= 2p.  With XV = X V (p x p) and U = V - 1/2 X^H XV (n x p), W^ = MX - 1/2 X^H X MX = U X,
// so W = A B with A = [U | -X^H] (n x 2p) and B = [X ; U^H] (2p x n).  Then (Woodbury)
//   buf' = W X^H = A (B X^H),   Z = (I + hW) X^H = X^H + h buf',
//   Y = (I - hW)^-1 Z = Z + h A (I_2p - h B A)^-1 B Z,
// the same quantities as the dense path (compute_Y, stiefel_optimizer_complex.py:66-74) in
// O(n^2 p) work (the 1-norm of W, column sums of |A B|) and O(n p) scratch instead of O(n^3) and
// O(n^2).  The 2p x 2p system is solved with partial pivoting.
// Scratch (after X p*n | V n*p): U n*p | Z n*p | XV p*p | BX 2p*p | S 2p*(3p) | n reals.
template <typename T, typename R>
__device__ void lowrank_step(Cx<R>* X, Cx<R>* V, R lr, T* buf, T* prm, int p, int n) {
  const int tid = threadIdx.x, q = 2 * p, sa = 3 * p;
  Cx<R>* U = V + n * p;
  Cx<R>* Z = U + n * p;
  Cx<R>* XV = Z + n * p;
  Cx<R>* BX = XV + p * p;
  Cx<R>* S = BX + q * p;
  R* red = reinterpret_cast<R*>(S + q * sa);   // (== the caller's `red`: X + 4pn + 9p^2)
  __shared__ R s_red[kThreads];
  __shared__ int s_piv;
  // A[i][c] and B[c][j] read in place from U and X
  auto Aat = [&](int i, int c) { return c < p ? U[i * p + c] : cx<R>(0) - conj(X[(c - p) * n + i]); };
  auto Bat = [&](int c, int j) { return c < p ? X[c * n + j] : conj(U[j * p + (c - p)]); };
  // XV = X V (p x p)
  mm<R, false, false>(XV, X, n, V, p, p, p, n);
  __syncthreads();
  // U = V - 1/2 X^H XV
  for (int e = tid; e < n * p; e += kThreads) {
    const int i = e / p, j = e % p;
    Cx<R> s = cx<R>(0);
    for (int k = 0; k < p; ++k) s = s + conj(X[k * n + i]) * XV[k * p + j];
    U[e] = V[e] - R(0.5) * s;
  }
  __syncthreads();
  // ||W||_1 = max_j sum_i |(A B)_ij|
  R cmax = 0;
  for (int j = tid; j < n; j += kThreads) {
    R s = 0;
    for (int i = 0; i < n; ++i) {
      Cx<R> w = cx<R>(0);
      for (int c = 0; c < q; ++c) w = w + Aat(i, c) * Bat(c, j);
      s += cabs(w);
    }
    cmax = s > cmax ? s : cmax;
  }
  s_red[tid] = cmax;
  __syncthreads();
  for (int w = kThreads / 2; w > 0; w >>= 1) {
    if (tid < w) s_red[tid] = s_red[tid + w] > s_red[tid] ? s_red[tid + w] : s_red[tid];
    __syncthreads();
  }
  const R nrm = s_red[0];
  const R t = R(0.5) * R(2) / (nrm + R(1e-8));
  const R h = (t < lr ? t : lr) / R(2);
  // BX = B X^H (2p x p)
  for (int e = tid; e < q * p; e += kThreads) {
    const int c = e / p, j = e % p;
    Cx<R> s = cx<R>(0);
    for (int k = 0; k < n; ++k) s = s + Bat(c, k) * conj(X[j * n + k]);
    BX[e] = s;
  }
  __syncthreads();
  // buf' = A BX (n x p) -> momentum buffer;  Z = X^H + h buf'
  for (int e = tid; e < n * p; e += kThreads) {
    const int i = e / p, j = e % p;
    Cx<R> s = cx<R>(0);
    for (int c = 0; c < q; ++c) s = s + Aat(i, c) * BX[c * p + j];
    st<T, R>(buf, e, s);
    Z[e] = conj(X[j * n + i]) + h * s;
  }
  __syncthreads();
  // augmented 2p x 3p system [I - h B A | B Z]
  for (int e = tid; e < q * sa; e += kThreads) {
    const int c = e / sa, d = e % sa;
    Cx<R> s = cx<R>(0);
    if (d < q) {
      for (int k = 0; k < n; ++k) s = s + Bat(c, k) * Aat(k, d);
      S[e] = (c == d ? cx<R>(1) : cx<R>(0)) - h * s;
    } else {
      for (int k = 0; k < n; ++k) s = s + Bat(c, k) * Z[k * p + (d - q)];
      S[e] = s;
    }
  }
  __syncthreads();
  // Gauss-Jordan with partial pivoting (2p rows)
  for (int k = 0; k < q; ++k) {
    if (tid == 0) {
      int best = k;
      R bv = abs2(S[k * sa + k]);
      for (int r = k + 1; r < q; ++r) {
        const R v = abs2(S[r * sa + k]);
        if (v > bv) { bv = v; best = r; }
      }
      s_piv = best;
    }
    __syncthreads();
    const int pr = s_piv;
    if (pr != k)
      for (int j = tid; j < sa; j += kThreads) {
        const Cx<R> a = S[k * sa + j];
        S[k * sa + j] = S[pr * sa + j];
        S[pr * sa + j] = a;
      }
    __syncthreads();
    const Cx<R> piv = S[k * sa + k];
    __syncthreads();
    for (int j = tid; j < sa; j += kThreads) S[k * sa + j] = cdiv(S[k * sa + j], piv);
    __syncthreads();
    for (int e = tid; e < q * sa; e += kThreads) {
      const int i = e / sa, j = e % sa;
      if (i != k && j != k) S[e] = S[e] - S[i * sa + k] * S[k * sa + j];
    }
    __syncthreads();
    for (int i = tid; i < q; i += kThreads)
      if (i != k) S[i * sa + k] = cx<R>(0);
    __syncthreads();
  }
  // Y = Z + h A R (R = the solved right block); parameter <- Y^H
  for (int64_t e = tid; e < (int64_t)p * n; e += kThreads) {
    const int r = (int)(e / n), i = (int)(e % n);
    Cx<R> s = cx<R>(0);
    for (int c = 0; c < q; ++c) s = s + Aat(i, c) * S[c * sa + q + r];
    st<T, R>(prm, e, conj(Z[i * p + r] + h * s));
  }
  (void)red;
}

template <typename T, typename R, bool GM>
__global__ void __launch_bounds__(kThreads) sgdg_kernel(const SgdgLaunch L) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const SgdgParam P = L.p[blockIdx.x];
  // GM launches hold only the large Stiefel parameters (and small ones: GM == false)
  if (GM != (P.ws != nullptr)) return;
  const int p = P.rows, n = P.cols;
  const int64_t numel = (int64_t)p * n;
  const int tid = threadIdx.x;
  T* prm = reinterpret_cast<T*>(P.param);
  T* grd = reinterpret_cast<T*>(P.grad);
  T* buf = reinterpret_cast<T*>(P.buf);
  const R lr = (R)L.lr, mom = (R)L.momentum;
  if (!(P.flags & kSgdgStiefel)) {
    // ---- plain SGD branch (stiefel_optimizer_complex.py:149-170), elementwise
    const R wd = (R)L.weight_decay, damp = (R)L.dampening;
    for (int64_t i = tid; i < numel; i += kThreads) {
      Cx<R> d = ld<T, R>(grd, i);
      const Cx<R> x = ld<T, R>(prm, i);
      if (L.weight_decay != 0.0) {
        d = d + wd * x;
        st<T, R>(grd, i, d);   // d_p.add_(weight_decay, p.data) updates p.grad in place
      }
      if (L.momentum != 0.0) {
        Cx<R> b;
        if (P.flags & kSgdgBufInit) b = mom * ld<T, R>(buf, i) + (R(1) - damp) * d;
        else b = d;            // first step: buf = d_p.clone()
        st<T, R>(buf, i, b);
        d = L.nesterov ? d + mom * b : b;
      }
      st<T, R>(prm, i, x - lr * d);
    }
    return;
  }
  // ---- Stiefel branch: LDS layout (complex<R>): X p*n | V n*p | MX n*n | T1 p*n | W n*n |
  //      aug n*(n+p) | norms
  Cx<R>* X = reinterpret_cast<Cx<R>*>(GM ? static_cast<char*>(P.ws) : smem_raw);
  Cx<R>* V = X + p * n;
  Cx<R>* MX = V + n * p;
  Cx<R>* T1 = MX + n * n;
  Cx<R>* W = T1 + p * n;
  Cx<R>* A = W + n * n;      // n x (n + p) augmented system
  // n reals of scratch: at the end of the layout the step uses (the low-rank form's scratch is
  // O(n p): the dense layout's offsets lie far beyond it)
  const bool lowrank = GM && 2 * p < n;
  R* red = lowrank ? reinterpret_cast<R*>(X + (size_t)p * n * 4 + (size_t)p * p * 9)
                   : reinterpret_cast<R*>(A + n * (n + p));
  const int na = n + p;
  // 1) X = unit(P): rows divided by (row 2-norm + 1e-8)           gutils.py:7-9
  for (int64_t i = tid; i < numel; i += kThreads) X[i] = ld<T, R>(prm, i);
  __syncthreads();
  for (int r = tid; r < p; r += kThreads) {
    R s = 0;
    for (int c = 0; c < n; ++c) s += abs2(X[r * n + c]);
    red[r] = sqrt(s) + R(1e-8);
  }
  __syncthreads();
  for (int64_t i = tid; i < numel; i += kThreads) X[i] = (R(1) / red[i / n]) * X[i];
  __syncthreads();
  // 2) optional qr_retraction (gutils.py:62-83): positive-diagonal QR of X^H == Gram-Schmidt of the
  //    rows of X in the inner product u^H v (one wave; p, n <= 32)
  if (P.flags & kSgdgRetract) {
    if (tid < 64) {
      for (int j = 0; j < p; ++j) {
        for (int i = 0; i < j; ++i) {
          // coefficient <x_i, x_j> = sum_k conj(x_i[k]) x_j[k]  (x_i already orthonormal)
          Cx<R> s = cx<R>(0);
          for (int k = 0; k < n; ++k) s = s + conj(X[i * n + k]) * X[j * n + k];
          __builtin_amdgcn_wave_barrier();
          for (int k = tid; k < n; k += 64) X[j * n + k] = X[j * n + k] - s * X[i * n + k];
          __builtin_amdgcn_wave_barrier();
        }
        R s = 0;
        for (int k = 0; k < n; ++k) s += abs2(X[j * n + k]);
        const R inv = R(1) / sqrt(s);
        __builtin_amdgcn_wave_barrier();
        for (int k = tid; k < n; k += 64) X[j * n + k] = inv * X[j * n + k];
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
  }
  // 3) V = momentum * buf - g^H   (n x p)
  for (int e = tid; e < n * p; e += kThreads) {
    const int i = e / p, j = e % p;
    const Cx<R> g = conj(ld<T, R>(grd, (int64_t)j * n + i));
    const Cx<R> b = (P.flags & kSgdgBufInit) ? ld<T, R>(buf, e) : cx<R>(0);
    V[e] = mom * b - g;
  }
  __syncthreads();
  if constexpr (GM) {
    if (lowrank) {   // W has rank <= 2p < n: the low-rank (Woodbury) form, O(n^2 p) not O(n^3)
      lowrank_step<T, R>(X, V, lr, buf, prm, p, n);
      return;
    }
  }
  // 4) MX = V X (n x n);  XMX = X MX (p x n);  XXMX = X^H XMX (n x n) -> W^ = MX - 1/2 XXMX
  mm<R, false, false>(MX, V, p, X, n, n, n, p);
  __syncthreads();
  mm<R, false, false>(T1, X, n, MX, n, p, n, n);
  __syncthreads();
  mm<R, true, false>(W, X, n, T1, n, n, n, p);   // W <- X^H XMX
  __syncthreads();
  for (int e = tid; e < n * n; e += kThreads) W[e] = MX[e] - R(0.5) * W[e];   // W <- W^
  __syncthreads();
  // W = W^ - W^^H: MX is free now, build there then swap roles
  for (int e = tid; e < n * n; e += kThreads) {
    const int i = e / n, j = e % n;
    MX[e] = W[e] - conj(W[j * n + i]);
  }
  __syncthreads();
  Cx<R>* Wf = MX;
  // 5) alpha = min(lr, 0.5 * 2 / (||W||_1 + 1e-8)), ||W||_1 = max column sum of |W|
  for (int c = tid; c < n; c += kThreads) {
    R s = 0;
    for (int r = 0; r < n; ++r) s += cabs(Wf[r * n + c]);
    red[c] = s;
  }
  __syncthreads();
  R nrm = 0;
  for (int c = 0; c < n; ++c) nrm = red[c] > nrm ? red[c] : nrm;
  const R t = R(0.5) * R(2) / (nrm + R(1e-8));
  const R alpha = t < lr ? t : lr;
  const R h = alpha / R(2);
  // 6) buf <- W X^H (n x p): V_new, the next step's momentum buffer
  mm<R, false, true>(V, Wf, n, X, n, n, p, n);
  __syncthreads();
  for (int e = tid; e < n * p; e += kThreads) st<T, R>(buf, e, V[e]);
  // 7) augmented system [I - h W | (I + h W) X^H]
  for (int e = tid; e < n * na; e += kThreads) {
    const int i = e / na, j = e % na;
    if (j < n) {
      A[e] = (i == j ? cx<R>(1) : cx<R>(0)) - h * Wf[i * n + j];
    } else {
      const int c = j - n;
      A[e] = conj(X[c * n + i]) + h * V[i * p + c];   // X^H + h W X^H
    }
  }
  __syncthreads();
  // 8) Gauss-Jordan: A <- [I | L^-1 R X^H]
  for (int k = 0; k < n; ++k) {
    const Cx<R> piv = A[k * na + k];
    __syncthreads();
    for (int j = tid; j < na; j += kThreads) A[k * na + j] = cdiv(A[k * na + j], piv);
    __syncthreads();
    for (int e = tid; e < n * na; e += kThreads) {
      const int i = e / na, j = e % na;
      if (i != k) {
        const Cx<R> f = A[i * na + k];
        if (j != k) A[e] = A[e] - f * A[k * na + j];
      }
    }
    __syncthreads();
    for (int i = tid; i < n; i += kThreads)
      if (i != k) A[i * na + k] = cx<R>(0);
    __syncthreads();
  }
  // 9) parameter <- Y^H  (Y = the n x p right block)
  for (int64_t e = tid; e < numel; e += kThreads) {
    const int r = (int)(e / n), c = (int)(e % n);
    st<T, R>(prm, e, conj(A[c * na + n + r]));
  }
}

// X p*n | V n*p | MX n*n | T1 p*n | W n*n | aug n*(n+p) | n reals
template <typename R>
size_t stiefel_bytes(int p, int n) {
  const size_t cells = (size_t)p * n * 2 + (size_t)n * n * 2 + (size_t)n * p + (size_t)n * (n + p);
  return cells * sizeof(Cx<R>) + (size_t)std::max(n, p) * sizeof(R) + 16;
}

// the global-scratch low-rank form (lowrank_step): X p*n | V n*p | U n*p | Z n*p | XV p*p |
// BX 2p*p | S 2p*3p | n reals
template <typename R>
size_t lowrank_bytes(int p, int n) {
  const size_t cells = (size_t)p * n * 4 + (size_t)p * p + (size_t)2 * p * p + (size_t)6 * p * p;
  return cells * sizeof(Cx<R>) + (size_t)n * sizeof(R) + 16;
}

template <typename R>
size_t global_bytes(int p, int n) {
  return 2 * p < n ? lowrank_bytes<R>(p, n) : stiefel_bytes<R>(p, n);
}

template <typename T, typename R>
int launch_t(const SgdgLaunch& L, hipStream_t stream) {
  int maxn = 1, maxp = 1;
  bool small = false, large = false;
  for (int i = 0; i < L.n; ++i) {
    large = large || L.p[i].ws != nullptr;
    small = small || L.p[i].ws == nullptr;
    if ((L.p[i].flags & kSgdgStiefel) && !L.p[i].ws) {
      maxn = std::max(maxn, L.p[i].cols);
      maxp = std::max(maxp, L.p[i].rows);
    }
  }
  if (small) {
    hipLaunchKernelGGL((sgdg_kernel<T, R, false>), dim3(L.n), dim3(kThreads), stiefel_bytes<R>(maxp, maxn), stream, L);
    TQ_HIP(hipGetLastError());
  }
  if (large) {
    hipLaunchKernelGGL((sgdg_kernel<T, R, true>), dim3(L.n), dim3(kThreads), 16, stream, L);
    TQ_HIP(hipGetLastError());
  }
  return TQ_OK;
}

}  // namespace

size_t sgdg_ws_bytes(int dtype, int rows, int cols) {
  return (dtype == TQ_F64 || dtype == TQ_C128) ? global_bytes<double>(rows, cols) : global_bytes<float>(rows, cols);
}

int sgdg_launch(int dtype, const SgdgLaunch& L, hipStream_t stream) {
  if (L.n <= 0) return TQ_OK;
  if (L.n > kSgdgMaxBatch) {
    set_error("sgdg: too many parameters in one launch");
    return TQ_ERR_INVALID;
  }
  for (int i = 0; i < L.n; ++i) {
    const SgdgParam& q = L.p[i];
    if (!q.param || !q.grad || (!q.buf && (q.flags & kSgdgStiefel || L.momentum != 0.0)) ||
        q.rows < 1 || q.cols < 1) {
      set_error("sgdg: bad parameter descriptor");
      return TQ_ERR_INVALID;
    }
    if ((q.flags & kSgdgStiefel) &&
        (q.rows > q.cols || q.cols > kSgdgMaxDimGlobal || (q.cols > kSgdgMaxDim && !q.ws))) {
      set_error("sgdg: Stiefel parameters need rows <= cols <= " + std::to_string(kSgdgMaxDimGlobal) +
                " (a global scratch above " + std::to_string(kSgdgMaxDim) + ")");
      return TQ_ERR_UNSUPPORTED;
    }
    if (q.ws && !(q.flags & kSgdgStiefel)) {
      set_error("sgdg: scratch given for a non-Stiefel parameter");
      return TQ_ERR_INVALID;
    }
  }
  switch (dtype) {
    case TQ_F32: return launch_t<float, float>(L, stream);
    case TQ_F64: return launch_t<double, double>(L, stream);
    case TQ_C64: return launch_t<c64, float>(L, stream);
    case TQ_C128: return launch_t<c128, double>(L, stream);
  }
  set_error("sgdg: bad dtype");
  return TQ_ERR_INVALID;
}

}  // namespace tq
