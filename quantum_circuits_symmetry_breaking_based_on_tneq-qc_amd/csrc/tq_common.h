// Shared internals of libtneqhip: error state, element traits, small helpers.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/tneqhip.h"

namespace tq {

// ---- error reporting (thread-local last error, surfaced through tq_last_error) ----------
void set_error(const std::string& msg);
const std::string& last_error();

#define TQ_CHECK_ARG(cond, msg)                                   \
  do {                                                            \
    if (!(cond)) {                                                \
      ::tq::set_error(std::string("invalid argument: ") + (msg)); \
      return TQ_ERR_INVALID;                                      \
    }                                                             \
  } while (0)

#define TQ_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      ::tq::set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " +     \
                      __FILE__ + ":" + std::to_string(__LINE__));                      \
      return TQ_ERR_HIP;                                                               \
    }                                                                                  \
  } while (0)

// ---- per-device cache of a launch parameter derived from the device (occupancy caps) -------
// One slot per (device ordinal, key); 0 = not computed yet.  Concurrent first uses may compute
// the value twice (the same value) but never race on the slot.
constexpr int kMaxDevices = 64;
template <int NKEYS>
struct DeviceCache {
  std::atomic<int> v[kMaxDevices][NKEYS] = {};
  // the cached value of `key` on the current device, computed by `fn()` on first use
  template <typename F>
  int get(int key, F&& fn) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return fn();
    int x = v[dev][key].load(std::memory_order_relaxed);
    if (x == 0) {
      x = fn();
      v[dev][key].store(x, std::memory_order_relaxed);
    }
    return x;
  }
};

#define TQ_TRY(expr)        \
  do {                      \
    int rc_ = (expr);       \
    if (rc_ != TQ_OK) return rc_; \
  } while (0)

inline size_t dtype_size(int dt) {
  switch (dt) {
    case TQ_F32: return 4;
    case TQ_F64: return 8;
    case TQ_C64: return 8;
    case TQ_C128: return 16;
    default: return 0;
  }
}
inline bool dtype_complex(int dt) { return dt == TQ_C64 || dt == TQ_C128; }
inline bool dtype_valid(int dt) { return dt >= TQ_F32 && dt <= TQ_C128; }

// Storage element types for the kernels.  Complex values are interleaved (re, im).
// Naturally aligned (8 B / 16 B) so that one element is one global / LDS access, not two.
struct alignas(8) c64 { float re, im; };
struct alignas(16) c128 { double re, im; };

template <typename T> struct Traits;
template <> struct Traits<float>  { using R = float;  static constexpr bool cplx = false; static constexpr int code = TQ_F32; };
template <> struct Traits<double> { using R = double; static constexpr bool cplx = false; static constexpr int code = TQ_F64; };
template <> struct Traits<c64>    { using R = float;  static constexpr bool cplx = true;  static constexpr int code = TQ_C64; };
template <> struct Traits<c128>   { using R = double; static constexpr bool cplx = true;  static constexpr int code = TQ_C128; };

__host__ __device__ inline c64 operator+(c64 a, c64 b) { return {a.re + b.re, a.im + b.im}; }
__host__ __device__ inline c128 operator+(c128 a, c128 b) { return {a.re + b.re, a.im + b.im}; }
__host__ __device__ inline c64 operator*(c64 a, float s) { return {a.re * s, a.im * s}; }
__host__ __device__ inline c128 operator*(c128 a, double s) { return {a.re * s, a.im * s}; }

// complex fused multiply-add acc += a*b (no conjugation)
__device__ __forceinline__ void cmac(float& acc, float a, float b) { acc = fmaf(a, b, acc); }
__device__ __forceinline__ void cmac(double& acc, double a, double b) { acc = fma(a, b, acc); }
__device__ __forceinline__ void cmac(c64& acc, c64 a, c64 b) {
  acc.re = fmaf(a.re, b.re, acc.re); acc.re = fmaf(-a.im, b.im, acc.re);
  acc.im = fmaf(a.re, b.im, acc.im); acc.im = fmaf(a.im, b.re, acc.im);
}
__device__ __forceinline__ void cmac(c128& acc, c128 a, c128 b) {
  acc.re = fma(a.re, b.re, acc.re); acc.re = fma(-a.im, b.im, acc.re);
  acc.im = fma(a.re, b.im, acc.im); acc.im = fma(a.im, b.re, acc.im);
}
template <typename T> __host__ __device__ inline T tzero() { return T{}; }

inline int64_t prod(const std::vector<int64_t>& v) {
  int64_t p = 1;
  for (auto x : v) p *= x;
  return p;
}

// ---- kernel launchers implemented in the .hip files -------------------------------------
// permute (tq_permute.hip)
int permute_launch(int dtype, int rank, const int64_t* shape, const int64_t* src_strides,
                   const void* src, void* dst, double beta, hipStream_t stream);
// gemm (tq_gemm.hip)
int gemm_launch(int dtype, int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch,
                const void* A, int64_t lda, int64_t strideA, const void* B, int64_t ldb,
                int64_t strideB, double beta, void* C, int64_t ldc, int64_t strideC,
                void* workspace, size_t ws_bytes, hipStream_t stream,
                const uint32_t* amax_a = nullptr, const uint32_t* amax_b = nullptr,
                const struct GemmPresplit* presplit = nullptr, int amax_bs_a = 0, int amax_bs_b = 0);
// Operands stored as f16 terms by their producers (S2Op::split_sc; complex64 K-outer f16 path):
// every element holds (h_re, h_im | l_re, l_im) of the value scaled by 2^sc.  The GEMM checks the
// producers' true max words against the scales: outside the window (max * 2^sc in [2^0, 2^15))
// it writes zeros and sets *bad = 1 (else 0), and the plan re-runs that slice on the split path.
struct GemmPresplit {
  const int32_t* sc_a = nullptr;
  const int32_t* sc_b = nullptr;
  uint32_t* bad = nullptr;
};
// plan-time / run-time eligibility of a GEMM for pre-split operands (the launch would take the
// f16 split kernel), the library switch (TQ_GEMM_PRESPLIT, "gemm_presplit") and the scale
// prediction offset (testing: "presplit_bias" forces the fallback)
bool gemm_c64_presplit_ok(int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch,
                          int64_t lda, int64_t ldb);
bool gemm_presplit_enabled();
// per slice, before the producers: sc[i] = scale for the next operand from the previous max
// (amax[i]; 0 = none yet), amax[i] = 0
int presplit_prep_launch(uint32_t* amax, int32_t* sc, int n, hipStream_t stream);
// amax_a / amax_b (optional, complex64): float bits of max |re|, |im| over A / B, written by the
// operands' producers (plan: the sweep ops that store them); the f16-split kernel then skips its
// own max pre-pass over A and B.  amax_bs_a / amax_bs_b: word stride between batch entries (0: one
// word for the whole batch; plan slice lanes: n_amax_slice, every lane scaled by its own max).
// Without the words the pre-pass keeps one max per batch entry and operand.
size_t gemm_workspace(int dtype, int64_t M, int64_t N, int64_t K, int64_t batch);
// Strided skinny contraction (tq_gemm.hip): C[m][n] (M x N contiguous, M * N <= 16, M, N powers
// of two) = sum_k A(m, k) B(k, n) where every index is a bit string of power-of-two modes read
// through per-bit element strides (w*), so no operand is permuted first -- the gradient steps of
// a reverse-mode tree (a gate's gradient against a large tensor in any mode order).
constexpr int kSkMaxKBits = 24;
struct SkinnyArgs {
  const void* A = nullptr;
  const void* B = nullptr;
  void* C = nullptr;
  void* W = nullptr;            // partials (P x M x N elements) when P > 1
  int64_t K = 0;
  int nkb = 0;                  // K = 2^nkb
  int M = 1, N = 1;
  double beta = 0;
  int64_t wam[4] = {}, wbn[4] = {};                     // bit b of m / n
  int64_t wak[kSkMaxKBits] = {}, wbk[kSkMaxKBits] = {}; // bit b of k
};
// partial blocks of a strided skinny contraction over K (its workspace = P x M x N elements)
int skinny_blocks(int64_t K);
int skinny_strided_launch(int dtype, const SkinnyArgs& a, hipStream_t stream);
// apply a small operand along (at most two runs of) contracted modes (tq_apply.hip):
//   C[o][n][m][i] = sum_{k1,k2} S[o][k1][m][k2][i] * G[k1*K2+k2][n]   (S, C, G contiguous)
int apply_launch(int dtype, int64_t O, int64_t K1, int64_t M, int64_t K2, int64_t I, int64_t N,
                 const void* S, const void* G, const int32_t* gidx, void* C, double beta,
                 hipStream_t stream);
int axpy_launch(int dtype, int64_t n, const void* x, void* y, double beta, hipStream_t stream);
// The boundary GEMM on operands pre-split by their producer into six f16 planes (tq_gemmp.hip):
// C = A^T B complex64 (K-outer operands), f32 accuracy on the f16 matrix cores (Gauss 3M x 3 term
// products).  Batch entry b's plane p of A is A + b sA + p psA, element (k, m) at k lda + m
// (planes re_h, re_l, im_h, im_l, s_h, s_l; s = re + im scaled one binade lower); B likewise.
struct PlanesGemmArgs {
  const _Float16* A = nullptr;
  const _Float16* B = nullptr;
  int64_t sA = 0, sB = 0, psA = 0, psB = 0, lda = 0, ldb = 0;
  int M = 0, N = 0, batch = 1, splits = 1;   // splits: set by the launcher
  int64_t K = 0;
  float* W = nullptr;                        // partials, planes_gemm_workspace bytes
  size_t ws_bytes = 0;                       // capacity of W (the launcher refuses a launch beyond it)
};
// C + j sC (complex64, row stride ldc; one output when lane_sum) = [sum over batch entries j]
// 2^-(sc_a[j stride] + sc_b[j stride]) x the complex product + beta C
struct PlanesCombineArgs {
  const float* W = nullptr;
  int M = 0, N = 0, batch = 1, splits = 1;   // set by the launcher
  const int32_t* sc_a = nullptr;
  const int32_t* sc_b = nullptr;
  int64_t sc_stride = 0;
  void* C = nullptr;
  int64_t ldc = 0, sC = 0;
  int lane_sum = 0;
  float beta = 0.f;
};
bool planes_gemm_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);
int planes_gemm_splits(int64_t M, int64_t N, int64_t K, int64_t batch);
size_t planes_gemm_workspace(int64_t M, int64_t N, int64_t K, int64_t batch);
int planes_gemm_kclock(unsigned long long* out, int n);   // -DTQ_KCLOCK builds (tq_kclock.h)
int kouter_kclock(unsigned long long* out, int n);
int planes_gemm_check(int64_t M, int64_t N, int64_t K, int64_t batch, int64_t lda, int64_t ldb, size_t ws_bytes);
int planes_gemm_launch(const PlanesGemmArgs& a, const PlanesCombineArgs& c, hipStream_t stream);
// y[i] = sum_{j < nl} y[i + j * stride] (elements), i < n: slice lanes summed into lane 0
int lane_sum_launch(int dtype, int64_t n, void* y, int64_t stride, int nl, hipStream_t stream);
// measurement data (tq_data.hip)
int hermite_launch(int dtype, int64_t n, int K, const double* x, const double* w, void* phi,
                   void* mx, hipStream_t stream);
int icdf_launch(int dtype, int64_t rows, int64_t grid_size, const void* density, int64_t ld,
                const void* grid_x, const float* u, void* out, int64_t out_stride,
                hipStream_t stream);
// fidelity loss of the symmetry-breaking fit (tq_loss.hip)
int fidelity_forward_launch(int dtype, int64_t n, const void* t, const void* o, double* stats, void* loss,
                            hipStream_t stream);
int fidelity_backward_launch(int dtype, int64_t n, const void* t, const void* o, const double* stats,
                             const void* g, void* grad, hipStream_t stream);

}  // namespace tq
