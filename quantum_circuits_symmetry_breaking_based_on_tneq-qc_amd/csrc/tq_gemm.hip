// Batched GEMM on gfx950 matrix cores for the inner product of every pairwise contraction.
//
// Replaces the GEMM under each tensordot of the reference's opt_einsum pairwise loop
// (tneq_qc/contractor/einsum_strategy.py:639-643 -> torch.tensordot -> at::mm) and the
// explicit partial bmm of the K-sharded reduce (tneq_qc/distributed/engine/distributed_engine.py:1477-1487).
//
//  * f32 / complex64  : v_mfma_f32_32x32x2_f32 (exact f32, 64 FLOP/clk/SIMD = FP32 peak).
//                       block 128x128, 4 waves of 64x64, BK = 16.
//  * f64 / complex128 : v_mfma_f64_16x16x4_f64. block 64x64, 4 waves of 32x32, BK = 16.
//  * complex = 4 real MFMAs per complex k-step on split re/im LDS planes
//      Cr += Ar*Br + (-Ai)*Bi ; Ci += Ar*Bi + Ai*Br     (8 real flops per complex MAC).
//  * operands staged global -> registers -> LDS (next tile's global loads are issued before the
//    current tile's MFMAs, written after the barrier), 16-byte vector loads where aligned.
//  * split-K over blockIdx.z with fp partial slabs + a deterministic reduce kernel when the
//    output tile count alone cannot fill 256 CUs.
//  * XCD-aware tile order: tiles that share an A row panel are dealt to the same XCD.
#include <algorithm>
#include <atomic>
#include <string>
#include <cstdlib>
#include <type_traits>

#include "tq_common.h"
#include "tq_kclock.h"

namespace tq {

// The fast path computes complex products with Gauss's 3 real multiplications (default; the C4
// amplitudes stay within 4.0e-6 of complex128, vs 2.7e-6 for the 4-multiplication product);
// TQ_GEMM_3M=0 selects the 4-multiplication kernel.
static int env_flag(const char* name) {
  const char* e = getenv(name);
  return (e && e[0] == '0') ? 0 : 1;
}
static std::atomic<int> g_gemm_3m{env_flag("TQ_GEMM_3M")};
static std::atomic<int> g_gemm_bf16{env_flag("TQ_GEMM_BF16")};
static std::atomic<int> g_gemm_f16{env_flag("TQ_GEMM_F16")};
static int env_int(const char* name, int dflt = 0) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
// f16-split tile variant: 0 = 8 waves of 64 x 32 with the 4-multiplication complex product,
// 1 = 4 waves of 64 x 64, 3 = tile 0 on a 4-slot LDS ring (one barrier per two K-steps), 2 = 4
// waves of 64 x 64 with Gauss's 3-multiplication product, 4 = tile 0 on v_mfma_f32_16x16x32_f16
// (K-chunks that are a multiple of 32; others run variant 0), 5 = tile 0 with Gauss's product: 9
// instead of 12 MFMAs per complex tile-step (the GEMM runs power-limited, so the fewer MFMAs are
// time: C4 r03 5.20 vs 5.60 ms per 4-slice launch), 6 (default) = variant 5 with 3 staging sets
// (loads two K-steps ahead), room made by the ordered term pairs (5.13 vs 5.19-5.25 ms).
// Measurements: DESIGN.md §3
static std::atomic<int> g_gemm_f16_var{env_int("TQ_GEMM_F16_VAR", 6)};
// static wave priority in the f16 split kernel (TQ_GEMM_PRIO=1): the second-dispatched half of
// the 8 waves (threads >= NT / 2) runs at s_setprio 1 for the whole main loop
// (cdna_hip_programming.md T5 static form: the younger half loses VALU arbitration otherwise)
static const int g_gemm_prio = env_int("TQ_GEMM_PRIO", 0);
int gemm_f16_var() { return g_gemm_f16_var.load(std::memory_order_relaxed); }
bool gemm_3m() { return g_gemm_3m.load(std::memory_order_relaxed) != 0; }
// The complex64 K-outer fast path runs on the bf16 matrix cores with an exact 3-term split of
// every f32 operand (gemm_c64_kouter_split_kernel<TileX, SplitBF16>, f32 accuracy); TQ_GEMM_BF16=0 (or
// tq_library_set("gemm_bf16", 0)) selects the f32-MFMA kernel.
bool gemm_bf16() { return g_gemm_bf16.load(std::memory_order_relaxed) != 0; }
// ... and, by default, on the f16 matrix cores with a 2-term split of the power-of-two-scaled
// operands (gemm_c64_kouter_split_kernel<TileH, SplitF16>, f32 accuracy, half the MFMAs of the
// bf16 3-term split); TQ_GEMM_F16=0 (or tq_library_set("gemm_f16", 0)) keeps the bf16 split.
bool gemm_f16() { return g_gemm_f16.load(std::memory_order_relaxed) != 0; }
// runtime switch (tq_library_set): affects launches issued after the call (plans replaying a
// captured hipGraph keep the kernels they captured)
// pre-split operands (GemmPresplit) are opt-in: measured on C4 (r02) the GEMM
// took 1.375 ms vs 1.34-1.39 ms on the split path while the producers' f16 stores added 0.37 ms
// of sweep time per step -- the split arithmetic is not what bounds the kernel
static int env_on(const char* name) {
  const char* e = getenv(name);
  return (e && e[0] == '1') ? 1 : 0;
}
static std::atomic<int> g_gemm_presplit{env_on("TQ_GEMM_PRESPLIT")};
static std::atomic<int> g_presplit_bias{env_int("TQ_PRESPLIT_BIAS")};
bool gemm_presplit_enabled() { return g_gemm_presplit.load(std::memory_order_relaxed) != 0; }
int presplit_bias() { return g_presplit_bias.load(std::memory_order_relaxed); }
bool gemm_configure(const char* key, int64_t v) {
  const std::string k(key);
  if (k == "gemm_presplit") { g_gemm_presplit = v ? 1 : 0; return true; }
  if (k == "presplit_bias") {
    if (v < -64 || v > 64) return false;
    g_presplit_bias = (int)v;
    return true;
  }
  if (k == "gemm_3m") { g_gemm_3m = v ? 1 : 0; return true; }
  if (k == "gemm_bf16") { g_gemm_bf16 = v ? 1 : 0; return true; }
  if (k == "gemm_f16") { g_gemm_f16 = v ? 1 : 0; return true; }
  if (k == "gemm_f16_var") {
    if (v < 0 || v > 9) return false;
    g_gemm_f16_var = (int)v;
    return true;
  }
  return false;
}

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

// Tile configuration per (real type, complex).  Measured (r02, scripts/gemm64_bench.py): wave tiles
// of 64 x 128 (f32) / 64 x 64 (f64) for the real GEMMs drop to one wave per SIMD in this
// register-staged, single-buffered kernel and lose 5-15 %, so every variant keeps 2 x 2 MFMA
// tiles per wave.
template <typename R, bool CPLX> struct Cfg;
template <bool CPLX> struct CfgF32 {
  static constexpr int MT = 32, KT = 2;          // MFMA tile M=N and K
  static constexpr int TI = 2, TJ = 2;           // MFMA tiles per wave (rows, cols)
  static constexpr int WM = MT * TI, WN = MT * TJ;
  static constexpr int BM = 2 * WM, BN = 2 * WN; // 2x2 waves
  static constexpr int BK = 16;
  static constexpr int PAD = 0;                  // ds_read_b32 halves read distinct rows: no conflict
  static constexpr int NACC = 16;                // accumulator values per MFMA tile per lane
};
template <bool CPLX> struct CfgF64 {
  static constexpr int MT = 16, KT = 4;
  static constexpr int TI = 2, TJ = 2;
  static constexpr int WM = MT * TI, WN = MT * TJ;
  static constexpr int BM = 2 * WM, BN = 2 * WN;
  static constexpr int BK = 16;
  static constexpr int PAD = 16;                 // rows k, k+1 of a ds_read_b64 half -> other banks
  static constexpr int NACC = 4;
};
template <> struct Cfg<float, false> : CfgF32<false> {};
template <> struct Cfg<float, true> : CfgF32<true> {};
template <> struct Cfg<double, false> : CfgF64<false> {};
template <> struct Cfg<double, true> : CfgF64<true> {};

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  void* W;  // split-K partial slabs (splits x batch x M x N elements) or null
  int64_t M, N, K, lda, ldb, ldc, sA, sB, sC, batch;
  int64_t kchunk;
  int splits;
  int mt, nt;  // tile counts
  int vecA, vecB;
  double beta;
};

constexpr int kThreads = 256;
// f16 split: max-word block behind the split-K slabs (two words per batch entry)
inline size_t amax_bytes(int64_t batch) { return ((size_t)batch * 8 + 255) / 256 * 256; }

// TQ_GEMM_FAST=0 disables the K-outer complex64 fast path (A/B timing of the two kernels)
bool fast_disabled() {
  static const int v = [] {
    const char* e = getenv("TQ_GEMM_FAST");
    return (e && e[0] == '0') ? 1 : 0;
  }();
  return v != 0;
}

// TQ_GEMM_SKINNY=0 sends the M * N <= 16 contractions to the tiled kernels (A/B timing)
bool skinny_disabled() {
  static const int v = [] {
    const char* e = getenv("TQ_GEMM_SKINNY");
    return (e && e[0] == '0') ? 1 : 0;
  }();
  return v != 0;
}

template <typename R>
__device__ __forceinline__ void mfma(R a, R b, typename std::conditional<sizeof(R) == 4, f32x16, f64x4>::type& c);
template <>
__device__ __forceinline__ void mfma<float>(float a, float b, f32x16& c) {
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mfma<double>(double a, double b, f64x4& c) {
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <typename R, bool CPLX, bool TA, bool TB>
__global__ void __launch_bounds__(kThreads) gemm_kernel(GemmArgs g) {
  using C_ = Cfg<R, CPLX>;
  using AccT = typename std::conditional<sizeof(R) == 4, f32x16, f64x4>::type;
  constexpr int EW = CPLX ? 2 : 1;                 // R values per element
  constexpr int VE = 16 / (EW * (int)sizeof(R));   // elements per 16-byte vector
  constexpr int BM = C_::BM, BN = C_::BN, BK = C_::BK;
  constexpr int LM = BM + C_::PAD, LN = BN + C_::PAD;  // LDS row strides
  constexpr int NVA = BM * BK / (VE * kThreads);
  constexpr int NVB = BK * BN / (VE * kThreads);
  constexpr int NPL = CPLX ? 2 : 1;

  __shared__ __attribute__((aligned(16))) R sA[NPL][BK][LM];
  __shared__ __attribute__((aligned(16))) R sB[NPL][BK][LN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  // ---- tile coordinates (XCD-aware: consecutive tiles along N of one M panel share an XCD)
  const int ntiles = g.mt * g.nt;
  int bid = blockIdx.x;
  {
    // bijective remap so that blocks b, b+8, b+16... (one XCD) get consecutive tiles
    const int q = ntiles / 8, r = ntiles % 8;
    const int xcd = bid % 8, idx = bid / 8;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    if (ntiles >= 8) bid = base + idx;
  }
  const int tm = bid / g.nt, tn = bid % g.nt;
  const int zb = blockIdx.z;
  const int split = zb % g.splits;
  const int64_t b = zb / g.splits;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = split * g.kchunk;
  const int64_t kend = min(g.K, kbeg + g.kchunk);

  const R* A = reinterpret_cast<const R*>(g.A) + b * g.sA * EW;
  const R* B = reinterpret_cast<const R*>(g.B) + b * g.sB * EW;

  AccT acc_re[C_::TI][C_::TJ];
  AccT acc_im[C_::TI][C_::TJ];
#pragma unroll
  for (int i = 0; i < C_::TI; ++i)
#pragma unroll
    for (int j = 0; j < C_::TJ; ++j) {
#pragma unroll
      for (int r = 0; r < C_::NACC; ++r) { acc_re[i][j][r] = 0; acc_im[i][j][r] = 0; }
    }

  R ra[NVA][VE * EW];
  R rb[NVB][VE * EW];

  // element (row, col) of a row-major matrix with leading dim ld, guarded
  auto load_vec = [&](const R* X, int64_t ld, int64_t row, int64_t col, int64_t rows,
                      int64_t cols, bool vec_ok, R* out) {
    // VE elements along `col`
    if (vec_ok && row < rows && col + VE <= cols) {
      const float4 v = *reinterpret_cast<const float4*>(X + (row * ld + col) * EW);
      const R* pv = reinterpret_cast<const R*>(&v);
#pragma unroll
      for (int e = 0; e < VE * EW; ++e) out[e] = pv[e];
    } else {
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        const bool in = row < rows && col + e < cols;
#pragma unroll
        for (int c = 0; c < EW; ++c) out[e * EW + c] = in ? X[(row * ld + col + e) * EW + c] : R(0);
      }
    }
  };

  auto global_load = [&](int64_t k0) {
#pragma unroll
    for (int s = 0; s < NVA; ++s) {
      const int q = tid + s * kThreads;
      if constexpr (!TA) {  // A is M x K, K contiguous: vectors along k
        const int m = q % BM, kv = q / BM;
        load_vec(A, g.lda, m0 + m, k0 + kv * VE, g.M, kend, g.vecA, ra[s]);
      } else {              // A is K x M, M contiguous: vectors along m
        const int mv = q % (BM / VE), k = q / (BM / VE);
        load_vec(A, g.lda, k0 + k, m0 + mv * VE, kend, g.M, g.vecA, ra[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < NVB; ++s) {
      const int q = tid + s * kThreads;
      if constexpr (!TB) {  // B is K x N, N contiguous
        const int nv = q % (BN / VE), k = q / (BN / VE);
        load_vec(B, g.ldb, k0 + k, n0 + nv * VE, kend, g.N, g.vecB, rb[s]);
      } else {              // B is N x K, K contiguous
        const int n = q % BN, kv = q / BN;
        load_vec(B, g.ldb, n0 + n, k0 + kv * VE, g.N, kend, g.vecB, rb[s]);
      }
    }
  };

  auto lds_store = [&]() {
#pragma unroll
    for (int s = 0; s < NVA; ++s) {
      const int q = tid + s * kThreads;
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        int m, k;
        if constexpr (!TA) { m = q % BM; k = (q / BM) * VE + e; }
        else { m = (q % (BM / VE)) * VE + e; k = q / (BM / VE); }
        sA[0][k][m] = ra[s][e * EW];
        if constexpr (CPLX) sA[1][k][m] = ra[s][e * EW + 1];
      }
    }
#pragma unroll
    for (int s = 0; s < NVB; ++s) {
      const int q = tid + s * kThreads;
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        int n, k;
        if constexpr (!TB) { n = (q % (BN / VE)) * VE + e; k = q / (BN / VE); }
        else { n = q % BN; k = (q / BN) * VE + e; }
        sB[0][k][n] = rb[s][e * EW];
        if constexpr (CPLX) sB[1][k][n] = rb[s][e * EW + 1];
      }
    }
  };

  // fragment lane maps (cdna_hip_programming.md §3):
  //   f32 32x32x2 : A[i = l&31][k = l>>5], B[k = l>>5][j = l&31]
  //   f64 16x16x4 : A[i = l&15][k = l>>4], B[k = l>>4][j = l&15]
  const int fr = lane % C_::MT;
  const int fk = lane / C_::MT;

  auto compute_tile = [&]() {
#pragma unroll
    for (int kk = 0; kk < BK; kk += C_::KT) {
      R ar[C_::TI], ai[C_::TI], br[C_::TJ], bi[C_::TJ];
#pragma unroll
      for (int i = 0; i < C_::TI; ++i) {
        const int m = wr * C_::WM + i * C_::MT + fr;
        ar[i] = sA[0][kk + fk][m];
        if constexpr (CPLX) ai[i] = sA[1][kk + fk][m];
      }
#pragma unroll
      for (int j = 0; j < C_::TJ; ++j) {
        const int n = wc * C_::WN + j * C_::MT + fr;
        br[j] = sB[0][kk + fk][n];
        if constexpr (CPLX) bi[j] = sB[1][kk + fk][n];
      }
#pragma unroll
      for (int i = 0; i < C_::TI; ++i)
#pragma unroll
        for (int j = 0; j < C_::TJ; ++j) {
          mfma<R>(ar[i], br[j], acc_re[i][j]);
          if constexpr (CPLX) {
            mfma<R>(-ai[i], bi[j], acc_re[i][j]);
            mfma<R>(ar[i], bi[j], acc_im[i][j]);
            mfma<R>(ai[i], br[j], acc_im[i][j]);
          }
        }
    }
  };

  if (kbeg < kend) {
    global_load(kbeg);
    for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
      lds_store();
      __syncthreads();
      if (k0 + BK < kend) global_load(k0 + BK);  // in flight during the MFMAs below
      compute_tile();
      __syncthreads();
    }
  }

  // ---- epilogue
  R* Cout;
  int64_t ldo;
  const bool partial = g.splits > 1;
  if (partial) {
    Cout = reinterpret_cast<R*>(g.W) + ((int64_t)split * g.batch + b) * g.M * g.N * EW;
    ldo = g.N;
  } else {
    Cout = reinterpret_cast<R*>(g.C) + b * g.sC * EW;
    ldo = g.ldc;
  }
  const R beta = partial ? R(0) : (R)g.beta;
#pragma unroll
  for (int i = 0; i < C_::TI; ++i)
#pragma unroll
    for (int j = 0; j < C_::TJ; ++j)
#pragma unroll
      for (int r = 0; r < C_::NACC; ++r) {
        int row, col;
        if constexpr (sizeof(R) == 4) {
          row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          col = lane & 31;
        } else {
          row = (lane >> 4) + 4 * r;
          col = lane & 15;
        }
        const int64_t gm = m0 + wr * C_::WM + i * C_::MT + row;
        const int64_t gn = n0 + wc * C_::WN + j * C_::MT + col;
        if (gm < g.M && gn < g.N) {
          R* p = Cout + (gm * ldo + gn) * EW;
          R vr = acc_re[i][j][r];
          if constexpr (CPLX) {
            R vi = acc_im[i][j][r];
            if (beta != R(0)) { vr += beta * p[0]; vi += beta * p[1]; }
            p[0] = vr;
            p[1] = vi;
          } else {
            if (beta != R(0)) vr += beta * p[0];
            p[0] = vr;
          }
        }
      }
}


// ---------------------------------------------------------------------------------------------
// Fast path: complex64 with both operands K-outer (A stored K x M, B stored K x N, M / N
// contiguous) — the layout the plan compiler gives the boundary GEMM of a sliced cut (the
// dominant contraction of the sliced amplitude workloads).
//
//  * 512 threads = 8 waves (2 per SIMD), block tile 256 (M) x 128 (N), wave tile 64 x 64 =
//    2 x 2 v_mfma_f32_32x32x2_f32 tiles x (re, im) accumulators = 128 AGPRs.
//  * operands reach LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR staging): one
//    wave-instruction moves 1 KiB = 128 complex of one k-row, so the LDS image is the global
//    row image [k][m] / [k][n] with (re, im) interleaved; a fragment is one ds_read_b64 that
//    yields (re, im) of one element — lanes 0-31 read 256 contiguous bytes of row k, lanes 32-63
//    of row k+1: conflict-free.
//  * 3-stage LDS ring (3 x 48 KiB), two K-tiles in flight: per K-tile one counted
//    `s_waitcnt vmcnt(6)` (6 DMAs per wave per tile) and ONE raw s_barrier, never vmcnt(0) in the
//    steady state (cdna_hip_programming.md §5 "Pipelining across barriers").
//  * split-K over the grid (slab reduce kernel below); a bijective XCD remap puts all tiles of one
//    K-split on one XCD so each XCD's L2 streams its K range of A and B from HBM exactly once.
namespace fastc64 {
// block configuration: WMW x WNW waves, each owning TI x TJ tiles of 32 x 32 outputs; K-tiles
// of BK rows in an NS-stage LDS ring (NS - 1 tiles in flight)
template <int WMW_, int WNW_, int TI_, int TJ_, int BK_ = 16, int NS_ = 3> struct Tile {
  static constexpr int WMW = WMW_, WNW = WNW_, TI = TI_, TJ = TJ_, BK = BK_, NS = NS_;
  static constexpr int NW = WMW * WNW, NT = 64 * NW;
  static constexpr int WM = 32 * TI, WN = 32 * TJ;            // wave tile
  static constexpr int BM = WMW * WM, BN = WNW * WN;           // block tile
  static constexpr int A_FLOATS = BK * BM * 2, B_FLOATS = BK * BN * 2, STAGE = A_FLOATS + B_FLOATS;
  static constexpr int A_ROW_PIECES = BM / 128;               // 1-KiB pieces per k-row of A
  static constexpr int A_PIECES_PER_WAVE = BK * A_ROW_PIECES / NW;
  static constexpr int B_ROW_PIECES = BN / 128;
  static constexpr int B_PIECES_PER_WAVE = BK * B_ROW_PIECES / NW;
  static constexpr int NDMA = A_PIECES_PER_WAVE + B_PIECES_PER_WAVE;  // DMAs per wave per tile
  static_assert(BK * A_ROW_PIECES % NW == 0 && BK * B_ROW_PIECES % NW == 0, "piece split");
};
// 4-multiplication complex product: 8 waves (2 per SIMD) of 64 x 64, block 256 x 128
using Tile4M = Tile<4, 2, 2, 2>;
// Gauss 3M (3 accumulator sets): 8 waves of 64 x 32 keep 96 accumulators (2 waves per SIMD),
// block 128 x 128
using Tile3M = Tile<2, 4, 2, 1>;
}

struct FastArgs {
  const float* A;  // K x M complex (lda complex elements between k-rows)
  const float* B;  // K x N complex
  float* C;        // output (ldc) or split-K slabs
  float* W;
  int64_t lda, ldb, ldc, sA, sB, sC, M, N;
  int64_t kchunk;  // K per split (multiple of BK)
  int mt, nt, splits, batch;
  float beta;
  const uint32_t* amax_a;  // f16 split kernel: max |x| bits of A / B (producer or absmax pre-pass)
  const uint32_t* amax_b;
  const int32_t* sc_a;     // pre-split operands (SplitPre): the producers' scales, window flag
  const int32_t* sc_b;
  uint32_t* bad;
  int amax_bs_a, amax_bs_b;  // max-word stride between batch entries (0: one word per operand)
  int prio;                  // f16 split kernel: s_setprio 1 for the second half of the waves
};

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// G3M: Gauss's 3-multiplication complex product (P1 = Ar Br, P2 = Ai Bi, P3 = (Ar+Ai)(Br+Bi);
// Cr = P1 - P2, Ci = P3 - P1 - P2): 3 real MFMAs per complex k-step instead of 4, all in f32.
template <bool G3M, typename TL>
__global__ void __launch_bounds__(TL::NT, 1) gemm_c64_kouter_kernel(FastArgs g) {
  using namespace fastc64;
  constexpr int BM = TL::BM, BN = TL::BN, WMW = TL::WMW, TI = TL::TI, TJ = TL::TJ;
  constexpr int STAGE = TL::STAGE, A_FLOATS = TL::A_FLOATS, BK = TL::BK, NSTAGE = TL::NS;
  constexpr int A_PIECES_PER_WAVE = TL::A_PIECES_PER_WAVE, B_PIECES_PER_WAVE = TL::B_PIECES_PER_WAVE;
  constexpr int NACC = G3M ? 3 : 2;
  __shared__ __attribute__((aligned(16))) float lds[NSTAGE * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WMW, wn = wid / WMW;

  // bijective XCD remap of the linear block id, then (batch, split, tile) with tile fastest
  const int nblk = gridDim.x;
  int L = blockIdx.x;
  {
    const int q = nblk / 8, r = nblk % 8, xcd = L % 8, idx = L / 8;
    if (nblk >= 8) L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int ntile = g.mt * g.nt;
  const int tile = L % ntile;
  const int split = (L / ntile) % g.splits;
  const int b = L / (ntile * g.splits);
  const int tm = tile / g.nt, tn = tile % g.nt;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * g.kchunk;
  const int nkt = (int)(g.kchunk / BK);

  const float* A = g.A + ((int64_t)b * g.sA + kbeg * g.lda + m0) * 2;
  const float* B = g.B + ((int64_t)b * g.sB + kbeg * g.ldb + n0) * 2;

  // this wave's DMA pieces (1 KiB = 128 complex of one k-row each).  The DMA is issued from
  // inline asm: hipcc would otherwise treat every in-flight LDS-DMA as a possible alias of the
  // next ds_read and drain it with vmcnt(0) (cdna_hip_programming.md §5 trap 4(a)); the counted
  // waits below are the only ordering, placed by hand.
  const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)lds;
  auto glds16 = [&](const float* gsrc, unsigned lds_off_floats) {
    unsigned keep;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_base + lds_off_floats * 4u);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto issue = [&](int t, int stage) {
    const unsigned sbase = stage * STAGE;
#pragma unroll
    for (int q = 0; q < A_PIECES_PER_WAVE; ++q) {
      const int p = wid * A_PIECES_PER_WAVE + q;
      const int kr = p / TL::A_ROW_PIECES, mp = p % TL::A_ROW_PIECES;
      glds16(A + (((int64_t)t * BK + kr) * g.lda + mp * 128 + lane * 2) * 2, sbase + p * 256);
    }
#pragma unroll
    for (int q = 0; q < B_PIECES_PER_WAVE; ++q) {
      const int p = wid * B_PIECES_PER_WAVE + q;
      const int kr = p / TL::B_ROW_PIECES, np = p % TL::B_ROW_PIECES;
      glds16(B + (((int64_t)t * BK + kr) * g.ldb + np * 128 + lane * 2) * 2, sbase + A_FLOATS + p * 256);
    }
  };

  f32x16 acc[NACC][TI][TJ];
#pragma unroll
  for (int x = 0; x < NACC; ++x)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][i][j][r] = 0.f;

  const int fr = lane & 31, fk = lane >> 5;
  // float offsets of this lane's fragments inside a stage (k-row kk + fk)
  const int a_off = (fk * BM + wm * TL::WM + fr) * 2;
  const int b_off = A_FLOATS + (fk * BN + wn * TL::WN + fr) * 2;

  for (int p = 0; p < NSTAGE - 1 && p < nkt; ++p) issue(p, p);
  for (int t = 0; t < nkt; ++t) {
    // tile t must have landed; tiles t+1 .. t+NSTAGE-2 may stay in flight (counted waits only)
    if (NSTAGE > 2 && t + 1 < nkt) vm_wait<TL::NDMA * (NSTAGE > 2 ? NSTAGE - 2 : 0)>();
    else vm_wait<0>();
    asm volatile("s_barrier" ::: "memory");
    if (t + NSTAGE - 1 < nkt) issue(t + NSTAGE - 1, (t + NSTAGE - 1) % NSTAGE);
    const float* s = lds + (t % NSTAGE) * STAGE;
    // fragments of k-step kk+2 are read while the MFMAs of k-step kk run
    float2 a[TI], bb[TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i) a[i] = *reinterpret_cast<const float2*>(s + a_off + (i * 32) * 2);
#pragma unroll
    for (int j = 0; j < TJ; ++j) bb[j] = *reinterpret_cast<const float2*>(s + b_off + (j * 32) * 2);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float2 na[TI], nb[TJ];
      if (kk + 2 < BK) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
          na[i] = *reinterpret_cast<const float2*>(s + a_off + ((kk + 2) * BM + i * 32) * 2);
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          nb[j] = *reinterpret_cast<const float2*>(s + b_off + ((kk + 2) * BN + j * 32) * 2);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the k+2 reads ahead of this k-step's MFMAs
      if constexpr (G3M) {
        float sa[TI], sb[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) sa[i] = a[i].x + a[i].y;
#pragma unroll
        for (int j = 0; j < TJ; ++j) sb[j] = bb[j].x + bb[j].y;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            acc[0][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, bb[j].x, acc[0][i][j], 0, 0, 0);
            acc[1][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, bb[j].y, acc[1][i][j], 0, 0, 0);
            acc[NACC - 1][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(sa[i], sb[j], acc[NACC - 1][i][j], 0, 0, 0);
          }
      } else {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            acc[0][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, bb[j].x, acc[0][i][j], 0, 0, 0);
            acc[1][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, bb[j].y, acc[1][i][j], 0, 0, 0);
          }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            acc[0][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(-a[i].y, bb[j].y, acc[0][i][j], 0, 0, 0);
            acc[1][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, bb[j].x, acc[1][i][j], 0, 0, 0);
          }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kk + 2 < BK) {
#pragma unroll
        for (int i = 0; i < TI; ++i) a[i] = na[i];
#pragma unroll
        for (int j = 0; j < TJ; ++j) bb[j] = nb[j];
      }
    }
  }

  // epilogue: 32x32 f32 MFMA accumulator r of lane -> row (r&3) + 8(r>>2) + 4(lane>>5), col lane&31
  const bool partial = g.splits > 1;
  float* Cout = partial ? g.W + (((int64_t)split * g.batch + b) * g.M * g.N) * 2 : g.C + (int64_t)b * g.sC * 2;
  const int64_t ldo = partial ? g.N : g.ldc;
  const float beta = partial ? 0.f : g.beta;
  auto store = [&](auto with_beta) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t gm = m0 + wm * TL::WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int64_t gn = n0 + wn * TL::WN + j * 32 + (lane & 31);
          float2* p = reinterpret_cast<float2*>(Cout + (gm * ldo + gn) * 2);
          float2 v;
          if constexpr (G3M) {
            const float p1 = acc[0][i][j][r], p2 = acc[1][i][j][r];
            v = make_float2(p1 - p2, acc[NACC - 1][i][j][r] - p1 - p2);
          } else {
            v = make_float2(acc[0][i][j][r], acc[1][i][j][r]);
          }
          if constexpr (decltype(with_beta)::value) {
            const float2 o = *p;
            v.x += beta * o.x;
            v.y += beta * o.y;
          }
          *p = v;
        }
  };
  if (beta != 0.f) store(std::true_type{});
  else store(std::false_type{});
}

// ---------------------------------------------------------------------------------------------
// complex64 on the 16-bit matrix cores with f32 accuracy (the K-outer complex64 fast path;
// TQ_GEMM_BF16=0 selects the f32-MFMA kernel above).  Every f32 operand value is split into
// 16-bit terms and each real product a*b becomes a few term products on the MFMA, accumulated
// in f32; the complex product is the 4-multiplication form (Cr += Ar Br + (-Ai) Bi,
// Ci += Ar Bi + Ai Br; -Ai by flipping the fragment's sign bits).  Two splits (SplitF16 /
// SplitBF16 below):
//  * f16 (default): x * 2^sc (sc from the operand's max |x|, so max |x| 2^sc is in [2^14, 2^15))
//    = h + l, two f16 terms good to 2^-24 relative; 3 term products (hh, hl, lh) = 12
//    v_mfma_f32_32x32x16_f16 per 32 x 32 x 16 complex tile-step.  The max comes from the operand's
//    producer (plan: the sweep op that stores it) or from a pre-pass (absmax_kouter_kernel).
//  * bf16 (TQ_GEMM_F16=0): x = h + m + l exactly by truncation, 6 term products = 24 MFMAs.
// Both run at the same cycles per MFMA, so the f16 split halves the MFMA work.
//
// Data path per K-step of 16 (block 128 x 128, one barrier per step): half of the threads stage
// A, half B; a thread owns 2 rows x 4 (8) consecutive k and loads them as 16-B vectors (one
// complex pair per k) with an SGPR base + 32-bit lane offset, NSET - 1 steps ahead, into
// register sets; the split of step t + 1 goes into the other half of a double-buffered LDS image
// of term planes (2 x NTERM planes of [row][16 k] 16-bit values, 32-B rows, swizzled: swz) while
// the MFMAs of step t run from fragments read at the start of the step (one ds_read_b128 each, in
// the order the MFMA pairs first use them).  The f16 kernel tells the scheduler to interleave the
// split with the MFMAs (sched_group_barrier).
//
// Measured at the C4 shape (1024 x 1024 x 65536, split-K 4; r02): f16 1.40-1.43 ms, MFMA busy
// 62 % at the 1.77 GHz the chip holds (PMC); bf16 2.49 ms.  Steps that mattered: 16-B staging
// loads instead of 8-B (the per-CU L2 request rate bounded the 8-B version: a loads-only variant
// took as long as the whole kernel), the producer-side operand max instead of a 1-GiB pre-pass
// (0.23 ms per launch).  Within 2-3 %: 3 vs 4 staging sets, one wave per SIMD with 64 x 64 wave
// tiles (TileH4), the interleave, fragment-read order, a conflict-free store swizzle.  With the
// MFMAs removed the kernel takes 0.66 ms at 2.3 GHz; with the loads removed 1.30 ms: the split
// and the MFMAs overlap only partly.
namespace xbf {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
template <int WMW_, int WNW_, int TI_, int TJ_, int NTERM_, int NSET_, bool ILV_, bool G3_ = false,
          int SLOTS_ = 2, bool ORD_ = false, bool POUT_ = false, bool STG_ = false, bool PIPE_ = false>
struct Tile {
  // PIPE (with STG): the step's barrier sits before its last product group, whose MFMAs then run
  // under the reads of the NEXT step's first group: a step starts on fragments already in
  // registers instead of waiting for its first LDS reads
  static constexpr bool PIPE = PIPE_;
  // STG (with POUT): a K-step's fragments are read one product group (re / im / re+im planes) at
  // a time, group h+1's under group h's MFMAs: two groups' fragments live instead of three
  static constexpr bool STG = STG_;
  // POUT (Gauss 3M): MFMAs ordered product-major -- the three term products of one real product
  // back to back on one accumulator, so consecutive MFMAs share an operand (A-l B-h, A-h B-h,
  // A-h B-l) instead of changing both
  static constexpr bool POUT = POUT_;
  // ORD (f16, 3 term pairs): pairs in the order (l, h), (h, h), (h, l); the B-l fragments are read
  // after the first third of the MFMAs, into the registers of the then-dead A-l fragments
  static constexpr bool ORD = ORD_;
  // LDS slots of a K-step each: 2 = double buffer, one barrier per K-step; 4 = a ring in which a
  // step's split lands two steps ahead, one barrier per TWO K-steps
  static constexpr int SLOTS = SLOTS_;
  // ILV: the scheduler is told to interleave the split (VALU, LDS stores) with the MFMAs
  static constexpr bool ILV = ILV_;
  // G3: Gauss's 3-multiplication product (planes re, im, re + im per term; 3 accumulator sets)
  static constexpr bool G3 = G3_;
  static constexpr int NGRP = G3_ ? 3 : 2;
  static constexpr int WMW = WMW_, WNW = WNW_, TI = TI_, TJ = TJ_, NTERM = NTERM_;
  // staging register sets: a K-step's loads go out NSET - 1 steps before its split
  static constexpr int NSET = NSET_;
  static constexpr int NW = WMW * WNW, NT = 64 * NW;
  static constexpr int WM = 32 * TI, WN = 32 * TJ, BM = WMW * WM, BN = WNW * WN, BK = 16;
  static constexpr int SUBA = BM * 32, SUBB = BN * 32;            // bytes per term plane
  static constexpr int BUF = NGRP * NTERM * (SUBA + SUBB);        // (re, im[, re+im]) x terms, A, B
  // split task per thread: 2 rows x KPT consecutive k of one operand
  static constexpr int KPT = 16 * BM / NT;
  static_assert(BM == BN && (KPT == 4 || KPT == 8), "task split");
  static_assert(SLOTS * BUF <= 160 * 1024, "LDS");
};
// 8 waves (two per SIMD) of 64 x 32, block 128 x 128, 64 accumulators per wave; 4-k split tasks
// (ds_write_b64).  bf16: 3 terms, 2 x 48 KiB LDS; f16: 2 terms, 2 x 32 KiB.
using TileX = Tile<2, 4, 2, 1, 3, 2, false>;   // bf16: 4 sets spill at 3 terms
// f16 default: 8 waves (two per SIMD) of 64 x 32, block 128 x 128, 4 staging sets, interleaved
using TileH = Tile<2, 4, 2, 1, 2, 4, true>;
// f16 alternative (TQ_GEMM_F16_VAR=1): 4 waves (one per SIMD, 512 registers) of 64 x 64 — twice
// the MFMAs per fragment read; measured within 2 % of the default
using TileH4 = Tile<2, 2, 2, 2, 2, 4, true>;
// f16, Gauss 3M (TQ_GEMM_F16_VAR=2): P1 = Ar Br, P2 = Ai Bi, P3 = (Ar + Ai)(Br + Bi), 9 MFMAs per
// complex tile-step instead of 12; 4 waves of 64 x 64 (3 x 64 accumulators), 3 staging sets
using TileH4G = Tile<2, 2, 2, 2, 2, 3, true, true>;
// f16, Gauss 3M on the default tile (TQ_GEMM_F16_VAR=5): 8 waves of 64 x 32, 3 x 32 accumulators,
// 2 staging sets (power: 25 % fewer MFMAs, 50 % more LDS term planes)
using TileH8G = Tile<2, 4, 2, 1, 2, 2, true, true>;
// the same with 3 staging sets (loads two K-steps ahead) and the ordered term pairs (var 6)
using TileH8G3 = Tile<2, 4, 2, 1, 2, 3, true, true, 2, true>;
// variant 5 with product-major MFMA order (var 7)
using TileH8GP = Tile<2, 4, 2, 1, 2, 2, true, true, 2, false, true>;
// product-major order, fragments read per product group, 3 staging sets (var 8)
using TileH8GS = Tile<2, 4, 2, 1, 2, 3, true, true, 2, false, true, true>;
// var 8 with the barrier before the last product group, next step's first group read early (var 9)
using TileH8GQ = Tile<2, 4, 2, 1, 2, 3, true, true, 2, false, true, true, true>;
// f16, one barrier per two K-steps (TQ_GEMM_F16_VAR=3): the default tile on a 4-slot LDS ring
using TileH2 = Tile<2, 4, 2, 1, 2, 4, true, false, 4>;

__device__ __forceinline__ uint32_t hi16(float x) { return __float_as_uint(x) & 0xffff0000u; }
// pack the bf16 held in the high halves of two dwords: lo <- a, hi <- b
__device__ __forceinline__ uint32_t pk(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

// bf16, three terms by truncation: h = x with the low 16 bits cleared, r = x - h (exact),
// m = r truncated the same way, l = r - m (exact, <= 8 significant bits): x == h + m + l exactly.
// Term pairs kept (A term, B term), smallest first: mh hm lh hl hh... the six down to 2^-16.
struct SplitBF16 {
  static constexpr int NTERM = 3, NPAIR = 6;
  static constexpr bool SCALED = false, PRE = false;
  static constexpr int pa(int q) { return q == 0 ? 1 : q == 2 ? 2 : q == 4 ? 1 : 0; }  // 1 0 2 0 1 0
  static constexpr int pb(int q) { return q == 0 ? 1 : q == 1 ? 2 : q == 3 ? 1 : 0; }  // 1 2 0 1 0 0
  template <int N>
  static __device__ __forceinline__ void split(const float (&v)[N], int, uint32_t (&t)[3][N / 2]) {
    uint32_t hb[N], mb[N], lb[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      hb[j] = hi16(v[j]);
      const float r = v[j] - __uint_as_float(hb[j]);
      mb[j] = hi16(r);
      lb[j] = __float_as_uint(r - __uint_as_float(mb[j]));
    }
#pragma unroll
    for (int j = 0; j < N / 2; ++j) {
      t[0][j] = pk(hb[2 * j], hb[2 * j + 1]);
      t[1][j] = pk(mb[2 * j], mb[2 * j + 1]);
      t[2][j] = pk(lb[2 * j], lb[2 * j + 1]);
    }
  }
  static __device__ __forceinline__ f32x16 mfma(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};

// f16, two terms of a power-of-two-scaled value: xs = x * 2^sc (sc from the operand's max |x|,
// so max |xs| is in [2^14, 2^15)), h = f16(xs) (round to nearest), r = xs - h (exact in f32,
// |r| <= 2^-12 |xs|), l = f16(r): xs == h + l within 2^-24 |xs| (l's rounding) — the f32 rounding
// level — for |xs| >= 2^-2 (l normal); below that l's absolute error is <= 2^-25, i.e. <= 2^-40 of
// the operand's max.  Pairs kept: lh, hl, hh; the dropped ll is <= 2^-24 relative.
struct SplitF16 {
  static constexpr int NTERM = 2, NPAIR = 3;
  static constexpr bool SCALED = true, PRE = false;
  static constexpr int pa(int q) { return q == 0 ? 1 : 0; }  // 1 0 0
  static constexpr int pb(int q) { return q == 1 ? 1 : 0; }  // 0 1 0
  // per pair of values: 2 v_ldexp_f32, v_cvt_pk_f16_f32 (h), 2 v_fma_mix_f32 (r = x - h, reading
  // the packed f16 halves directly), v_cvt_pk_f16_f32 (l): 3 VALU per value
  template <int N>
  static __device__ __forceinline__ void split(const float (&v)[N], int sc, uint32_t (&t)[2][N / 2]) {
#ifdef TQ_GEMM_DIAG_HALFSPLIT
    // development diagnostic (wrong results): h as in the split, l = h with flipped low bits (4
    // VALU per pair instead of 6) -- the split's VALU cost at the same data flow.  Measured r03:
    // 5.17 -> 5.08 ms per C4 launch (-1.7 %), clock +1 %: all of the split's VALU is worth ~5 %
    // (raw f32 bits as the terms instead, no VALU, ran 9.7 ms: NaN / Inf f16 patterns)
#pragma unroll
    for (int j = 0; j < N / 2; ++j) {
      const float x0 = ldexpf(v[2 * j], sc), x1 = ldexpf(v[2 * j + 1], sc);
      const f16x2 hv = {(_Float16)x0, (_Float16)x1};
      const uint32_t h = __builtin_bit_cast(uint32_t, hv);
      t[0][j] = h;
      t[1][j] = h ^ 0x00030003u;
    }
    return;
#endif
#pragma unroll
    for (int j = 0; j < N / 2; ++j) {
      const float x0 = ldexpf(v[2 * j], sc), x1 = ldexpf(v[2 * j + 1], sc);
      const f16x2 hv = {(_Float16)x0, (_Float16)x1};
      const uint32_t h = __builtin_bit_cast(uint32_t, hv);
      float r0, r1;
      asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r0) : "v"(x0), "v"(h));
      asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r1) : "v"(x1), "v"(h));
      const f16x2 lv = {(_Float16)r0, (_Float16)r1};
      t[0][j] = h;
      t[1][j] = __builtin_bit_cast(uint32_t, lv);
    }
  }
  static __device__ __forceinline__ f32x16 mfma(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

// f16 terms split by the operand's producer (S2Op::split_sc): every complex64 element holds
// (h_re, h_im | l_re, l_im) as four f16 of the value scaled by 2^sc; the GEMM only regroups the
// halves into its term planes (v_perm_b32, 2 per 4 k of a row and plane)
struct SplitPre : SplitF16 {
  static constexpr bool PRE = true;
};

// scheduling pattern (sched_group_barrier, one scheduling region): MFMA i, then up to V VALU,
// and one LDS store after every E-th MFMA
template <int I, int NM, int V, int E> struct Interleave {
  static __device__ __forceinline__ void run() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
    if constexpr (I % E == E - 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    Interleave<I + 1, NM, V, E>::run();
  }
};
template <int NM, int V, int E> struct Interleave<NM, NM, V, E> {
  static __device__ __forceinline__ void run() {}
};

// exponent sc with max|x| * 2^sc in [2^14, 2^15) from the bits of max|x| (0 -> 0; inf/nan -> 0)
__device__ __forceinline__ int scale_exp(uint32_t bits) {
  const int E = (int)((bits >> 23) & 0xff);
  if (bits == 0 || E == 255) return 0;
  const int e = E ? E - 127 : (31 - __clz((int)(bits & 0x7fffff))) - 149;
  return 14 - e;
}

// pre-split operands: floor(log2 max) + sc in [0, 14] (max == 0: every term is zero, valid)
__device__ __forceinline__ bool presplit_in_window(uint32_t bits, int sc) {
  const int E = (int)((bits >> 23) & 0xff);
  if (bits == 0) return true;
  if (E == 255) return false;
  const int e = E ? E - 127 : (31 - __clz((int)(bits & 0x7fffff))) - 149;
  return e + sc >= 0 && e + sc <= 14;
}

// scale of the next slice's operand from this slice's max: max * 2^sc near 2^7 (7 binades of
// headroom either way); no max yet: sc = 10 (|x| ~ 1e-3 .. 16)
__global__ void presplit_prep_kernel(uint32_t* amax, int32_t* sc, int n, int bias) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t bits = amax[i];
    const int E = (int)((bits >> 23) & 0xff);
    int s = 10;
    if (bits != 0 && E != 255) {
      const int e = E ? E - 127 : (31 - __clz((int)(bits & 0x7fffff))) - 149;
      s = 7 - e;
    }
    sc[i] = s + bias;
    amax[i] = 0;
  }
}

template <int N>
__device__ __forceinline__ void st_lds(char* p, const uint32_t (&w)[N / 2]) {
  if constexpr (N == 8) *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  else *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
}

// byte offset of (row, k-half) inside a term plane: rows of 32 B; on every other group of 8 rows
// the two 16-B k-halves are swapped, and rows 2i / 2i+1 trade places where row bit 2 is set.
// ds_read_b128 (bank = byte/4 mod 64, lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, +32):
// a group's 16 rows land on 16 distinct (row mod 8, half) slots; ds_write_b64 (bank = byte/4
// mod 32, 16 contiguous lanes): the staging stores of a group — rows 2r or 2r+1, r = 4q..4q+3,
// x four 8-B k-groups — land on 4 distinct 32-B blocks mod 128 B (PMC SQ_LDS_BANK_CONFLICT 0;
// without the row swap, rows 2r and 2r+4 were 2-way on every store)
__device__ __forceinline__ int swz(int row, int kh) {
  return (row ^ ((row >> 2) & 1)) * 32 + ((kh ^ ((row >> 3) & 1)) << 4);
}
// sign flip of 8 packed 16-bit floats (bf16 and f16 keep the sign in bit 15)
__device__ __forceinline__ uint4 neg8(uint4 v) {
  return make_uint4(v.x ^ 0x80008000u, v.y ^ 0x80008000u, v.z ^ 0x80008000u, v.w ^ 0x80008000u);
}

// max |re|, |im| over the K x M (A) and K x N (B) operands of batch entry blockIdx.z, as float
// bits atomically max-ed into amax[b] (A) / amax[batch + b] (B) (zeroed before).  One wave per
// k-row, 64 lanes x 16 B per load, four loads in flight; rows are M / 2 float4 (M % 128 == 0).
__global__ void __launch_bounds__(256) absmax_kouter_kernel(const float4* A, int64_t lda4, int64_t sA4,
                                                            const float4* B, int64_t ldb4, int64_t sB4,
                                                            int64_t K, int64_t w4A, int64_t w4B,
                                                            int64_t batch, uint32_t* amax) {
  const int op = blockIdx.y;
  const int64_t b = blockIdx.z;
  const float4* base = op ? B : A;
  const int64_t ld = op ? ldb4 : lda4, s = op ? sB4 : sA4, w = op ? w4B : w4A;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  float m = 0.f;
  for (int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); k < K; k += nw) {
    const float4* p = base + b * s + k * ld + lane;
    for (int64_t c = 0; c < w; c += 256) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = (c + 64 * u < w) ? p[c + 64 * u] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float red[4];
  if (lane == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(amax + op * batch + b, __float_as_uint(m));
  }
}
}  // namespace xbf

TQ_KCLOCK_DEFINE(g_kclk_kouter)
template <typename TL, typename SP>
__global__ void __launch_bounds__(TL::NT, 1) gemm_c64_kouter_split_kernel(FastArgs g) {
  using namespace xbf;
  constexpr int BM = TL::BM, BN = TL::BN, BK = TL::BK, WMW = TL::WMW, TI = TL::TI, TJ = TL::TJ;
  constexpr int SUBA = TL::SUBA, SUBB = TL::SUBB, BUF = TL::BUF, NTM = SP::NTERM;
  constexpr bool G3 = TL::G3;
  constexpr int NGRP = TL::NGRP, NACC = G3 ? 3 : 2;
  static_assert(TL::NTERM == SP::NTERM, "tile / split terms");
  __shared__ __attribute__((aligned(16))) char lds[TL::SLOTS * BUF];
  TQ_KCLOCK_BEGIN()

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WMW, wn = wid / WMW;

  const int nblk = gridDim.x;
  int L = blockIdx.x;
  {
    const int q = nblk / 8, r = nblk % 8, xcd = L % 8, idx = L / 8;
    if (nblk >= 8) L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int ntile = g.mt * g.nt;
  const int tile = L % ntile;
  const int split = (L / ntile) % g.splits;
  const int b = L / (ntile * g.splits);
  const int tm = tile / g.nt, tn = tile % g.nt;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * g.kchunk;
  const int nkt = (int)(g.kchunk / BK);

  const float2* A = reinterpret_cast<const float2*>(g.A) + ((int64_t)b * g.sA + kbeg * g.lda + m0);
  const float2* B = reinterpret_cast<const float2*>(g.B) + ((int64_t)b * g.sB + kbeg * g.ldb + n0);
  // power-of-two operand scales (f16 terms): from the operands' max |x| (absmax_kouter_kernel)
  int sca = 0, scb = 0;
  if constexpr (SP::PRE) {
    // the producers scaled by sc_a / sc_b (predicted from the previous slice): valid while the
    // true max lands in [2^0, 2^15) -- no f16 overflow, rounding <= 2^-25 of the max; otherwise
    // this launch writes zeros and flags the slice for the split path
    sca = *g.sc_a;
    scb = *g.sc_b;
    const bool ok = presplit_in_window(*g.amax_a, sca) && presplit_in_window(*g.amax_b, scb);
    if (L == 0 && tid == 0) *g.bad = ok ? 0u : 1u;
    if (!ok) {
      const bool part = g.splits > 1;
      float* Co = part ? g.W + (((int64_t)split * g.batch + b) * g.M * g.N) * 2 : g.C + (int64_t)b * g.sC * 2;
      const int64_t ldz = part ? g.N : g.ldc;
      for (int e = tid; e < BM * BN; e += TL::NT) {
        const int64_t gm = m0 + e / BN, gn = n0 + e % BN;
        float2* p = reinterpret_cast<float2*>(Co + (gm * ldz + gn) * 2);
        *p = (part || g.beta == 0.f) ? make_float2(0.f, 0.f) : make_float2(p->x * g.beta, p->y * g.beta);
      }
      return;
    }
  } else if constexpr (SP::SCALED) {
    // every batch entry (slice lane) scaled by its own operand max
    sca = scale_exp(g.amax_a[(int64_t)b * g.amax_bs_a]);
    scb = scale_exp(g.amax_b[(int64_t)b * g.amax_bs_b]);
  }

  // staging registers, NSET sets (K-step mod NSET).  Threads 0 .. NT/2-1 stage A, the rest B
  // (wave-uniform); a thread owns rows 2r, 2r+1 (r = lane-group index) x KPT = 4 consecutive k
  // (k-group tkg = tid % 4): per K-step four 16-B loads (one k, both rows: a wave-instruction
  // covers 4 k-rows x 256 B) and, per row and term plane, one 8-B LDS store (a 16-lane group
  // writes rows 0, 2, 4, 6 (+8..) x 32 B: distinct banks).  Per-CU L2 -> L1 request concurrency,
  // not bandwidth, bounded the 8-B-per-lane version (512 B per wave-load): ~7.5 B/clk/CU with the
  // MFMAs removed.  A K-step's loads are issued NSET - 1 K-steps before its split.
  constexpr int KPT = TL::KPT, KG = 16 / KPT, NSET = TL::NSET;
  static_assert(BM == BN && (TL::NT / 2) * 2 * KPT == BM * 16, "two operands x BM/2 row pairs x KG k-groups");
  const int op = __builtin_amdgcn_readfirstlane(tid >= TL::NT / 2 ? 1 : 0);  // wave-uniform: SGPR
  const int ot = tid & (TL::NT / 2 - 1);
  const int trow = 2 * (ot / KG), tkg = ot % KG;
  float4 rv[NSET][KPT];
  // wave-uniform K-step base (SGPR pair) + per-lane 32-bit byte offsets fixed over the loop (no
  // per-step address VALU; launch: lda, ldb < 2^24 complex)
  const int64_t ld = op ? g.ldb : g.lda;
  const char* src = reinterpret_cast<const char*>(op ? B : A);
  uint32_t off[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) off[j] = (uint32_t)(((tkg * KPT + j) * ld + trow) * 8);
  const int64_t stepb = (int64_t)BK * ld * 8;
  auto load = [&](auto set, int t) {
    constexpr int S = decltype(set)::value;
    const char* p = src + t * stepb;
#pragma unroll
    for (int j = 0; j < KPT; ++j) rv[S][j] = *reinterpret_cast<const float4*>(p + off[j]);
  };
  // term planes: 0..NTM-1 = re terms (largest first), NTM..2 NTM-1 = im terms
  const int sc = op ? scb : sca;
  const int sub = op ? SUBB : SUBA;
  const int obase = op ? NGRP * NTM * SUBA : 0;
  const int toff0 = swz(trow, (tkg * KPT) >> 3) + ((tkg * KPT) & 7) * 2;
  const int toff1 = swz(trow + 1, (tkg * KPT) >> 3) + ((tkg * KPT) & 7) * 2;
  auto put = [&](const float (&re)[KPT], const float (&im)[KPT], char* base, int toff) {
    if constexpr (SP::PRE) {
      // re[j] = bits of (h_re, h_im), im[j] = bits of (l_re, l_im) of k = j: planes h_re, l_re,
      // h_im, l_im from the low / high halves
      uint32_t q[4][KPT / 2];
#pragma unroll
      for (int j = 0; j < KPT / 2; ++j) {
        const uint32_t a0 = __float_as_uint(re[2 * j]), a1 = __float_as_uint(re[2 * j + 1]);
        const uint32_t b0 = __float_as_uint(im[2 * j]), b1 = __float_as_uint(im[2 * j + 1]);
        q[0][j] = __builtin_amdgcn_perm(a1, a0, 0x05040100u);
        q[1][j] = __builtin_amdgcn_perm(b1, b0, 0x05040100u);
        q[2][j] = __builtin_amdgcn_perm(a1, a0, 0x07060302u);
        q[3][j] = __builtin_amdgcn_perm(b1, b0, 0x07060302u);
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) st_lds<KPT>(base + x * sub + toff, q[x]);
      return;
    }
    uint32_t t[NTM][KPT / 2];
    SP::template split<KPT>(re, sc, t);
#pragma unroll
    for (int x = 0; x < NTM; ++x) st_lds<KPT>(base + x * sub + toff, t[x]);
    SP::template split<KPT>(im, sc, t);
#pragma unroll
    for (int x = 0; x < NTM; ++x) st_lds<KPT>(base + (NTM + x) * sub + toff, t[x]);
    if constexpr (G3) {
      // re + im, scaled one binade lower (|re + im| <= 2 max(|re|, |im|))
      float sm[KPT];
#pragma unroll
      for (int j = 0; j < KPT; ++j) sm[j] = re[j] + im[j];
      SP::template split<KPT>(sm, sc - 1, t);
#pragma unroll
      for (int x = 0; x < NTM; ++x) st_lds<KPT>(base + (2 * NTM + x) * sub + toff, t[x]);
    }
  };
  // development diagnostics (wrong results, realistic operand values: the MFMAs keep multiplying
  // step 0's real operands, so the chip's power and clock stay those of real data):
  //  TQ_GEMM_DIAG_NOSTORE: the prologue splits step 0 into BOTH LDS halves, the main loop splits
  //    every step but stores nothing (the values are kept alive) -- the LDS stores' share
  //  TQ_GEMM_DIAG_NOREAD: the fragments are read once before the main loop and kept -- the
  //    fragment reads' share
  auto keep_split = [&](auto set) {
    constexpr int S = decltype(set)::value;
#pragma unroll
    for (int rw = 0; rw < 2; ++rw) {
      float re[KPT], im[KPT], sm[KPT];
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        re[j] = rw ? rv[S][j].z : rv[S][j].x;
        im[j] = rw ? rv[S][j].w : rv[S][j].y;
        sm[j] = re[j] + im[j];
      }
      uint32_t t[NTM][KPT / 2];
      SP::template split<KPT>(re, sc, t);
#pragma unroll
      for (int x = 0; x < NTM; ++x)
#pragma unroll
        for (int q = 0; q < KPT / 2; ++q) asm volatile("" ::"v"(t[x][q]));
      SP::template split<KPT>(im, sc, t);
#pragma unroll
      for (int x = 0; x < NTM; ++x)
#pragma unroll
        for (int q = 0; q < KPT / 2; ++q) asm volatile("" ::"v"(t[x][q]));
      if constexpr (G3) {
        SP::template split<KPT>(sm, sc - 1, t);
#pragma unroll
        for (int x = 0; x < NTM; ++x)
#pragma unroll
          for (int q = 0; q < KPT / 2; ++q) asm volatile("" ::"v"(t[x][q]));
      }
    }
  };
  (void)keep_split;
  auto store_stage = [&](auto set, int buf) {
    constexpr int S = decltype(set)::value;
    char* base = lds + buf * BUF + obase;
    float r0[KPT], i0[KPT], r1[KPT], i1[KPT];
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      r0[j] = rv[S][j].x; i0[j] = rv[S][j].y; r1[j] = rv[S][j].z; i1[j] = rv[S][j].w;
    }
    put(r0, i0, base, toff0);
    put(r1, i1, base, toff1);
  };

  f32x16 acc[NACC][TI][TJ];
#pragma unroll
  for (int x = 0; x < NACC; ++x)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][i][j][r] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  int a_off[TI], b_off[TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i) a_off[i] = swz(wm * TL::WM + i * 32 + fr, fh);
#pragma unroll
  for (int j = 0; j < TJ; ++j) b_off[j] = NGRP * NTM * SUBA + swz(wn * TL::WN + j * 32 + fr, fh);

  typedef uint4 FragA[NGRP * NTM][TI];
  typedef uint4 FragB[NGRP * NTM][TJ];
  // planes in the order the MFMA pairs first use them (pair 0's four first), so the first MFMAs
  // of a step wait for a third to a half of the step's fragment reads, not all of them
  static_assert(!TL::ORD || SP::NPAIR == 3, "ordered pairs: the f16 split");
  constexpr int QO[3] = {0, TL::ORD ? 2 : 1, TL::ORD ? 1 : 2};
  auto qat = [&](int qq) { return SP::NPAIR == 3 ? QO[qq] : qq; };
  auto read_frags = [&](const char* s, FragA& fa, FragB& fb) {
    bool ra[NTM] = {}, rb[NTM] = {};
#pragma unroll
    for (int qq = 0; qq < SP::NPAIR; ++qq) {
      const int q = qat(qq);
      const int xa = SP::pa(q), xb = SP::pb(q);
      if (!ra[xa]) {
        ra[xa] = true;
#pragma unroll
        for (int h = 0; h < NGRP; ++h)
#pragma unroll
          for (int i = 0; i < TI; ++i)
            fa[h * NTM + xa][i] = *reinterpret_cast<const uint4*>(s + (h * NTM + xa) * SUBA + a_off[i]);
      }
      if (!rb[xb]) {
        rb[xb] = true;
#pragma unroll
        for (int h = 0; h < NGRP; ++h)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            fb[h * NTM + xb][j] = *reinterpret_cast<const uint4*>(s + (h * NTM + xb) * SUBB + b_off[j]);
      }
    }
  };
  // pairs of (A term, B term), smallest first
  // one product group's fragments (planes h * NTM + term of A and B) / MFMAs (TL::STG)
  auto read_group = [&](const char* s, int h, FragA& fa, FragB& fb) {
#pragma unroll
    for (int x = 0; x < NTM; ++x) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
        fa[h * NTM + x][i] = *reinterpret_cast<const uint4*>(s + (h * NTM + x) * SUBA + a_off[i]);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        fb[h * NTM + x][j] = *reinterpret_cast<const uint4*>(s + (h * NTM + x) * SUBB + b_off[j]);
    }
  };
  auto mfma_group = [&](int h, const FragA& fa, const FragB& fb) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int qq = 0; qq < SP::NPAIR; ++qq) {
          const int q = qat(qq);
          acc[h][i][j] = SP::mfma(fa[h * NTM + SP::pa(q)][i], fb[h * NTM + SP::pb(q)][j], acc[h][i][j]);
        }
  };
  auto mfmas = [&](const FragA& fa, const FragB& fb) {
    if constexpr (TL::POUT) {
      static_assert(G3 && SP::NPAIR == 3, "product-major order: Gauss 3M on the f16 split");
#pragma unroll
      for (int h = 0; h < 3; ++h)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int qq = 0; qq < 3; ++qq) {
              const int q = qat(qq);
              acc[h][i][j] = SP::mfma(fa[h * NTM + SP::pa(q)][i], fb[h * NTM + SP::pb(q)][j], acc[h][i][j]);
            }
      return;
    }
#pragma unroll
    for (int qq = 0; qq < SP::NPAIR; ++qq)
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int q = qat(qq);
        const uint4 ar = fa[SP::pa(q)][i];
        const uint4 ai = fa[NTM + SP::pa(q)][i];
        if constexpr (G3) {
          const uint4 as = fa[2 * NTM + SP::pa(q)][i];
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            acc[0][i][j] = SP::mfma(ar, fb[SP::pb(q)][j], acc[0][i][j]);
            acc[1][i][j] = SP::mfma(ai, fb[NTM + SP::pb(q)][j], acc[1][i][j]);
            acc[2][i][j] = SP::mfma(as, fb[2 * NTM + SP::pb(q)][j], acc[2][i][j]);
          }
          continue;
        }
        const uint4 nai = neg8(ai);
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const uint4 br = fb[SP::pb(q)][j];
          const uint4 bi = fb[NTM + SP::pb(q)][j];
          acc[0][i][j] = SP::mfma(ar, br, acc[0][i][j]);
          acc[1][i][j] = SP::mfma(ar, bi, acc[1][i][j]);
          acc[0][i][j] = SP::mfma(nai, bi, acc[0][i][j]);
          acc[1][i][j] = SP::mfma(ai, br, acc[1][i][j]);
        }
      }
  };
  // one steady-state K-step t (t + 1 < nkt, P = t mod NSET): loads of step t + NSET into the
  // register set step t used (split one step ago) issued first; the split of step t + 1 into the
  // other LDS half and the MFMAs of step t (fragments already in registers) interleave; after the
  // barrier the fragments of step t + 1 are read, so they land under the next step's load issue
  // and split instead of stalling its first MFMAs (one fragment set live at a time)
  // body P (t = P mod U): register set P mod NSET, LDS half P & 1.  (Reading the next step's
  // fragments right after the barrier, into a second fragment set, spilled at 256 registers and
  // measured slower at 512 with fewer staging sets.)
  FragA fa;
  FragB fb;
  using I0_ = std::integral_constant<int, 0>;
  using I1_ = std::integral_constant<int, 1>;
  using I2_ = std::integral_constant<int, 2>;
  using I3_ = std::integral_constant<int, 3>;
  auto body = [&](auto par, int t) {
    constexpr int P = decltype(par)::value;
    load(std::integral_constant<int, P % NSET>{}, t + NSET < nkt ? t + NSET : nkt - 1);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (TL::PIPE) {
      static_assert(TL::STG, "pipelined groups: staged group reads");
      // group 0 of this step is in registers (read behind the previous step's barrier)
      const char* sb = lds + (P & 1) * BUF;
      read_group(sb, 1, fa, fb);
      store_stage(std::integral_constant<int, (P + 1) % NSET>{}, (P & 1) ^ 1);
      mfma_group(0, fa, fb);
      read_group(sb, 2, fa, fb);
      mfma_group(1, fa, fb);
      constexpr int NMG = SP::NPAIR * TI * TJ;
      constexpr int NRG = NTM * (TI + TJ);
      constexpr int NWR = 2 * NGRP * NTM;
      constexpr int E = 2 * NMG / NWR > 0 ? 2 * NMG / NWR : 1;
      __builtin_amdgcn_sched_group_barrier(0x100, NRG, 0);
      Interleave<0, NMG, 6, E>::run();
      __builtin_amdgcn_sched_group_barrier(0x100, NRG, 0);
      Interleave<NMG, 2 * NMG, 6, E>::run();
      __builtin_amdgcn_sched_barrier(0);
      // the split of step t + 1 is in LDS, this step's reads of its buffer are done
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      read_group(lds + ((P & 1) ^ 1) * BUF, 0, fa, fb);   // step t + 1, group 0
      mfma_group(2, fa, fb);
      __builtin_amdgcn_sched_group_barrier(0x100, NRG, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NMG, 0);
      __builtin_amdgcn_sched_barrier(0);
      return;
    }
    if constexpr (TL::STG) {
      static_assert(TL::POUT && TL::ILV, "staged group reads: product-major, interleaved");
      const char* sb = lds + (P & 1) * BUF;
      read_group(sb, 0, fa, fb);
      store_stage(std::integral_constant<int, (P + 1) % NSET>{}, (P & 1) ^ 1);
      read_group(sb, 1, fa, fb);
      mfma_group(0, fa, fb);
      read_group(sb, 2, fa, fb);
      mfma_group(1, fa, fb);
      mfma_group(2, fa, fb);
      constexpr int NMG = SP::NPAIR * TI * TJ;      // MFMAs per product group
      constexpr int NRG = NTM * (TI + TJ);          // fragment reads per product group
      constexpr int NWR = 2 * NGRP * NTM;
      constexpr int E = 3 * NMG / NWR > 0 ? 3 * NMG / NWR : 1;
      __builtin_amdgcn_sched_group_barrier(0x100, NRG, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, NRG, 0);
      Interleave<0, NMG, 3, E>::run();
      __builtin_amdgcn_sched_group_barrier(0x100, NRG, 0);
      Interleave<NMG, 3 * NMG, 3, E>::run();
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      return;
    }
#ifdef TQ_GEMM_DIAG_NOREAD
#pragma unroll
    for (int x = 0; x < NGRP * NTM; ++x) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
        asm volatile("" : "+v"(fa[x][i].x), "+v"(fa[x][i].y), "+v"(fa[x][i].z), "+v"(fa[x][i].w));
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        asm volatile("" : "+v"(fb[x][j].x), "+v"(fb[x][j].y), "+v"(fb[x][j].z), "+v"(fb[x][j].w));
    }
#else
    read_frags(lds + (P & 1) * BUF, fa, fb);
#endif
#ifdef TQ_GEMM_DIAG_NOSTORE
    keep_split(std::integral_constant<int, (P + 1) % NSET>{});
#else
    store_stage(std::integral_constant<int, (P + 1) % NSET>{}, (P & 1) ^ 1);
#endif
    mfmas(fa, fb);
    if constexpr (TL::ILV) {
      // fragment reads first, then every MFMA followed by up to 3 VALU (the split, the sign
      // flips), the split's LDS stores spread evenly: without this the compiler issued the split
      // and the MFMAs largely back to back (the no-MFMA variant's time added to the MFMA time)
      constexpr int NM = SP::NPAIR * TI * TJ * (G3 ? 3 : 4);
      constexpr int NR = NGRP * NTM * (TI + TJ);
      constexpr int NWR = 2 * NGRP * NTM;  // LDS stores per thread: 2 rows x planes
      constexpr int E = NM / NWR > 0 ? NM / NWR : 1;
      if constexpr (TL::ORD) {
        __builtin_amdgcn_sched_group_barrier(0x100, NR - NGRP * TJ, 0);
        Interleave<0, NM / 3, 3, E>::run();
        __builtin_amdgcn_sched_group_barrier(0x100, NGRP * TJ, 0);
        Interleave<NM / 3, NM, 3, E>::run();
      } else {
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
        Interleave<0, NM, 3, E>::run();
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // the MFMAs of step t stay above the barrier
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I5 = std::integral_constant<int, 5>;

  static_assert(NSET >= 2 && NSET <= 4, "register sets");
  // wave-uniform guard (readfirstlane): s_setprio ignores EXEC
  if (g.prio && __builtin_amdgcn_readfirstlane(tid) >= TL::NT / 2) __builtin_amdgcn_s_setprio(1);
  if constexpr (TL::SLOTS == 4) {
    // 4-slot ring: K-step u is loaded 5 steps ahead into set u % 4, split at step u - 2 into
    // slot u % 4, read and multiplied at step u; a barrier after every odd step -- between any
    // slot's write (step u - 2) and read (step u), and between its read and next write, one of
    // two consecutive steps is odd
    static_assert(NSET == 4, "4 staging sets");
    auto ck = [&](int u) { return u < nkt ? u : nkt - 1; };
    load(I0_{}, 0);
    load(I1_{}, ck(1));
    load(I2_{}, ck(2));
    load(I3_{}, ck(3));
    store_stage(I0_{}, 0);
    store_stage(I1_{}, 1);
    load(I0_{}, ck(4));
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    auto body4 = [&](auto par, int t) {
      constexpr int P = decltype(par)::value;   // t % 4
      load(std::integral_constant<int, (P + 1) % 4>{}, ck(t + 5));
      __builtin_amdgcn_sched_barrier(0);
      read_frags(lds + P * BUF, fa, fb);
      store_stage(std::integral_constant<int, (P + 2) % 4>{}, (P + 2) % 4);
      mfmas(fa, fb);
      if constexpr (TL::ILV) {
        constexpr int NM = SP::NPAIR * TI * TJ * (G3 ? 3 : 4);
        constexpr int NR = NGRP * NTM * (TI + TJ);
        constexpr int NWR = 2 * NGRP * NTM;
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
        Interleave<0, NM, 3, (NM / NWR > 0 ? NM / NWR : 1)>::run();
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (P & 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    int t = 0;
    for (; t + 4 <= nkt; t += 4) {
      body4(I0_{}, t);
      body4(I1_{}, t + 1);
      body4(I2_{}, t + 2);
      body4(I3_{}, t + 3);
    }
    if (t < nkt) body4(I0_{}, t);
    if (t + 1 < nkt) body4(I1_{}, t + 1);
    if (t + 2 < nkt) body4(I2_{}, t + 2);
  } else {
  constexpr int U = NSET == 3 ? 6 : NSET;  // unroll: a multiple of NSET and of 2 (LDS halves)
  load(std::integral_constant<int, 0>{}, 0);
  load(std::integral_constant<int, 1>{}, nkt > 1 ? 1 : nkt - 1);
  if constexpr (NSET >= 3) load(std::integral_constant<int, NSET >= 3 ? 2 : 0>{}, nkt > 2 ? 2 : nkt - 1);
  if constexpr (NSET >= 4) load(std::integral_constant<int, NSET >= 4 ? 3 : 0>{}, nkt > 3 ? 3 : nkt - 1);
  store_stage(std::integral_constant<int, 0>{}, 0);
#ifdef TQ_GEMM_DIAG_NOSTORE
  store_stage(std::integral_constant<int, 0>{}, 1);
#endif
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#ifdef TQ_GEMM_DIAG_NOREAD
  read_frags(lds, fa, fb);
#endif
  if constexpr (TL::PIPE) read_group(lds, 0, fa, fb);
  int t = 0;
  for (; t + U < nkt; t += U) {
    body(I0{}, t);
    body(I1{}, t + 1);
    if constexpr (U >= 4) { body(I2{}, t + 2); body(I3{}, t + 3); }
    if constexpr (U >= 6) { body(I4{}, t + 4); body(I5{}, t + 5); }
  }
  // 1 .. U steps left: all but the last split their successor
  if (t + 1 < nkt) body(I0{}, t);
  if constexpr (U >= 4) {
    if (t + 2 < nkt) body(I1{}, t + 1);
    if (t + 3 < nkt) body(I2{}, t + 2);
  }
  if constexpr (U >= 6) {
    if (t + 4 < nkt) body(I3{}, t + 3);
    if (t + 5 < nkt) body(I4{}, t + 4);
  }
  if constexpr (TL::PIPE) {   // step nkt - 1: group 0 already in registers
    const char* sb = lds + ((nkt - 1) & 1) * BUF;
    read_group(sb, 1, fa, fb);
    read_group(sb, 2, fa, fb);
    mfma_group(0, fa, fb);
    mfma_group(1, fa, fb);
    mfma_group(2, fa, fb);
  } else {
    read_frags(lds + ((nkt - 1) & 1) * BUF, fa, fb);
    mfmas(fa, fb);  // step nkt - 1
  }
  }

  const bool partial = g.splits > 1;
  float* Cout = partial ? g.W + (((int64_t)split * g.batch + b) * g.M * g.N) * 2 : g.C + (int64_t)b * g.sC * 2;
  const int64_t ldo = partial ? g.N : g.ldc;
  const float beta = partial ? 0.f : g.beta;
  const int unsc = -(sca + scb);
  auto store = [&](auto with_beta) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t gm = m0 + wm * TL::WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int64_t gn = n0 + wn * TL::WN + j * 32 + (lane & 31);
          float2* p = reinterpret_cast<float2*>(Cout + (gm * ldo + gn) * 2);
          float2 v;
          if constexpr (G3) {
            // P3 was accumulated from sums scaled one binade lower on both sides: 4 P3 (exact)
            const float p1 = acc[0][i][j][r], p2 = acc[1][i][j][r];
            v = make_float2(ldexpf(p1 - p2, unsc), ldexpf(4.f * acc[2][i][j][r] - p1 - p2, unsc));
          } else {
            v = make_float2(ldexpf(acc[0][i][j][r], unsc), ldexpf(acc[1][i][j][r], unsc));
          }
          if constexpr (decltype(with_beta)::value) {
            const float2 o = *p;
            v.x += beta * o.x;
            v.y += beta * o.y;
          }
          *p = v;
        }
  };
  if (beta != 0.f) store(std::true_type{});
  else store(std::false_type{});
  TQ_KCLOCK_END(g_kclk_kouter)
}

// ---------------------------------------------------------------------------------------------
// The same f16 split on v_mfma_f32_16x16x32_f16 (TQ_GEMM_F16_VAR=4).  MI355X_MICROARCH.md
// ('DVFS give-back' item 7): with every operand re-read from LDS the chip holds a higher clock on
// the 16x16x32 shape than on 32x32x16 at equal cycles per flop — this GEMM runs power-limited
// (1.56-1.63 GHz under load, profiles/pmc_gemm_f16_r03.json).
//
//  * block 128 x 128, 8 waves (two per SIMD) of 64 x 32 = 4 x 2 tiles of 16 x 16 (64 accumulator
//    VGPRs, as the 32x32 kernel); an MFMA consumes 32 k, so a main-loop step covers two K-slabs of
//    16 (one barrier per 32 k) and reads 24 fragments for 96 MFMAs.
//  * staging as the 32x32 kernel (a thread splits 2 rows x 4 k per slab, 16-B loads one step
//    ahead in 4 register sets = two steps of two slabs); the LDS holds two steps x two slabs
//    (128 KiB) of term planes [re h, re l, im h, im l] for A then B.
//  * plane layout per slab: 16-row blocks of 512 B, [row / 16][k-half h][row % 16 ^ h][16 B]
//    (swz16): a fragment read (lane l: row l % 16, k-chunk l / 16 = (slab, half)) puts each
//    ds_read_b128 lane group on 16 distinct 16-B slots, and the staging stores (ds_write_b64,
//    16 lanes = rows {0, 2, 4, 6} (+1) x four 8-B k-groups) on 16 distinct 8-B slots mod 128 B.
namespace xbf {
struct Tile16 {
  static constexpr int NT = 512, WMW = 2, WNW = 4, TI = 4, TJ = 2;
  static constexpr int WM = 16 * TI, WN = 16 * TJ, BM = WMW * WM, BN = WNW * WN, BK = 32, NTM = 2;
  static constexpr int SUBA = BM * 32, SUBB = BN * 32;         // bytes per term plane and slab
  static constexpr int SLAB = 2 * NTM * (SUBA + SUBB);         // one 16-k slab of A and B
  static constexpr int KPT = 4, NSET = 4;
  static_assert(BM == 128 && BN == 128 && 4 * SLAB <= 160 * 1024, "tile");
};
__device__ __forceinline__ int swz16(int row, int kg) {
  const int h = kg >> 1;
  return ((((row >> 4) << 1) + h) << 8) + (((row & 15) ^ h) << 4) + ((kg & 1) << 3);
}
__device__ __forceinline__ f32x4 mfma16(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
}  // namespace xbf

__global__ void __launch_bounds__(512, 1) gemm_c64_kouter_split16_kernel(FastArgs g) {
  using namespace xbf;
  using TL = Tile16;
  using SP = SplitF16;
  constexpr int BM = TL::BM, BN = TL::BN, TI = TL::TI, TJ = TL::TJ, NTM = TL::NTM;
  constexpr int SUBA = TL::SUBA, SUBB = TL::SUBB, SLAB = TL::SLAB, KPT = TL::KPT;
  __shared__ __attribute__((aligned(16))) char lds[4 * SLAB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % TL::WMW, wn = wid / TL::WMW;

  const int nblk = gridDim.x;
  int L = blockIdx.x;
  {
    const int q = nblk / 8, r = nblk % 8, xcd = L % 8, idx = L / 8;
    if (nblk >= 8) L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int ntile = g.mt * g.nt;
  const int tile = L % ntile;
  const int split = (L / ntile) % g.splits;
  const int b = L / (ntile * g.splits);
  const int tm = tile / g.nt, tn = tile % g.nt;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * g.kchunk;
  const int nks = (int)(g.kchunk / 16);  // slabs
  const int nv = nks / 2;                // steps (launch: kchunk % 32 == 0)

  const float2* A = reinterpret_cast<const float2*>(g.A) + ((int64_t)b * g.sA + kbeg * g.lda + m0);
  const float2* B = reinterpret_cast<const float2*>(g.B) + ((int64_t)b * g.sB + kbeg * g.ldb + n0);
  const int sca = scale_exp(g.amax_a[(int64_t)b * g.amax_bs_a]);
  const int scb = scale_exp(g.amax_b[(int64_t)b * g.amax_bs_b]);

  // staging: threads 0..255 A, 256..511 B; rows 2r, 2r+1 x k-group tkg (4 k) of a slab
  const int op = __builtin_amdgcn_readfirstlane(tid >= TL::NT / 2 ? 1 : 0);
  const int ot = tid & (TL::NT / 2 - 1);
  const int trow = 2 * (ot / 4), tkg = ot % 4;
  float4 rv[TL::NSET][KPT];
  const int64_t ld = op ? g.ldb : g.lda;
  const char* src = reinterpret_cast<const char*>(op ? B : A);
  uint32_t off[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) off[j] = (uint32_t)(((tkg * KPT + j) * ld + trow) * 8);
  const int64_t slabb = (int64_t)16 * ld * 8;
  auto ck = [&](int s) { return s < nks ? s : nks - 1; };
  auto load = [&](auto set, int s) {
    constexpr int S = decltype(set)::value;
    const char* p = src + s * slabb;
#pragma unroll
    for (int j = 0; j < KPT; ++j) rv[S][j] = *reinterpret_cast<const float4*>(p + off[j]);
  };
  const int sc = op ? scb : sca;
  const int sub = op ? SUBB : SUBA;
  const int obase = op ? 2 * NTM * SUBA : 0;
  const int toff0 = swz16(trow, tkg), toff1 = swz16(trow + 1, tkg);
  auto put = [&](const float (&re)[KPT], const float (&im)[KPT], char* base, int toff) {
    uint32_t t[NTM][KPT / 2];
    SP::template split<KPT>(re, sc, t);
#pragma unroll
    for (int x = 0; x < NTM; ++x) st_lds<KPT>(base + x * sub + toff, t[x]);
    SP::template split<KPT>(im, sc, t);
#pragma unroll
    for (int x = 0; x < NTM; ++x) st_lds<KPT>(base + (NTM + x) * sub + toff, t[x]);
  };
  auto store_stage = [&](auto set, int slot) {
    constexpr int S = decltype(set)::value;
    char* base = lds + slot * SLAB + obase;
    float r0[KPT], i0[KPT], r1[KPT], i1[KPT];
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      r0[j] = rv[S][j].x; i0[j] = rv[S][j].y; r1[j] = rv[S][j].z; i1[j] = rv[S][j].w;
    }
    put(r0, i0, base, toff0);
    put(r1, i1, base, toff1);
  };

  f32x4 acc[2][TI][TJ];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[x][i][j][r] = 0.f;

  // fragment of lane l: row l % 16 of a 16-row block, k-chunk c = l / 16 -> slab c / 2, half c % 2
  const int fr = lane & 15, fc = lane >> 4, fs = fc >> 1, fhh = fc & 1;
  int a_off[TI], b_off[TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i) a_off[i] = fs * SLAB + ((((wm * TI + i) << 1) + fhh) << 8) + ((fr ^ fhh) << 4);
#pragma unroll
  for (int j = 0; j < TJ; ++j)
    b_off[j] = fs * SLAB + 2 * NTM * SUBA + ((((wn * TJ + j) << 1) + fhh) << 8) + ((fr ^ fhh) << 4);

  uint4 fa[2 * NTM][TI], fb[2 * NTM][TJ];
  // term pairs in the order (l, h), (h, h), (h, l): the A-l fragments are dead after the first
  // third of the MFMAs and the B-l fragments, read last, reuse their registers (80 fragment
  // VGPRs live instead of 96)
  constexpr int QORD[3] = {0, 2, 1};
  auto read_frags = [&](const char* s) {
    bool ra[NTM] = {}, rb[NTM] = {};
#pragma unroll
    for (int qq = 0; qq < SP::NPAIR; ++qq) {
      const int q = QORD[qq];
      const int xa = SP::pa(q), xb = SP::pb(q);
      if (!ra[xa]) {
        ra[xa] = true;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < TI; ++i) fa[h * NTM + xa][i] = *reinterpret_cast<const uint4*>(s + (h * NTM + xa) * SUBA + a_off[i]);
      }
      if (!rb[xb]) {
        rb[xb] = true;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int j = 0; j < TJ; ++j) fb[h * NTM + xb][j] = *reinterpret_cast<const uint4*>(s + (h * NTM + xb) * SUBB + b_off[j]);
      }
    }
  };
  auto mfmas = [&]() {
#pragma unroll
    for (int qq = 0; qq < SP::NPAIR; ++qq)
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int q = QORD[qq];
        const uint4 ar = fa[SP::pa(q)][i];
        const uint4 ai = fa[NTM + SP::pa(q)][i];
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          // -Bi: the wave tile has half as many B fragments as A fragments to flip
          const uint4 br = fb[SP::pb(q)][j];
          const uint4 bi = fb[NTM + SP::pb(q)][j];
          acc[0][i][j] = mfma16(ar, br, acc[0][i][j]);
          acc[1][i][j] = mfma16(ar, bi, acc[1][i][j]);
          acc[0][i][j] = mfma16(ai, neg8(bi), acc[0][i][j]);
          acc[1][i][j] = mfma16(ai, br, acc[1][i][j]);
        }
      }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  // step v (parity P = v & 1): slabs 2v, 2v+1 sit in LDS slots 2P, 2P+1 (split last step from
  // register sets 2P, 2P+1, now free: the loads of step v + 2 go there); the split of step v + 1
  // (sets / slots 2(1-P), 2(1-P)+1) interleaves with this step's MFMAs; one barrier
  auto body = [&](auto par, int v) {
    constexpr int P = decltype(par)::value;
    load(std::integral_constant<int, 2 * P>{}, ck(2 * v + 4));
    load(std::integral_constant<int, 2 * P + 1>{}, ck(2 * v + 5));
    __builtin_amdgcn_sched_barrier(0);
    read_frags(lds + 2 * P * SLAB);
    store_stage(std::integral_constant<int, 2 * (1 - P)>{}, 2 * (1 - P));
    store_stage(std::integral_constant<int, 2 * (1 - P) + 1>{}, 2 * (1 - P) + 1);
    mfmas();
    {
      constexpr int NM = SP::NPAIR * TI * TJ * 4;   // 96
      constexpr int NR = 2 * NTM * (TI + TJ);       // 24
      constexpr int NWR = 2 * 2 * 2 * NTM;          // 2 slabs x 2 rows x 4 planes
      __builtin_amdgcn_sched_group_barrier(0x100, NR - 2 * TJ, 0);
      Interleave<0, NM / 3, 2, NM / NWR>::run();
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * TJ, 0);
      Interleave<NM / 3, NM, 2, NM / NWR>::run();
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  load(I0{}, 0);
  load(I1{}, ck(1));
  load(I2{}, ck(2));
  load(I3{}, ck(3));
  store_stage(I0{}, 0);
  store_stage(I1{}, 1);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  int v = 0;
  for (; v + 2 < nv; v += 2) {
    body(I0{}, v);
    body(I1{}, v + 1);
  }
  if (v + 1 < nv) {
    body(I0{}, v);
    read_frags(lds + 2 * SLAB);  // last step, parity 1
  } else {
    read_frags(lds);             // last step, parity 0
  }
  mfmas();

  const bool partial = g.splits > 1;
  float* Cout = partial ? g.W + (((int64_t)split * g.batch + b) * g.M * g.N) * 2 : g.C + (int64_t)b * g.sC * 2;
  const int64_t ldo = partial ? g.N : g.ldc;
  const float beta = partial ? 0.f : g.beta;
  const int unsc = -(sca + scb);
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + wm * TL::WM + i * 16 + (lane >> 4) * 4 + r;
        const int64_t gn = n0 + wn * TL::WN + j * 16 + (lane & 15);
        float2* p = reinterpret_cast<float2*>(Cout + (gm * ldo + gn) * 2);
        float2 o = make_float2(ldexpf(acc[0][i][j][r], unsc), ldexpf(acc[1][i][j][r], unsc));
        if (beta != 0.f) {
          const float2 c = *p;
          o.x += beta * c.x;
          o.y += beta * c.y;
        }
        *p = o;
      }
}

// ---------------------------------------------------------------------------------------------
// FP64 fast path: float64 / complex128 with both operands K-outer (A stored K x M, B K x N) — the
// same layout as the complex64 fast path, for the fp64 workloads (the symmetry-breaking ansatz,
// BASELINE config 5) — on v_mfma_f64_16x16x4_f64.
//
//  * operands reach LDS by LDS-DMA (global_load_lds_dwordx4: one wave-instruction = 1 KiB of one
//    k-row), in an NS-stage ring with NS - 1 K-tiles in flight, one counted vmcnt wait and one
//    raw s_barrier per K-tile (as the complex64 kernel above);
//  * fragments: lane l reads element (k = kk + l/16, m = .. + l%16) — 16 consecutive elements
//    of one k-row per 16 lanes: one ds_read_b64 (f64) / ds_read_b128 (re, im of a complex128)
//    per MFMA operand, conflict-free; the next k-step's fragments are read under this one's MFMAs;
//  * complex128: Gauss 3M (3 real MFMAs per complex k-step, default) or 4M (TQ_GEMM_3M=0);
//  * C/D of the f64 MFMA: col = lane%16, row = lane/16 + 4 r (cdna_hip_programming.md §3);
//  * split-K over the grid with the deterministic slab reduce, bijective XCD remap.
namespace fast64 {
template <int WMW_, int WNW_, int TI_, int TJ_, int BK_, int NS_, int ESZ_> struct Tile {
  static constexpr int WMW = WMW_, WNW = WNW_, TI = TI_, TJ = TJ_, BK = BK_, NS = NS_, ESZ = ESZ_;
  static constexpr int NW = WMW * WNW, NT = 64 * NW;
  static constexpr int WM = 16 * TI, WN = 16 * TJ;
  static constexpr int BM = WMW * WM, BN = WNW * WN;
  static constexpr int A_BYTES = BK * BM * ESZ, B_BYTES = BK * BN * ESZ, STAGE = A_BYTES + B_BYTES;
  static constexpr int A_ROW_PIECES = BM * ESZ / 1024, B_ROW_PIECES = BN * ESZ / 1024;
  static constexpr int A_PIECES_PER_WAVE = BK * A_ROW_PIECES / NW;
  static constexpr int B_PIECES_PER_WAVE = BK * B_ROW_PIECES / NW;
  static constexpr int NDMA = A_PIECES_PER_WAVE + B_PIECES_PER_WAVE;
  static_assert(BM * ESZ % 1024 == 0 && BN * ESZ % 1024 == 0, "1-KiB row pieces");
  static_assert(BK * A_ROW_PIECES % NW == 0 && BK * B_ROW_PIECES % NW == 0, "piece split");
  static_assert(BK % 4 == 0, "MFMA k-step");
};
// float64: 8 waves of 64 x 32 (4 x 2 MFMA tiles, 64 accumulator VGPRs), block 128 x 128,
// BK 16, 3 x 32 KiB stages
using TileF64 = Tile<2, 4, 4, 2, 16, 3, 8>;
// complex128: 8 waves of 32 x 32 (2 x 2 tiles x 3 (3M) accumulator sets = 96 VGPRs), block
// 64 x 128, BK 8, 3 x 24 KiB stages
using TileC128 = Tile<2, 4, 2, 2, 8, 3, 16>;
}

struct FastArgs64 {
  const double* A;  // K x M elements (lda elements between k-rows)
  const double* B;  // K x N elements
  double* C;        // output (ldc) or split-K slabs
  double* W;
  int64_t lda, ldb, ldc, sA, sB, sC, M, N;
  int64_t kchunk;
  int mt, nt, splits, batch;
  double beta;
};

template <bool CPLX, bool G3M, typename TL>
__global__ void __launch_bounds__(TL::NT, 1) gemm_f64_kouter_kernel(FastArgs64 g) {
  using namespace fast64;
  constexpr int BM = TL::BM, BN = TL::BN, WMW = TL::WMW, TI = TL::TI, TJ = TL::TJ, BK = TL::BK;
  constexpr int STAGE = TL::STAGE, A_BYTES = TL::A_BYTES, NSTAGE = TL::NS, ESZ = TL::ESZ;
  constexpr int EW = CPLX ? 2 : 1;
  constexpr int NACC = CPLX ? (G3M ? 3 : 2) : 1;
  static_assert(ESZ == 8 * EW, "element size");
  __shared__ __attribute__((aligned(16))) char lds[NSTAGE * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WMW, wn = wid / WMW;
  const int nblk = gridDim.x;
  int L = blockIdx.x;
  {
    const int q = nblk / 8, r = nblk % 8, xcd = L % 8, idx = L / 8;
    if (nblk >= 8) L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int ntile = g.mt * g.nt;
  const int tile = L % ntile;
  const int split = (L / ntile) % g.splits;
  const int b = L / (ntile * g.splits);
  const int tm = tile / g.nt, tn = tile % g.nt;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * g.kchunk;
  const int nkt = (int)(g.kchunk / BK);
  const char* A = reinterpret_cast<const char*>(g.A + ((int64_t)b * g.sA + kbeg * g.lda + m0) * EW);
  const char* B = reinterpret_cast<const char*>(g.B + ((int64_t)b * g.sB + kbeg * g.ldb + n0) * EW);
  const int64_t lda_b = g.lda * ESZ, ldb_b = g.ldb * ESZ;

  const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds;
  auto glds16 = [&](const char* gsrc, unsigned lds_off) {
    unsigned keep;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_base + lds_off);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto issue = [&](int t, int stage) {
    const unsigned sbase = stage * STAGE;
#pragma unroll
    for (int q = 0; q < TL::A_PIECES_PER_WAVE; ++q) {
      const int p = wid * TL::A_PIECES_PER_WAVE + q;
      const int kr = p / TL::A_ROW_PIECES, mp = p % TL::A_ROW_PIECES;
      glds16(A + ((int64_t)t * BK + kr) * lda_b + mp * 1024 + lane * 16, sbase + p * 1024);
    }
#pragma unroll
    for (int q = 0; q < TL::B_PIECES_PER_WAVE; ++q) {
      const int p = wid * TL::B_PIECES_PER_WAVE + q;
      const int kr = p / TL::B_ROW_PIECES, np = p % TL::B_ROW_PIECES;
      glds16(B + ((int64_t)t * BK + kr) * ldb_b + np * 1024 + lane * 16, sbase + A_BYTES + p * 1024);
    }
  };

  f64x4 acc[NACC][TI][TJ];
#pragma unroll
  for (int x = 0; x < NACC; ++x)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[x][i][j][r] = 0.0;

  const int fr = lane & 15, fk = lane >> 4;
  const int a_off = (fk * BM + wm * TL::WM + fr) * ESZ;
  const int b_off = A_BYTES + (fk * BN + wn * TL::WN + fr) * ESZ;
  using Frag = typename std::conditional<CPLX, double2, double>::type;

  for (int p = 0; p < NSTAGE - 1 && p < nkt; ++p) issue(p, p);
  for (int t = 0; t < nkt; ++t) {
    if (NSTAGE > 2 && t + 1 < nkt) vm_wait<TL::NDMA * (NSTAGE > 2 ? NSTAGE - 2 : 0)>();
    else vm_wait<0>();
    asm volatile("s_barrier" ::: "memory");
    if (t + NSTAGE - 1 < nkt) issue(t + NSTAGE - 1, (t + NSTAGE - 1) % NSTAGE);
    const char* s = lds + (t % NSTAGE) * STAGE;
    Frag a[TI], bb[TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i) a[i] = *reinterpret_cast<const Frag*>(s + a_off + i * 16 * ESZ);
#pragma unroll
    for (int j = 0; j < TJ; ++j) bb[j] = *reinterpret_cast<const Frag*>(s + b_off + j * 16 * ESZ);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      Frag na[TI], nb[TJ];
      if (kk + 4 < BK) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
          na[i] = *reinterpret_cast<const Frag*>(s + a_off + ((kk + 4) * BM + i * 16) * ESZ);
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          nb[j] = *reinterpret_cast<const Frag*>(s + b_off + ((kk + 4) * BN + j * 16) * ESZ);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!CPLX) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[0][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], bb[j], acc[0][i][j], 0, 0, 0);
      } else if constexpr (G3M) {
        double sa[TI], sb[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) sa[i] = a[i].x + a[i].y;
#pragma unroll
        for (int j = 0; j < TJ; ++j) sb[j] = bb[j].x + bb[j].y;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            acc[0][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i].x, bb[j].x, acc[0][i][j], 0, 0, 0);
            acc[1][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i].y, bb[j].y, acc[1][i][j], 0, 0, 0);
            acc[2][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[i], sb[j], acc[2][i][j], 0, 0, 0);
          }
      } else {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            acc[0][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i].x, bb[j].x, acc[0][i][j], 0, 0, 0);
            acc[1][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i].x, bb[j].y, acc[1][i][j], 0, 0, 0);
          }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            acc[0][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[i].y, bb[j].y, acc[0][i][j], 0, 0, 0);
            acc[1][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i].y, bb[j].x, acc[1][i][j], 0, 0, 0);
          }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kk + 4 < BK) {
#pragma unroll
        for (int i = 0; i < TI; ++i) a[i] = na[i];
#pragma unroll
        for (int j = 0; j < TJ; ++j) bb[j] = nb[j];
      }
    }
  }

  const bool partial = g.splits > 1;
  double* Cout = partial ? g.W + (((int64_t)split * g.batch + b) * g.M * g.N) * EW : g.C + (int64_t)b * g.sC * EW;
  const int64_t ldo = partial ? g.N : g.ldc;
  const double beta = partial ? 0.0 : g.beta;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + wm * TL::WM + i * 16 + (lane >> 4) + 4 * r;
        const int64_t gn = n0 + wn * TL::WN + j * 16 + (lane & 15);
        double* p = Cout + (gm * ldo + gn) * EW;
        if constexpr (!CPLX) {
          const double v = acc[0][i][j][r];
          p[0] = beta != 0.0 ? v + beta * p[0] : v;
        } else {
          double2 v;
          if constexpr (G3M) {
            const double p1 = acc[0][i][j][r], p2 = acc[1][i][j][r];
            v = make_double2(p1 - p2, acc[2][i][j][r] - p1 - p2);
          } else {
            v = make_double2(acc[0][i][j][r], acc[1][i][j][r]);
          }
          if (beta != 0.0) {
            const double2 o = *reinterpret_cast<const double2*>(p);
            v.x += beta * o.x;
            v.y += beta * o.y;
          }
          *reinterpret_cast<double2*>(p) = v;
        }
      }
}

template <typename TL>
int fast_f64_splits_t(int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch) {
  constexpr int BK = TL::BK;
  if (!(transA == 1 && transB == 0)) return 0;
  if (M % TL::BM || N % TL::BN || K % BK || K == 0) return 0;
  const int64_t tiles = (M / TL::BM) * (N / TL::BN) * batch;
  int s = 1;
  while (tiles * s * 2 <= 256 && K % ((int64_t)s * 2 * BK) == 0 && K / ((int64_t)s * 2 * BK) >= 32) s *= 2;
  if (tiles * s > INT32_MAX) return 0;
  return s;
}
int fast_f64_splits(int dtype, int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch) {
  if (dtype == TQ_F64) return fast_f64_splits_t<fast64::TileF64>(transA, transB, M, N, K, batch);
  if (dtype == TQ_C128) return fast_f64_splits_t<fast64::TileC128>(transA, transB, M, N, K, batch);
  return 0;
}

// eligibility and split choice of the fast path (shared by launch and workspace sizing)
template <typename TL>
int fast_c64_splits_t(int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch) {
  constexpr int BK = TL::BK;
  if (!(transA == 1 && transB == 0)) return 0;
  if (M % TL::BM || N % TL::BN || K % BK || K == 0) return 0;
  const int64_t tiles = (M / TL::BM) * (N / TL::BN) * batch;
  int s = 1;
  // fill the 256 CUs with one block each; keep >= 8 K-tiles per split (C3's boundary GEMM,
  // 256 x 256 x 512, ran on 4 blocks with the earlier 32)
  while (tiles * s * 2 <= 256 && K % ((int64_t)s * 2 * BK) == 0 && K / ((int64_t)s * 2 * BK) >= 8) s *= 2;
  if (tiles * s > INT32_MAX) return 0;
  return s;
}
int fast_c64_splits(int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch) {
  if (gemm_bf16()) return fast_c64_splits_t<xbf::TileX>(transA, transB, M, N, K, batch);
  if (!gemm_3m()) return fast_c64_splits_t<fastc64::Tile4M>(transA, transB, M, N, K, batch);
  return fast_c64_splits_t<fastc64::Tile3M>(transA, transB, M, N, K, batch);
}

}  // namespace

bool gemm_c64_presplit_ok(int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch,
                          int64_t lda, int64_t ldb) {
  return gemm_presplit_enabled() && gemm_bf16() && gemm_f16() && gemm_f16_var() == 0 && !fast_disabled() &&
         batch >= 1 && lda % 2 == 0 && ldb % 2 == 0 && lda < (int64_t(1) << 24) && ldb < (int64_t(1) << 24) &&
         fast_c64_splits_t<xbf::TileX>(transA, transB, M, N, K, batch) > 0;
}

int presplit_prep_launch(uint32_t* amax, int32_t* sc, int n, hipStream_t stream) {
  if (n <= 0) return TQ_OK;
  hipLaunchKernelGGL(xbf::presplit_prep_kernel, dim3(1), dim3(64), 0, stream, amax, sc, n, presplit_bias());
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

namespace {

// C_b = sum_s W[s][b] + beta * C_b
template <typename R>
__global__ void __launch_bounds__(kThreads)
splitk_reduce_kernel(const R* __restrict__ W, R* __restrict__ C, int64_t M, int64_t N,
                     int64_t ldc, int64_t sC, int64_t batch, int splits, int ew, R beta) {
  const int64_t per = M * N * ew;
  const int64_t total = per * batch;
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int64_t b = i / per, r = i % per;
    const int64_t e = r / ew, c = r % ew;
    const int64_t m = e / N, n = e % N;
    R s = 0;
    for (int k = 0; k < splits; ++k) s += W[(int64_t)k * total + i];
    R* p = C + b * sC * ew + (m * ldc + n) * ew + c;
    *p = beta != R(0) ? s + beta * *p : s;
  }
}

// ---------------------------------------------------------------------------------------------
// Skinny contraction: C (M x N with M * N <= 16, M and N powers of two) = op(A) op(B) over a
// long K -- the gradient steps of the reverse-mode tree (a gate's 4 x 4 / 8 x 2 / 2 x 8 gradient
// contracted over 2^6-2^14 elements of the running tensor: ~250 of them per C5 training step,
// engine_siamese.py:351-554 / symmetry_breaking_quantum.py:210-224), where a 64 x 64 MFMA tile
// would be 1/256 used and split 64 ways over K.  A block sums a K-range into per-thread registers
// (one k per thread per iteration, all M * N products), reduces across its waves and writes one
// partial (or C itself when it is the only block); skinny_reduce_kernel sums the partials in a
// fixed order and applies beta.  Element strides make every transposition one kernel.
template <typename R, bool CPLX, int SM, int SN>
__global__ void __launch_bounds__(256) gemm_skinny_kernel(GemmArgs g, int64_t sam, int64_t sak,
                                                         int64_t sbk, int64_t sbn, int P) {
  constexpr int EW = CPLX ? 2 : 1, MN = SM * SN, NW = 256 / 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int p = blockIdx.x;
  const int64_t b = blockIdx.y;
  const int64_t kc = (g.K + P - 1) / P;
  const int64_t k0 = (int64_t)p * kc, k1 = k0 + kc < g.K ? k0 + kc : g.K;
  const R* A = reinterpret_cast<const R*>(g.A) + b * g.sA * EW;
  const R* B = reinterpret_cast<const R*>(g.B) + b * g.sB * EW;
  R cr[MN], ci[MN];
#pragma unroll
  for (int e = 0; e < MN; ++e) cr[e] = ci[e] = R(0);
  for (int64_t k = k0 + tid; k < k1; k += 256) {
    R ar[SM], ai[SM], br[SN], bi[SN];
#pragma unroll
    for (int m = 0; m < SM; ++m) {
      const R* q = A + (m * sam + k * sak) * EW;
      ar[m] = q[0];
      ai[m] = CPLX ? q[1] : R(0);
    }
#pragma unroll
    for (int n = 0; n < SN; ++n) {
      const R* q = B + (k * sbk + n * sbn) * EW;
      br[n] = q[0];
      bi[n] = CPLX ? q[1] : R(0);
    }
#pragma unroll
    for (int m = 0; m < SM; ++m)
#pragma unroll
      for (int n = 0; n < SN; ++n) {
        cr[m * SN + n] += ar[m] * br[n];
        if constexpr (CPLX) {
          cr[m * SN + n] -= ai[m] * bi[n];
          ci[m * SN + n] += ar[m] * bi[n] + ai[m] * br[n];
        }
      }
  }
#pragma unroll
  for (int e = 0; e < MN; ++e)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      cr[e] += __shfl_xor(cr[e], o);
      if constexpr (CPLX) ci[e] += __shfl_xor(ci[e], o);
    }
  __shared__ R red[NW][MN * EW];
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < MN; ++e) {
      red[wv][e * EW] = cr[e];
      if constexpr (CPLX) red[wv][e * EW + 1] = ci[e];
    }
  }
  __syncthreads();
  if (tid < MN * EW) {
    R v = red[0][tid];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += red[w][tid];
    if (P > 1) {
      reinterpret_cast<R*>(g.W)[((int64_t)p * g.batch + b) * MN * EW + tid] = v;
    } else {
      const int e = tid / EW, c = tid % EW;
      R* cp = reinterpret_cast<R*>(g.C) + (b * g.sC + (int64_t)(e / SN) * g.ldc + (e % SN)) * EW + c;
      *cp = g.beta != 0.0 ? v + (R)g.beta * *cp : v;
    }
  }
}

// C_b = sum_p W[p][b] + beta * C_b for the skinny kernel's partials (fixed summation order)
template <typename R>
__global__ void __launch_bounds__(64) skinny_reduce_kernel(const R* __restrict__ W, R* __restrict__ C,
                                                          int64_t N, int64_t ldc, int64_t sC,
                                                          int64_t batch, int P, int mne, int ew, double beta) {
  const int e = threadIdx.x;
  const int64_t b = blockIdx.x;
  if (e >= mne) return;
  R s[8] = {};
  int p = 0;
  for (; p + 8 <= P; p += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += W[((int64_t)(p + u) * batch + b) * mne + e];
  }
  for (; p < P; ++p) s[0] += W[((int64_t)p * batch + b) * mne + e];
  R v = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  const int el = e / ew, c = e % ew;
  R* cp = C + (b * sC + (int64_t)(el / N) * ldc + (el % N)) * ew + c;
  *cp = beta != 0.0 ? v + (R)beta * *cp : v;
}

// the skinny path for M * N <= 16 (M, N powers of two): launched here (TQ_OK or a launch error);
// 1 when the shape is not one of its shapes
template <typename R, bool CPLX>
int launch_skinny(int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch,
                  const void* A, int64_t lda, int64_t sA, const void* B, int64_t ldb, int64_t sB,
                  double beta, void* C, int64_t ldc, int64_t sC, void* W, size_t wsb, hipStream_t stream) {
  auto p2 = [](int64_t v) { return v >= 1 && v <= 16 && (v & (v - 1)) == 0; };
  if (!p2(M) || !p2(N) || M * N > 16 || K < 64 || batch > 65535 || skinny_disabled()) return 1;
  constexpr int EW = CPLX ? 2 : 1;
  // ~2048 k per block (8 per thread); the partials must fit the workspace
  int P = (int)std::min<int64_t>(64, std::max<int64_t>(1, (K + 2047) / 2048));
  const size_t per = (size_t)batch * M * N * EW * sizeof(R);
  if (P > 1 && (W == nullptr || wsb < (size_t)P * per)) P = W ? (int)std::max<size_t>(1, std::min<size_t>(P, wsb / per)) : 1;
  GemmArgs g{};
  g.A = A; g.B = B; g.C = C; g.W = W;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.sA = sA; g.sB = sB; g.sC = sC; g.batch = batch; g.beta = beta;
  const int64_t sam = transA ? 1 : lda, sak = transA ? lda : 1;
  const int64_t sbk = transB ? 1 : ldb, sbn = transB ? ldb : 1;
  const dim3 grid((unsigned)P, (unsigned)batch);
#define TQ_SK(m, n) \
  if (M == m && N == n) hipLaunchKernelGGL((gemm_skinny_kernel<R, CPLX, m, n>), grid, dim3(256), 0, stream, g, sam, sak, sbk, sbn, P);
  TQ_SK(1, 1) TQ_SK(1, 2) TQ_SK(1, 4) TQ_SK(1, 8) TQ_SK(1, 16)
  TQ_SK(2, 1) TQ_SK(2, 2) TQ_SK(2, 4) TQ_SK(2, 8)
  TQ_SK(4, 1) TQ_SK(4, 2) TQ_SK(4, 4)
  TQ_SK(8, 1) TQ_SK(8, 2)
  TQ_SK(16, 1)
#undef TQ_SK
  TQ_HIP(hipGetLastError());
  if (P > 1) {
    hipLaunchKernelGGL((skinny_reduce_kernel<R>), dim3((unsigned)batch), dim3(64), 0, stream, (const R*)W, (R*)C,
                       N, ldc, sC, batch, P, (int)(M * N * EW), EW, beta);
    TQ_HIP(hipGetLastError());
  }
  return TQ_OK;
}

// The strided form (SkinnyArgs): the same sums, each operand index a bit string read through
// per-bit element strides -- one thread's k keeps its low 8 bits (its lane id) for the whole
// range, so those weights are summed once and the higher bits per 256-k step, wave-uniform.
template <typename R, bool CPLX, int SM, int SN>
__global__ void __launch_bounds__(256) gemm_skinny_strided_kernel(SkinnyArgs a, int P, int64_t kc) {
  constexpr int EW = CPLX ? 2 : 1, MN = SM * SN, NW = 256 / 64;
  constexpr int MB = SM == 16 ? 4 : SM == 8 ? 3 : SM == 4 ? 2 : SM == 2 ? 1 : 0;
  constexpr int NB = SN == 16 ? 4 : SN == 8 ? 3 : SN == 4 ? 2 : SN == 2 ? 1 : 0;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int p = blockIdx.x;
  const int64_t k0 = (int64_t)p * kc, k1 = k0 + kc < a.K ? k0 + kc : a.K;
  int64_t loA = 0, loB = 0;
#pragma unroll
  for (int b = 0; b < 8; ++b)
    if (b < a.nkb && ((tid >> b) & 1)) { loA += a.wak[b]; loB += a.wbk[b]; }
  int64_t oa[SM], ob[SN];
#pragma unroll
  for (int m = 0; m < SM; ++m) {
    oa[m] = 0;
#pragma unroll
    for (int b = 0; b < MB; ++b) if ((m >> b) & 1) oa[m] += a.wam[b];
  }
#pragma unroll
  for (int n = 0; n < SN; ++n) {
    ob[n] = 0;
#pragma unroll
    for (int b = 0; b < NB; ++b) if ((n >> b) & 1) ob[n] += a.wbn[b];
  }
  const R* A = reinterpret_cast<const R*>(a.A);
  const R* B = reinterpret_cast<const R*>(a.B);
  R cr[MN], ci[MN];
#pragma unroll
  for (int e = 0; e < MN; ++e) cr[e] = ci[e] = R(0);
  for (int64_t kb = k0; kb < k1; kb += 256) {
    int64_t hiA = 0, hiB = 0;
    const int64_t h = kb >> 8;   // kc and k0 are multiples of 256: bits >= 8 are uniform
    for (int b = 8; b < a.nkb; ++b)
      if ((h >> (b - 8)) & 1) { hiA += a.wak[b]; hiB += a.wbk[b]; }
    if (kb + tid < k1) {
      const R* pa = A + (loA + hiA) * EW;
      const R* pb = B + (loB + hiB) * EW;
      R ar[SM], ai[SM], br[SN], bi[SN];
#pragma unroll
      for (int m = 0; m < SM; ++m) {
        ar[m] = pa[oa[m] * EW];
        ai[m] = CPLX ? pa[oa[m] * EW + 1] : R(0);
      }
#pragma unroll
      for (int n = 0; n < SN; ++n) {
        br[n] = pb[ob[n] * EW];
        bi[n] = CPLX ? pb[ob[n] * EW + 1] : R(0);
      }
#pragma unroll
      for (int m = 0; m < SM; ++m)
#pragma unroll
        for (int n = 0; n < SN; ++n) {
          cr[m * SN + n] += ar[m] * br[n];
          if constexpr (CPLX) {
            cr[m * SN + n] -= ai[m] * bi[n];
            ci[m * SN + n] += ar[m] * bi[n] + ai[m] * br[n];
          }
        }
    }
  }
#pragma unroll
  for (int e = 0; e < MN; ++e)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      cr[e] += __shfl_xor(cr[e], o);
      if constexpr (CPLX) ci[e] += __shfl_xor(ci[e], o);
    }
  __shared__ R red[NW][MN * EW];
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < MN; ++e) {
      red[wv][e * EW] = cr[e];
      if constexpr (CPLX) red[wv][e * EW + 1] = ci[e];
    }
  }
  __syncthreads();
  if (tid < MN * EW) {
    R v = red[0][tid];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += red[w][tid];
    if (P > 1) {
      reinterpret_cast<R*>(a.W)[(int64_t)p * MN * EW + tid] = v;
    } else {
      R* cp = reinterpret_cast<R*>(a.C) + tid;
      *cp = a.beta != 0.0 ? v + (R)a.beta * *cp : v;
    }
  }
}

template <typename R, bool CPLX>
int skinny_strided_typed(const SkinnyArgs& a, hipStream_t stream) {
  constexpr int EW = CPLX ? 2 : 1;
  const int P = skinny_blocks(a.K);
  const int64_t kc = ((a.K + P - 1) / P + 255) / 256 * 256;
  bool hit = false;
#define TQ_SKS(m, n)                                                                                   \
  if (a.M == m && a.N == n) {                                                                          \
    hipLaunchKernelGGL((gemm_skinny_strided_kernel<R, CPLX, m, n>), dim3((unsigned)P), dim3(256), 0, stream, a, P, kc); \
    hit = true;                                                                                        \
  }
  TQ_SKS(1, 1) TQ_SKS(1, 2) TQ_SKS(1, 4) TQ_SKS(1, 8) TQ_SKS(1, 16)
  TQ_SKS(2, 1) TQ_SKS(2, 2) TQ_SKS(2, 4) TQ_SKS(2, 8)
  TQ_SKS(4, 1) TQ_SKS(4, 2) TQ_SKS(4, 4)
  TQ_SKS(8, 1) TQ_SKS(8, 2)
  TQ_SKS(16, 1)
#undef TQ_SKS
  if (!hit) {
    set_error("skinny: M x N must be powers of two with M * N <= 16");
    return TQ_ERR_INVALID;
  }
  TQ_HIP(hipGetLastError());
  if (P > 1) {
    hipLaunchKernelGGL((skinny_reduce_kernel<R>), dim3(1), dim3(64), 0, stream, (const R*)a.W, (R*)a.C,
                       (int64_t)a.N, (int64_t)a.N, (int64_t)a.M * a.N, (int64_t)1, P, a.M * a.N * EW, EW, a.beta);
    TQ_HIP(hipGetLastError());
  }
  return TQ_OK;
}

template <typename R> int ew_of(int dtype) { return dtype_complex(dtype) ? 2 : 1; }

int choose_splits(int64_t tiles, int64_t K, int BK) {
  // aim for >= 512 workgroups (2 per CU) but keep >= 8 K-tiles per split
  int s = 1;
  while (tiles * s < 512 && K / ((int64_t)(s * 2) * BK) >= 8 && s < 64) s *= 2;
  return s;
}

template <typename R, bool CPLX>
int launch_typed(int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch,
                 const void* A, int64_t lda, int64_t sA, const void* B, int64_t ldb, int64_t sB,
                 double beta, void* C, int64_t ldc, int64_t sC, void* W, size_t wsb,
                 hipStream_t stream, const uint32_t* amax_a, const uint32_t* amax_b,
                 const GemmPresplit* ps, int amax_bs_a, int amax_bs_b) {
  using C_ = Cfg<R, CPLX>;
  constexpr int EW = CPLX ? 2 : 1;
  constexpr int VE = 16 / (EW * (int)sizeof(R));
  if constexpr (CPLX && sizeof(R) == 4) {
    const int fs = fast_c64_splits(transA, transB, M, N, K, batch);
    const bool al = ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 && lda % 2 == 0 &&
                    ldb % 2 == 0 && (batch == 1 || (sA % 2 == 0 && sB % 2 == 0)) &&
                    lda < (int64_t(1) << 24) && ldb < (int64_t(1) << 24);
    const size_t need = (size_t)fs * batch * M * N * 8;
    if (ps && !(fs > 0 && al && (fs == 1 || (W != nullptr && wsb >= need)) && !fast_disabled() &&
                gemm_bf16() && gemm_f16())) {
      set_error("gemm: pre-split operands but the f16 split path is not available");
      return TQ_ERR_INVALID;
    }
    if (fs > 0 && al && (fs == 1 || (W != nullptr && wsb >= need)) && !fast_disabled()) {
      FastArgs f{};
      f.A = (const float*)A; f.B = (const float*)B; f.C = (float*)C; f.W = (float*)W;
      f.lda = lda; f.ldb = ldb; f.ldc = ldc; f.sA = sA; f.sB = sB; f.sC = sC; f.M = M; f.N = N;
      const bool g3 = gemm_3m();
      f.kchunk = K / fs;
      f.splits = fs; f.batch = (int)batch; f.beta = (float)beta;
      f.prio = g_gemm_prio;
      if (gemm_bf16()) {
        using TX = xbf::TileX;
        static_assert(TX::BM == xbf::TileH::BM && TX::BN == xbf::TileH::BN && TX::BM == xbf::TileH4::BM, "same split-K tiling");
        f.mt = (int)(M / TX::BM);
        f.nt = (int)(N / TX::BN);
        const int64_t nb = (int64_t)f.mt * f.nt * fs * batch;
        // the f16 split needs the two max words behind the split-K slabs
        const size_t slab = fs > 1 ? need : 0;
        const bool ext = amax_a != nullptr && amax_b != nullptr;
        if (gemm_f16() && (ext || (W != nullptr && wsb >= slab + amax_bytes(batch) && batch <= 65535))) {
          if (ext) {
            f.amax_a = amax_a;
            f.amax_b = amax_b;
            f.amax_bs_a = amax_bs_a;
            f.amax_bs_b = amax_bs_b;
          } else {
            // one max per batch entry and operand: every entry scaled by its own max
            uint32_t* amax = reinterpret_cast<uint32_t*>(static_cast<char*>(W) + slab);
            TQ_HIP(hipMemsetAsync(amax, 0, 2 * batch * sizeof(uint32_t), stream));
            const int64_t per = std::max<int64_t>(1, 1024 / batch);
            const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((K + 3) / 4, per));
            hipLaunchKernelGGL(xbf::absmax_kouter_kernel, dim3(gx, 2, (unsigned)batch), dim3(256), 0, stream,
                               (const float4*)A, lda / 2, sA / 2, (const float4*)B, ldb / 2, sB / 2, K,
                               M / 2, N / 2, batch, amax);
            TQ_HIP(hipGetLastError());
            f.amax_a = amax;
            f.amax_b = amax + batch;
            f.amax_bs_a = f.amax_bs_b = 1;
          }
          const int var = gemm_f16_var();
          if (ps) {
            f.sc_a = ps->sc_a;
            f.sc_b = ps->sc_b;
            f.bad = ps->bad;
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH, xbf::SplitPre>), dim3((unsigned)nb),
                               dim3(xbf::TileH::NT), 0, stream, f);
          } else if (var == 9)
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH8GQ, xbf::SplitF16>), dim3((unsigned)nb),
                               dim3(xbf::TileH8GQ::NT), 0, stream, f);
          else if (var == 8)
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH8GS, xbf::SplitF16>), dim3((unsigned)nb),
                               dim3(xbf::TileH8GS::NT), 0, stream, f);
          else if (var == 7)
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH8GP, xbf::SplitF16>), dim3((unsigned)nb),
                               dim3(xbf::TileH8GP::NT), 0, stream, f);
          else if (var == 6)
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH8G3, xbf::SplitF16>), dim3((unsigned)nb),
                               dim3(xbf::TileH8G3::NT), 0, stream, f);
          else if (var == 5)
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH8G, xbf::SplitF16>), dim3((unsigned)nb),
                               dim3(xbf::TileH8G::NT), 0, stream, f);
          else if (var == 4 && f.kchunk % xbf::Tile16::BK == 0)
            hipLaunchKernelGGL(gemm_c64_kouter_split16_kernel, dim3((unsigned)nb), dim3(xbf::Tile16::NT), 0, stream, f);
          else if (var == 3)
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH2, xbf::SplitF16>), dim3((unsigned)nb),
                               dim3(xbf::TileH2::NT), 0, stream, f);
          else if (var == 1)
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH4, xbf::SplitF16>), dim3((unsigned)nb),
                               dim3(xbf::TileH4::NT), 0, stream, f);
          else if (var == 2)
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH4G, xbf::SplitF16>), dim3((unsigned)nb),
                               dim3(xbf::TileH4G::NT), 0, stream, f);
          else
            hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<xbf::TileH, xbf::SplitF16>), dim3((unsigned)nb),
                               dim3(xbf::TileH::NT), 0, stream, f);
        } else {
          hipLaunchKernelGGL((gemm_c64_kouter_split_kernel<TX, xbf::SplitBF16>), dim3((unsigned)nb),
                             dim3(TX::NT), 0, stream, f);
        }
        TQ_HIP(hipGetLastError());
        if (fs > 1) {
          const int64_t total = batch * M * N * 2;
          const int blocks = (int)std::min<int64_t>((total + kThreads - 1) / kThreads, 4096);
          hipLaunchKernelGGL((splitk_reduce_kernel<float>), dim3(blocks), dim3(kThreads), 0, stream,
                             (const float*)W, (float*)C, M, N, ldc, sC, batch, fs, 2, (float)beta);
          TQ_HIP(hipGetLastError());
        }
        return TQ_OK;
      }
      f.mt = (int)(M / (g3 ? fastc64::Tile3M::BM : fastc64::Tile4M::BM));
      f.nt = (int)(N / (g3 ? fastc64::Tile3M::BN : fastc64::Tile4M::BN));
      f.splits = fs; f.batch = (int)batch; f.beta = (float)beta;
      const int64_t nblk = (int64_t)f.mt * f.nt * fs * batch;
      if (g3)
        hipLaunchKernelGGL((gemm_c64_kouter_kernel<true, fastc64::Tile3M>), dim3((unsigned)nblk),
                           dim3(fastc64::Tile3M::NT), 0, stream, f);
      else
        hipLaunchKernelGGL((gemm_c64_kouter_kernel<false, fastc64::Tile4M>), dim3((unsigned)nblk),
                           dim3(fastc64::Tile4M::NT), 0, stream, f);
      TQ_HIP(hipGetLastError());
      if (fs > 1) {
        const int64_t total = batch * M * N * 2;
        const int blocks = (int)std::min<int64_t>((total + kThreads - 1) / kThreads, 4096);
        hipLaunchKernelGGL((splitk_reduce_kernel<float>), dim3(blocks), dim3(kThreads), 0, stream,
                           (const float*)W, (float*)C, M, N, ldc, sC, batch, fs, 2, (float)beta);
        TQ_HIP(hipGetLastError());
      }
      return TQ_OK;
    }
  }
  if constexpr (sizeof(R) == 8) {
    const int dt = CPLX ? TQ_C128 : TQ_F64;
    const int fs = fast_f64_splits(dt, transA, transB, M, N, K, batch);
    const bool al = ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 &&
                    (CPLX || (lda % 2 == 0 && ldb % 2 == 0 && (batch == 1 || (sA % 2 == 0 && sB % 2 == 0))));
    const size_t need = (size_t)fs * batch * M * N * EW * sizeof(double);
    if (fs > 0 && al && (fs == 1 || (W != nullptr && wsb >= need)) && !fast_disabled()) {
      FastArgs64 f{};
      f.A = (const double*)A; f.B = (const double*)B; f.C = (double*)C; f.W = (double*)W;
      f.lda = lda; f.ldb = ldb; f.ldc = ldc; f.sA = sA; f.sB = sB; f.sC = sC; f.M = M; f.N = N;
      f.kchunk = K / fs;
      f.splits = fs; f.batch = (int)batch; f.beta = beta;
      auto go = [&](auto tl, auto g3c) {
        using TL = decltype(tl);
        f.mt = (int)(M / TL::BM);
        f.nt = (int)(N / TL::BN);
        const int64_t nblk = (int64_t)f.mt * f.nt * fs * batch;
        hipLaunchKernelGGL((gemm_f64_kouter_kernel<CPLX, decltype(g3c)::value, TL>), dim3((unsigned)nblk),
                           dim3(TL::NT), 0, stream, f);
      };
      if constexpr (CPLX) {
        if (gemm_3m()) go(fast64::TileC128{}, std::true_type{});
        else go(fast64::TileC128{}, std::false_type{});
      } else {
        go(fast64::TileF64{}, std::false_type{});
      }
      TQ_HIP(hipGetLastError());
      if (fs > 1) {
        const int64_t total = batch * M * N * EW;
        const int blocks = (int)std::min<int64_t>((total + kThreads - 1) / kThreads, 4096);
        hipLaunchKernelGGL((splitk_reduce_kernel<double>), dim3(blocks), dim3(kThreads), 0, stream,
                           (const double*)W, (double*)C, M, N, ldc, sC, batch, fs, EW, beta);
        TQ_HIP(hipGetLastError());
      }
      return TQ_OK;
    }
  }
  if (const int rc = launch_skinny<R, CPLX>(transA, transB, M, N, K, batch, A, lda, sA, B, ldb, sB, beta, C, ldc,
                                            sC, W, wsb, stream);
      rc != 1)
    return rc;
  GemmArgs g{};
  g.A = A; g.B = B; g.C = C; g.W = W;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.sA = sA; g.sB = sB; g.sC = sC; g.batch = batch; g.beta = beta;
  g.mt = (int)((M + C_::BM - 1) / C_::BM);
  g.nt = (int)((N + C_::BN - 1) / C_::BN);
  const int64_t tiles = (int64_t)g.mt * g.nt * batch;
  int splits = choose_splits(tiles, K, C_::BK);
  const size_t need = (size_t)splits * batch * M * N * EW * sizeof(R);
  if (splits > 1 && (W == nullptr || wsb < need)) splits = 1;
  g.splits = splits;
  g.kchunk = ((K + splits - 1) / splits + C_::BK - 1) / C_::BK * C_::BK;
  auto aligned = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  g.vecA = aligned(A) && lda % VE == 0 && (batch == 1 || sA % VE == 0);
  g.vecB = aligned(B) && ldb % VE == 0 && (batch == 1 || sB % VE == 0);
  if ((int64_t)g.mt * g.nt > INT32_MAX) {
    set_error("gemm: grid too large");
    return TQ_ERR_UNSUPPORTED;
  }
  // grid.z holds batch x splits (<= 65535): larger batches (e.g. the S*G measurement batch of
  // EngineSiamese.sample) run as several launches over batch ranges (split-K is 1 there: such
  // batches already give >= 512 tiles)
  const int64_t bchunk = splits > 1 ? batch : std::min<int64_t>(batch, 65535);
  if (bchunk * splits > 65535) {
    set_error("gemm: grid too large");
    return TQ_ERR_UNSUPPORTED;
  }
  const size_t esz = (size_t)EW * sizeof(R);
  for (int64_t b0 = 0; b0 < batch; b0 += bchunk) {
    const int64_t nb = std::min<int64_t>(bchunk, batch - b0);
    GemmArgs gb = g;
    gb.A = (const char*)A + (size_t)(b0 * sA) * esz;
    gb.B = (const char*)B + (size_t)(b0 * sB) * esz;
    gb.C = (char*)C + (size_t)(b0 * sC) * esz;
    gb.batch = nb;
    dim3 grid(g.mt * g.nt, 1, (unsigned)(nb * splits));
#define TQ_GEMM_CASE(ta, tb)                                                               \
    if (transA == ta && transB == tb) {                                                    \
      hipLaunchKernelGGL((gemm_kernel<R, CPLX, ta, tb>), grid, dim3(kThreads), 0, stream, gb); \
    }
    TQ_GEMM_CASE(0, 0)
    TQ_GEMM_CASE(0, 1)
    TQ_GEMM_CASE(1, 0)
    TQ_GEMM_CASE(1, 1)
#undef TQ_GEMM_CASE
  }
  TQ_HIP(hipGetLastError());
  if (splits > 1) {
    const int64_t total = batch * M * N * EW;
    const int blocks = (int)std::min<int64_t>((total + kThreads - 1) / kThreads, 4096);
    hipLaunchKernelGGL((splitk_reduce_kernel<R>), dim3(blocks), dim3(kThreads), 0, stream,
                       (const R*)W, (R*)C, M, N, ldc, sC, batch, splits, EW, (R)beta);
    TQ_HIP(hipGetLastError());
  }
  return TQ_OK;
}

}  // namespace

int skinny_blocks(int64_t K) { return (int)std::min<int64_t>(64, std::max<int64_t>(1, (K + 2047) / 2048)); }

int skinny_strided_launch(int dtype, const SkinnyArgs& a, hipStream_t stream) {
  if (a.K <= 0 || a.nkb < 0 || a.nkb > kSkMaxKBits || (int64_t(1) << a.nkb) != a.K ||
      (skinny_blocks(a.K) > 1 && a.W == nullptr)) {
    set_error("skinny: bad K / workspace");
    return TQ_ERR_INVALID;
  }
  switch (dtype) {
    case TQ_F32: return skinny_strided_typed<float, false>(a, stream);
    case TQ_C64: return skinny_strided_typed<float, true>(a, stream);
    case TQ_F64: return skinny_strided_typed<double, false>(a, stream);
    case TQ_C128: return skinny_strided_typed<double, true>(a, stream);
    default: set_error("skinny: dtype"); return TQ_ERR_INVALID;
  }
}

int kouter_kclock(unsigned long long* out, int n) { return TQ_KCLOCK_READ(g_kclk_kouter, out, n); }

size_t gemm_workspace(int dtype, int64_t M, int64_t N, int64_t K, int64_t batch) {
  int64_t bm, bn, bk;
  switch (dtype) {
    case TQ_F32: bm = Cfg<float, false>::BM; bn = Cfg<float, false>::BN; bk = Cfg<float, false>::BK; break;
    case TQ_C64: bm = Cfg<float, true>::BM; bn = Cfg<float, true>::BN; bk = Cfg<float, true>::BK; break;
    case TQ_F64: bm = Cfg<double, false>::BM; bn = Cfg<double, false>::BN; bk = Cfg<double, false>::BK; break;
    default: bm = Cfg<double, true>::BM; bn = Cfg<double, true>::BN; bk = Cfg<double, true>::BK; break;
  }
  const int64_t tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn) * batch;
  int s = choose_splits(tiles, K, (int)bk);
  // the complex64 fast path also keeps the f16 split's operand max words (amax_bytes)
  const int fs = dtype == TQ_C64 ? fast_c64_splits(1, 0, M, N, K, batch) : 0;
  s = std::max(s, fs);
  if (dtype == TQ_F64 || dtype == TQ_C128) s = std::max(s, fast_f64_splits(dtype, 1, 0, M, N, K, batch));
  const size_t slabs = s <= 1 ? 0 : (size_t)s * batch * M * N * dtype_size(dtype);
  return fs > 0 ? slabs + amax_bytes(batch) : slabs;
}

int gemm_launch(int dtype, int transA, int transB, int64_t M, int64_t N, int64_t K, int64_t batch,
                const void* A, int64_t lda, int64_t strideA, const void* B, int64_t ldb,
                int64_t strideB, double beta, void* C, int64_t ldc, int64_t strideC,
                void* workspace, size_t ws_bytes, hipStream_t stream, const uint32_t* amax_a,
                const uint32_t* amax_b, const GemmPresplit* presplit, int amax_bs_a, int amax_bs_b) {
  TQ_CHECK_ARG(dtype_valid(dtype), "dtype");
  TQ_CHECK_ARG(presplit == nullptr || (dtype == TQ_C64 && amax_a && amax_b && presplit->sc_a &&
                                       presplit->sc_b && presplit->bad &&
                                       gemm_c64_presplit_ok(transA, transB, M, N, K, batch, lda, ldb)),
               "pre-split operands need the complex64 f16 split path");
  TQ_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && batch >= 0, "negative size");
  TQ_CHECK_ARG(transA == 0 || transA == 1, "transA");
  TQ_CHECK_ARG(transB == 0 || transB == 1, "transB");
  if (M == 0 || N == 0 || batch == 0) return TQ_OK;
  TQ_CHECK_ARG(ldc >= N, "ldc < N");
  TQ_CHECK_ARG(transA ? lda >= M : lda >= K, "lda");
  TQ_CHECK_ARG(transB ? ldb >= K : ldb >= N, "ldb");
  switch (dtype) {
    case TQ_F32:
      return launch_typed<float, false>(transA, transB, M, N, K, batch, A, lda, strideA, B, ldb,
                                        strideB, beta, C, ldc, strideC, workspace, ws_bytes, stream, amax_a, amax_b, presplit,
                                        amax_bs_a, amax_bs_b);
    case TQ_C64:
      return launch_typed<float, true>(transA, transB, M, N, K, batch, A, lda, strideA, B, ldb,
                                       strideB, beta, C, ldc, strideC, workspace, ws_bytes, stream, amax_a, amax_b, presplit,
                                        amax_bs_a, amax_bs_b);
    case TQ_F64:
      return launch_typed<double, false>(transA, transB, M, N, K, batch, A, lda, strideA, B, ldb,
                                         strideB, beta, C, ldc, strideC, workspace, ws_bytes, stream, amax_a, amax_b, presplit,
                                        amax_bs_a, amax_bs_b);
    case TQ_C128:
      return launch_typed<double, true>(transA, transB, M, N, K, batch, A, lda, strideA, B, ldb,
                                        strideB, beta, C, ldc, strideC, workspace, ws_bytes, stream, amax_a, amax_b, presplit,
                                        amax_bs_a, amax_bs_b);
  }
  return TQ_ERR_INVALID;
}

}  // namespace tq
