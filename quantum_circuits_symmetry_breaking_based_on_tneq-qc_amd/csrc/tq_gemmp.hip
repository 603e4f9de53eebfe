// The boundary GEMM on pre-split operands ("planes"): complex64 C = A^T B (both K-outer) with f32
// accuracy on the f16 matrix cores, where the f32 -> f16 term split has already been done by the
// operands' producer (the dense sweep, tq_sweepd.hip planes mode).  The contraction it replaces is
// the tensordot of the cut network's two halves (einsum_strategy.py:639-643 through opt_einsum;
// SURVEY.md §8(a) row a5), the dominant kernel of the C4 step.
//
// Operand form (per batch entry = slice lane, per operand): six f16 planes, each [k][m] with
// element (k, m) at k * ld + m, plane p at p * ps:
//   0 re_h, 1 re_l, 2 im_h, 3 im_l, 4 s_h, 5 s_l      (s = re + im, scaled one binade lower)
// where x * 2^sc = h + l (h = f16(x 2^sc), l = f16(x 2^sc - h)), sc a power-of-two scale per
// operand and lane from an a-priori bound of the operand (so max |x| 2^sc < 2^15: no overflow;
// values far below the bound lose nothing that matters at the f32 level of the result).
//
// Gauss's three real products P1 = Ar Br, P2 = Ai Bi, P3 = (Ar + Ai)(Br + Bi), each with the
// three term products (h h, h l, l h) -- 18 M N K MFMA flops per complex GEMM, as the
// GEMM-side split kernel (tq_gemm.hip) executes, but without its split VALU, its LDS term-plane
// stores and its register staging:
//   * one workgroup = one real product x one 256 x 256 output tile x one K range (split-K);
//     8 waves (2 over M x 4 over N) of 128 x 64 on v_mfma_f32_16x16x32_f16;
//   * per 32-deep K-step the h and l planes of A and B (4 x 16 KiB) reach LDS by LDS-DMA
//     (global_load_lds_dwordx4, two buffers: the next step's DMA flies under this step's MFMAs),
//     into an image whose 32-byte chunks are XOR-swizzled by k so that the transposed fragment
//     reads (ds_read_b64_tr_b16: the operands are K-outer) are bank-conflict free;
//   * a wave reads Ah, Bh, Bl, Al fragments once and runs the 3 term products (96 MFMAs);
//   * f32 partial tiles [batch][product][split][M][N]; planes_combine_kernel sums the K splits,
//     forms Cr = P1 - P2, Ci = 4 P3 - P1 - P2, unscales by 2^-(sc_a + sc_b) per lane and sums the
//     slice lanes (the plan's lane sum) in one pass.
// Probe (probes/f16gemm_probe.hip, C4 shape, same executed flops as the split kernel's 5.1 ms):
// 3.4-3.6 ms per 4-lane launch, 1.39-1.46 PF executed at 1.78-1.88 GHz.
#include <algorithm>

#include "tq_common.h"
#include "tq_kclock.h"

namespace tq {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define TQ_LDS __attribute__((address_space(3)))

constexpr int kBM = 256, kBN = 256, kBK = 32, kNT = 512;
TQ_KCLOCK_DEFINE(g_kclk_gemmp)
constexpr int kTB = kBK * kBM * 2;   // bytes of one plane tile (16 KiB)

// chunk swizzle: the 32-byte chunk c of LDS row k holds global chunk c ^ f(k)
__device__ __forceinline__ int fsw(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

__global__ void __launch_bounds__(kNT) gemm_planes_kernel(PlanesGemmArgs g) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * 4 * kTB];
  TQ_KCLOCK_BEGIN()
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;
  // XCD-aware order (bijective for any count): the 8 round-robin XCD groups of workgroups
  // take consecutive tile indices, so a (lane, product, split) group of tiles sharing operand
  // panels runs on one XCD
  const int nwg = gridDim.x;
  int L = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = L % 8, idx = L / 8;
    if (nwg >= 8) L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int nt = g.N / kBN, ntile = (g.M / kBM) * nt;
  const int tile = L % ntile, grp = L / ntile;
  const int split = grp % g.splits, prod = (grp / g.splits) % 3, b = grp / (g.splits * 3);
  const int m0 = (tile / nt) * kBM, n0 = (tile % nt) * kBN;
  const int64_t kc = g.K / g.splits, k0 = split * kc;
  const int nk = (int)(kc / kBK);
  // h plane of this product (l = h + 1 plane)
  const _Float16* Ah = g.A + b * g.sA + (2 * prod) * g.psA + k0 * g.lda + m0;
  const _Float16* Bh = g.B + b * g.sB + (2 * prod) * g.psB + k0 * g.ldb + n0;

  // LDS-DMA: wave-instruction i of wave w fills 1 KiB = tile rows 2 (8 i + w), +1 of a plane
  // image; lane l: row r, chunk c' = (l & 31) >> 1, half l & 1, holding global chunk c' ^ f(r)
  uint32_t goA[2], goB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 2 * (8 * i + w) + (lane >> 5);
    const int c = ((lane & 31) >> 1) ^ fsw(r);
    goA[i] = (uint32_t)(r * g.lda + c * 16 + (lane & 1) * 8);
    goB[i] = (uint32_t)(r * g.ldb + c * 16 + (lane & 1) * 8);
  }
  // the DMA is issued from inline asm: hipcc treats an in-flight LDS-DMA as a possible alias of
  // the next ds_read and would drain it with vmcnt(0) before every fragment read; the waits below
  // are placed by hand
  const unsigned lbase = (unsigned)(uintptr_t)(TQ_LDS char*)lds;
  auto glds16 = [&](const void* src, unsigned off) {
    unsigned keep;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lbase + off);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  };
  auto stage = [&](int t, int buf) {
    const _Float16* pa = Ah + (int64_t)t * kBK * g.lda;
    const _Float16* pb = Bh + (int64_t)t * kBK * g.ldb;
    const unsigned o = buf * 4 * kTB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      glds16(pa + goA[i], o + (8 * i + w) * 1024);
      glds16(pa + g.psA + goA[i], o + kTB + (8 * i + w) * 1024);
      glds16(pb + goB[i], o + 2 * kTB + (8 * i + w) * 1024);
      glds16(pb + g.psB + goB[i], o + 3 * kTB + (8 * i + w) * 1024);
    }
  };
  // transposed fragment reads: lane l = 16 g4 + 4 q + p reads image row k = 8 g4 + 4 u + q,
  // 8 B at columns 4p .. 4p+3 of 16-column chunk c (stored at chunk c ^ f(k), f(k) = x)
  const int g4 = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int x = q | ((g4 & 1) << 2);
  const int rowb = (8 * g4 + q) * (kBM * 2) + 8 * p;
  int aoff[8], boff[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) aoff[i] = rowb + ((wm * 8 + i) ^ x) * 32;
#pragma unroll
  for (int j = 0; j < 4; ++j) boff[j] = 2 * kTB + rowb + ((wn * 4 + j) ^ x) * 32;
  auto rd = [&](const char* s, int off) -> f16x8 {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((TQ_LDS s16x4*)(s + off));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((TQ_LDS s16x4*)(s + off + 4 * kBM * 2));
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int t = 0; t < nk; ++t) {
    const char* s = lds + (t & 1) * 4 * kTB;
    // the other buffer was last read in step t - 1, whose reads every wave finished before the
    // barrier that ended it
    if (t + 1 < nk) stage(t + 1, (t & 1) ^ 1);
    f16x8 ah[8], al[8], bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bh[j] = rd(s, boff[j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) ah[i] = rd(s, aoff[i]);
#pragma unroll
    for (int j = 0; j < 4; ++j) bl[j] = rd(s, boff[j] + kTB);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) al[i] = rd(s, aoff[i] + kTB);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
    // the MFMAs stay above the wait (hipcc would otherwise hoist the wait for the next step's DMA
    // in front of them and expose its latency every step); then: next buffer landed, this
    // buffer's reads done, for every wave
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // partial tile: C/D of 16x16x32: column lane & 15, row 4 (lane >> 4) + register
  float* W = g.W + (((int64_t)b * 3 + prod) * g.splits + split) * (int64_t)g.M * g.N;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 128 + i * 16 + g4 * 4 + r;
        const int n = n0 + wn * 64 + j * 16 + (lane & 15);
        W[(int64_t)m * g.N + n] = acc[i][j][r];
      }
  TQ_KCLOCK_END(g_kclk_gemmp)
}

// out(m, n) = sum over lanes j (lane_sum) or lane j alone of
//   2^-(sc_a[j] + sc_b[j]) (P1 - P2, 4 P3 - P1 - P2),  Px = sum over the K splits
// (+ beta * out).  Four consecutive n per thread.
__global__ void __launch_bounds__(256) planes_combine_kernel(PlanesCombineArgs c) {
  const int64_t n4 = c.N / 4;
  const int64_t total = (int64_t)c.M * n4 * (c.lane_sum ? 1 : c.batch);
  const int64_t MN = (int64_t)c.M * c.N;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t mn4 = e % ((int64_t)c.M * n4);
    const int jo = (int)(e / ((int64_t)c.M * n4));
    const int64_t m = mn4 / n4, n = (mn4 % n4) * 4;
    float4 re = make_float4(0.f, 0.f, 0.f, 0.f), im = re;
    const int jb = c.lane_sum ? 0 : jo, je = c.lane_sum ? c.batch : jo + 1;
    for (int j = jb; j < je; ++j) {
      float4 P[3];
      for (int x = 0; x < 3; ++x) {
        P[x] = make_float4(0.f, 0.f, 0.f, 0.f);
        const float* base = c.W + (((int64_t)j * 3 + x) * c.splits) * MN + m * c.N + n;
        for (int s = 0; s < c.splits; ++s) {
          const float4 v = *reinterpret_cast<const float4*>(base + s * MN);
          P[x].x += v.x; P[x].y += v.y; P[x].z += v.z; P[x].w += v.w;
        }
      }
      const int us = -(c.sc_a[j * c.sc_stride] + c.sc_b[j * c.sc_stride]);
      re.x += ldexpf(P[0].x - P[1].x, us); re.y += ldexpf(P[0].y - P[1].y, us);
      re.z += ldexpf(P[0].z - P[1].z, us); re.w += ldexpf(P[0].w - P[1].w, us);
      im.x += ldexpf(4.f * P[2].x - P[0].x - P[1].x, us); im.y += ldexpf(4.f * P[2].y - P[0].y - P[1].y, us);
      im.z += ldexpf(4.f * P[2].z - P[0].z - P[1].z, us); im.w += ldexpf(4.f * P[2].w - P[0].w - P[1].w, us);
    }
    float4* o = reinterpret_cast<float4*>(reinterpret_cast<float2*>(c.C) + jo * c.sC + m * c.ldc + n);
    float4 v0 = make_float4(re.x, im.x, re.y, im.y), v1 = make_float4(re.z, im.z, re.w, im.w);
    if (c.beta != 0.f) {
      const float4 a = o[0], bq = o[1];
      v0.x += c.beta * a.x; v0.y += c.beta * a.y; v0.z += c.beta * a.z; v0.w += c.beta * a.w;
      v1.x += c.beta * bq.x; v1.y += c.beta * bq.y; v1.z += c.beta * bq.z; v1.w += c.beta * bq.w;
    }
    o[0] = v0;
    o[1] = v1;
  }
}

}  // namespace

int planes_gemm_splits(int64_t M, int64_t N, int64_t K, int64_t batch) {
  // workgroup count = batch x 3 x tiles x splits: the split count that fills whole rounds of
  // the 256 CUs best (ties: fewer splits, less partial traffic), at least two rounds when K allows
  const int64_t base = batch * 3 * (M / kBM) * (N / kBN);
  int best = 1;
  double best_eff = -1;
  for (int s = 1; s <= 16; s *= 2) {
    if (K % ((int64_t)s * kBK)) break;
    const int64_t n = base * s;
    const double rounds = (double)((n + 255) / 256);
    double eff = (double)n / (rounds * 256.0);
    if (n < 512 && s < 16 && K % ((int64_t)2 * s * kBK) == 0) eff *= 0.9;   // prefer >= 2 rounds
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = s;
    }
  }
  return best;
}

bool planes_gemm_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  return M % kBM == 0 && N % kBN == 0 && K % kBK == 0 && K > 0 && lda >= M && ldb >= N && lda % 8 == 0 &&
         ldb % 8 == 0 && (int64_t)kBK * lda < (int64_t(1) << 31) && (int64_t)kBK * ldb < (int64_t(1) << 31);
}

static size_t planes_ws_one(int64_t M, int64_t N, int64_t K, int64_t batch) {
  return (size_t)batch * 3 * planes_gemm_splits(M, N, K, batch) * M * N * sizeof(float);
}

// partials of a launch of up to `batch` entries: a partial lane batch (a slice range that is not a
// multiple of the lanes) may pick more splits than a full one (C4, 4 lanes: 4 splits; 3: 16)
size_t planes_gemm_workspace(int64_t M, int64_t N, int64_t K, int64_t batch) {
  size_t w = 0;
  for (int64_t b = 1; b <= batch; ++b) w = std::max(w, planes_ws_one(M, N, K, b));
  return w;
}

int planes_gemm_kclock(unsigned long long* out, int n) { return TQ_KCLOCK_READ(g_kclk_gemmp, out, n); }

// the launcher's argument checks, host only (tq_planes_gemm_check: CPU tests of the sizing)
int planes_gemm_check(int64_t M, int64_t N, int64_t K, int64_t batch, int64_t lda, int64_t ldb, size_t ws_bytes) {
  if (!planes_gemm_ok(M, N, K, lda, ldb) || batch < 1) {
    set_error("planes gemm: unsupported shape");
    return TQ_ERR_INVALID;
  }
  if (planes_ws_one(M, N, K, batch) > ws_bytes) {
    set_error("planes gemm: partials exceed the workspace");
    return TQ_ERR_INVALID;
  }
  return TQ_OK;
}

int planes_gemm_launch(const PlanesGemmArgs& a0, const PlanesCombineArgs& c0, hipStream_t stream) {
  TQ_TRY(planes_gemm_check(a0.M, a0.N, a0.K, a0.batch, a0.lda, a0.ldb, a0.ws_bytes));
  PlanesGemmArgs a = a0;
  a.splits = planes_gemm_splits(a.M, a.N, a.K, a.batch);
  const int64_t nwg = (int64_t)a.batch * 3 * a.splits * (a.M / kBM) * (a.N / kBN);
  hipLaunchKernelGGL(gemm_planes_kernel, dim3((unsigned)nwg), dim3(kNT), 0, stream, a);
  TQ_HIP(hipGetLastError());
  PlanesCombineArgs c = c0;
  c.W = a.W;
  c.M = a.M;
  c.N = a.N;
  c.batch = a.batch;
  c.splits = a.splits;
  const int64_t work = (int64_t)c.M * (c.N / 4) * (c.lane_sum ? 1 : c.batch);
  const int blocks = (int)std::min<int64_t>((work + 255) / 256, 4096);
  hipLaunchKernelGGL(planes_combine_kernel, dim3(blocks), dim3(256), 0, stream, c);
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

}  // namespace tq
