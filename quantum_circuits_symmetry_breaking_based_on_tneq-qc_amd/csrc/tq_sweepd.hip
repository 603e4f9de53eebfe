// Dense sweep: the expanding tail of a qubit-line sweep as one streaming pass,
//   Y[outer, r] = sum_{k < tin} M[r][k] * X[outer, k]     (complex64, tin <= 16, tout <= 256).
//
// The per-slice sweep ops that grow the running tensor from a handful of legs to the boundary
// GEMM's operand (C4: 2^22 -> 2^26 elements, 16 -> 256 per column; the opt_einsum pairwise
// absorptions of einsum_strategy.py:639-643 / greedy_strategy.py:461-585) write 16x what they
// read.  As in-place butterfly passes (tq_sweep2.hip) they are bound by the latency of their LDS
// pass chains (three barriered passes per chunk, one chunk in flight per workgroup: 2.7 TB/s).
// Here the whole chain is ONE dense tout x tin matrix per op (composed on the device by a tiny
// sweep2 op on the identity, since the gates are device data), applied as a small-K complex
// GEMM on the f32 matrix cores (exact f32 products, f32 accumulation):
//   * D[r][c] = sum_k M[r][k] X[c][k] with v_mfma_f32_32x32x2_f32: A = M (32 outputs x 2 k, from
//     LDS planes [k][r]: conflict-free fragment reads), B = X (2 k x 32 columns, straight from
//     HBM: a half-wave reads 32 consecutive columns = 256 B; the plan only picks ops whose six
//     lowest column bits are the memory-fastest bits of X and Y);
//   * Gauss's 3M product (P1 = Mr Xr, P2 = Mi Xi, P3 = (Mr + Mi)(Xr + Xi); Dr = P1 - P2,
//     Di = P3 - P1 - P2): 3 MFMAs per k-step and 32 x 32 tile; the sums Mr + Mi are an LDS plane
//     of their own, Xr + Xi are formed once per column tile;
//   * a wave owns a 64-column group at a time, loads its tin inputs once and streams every
//     32-output tile of both 32-column halves out of the accumulators (lane -> column: a store
//     instruction writes two 256-B row segments; a row's two halves leave back to back).
// A first version on the vector ALUs (coefficients by scalar loads) ran 1.9-4.7 TB/s: the
// tout x tin coefficients (32 KiB at tin 16) stream through the scalar cache once per column
// group.  Algorithmic bytes per op = (numel(X) + numel(Y)) * 8; 8 * tin flops per output.
#include <type_traits>

#include "tq_common.h"
#include "tq_sweep2.h"

namespace tq {

namespace {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
template <typename T> using cst = __attribute__((address_space(4))) const T;

template <typename T>
__device__ __forceinline__ cst<T>* as_const(const void* p) {
  return (cst<T>*)(uintptr_t)p;
}

// f16 terms of v * 2^sc (S2DOp::split_sc; the consuming GEMM's pre-split operand form, as
// tq_sweep2.hip's f16_terms)
__device__ __forceinline__ f2v f16_terms(f2v v, int sc) {
  const float x0 = ldexpf(v.x, sc), x1 = ldexpf(v.y, sc);
  const f16x2 hv = {(_Float16)x0, (_Float16)x1};
  const uint32_t h = __builtin_bit_cast(uint32_t, hv);
  float r0, r1;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r0) : "v"(x0), "v"(h));
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r1) : "v"(x1), "v"(h));
  const f16x2 lv = {(_Float16)r0, (_Float16)r1};
  return f2v{__uint_as_float(h), __uint_as_float(__builtin_bit_cast(uint32_t, lv))};
}

constexpr int kWaves = 4;   // waves per workgroup

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int TIN>
__global__ void __launch_bounds__(64 * kWaves) sweepd_kernel(S2DLaunch L) {
  static_assert(TIN % 2 == 0 && TIN <= kS2DMaxTin, "k-steps of 2");
  constexpr int KS = TIN / 2;
  __shared__ float mp[3][TIN * kS2DMaxTout];   // planes Mr, Mi, Mr + Mi as [k][r]
  __shared__ int32_t ooff[kS2DMaxTout];        // output offsets (elements)
  int j = 0;
  for (int q = 1; q < L.nops; ++q)
    if ((int)blockIdx.x >= L.op[q].block_begin) j = q;
  const S2DOp& op = L.op[j];
  cst<S2Dense>* d = as_const<S2Dense>(op.desc);
  const int tout = d->tout, colbits = d->colbits;
  {
    const float2* M = reinterpret_cast<const float2*>(op.M);   // [r][k], written by the compose op
    for (int i = threadIdx.x; i < tout * TIN; i += 64 * kWaves) {
      const int r = i / TIN, k = i % TIN;
      const float2 v = M[i];
      mp[0][k * tout + r] = v.x;
      mp[1][k * tout + r] = v.y;
      mp[2][k * tout + r] = v.x + v.y;
    }
    for (int r = threadIdx.x; r < tout; r += 64 * kWaves) ooff[r] = (int32_t)d->out_off[r];
  }
  __syncthreads();
  const f2v* __restrict__ X = reinterpret_cast<const f2v*>(op.X);
  f2v* __restrict__ Y = reinterpret_cast<f2v*>(op.Y);
  const int lane = threadIdx.x & 63, fr = lane & 31, fk = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t ngroups = d->ncols >> 6;
  const int64_t nw = (int64_t)op.nblocks * kWaves;
  const bool use_beta = op.use_beta;
  const float beta = (float)op.beta;
  const bool split = op.split_sc != nullptr;
  const int sc = split ? *op.split_sc : 0;
  const bool track = op.amax != nullptr;
  float vmax = 0.f;
  int64_t io[KS];   // this lane's input offsets: element 2s + fk of the tile
#pragma unroll
  for (int s = 0; s < KS; ++s) io[s] = d->in_off[2 * s + fk];
  // a wave owns a 64-column group (two 32-column MFMA tiles, h = 0 / 1): every 32-output tile
  // is computed and stored for both halves back to back, so the two 256-B halves of each
  // 512-B output row segment leave within a few hundred cycles of each other
  for (int64_t g = (int64_t)((int)blockIdx.x - op.block_begin) * kWaves + wave; g < ngroups; g += nw) {
    int64_t bi = 0, bo = 0;
    for (int b = 6; b < colbits; ++b)
      if ((g >> (b - 6)) & 1) { bi += d->w_in[b]; bo += d->w_out[b]; }
    float xr[2][KS], xi[2][KS], xs[2][KS];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const f2v v = X[bi + io[s] + h * 32 + fr];
        xr[h][s] = v.x;
        xi[h][s] = v.y;
        xs[h][s] = v.x + v.y;
      }
    for (int rt = 0; rt < tout; rt += 32) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x16 p1 = {}, p2 = {}, p3 = {};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int a = (2 * s + fk) * tout + rt + fr;
          p1 = __builtin_amdgcn_mfma_f32_32x32x2f32(mp[0][a], xr[h][s], p1, 0, 0, 0);
          p2 = __builtin_amdgcn_mfma_f32_32x32x2f32(mp[1][a], xi[h][s], p2, 0, 0, 0);
          p3 = __builtin_amdgcn_mfma_f32_32x32x2f32(mp[2][a], xs[h][s], p3, 0, 0, 0);
        }
        // accumulator e of a lane: output row rt + (e & 3) + 8 (e >> 2) + 4 fk, column h*32 + fr
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = rt + (e & 3) + 8 * (e >> 2) + 4 * fk;
          f2v v = {p1[e] - p2[e], p3[e] - p1[e] - p2[e]};
          f2v* p = Y + (bo + ooff[r] + h * 32 + fr);
          if (use_beta) v += *p * beta;
          if (track) vmax = fmaxf(vmax, fmaxf(fabsf(v.x), fabsf(v.y)));
          *p = split ? f16_terms(v, sc) : v;
          // keeps the 16 store addresses from being formed (and held) all at once
          if ((e & 3) == 3) asm volatile("" ::: "memory");
        }
      }
    }
  }
  if (track) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
    if (lane == 0) atomicMax(op.amax, __float_as_uint(vmax));
  }
}

}  // namespace

int sweepd_launch(int dtype, const S2DLaunch& L, hipStream_t stream) {
  if (dtype != TQ_C64) {
    set_error("sweepd: complex64 only");
    return TQ_ERR_INVALID;
  }
  if (L.nops < 1 || L.nops > kS2MaxOps) {
    set_error("sweepd: bad op count");
    return TQ_ERR_INVALID;
  }
  int blocks = 0;
  const int tin = L.op[0].tin;
  for (int q = 0; q < L.nops; ++q) {
    if (L.op[q].tin != tin) {
      set_error("sweepd: one input tile size per launch");
      return TQ_ERR_INVALID;
    }
    // the kernel stores whole 32-output tiles and stages at most kS2DMaxTout offsets
    if (L.op[q].tout < 32 || L.op[q].tout % 32 || L.op[q].tout > kS2DMaxTout || !L.op[q].desc || !L.op[q].M) {
      set_error("sweepd: bad output tile");
      return TQ_ERR_INVALID;
    }
    blocks = std::max(blocks, L.op[q].block_begin + L.op[q].nblocks);
  }
  if (blocks <= 0) return TQ_OK;
  switch (tin) {
    case 2: hipLaunchKernelGGL(sweepd_kernel<2>, dim3(blocks), dim3(64 * kWaves), 0, stream, L); break;
    case 4: hipLaunchKernelGGL(sweepd_kernel<4>, dim3(blocks), dim3(64 * kWaves), 0, stream, L); break;
    case 8: hipLaunchKernelGGL(sweepd_kernel<8>, dim3(blocks), dim3(64 * kWaves), 0, stream, L); break;
    case 16: hipLaunchKernelGGL(sweepd_kernel<16>, dim3(blocks), dim3(64 * kWaves), 0, stream, L); break;
    default:
      set_error("sweepd: tin must be 2, 4, 8 or 16");
      return TQ_ERR_INVALID;
  }
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

}  // namespace tq
