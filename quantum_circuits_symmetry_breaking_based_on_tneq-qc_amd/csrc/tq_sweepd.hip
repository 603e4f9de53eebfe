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
//     Di = P3 - P1 - P2): 3 MFMAs per k-step and 32 x 32 tile; the sums Mr + Mi and Xr + Xi
//     are formed in registers;
//   * a wave owns a 32-column tile at a time (inputs loaded once, column bases from small LDS
//     tables) and streams every 32-output tile out of the accumulators; lane pairs trade one
//     value per two rows so that every lane stores 16 B (two columns of one row): 4 x 256-B row
//     segments per store instruction.
// Measured (C4, one 4-lane launch = 2 GiB of stores): 450-490 us, ~4.5 TB/s, against 1.6 ms for the
// same ops as sweep2 passes.  What does not bound it: the MFMAs (removed: -10 %), the stores'
// instruction count (8-B -> 16-B stores: +-0), the tile shape (64-column groups, two output tiles
// in flight per wave: +-0 / -15 %), a dedicated loader wave feeding the inputs through LDS
// (-30 %: the per-round barrier aligns the waves' MFMA phases).  The tin = 8 op sits at the same
// 450 us as tin = 16 with half the MFMA work: the output stream itself (2^21 separate 256-B row
// segments per op, each written once) runs at ~4.5 TB/s, where a linear fill reaches 6.35 TB/s.
// A first version on the vector ALUs (coefficients by scalar loads) ran 1.9-4.7 TB/s: the
// tout x tin coefficients (32 KiB at tin 16) stream through the scalar cache once per column
// group.  Algorithmic bytes per op = (numel(X) + numel(Y)) * 8; 8 * tin flops per output.
#include <type_traits>
#include <utility>

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
// f16 terms (h, l) of two values already scaled: h = f16(x), l = f16(x - h)
__device__ __forceinline__ f2v f16_terms_scaled(f2v v) {
  const f16x2 hv = {(_Float16)v.x, (_Float16)v.y};
  const uint32_t h = __builtin_bit_cast(uint32_t, hv);
  float r0, r1;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r0) : "v"(v.x), "v"(h));
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r1) : "v"(v.y), "v"(h));
  const f16x2 lv = {(_Float16)r0, (_Float16)r1};
  return f2v{__uint_as_float(h), __uint_as_float(__builtin_bit_cast(uint32_t, lv))};
}
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

#ifndef TQ_S2D_DIAG
// development diagnostics (a separate build, make EXTRA=-DTQ_S2D_DIAG=n): 1 no MFMAs, 2 no
// stores, 3 no MFMAs and no f16 split (the planes path's store stream alone)
#define TQ_S2D_DIAG 0
#endif

constexpr int kWaves = 4;             // waves per workgroup
constexpr int kLevels = 7;            // column-base tables: 6 column bits each, bits 6 .. 47

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

// LDS of one workgroup: the coefficient planes Mr, Mi as [k][r] (room for TMAX input elements),
// output offsets (elements), column-group bases (in, out) per 6-bit level, column-bit weights
template <int TMAX>
struct SdSmem {
  float mp[2][TMAX * kS2DMaxTout];
  float red[kWaves];
  int32_t ooff[kS2DMaxTout];
  int64_t btab[2][kLevels][64];
  int64_t wcol[2][kS2MaxColBits];
  // planes mode: each wave's next 64-column group of X, [k][64 columns] (LDS-DMA target)
  __attribute__((aligned(16))) float2 xs[kWaves][TMAX * 64];
};

// one op's share of the launch (its workgroups stride over its 32-column tiles)
template <int TIN, bool NTS, int TMAX>
__device__ __forceinline__ void sweepd_op(const S2DOp& op, SdSmem<TMAX>& sm) {
  static_assert(TIN % 2 == 0 && TIN <= TMAX && TMAX <= kS2DMaxTin, "k-steps of 2");
  constexpr int KS = TIN / 2;
  auto& mp = sm.mp;
  auto& ooff = sm.ooff;
  auto& btab = sm.btab;
  auto& wcol = sm.wcol;
  cst<S2Dense>* d = as_const<S2Dense>(op.desc);
  const int tout = d->tout, colbits = d->colbits;
  const int tid = threadIdx.x;
  {
    const float2* M = reinterpret_cast<const float2*>(op.M);   // [r][k], written by the compose op
    for (int i = tid; i < tout * TIN; i += 64 * kWaves) {
      const int r = i % tout, k = i / tout;                    // LDS-write order: conflict-free
      const float2 v = M[r * TIN + k];
      mp[0][k * tout + r] = v.x;
      mp[1][k * tout + r] = v.y;
    }
    for (int r = tid; r < tout; r += 64 * kWaves) ooff[r] = (int32_t)d->out_off[r];
    for (int i = tid; i < 2 * kS2MaxColBits; i += 64 * kWaves)
      wcol[i / kS2MaxColBits][i % kS2MaxColBits] = (i / kS2MaxColBits) ? d->w_out[i % kS2MaxColBits] : d->w_in[i % kS2MaxColBits];
  }
  __syncthreads();
  // planes mode: the operand scale from an a-priori bound of the output, identical in every
  // workgroup of the op (so every lane of the operand is scaled alike)
  const bool planes = op.planes != nullptr;
  int psc = 0, xsc = 0;
  if (planes) {
    float rs = 0.f;
    for (int r = tid; r < tout; r += 64 * kWaves) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < TIN; ++k) a += sqrtf(mp[0][k * tout + r] * mp[0][k * tout + r] + mp[1][k * tout + r] * mp[1][k * tout + r]);
      rs = fmaxf(rs, a);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) rs = fmaxf(rs, __shfl_xor(rs, o));
    if ((tid & 63) == 0) sm.red[tid >> 6] = rs;
    __syncthreads();
    rs = sm.red[0];
#pragma unroll
    for (int i = 1; i < kWaves; ++i) rs = fmaxf(rs, sm.red[i]);
    // |Y| <= |X|max * rs, |X|max <= sqrt(2) max(|re|, |im|); margin for the rounding of the bound
    const float bound = __uint_as_float(*op.amax_in) * 1.41421356f * rs * 1.001f;
    const uint32_t bits = __float_as_uint(bound);
    const int E = (int)((bits >> 23) & 0xff);
    if (bits != 0 && E != 255) {
      const int e = E ? E - 127 : (31 - __clz((int)(bits & 0x7fffff))) - 149;
      psc = 14 - e;   // bound * 2^psc in [2^14, 2^15): no f16 overflow (65504)
    }
    if (blockIdx.x == (unsigned)op.block_begin && tid == 0) *op.sc_out = psc;
    // the scale is applied to the operands instead of every output: X by 2^xsc (its max to
    // [1, 2), exact) as it is loaded, M by 2^(psc - xsc) here (exact: |M 2^(psc - xsc)| <=
    // 2^16 by the bound), so the products come out scaled
    const uint32_t xb = *op.amax_in;
    const int XE = (int)((xb >> 23) & 0xff);
    xsc = (xb == 0 || XE == 255) ? 0 : -(XE ? XE - 127 : (31 - __clz((int)(xb & 0x7fffff))) - 149);
    __syncthreads();   // every wave has read M for the bound
    for (int i = tid; i < tout * TIN; i += 64 * kWaves) {
      mp[0][i] = ldexpf(mp[0][i], psc - xsc);
      mp[1][i] = ldexpf(mp[1][i], psc - xsc);
    }
    __syncthreads();
  }
  // btab[io][l][v] = sum of the weights of the set bits of v among column bits 6+6l .. 6+6l+5
  for (int i = tid; i < 2 * kLevels * 64; i += 64 * kWaves) {
    const int io = i / (kLevels * 64), l = (i / 64) % kLevels, v = i % 64;
    int64_t acc = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int cb = 6 + 6 * l + b;
      if (((v >> b) & 1) && cb < colbits) acc += wcol[io][cb];
    }
    btab[io][l][v] = acc;
  }
  __syncthreads();
  auto base = [&](int io, int64_t g) {
    int64_t b = 0;
#pragma unroll
    for (int l = 0; l < kLevels; ++l) b += btab[io][l][(g >> (6 * l)) & 63];
    return b;
  };
  const f2v* __restrict__ X = reinterpret_cast<const f2v*>(op.X);
  f2v* __restrict__ Y = reinterpret_cast<f2v*>(op.Y);
  const int lane = tid & 63, fr = lane & 31, fk = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t ntiles = d->ncols >> 5;
  const int64_t nw = (int64_t)op.nblocks * kWaves;
  const bool use_beta = op.use_beta;
  const float beta = (float)op.beta;
  const bool split = op.split_sc != nullptr;
  const int sc = split ? *op.split_sc : 0;
  const bool track = op.amax != nullptr;
  const bool odd = lane & 1;
  float vmax = 0.f;
  int32_t io[KS];   // this lane's input offsets: element 2s + fk of the tile (< 2^31, plan)
#pragma unroll
  for (int s = 0; s < KS; ++s) io[s] = (int32_t)d->in_off[2 * s + fk];
  // one 32-output tile's results (Cr, Ci accumulators) out as 16-B stores: accumulator e of a
  // lane is output row rt + (e & 3) + 8 (e >> 2) + 4 fk, column fr; rows of e and e + 1 are
  // adjacent, so the lane pair (2i, 2i+1) trades one value and the even lane stores row(e), the
  // odd lane row(e+1), both columns
  auto emit = [&](const f32x16& cr, const f32x16& ci, const f2v* Yt, int rt) {
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      const f2v v0 = {cr[e], ci[e]};
      const f2v v1 = {cr[e + 1], ci[e + 1]};
      if (track) vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v0.x), fabsf(v0.y)), fmaxf(fabsf(v1.x), fabsf(v1.y))));
      const f2v send = odd ? v0 : v1;
      f2v recv;   // quad_perm [1, 0, 3, 2]: the partner lane's value
      recv.x = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send.x), 0xB1, 0xF, 0xF, false));
      recv.y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send.y), 0xB1, 0xF, 0xF, false));
      f4v w = odd ? f4v{recv.x, recv.y, v1.x, v1.y} : f4v{v0.x, v0.y, recv.x, recv.y};
      const int r = rt + (e & 3) + 8 * (e >> 2) + 4 * fk + (odd ? 1 : 0);
      f4v* p = reinterpret_cast<f4v*>(const_cast<f2v*>(Yt) + ooff[r]);
      if (use_beta) w += *p * beta;
      if (split) {
        const f2v a = f16_terms(f2v{w.x, w.y}, sc), b = f16_terms(f2v{w.z, w.w}, sc);
        w = f4v{a.x, a.y, b.x, b.y};
      }
#if TQ_S2D_DIAG == 2
      if (w.x == 12345.f) *p = w;   // development diagnostic: no stores
#else
      if constexpr (NTS) __builtin_nontemporal_store(w, p);   // streaming stores (TQ_S2D_NT=1)
      else *p = w;
#endif
    }
  };
  // planes mode: per wave a 64-column group (both 32-column tiles of a column-bit-5 pair) and 32
  // output rows at a time, computed transposed (D^T[c][r]: lane = row rt + (lane & 31), registers =
  // columns (e & 3) + 8 (e >> 2) + 4 fk); a permlane32 swap per register pair leaves every lane two
  // runs of 8 consecutive columns per tile, split into the six f16 planes and stored 16 B per
  // plane and run.  The dense op's output rows are consecutive 64-element runs of the operand
  // (out_off = 64 r), so a wave's 32 x 64 tile is 4 KiB of each plane, written whole by the 4
  // store instructions of that plane (both column tiles' runs are emitted per plane: writing one
  // tile's halves of all rows first left half-written lines and ran 2.5x slower)
  // the planes' base and stride as locals: read through `op` (the kernel-argument block, not
  // provably unaliased by the stores) they were re-loaded by scalar loads inside the store loop
  _Float16* const Pl = reinterpret_cast<_Float16*>(op.planes);
  const int64_t pstride = op.pstride;
  auto emit_planes = [&](f32x16 (&d)[2][2], int64_t gbase, int rt) {
#pragma unroll
    for (int tl = 0; tl < 2; ++tl)
#pragma unroll
      for (int ri = 0; ri < 2; ++ri)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int a = 8 * h + i, b = 8 * h + 4 + i;
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(d[tl][ri][a]), __float_as_uint(d[tl][ri][b]), false, false);
            d[tl][ri][a] = __uint_as_float(sw[0]);
            d[tl][ri][b] = __uint_as_float(sw[1]);
          }
    {
      // each lane stores its own four 16-B runs per plane: a store instruction covers 32 rows x
      // 32 contiguous bytes, and the plane's 4 instructions fill the wave's 4 KiB (32 rows x
      // 128 B) of that plane back to back (an LDS-staged form storing 8 whole rows per
      // instruction measured the same)
      const int64_t rb = gbase + ooff[rt + fr] + 8 * fk;
#pragma unroll
      for (int pl = 0; pl < 6; ++pl)
#pragma unroll
        for (int tl = 0; tl < 2; ++tl)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            uint32_t w4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int e0 = 8 * h + 2 * j;
              const f2v re = {d[tl][0][e0], d[tl][0][e0 + 1]}, im = {d[tl][1][e0], d[tl][1][e0 + 1]};
              f2v t;
#if TQ_S2D_DIAG == 3
              t = (pl & 2) ? im : re;   // development diagnostic: no split
#else
              if (pl < 2) t = f16_terms_scaled(re);
              else if (pl < 4) t = f16_terms_scaled(im);
              else t = f16_terms_scaled((re + im) * 0.5f);   // one binade lower (exact)
#endif
              w4[j] = __float_as_uint((pl & 1) ? t.y : t.x);
            }
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4* dst = reinterpret_cast<u32x4*>(Pl + pl * pstride + rb + 32 * tl + 16 * h);
            const u32x4 v = {w4[0], w4[1], w4[2], w4[3]};
#if TQ_S2D_DIAG == 2
            if (w4[0] == 12345u) *dst = v;   // development diagnostic: no stores
#else
            if constexpr (NTS) __builtin_nontemporal_store(v, dst);
            else *dst = v;
#endif
          }
    }
  };
  // tile order: grid-strided (default: concurrently running workgroups write neighbouring 1-KiB
  // pieces of the same output rows) or blocked (op.order == 1, TQ_S2D_BLOCKED=1: each workgroup
  // walks its own contiguous range of tiles, i.e. whole runs of one row set)
  const int64_t blk = (int)blockIdx.x - op.block_begin;
  int64_t t0 = blk * kWaves + wave, t_end = ntiles, t_step = nw;
  if (op.order == 1) {
    const int64_t per = ((ntiles + op.nblocks - 1) / op.nblocks + kWaves - 1) / kWaves * kWaves;
    t0 = blk * per + wave;
    t_end = ntiles < (blk + 1) * per ? ntiles : (blk + 1) * per;
    t_step = kWaves;
  }
  if (planes) {
    // 64-column groups (column bits 0..5), the same products with the operands swapped (the
    // transposed tile: columns in registers)
    const int64_t ngroups = ntiles >> 1;
    int64_t g_0 = (int64_t)blk * kWaves + wave, g_end = ngroups, g_step = nw;
    if (op.order == 1) {   // blocked: each wave its own contiguous range of groups
      const int64_t per = (ngroups + nw - 1) / nw;
      g_0 = ((int64_t)blk * kWaves + wave) * per;
      g_end = ngroups < g_0 + per ? ngroups : g_0 + per;
      g_step = 1;
    }
    // The group's inputs arrive by LDS-DMA into the wave's slot, issued at the previous group's
    // start (right after that group's inputs left the slot): the group waits with vmcnt(N), N the
    // stores issued after the DMA (up to 63), not vmcnt(0) -- a register load at the group start
    // waited for every store the wave had in flight and then for the load itself behind the
    // saturated write stream (probes/planes_store_probe.hip: 1.69 -> 1.45 ms for the launch's
    // store pattern with its reads, issued without waits)
    const uint32_t slot = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&sm.xs[wave][0]);
    const char* const Xb = reinterpret_cast<const char*>(op.X);
    // SGPR base (the group's column base, uniform) + a 32-bit lane byte offset per instruction
    // (loop invariant): no 64-bit address VGPRs in the group loop
    uint32_t doff[KS];
#pragma unroll
    for (int i = 0; i < KS; ++i) doff[i] = (uint32_t)((io[i] + 2 * fr) * 8);
    auto dma = [&](int64_t g) {   // X[k][64 columns of group g] -> slot, KS x 1 KiB
      const int64_t bi = base(0, g);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bi), hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)bi >> 32));
      const char* const gbase = Xb + (int64_t)(((uint64_t)hi << 32) | lo) * 8;
#pragma unroll
      for (int i = 0; i < KS; ++i) {
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(doff[i]), "s"(gbase), "s"(slot + 1024u * i) : "memory");
      }
    };
    const int nrt = tout / 32;
    if (g_0 < g_end) {
      dma(g_0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (int64_t g = g_0; g < g_end; g += g_step) {
      float xr[2][KS], xi[2][KS];
      {
        const float2* xsl = sm.xs[wave];
#pragma unroll
        for (int tl = 0; tl < 2; ++tl)
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const float2 v = xsl[(2 * s + fk) * 64 + 32 * tl + fr];
            xr[tl][s] = ldexpf(v.x, xsc);
            xi[tl][s] = ldexpf(v.y, xsc);
          }
      }
      // every lane's reads of the slot are complete before the next DMA overwrites it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // (unconditional: the last group re-reads its own inputs -- a branch here doubled the
      // kernel's registers)
      const bool more = g + g_step < g_end;
      dma(more ? g + g_step : g);
      const int64_t gb = base(1, g);
#pragma unroll 1
      for (int rt = 0; rt < tout; rt += 32) {
        f32x16 d[2][2];
#pragma unroll
        for (int tl = 0; tl < 2; ++tl) {
          f32x16 p1 = {}, p2 = {}, p3 = {};
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const int a = (2 * s + fk) * tout + rt + fr;
            const float mr = mp[0][a], mi = mp[1][a];
#if TQ_S2D_DIAG == 1 || TQ_S2D_DIAG == 3
            p1[s] = xr[tl][s] * mr;   // development diagnostics: no MFMAs
            p2[s] = xi[tl][s] * mi;
            p3[s] = mr + mi;
            continue;
#endif
            p1 = __builtin_amdgcn_mfma_f32_32x32x2f32(xr[tl][s], mr, p1, 0, 0, 0);
            p2 = __builtin_amdgcn_mfma_f32_32x32x2f32(xi[tl][s], mi, p2, 0, 0, 0);
            p3 = __builtin_amdgcn_mfma_f32_32x32x2f32(xr[tl][s] + xi[tl][s], mr + mi, p3, 0, 0, 0);
          }
          d[tl][0] = p1 - p2;
          d[tl][1] = p3 - p1 - p2;
        }
        emit_planes(d, gb, rt);
      }
      // the next group's DMA is older than this group's 24 x nrt stores: all but the most recent
      // min(63, 24 nrt) operations complete => the DMA has landed
      if (nrt >= 3) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
      else if (nrt == 2) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    }
    return;
  }
  for (int64_t t = t0; t < t_end; t += t_step) {
    // column tile t: columns 32t .. 32t+31 (bits 0..4 = lane, bit 5 = t & 1, bits >= 6: tables)
    const int64_t g = t >> 1;
    const int cl = (int)(t & 1) * 32 + fr;
    const int64_t bi = base(0, g);
    float xr[KS], xi[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const f2v v = X[bi + io[s] + cl];
      xr[s] = v.x;
      xi[s] = v.y;
    }
    const f2v* Yt = Y + (base(1, g) + (cl & ~1));   // a lane pair stores columns (cl & ~1), +1
    // one 32-output tile per iteration; Gauss's 3M product (three accumulator sets)
    for (int rt = 0; rt < tout; rt += 32) {
      f32x16 p1 = {}, p2 = {}, p3 = {};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#if TQ_S2D_DIAG == 1 || TQ_S2D_DIAG == 3
        break;   // development diagnostics: no MFMAs
#endif
        const int a = (2 * s + fk) * tout + rt + fr;
        const float mr = mp[0][a], mi = mp[1][a];
        p1 = __builtin_amdgcn_mfma_f32_32x32x2f32(mr, xr[s], p1, 0, 0, 0);
        p2 = __builtin_amdgcn_mfma_f32_32x32x2f32(mi, xi[s], p2, 0, 0, 0);
        p3 = __builtin_amdgcn_mfma_f32_32x32x2f32(mr + mi, xr[s] + xi[s], p3, 0, 0, 0);
      }
      emit(p1 - p2, p3 - p1 - p2, Yt, rt);
    }
  }
  if (track) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
    if (lane == 0 &&   // only when it raises the word (same-address atomics serialise: tq_sweep2.hip)
        __float_as_uint(vmax) > __hip_atomic_load(op.amax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(op.amax, __float_as_uint(vmax));
  }
}

// TB == 0: every op of the launch has input tile TA; else each op has TA or TB (one dependency
// level's dense ops of both subtrees of a cut network in one launch: their tails overlap)
template <int TA, int TB, bool NTS>
#ifndef TQ_S2D_OCC
#define TQ_S2D_OCC 2
#endif
__global__ void __launch_bounds__(64 * kWaves, TQ_S2D_OCC) sweepd_kernel(S2DLaunch L) {
  constexpr int TMAX = TA > TB ? TA : TB;
  __shared__ SdSmem<TMAX> sm;
  int j = 0;
  for (int q = 1; q < L.nops; ++q)
    if ((int)blockIdx.x >= L.op[q].block_begin) j = q;
  const S2DOp& op = L.op[j];
  if constexpr (TB == 0) {
    sweepd_op<TA, NTS, TMAX>(op, sm);
  } else {
    if (op.tin == TA) sweepd_op<TA, NTS, TMAX>(op, sm);
    else sweepd_op<TB, NTS, TMAX>(op, sm);
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
  // at most two input tile sizes per launch (ta > tb; tb = 0: one)
  int ta = L.op[0].tin, tb = 0;
  for (int q = 0; q < L.nops; ++q) {
    const int t = L.op[q].tin;
    if (t != ta && t != tb) {
      if (tb != 0) {
        set_error("sweepd: at most two input tile sizes per launch");
        return TQ_ERR_INVALID;
      }
      tb = t;
    }
    // the kernel stores whole 32-output tiles and stages at most kS2DMaxTout offsets
    if (L.op[q].tout < 32 || L.op[q].tout % 32 || L.op[q].tout > kS2DMaxTout || !L.op[q].desc || !L.op[q].M) {
      set_error("sweepd: bad output tile");
      return TQ_ERR_INVALID;
    }
  }
  // one round of resident workgroups over the launch's ops (the kernel strides over its tiles):
  // a second, partial round of workgroups left most CUs idle (1024 blocks on 768 slots)
  static const bool nts = [] {
    const char* e = getenv("TQ_S2D_NT");
    return e && e[0] == '1';
  }();
  static const int order = [] {
    const char* e = getenv("TQ_S2D_BLOCKED");
    return e && e[0] == '1' ? 1 : 0;
  }();
  if (tb > ta) std::swap(ta, tb);
  auto pow2tin = [](int t) { return t == 2 || t == 4 || t == 8 || t == 16; };
  if (!pow2tin(ta) || (tb && !pow2tin(tb))) {
    set_error("sweepd: tin must be 2, 4, 8 or 16");
    return TQ_ERR_INVALID;
  }
  if (tb && nts) {
    set_error("sweepd: mixed input tile sizes only with plain stores");
    return TQ_ERR_INVALID;
  }
  const void* fn = nullptr;
#define TQ_SD_FN(T) (nts ? reinterpret_cast<const void*>(&sweepd_kernel<T, 0, true>) \
                         : reinterpret_cast<const void*>(&sweepd_kernel<T, 0, false>))
#define TQ_SD_MIX(A, B) reinterpret_cast<const void*>(&sweepd_kernel<A, B, false>)
  switch (ta * 32 + tb) {
    case 2 * 32: fn = TQ_SD_FN(2); break;
    case 4 * 32: fn = TQ_SD_FN(4); break;
    case 8 * 32: fn = TQ_SD_FN(8); break;
    case 16 * 32: fn = TQ_SD_FN(16); break;
    case 4 * 32 + 2: fn = TQ_SD_MIX(4, 2); break;
    case 8 * 32 + 2: fn = TQ_SD_MIX(8, 2); break;
    case 8 * 32 + 4: fn = TQ_SD_MIX(8, 4); break;
    case 16 * 32 + 2: fn = TQ_SD_MIX(16, 2); break;
    case 16 * 32 + 4: fn = TQ_SD_MIX(16, 4); break;
    case 16 * 32 + 8: fn = TQ_SD_MIX(16, 8); break;
    default: break;
  }
#undef TQ_SD_FN
#undef TQ_SD_MIX
  // resident workgroups of this instantiation on the current device (cached per device)
  static DeviceCache<(kS2DMaxTin + 1) * 32> slot_cache;
  const int key = ta * 32 + tb;
  const int slots = slot_cache.get(key, [&] {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 64 * kWaves, 0) != hipSuccess)
      return 256;
    return std::max(1, cus * std::max(1, per));
  });
  S2DLaunch R = L;
  // the round of resident workgroups shared by the ops in proportion to their output: the ops are
  // bound by their store streams, not their products (C4's tin-16 and tin-8 ops store the same
  // bytes; shared by products (8 + tin), the tin-8 ops' workgroups finished last: 1.67 vs 1.48 ms
  // per launch on one box), plus 16 rows' worth per column for the per-column-group work (input
  // loads, bases: 1.45 ms; 48: 1.48, -16: 1.51)
  // (TQ_S2D_SHARE=0: by products, the r04 rule, for A/B)
  static const bool by_products = [] {
    const char* e = getenv("TQ_S2D_SHARE");
    return e && e[0] == '0';
  }();
  auto work = [&](const S2DOp& o) {
    const double c = (double)std::max<int64_t>(o.ncols, 1);
    return by_products ? c * o.tout * (8.0 + o.tin) : c * (o.tout + 16.0);
  };
  double wsum = 0;
  for (int q = 0; q < R.nops; ++q) wsum += work(R.op[q]);
  int blocks = 0;
  for (int q = 0; q < R.nops; ++q) {
    const double wq = work(R.op[q]);
    const int want = std::max(1, (int)((double)slots * wq / wsum));
    R.op[q].nblocks = std::max(1, std::min(R.op[q].nblocks, want));
    R.op[q].block_begin = blocks;
    R.op[q].order = order;
    blocks += R.op[q].nblocks;
  }
  hipLaunchKernelGGL(reinterpret_cast<void (*)(S2DLaunch)>(const_cast<void*>(fn)), dim3(blocks), dim3(64 * kWaves), 0,
                     stream, R);
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

}  // namespace tq
