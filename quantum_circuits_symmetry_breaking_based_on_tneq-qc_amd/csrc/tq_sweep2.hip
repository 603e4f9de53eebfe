// In-place butterfly sweep: a chain of small-operand absorptions in ONE HBM pass, several
// independent chains per launch.
//
// The contraction trees of the amplitude workloads (each
// opt_einsum pairwise step at einsum_strategy.py:639-643 absorbs one (2,2,2,2) gate, or a
// gate with an input state / output projector folded in, into a running tensor) are long
// chains of steps that each touch a few legs.  For chains whose modes all have power-of-two
// extents the plan compiler (tq_plan.cpp) gives every mode bit of the working set a fixed
// position bit of a tile index; a gate with K inputs and N outputs then works on disjoint
// groups (one assignment of the positions it does not touch): read K tile elements, write N —
// outputs take the positions the gate frees, so the tile is updated in place and every gate
// costs one LDS read + one LDS write per element (the table-driven sweep costs K reads).
//
// A workgroup owns chunks of C columns (assignments of the untouched modes) x the tile; the
// LDS image of element (position p, column c) is p*C + (c ^ swz(p)) with a per-op linear XOR
// swizzle chosen at plan time, so the gate passes (32 consecutive columns per half-wave) and
// the load / store phases (elements enumerated in memory order: every half-wave touches 256
// contiguous bytes when the tensor allows it) are LDS-bank-conflict free.  The next chunk's
// loads are issued into registers before the current chunk's stores.  Independent ops (the
// two subtrees of a cut network, the tiny vector pre-absorption chains) share one launch:
// blockIdx ranges select the op.
//
// Latency: the op descriptor is copied to LDS by one coalesced pass at kernel start (no chains
// of dependent scalar loads), gate passes are instantiated per exact (K, N) (powers of two
// K <= 4, N <= 8: no predication in the inner loop), the gate coefficients are staged once per
// workgroup in LDS (and held in registers for small gates), and complex64 products use packed
// FP32 FMAs (v_pk_fma_f32: 2 instead of 4 FMAs per complex multiply-add).  At most 128 VGPRs
// per lane (launch bound), so two 512-thread workgroups share a CU.
// Algorithmic bytes per op = (numel(X) + numel(Y)) * sizeof.
#include <algorithm>
#include <type_traits>

#include "tq_common.h"
#include "tq_sweep2.h"
#include "tq_kclock.h"

namespace tq {

namespace {

TQ_KCLOCK_DEFINE(g_kclk_sweep2)

constexpr int NT = 512, LOG_NT = 9;
// the pass-barrier elision (kS2PmSync) assumes gi == threadIdx.x (mod NT) in gate_pass_u and
// block_pass and 64-lane waves: wave = gi bits [kS2WaveBits, kS2LogThreads)
static_assert(NT == (1 << kS2LogThreads) && LOG_NT == kS2LogThreads, "sweep2 thread count vs the planner's");
static_assert(kS2WaveBits == 6 && kS2LogThreads > kS2WaveBits, "wave-select group bits");
constexpr int kLut = 64;                     // per-gate group tables: 32 entries for the low 5 pass bits,
                                             // 32 for the high ones (<= 9 pass positions)
constexpr int kCf = kS2MaxK * kS2MaxKN;      // coefficient slots per gate
// per-gate fields the gate passes read, staged in LDS: read in every pass of every chunk, they
// must not queue behind the chunk's HBM stores (descriptor loads are vector loads)
constexpr int kGmK = kS2GmK, kGmN = kS2GmN, kGmPass = kS2GmPass, kGmKaddr = kS2GmKaddr,
              kGmNaddr = kS2GmNaddr;
constexpr int kGm = 16;
constexpr int kDescWords2 = kS2DescHotBytes / 8;   // the kernel-read part of S2Desc
constexpr int kKeepWords2 = kS2KeepOff / 8;        // words before S2Desc::k (-> tile buffer)

static_assert(kGmNaddr + kS2MaxKN <= kGm, "gate meta layout");
static_assert(kLut == 64, "lut layout shared with S2Desc::lut");

#if defined(TQ_S2_DIAG) && TQ_S2_DIAG == 2
// development diagnostic: no HBM stores (a runtime condition that never holds keeps the work)
#define TQ_ST(p, v) do { if (use_beta == 12345) *(p) = (v); } while (0)
#else
#define TQ_ST(p, v) (*(p) = (v))
#endif

#ifdef TQ_S2_TIMING
// development instrumentation (built only with -DTQ_S2_TIMING): workgroup 0 of every op records
// wall-clock stamps (100 MHz) at its phase boundaries
// record: [0..6] phase stamps, [7] blocks|chunks, [8] first chunk's gate clocks,
// [9..24] clock at the end of each pass of the first chunk, [25..40] pass kind (B<<16|K<<8|N)
constexpr int kTsMax = 2048, kTsPh = 48;   // [41..47]: sub-stamps of the tables phase
__device__ unsigned long long g_s2_ts[kTsMax][kTsPh];
__device__ unsigned int g_s2_seq;
#define TQ_TS(ph) do { if (ts_rec && threadIdx.x == 0) g_s2_ts[ts_idx][ph] = wall_clock64(); } while (0)
#else
#define TQ_TS(ph) do {} while (0)
#endif

template <typename T>
__device__ __forceinline__ T scale_add(T v, T y, double beta) {
  if constexpr (sizeof(typename Traits<T>::R) == 4) return v + y * (float)beta;
  else return v + y * beta;
}

typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// f16 terms of v * 2^sc (S2Op::split_sc; the consuming GEMM's xbf::SplitPre): h = f16(xs) (round
// to nearest), l = f16(xs - h) (xs - h exact in f32, read from the packed halves by
// v_fma_mix_f32); the element's 8 bytes become (h_re, h_im | l_re, l_im)
__device__ __forceinline__ c64 f16_terms(c64 v, int sc) {
  const float x0 = ldexpf(v.re, sc), x1 = ldexpf(v.im, sc);
  const f16x2 hv = {(_Float16)x0, (_Float16)x1};
  const uint32_t h = __builtin_bit_cast(uint32_t, hv);
  float r0, r1;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r0) : "v"(x0), "v"(h));
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r1) : "v"(x1), "v"(h));
  const f16x2 lv = {(_Float16)r0, (_Float16)r1};
  return c64{__uint_as_float(h), __uint_as_float(__builtin_bit_cast(uint32_t, lv))};
}

// uniform base + zero-extended 32-bit lane byte offset: global_load/store with an SGPR-pair base
// and one VGPR offset shared by every register slot (no 64-bit VGPR address per slot)
template <typename T>
__device__ __forceinline__ T* lane_at(T* base, uint32_t byte_off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + byte_off);
}
template <typename T>
__device__ __forceinline__ const T* lane_at(const T* base, uint32_t byte_off) {
  return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}

// Cooperative chain ops (S2Launch::sync): a tensor one workgroup stores and another loads in the
// same launch moves through vector buffer accesses with the sc1 policy (write-through stores,
// L1-bypassing loads, coherent across the XCDs' L2s), one element per lane -- the hand-off form the
// MI355X guide measures valid with a counter between them (stores drained by every wave, a
// workgroup barrier, one agent-scope add; one polling lane, a barrier, then the loads).
// `base` is wave-uniform (the buffer descriptor is built in scalar registers), `off` the lane's
// byte offset.
constexpr int kSc1 = 16;   // cache-policy bits of a buffer access: sc1
template <typename W>
__device__ __forceinline__ W ld_coherent(const void* base, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
  if constexpr (sizeof(W) == 16) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1);
    return __builtin_bit_cast(W, v);
  } else if constexpr (sizeof(W) == 8) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kSc1);
    return __builtin_bit_cast(W, v);
  } else {
    static_assert(sizeof(W) == 4, "4-, 8- or 16-byte elements");
    const auto v = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kSc1);
    return __builtin_bit_cast(W, v);
  }
}
template <typename W>
__device__ __forceinline__ void st_coherent(void* base, uint32_t off, const W& w) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, -1, 0x00020000);
  if constexpr (sizeof(W) == 16) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(int __attribute__((ext_vector_type(4))), w), r, off, 0,
                                           kSc1);
  } else if constexpr (sizeof(W) == 8) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(int __attribute__((ext_vector_type(2))), w), r, off, 0,
                                          kSc1);
  } else {
    static_assert(sizeof(W) == 4, "4-, 8- or 16-byte elements");
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, w), r, off, 0, kSc1);
  }
}
// bounded polls of a cooperative chain's counter (~1 s): a lost arrival cannot hang the GPU
constexpr int kCoopSpin = 1 << 20;

// acc += a * b on packed f32: (a.re, a.re) * (b.re, b.im) + (a.im, a.im) * (-b.im, b.re).
// The broadcasts and the swap / negation are operand modifiers (op_sel / neg), not copies.
__device__ __forceinline__ f2v pmac(f2v acc, f2v a, f2v b) {
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "+v"(acc) : "v"(a), "v"(b));
  return acc;
}

// a * b on packed f32 (the first product of a sum: no zeroed accumulator to initialise)
__device__ __forceinline__ f2v pmul(f2v a, f2v b) {
  f2v acc;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(acc) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "+v"(acc) : "v"(a), "v"(b));
  return acc;
}

template <typename T>
__device__ __forceinline__ T mul(const T& a, const T& b) {
#if defined(TQ_S2_DIAG) && TQ_S2_DIAG == 1
  (void)b;
  return a;
#endif
  if constexpr (std::is_same<T, c64>::value) {
    const f2v r = pmul(f2v{a.re, a.im}, f2v{b.re, b.im});
    return c64{r.x, r.y};
  } else {
    T acc = tzero<T>();
    cmac(acc, a, b);
    return acc;
  }
}

template <typename T>
__device__ __forceinline__ void mac(T& acc, const T& a, const T& b) {
#if defined(TQ_S2_DIAG) && TQ_S2_DIAG == 1
  // development diagnostic: no arithmetic (the data movement of every pass stays)
  (void)b;
  acc = a;
  return;
#endif
  if constexpr (std::is_same<T, c64>::value) {
    const f2v r = pmac(f2v{acc.re, acc.im}, f2v{a.re, a.im}, f2v{b.re, b.im});
    acc = c64{r.x, r.y};
  } else {
    cmac(acc, a, b);
  }
}

// A pass's head (S2Keep::pmeta row, wave-uniform, in scalar registers): everything a pass needs
// before its element addresses.  One batch of LDS reads, issued together with the pass's group
// table reads (rows by pass), so a pass is head + table -> elements -> barrier: two dependent
// LDS round trips where it was four (r04: ~2600 clocks per pass on tiny chunks -- pass row, gate
// row, group table, elements, and the barrier).
struct PassHead {
  int32_t w[16];   // pmeta row: first gate, count (| K*16+N << 8 for a single gate), B, pass mask, ...
};

// One gate over all groups of the chunk.  Every LDS address is an XOR of contributions:
// group (lut[pp] ^ c) ^ input k (kaddr[k]) / output n (naddr[n]).  U groups per thread in
// flight; all K inputs of a group are read before any of its N outputs is written (outputs
// reuse the input positions).
template <typename T, int K, int N, int U>
__device__ __forceinline__ void gate_pass_u(T* __restrict__ buf, const T* __restrict__ cf, const PassHead& h,
                                            const int32_t* __restrict__ lut, int logC) {
  // coefficients held in registers (up to 32 VGPRs for FP32 data, 16 for FP64); larger gates
  // re-read them from LDS per group
  constexpr bool kReg = K * N * sizeof(T) <= (sizeof(typename Traits<T>::R) == 4 ? 128 : 64);
  constexpr int SH = sizeof(T) == 4 ? 2 : sizeof(T) == 8 ? 3 : 4;   // element -> byte offset
  char* const bb = reinterpret_cast<char*>(buf);
  const int tid = threadIdx.x;
  static_assert(U <= 4, "head group slots");
  const int ngroups = (1 << logC) << __popc((uint32_t)h.w[kS2PmPass]);
  const int cmb = ((1 << logC) - 1) << SH;
  int ka[K], na[N];   // byte offsets (the LUT entries are staged as byte offsets too)
#pragma unroll
  for (int k = 0; k < K; ++k) ka[k] = h.w[kS2PmAddr + k] << SH;
#pragma unroll
  for (int n = 0; n < N; ++n) na[n] = h.w[kS2PmCode + n] << SH;
  T creg[kReg ? K * N : 1];
  if constexpr (kReg) {
#pragma unroll
    for (int i = 0; i < K * N; ++i) creg[i] = cf[i];
  }
  for (int g0 = tid; g0 < ngroups; g0 += U * NT) {
    // keeps the compiler from hoisting the (loop-invariant) LDS coefficient reads of large gates
    // out of the loop, which would pin K*N coefficients in registers
    if constexpr (!kReg) asm volatile("" ::: "memory");
    int a0[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int gi = g0 + u * NT;
      ok[u] = gi < ngroups;
      gi = ok[u] ? gi : g0;
      const int gp = gi >> logC;
      a0[u] = lut[gp & 31] ^ lut[32 + (gp >> 5)] ^ ((gi << SH) & cmb);
    }
    T x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < K; ++k) x[u][k] = *reinterpret_cast<const T*>(bb + (a0[u] ^ ka[k]));
#pragma unroll
    for (int n = 0; n < N; ++n) {
      T c[K];
      if constexpr (kReg) {
#pragma unroll
        for (int k = 0; k < K; ++k) c[k] = creg[k * N + n];
      } else {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < K; ++k) c[k] = cf[k * N + n];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        T acc = mul(x[u][0], c[0]);
#pragma unroll
        for (int k = 1; k < K; ++k) mac(acc, x[u][k], c[k]);
        if (ok[u]) *reinterpret_cast<T*>(bb + (a0[u] ^ na[n])) = acc;
      }
    }
  }
}

// U groups per thread in flight; a chunk of at most one group per thread (the small tiles: C2's
// 2048-element chunks under a 4x4 gate, 512 groups) runs the one-group form -- the U-wide one
// computed U - 1 duplicate groups there, half or more of the pass's VALU (r04 probe,
// probes/pass_probe.hip: a 4x4 pass over 2048 elements is VALU-issue bound at ~1000 clocks with
// one group per thread)
template <typename T, int K, int N>
__device__ __forceinline__ void gate_pass(T* __restrict__ buf, const T* __restrict__ cf, const PassHead& h,
                                          const int32_t* __restrict__ lut, int logC) {
  constexpr int U = sizeof(T) > 8 ? (K * N >= 8 ? 1 : 2) : (K * N >= 16 ? 2 : 4);
  if constexpr (U > 1) {
    const int ngroups = (1 << logC) << __popc((uint32_t)h.w[kS2PmPass]);
    if (ngroups <= NT) {
      gate_pass_u<T, K, N, 1>(buf, cf, h, lut, logC);
      return;
    }
    if constexpr (U > 2) {
      if (ngroups <= 2 * NT) {
        gate_pass_u<T, K, N, 2>(buf, cf, h, lut, logC);
        return;
      }
    }
  }
  gate_pass_u<T, K, N, U>(buf, cf, h, lut, logC);
}

// ---- register blocks (S2Desc::pmeta): a run of square gates applied to 2^B elements per group
// held in registers.  Block bit b of element e is bit b of e; a gate's index bits 0 / 1 sit on
// block bits I / J (compile-time, one instantiation per placement).
template <int B, int I, int J>
__device__ __forceinline__ constexpr int deposit2(int r) {
  // bits of r into the block bits other than I and J, ascending
  int v = 0, t = 0;
  for (int b = 0; b < B; ++b) {
    if (b == I || b == J) continue;
    v |= ((r >> t) & 1) << b;
    ++t;
  }
  return v;
}

// wave-uniform value -> scalar registers (the block passes keep their VGPRs for the elements)
template <typename T>
__device__ __forceinline__ T uniform(T v) {
  static_assert(sizeof(T) % 4 == 0, "dword granularity");
  union { T t; int w[sizeof(T) / 4]; } u;
  u.t = v;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) u.w[i] = __builtin_amdgcn_readfirstlane(u.w[i]);
  return u.t;
}

// Coefficients are wave-uniform.  complex64: read from LDS at a uniform address straight into
// VGPRs (broadcast) -- the packed FMAs take VGPR operands only, so scalar copies (readfirstlane)
// would be moved back into VGPRs before every use, 2 extra VALU instructions per dword.  Other
// types: scalar registers (the FMAs read them directly; VGPRs are what the 16-element blocks
// need).
template <typename T>
__device__ __forceinline__ T coef(const T* cf, int i) {
  if constexpr (std::is_same<T, c64>::value) return cf[i];
  else return uniform(cf[i]);
}
template <typename T, int B, int I, int J>
__device__ __forceinline__ void blk_apply4(T (&x)[1 << B], const T* __restrict__ cf) {
  T c[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) c[i] = coef(cf, i);
#pragma unroll
  for (int r = 0; r < (1 << (B - 2)); ++r) {
    const int base = deposit2<B, I, J>(r);
    T in[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) in[k] = x[base | ((k & 1) << I) | ((k >> 1) << J)];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      T acc = mul(in[0], c[n]);
#pragma unroll
      for (int k = 1; k < 4; ++k) mac(acc, in[k], c[k * 4 + n]);
      x[base | ((n & 1) << I) | ((n >> 1) << J)] = acc;
    }
  }
}

template <typename T, int B, int I>
__device__ __forceinline__ void blk_apply2(T (&x)[1 << B], const T* __restrict__ cf) {
  T c[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = coef(cf, i);
#pragma unroll
  for (int r = 0; r < (1 << (B - 1)); ++r) {
    const int base = deposit2<B, I, I>(r) ;
    const T a = x[base], b = x[base | (1 << I)];
    T y0 = mul(a, c[0]), y1 = mul(a, c[1]);
    mac(y0, b, c[2]);
    mac(y1, b, c[3]);
    x[base] = y0;
    x[base | (1 << I)] = y1;
  }
}

template <typename T, int B>
__device__ __forceinline__ void blk_gate(T (&x)[1 << B], const T* cf, int code) {
#define TQ_B4(i, j) case 16 | (j << 2) | i: blk_apply4<T, B, i, j>(x, cf); break;
#define TQ_B2(i) case i: blk_apply2<T, B, i>(x, cf); break;
  // the plan compiler emits I < J only (it swaps a gate's legs otherwise): 6 / 3 bodies
  if constexpr (B == 4) {
    switch (code) {
      TQ_B4(0, 1) TQ_B4(0, 2) TQ_B4(0, 3) TQ_B4(1, 2) TQ_B4(1, 3) TQ_B4(2, 3)
      TQ_B2(0) TQ_B2(1) TQ_B2(2) TQ_B2(3)
      default: break;
    }
  } else {
    switch (code) {
      TQ_B4(0, 1) TQ_B4(0, 2) TQ_B4(1, 2)
      TQ_B2(0) TQ_B2(1) TQ_B2(2)
      default: break;
    }
  }
#undef TQ_B4
#undef TQ_B2
}

// A lane block's swap (code kS2SwapCode | L << 2 | r): register bit r and lane bit 4 (L = 0) or 5
// (L = 1) trade positions.  For every element pair (e, e | 1 << r) the pair's values transpose
// across the two lane halves -- v_permlane16_swap (rows of 16 lanes) / v_permlane32_swap (halves
// of the wave) on each dword: the value at (lane l, bit r = v) becomes the value that was at
// (lane bit := v, bit r := lane bit of l)
template <typename T, int B, int R, bool L5>
__device__ __forceinline__ void blk_swap_rl(T (&x)[1 << B]) {
  static_assert(sizeof(T) % 4 == 0, "dword elements");
  constexpr int W = (int)(sizeof(T) / 4);
#pragma unroll
  for (int e = 0; e < (1 << B); ++e) {
    if ((e >> R) & 1) continue;
    union U { T t; uint32_t w[W]; } lo, hi;
    lo.t = x[e];
    hi.t = x[e | (1 << R)];
#pragma unroll
    for (int i = 0; i < W; ++i) {
      const auto r = L5 ? __builtin_amdgcn_permlane32_swap(lo.w[i], hi.w[i], false, false)
                        : __builtin_amdgcn_permlane16_swap(lo.w[i], hi.w[i], false, false);
      lo.w[i] = r[0];
      hi.w[i] = r[1];
    }
    x[e] = lo.t;
    x[e | (1 << R)] = hi.t;
  }
}

template <typename T>
__device__ __forceinline__ void blk_swap(T (&x)[16], int code) {
  switch (code & 7) {
    case 0: blk_swap_rl<T, 4, 0, false>(x); break;
    case 1: blk_swap_rl<T, 4, 1, false>(x); break;
    case 2: blk_swap_rl<T, 4, 2, false>(x); break;
    case 3: blk_swap_rl<T, 4, 3, false>(x); break;
    case 4: blk_swap_rl<T, 4, 0, true>(x); break;
    case 5: blk_swap_rl<T, 4, 1, true>(x); break;
    case 6: blk_swap_rl<T, 4, 2, true>(x); break;
    default: blk_swap_rl<T, 4, 3, true>(x); break;
  }
}

template <typename T, int B>
__device__ __forceinline__ void block_pass(T* __restrict__ buf, const T* __restrict__ cf_all, const PassHead& h,
                                           const int32_t* __restrict__ pml, const int32_t* __restrict__ lut,
                                           int logC) {
  constexpr int E = 1 << B;
  constexpr int SH = sizeof(T) == 4 ? 2 : sizeof(T) == 8 ? 3 : 4;
  char* const bb = reinterpret_cast<char*>(buf);
  const int32_t* const pm = h.w;   // constant indices only (a register copy); codes from pml (LDS)
  const int ngroups = (1 << logC) << __popc((uint32_t)pm[kS2PmPass]);
  const int cmb = ((1 << logC) - 1) << SH;
  // block-bit address parts are wave-uniform: scalar registers, element offsets formed by SALU
  int ba[B];
#pragma unroll
  for (int b = 0; b < B; ++b) ba[b] = pm[kS2PmAddr + b] << SH;
  auto off = [&](int e) {
    int o = 0;
#pragma unroll
    for (int b = 0; b < B; ++b)
      if ((e >> b) & 1) o ^= ba[b];
    return o;
  };
  const int first = pm[kS2PmFirst], cnt = pm[kS2PmCount] & 0xff;
  const bool lanes = (pm[kS2PmB] & kS2PmLanes) != 0;
  for (int g0 = threadIdx.x; g0 < ngroups; g0 += NT) {
    const int gp = g0 >> logC;
    int a0 = lut[gp & 31] ^ lut[32 + (gp >> 5)] ^ ((g0 << SH) & cmb);
    T x[E];
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = *reinterpret_cast<const T*>(bb + (a0 ^ off(e)));
    // the element addresses are recomputed for the write-back (not held across the gates)
    asm volatile("" : "+v"(a0));
    // gates (and a lane block's swaps; the gate row advances on gates only)
    int gq = first;
    for (int q = 0; q < cnt; ++q) {
      const int code = pml[kS2PmCode + q];
      if constexpr (B == 4) {
        if (code & kS2SwapCode) {
          blk_swap<T>(x, code);
          continue;
        }
      }
      blk_gate<T, B>(x, cf_all + gq * kCf, code);
      ++gq;
    }
    // write-back in the end layout (S2Keep::pmeta [16, 22): a plain block's is its start layout)
    int be[B];
#pragma unroll
    for (int b = 0; b < B; ++b) be[b] = ba[b];
    int aw = a0;
    if (lanes) {
#pragma unroll
      for (int b = 0; b < B; ++b) be[b] = __builtin_amdgcn_readfirstlane(pml[kS2PmAddrEnd + b]) << SH;
      const int d4 = __builtin_amdgcn_readfirstlane(pml[kS2PmLaneDelta]) << SH;
      const int d5 = __builtin_amdgcn_readfirstlane(pml[kS2PmLaneDelta + 1]) << SH;
      const int lane = threadIdx.x & 63;
      aw ^= ((lane & 16) ? d4 : 0) ^ ((lane & 32) ? d5 : 0);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      int o = 0;
#pragma unroll
      for (int b = 0; b < B; ++b)
        if ((e >> b) & 1) o ^= be[b];
      *reinterpret_cast<T*>(bb + (aw ^ o)) = x[e];
    }
  }
}

template <typename T>
__device__ __forceinline__ void run_gate(T* buf, const T* cf, const PassHead& h, const int32_t* lut, int logC) {
#define TQ_GATE(k, n) \
  case k * 16 + n: gate_pass<T, k, n>(buf, cf, h, lut, logC); break;
  switch ((h.w[kS2PmCount] >> 8) & 0xff) {   // K * 16 + N
    TQ_GATE(1, 1) TQ_GATE(1, 2) TQ_GATE(1, 4) TQ_GATE(1, 8)
    TQ_GATE(2, 1) TQ_GATE(2, 2) TQ_GATE(2, 4) TQ_GATE(2, 8)
    TQ_GATE(4, 1) TQ_GATE(4, 2) TQ_GATE(4, 4) TQ_GATE(4, 8)
    default: break;   // the plan compiler only emits K in {1, 2, 4}, N in {1, 2, 4, 8}
  }
#undef TQ_GATE
}

// SEQ: the chain-launch form (S2Launch::seq): one workgroup per CU (its streams are a few
// workgroups; the LDS hand-off block takes 64 KiB more), so up to 256 VGPRs -- the op loop around
// the body does not fit the 128 of the two-per-CU form without spilling
template <typename T, int CB, bool SEQ>
__global__ void __launch_bounds__(NT, SEQ ? 1 : 4) sweep2_kernel(S2Launch L) {
  constexpr int RMAX = (1 << CB) / NT;
  // register copies of elements as plain vector words (16-byte struct arrays behind runtime
  // conditions are otherwise demoted to scratch)
  using Raw = typename std::conditional<sizeof(T) == 16, double __attribute__((ext_vector_type(2))),
                                        typename std::conditional<sizeof(T) == 8, double, float>::type>::type;
  static_assert(sizeof(Raw) == sizeof(T), "raw slot word");
  static_assert(RMAX <= kS2MaxSlots, "register slots");
  // the gate coefficients first: their LDS addresses fit the 16-bit immediate offset of a
  // ds_read (behind the 64-KiB tile a gate's 8 coefficient reads took a v_mov + s_add each)
  struct alignas(16) Lds {
    T cf[kS2MaxGates * kCf];                             // gate coefficients, k*N+n
    T buf[1 << CB];
  };
  __shared__ Lds lds_main;
  T* const cf = lds_main.cf;
  T* const buf = lds_main.buf;
  static_assert(sizeof(S2Keep) % 8 == 0, "kept-table copy granularity");
  __shared__ uint2 keep_raw[sizeof(S2Keep) / 8];          // S2Desc::k, staged once
  // chain launches (S2Launch::seq) with LDS hand-offs: the dynamic LDS holds the tensor an op
  // passes to the next op of its stream, in its memory layout (S2Op::lds_io; <= 64 KiB)
  extern __shared__ __attribute__((aligned(16))) uint4 s2_dyn[];   // 16-B slots (complex128)
  Raw* const mir = reinterpret_cast<Raw*>(s2_dyn);
  const S2Keep& keep = *reinterpret_cast<const S2Keep*>(keep_raw);
  const int32_t* const gmeta = &keep.gmeta[0][0];        // K, N, pass mask, kaddr, naddr
  const int32_t* const pmeta = &keep.pmeta[0][0];        // passes
  const int32_t* const lut = &keep.lut[0][0];            // group -> LDS byte offset part
  const int tid = threadIdx.x;
  if (__builtin_amdgcn_wavefrontsize() != (1 << kS2WaveBits)) __builtin_trap();   // folded: wave64
  TQ_KCLOCK_BEGIN()
  // ---- which op this workgroup works on: one op of a level (blockIdx ranges select it,
  // wave-uniform scan), or -- S2Launch::seq, one workgroup -- every op of a dependent chain in
  // order: op j + 1 reads what op j stored (same CU: its stores are complete before the next
  // op's loads, below), and from the second op on the code is in this CU's instruction cache
  int j = 0;
  for (int q = 1; q < L.nops; ++q)
    if ((int)blockIdx.x >= L.op[q].block_begin) j = q;
  const int j_end = SEQ ? L.nops : j + 1;
  if (SEQ) j = 0;
  // descriptor words / gate-tensor elements per thread of the coalesced staging copy
  constexpr int kIt = (kDescWords2 + NT - 1) / NT, kGt = (kS2MaxGates * kS2GateRaw + NT - 1) / NT;
  // elements of gate gi (wave-uniform) an op stages: S2Op::gnum through the scalar unit (its
  // dword: no byte loads there) -- a per-lane index made it a vector load of the argument block,
  // waited for (with every load in flight) before the gate elements could be requested
  using KArg = const __attribute__((address_space(4))) S2Op*;
  using KWord = const __attribute__((address_space(4))) uint32_t*;
  auto gate_count = [](const S2Op& o, int gi) {
    const KArg ko = (KArg)&o;
    return gi < kS2MaxGates ? (int)((((KWord)ko->gnum)[gi >> 2] >> ((gi & 3) * 8)) & 0xff) : 0;
  };
  // descriptor words an op reads (S2Op::rows): S2Keep's group tables / pass rows below npass,
  // gate rows below ngates, column weights below colbits; everything else is always staged
  auto word_used = [](int i, int rows) {
    if (rows == 0) return true;
    const int b = i * 8 - kS2KeepOff;   // byte offset inside S2Keep
    const int np = rows & 0xff, ng = (rows >> 8) & 0xff, cb = (rows >> 16) & 0xff;
    constexpr int oWi = (int)offsetof(S2Keep, w_in), oWo = (int)offsetof(S2Keep, w_out),
                  oHa = (int)offsetof(S2Keep, ld_ha), oL = (int)offsetof(S2Keep, lut),
                  oG = (int)offsetof(S2Keep, gmeta), oP = (int)offsetof(S2Keep, pmeta);
    if (b < oWi) return true;
    if (b < oWo) return (b - oWi) / 8 < cb;
    if (b < oHa) return (b - oWo) / 8 < cb;
    if (b < oL) return true;
    if (b < oG) return (b - oL) / (64 * 4) < np;
    if (b < oP) return (b - oG) / (16 * 4) < ng;
    return (b - oP) / (kS2PmWords * 4) < np;
  };
  auto load_desc = [&](const S2Op& o, uint2 (&w)[kIt], Raw (&g)[kGt]) {
    const uint2* __restrict__ gd = reinterpret_cast<const uint2*>(o.desc);
    const int rows = ((KArg)&o)->rows;   // a kernel argument (scalar)
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int i = tid + it * NT;
      if (i < kDescWords2 && word_used(i, rows)) w[it] = gd[i];
    }
    // gate gi = (i / kS2GateRaw) is wave-uniform (kS2GateRaw = the wave size): its element count
    // and pointer come from the kernel argument through the scalar cache
    static_assert(kS2GateRaw == 64 && NT % 64 == 0, "one gate per wave and slot");
    const KArg ko = (KArg)&o;
#pragma unroll
    for (int it = 0; it < kGt; ++it) {
      const int i = tid + it * NT;
      const int gi = __builtin_amdgcn_readfirstlane(i / kS2GateRaw), e = i % kS2GateRaw;
      if (e < gate_count(o, gi)) g[it] = reinterpret_cast<const Raw*>(ko->G[gi])[e];
    }
  };
  // SEQ: the next op of this stream's descriptor and gate elements, loaded into registers while
  // this op runs (S2Op::lds_io bit 2: no earlier op of the launch writes its gate tensors)
  uint2 pdw[kIt];
  Raw pgw[kGt];
  bool have_pf = false;
  for (; j < j_end; ++j) {
  // another stream's op
  if (SEQ && ((int)blockIdx.x < L.op[j].block_begin || (int)blockIdx.x >= L.op[j].block_begin + L.op[j].nblocks))
    continue;
  const S2Op& op = L.op[j];
  const S2Desc* __restrict__ d = op.desc;
  // host-built per-thread lane offsets and per-chunk bases (S2Op::lanes / cbase, tq_plan.cpp
  // s2_blob): loaded from memory together with the descriptor staging below -- no LDS table walk
  // (and no barrier) between the descriptor and the first chunk's loads
  const bool host_lanes = op.lanes != nullptr, host_cb = op.cbase != nullptr;
  uint4 lane_e = {0u, 0u, 0u, 0u};
  if (host_lanes) lane_e = op.lanes[tid];
  int64_t hcb_in = 0, hcb_out = 0;
  if (host_cb) {
    const int64_t chl = ((int)blockIdx.x - op.block_begin) + (int64_t)(tid & 63) * op.nblocks;
    if (chl < d->nchunks) {
      hcb_in = op.cbase[2 * chl];
      hcb_out = op.cbase[2 * chl + 1];
    }
  }
#ifdef TQ_S2_TIMING
  const bool ts_rec = (int)blockIdx.x == op.block_begin;
  __shared__ unsigned int ts_slot;
  if (ts_rec && threadIdx.x == 0) ts_slot = atomicAdd(&g_s2_seq, 1u) % kTsMax;
  __syncthreads();
  const unsigned ts_idx = ts_slot;
  TQ_TS(0);
  if (ts_rec && threadIdx.x == 0)
    for (int q = 9; q < kTsPh; ++q) g_s2_ts[ts_idx][q] = 0;
#endif
  // ---- the descriptor is staged by one coalesced pass: its prologue part into the (not yet
  // used) tile buffer, S2Desc::k straight into its own LDS block, kept for the whole launch (no
  // chains of dependent scalar loads, no second LDS copy); the gate tensors' raw elements go to
  // the tile buffer behind the prologue part in the same pass (pointers and element counts are
  // kernel arguments)
  constexpr int kGrawOff = (kS2KeepOff + 255) / 256 * 256 / (int)sizeof(T);
  static_assert(kGrawOff + kS2MaxGates * kS2GateRaw <= (1 << CB), "descriptor + raw gates fit the tile");
  T* graw = buf + kGrawOff;
  {
    uint2* bd = reinterpret_cast<uint2*>(buf);
    uint2* kd = keep_raw;
    // every load is issued before the first LDS store (one memory round trip, not one per
    // loop iteration)
    uint2 dw[kIt];
    Raw gw[kGt];
    if (SEQ && have_pf) {
#pragma unroll
      for (int it = 0; it < kIt; ++it) dw[it] = pdw[it];
#pragma unroll
      for (int it = 0; it < kGt; ++it) gw[it] = pgw[it];
    } else {
      load_desc(op, dw, gw);
    }
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int i = tid + it * NT;
      if (i < kKeepWords2) bd[i] = dw[it];
      else if (i < kDescWords2) kd[i - kKeepWords2] = dw[it];
    }
#pragma unroll
    for (int it = 0; it < kGt; ++it) {
      const int i = tid + it * NT;
      const int g = __builtin_amdgcn_readfirstlane(i / kS2GateRaw), e = i % kS2GateRaw;
      if (e < gate_count(op, g)) reinterpret_cast<Raw*>(graw)[i] = gw[it];
    }
  }
  const T* __restrict__ X = reinterpret_cast<const T*>(op.X);
  T* __restrict__ Y = reinterpret_cast<T*>(op.Y);
  const int lb = (int)blockIdx.x - op.block_begin, nb = op.nblocks;
  const int logC = d->logC, colbits = d->colbits, npass = d->npass;
  const int cm = (1 << logC) - 1;
  const int64_t nchunks = d->nchunks;
  const int nld = d->nld, nst = d->nst;
  const int nin = 1 << nld, nout = 1 << nst;
  const int rin = (nin + NT - 1) / NT, rout = (nout + NT - 1) / NT;  // slots in use (powers of 2)
  const bool use_beta = op.use_beta;
  const double beta = op.beta;
  const bool x_lds = SEQ && (op.lds_io & 1) != 0, y_lds = SEQ && (op.lds_io & 2) != 0;   // chain hand-offs
  const bool coop = SEQ && (op.lds_io & kS2Coop) != 0;   // cooperative chain (S2Launch::sync)
  // producer-side max of a complex64 GEMM operand (S2Op::amax): max |re|, |im| of the values
  // this thread stores, one atomic per wave after the chunk loop
  constexpr bool kC64 = std::is_same<T, c64>::value;
  uint32_t* const amax = kC64 ? op.amax : nullptr;
  float vmax = 0.f;
  auto track = [&](const T& v) {
    if constexpr (kC64) vmax = fmaxf(vmax, fmaxf(fabsf(v.re), fabsf(v.im)));
  };
  // S2Op::split_sc: the stored form is the f16 terms (uniform branch)
  const bool split = kC64 && op.split_sc != nullptr;
  const int split_sc = split ? *op.split_sc : 0;
  auto stored = [&](const T& v) -> T {
    if constexpr (kC64) {
      if (split) return f16_terms(v, split_sc);
    }
    return v;
  };
  // a chain's previous op: its stores were issued before this op's descriptor loads and are
  // complete (in L2, visible to this CU) before any wave loads this op's input
  if (SEQ) __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  TQ_TS(1);
  if constexpr (SEQ) {
    int jn = j + 1;
    while (jn < L.nops && ((int)blockIdx.x < L.op[jn].block_begin ||
                           (int)blockIdx.x >= L.op[jn].block_begin + L.op[jn].nblocks))
      ++jn;
    have_pf = jn < L.nops && (L.op[jn].lds_io & 4) != 0;
    if (have_pf) load_desc(L.op[jn], pdw, pgw);
  }
  TQ_TS(44);   // next descriptor's loads issued
  const S2Desc* ds = reinterpret_cast<const S2Desc*>(buf);
  const int ngates = ds->ngates;
  const int epi = ds->epi;   // S2Desc::epi (read before the tile overwrites the descriptor copy)
  // ---- per-thread part of the load / store enumerations (low LOG_NT chunk bits); threads
  // beyond a small chunk duplicate element tid % n (same value to the same place)
  int64_t ldm = 0, stm = 0;
  int lda = 0, sta = 0;
  constexpr int ESH = sizeof(T) == 4 ? 2 : sizeof(T) == 8 ? 3 : 4;
  if (host_lanes) {
    ldm = (int64_t)(lane_e.x >> ESH);
    stm = (int64_t)(lane_e.y >> ESH);
    lda = (int)lane_e.z;
    sta = (int)lane_e.w;
  } else {
    const int ti = tid & (nin - 1), to = tid & (nout - 1);
#pragma unroll
    for (int b = 0; b < LOG_NT; ++b) {
      const int64_t lw = ds->ld_w[b], sw = ds->st_w[b];
      const int la = ds->ld_a[b], sa = ds->st_a[b];
      const bool lb_on = b < nld && ((ti >> b) & 1), sb_on = b < nst && ((to >> b) & 1);
      ldm += lb_on ? lw : 0;
      lda ^= lb_on ? la : 0;
      stm += sb_on ? sw : 0;
      sta ^= sb_on ? sa : 0;
    }
  }
  TQ_TS(45);   // lane offsets
  const bool st_lane = tid < nout;
  // uniform part (chunk + register slot) in scalar registers, lane part as a 32-bit byte offset
  const uint32_t ldo = (uint32_t)(ldm * (int64_t)sizeof(T)), sto = (uint32_t)(stm * (int64_t)sizeof(T));
  auto chunk_base = [&](int64_t ch, const int64_t* w) {
    int64_t o = 0;
    for (int b = logC; b < colbits; ++b)
      if ((ch >> (b - logC)) & 1) o += w[b];
    return o;
  };
  // Chunk base offsets of this workgroup's chunks lb + i*nb, i < 64: lane i of every wave holds
  // chunk i's (built once, all column-bit weights read in one batch); the chunk loop takes them
  // with a lane read instead of a chain of dependent LDS reads per chunk.
  const int64_t nloc = (nchunks - lb + nb - 1) / nb;
  const bool lane_bases = nloc <= 64;
  int64_t cb_in = hcb_in, cb_out = hcb_out;
  if (!host_cb) {
    const int64_t chl = lb + (int64_t)(tid & 63) * nb;
    for (int b0 = logC & ~7; b0 < colbits; b0 += 8) {   // batches of 8 weights in flight
      int64_t wi[8], wo[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {   // every read issued before the first is used
        const int bb = b0 + q < kS2MaxColBits ? b0 + q : kS2MaxColBits - 1;
        wi[q] = keep.w_in[bb];
        wo[q] = keep.w_out[bb];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int b = b0 + q;
        const bool on = b >= logC && b < colbits && ((chl >> (b - logC)) & 1);
        cb_in += on ? wi[q] : 0;
        cb_out += on ? wo[q] : 0;
      }
    }
  }
  TQ_TS(46);   // chunk bases
  auto lane64 = [](int64_t v, int i) {
    const int lo = __builtin_amdgcn_readlane((int)(uint32_t)v, i);
    const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), i);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  };
  // a chunk beyond the lanes' 64: from the host table through the scalar cache (a uniform read),
  // else summed from the column-bit weights
  using KI64 = const __attribute__((address_space(4))) int64_t*;
  auto base_in = [&](int i, int64_t ch) {
    return lane_bases ? lane64(cb_in, i) : host_cb ? ((KI64)op.cbase)[2 * ch] : chunk_base(ch, keep.w_in);
  };
  auto base_out = [&](int i, int64_t ch) {
    return lane_bases ? lane64(cb_out, i) : host_cb ? ((KI64)op.cbase)[2 * ch + 1] : chunk_base(ch, keep.w_out);
  };
  // The first chunk is loaded into RMAX register slots before the tables are staged (those
  // registers are free again before the gate passes).  Inside the chunk loop only chunks of at
  // most RPF slots are prefetched under the gate passes (the register-block passes need the
  // VGPRs); such ops are the multi-chunk ones (small input tile, large output tile).  Larger
  // chunks are loaded when they enter the tile.
  constexpr int RPF = RMAX > 2 ? 2 : RMAX;
  Raw reg[RPF];
  const bool pf = rin <= RPF;
  Raw* const bufr = reinterpret_cast<Raw*>(buf);
  const Raw* const Xr = reinterpret_cast<const Raw*>(X);
  // slot loops run a compile-time count (a power of two): loads / LDS accesses issue back to back
#define TQ_SLOTS(CAP, R, BODY)                                   \
  if constexpr ((CAP) >= (R)) {                                  \
    _Pragma("unroll") for (int r = 0; r < (R); ++r) BODY;        \
  }
#define TQ_BY_COUNT(CAP, n, BODY)                                \
  do {                                                           \
    if ((n) >= 16) { TQ_SLOTS(CAP, 16, BODY) }                   \
    else if ((n) >= 8) { TQ_SLOTS(CAP, 8, BODY) }                \
    else if ((n) >= 4) { TQ_SLOTS(CAP, 4, BODY) }                \
    else if ((n) >= 2) { TQ_SLOTS(CAP, 2, BODY) }                \
    else { TQ_SLOTS(CAP, 1, BODY) }                              \
  } while (0)
  auto prefetch = [&](int i, int64_t ch) {
    if (!pf) return;
    const int64_t base = base_in(i, ch);
    if (coop) {
      TQ_BY_COUNT(RPF, rin, reg[r] = ld_coherent<Raw>(Xr + uniform(base + keep.ld_hm[r]), ldo));
      return;
    }
    TQ_BY_COUNT(RPF, rin, reg[r] = *lane_at(Xr + uniform(base + keep.ld_hm[r]), ldo));
  };
  auto fill = [&](int i, int64_t ch) {   // the chunk's elements -> tile
    if (pf) {
      TQ_BY_COUNT(RPF, rin, bufr[lda ^ keep.ld_ha[r]] = reg[r]);
      return;
    }
    const int64_t base = base_in(i, ch);
    Raw t[RMAX];
    if (coop) TQ_BY_COUNT(RMAX, rin, t[r] = ld_coherent<Raw>(Xr + uniform(base + keep.ld_hm[r]), ldo));
    else TQ_BY_COUNT(RMAX, rin, t[r] = *lane_at(Xr + uniform(base + keep.ld_hm[r]), ldo));
    TQ_BY_COUNT(RMAX, rin, bufr[lda ^ keep.ld_ha[r]] = t[r]);
  };
  // a pass's head (PassHead): the pmeta row, one batch of LDS reads into scalar registers (the
  // pass's group-table reads do not depend on it: rows by pass)
  auto read_head = [&](int p, PassHead& h) {
    const int32_t* const pm = pmeta + p * kS2PmWords;
#pragma unroll
    for (int i = 0; i < 16; ++i) h.w[i] = __builtin_amdgcn_readfirstlane(pm[i]);
  };
  Raw reg0[RMAX];
  // ---- a cooperative op waits for every workgroup's arrival after the previous ops (their
  // stores complete): one lane polls the counter, the others wait at the barrier.  Every
  // workgroup waits, one with no chunk of this op too, so the count cannot run ahead of a slow one
  if constexpr (SEQ) {
    const uint32_t need = (uint32_t)op.lds_io >> 8;
    if (coop && need) {
      if (tid == 0) {
        int n = 0;
        while (__hip_atomic_load(L.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need && ++n < kCoopSpin)
          __builtin_amdgcn_s_sleep(2);
        if (n == kCoopSpin) __hip_atomic_fetch_add(L.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
    }
  }
  TQ_TS(47);   // cooperative wait
  // ---- the first chunk's loads go out now (addresses from the staged descriptor) and land
  // while the tables are staged
  int64_t ch = lb;
  if (ch < nchunks) {
    const int64_t base = lane_bases ? lane64(cb_in, 0) : chunk_base(ch, keep.w_in);
    if (x_lds) {   // the previous op of this stream left the tensor in LDS (one chunk)
      const int lm = (int)ldm;
      TQ_BY_COUNT(RMAX, rin, reg0[r] = mir[(int)(base + keep.ld_hm[r]) + lm]);
    } else if (coop) {
      TQ_BY_COUNT(RMAX, rin, reg0[r] = ld_coherent<Raw>(Xr + uniform(base + keep.ld_hm[r]), ldo));
    } else {
      TQ_BY_COUNT(RMAX, rin, reg0[r] = *lane_at(Xr + uniform(base + keep.ld_hm[r]), ldo));
    }
  }
  TQ_TS(41);   // first chunk's loads issued
  // ---- gate coefficients -> LDS
  for (int i = tid; i < ngates * kCf; i += NT) {
    const int g = i / kCf, t = i % kCf;
    if (t < keep.gmeta[g][kS2GmK] * keep.gmeta[g][kS2GmN]) cf[i] = graw[g * kS2GateRaw + ds->cgidx[g][t]];
  }
  TQ_TS(42);   // coefficients staged
  TQ_TS(43);   // tables staged (before the barrier)
  __syncthreads();   // every wave is done with the descriptor copy: the tile may be written
  TQ_TS(2);
  // Chunk pipeline.  On this ISA one counter (vmcnt) covers loads and stores, and a wait for a
  // load issued before some stores waits for those stores too (they may complete out of order),
  // so the order below keeps every wait where nothing else is pending:
  //   next chunk's loads -> gate passes -> wait(all) -> store this chunk -> tile <- next chunk
  // the stores of a chunk then drain under the next chunk's gate passes and the loads of the
  // chunk after it, instead of being waited for before that chunk can enter the tile.
  if (ch < nchunks) TQ_BY_COUNT(RMAX, rin, bufr[lda ^ keep.ld_ha[r]] = reg0[r]);
  __syncthreads();
  TQ_TS(3);
#ifdef TQ_S2_TIMING
  const unsigned long long clk0 = clock64();
  unsigned long long clk_gates = 0;
#endif
  for (int i = 0; ch < nchunks; ch += nb, ++i) {
    const int64_t nxt = ch + nb;
    const bool more = nxt < nchunks;
    if (more) prefetch(i + 1, nxt);
    for (int p = 0; p < npass; ++p) {
      PassHead cur;
      read_head(p, cur);
      // the workgroup barrier before a pass only where another wave may own its elements
      // (kS2PmSync, tq_plan.cpp s2_layout); otherwise every element this pass touches was
      // last touched by this wave, whose LDS accesses complete in order
      if (p > 0 && (cur.w[kS2PmCount] & kS2PmSync)) __syncthreads();
      asm volatile("" ::: "memory");
      const int g = cur.w[kS2PmFirst];
      const int bk = cur.w[kS2PmB];
      const int32_t* const lp = lut + p * kLut;   // the pass's group table (rows by pass)
      if (bk == 0) run_gate<T>(buf, cf + g * kCf, cur, lp, logC);
      else if ((bk & 0xff) == 4) {
        if constexpr (sizeof(T) <= 8) block_pass<T, 4>(buf, cf, cur, pmeta + p * kS2PmWords, lp, logC);
      }
      else block_pass<T, 3>(buf, cf, cur, pmeta + p * kS2PmWords, lp, logC);
      asm volatile("" ::: "memory");
#ifdef TQ_S2_TIMING
      if (ch == lb && ts_rec && threadIdx.x == 0 && p < 16) {
        g_s2_ts[ts_idx][9 + p] = clock64() - clk0;
        g_s2_ts[ts_idx][25 + p] = ((unsigned long long)bk << 16) | (gmeta[g * kGm + kGmK] << 8) |
                                  gmeta[g * kGm + kGmN] | ((unsigned long long)(cur.w[kS2PmCount] & 0xff) << 24);
      }
#endif
    }
    __syncthreads();   // the store phase reads the tile in its own enumeration
    if (ch == lb) TQ_TS(4);
#ifdef TQ_S2_TIMING
    if (ch == lb) clk_gates = clock64() - clk0;
#endif
    // vmcnt(0) (expcnt / lgkmcnt unconstrained): the next chunk is in registers, the previous
    // chunk's stores are done
    __builtin_amdgcn_s_waitcnt(0x0F70);
    const int64_t base = base_out(i, ch);
    // the tile leaves LDS in batches of 4 register slots, each batch stored before the next is
    // read (keeps the register budget)
    // the max of the stored values is always tracked (3 VALU per complex64 element; the atomic
    // only runs for an S2Op::amax): one instantiation of each store form instead of two, the
    // code sits in the 64-KB instruction cache two CUs share (r04: -9 KB of 72)
    auto store_chunk = [&]() {
      if (rout >= 4) {
        for (int r0 = 0; r0 < rout; r0 += 4) {
          T t[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) t[q] = buf[sta ^ keep.st_ha[r0 + q]];
          if (st_lane && y_lds) {
#pragma unroll
            for (int q = 0; q < 4; ++q) reinterpret_cast<T*>(mir)[(int)(base + keep.st_hm[r0 + q]) + (int)stm] = t[q];
          } else if (st_lane && coop) {   // (no beta, no split, no max: the planner's cooperative ops)
#pragma unroll
            for (int q = 0; q < 4; ++q) st_coherent(Y + uniform(base + keep.st_hm[r0 + q]), sto, t[q]);
          } else if (st_lane) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              T* p = lane_at(Y + uniform(base + keep.st_hm[r0 + q]), sto);
              const T v = use_beta ? scale_add(t[q], *p, beta) : t[q];
              TQ_ST(p, stored(v));
              track(v);
            }
          }
          asm volatile("" ::: "memory");
        }
      } else {
        T t[4];
        TQ_BY_COUNT(4, rout, t[r] = buf[sta ^ keep.st_ha[r]]);
        if (st_lane && y_lds) {
          TQ_BY_COUNT(4, rout, reinterpret_cast<T*>(mir)[(int)(base + keep.st_hm[r]) + (int)stm] = t[r]);
        } else if (st_lane && coop) {
          TQ_BY_COUNT(4, rout, st_coherent(Y + uniform(base + keep.st_hm[r]), sto, t[r]));
        } else if (st_lane) {
          TQ_BY_COUNT(4, rout, {
            T* p = lane_at(Y + uniform(base + keep.st_hm[r]), sto);
            const T v = use_beta ? scale_add(t[r], *p, beta) : t[r];
            TQ_ST(p, stored(v));
            track(v);
          });
        }
      }
    };
    // S2Desc::epi: the last gate is applied here, in registers -- a thread reads the K inputs of
    // a group (slots r0 .. r0+K-1 of the pre-gate tile) and stores its N outputs (slots r0 ..
    // r0+N-1); the coefficients are wave-uniform (scalar registers)
    auto store_epi = [&](auto kt, auto nt) {
      constexpr int K = decltype(kt)::value, N = decltype(nt)::value;
      // the coefficient row's offset is re-materialised per chunk: hoisted out of the chunk loop,
      // the per-case LDS addresses of every (K, N) instantiation were spilled to scratch and
      // reloaded one dependent round trip per read
      int cb = __builtin_amdgcn_readfirstlane((epi - 1) * kCf);
      asm volatile("" : "+s"(cb));
      const T* ce = cf + cb;
      T c[K * N];
#pragma unroll
      for (int q = 0; q < K * N; ++q) c[q] = uniform(ce[q]);
      for (int r0 = 0; r0 < rout; r0 += N) {
        T x[K];
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = buf[sta ^ keep.st_ha[r0 + k]];
        if (st_lane) {
#pragma unroll
          for (int n = 0; n < N; ++n) {
            T acc = mul(x[0], c[n]);
#pragma unroll
            for (int k = 1; k < K; ++k) mac(acc, x[k], c[k * N + n]);
            if (y_lds) {
              reinterpret_cast<T*>(mir)[(int)(base + keep.st_hm[r0 + n]) + (int)stm] = acc;
              continue;
            }
            if (coop) {
              st_coherent(Y + uniform(base + keep.st_hm[r0 + n]), sto, acc);
              continue;
            }
            T* p = lane_at(Y + uniform(base + keep.st_hm[r0 + n]), sto);
            const T v = use_beta ? scale_add(acc, *p, beta) : acc;
            TQ_ST(p, stored(v));
            track(v);
          }
        }
        asm volatile("" ::: "memory");
      }
    };
    auto store_epi_kn = [&]() {
      using std::integral_constant;
#define TQ_EPI(k, n) \
  case k * 16 + n: store_epi(integral_constant<int, k>{}, integral_constant<int, n>{}); break;
      const int32_t* gm = gmeta + (epi - 1) * kGm;
      switch (gm[kGmK] * 16 + gm[kGmN]) {
        TQ_EPI(1, 2) TQ_EPI(1, 4) TQ_EPI(1, 8) TQ_EPI(2, 2) TQ_EPI(2, 4) TQ_EPI(2, 8) TQ_EPI(4, 4)
        default: break;   // the plan compiler only emits these (K <= N, K * N <= 16)
      }
#undef TQ_EPI
    };
    if (epi) store_epi_kn();
    else store_chunk();
    __syncthreads();  // every wave has read the tile
    if (ch == lb) TQ_TS(5);
    if (more) fill(i + 1, nxt);
    __syncthreads();
  }
  // a cooperative op's arrival: every wave's stores have completed (vmcnt(0)), then the
  // workgroup barrier, then one agent-scope add; the launch's last arrival resets the counter
  if constexpr (SEQ) {
    if (coop) {
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (tid == 0) {
        const uint32_t n = __hip_atomic_fetch_add(L.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n + 1 == (uint32_t)L.sync_total) __hip_atomic_store(L.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (amax) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
    // one atomic per wave only when it raises the word: every wave of a big op finishes at about
    // the same time, and thousands of same-address atomics serialise in one L2 channel (a 2^21-
    // element operand took 58 us); a relaxed read first skips the ones that cannot win
    if ((threadIdx.x & 63) == 0 &&
        __float_as_uint(vmax) > __hip_atomic_load(amax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(amax, __float_as_uint(vmax));
  }
#ifdef TQ_S2_TIMING
  __builtin_amdgcn_s_waitcnt(0);
  TQ_TS(6);
  if (ts_rec && threadIdx.x == 0) g_s2_ts[ts_idx][7] = ((unsigned long long)op.nblocks << 32) | (unsigned)nchunks;
  if (ts_rec && threadIdx.x == 0) g_s2_ts[ts_idx][8] = clk_gates;
#endif
#undef TQ_BY_COUNT
#undef TQ_SLOTS
  }  // ops
  TQ_KCLOCK_END(g_kclk_sweep2)
}

template <typename T>
int launch_t(const S2Launch& L, hipStream_t stream) {
  constexpr int CB = sizeof(T) > 8 ? 12 : 13;
  if (L.seq) {   // dependent chains: workgroup b runs the ops of stream b in order
    int streams = 0;
    bool lds = false;
    for (int q = 0; q < L.nops; ++q) {
      if (L.op[q].block_begin < 0 || L.op[q].nblocks < 1 ||
          L.op[q].block_begin + L.op[q].nblocks > kS2SeqMaxStreams) {
        set_error("sweep2: a chain launch runs at most kS2SeqMaxStreams workgroups");
        return TQ_ERR_INVALID;
      }
      streams = std::max(streams, L.op[q].block_begin + L.op[q].nblocks);
      lds = lds || L.op[q].lds_io != 0;
    }
    // a cooperative chain: every op on all the launch's workgroups, op k waiting for k x n
    // arrivals, no LDS hand-off (a mixed launch could strand a workgroup at a wait)
    int ncoop = 0;
    for (int q = 0; q < L.nops; ++q) ncoop += (L.op[q].lds_io & kS2Coop) != 0;
    if (ncoop) {
      bool ok = ncoop == L.nops && L.sync != nullptr && L.sync_total == ncoop * streams;
      for (int q = 0; q < L.nops && ok; ++q)
        ok = L.op[q].block_begin == 0 && L.op[q].nblocks == streams && (L.op[q].lds_io & 3) == 0 &&
             (L.op[q].lds_io >> 8) == q * streams && !L.op[q].use_beta && !L.op[q].amax && !L.op[q].split_sc;
      if (!ok) {
        set_error("sweep2: malformed cooperative chain launch");
        return TQ_ERR_INVALID;
      }
    }
    // LDS hand-offs: a 64-KiB dynamic block beside the kernel's ~76 KiB (one workgroup per CU;
    // every cooperative chain takes it too: the sc1 hand-off between its workgroups is the form
    // measured with one workgroup per CU)
    const unsigned dyn = lds ? (unsigned)kS2ChunkBytes : 0u;
    if (dyn) {
      static DeviceCache<1> attr;
      if (attr.get(0, [] {
            return hipFuncSetAttribute(reinterpret_cast<const void*>(&sweep2_kernel<T, CB, true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kS2ChunkBytes) == hipSuccess ? 1 : -1;
          }) < 0) {
        set_error("sweep2: dynamic LDS for chain hand-offs");
        return TQ_ERR_INVALID;
      }
    }
    hipLaunchKernelGGL((sweep2_kernel<T, CB, true>), dim3((unsigned)streams), dim3(NT), dyn, stream, L);
    TQ_HIP(hipGetLastError());
    return TQ_OK;
  }
  int blocks = 0;
  for (int q = 0; q < L.nops; ++q) blocks = std::max(blocks, L.op[q].block_begin + L.op[q].nblocks);
  if (blocks <= 0) return TQ_OK;
  // A launch of more workgroups than fit on the GPU at once (the lane-merged per-slice levels:
  // 8-16 lanes x 2 ops x 64-512 chunks) is scaled to one resident round (TQ_S2_CAP = rounds,
  // default 1; 0 = off): every workgroup strides over several chunks, so its ~5-us prologue
  // (descriptor + tables) is paid once and each chunk's stores drain under the next chunk's gate
  // passes (the chunk pipeline below) instead of at the end of a one-chunk workgroup.  Measured
  // (r03, same box): C3 1.84 -> 1.27 ms per step (its per-slice launch of 1536 one-chunk
  // workgroups spent ~80 us per round in the store / drain phases, waves waiting 75 %), C4 +-0
  // (13.36 / 13.29 ms; 2 rounds 13.29, 4 rounds 13.24), C3 with 2 rounds 1.56 ms.
  static const double rounds = [] {
    const char* e = getenv("TQ_S2_CAP");
    return e ? atof(e) : 1.0;   // resident rounds per launch (0 = no cap)
  }();
  // per device (cached; -1 = no cap)
  static DeviceCache<1> cap_cache;
  const int cap = !(rounds > 0) ? 0 : std::max(0, cap_cache.get(0, [] {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&sweep2_kernel<T, CB, false>), NT, 0) != hipSuccess)
      return -1;
    return std::max(1, (int)(cus * std::max(1, per) * rounds));
  }));
  if (cap > 0 && blocks > cap) {
    S2Launch R = L;
    int b = 0;
    for (int q = 0; q < R.nops; ++q) {
      R.op[q].nblocks = std::max(1, (int)((int64_t)L.op[q].nblocks * cap / blocks));
      R.op[q].block_begin = b;
      b += R.op[q].nblocks;
    }
    hipLaunchKernelGGL((sweep2_kernel<T, CB, false>), dim3((unsigned)b), dim3(NT), 0, stream, R);
    TQ_HIP(hipGetLastError());
    return TQ_OK;
  }
  hipLaunchKernelGGL((sweep2_kernel<T, CB, false>), dim3((unsigned)blocks), dim3(NT), 0, stream, L);
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

}  // namespace

// copies up to n records of 8 stamps (see g_s2_ts) and resets the sequence; 0 without the
// instrumentation
int sweep2_timing(unsigned long long* out, int n) {
#ifdef TQ_S2_TIMING
  unsigned seq = 0;
  if (hipMemcpyFromSymbol(&seq, HIP_SYMBOL(g_s2_seq), sizeof(seq)) != hipSuccess) return -1;
  const int cnt = (int)std::min<unsigned>(seq, (unsigned)std::min(n, kTsMax));
  if (cnt > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_s2_ts), sizeof(unsigned long long) * kTsPh * cnt) != hipSuccess)
    return -1;
  const unsigned zero = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_s2_seq), &zero, sizeof(zero)) != hipSuccess) return -1;
  return cnt;
#else
  (void)out; (void)n;
  return 0;
#endif
}

int sweep2_kclock(unsigned long long* out, int n) { return TQ_KCLOCK_READ(g_kclk_sweep2, out, n); }

int sweep2_launch(int dtype, const S2Launch& L, hipStream_t stream) {
  if (L.nops < 1 || L.nops > kS2MaxOps) {
    set_error("sweep2: bad op count");
    return TQ_ERR_INVALID;
  }
  switch (dtype) {
    case TQ_F32: return launch_t<float>(L, stream);
    case TQ_F64: return launch_t<double>(L, stream);
    case TQ_C64: return launch_t<c64>(L, stream);
    case TQ_C128: return launch_t<c128>(L, stream);
  }
  set_error("sweep2: bad dtype");
  return TQ_ERR_INVALID;
}

}  // namespace tq
