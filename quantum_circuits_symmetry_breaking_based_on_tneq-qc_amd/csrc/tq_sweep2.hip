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

namespace tq {

namespace {

constexpr int NT = 512, LOG_NT = 9;
constexpr int kLut = 64;                     // per-gate group tables: 32 entries for the low 5 pass bits,
                                             // 32 for the high ones (<= 9 pass positions)
constexpr int kCf = kS2MaxK * kS2MaxKN;      // coefficient slots per gate
// per-gate fields the gate passes read, staged in LDS: read in every pass of every chunk, they
// must not queue behind the chunk's HBM stores (descriptor loads are vector loads)
constexpr int kGmK = kS2GmK, kGmN = kS2GmN, kGmPass = kS2GmPass, kGmKaddr = kS2GmKaddr,
              kGmNaddr = kS2GmNaddr;
constexpr int kGm = 16;
constexpr int kDescWords2 = (int)(sizeof(S2Desc) / 8);
static_assert(sizeof(S2Desc) % 8 == 0, "descriptor copy granularity");

// per-chunk tables of the load / store phases, staged in LDS for the same reason
struct S2Hot {
  int64_t ld_hm[kS2MaxSlots], st_hm[kS2MaxSlots];
  int64_t w_in[kS2MaxColBits], w_out[kS2MaxColBits];
  int32_t ld_ha[kS2MaxSlots], st_ha[kS2MaxSlots];
};
static_assert(kGmNaddr + kS2MaxKN <= kGm, "gate meta layout");
static_assert(kLut == 64, "lut layout shared with S2Desc::lut");

#ifdef TQ_S2_TIMING
// development instrumentation (built only with -DTQ_S2_TIMING): workgroup 0 of every op records
// wall-clock stamps (100 MHz) at its phase boundaries
constexpr int kTsMax = 4096, kTsPh = 9;
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

// acc += a * b on packed f32: (a.re, a.re) * (b.re, b.im) + (a.im, a.im) * (-b.im, b.re).
// The broadcasts and the swap / negation are operand modifiers (op_sel / neg), not copies.
__device__ __forceinline__ f2v pmac(f2v acc, f2v a, f2v b) {
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "+v"(acc) : "v"(a), "v"(b));
  return acc;
}

template <typename T>
__device__ __forceinline__ void mac(T& acc, const T& a, const T& b) {
  if constexpr (std::is_same<T, c64>::value) {
    const f2v r = pmac(f2v{acc.re, acc.im}, f2v{a.re, a.im}, f2v{b.re, b.im});
    acc = c64{r.x, r.y};
  } else {
    cmac(acc, a, b);
  }
}

// One gate over all groups of the chunk.  Every LDS address is an XOR of contributions:
// group (lut[pp] ^ c) ^ input k (kaddr[k]) / output n (naddr[n]).  U groups per thread in
// flight; all K inputs of a group are read before any of its N outputs is written (outputs
// reuse the input positions).
template <typename T, int K, int N>
__device__ __forceinline__ void gate_pass(T* __restrict__ buf, const T* __restrict__ cf,
                                          const int32_t* __restrict__ gm,
                                          const int32_t* __restrict__ lut, int logC) {
  constexpr int U = sizeof(T) > 8 ? (K * N >= 8 ? 1 : 2) : (K * N >= 16 ? 2 : 4);
  constexpr bool kReg = K * N * sizeof(T) <= 64;   // coefficients held in registers
  const int tid = threadIdx.x;
  const int ngroups = (1 << logC) << __popc((uint32_t)gm[kGmPass]);
  const int cm = (1 << logC) - 1;
  int ka[K], na[N];
#pragma unroll
  for (int k = 0; k < K; ++k) ka[k] = gm[kGmKaddr + k];
#pragma unroll
  for (int n = 0; n < N; ++n) na[n] = gm[kGmNaddr + n];
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
      a0[u] = lut[gp & 31] ^ lut[32 + (gp >> 5)] ^ (gi & cm);
    }
    T x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < K; ++k) x[u][k] = buf[a0[u] ^ ka[k]];
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
        T acc = tzero<T>();
#pragma unroll
        for (int k = 0; k < K; ++k) mac(acc, x[u][k], c[k]);
        if (ok[u]) buf[a0[u] ^ na[n]] = acc;
      }
    }
  }
}

template <typename T>
__device__ __forceinline__ void run_gate(T* buf, const T* cf, const int32_t* gm, const int32_t* lut,
                                         int logC) {
#define TQ_GATE(k, n) \
  case k * 16 + n: gate_pass<T, k, n>(buf, cf, gm, lut, logC); break;
  switch (gm[kGmK] * 16 + gm[kGmN]) {
    TQ_GATE(1, 1) TQ_GATE(1, 2) TQ_GATE(1, 4) TQ_GATE(1, 8)
    TQ_GATE(2, 1) TQ_GATE(2, 2) TQ_GATE(2, 4) TQ_GATE(2, 8)
    TQ_GATE(4, 1) TQ_GATE(4, 2) TQ_GATE(4, 4) TQ_GATE(4, 8)
    default: break;   // the plan compiler only emits K in {1, 2, 4}, N in {1, 2, 4, 8}
  }
#undef TQ_GATE
}

template <typename T, int CB>
__global__ void __launch_bounds__(NT, 4) sweep2_kernel(S2Launch L) {
  constexpr int RMAX = (1 << CB) / NT;
  static_assert(RMAX <= kS2MaxSlots, "register slots");
  __shared__ T buf[1 << CB];
  __shared__ int32_t lut[kS2MaxGates * kLut];            // group -> LDS address part
  __shared__ T cf[kS2MaxGates * kCf];                    // gate coefficients, k*N+n
  __shared__ int32_t gmeta[kS2MaxGates * kGm];           // K, N, pass mask, kaddr, naddr
  __shared__ S2Hot hot;
  const int tid = threadIdx.x;
  // ---- which op this workgroup works on (wave-uniform scan over <= 16 ranges)
  int j = 0;
  for (int q = 1; q < L.nops; ++q)
    if ((int)blockIdx.x >= L.op[q].block_begin) j = q;
  const S2Op& op = L.op[j];
  const S2Desc* __restrict__ d = op.desc;
#ifdef TQ_S2_TIMING
  const bool ts_rec = (int)blockIdx.x == op.block_begin;
  __shared__ unsigned int ts_slot;
  if (ts_rec && threadIdx.x == 0) ts_slot = atomicAdd(&g_s2_seq, 1u) % kTsMax;
  __syncthreads();
  const unsigned ts_idx = ts_slot;
  TQ_TS(0);
#endif
  // ---- the descriptor is staged in the (not yet used) tile buffer by one coalesced pass; the
  // tables below are built from that copy (no chains of dependent scalar loads)
  // the gate tensors' raw elements go to the tile buffer behind the descriptor in the same pass
  // (pointers and element counts are kernel arguments)
  constexpr int kGrawOff = ((int)sizeof(S2Desc) + 255) / 256 * 256 / (int)sizeof(T);
  static_assert(kGrawOff + kS2MaxGates * kS2GateRaw <= (1 << CB), "descriptor + raw gates fit the tile");
  T* graw = buf + kGrawOff;
  {
    const uint2* __restrict__ gd = reinterpret_cast<const uint2*>(d);
    uint2* bd = reinterpret_cast<uint2*>(buf);
    for (int i = tid; i < kDescWords2; i += NT) bd[i] = gd[i];
    for (int i = tid; i < kS2MaxGates * kS2GateRaw; i += NT) {
      const int g = i / kS2GateRaw, e = i % kS2GateRaw;
      if (e < (int)op.gnum[g]) graw[i] = reinterpret_cast<const T*>(op.G[g])[e];
    }
  }
  const T* __restrict__ X = reinterpret_cast<const T*>(op.X);
  T* __restrict__ Y = reinterpret_cast<T*>(op.Y);
  const int lb = (int)blockIdx.x - op.block_begin, nb = op.nblocks;
  const int logC = d->logC, colbits = d->colbits, ngates = d->ngates;
  const int cm = (1 << logC) - 1;
  const int64_t nchunks = d->nchunks;
  const int nld = d->nld, nst = d->nst;
  const int nin = 1 << nld, nout = 1 << nst;
  const int rin = (nin + NT - 1) / NT, rout = (nout + NT - 1) / NT;  // slots in use (powers of 2)
  const bool use_beta = op.use_beta;
  const double beta = op.beta;
  __syncthreads();
  TQ_TS(1);
  const S2Desc* ds = reinterpret_cast<const S2Desc*>(buf);
  // ---- gate coefficients -> LDS
  for (int i = tid; i < ngates * kCf; i += NT) {
    const int g = i / kCf, t = i % kCf;
    const S2Gate& gt = ds->gate[g];
    if (t < gt.K * gt.N) cf[i] = graw[g * kS2GateRaw + gt.gidx[t]];
  }
  // ---- per-chunk tables -> LDS
  for (int i = tid; i < kS2MaxSlots; i += NT) {
    hot.ld_hm[i] = ds->ld_hm[i];
    hot.st_hm[i] = ds->st_hm[i];
    hot.ld_ha[i] = ds->ld_ha[i];
    hot.st_ha[i] = ds->st_ha[i];
  }
  for (int i = tid; i < kS2MaxColBits; i += NT) {
    hot.w_in[i] = ds->w_in[i];
    hot.w_out[i] = ds->w_out[i];
  }
  // ---- gate fields and group tables -> LDS (built on the host, S2Desc::gmeta / lut)
  for (int i = tid; i < ngates * kGm; i += NT) gmeta[i] = ds->gmeta[i / kGm][i % kGm];
  for (int i = tid; i < ngates * kLut; i += NT) lut[i] = ds->lut[i / kLut][i % kLut];
  // ---- per-thread part of the load / store enumerations (low LOG_NT chunk bits); threads
  // beyond a small chunk duplicate element tid % n (same value to the same place)
  int64_t ldm = 0, stm = 0;
  int lda = 0, sta = 0;
  {
    const int ti = tid & (nin - 1), to = tid & (nout - 1);
    for (int b = 0; b < LOG_NT; ++b) {
      if (b < nld && ((ti >> b) & 1)) { ldm += ds->ld_w[b]; lda ^= ds->ld_a[b]; }
      if (b < nst && ((to >> b) & 1)) { stm += ds->st_w[b]; sta ^= ds->st_a[b]; }
    }
  }
  const bool st_lane = tid < nout;
  // uniform part (chunk + register slot) in scalar registers, lane part as a 32-bit byte offset
  const uint32_t ldo = (uint32_t)(ldm * (int64_t)sizeof(T)), sto = (uint32_t)(stm * (int64_t)sizeof(T));
  __syncthreads();
  TQ_TS(2);
  auto chunk_base = [&](int64_t ch, const int64_t* w) {
    int64_t o = 0;
    for (int b = logC; b < colbits; ++b)
      if ((ch >> (b - logC)) & 1) o += w[b];
    return o;
  };
  T reg[RMAX];
  // slot loops run a compile-time count (a power of two): loads / LDS accesses issue back to back
#define TQ_SLOTS(R, BODY)                                  \
  if constexpr (RMAX >= (R)) {                             \
    _Pragma("unroll") for (int r = 0; r < (R); ++r) BODY;  \
  }
#define TQ_BY_COUNT(n, BODY)                                     \
  do {                                                           \
    if ((n) >= 16) { TQ_SLOTS(16, BODY) }                        \
    else if ((n) >= 8) { TQ_SLOTS(8, BODY) }                     \
    else if ((n) >= 4) { TQ_SLOTS(4, BODY) }                     \
    else if ((n) >= 2) { TQ_SLOTS(2, BODY) }                     \
    else { TQ_SLOTS(1, BODY) }                                   \
  } while (0)
  auto prefetch = [&](int64_t ch) {
    const int64_t base = chunk_base(ch, hot.w_in);
    TQ_BY_COUNT(rin, reg[r] = *lane_at(X + base + hot.ld_hm[r], ldo));
  };
  // Chunk pipeline.  On this ISA one counter (vmcnt) covers loads and stores, and a wait for a
  // load issued before some stores waits for those stores too (they may complete out of order),
  // so the order below keeps every wait where nothing else is pending:
  //   next chunk's loads -> gate passes -> wait(all) -> store this chunk -> tile <- next chunk
  // the stores of a chunk then drain under the next chunk's gate passes and the loads of the
  // chunk after it, instead of being waited for before that chunk can enter the tile.
  int64_t ch = lb;
  if (ch < nchunks) {
    prefetch(ch);
    TQ_BY_COUNT(rin, buf[lda ^ hot.ld_ha[r]] = reg[r]);
  }
  __syncthreads();
  TQ_TS(3);
#ifdef TQ_S2_TIMING
  const unsigned long long clk0 = clock64();
  unsigned long long clk_gates = 0;
#endif
  for (; ch < nchunks; ch += nb) {
    const int64_t nxt = ch + nb;
    const bool more = nxt < nchunks;
    if (more) prefetch(nxt);
    for (int g = 0; g < ngates; ++g) {
      run_gate<T>(buf, cf + g * kCf, gmeta + g * kGm, lut + g * kLut, logC);
      __syncthreads();
    }
    if (ch == lb) TQ_TS(4);
#ifdef TQ_S2_TIMING
    if (ch == lb) clk_gates = clock64() - clk0;
#endif
    // vmcnt(0) (expcnt / lgkmcnt unconstrained): the next chunk is in registers, the previous
    // chunk's stores are done
    __builtin_amdgcn_s_waitcnt(0x0F70);
    const int64_t base = chunk_base(ch, hot.w_out);
    // the tile leaves LDS in batches of 4 register slots, each batch stored before the next is
    // read (keeps the register budget)
    if (rout >= 4) {
      for (int r0 = 0; r0 < rout; r0 += 4) {
        T t[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] = buf[sta ^ hot.st_ha[r0 + q]];
        if (st_lane) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            T* p = lane_at(Y + base + hot.st_hm[r0 + q], sto);
            *p = use_beta ? scale_add(t[q], *p, beta) : t[q];
          }
        }
        asm volatile("" ::: "memory");
      }
    } else {
      T t[4];
      TQ_BY_COUNT(rout, t[r] = buf[sta ^ hot.st_ha[r]]);
      if (st_lane) {
        TQ_BY_COUNT(rout, {
          T* p = lane_at(Y + base + hot.st_hm[r], sto);
          *p = use_beta ? scale_add(t[r], *p, beta) : t[r];
        });
      }
    }
    __syncthreads();  // every wave has read the tile
    if (ch == lb) TQ_TS(5);
    if (more) TQ_BY_COUNT(rin, buf[lda ^ hot.ld_ha[r]] = reg[r]);
    __syncthreads();
  }
#ifdef TQ_S2_TIMING
  __builtin_amdgcn_s_waitcnt(0);
  TQ_TS(6);
  if (ts_rec && threadIdx.x == 0) g_s2_ts[ts_idx][7] = ((unsigned long long)op.nblocks << 32) | (unsigned)nchunks;
  if (ts_rec && threadIdx.x == 0) g_s2_ts[ts_idx][8] = clk_gates;
#endif
#undef TQ_BY_COUNT
#undef TQ_SLOTS
}

template <typename T>
int launch_t(const S2Launch& L, hipStream_t stream) {
  constexpr int CB = sizeof(T) > 8 ? 12 : 13;
  int blocks = 0;
  for (int q = 0; q < L.nops; ++q) blocks = std::max(blocks, L.op[q].block_begin + L.op[q].nblocks);
  if (blocks <= 0) return TQ_OK;
  hipLaunchKernelGGL((sweep2_kernel<T, CB>), dim3((unsigned)blocks), dim3(NT), 0, stream, L);
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
