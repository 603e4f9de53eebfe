// In-place butterfly sweep (tq_sweep2.hip): descriptors shared by the plan compiler and the
// kernel.  A sweep op applies a chain of small operands ("gates") to a big tensor X in one HBM
// pass, Y[outer, t_out] = (G_q o ... o G_1)(X[outer, t_in]), for chains whose modes all have
// power-of-two extents.  Every mode bit of the working set owns a fixed *position* bit of an
// LDS tile index; a gate reads its K inputs and writes its N outputs at the positions of its
// index bits (outputs reuse the positions the gate frees), so the tile is updated in place.
#pragma once
#include <cstddef>
#include <cstdint>

#include <hip/hip_runtime.h>

namespace tq {

constexpr int kS2MaxGates = 16;
constexpr int kS2MaxKN = 8;            // N <= 8 per gate (coefficient slots: 8 x 8)
constexpr int kS2MaxK = 4;             // K <= 4 per gate (exact-shape gate passes)
#ifndef TQ_S2_MAX_OPS
#define TQ_S2_MAX_OPS 32
#endif
// independent sweep ops batched into one launch (a level's ops of every slice lane: C3's 16
// lanes x 2 ops in one launch -- 0.995 -> 0.785 ms per step against 16; S2Launch is a ~7-KB
// kernel argument)
constexpr int kS2MaxOps = TQ_S2_MAX_OPS;
constexpr int kS2GateRaw = 64;         // gate-tensor elements staged per gate
constexpr int kS2ChunkBytes = 65536;   // LDS tile per workgroup
constexpr int kS2MaxChunkBits = 13;    // log2(chunk elements) for 8-byte elements
constexpr int kS2MaxColBits = 48;
constexpr int kS2LogThreads = 9;       // 512 threads per workgroup
// Pass barriers (kS2PmSync, planned in tq_plan.cpp s2_layout): thread t takes the groups
// gi == t (mod 2^kS2LogThreads) of every pass, so the 64-lane wave w owns exactly the groups whose
// gi bits [kS2WaveBits, kS2LogThreads) equal w.  The kernel asserts both constants.
constexpr int kS2WaveBits = 6;         // log2(wave size): CDNA waves are 64 lanes
constexpr int kS2MaxSlots = 16;        // chunk elements per thread (load / store register slots)
constexpr int kS2MaxPos = 10;         // tile positions (index bits), at most
inline int s2_max_pos(int esz) { return esz > 8 ? 9 : 10; }
inline int s2_chunk_bits(int esz) { return esz > 8 ? 12 : 13; }

// chunk-element code: column bits [0,13), position bits [13,23), swizzle [23,28); all XOR-combined
constexpr int kS2CodeP = 13, kS2CodeS = 23;

struct S2Gate {
  int K = 0, N = 0;
  uint32_t pass_mask = 0;                 // live positions the gate does not contract
  int32_t kdep[kS2MaxKN] = {}, ndep[kS2MaxKN] = {};  // position bits of input k / output n
  int32_t ksw[kS2MaxKN] = {}, nsw[kS2MaxKN] = {};    // their swizzle contributions
  // LDS element-address XOR masks of input k / output n (linear in the position bits):
  // (dep << logC) ^ sw
  int32_t kaddr[kS2MaxKN] = {}, naddr[kS2MaxKN] = {};
  int32_t gidx[kS2MaxKN * kS2MaxKN] = {};             // coefficient k*N+n -> element of G
};

// The tables every chunk and gate pass of the kernel reads: staged from the descriptor straight
// into their own LDS block once per workgroup and kept for the whole launch.
struct S2Keep {
  // register slot r (chunk bits >= kS2LogThreads of element r*512+tid): memory offset and LDS
  // address; slots beyond the chunk repeat slot r % slots (a duplicate, harmless access)
  int64_t ld_hm[kS2MaxSlots] = {}, st_hm[kS2MaxSlots] = {};
  int64_t w_in[kS2MaxColBits] = {}, w_out[kS2MaxColBits] = {};  // column-bit weights
  int32_t ld_ha[kS2MaxSlots] = {}, st_ha[kS2MaxSlots] = {};
  // Built on the host (plan compile):
  //  lut[p][j]: LDS BYTE offset part of group index bits -> ((pass positions << logC) ^ swizzle)
  //             * element size, j < 32 for the low 5 pass bits, 32 + j for the high ones
  //             (XOR-linear, combined by ^)
  //  gmeta[g][f]: K, N, pass mask, kaddr[0..3], naddr[0..7] (kS2GmK.. layout; element units)
  int32_t lut[kS2MaxGates][64] = {};
  int32_t gmeta[kS2MaxGates][16] = {};
  // Passes over the tile (one barrier each).  A pass is one gate, or a register block: a run of
  // consecutive square gates (K == N, outputs on their inputs' positions) whose positions fit B
  // bits; every thread then holds 2^B elements of a group in registers and applies the whole
  // run to them (one LDS read + write per element for the run instead of per gate).
  //  pmeta[p]: first gate, gate count, B (0 = single gate), pass mask (live positions outside the
  //            block), block-bit address parts [4, 4+B), per-gate local codes [8, 8+count):
  //            bits 0-1 / 2-3 = block bits of the gate's index bits 0 / 1, bit 4 = 4x4 (else 2x2).
  //            A single-gate pass (B = 0) carries its gate instead: count | (K*16+N) << 8, the
  //            gate's pass mask, kaddr [4, 8), naddr [8, 16) -- a pass's head is one read batch
  //  lut rows are by PASS (row p: the group table of pass p; a block's own table)
  //  A lane block (B word kS2PmLanes | 4) spans 6 positions: 4 in the registers, 2 on lane bits 4
  //  and 5 of the thread (group-index bits 4 and 5); its codes mix gates and swap codes
  //  (kS2SwapCode | lane bit (4: 0, 5: 1) << 2 | register bit: a register bit and a lane bit
  //  trade positions, v_permlane16 / 32_swap), and [16, 22) hold the end layout for the
  //  write-back: the register bits' address parts, then the XOR deltas of lane bits 4 and 5
  int32_t pmeta[kS2MaxGates][24] = {};
};

struct S2Desc {
  // ---- staged into the (not yet used) tile buffer, read in the kernel's prologue only
  int64_t ncols = 0, nchunks = 0;
  int logC = 0, colbits = 0;     // columns per chunk (log2), column index bits
  int nld = 0, nst = 0;          // chunk bits of the load (X) / store (Y) enumerations
  int ngates = 0;
  // 1 + index of the last gate when the store phase applies it in registers (0: every gate is a
  // pass): its output index bits are the lowest register-slot bits of the store enumeration, so
  // a thread's slots r0 .. r0+N-1 hold one group's outputs and r0 .. r0+K-1 its inputs
  int epi = 0;
  int64_t ld_w[16] = {}, st_w[16] = {};      // memory weight of each chunk bit (ascending)
  // LDS element address of each chunk bit: every LDS address is an XOR of these
  int32_t ld_a[16] = {}, st_a[16] = {};
  // coefficient k*N+n of gate g -> element of its gate tensor (S2Gate::gidx, < kS2GateRaw)
  uint8_t cgidx[kS2MaxGates][kS2MaxK * kS2MaxKN] = {};
  int32_t npass = 0, pad2 = 0;
  // ---- kept in LDS for the whole launch
  S2Keep k;
  // ---- host-side build records (not staged)
  int32_t ld_code[16] = {}, st_code[16] = {};
  int32_t ld_hc[kS2MaxSlots] = {}, st_hc[kS2MaxSlots] = {};
  int32_t vsw[12] = {};          // swizzle vector of each position (kS2MaxPos used)
  // modeled extra LDS bank-conflict cycles / conflict-free cycles of a chunk: the r04 column-only
  // swizzle, the chosen one (tq_plan.cpp s2_layout)
  float lds_model[2] = {};
  int32_t nsync = 0;             // passes preceded by a workgroup barrier (kS2PmSync)
  // byte offsets (in the plan's descriptor blob) of the host-built lane / chunk-base tables
  // (S2Op::lanes / cbase), 0 = none
  int32_t aux_lanes = 0, aux_cb = 0;
  alignas(8) S2Gate gate[kS2MaxGates];
};
constexpr int kS2KeepOff = (int)offsetof(S2Desc, k);
constexpr int kS2DescHotBytes = (int)(offsetof(S2Desc, k) + sizeof(S2Keep));   // the staged part
static_assert(kS2KeepOff % 8 == 0 && kS2DescHotBytes % 8 == 0, "descriptor copy granularity");
constexpr int kS2GmK = 0, kS2GmN = 1, kS2GmPass = 2, kS2GmKaddr = 3, kS2GmNaddr = kS2GmKaddr + kS2MaxK;
static_assert(kS2GmNaddr + kS2MaxKN <= 16, "gate meta layout");
constexpr int kS2PmFirst = 0, kS2PmCount = 1, kS2PmB = 2, kS2PmPass = 3, kS2PmAddr = 4, kS2PmCode = 8;
constexpr int kS2PmAddrEnd = 16, kS2PmLaneDelta = 20, kS2PmWords = 24;   // lane blocks (S2Keep::pmeta)
constexpr int kS2PmLanes = 1 << 8;     // B-word flag: a lane block
constexpr int kS2SwapCode = 32;        // block code flag: swap a register bit with lane bit 4 / 5
static_assert(sizeof(S2Keep::pmeta[0]) == kS2PmWords * sizeof(int32_t), "pass row words");
constexpr int kS2PmSync = 1 << 16;   // count-word flag: a workgroup barrier before this pass
constexpr int kS2BlkMaxGates = 8;      // gates per register block
inline int s2_block_bits(int esz, int64_t tile_elems) {
  // 2^B elements per thread: 16 (FP32 data, tiles of >= 8192 elements) or 8
  return (esz <= 8 && tile_elems >= 8192) ? 4 : 3;
}

struct S2Op {
  const S2Desc* desc = nullptr;
  const void* X = nullptr;
  void* Y = nullptr;
  const void* G[kS2MaxGates] = {};
  // elements of G[g] the gate reads (max gidx + 1, <= kS2GateRaw): staged by the kernel together
  // with the descriptor, so the coefficient fetch is not a second dependent global round trip
  uint8_t gnum[kS2MaxGates] = {};
  int block_begin = 0, nblocks = 0;
  double beta = 0.0;
  // lds_io (chain launches only, one-chunk ops of <= kS2ChunkBytes): bit 0 = X is in the launch's
  // dynamic LDS block (left there by the previous op of this stream), bit 1 = Y goes there
  // instead of memory (the next op of this stream is its only reader; no beta, no split, no max),
  // bit 2 = no op of the launch writes this op's gate tensors (its descriptor and gate elements
  // may be loaded while the previous op of its stream runs), bit 3 (kS2Coop) = a cooperative op
  // (S2Launch::sync): its X / Y move through L2-coherent accesses, and bits 8.. hold the count of
  // arrivals it waits for before its loads (every workgroup of the launch arrives once per op)
  int use_beta = 0, lds_io = 0;
  // complex64 only, optional: the op atomically max-es the float bits of max |re|, |im| over
  // every value it stores into *amax (zeroed before; the max a consuming f16-split GEMM scales by)
  uint32_t* amax = nullptr;
  // complex64 only, optional: store every value as the f16 terms of v * 2^sc, sc = *split_sc
  // ((h_re, h_im | l_re, l_im) in the element's 8 bytes; the consuming GEMM's SplitPre); amax
  // still tracks the unscaled values
  const int32_t* split_sc = nullptr;
  // host-built tables behind the descriptor (tq_plan.cpp s2_blob; nullptr = computed in the
  // kernel): per thread (byte offset of its load / store element, LDS address of both), and per
  // chunk (memory base of its load / store elements) -- S2Desc::aux_lanes / aux_cb
  const uint4* lanes = nullptr;
  const int64_t* cbase = nullptr;
  // the descriptor rows in use (host-filled from it; 0 = stage every row): npass | ngates << 8 |
  // colbits << 16 -- the prologue stages only the group-table / pass / gate rows and column
  // weights the op reads (a 2-pass op stages ~2 KiB of the 7-KiB S2Keep)
  int32_t rows = 0, pad_rows = 0;
};
constexpr int kS2MaxCbTab = 4096;   // chunks with a host-built base table, at most

// streams of a chain launch (S2Launch::seq), a workgroup each
constexpr int kS2SeqMaxStreams = 8;
constexpr int kS2Coop = 8;   // S2Op::lds_io: a cooperative op
struct S2Launch {
  // seq = 0: independent ops (one dependency level), blockIdx ranges select the op; seq = 1:
  // dependent chains -- workgroup b runs, in order, every op whose range [block_begin,
  // block_begin + nblocks) holds b (a stream: nblocks 1; an op reads only what earlier ops of
  // its stream wrote): no launch gap between the small ops of a long chain, and the kernel's
  // code stays in one CU's instruction cache
  int nops = 0, seq = 0;
  // cooperative chain (seq = 1, every op kS2Coop over the same workgroups [0, n)): op k's
  // chunks are spread over the n workgroups, and op k + 1 reads what ANY of them stored, so a
  // counter barrier separates the ops: every workgroup adds 1 to sync[0] after its op-k stores
  // have completed, and loads op k + 1's input once sync[0] >= (k + 1) n.  sync[0] is zero when
  // the launch starts; the last arrival (sync_total = ops x n) resets it.  sync[1] counts
  // waits that gave up (a bounded spin: never expected; the results are then invalid)
  uint32_t* sync = nullptr;
  int sync_total = 0, pad = 0;
  S2Op op[kS2MaxOps];
};

// The kernel addresses a lane's element as (uniform 64-bit base) + (32-bit byte offset), the
// offset being the summed memory weights of the low kS2LogThreads load / store chunk bits: an
// op whose lane offsets could reach 4 GiB must not be lowered to sweep2.
inline bool s2_lane_offsets_fit(const int64_t* ld_w, int nld, const int64_t* st_w, int nst,
                                int64_t esz) {
  int64_t l = 0, s = 0;
  for (int b = 0; b < kS2LogThreads && b < nld; ++b) l += ld_w[b];
  for (int b = 0; b < kS2LogThreads && b < nst; ++b) s += st_w[b];
  return (l > s ? l : s) * esz < (int64_t(1) << 32);
}

// blocks a sweep op gets when launched (chunks are strided over them)
inline int s2_blocks(int64_t nchunks) { return (int)(nchunks < 512 ? nchunks : 512); }

int sweep2_launch(int dtype, const S2Launch& L, hipStream_t stream);

// ---- dense sweep (tq_sweepd.hip): an expanding chain with a small input tile (tin <= 16) on a
// big tensor, Y[outer, r] = sum_k M[r][k] X[outer, k].  M (tout x tin, row-major: the tin
// coefficients of output r contiguous) is the chain composed on the identity by a separate tiny
// sweep2 op (the plan's "compose" op; the gates are device data).  No LDS tile and no gate
// passes: a small-K complex GEMM on the f32 matrix cores per 32-column tile, the columns being
// the memory-fastest bits of X and Y (coalesced loads and 256-B store segments).
constexpr int kS2DMaxTin = 16;
constexpr int kS2DMaxTout = 256;
struct S2Dense {
  int64_t ncols = 0;             // columns (outer index), a multiple of 64
  int colbits = 0, tin = 0, tout = 0, pad = 0;
  int64_t w_in[kS2MaxColBits] = {}, w_out[kS2MaxColBits] = {};  // column-bit weights (bits >= 6 used)
  int64_t in_off[kS2DMaxTin] = {};     // memory offset of input tile element k
  int64_t out_off[kS2DMaxTout] = {};   // memory offset of output tile element r
};
struct S2DOp {
  const S2Dense* desc = nullptr;   // device copy (plan tables)
  const void* X = nullptr;
  void* Y = nullptr;
  const void* M = nullptr;         // tout x tin coefficients
  int block_begin = 0, nblocks = 0;
  int tin = 0, tout = 0;           // host copies of the descriptor's (launch checks)
  int use_beta = 0, pad = 0;
  double beta = 0.0;
  uint32_t* amax = nullptr;        // as S2Op::amax
  const int32_t* split_sc = nullptr;  // as S2Op::split_sc
  int order = 0, pad2 = 0;         // tile order (tq_sweepd.hip): 0 grid-strided, 1 blocked
  int64_t ncols = 0;               // host copy (the launcher shares the workgroups by work)
  // planes mode (the pre-split boundary GEMM, tq_gemmp.hip): Y is not written; instead the six f16
  // term planes (re_h, re_l, im_h, im_l, s_h, s_l) of Y * 2^sc go to planes + p * pstride (element
  // offsets as Y's), sc from the bound max|Y| <= sqrt(2) max(|re X|, |im X|) max_r sum_k |M[r][k]|
  // (amax_in: X's producer's max word); sc is stored to *sc_out for the GEMM's unscaling
  void* planes = nullptr;
  int64_t pstride = 0;
  const uint32_t* amax_in = nullptr;
  int32_t* sc_out = nullptr;
};
struct S2DLaunch {
  int nops = 0, pad = 0;
  S2DOp op[kS2MaxOps];
};
// blocks of a dense op (4 waves each, one 32-column tile per wave and iteration)
// workgroups a dense op may use (4 waves, one 32-column tile per wave at a time); the launcher
// caps the launch at one round of resident workgroups shared by its ops (a single-lane op then
// gets all of them: 1 workgroup per CU left 3 of 4 slots idle at 3.0 TB/s)
inline int s2d_blocks(int64_t ncols) {
  const int64_t tiles = ncols / 32;
  const int64_t b = (tiles + 3) / 4;
  return (int)(b < 2048 ? b : 2048);
}
int sweepd_launch(int dtype, const S2DLaunch& L, hipStream_t stream);
int sweep2_timing(unsigned long long* out, int n);   // development instrumentation
int sweep2_kclock(unsigned long long* out, int n);   // in-kernel clock records (-DTQ_KCLOCK builds)

}  // namespace tq
