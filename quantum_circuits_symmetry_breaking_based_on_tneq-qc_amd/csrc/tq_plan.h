// Contraction-plan compiler and executor (host C++ over the HIP kernels).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "tq_common.h"
#include "tq_permute.h"
#include "tq_sweep2.h"

namespace tq {

// where an operand lives
enum BufKind { BUF_INPUT = 0, BUF_ARENA = 1, BUF_OUTPUT = 2, BUF_TABLE = 3, BUF_PINNED = 4,
               BUF_PENDING = 5 /* compile time only: result of an open sweep chain */ };
struct BufRef {
  int kind = BUF_ARENA;
  int64_t index = 0;  // input id for BUF_INPUT
  int64_t off = 0;    // element offset (bytes for BUF_TABLE)
  int region = 0;     // compile time: arena region (branch) the offset is relative to
};

enum OpKind { OP_PERMUTE = 0, OP_GEMM = 1, OP_APPLY = 2, OP_AXPY = 3, OP_SWEEP = 4,
              OP_SWEEP2 = 5 /* in-place butterfly sweep (profiled as OP_SWEEP) */ };

// one gate of a fused sweep op (OP_SWEEP): small operand + its gather table + index table
struct SweepGate {
  BufRef g;
  int gtab = -1;
  int K = 0, N = 0, W = 0;
  int64_t n = 0;        // elements of the gate operand (hazard analysis)
  size_t tab_off = 0;   // entry offset of its [W][K+1] int16 table in the op's packed tables
};

struct Op {
  int kind = OP_PERMUTE;
  BufRef a, b, c;       // permute: a -> c ; gemm: c = a*b ; apply: c = a (x) b ; axpy: c += a
  bool writes_output = false;
  bool invariant = false;  // reads no sliced input: run once per execute call (hoisted)
  int branch = 0;          // 0 / 1: the two independent subtrees of the final step (own arena
                           // regions; their sweeps share launches); 2: the join (final step)
  // permute
  int perm = -1;        // index into Plan::perms
  // gemm
  int transA = 0, transB = 0;
  int64_t M = 0, N = 0, K = 0, batch = 1, lda = 0, ldb = 0, ldc = 0, sA = 0, sB = 0, sC = 0;
  BufRef ws;
  size_t ws_bytes = 0;
  // apply: S = [O][K][M][K2][I] -> C = [O][N][M][I]   (K, N above)
  int64_t O = 0, I = 0, K2 = 1;
  int gtab = -1;         // gather table of the small operand (index into Plan::gtabs)
  // axpy
  int64_t n = 0;
  // sweep (fused chain of APPLY steps): a = chain input, c = chain output, gates in order
  std::vector<SweepGate> sgates;
  int stab = -1;                 // index into Plan::stabs (tin_off | tout_off | gate tables)
  int tin = 0, tout = 0;
  int nruns = 0;
  int64_t run_ext[8] = {}, run_in[8] = {}, run_out[8] = {};
  int64_t ncols = 0;
  size_t tout_off_at = 0;        // byte offset of tout_off inside the blob (tin_off at 0)
  size_t tabs_at = 0;            // byte offset of the packed gate tables inside the blob
  int tab_len = 0;
  int load_colfast = 1, store_colfast = 1;
  // sweep2: descriptor blob = stabs[stab] (an S2Desc), launched with s2_blocks(s2_nchunks)
  int64_t s2_nchunks = 0;
  // sweep2 whose whole tensor fits one LDS tile: the one-chunk layout of the same chain
  // (stabs[stab1]; == stab when the default layout is one chunk already, -1: none), the form a
  // chain launch (Plan::seq_once) runs
  int stab1 = -1;
  // chain launches: bit 0 = X comes from the workgroup's LDS (the previous op of its stream left
  // it there), bit 1 = Y stays in LDS for the next op of its stream (S2Op::lds_io)
  int lds_io = 0;
  // dense sweep (tq_sweepd.hip): stabs[stab] is an S2Dense, b = the tout x tin coefficient
  // matrix written by the preceding compose op (a sweep2 op of the same chain on the identity)
  bool s2_dense = false;
  // operand-max words (complex64 f16-split GEMM): a sweep2 op that produces a GEMM operand
  // max-es its stored values into word amax_word; the GEMM reads words amax_a / amax_b
  int amax_word = -1, amax_a = -1, amax_b = -1;
  // pre-split operands (GemmPresplit): a per-slice GEMM whose two operands are each stored in
  // full by one per-slice sweep2 op and read by nothing else may take them as f16 terms
  // (ps_cand); its producers (ps_gemm = that GEMM) then store the terms (S2Op::split_sc)
  bool ps_cand = false;
  int ps_gemm = -1;
  // pre-split boundary GEMM ("planes", tq_gemmp.hip): the GEMM (Plan::planes_gemm) and its two
  // dense producers (planes_role 1 = A, 2 = B), which then store the six f16 term planes of their
  // output instead of the complex64 values; planes_in_amax = the max word of the dense op's input
  // (written by that input's producer) from which the producer bounds its output
  int planes_role = 0;
  int planes_in_amax = -1;
  // per-slice GEMM on lane-local (or pinned) operands: the lanes of a batch run as ONE batched
  // launch (strides = Plan::lane_stride, workspace at Plan::lane_ws_off)
  bool lane_batch = false;
  // lane_sum (a lane-batched GEMM): its result is read only by one output permute, so the
  // lanes' results are summed into lane 0's and that permute (lane_once) runs once per batch
  bool lane_sum = false, lane_once = false;
  // strided skinny contraction (an OP_GEMM with M * N <= 16 whose operands are read in place
  // through per-bit strides instead of being permuted first): weights in sk, pointers at launch
  bool skinny = false;
  SkinnyArgs sk;
  // element counts of a / b / c / ws (hazard analysis of the launch schedule)
  int64_t na = 0, nb = 0, nc = 0, nws = 0;
  // bookkeeping
  int step = -1;
  double flops = 0, bytes = 0;
  std::string note;
};

struct InputView {
  std::vector<int> modes;      // modes after removing sliced ones
  std::vector<int64_t> ext;
  std::vector<int64_t> stride;
  std::vector<int64_t> slice_stride;  // per sliced mode (0 if absent)
};

// the arguments a plan was compiled from (kept for plan_recompile)
struct CompileArgs {
  std::vector<int32_t> in_ranks, in_modes, out_modes, path, sliced;
  std::vector<int64_t> in_extents, in_strides;
};

struct Plan {
  int dtype = TQ_C64;
  CompileArgs args;
  int group_hint = 1;       // compiled for lockstep groups of this many plans (wider sweep chunks)
  int min_chunks = 0;       // smallest chunk count of a big sweep op (0: TQ_S2_MINCHUNKS, default 128)
  size_t esz = 8;
  int n_inputs = 0;
  std::vector<InputView> inputs;
  std::vector<int> out_modes;
  std::vector<int64_t> out_ext;
  int64_t out_numel = 1;
  std::vector<int> sliced;
  std::vector<int64_t> sliced_ext;
  int64_t n_slices = 1;
  std::vector<Op> ops;
  std::vector<PermPlan> perms;
  std::vector<size_t> perm_tab_off;   // byte offset in the table buffer
  std::vector<std::vector<int32_t>> gtabs;  // APPLY small-operand gather tables
  std::vector<size_t> gtab_off;
  std::vector<std::vector<char>> stabs;     // OP_SWEEP table blobs
  std::vector<size_t> stab_off;
  size_t table_bytes = 0;
  // operand-max words behind the tables (zeroed per execute call: the first n_amax_once, written
  // by slice-invariant producers; per slice batch: the next n_amax_slice x lanes, lane j's set at
  // n_amax_once + j * n_amax_slice)
  size_t amax_off = 0;
  int n_amax_once = 0, n_amax_slice = 0;
  // pre-split GEMMs: scale words (one per per-slice max word), one window flag per slice, and
  // the host copy of the flags (read after an execute call that ran pre-split GEMMs)
  size_t sc_off = 0, bad_off = 0;
  int n_ps = 0;               // pre-split candidate GEMMs
  uint32_t* h_bad = nullptr;  // pinned, n_slices words
  int run_mode = 0;           // 1: this execute call runs the candidates pre-split
  // pre-split boundary GEMM (Op::planes_role): one per plan; device buffer d_planes (plan-owned,
  // allocated at materialize) = per lane [A planes][B planes] (6 planes of the operand's element
  // count each, 2 B), then the GEMM's f32 partials, then per lane two scale words (A, B)
  int planes_gemm = -1;
  int64_t planes_n[2] = {0, 0};     // elements of the A / B operand (one plane)
  size_t planes_lane_bytes = 0, planes_ws_off = 0, planes_sc_off = 0, planes_bytes = 0;
  void* d_planes = nullptr;
  bool use_planes = true;           // TQ_GEMM_PLANES (default 1) / tq_plan_set "gemm_planes"
  int64_t ps_fallbacks = 0;   // slices re-run on the split path (operand max left the window)
  size_t arena_bytes = 0;
  size_t pinned_base = 0;             // pinned (hoisted, slice-invariant) results live above this
  // slice lanes: slices run in batches of `lanes`; lane j > 0 has its own copy of the per-slice
  // part [0, pinned_base) at lane0_bytes + (j-1) * pinned_base (arena_bytes includes the copies).
  // Small per-slice working sets only (C3: 64 latency-bound slices), 1 otherwise (C4)
  int lanes = 1;
  size_t lane0_bytes = 0;
  // physical arena: [pinned part][lane 0][lane 1]...[lane-batched GEMM workspace]; lane j's copy
  // of [0, pinned_base) starts at lane_phys + j * lane_stride (a uniform stride, so a per-slice
  // GEMM of all lanes is ONE batched launch); the logical offsets used by the compiler's
  // analyses are unchanged (arena [0, pinned_base), pinned above)
  size_t lane_phys = 0, lane_stride = 0, lane_ws_off = 0, lane_ws_bytes = 0;
  void* d_arena = nullptr;
  void* d_tables = nullptr;
  bool owns_device = false;
  int device = -1;          // HIP device the arena / tables / graphs belong to (set at materialize)
  uint64_t serial = 0;      // process-unique id (set at materialize; group graph keys)
  // optional per-op-kind timing with HIP events on the execution stream (bench evidence)
  unsigned profile = 0;  // bit k set: time ops of kind k
  struct Ev { hipEvent_t a, b; int kind; double flops, bytes; };
  std::vector<Ev> ev_used, ev_free;
  double flops = 0, bytes = 0;              // whole execute (all slices)
  double flops_once = 0, bytes_once = 0;    // slice-invariant (hoisted) part
  double flops_slice = 0, bytes_slice = 0;  // per slice
  int n_gemm = 0, n_apply = 0, n_permute = 0, n_sweep = 0, n_sweep_gates = 0;
  // launch schedule: ops grouped by dependency level; independent sweep2 ops of one level share
  // a launch.  `once` = slice-invariant ops (first slice of an execute call), `slice` = per slice
  std::vector<std::vector<int>> sched_once, sched_slice;
  int n_launch_once = 0, n_launch_slice = 0;
  // chain launches: runs [first, last) of consecutive sched_once entries that are each ONE small
  // sweep2 op (a one-chunk layout exists), run in order by one workgroup in one launch
  // (S2Launch::seq) when use_seq (env TQ_S2_SEQ, default 1; tq_plan_set "sweep_chain")
  std::vector<std::pair<int, int>> seq_once;
  std::vector<int> seq_stream;   // per op: its stream (workgroup) in a chain launch, -1 none
  bool use_seq = true;
  // cooperative chain launches: runs [first, last) of consecutive sched_once entries that are
  // each ONE multi-chunk sweep2 op (C2's 27 levels of 4-chunk ops), run by coop_width[r]
  // workgroups in one launch with a counter barrier between the ops (S2Launch::sync = the
  // 256-byte slot r at sync_off of the tables) when use_coop (env TQ_S2_COOP; tq_plan_set
  // "sweep_coop")
  static constexpr size_t kSyncSlot = 256;
  std::vector<std::pair<int, int>> coop_once;
  std::vector<int> coop_width;
  size_t sync_off = 0;
  bool use_coop = false;     // TQ_S2_COOP (default off) / tq_plan_set "sweep_coop"
  std::string describe;
  // hipGraph of the whole launch sequence of one execute call, replayed while the call's
  // pointers / slice range / flags are unchanged (a plan is hundreds of small launches)
  struct GraphKey {
    std::vector<const void*> inputs;
    void* out = nullptr;
    int64_t b = 0, e = 0, s = 0;
    int acc = 0;
    int mode = 0;   // Plan::run_mode the graph was captured with
    int planes = 0; // the pre-split boundary GEMM was on
    bool seq = true;  // Plan::use_seq
    bool coop = false;  // Plan::use_coop
    // a group execute (plan_run_group): every member's output and serial
    std::vector<const void*> group;
    bool operator==(const GraphKey& o) const {
      return inputs == o.inputs && out == o.out && b == o.b && e == o.e && s == o.s && acc == o.acc &&
             mode == o.mode && seq == o.seq && coop == o.coop && planes == o.planes && group == o.group;
    }
  };
  bool use_graph = true;
  // small cache of instantiated graphs (alternating slice ranges / buffers do not re-capture);
  // an entry is destroyed only after the event recorded behind its last launch has completed
  struct GraphEntry {
    GraphKey key;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    hipEvent_t done = nullptr;
    uint64_t used = 0;
  };
  std::vector<GraphEntry> graphs;
  uint64_t graph_clock = 0;
  hipStream_t cap_stream = nullptr;
  // a group execute led by this plan: side streams / events of its per-member branches
  std::vector<hipStream_t> side_streams;
  std::vector<hipEvent_t> side_events;
  int64_t graph_builds = 0, graph_launches = 0;
};

int plan_compile(Plan& P, int dtype, int n_inputs, const int32_t* in_ranks, const int32_t* in_modes,
                 const int64_t* in_extents, const int64_t* in_strides, int out_rank,
                 const int32_t* out_modes, int n_steps, const int32_t* path, int n_sliced,
                 const int32_t* sliced_modes, int group_hint = 1, int min_chunks = 0);
// compile the plan again for lockstep groups of `group_hint` plans and with `min_chunks` (0:
// the default) chunks per big sweep op at least (before its first execute)
int plan_recompile(Plan& P, int group_hint, int min_chunks);
// a copy of a compiled plan without any device state (arena, tables, graphs, events): the
// same schedule for another stream / block (tq_plan_clone)
void plan_clone_compiled(const Plan& src, Plan& dst);
// the pre-split boundary GEMM's buffer layout (planes, partials, scale words): host only
void plan_planes_layout(Plan& P);
// upload tables / allocate arena (owned) — or use caller memory when `arena`/`tables` are given
int plan_materialize(Plan& P, void* arena, void* tables, hipStream_t stream);
int plan_run(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
             int64_t s_step, int accumulate, hipStream_t stream);
// a group of plans compiled from the same network, run in lockstep on one stream: every sweep2 /
// dense-sweep level and chain launch of all members is one launch (blocks as lanes); inputs[k] /
// outs[k] are member k's.  Replayed as one hipGraph (cached in plans[0]).
int plan_run_group(Plan* const* plans, int n, const void* const* const* inputs, void* const* outs,
                   int64_t s_begin, int64_t s_end, int64_t s_step, int accumulate, hipStream_t stream);
int plan_release(Plan& P);   // TQ_OK, or TQ_ERR_HIP with what is left still held (retry later)
int plan_profile_read(Plan& P, int kind, double* ms, int64_t* launches, double* flops, double* bytes);

}  // namespace tq
