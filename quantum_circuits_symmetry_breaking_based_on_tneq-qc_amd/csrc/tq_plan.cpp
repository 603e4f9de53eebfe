// Contraction-plan compiler and executor: the GPU-resident replacement of the reference's
// opt_einsum ContractExpression (tneq_qc/contractor/einsum_strategy.py:622-643, executed by
// ComputeBackend.execute_expression, tneq_qc/backends/backend_pytorch.py:99-105).
//
// Compile time (host, once per expression + dtype + strides):
//   * walks the SSA pairwise path, tracks which modes are still needed (mode reference counts),
//     classifies every mode of each pair (batch / contracted / free / single-side sum),
//   * picks per step the cheapest lowering:
//       APPLY  one operand small (<= 32 x 32) and its contracted modes forming at most two runs
//              in the big operand -> one streaming pass, no transpose (tq_apply.hip); the small
//              operand is read in any layout through a gather table (no extra launch);
//       GEMM   TTGT: reuse any operand whose layout is already [batch][M][K] / [batch][K][M]
//              (no transpose), otherwise permute it (tq_permute.hip); operand roles and the
//              K order are chosen to minimise transposed bytes; MFMA GEMM (tq_gemm.hip);
//   * lays intermediates out in one arena with a first-fit allocator over their live ranges,
//   * tabulates every permute's tile tables once (uploaded with the plan).
// Run time: a flat list of kernel launches on one stream per slice; sliced modes are removed
// from the input views, each slice only shifts input base pointers; slices are summed into the
// output by the final op's beta.
#include "tq_plan.h"
#include "tq_sweep.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <numeric>
#include <set>
#include <sstream>

namespace tq {

namespace {

constexpr int64_t kAlign = 256;

std::vector<int64_t> contig_strides(const std::vector<int64_t>& ext) {
  std::vector<int64_t> s(ext.size());
  int64_t p = 1;
  for (int d = (int)ext.size() - 1; d >= 0; --d) { s[d] = p; p *= ext[d]; }
  return s;
}

struct Live {
  std::vector<int> modes;
  std::vector<int64_t> ext;
  std::vector<int64_t> stride;
  BufRef buf;
  bool owned = false;  // arena intermediate that must be freed after use
  bool dep = false;    // depends on a sliced input (otherwise computed once per execute)
  int64_t numel() const { return prod(ext); }
  bool contiguous() const {
    auto cs = contig_strides(ext);
    for (size_t d = 0; d < ext.size(); ++d)
      if (ext[d] != 1 && stride[d] != cs[d]) return false;
    return true;
  }
  int pos(int m) const {
    for (size_t i = 0; i < modes.size(); ++i) if (modes[i] == m) return (int)i;
    return -1;
  }
};

class Arena {
 public:
  int64_t alloc(int64_t bytes) {
    bytes = std::max<int64_t>(kAlign, (bytes + kAlign - 1) / kAlign * kAlign);
    int64_t cur = 0;
    auto it = used_.begin();
    for (; it != used_.end(); ++it) {
      if (it->first - cur >= bytes) break;
      cur = it->first + it->second;
    }
    used_.insert(it, {cur, bytes});
    peak_ = std::max(peak_, cur + bytes);
    return cur;
  }
  void release(int64_t off) {
    for (auto it = used_.begin(); it != used_.end(); ++it)
      if (it->first == off) { used_.erase(it); return; }
  }
  int64_t peak() const { return peak_; }

 private:
  std::vector<std::pair<int64_t, int64_t>> used_;  // sorted by offset
  int64_t peak_ = 0;
};

std::string modes_str(const std::vector<int>& m) {
  std::ostringstream o;
  o << "(";
  for (size_t i = 0; i < m.size(); ++i) o << (i ? "," : "") << m[i];
  o << ")";
  return o.str();
}

// A sweep2 op's descriptor blob: the S2Desc, then the host-built tables the kernel reads instead
// of walking the descriptor in LDS (S2Op::lanes / cbase): per thread of the 512 its load / store
// element's byte offset and LDS address (threads beyond a small chunk duplicate element tid % n,
// as the kernel's own enumeration), and per chunk (when there are at most kS2MaxCbTab) the memory
// base of its load / store elements.
std::vector<char> s2_blob(const S2Desc& d0, size_t esz) {
  S2Desc d = d0;
  auto al16 = [](size_t b) { return (b + 15) / 16 * 16; };
  const size_t off_l = al16(sizeof(S2Desc));
  const size_t off_c = off_l + (size_t)(1 << kS2LogThreads) * 16;
  const bool cb = d.nchunks >= 1 && d.nchunks <= kS2MaxCbTab;
  d.aux_lanes = (int32_t)off_l;
  d.aux_cb = cb ? (int32_t)off_c : 0;
  std::vector<char> blob(off_c + (cb ? (size_t)d.nchunks * 16 : 0), 0);
  std::memcpy(blob.data(), &d, sizeof(S2Desc));
  const int nin = 1 << d.nld, nout = 1 << d.nst;
  uint32_t* lt = reinterpret_cast<uint32_t*>(blob.data() + off_l);
  for (int tid = 0; tid < (1 << kS2LogThreads); ++tid) {
    const int ti = tid & (nin - 1), to = tid & (nout - 1);
    int64_t ldm = 0, stm = 0;
    int lda = 0, sta = 0;
    for (int b = 0; b < kS2LogThreads; ++b) {
      if (b < d.nld && ((ti >> b) & 1)) { ldm += d.ld_w[b]; lda ^= d.ld_a[b]; }
      if (b < d.nst && ((to >> b) & 1)) { stm += d.st_w[b]; sta ^= d.st_a[b]; }
    }
    lt[4 * tid + 0] = (uint32_t)(ldm * (int64_t)esz);
    lt[4 * tid + 1] = (uint32_t)(stm * (int64_t)esz);
    lt[4 * tid + 2] = (uint32_t)lda;
    lt[4 * tid + 3] = (uint32_t)sta;
  }
  if (cb) {
    int64_t* ct = reinterpret_cast<int64_t*>(blob.data() + off_c);
    for (int64_t ch = 0; ch < d.nchunks; ++ch) {
      int64_t bi = 0, bo = 0;
      for (int b = d.logC; b < d.colbits; ++b)
        if ((ch >> (b - d.logC)) & 1) { bi += d.k.w_in[b]; bo += d.k.w_out[b]; }
      ct[2 * ch] = bi;
      ct[2 * ch + 1] = bo;
    }
  }
  return blob;
}

class Compiler {
 public:
  // lanes_hint > 1: the plan will run its slices in batches of that many lanes, so a
  // slice-dependent sweep op needs only min_chunks / lanes chunks to fill the GPU
  // group_hint > 1: the plan will run in lockstep groups of that many plans (blocks as lanes,
  // plan_run_group), so every sweep op shares its launches with group_hint - 1 others
  // min_chunks > 0: the smallest chunk count of a big sweep op (else TQ_S2_MINCHUNKS / 128)
  Compiler(Plan& P, int lanes_hint = 1, int group_hint = 1, int min_chunks = 0)
      : P_(P), lanes_hint_(lanes_hint), group_hint_(std::max(1, group_hint)), min_chunks_(min_chunks) {}

  int run(int n_inputs, const int32_t* in_ranks, const int32_t* in_modes, const int64_t* in_ext,
          const int64_t* in_strides, int out_rank, const int32_t* out_modes, int n_steps,
          const int32_t* path, int n_sliced, const int32_t* sliced) {
    P_.esz = dtype_size(P_.dtype);
    cplx_ = dtype_complex(P_.dtype);
    P_.n_inputs = n_inputs;
    n_inputs_ = n_inputs;
    std::set<int> sl(sliced, sliced + n_sliced);
    TQ_CHECK_ARG((int)sl.size() == n_sliced, "duplicate sliced mode");
    P_.sliced.assign(sliced, sliced + n_sliced);
    P_.sliced_ext.assign(n_sliced, 0);
    // ---- inputs
    size_t cur = 0;
    for (int i = 0; i < n_inputs; ++i) {
      TQ_CHECK_ARG(in_ranks[i] >= 0 && in_ranks[i] <= TQ_MAX_RANK, "input rank");
      InputView v;
      Live L;
      std::vector<int64_t> ext(in_ext + cur, in_ext + cur + in_ranks[i]);
      std::vector<int64_t> st;
      if (in_strides) st.assign(in_strides + cur, in_strides + cur + in_ranks[i]);
      else st = contig_strides(ext);
      v.slice_stride.assign(n_sliced, 0);
      for (int d = 0; d < in_ranks[i]; ++d) {
        const int m = in_modes[cur + d];
        TQ_CHECK_ARG(ext[d] >= 1, "input extent < 1");
        TQ_TRY(note_extent(m, ext[d]));
        for (int q = 0; q < d; ++q)
          TQ_CHECK_ARG(in_modes[cur + q] != m, "repeated mode within one input (diagonal) unsupported");
        auto it = std::find(P_.sliced.begin(), P_.sliced.end(), m);
        if (it != P_.sliced.end()) {
          const int si = (int)(it - P_.sliced.begin());
          v.slice_stride[si] = st[d];
          P_.sliced_ext[si] = ext[d];
          continue;
        }
        v.modes.push_back(m); v.ext.push_back(ext[d]); v.stride.push_back(st[d]);
      }
      cur += in_ranks[i];
      L.modes = v.modes; L.ext = v.ext; L.stride = v.stride;
      L.buf.kind = BUF_INPUT; L.buf.index = i; L.buf.off = 0;
      for (int64_t ss : v.slice_stride) L.dep |= ss != 0;
      P_.inputs.push_back(v);
      live_.push_back(L);
    }
    for (int s = 0; s < n_sliced; ++s) {
      TQ_CHECK_ARG(P_.sliced_ext[s] > 0, "sliced mode not present in any input");
      P_.n_slices *= P_.sliced_ext[s];
    }
    // ---- output
    std::set<int> outset;
    for (int d = 0; d < out_rank; ++d) {
      const int m = out_modes[d];
      TQ_CHECK_ARG(!outset.count(m), "repeated output mode");
      TQ_CHECK_ARG(!sl.count(m), "sliced mode in output");
      TQ_CHECK_ARG(ext_.count(m), "output mode not in any input");
      outset.insert(m);
      P_.out_modes.push_back(m);
      P_.out_ext.push_back(ext_[m]);
    }
    P_.out_numel = prod(P_.out_ext);
    // reference counts: live tensors + output
    for (auto& L : live_) for (int m : L.modes) cnt_[m]++;
    for (int m : P_.out_modes) cnt_[m]++;
    // ---- pre-pass: which SSA ids depend on a sliced input, and which slice-invariant results
    // are read by slice-dependent steps (those are "pinned": kept in a region of their own that
    // no slice-dependent buffer ever reuses, since invariant ops do not re-run per slice)
    {
      std::vector<char> dep(n_inputs + n_steps, 0);
      for (int i = 0; i < n_inputs; ++i) dep[i] = live_[i].dep;
      pinned_.assign(n_inputs + n_steps, 0);
      for (int s = 0; s < n_steps; ++s) {
        const int x = path[2 * s], y = path[2 * s + 1];
        if (x < 0 || y < 0 || x >= n_inputs + s || y >= n_inputs + s) break;  // checked below
        dep[n_inputs + s] = dep[x] || dep[y];
        if (dep[n_inputs + s]) {
          if (!dep[x] && x >= n_inputs) pinned_[x] = 1;
          if (!dep[y] && y >= n_inputs) pinned_[y] = 1;
        }
      }
    }
    // ---- branches: the two subtrees of the join step are independent (run concurrently, arena
    // regions of their own); the join and every step outside its subtrees are branch 2 (region
    // 0).  The join is the step whose smaller subtree holds the most inputs: the final step of a
    // plain partition path, the boundary contraction when the sweeps' tails are absorbed after
    // it (einsum.partition_path defer=...)
    step_branch_.assign(n_steps, 2);
    if (n_steps >= 1) {
      std::vector<int> leaves(n_inputs + n_steps, 1);
      int last = n_steps - 1, best = -1;
      for (int s = 0; s < n_steps; ++s) {
        const int x = path[2 * s], y = path[2 * s + 1];
        if (x < 0 || y < 0 || x >= n_inputs + s || y >= n_inputs + s) break;  // checked below
        leaves[n_inputs + s] = leaves[x] + leaves[y];
        const int m = std::min(leaves[x], leaves[y]);
        if (m >= best) { best = m; last = s; }
      }
      step_branch_[last] = 2;
      for (int side = 0; side < 2; ++side) {
        std::vector<int> stack{path[2 * last + side]};
        while (!stack.empty()) {
          const int id = stack.back();
          stack.pop_back();
          if (id < n_inputs || id - n_inputs >= last) continue;
          step_branch_[id - n_inputs] = side;
          stack.push_back(path[2 * (id - n_inputs)]);
          stack.push_back(path[2 * (id - n_inputs) + 1]);
        }
      }
    }
    // ---- steps
    std::vector<bool> used(n_inputs + n_steps, false);
    for (int s = 0; s < n_steps; ++s) {
      const int x = path[2 * s], y = path[2 * s + 1];
      const int nid = n_inputs + s;
      TQ_CHECK_ARG(x >= 0 && x < nid && y >= 0 && y < nid && x != y, "path id out of range");
      TQ_CHECK_ARG(!used[x] && !used[y], "path uses a tensor twice");
      used[x] = used[y] = true;
      Live res;
      pin_next_ = pinned_[nid];
      br_ = step_branch_[s];
      TQ_TRY(step(s, live_[x], live_[y], s == n_steps - 1, res));
      live_.push_back(res);
    }
    TQ_TRY(flush_chain(false));  // (the final step always closes a chain; kept for safety)
    int remaining = 0, last = -1;
    for (int i = 0; i < n_inputs + n_steps; ++i) if (!used[i]) { ++remaining; last = i; }
    TQ_CHECK_ARG(remaining == 1, "path does not reduce to a single tensor");
    if (n_steps == 0) {
      // single input: permute (and sum) into the output
      Live& L = live_[last];
      for (int m : L.modes)
        TQ_CHECK_ARG(outset.count(m), "single-input trace/sum is unsupported");
      TQ_TRY(emit_permute(L, P_.out_modes, {}, BufRef{BUF_OUTPUT, 0, 0}, true, -1, "copy->out"));
    }
    // arena layout: [region 0][region 1] | pinned: [region 0][region 1]; offsets become absolute
    {
      auto al = [](int64_t b) { return (b + kAlign - 1) / kAlign * kAlign; };
      const int64_t abase[2] = {0, al(arenas_[0].peak())};
      const int64_t pbase[2] = {0, al(pinned_arenas_[0].peak())};
      P_.pinned_base = (size_t)al(abase[1] + arenas_[1].peak());
      P_.arena_bytes = P_.pinned_base + (size_t)(pbase[1] + pinned_arenas_[1].peak());
      P_.lane0_bytes = P_.arena_bytes;
      P_.lanes = 1;
      if (const int want = slice_lanes(); P_.n_slices > 1 && want > 1 && P_.pinned_base > 0) {
        const int64_t cap = std::min<int64_t>({(int64_t)want, P_.n_slices,
                                               (int64_t)(lane_arena_budget() / P_.pinned_base)});
        while (P_.lanes * 2 <= cap) P_.lanes *= 2;   // a power of two
      }
      P_.lane_phys = (size_t)al((int64_t)(P_.arena_bytes - P_.pinned_base));
      P_.lane_stride = P_.pinned_base;
      P_.lane_ws_off = P_.lane_phys + (size_t)P_.lanes * P_.lane_stride;
      P_.arena_bytes = P_.lane_ws_off;   // + the lane-batched GEMM workspace (run(), after lowering)
      // lane-batched GEMMs and their shared workspace
      if (P_.lanes > 1) {
        size_t wsmax = 0;
        for (auto& op : P_.ops) {
          const bool okab = (op.a.kind == BUF_ARENA || op.a.kind == BUF_PINNED) &&
                            (op.b.kind == BUF_ARENA || op.b.kind == BUF_PINNED);
          if (op.kind != OP_GEMM || op.skinny || op.invariant || op.batch != 1 || op.writes_output || !okab ||
              op.c.kind != BUF_ARENA || (P_.lane_stride / P_.esz) % 2)
            continue;
          op.lane_batch = true;
          op.note += " lanes";
          wsmax = std::max(wsmax, gemm_workspace(P_.dtype, op.M, op.N, op.K, P_.lanes));
        }
        // a lane-batched GEMM or a lane-merged sweep2 level (a per-slice op: every lane's copy in
        // one launch) whose result only an output permute reads: sum the lanes first, then permute
        // once per batch instead of once per lane
        for (size_t i = 0; i < P_.ops.size(); ++i) {
          Op& g = P_.ops[i];
          const bool s2 = g.kind == OP_SWEEP2 && !g.s2_dense && !g.invariant && !g.writes_output &&
                          g.c.kind == BUF_ARENA;
          if (!g.lane_batch && !s2) continue;
          const int64_t lo = g.c.off, hi = g.c.off + g.nc;
          int reader = -1, nread = 0;
          for (size_t k = i + 1; k < P_.ops.size(); ++k) {
            const Op& o = P_.ops[k];
            auto rd = [&](const BufRef& r, int64_t n) { return r.kind == BUF_ARENA && r.off < hi && lo < r.off + n; };
            if (rd(o.a, o.na) || rd(o.b, o.nb) || (o.kind == OP_AXPY && rd(o.c, o.nc))) { ++nread; reader = (int)k; }
            for (auto& sg : o.sgates) if (rd(sg.g, std::max<int64_t>(sg.n, 1))) ++nread;
            if (o.c.kind == BUF_ARENA && o.c.off < hi && lo < o.c.off + o.nc) break;   // overwritten
          }
          if (nread != 1) continue;
          Op& pm = P_.ops[reader];
          if (pm.kind != OP_PERMUTE || !pm.writes_output || pm.invariant || pm.a.off != g.c.off) continue;
          g.lane_sum = pm.lane_once = true;
          g.note += " lane-sum";
        }
        P_.lane_ws_bytes = (size_t)al((int64_t)wsmax);
        P_.arena_bytes += P_.lane_ws_bytes;
      }
      const int64_t esz = (int64_t)P_.esz;
      auto fix = [&](BufRef& b) {
        if (b.kind == BUF_ARENA) b.off += abase[b.region] / esz;
        else if (b.kind == BUF_PINNED) b.off += pbase[b.region] / esz;
        b.region = 0;
      };
      for (auto& op : P_.ops) {
        fix(op.a); fix(op.b); fix(op.c); fix(op.ws);
        for (auto& g : op.sgates) fix(g.g);
      }
    }
    assign_amax();
    // table layout
    size_t tb = 0;
    P_.perm_tab_off.clear();
    for (auto& pp : P_.perms) {
      P_.perm_tab_off.push_back(tb);
      tb += (perm_plan_table_bytes(pp) + kAlign - 1) / kAlign * kAlign;
    }
    P_.gtab_off.clear();
    for (auto& g : P_.gtabs) {
      P_.gtab_off.push_back(tb);
      tb += (g.size() * sizeof(int32_t) + kAlign - 1) / kAlign * kAlign;
    }
    P_.stab_off.clear();
    for (auto& b : P_.stabs) {
      P_.stab_off.push_back(tb);
      tb += (b.size() + kAlign - 1) / kAlign * kAlign;
    }
    // constant operands in the tables (the compose ops' identity matrices): BufRef::index = blob
    for (auto& op : P_.ops)
      for (BufRef* r : {&op.a, &op.b})
        if (r->kind == BUF_TABLE) r->off = (int64_t)P_.stab_off[r->index];
    P_.amax_off = tb;
    // per-slice words: one set per slice lane (every lane's operands scaled by their own max)
    tb += ((size_t)(P_.n_amax_once + P_.n_amax_slice * std::max(1, P_.lanes)) * sizeof(uint32_t) + kAlign - 1) /
          kAlign * kAlign;
    P_.sc_off = tb;
    tb += ((size_t)P_.n_amax_slice * sizeof(int32_t) + kAlign - 1) / kAlign * kAlign;
    P_.bad_off = tb;
    if (P_.n_ps) tb += ((size_t)P_.n_slices * sizeof(uint32_t) + kAlign - 1) / kAlign * kAlign;
    P_.table_bytes = tb;
    for (auto& op : P_.ops) {
      (op.invariant ? P_.flops_once : P_.flops_slice) += op.flops;
      (op.invariant ? P_.bytes_once : P_.bytes_slice) += op.bytes;
      P_.n_gemm += op.kind == OP_GEMM;
      P_.n_apply += op.kind == OP_APPLY;
      P_.n_permute += op.kind == OP_PERMUTE;
      P_.n_sweep += op.kind == OP_SWEEP || op.kind == OP_SWEEP2;
      if (op.kind == OP_SWEEP || op.kind == OP_SWEEP2) P_.n_sweep_gates += (int)op.sgates.size();
    }
    build_schedule();
    // cooperative chain counters (S2Launch::sync): a 256-byte slot each, behind the other tables
    // (zero from the upload; every launch leaves its counter at zero)
    P_.sync_off = P_.table_bytes;
    P_.table_bytes += P_.coop_once.size() * Plan::kSyncSlot;
    P_.flops = P_.flops_once + P_.flops_slice * (double)P_.n_slices;
    P_.bytes = P_.bytes_once + P_.bytes_slice * (double)P_.n_slices;
    std::ostringstream d;
    for (size_t i = 0; i < P_.ops.size(); ++i)
      d << (P_.ops[i].invariant ? "[once]  " : "[slice] ") << "b" << P_.ops[i].branch << " "
        << P_.ops[i].note << "\n";
    d << "# schedule (launch: op indices)\n";
    for (int set = 0; set < 2; ++set)
      for (auto& g : set == 0 ? P_.sched_once : P_.sched_slice) {
        d << "# " << (set == 0 ? "once " : "slice");
        for (int j : g) d << " " << j;
        d << "\n";
      }
    for (auto& r : P_.seq_once) {
      d << "# chain launch (a workgroup per stream, one-chunk layouts): once entries " << r.first << ".."
        << r.second - 1 << ", ops";
      for (int i = r.first; i < r.second; ++i)
        for (int j : P_.sched_once[i])
          d << " " << j << "/s" << P_.seq_stream[j] << ((P_.ops[j].lds_io & 1) ? "<" : "")
            << ((P_.ops[j].lds_io & 2) ? ">" : "");
      d << "   (< input from LDS, > result left in LDS)\n";
    }
    for (size_t r = 0; r < P_.coop_once.size(); ++r) {
      d << "# cooperative chain launch (" << P_.coop_width[r]
        << " workgroups, a counter barrier between ops): once entries " << P_.coop_once[r].first << ".."
        << P_.coop_once[r].second - 1 << ", ops";
      for (int i = P_.coop_once[r].first; i < P_.coop_once[r].second; ++i) d << " " << P_.sched_once[i][0];
      d << "\n";
    }
    P_.describe = d.str();
    return TQ_OK;
  }

  // Operand-max words for the complex64 f16-split GEMM (tq_gemm.hip): when a GEMM that can take
  // the K-outer fast path reads an operand that one sweep2 op stored in full (same buffer, same
  // element count, no other writer in between), that sweep op max-es |re|, |im| of what it
  // stores into a word the GEMM reads, instead of the GEMM re-reading both operands (1 GiB per
  // C4 slice) for their max.  Words of slice-invariant producers are zeroed once per execute
  // call, the others before every slice.
  void assign_amax() {
    P_.n_amax_once = P_.n_amax_slice = 0;
    if (P_.dtype != TQ_C64) return;
    const int64_t esz = (int64_t)P_.esz;
    auto span = [&](const BufRef& b, int64_t n, int* space, int64_t* lo, int64_t* hi) {
      if (b.kind == BUF_ARENA) { *space = 0; *lo = b.off * esz; }
      else if (b.kind == BUF_PINNED) { *space = 0; *lo = (int64_t)P_.pinned_base + b.off * esz; }
      else if (b.kind == BUF_OUTPUT) { *space = 1; *lo = b.off * esz; }
      else return false;
      *hi = *lo + n * esz;
      return true;
    };
    std::vector<int> once, slice;  // producer op indices, in word order
    auto producer = [&](int gi, const BufRef& r, int64_t n) -> int {
      int sp, spw;
      int64_t lo, hi, wlo, whi;
      if (!span(r, n, &sp, &lo, &hi)) return -1;
      for (int j = gi - 1; j >= 0; --j) {
        const Op& w = P_.ops[j];
        if (!span(w.c, w.nc, &spw, &wlo, &whi)) continue;
        if (spw != sp || whi <= lo || hi <= wlo) continue;
        // the latest writer of these bytes: usable only if it stored exactly this operand
        if (w.kind == OP_SWEEP2 && !w.writes_output && wlo == lo && whi == hi) return j;
        return -1;
      }
      return -1;
    };
    std::vector<int> prod_a(P_.ops.size(), -1), prod_b(P_.ops.size(), -1);
    for (size_t i = 0; i < P_.ops.size(); ++i) {
      const Op& g = P_.ops[i];
      if (g.kind != OP_GEMM || g.transA != 1 || g.transB != 0) continue;
      if (g.M % 128 || g.N % 128 || g.K % 16 || g.lda % 2 || g.ldb % 2) continue;
      if (g.lda >= (int64_t(1) << 24) || g.ldb >= (int64_t(1) << 24)) continue;
      if (g.batch > 1 && (g.sA % 2 || g.sB % 2)) continue;
      const int pa = producer((int)i, g.a, g.na), pb = producer((int)i, g.b, g.nb);
      if (pa < 0 || pb < 0) continue;
      prod_a[i] = pa;
      prod_b[i] = pb;
      for (int j : {pa, pb}) {
        auto& v = P_.ops[j].invariant ? once : slice;
        if (std::find(v.begin(), v.end(), j) == v.end()) v.push_back(j);
      }
    }
    // the pre-split boundary GEMM (tq_gemmp.hip): a per-slice GEMM whose operands are each stored
    // in full by one per-slice dense sweep op and read by nothing else; those ops then store the
    // operand as six f16 term planes, scaled from a bound built on the max of their own input,
    // whose producer (a sweep2 op storing exactly that input) gets a max word too.  The largest
    // such GEMM of the plan (C4 / C3: the boundary contraction of the cut network)
    P_.planes_gemm = -1;
    std::vector<int> planes_x(P_.ops.size(), -1);
    if (planes_enabled()) {
      auto only_reader = [&](int j, int gi) {
        int sp, spo;
        int64_t lo, hi, olo, ohi;
        const Op& w = P_.ops[j];
        if (!span(w.c, w.nc, &sp, &lo, &hi)) return false;
        auto hits = [&](const BufRef& r, int64_t n) {
          return span(r, n, &spo, &olo, &ohi) && spo == sp && olo < hi && lo < ohi;
        };
        for (size_t k = j + 1; k < P_.ops.size(); ++k) {
          const Op& o = P_.ops[k];
          if ((int)k != gi) {
            if (hits(o.a, o.na) || hits(o.b, o.nb) || (o.kind == OP_AXPY && hits(o.c, o.nc))) return false;
            for (auto& g : o.sgates) if (hits(g.g, std::max<int64_t>(g.n, 1))) return false;
          }
          if (hits(o.c, o.nc) || (o.nws && hits(o.ws, o.nws))) break;
        }
        return true;
      };
      double best = 0;
      for (size_t i = 0; i < P_.ops.size(); ++i) {
        const Op& g = P_.ops[i];
        const int pa = prod_a[i], pb = prod_b[i];
        if (pa < 0 || pa == pb || g.invariant || g.batch != 1 || g.writes_output || g.skinny) continue;
        if (!planes_gemm_ok(g.M, g.N, g.K, g.lda, g.ldb)) continue;
        const Op& da = P_.ops[pa];
        const Op& db = P_.ops[pb];
        if (!da.s2_dense || !db.s2_dense || da.invariant || db.invariant || da.writes_output || db.writes_output) continue;
        if (!only_reader(pa, (int)i) || !only_reader(pb, (int)i)) continue;
        const int xa = producer(pa, da.a, da.na), xb = producer(pb, db.a, db.na);
        if (xa < 0 || xb < 0 || P_.ops[xa].s2_dense || P_.ops[xb].s2_dense) continue;
        if (P_.ops[xa].invariant != P_.ops[xb].invariant) continue;
        const double w = (double)g.M * g.N * g.K;
        if (w > best) {
          best = w;
          P_.planes_gemm = (int)i;
          planes_x[pa] = xa;
          planes_x[pb] = xb;
        }
      }
      if (P_.planes_gemm >= 0) {
        const Op& g = P_.ops[P_.planes_gemm];
        const int pab[2] = {prod_a[P_.planes_gemm], prod_b[P_.planes_gemm]};
        for (int r = 0; r < 2; ++r) {
          const int j = pab[r], x = planes_x[j];
          P_.ops[j].planes_role = r + 1;
          auto& v = P_.ops[x].invariant ? once : slice;
          if (std::find(v.begin(), v.end(), x) == v.end()) v.push_back(x);
          // the planes (12 B per element) replace the complex64 store (8 B)
          P_.ops[j].bytes += (double)P_.ops[j].nc * 4.0;
          P_.ops[j].note += r ? " planes(B)" : " planes(A)";
        }
        P_.planes_n[0] = g.na;
        P_.planes_n[1] = g.nb;
        P_.ops[P_.planes_gemm].note += " planes";
      }
    }
    P_.n_amax_once = (int)once.size();
    P_.n_amax_slice = (int)slice.size();
    for (size_t q = 0; q < once.size(); ++q) P_.ops[once[q]].amax_word = (int)q;
    for (size_t q = 0; q < slice.size(); ++q) P_.ops[slice[q]].amax_word = P_.n_amax_once + (int)q;
    for (size_t j = 0; j < P_.ops.size(); ++j)
      if (P_.ops[j].planes_role) P_.ops[j].planes_in_amax = P_.ops[planes_x[j]].amax_word;
    for (size_t i = 0; i < P_.ops.size(); ++i) {
      if (prod_a[i] < 0) continue;
      P_.ops[i].amax_a = P_.ops[prod_a[i]].amax_word;
      P_.ops[i].amax_b = P_.ops[prod_b[i]].amax_word;
      P_.ops[i].note += " amax<-op" + std::to_string(prod_a[i]) + ",op" + std::to_string(prod_b[i]);
    }
    // pre-split candidates: per-slice GEMM, per-slice producers that store nothing else read
    // (scan forward from the producer until its bytes are overwritten), batch 1, no beta
    P_.n_ps = 0;
    auto exclusive = [&](int j, int gi) {
      int sp, spo;
      int64_t lo, hi, olo, ohi;
      const Op& w = P_.ops[j];
      if (!span(w.c, w.nc, &sp, &lo, &hi)) return false;
      auto hits = [&](const BufRef& r, int64_t n) {
        return span(r, n, &spo, &olo, &ohi) && spo == sp && olo < hi && lo < ohi;
      };
      for (size_t k = j + 1; k < P_.ops.size(); ++k) {
        const Op& o = P_.ops[k];
        if ((int)k != gi) {
          if (hits(o.a, o.na) || hits(o.b, o.nb) || (o.kind == OP_AXPY && hits(o.c, o.nc))) return false;
          for (auto& g : o.sgates) if (hits(g.g, std::max<int64_t>(g.n, 1))) return false;
        }
        if (hits(o.c, o.nc) || (o.nws && hits(o.ws, o.nws))) break;
      }
      return true;
    };
    const int64_t max_slices = 1 << 16;
    for (size_t i = 0; i < P_.ops.size(); ++i) {
      Op& g = P_.ops[i];
      const int pa = prod_a[i], pb = prod_b[i];
      if (pa < 0 || pa == pb || g.invariant || g.batch != 1 || P_.n_slices > max_slices) continue;
      if ((int)i == P_.planes_gemm) continue;
      if (P_.ops[pa].invariant || P_.ops[pb].invariant) continue;
      if (P_.ops[pa].ps_gemm >= 0 || P_.ops[pb].ps_gemm >= 0) continue;
      if (!exclusive(pa, (int)i) || !exclusive(pb, (int)i)) continue;
      g.ps_cand = true;
      P_.ops[pa].ps_gemm = P_.ops[pb].ps_gemm = (int)i;
      g.note += " presplit";
      ++P_.n_ps;
    }
  }

  // Launch schedule.  Ops of one set (slice-invariant / per slice) are ordered by dependency
  // level: an op's level is one more than that of every earlier op it conflicts with (RAW, WAR
  // or WAW on overlapping bytes of the arena, the output or a workspace; inputs are read-only).
  // Ops of one level commute, so the independent in-place sweeps of a level (e.g. the left and
  // right subtrees of a cut network, or the tiny vector pre-absorption chains) share a launch.
  void build_schedule() {
    struct Acc { int space; int64_t lo, hi; };
    const int64_t esz = (int64_t)P_.esz;
    auto add = [&](std::vector<Acc>& v, const BufRef& b, int64_t n) {
      if (n <= 0) return;
      switch (b.kind) {
        case BUF_ARENA: v.push_back({0, b.off * esz, (b.off + n) * esz}); break;
        case BUF_PINNED:
          v.push_back({0, (int64_t)P_.pinned_base + b.off * esz, (int64_t)P_.pinned_base + (b.off + n) * esz});
          break;
        case BUF_OUTPUT: v.push_back({1, b.off * esz, (b.off + n) * esz}); break;
        default: break;  // inputs are never written
      }
    };
    const size_t n = P_.ops.size();
    std::vector<std::vector<Acc>> rd(n), wr(n);
    for (size_t i = 0; i < n; ++i) {
      const Op& op = P_.ops[i];
      add(rd[i], op.a, op.na);
      add(rd[i], op.b, op.nb);
      add(wr[i], op.c, op.nc);
      add(rd[i], op.c, op.nc);    // beta accumulation reads the target
      add(wr[i], op.ws, op.nws);
      add(rd[i], op.ws, op.nws);
      for (auto& g : op.sgates) add(rd[i], g.g, g.n);
    }
    auto overlap = [](const std::vector<Acc>& x, const std::vector<Acc>& y) {
      for (auto& a : x)
        for (auto& b : y)
          if (a.space == b.space && a.lo < b.hi && b.lo < a.hi) return true;
      return false;
    };
    for (int set = 0; set < 2; ++set) {
      std::vector<int> ids;
      for (size_t i = 0; i < n; ++i) if (P_.ops[i].invariant == (set == 0)) ids.push_back((int)i);
      std::vector<int> lev(ids.size(), 0);
      int maxlev = -1;
      for (size_t b = 0; b < ids.size(); ++b) {
        const int j = ids[b];
        for (size_t a = 0; a < b; ++a) {
          const int i = ids[a];
          if (lev[a] + 1 <= lev[b]) continue;
          if (overlap(wr[i], rd[j]) || overlap(wr[i], wr[j]) || overlap(rd[i], wr[j])) lev[b] = lev[a] + 1;
        }
        maxlev = std::max(maxlev, lev[b]);
      }
      auto& sched = set == 0 ? P_.sched_once : P_.sched_slice;
      sched.clear();
      for (int L = 0; L <= maxlev; ++L) {
        std::vector<int> grp;
        for (size_t b = 0; b < ids.size(); ++b) {
          if (lev[b] != L) continue;
          const int j = ids[b];
          if (P_.ops[j].kind != OP_SWEEP2) { sched.push_back({j}); continue; }
          grp.push_back(j);
          if ((int)grp.size() == kS2MaxOps) { sched.push_back(grp); grp.clear(); }
        }
        if (!grp.empty()) sched.push_back(grp);
      }
    }
    P_.n_launch_once = (int)P_.sched_once.size();
    P_.n_launch_slice = (int)P_.sched_slice.size();
    // chain launches: consecutive hoisted levels that are each one small sweep2 op (C2's whole
    // contraction, the first levels of C3 / C4's hoisted chains: 1-4 workgroups per launch) run
    // in order by one workgroup in one launch
    // Levels of several such ops (the left and right halves of a cut network) run as several
    // streams of one launch, a workgroup each, when every op conflicts (RAW / WAR / WAW) with
    // earlier ops of at most one stream: that stream's workgroup runs it after them.
    P_.seq_once.clear();
    P_.seq_stream.assign(n, -1);
    P_.use_seq = s2_seq_enabled();
    auto chainable = [&](const std::vector<int>& g) {
      if (g.empty() || (int)g.size() > kS2SeqMaxStreams) return false;
      for (int j : g) {
        const Op& op = P_.ops[j];
        if (op.kind != OP_SWEEP2 || op.s2_dense || op.stab1 < 0) return false;
      }
      return true;
    };
    auto conflict = [&](int i, int j) {
      return overlap(wr[i], rd[j]) || overlap(wr[i], wr[j]) || overlap(rd[i], wr[j]);
    };
    const int ns = (int)P_.sched_once.size();
    for (int i = 0; i < ns;) {
      if (!chainable(P_.sched_once[i])) { ++i; continue; }
      std::vector<int> in_run;   // ops of the run so far
      int nstreams = 0, nops = 0, e = i;
      for (; e < ns && chainable(P_.sched_once[e]); ++e) {
        const auto& g = P_.sched_once[e];
        if (nops + (int)g.size() > kS2MaxOps) break;
        std::vector<int> st(g.size(), -1);
        int fresh = nstreams;
        bool ok = true;
        for (size_t q = 0; q < g.size() && ok; ++q) {
          int s = -1;
          for (int k : in_run)
            if (conflict(k, g[q])) {
              if (s >= 0 && P_.seq_stream[k] != s) { ok = false; break; }
              s = P_.seq_stream[k];
            }
          st[q] = s >= 0 ? s : fresh++;
        }
        if (!ok || fresh > kS2SeqMaxStreams) break;
        for (size_t q = 0; q < g.size(); ++q) { P_.seq_stream[g[q]] = st[q]; in_run.push_back(g[q]); }
        nstreams = fresh;
        nops += (int)g.size();
      }
      if (e - i >= 2) {
        P_.seq_once.push_back({i, e});
      } else {
        for (int k : in_run) P_.seq_stream[k] = -1;
        e = std::max(e, i + 1);
      }
      i = e;
    }
    // LDS hand-offs inside a chain launch: op j's result stays in the workgroup's LDS for the
    // next op k of its stream when k reads exactly that tensor, it fits 64 KiB, and no other op
    // reads it before it is overwritten (true reads: a, b, gate tensors; the scan follows the
    // execution order: the rest of the hoisted launches, then every per-slice launch)
    for (auto& o : P_.ops) o.lds_io = 0;
    std::vector<int> order;   // execution order of the ops (hoisted, then per slice)
    for (auto& g : P_.sched_once) for (int j : g) order.push_back(j);
    for (auto& g : P_.sched_slice) for (int j : g) order.push_back(j);
    std::vector<int> at(n, -1);
    for (size_t q = 0; q < order.size(); ++q) at[order[q]] = (int)q;
    auto true_reads = [&](int i) {
      std::vector<Acc> v;
      const Op& op = P_.ops[i];
      add(v, op.a, op.na);
      add(v, op.b, op.nb);
      for (auto& g : op.sgates) add(v, g.g, g.n);
      return v;
    };
    for (auto& r : P_.seq_once) {
      std::vector<int> run;
      for (int i = r.first; i < r.second; ++i) for (int j : P_.sched_once[i]) run.push_back(j);
      // bit 2: no op of the launch writes this op's gate tensors (prefetch while the previous
      // op of its stream runs)
      for (int k : run) {
        std::vector<Acc> gr;
        for (auto& g : P_.ops[k].sgates) add(gr, g.g, g.n);
        bool clean = true;
        for (int i : run) clean = clean && !overlap(wr[i], gr);
        if (clean && s2_seq_prefetch()) P_.ops[k].lds_io |= 4;
      }
      for (size_t x = 0; x < run.size(); ++x) {
        const int j = run[x];
        int k = -1;
        for (size_t y = x + 1; y < run.size() && k < 0; ++y)
          if (P_.seq_stream[run[y]] == P_.seq_stream[j]) k = run[y];
        if (k < 0) continue;
        const Op& oj = P_.ops[j];
        const Op& ok = P_.ops[k];
        if (oj.writes_output || oj.amax_word >= 0 || oj.ps_gemm >= 0 || oj.c.kind != ok.a.kind ||
            oj.c.off != ok.a.off || oj.c.index != ok.a.index || oj.c.region != ok.a.region || oj.nc != ok.na || oj.nc * esz > kS2ChunkBytes)
          continue;
        std::vector<Acc> out;
        add(out, oj.c, oj.nc);
        if (out.size() != 1) continue;
        bool alone = true;
        for (size_t q = (size_t)at[j] + 1; q < order.size() && alone; ++q) {
          const int i = order[q];
          if (i == k) continue;
          if (overlap(true_reads(i), out)) { alone = false; break; }
          std::vector<Acc> w;
          add(w, P_.ops[i].c, P_.ops[i].nc);
          add(w, P_.ops[i].ws, P_.ops[i].nws);
          bool covered = false;
          for (auto& a : w) covered = covered || (a.space == out[0].space && a.lo <= out[0].lo && a.hi >= out[0].hi);
          if (covered) break;   // overwritten: no later op reads j's values
        }
        if (!alone) continue;
        P_.ops[j].lds_io |= 2;
        P_.ops[k].lds_io |= 1;
      }
    }
    // cooperative chain launches: consecutive hoisted levels that are each ONE multi-chunk sweep2
    // op outside a chain launch (C2: 27 levels of 4-chunk ops after its one-chunk chain) run as
    // one launch of n workgroups, every op's chunks spread over all of them and a counter barrier
    // between consecutive ops (S2Launch::sync).  Plain ops only (no beta / max / split / output:
    // their stores and loads are the coherent forms), and no op of a run writes a gate tensor of
    // the run (gates are read through the caches, and prefetched)
    P_.coop_once.clear();
    P_.coop_width.clear();
    P_.use_coop = s2_coop_enabled();
    std::vector<char> in_chain(ns, 0);
    for (auto& r : P_.seq_once)
      for (int i = r.first; i < r.second; ++i) in_chain[i] = 1;
    auto coop_ok = [&](int i) {
      if (in_chain[i] || P_.sched_once[i].size() != 1) return false;
      const Op& op = P_.ops[P_.sched_once[i][0]];
      return op.kind == OP_SWEEP2 && !op.s2_dense && !op.writes_output && op.amax_word < 0 && op.ps_gemm < 0 &&
             op.s2_nchunks >= 2 && op.s2_nchunks <= s2_coop_max_chunks();
    };
    for (int i = 0; i < ns;) {
      if (!coop_ok(i)) { ++i; continue; }
      std::vector<Acc> gates, writes;
      int e = i;
      for (; e < ns && coop_ok(e) && e - i < kS2MaxOps; ++e) {
        const int j = P_.sched_once[e][0];
        std::vector<Acc> g;
        for (auto& sg : P_.ops[j].sgates) add(g, sg.g, sg.n);
        if (overlap(wr[j], gates) || overlap(writes, g) || overlap(wr[j], g)) break;
        gates.insert(gates.end(), g.begin(), g.end());
        writes.insert(writes.end(), wr[j].begin(), wr[j].end());
      }
      if (e - i >= 2) {
        // workgroups: the most common chunk count of the run (an op of more chunks strides them)
        std::vector<int> cnt(17, 0);
        for (int q = i; q < e; ++q) ++cnt[(int)P_.ops[P_.sched_once[q][0]].s2_nchunks];
        int w = 2;
        for (int c = 2; c <= 16; ++c) if (cnt[c] > cnt[w]) w = c;
        P_.coop_once.push_back({i, e});
        P_.coop_width.push_back(std::min(w, kS2SeqMaxStreams));
        // the next op's descriptor and gates prefetched (no op of the run writes a gate of it)
        for (int q = i; q < e; ++q) P_.ops[P_.sched_once[q][0]].lds_io = s2_seq_prefetch() ? 4 : 0;
      }
      i = std::max(e, i + 1);
    }
  }
  // cooperative chain launches (TQ_S2_COOP=1, default 0; tq_plan_set "sweep_coop") for levels of
  // ops of at most TQ_S2_COOPCH chunks (default 16).  Measured r04 (C2, complex64, 26 levels in
  // one launch of 4 workgroups): 0.379 ms against 0.363 one launch per level -- the launch gaps
  // it removes (~1.7 us each, 46 us in all) come back as longer ops (write-through stores
  // drained before the arrival, the poll, L2-missing loads: +1.1 us per op), so it is off
  static bool s2_coop_enabled() {
    static const bool v = [] {
      const char* e = getenv("TQ_S2_COOP");
      return e && e[0] == '1';
    }();
    return v;
  }
  static int s2_coop_max_chunks() {
    static const int v = [] {
      const char* e = getenv("TQ_S2_COOPCH");
      return e ? std::min(16, atoi(e)) : 16;
    }();
    return v;
  }
  // chain launches take small ops of at most this many chunks, in their one-chunk layout
  // (TQ_S2_SEQCH, default 2).  Measured r04: C2's 29 levels of 4-chunk ops as one chain are
  // 0.404 ms against 0.363 one launch per level on a fast box -- ~6 us of gate passes per op on
  // ONE CU cost more than the ~3 us launch gap they save -- though 0.596 against 0.677 on a box
  // with slow memory round trips; C3's 2-chunk levels: 0.677 against 0.684 ms
  static int s2_seq_max_chunks() {
    static const int v = [] {
      const char* e = getenv("TQ_S2_SEQCH");
      return e ? atoi(e) : 2;
    }();
    return v;
  }
  // chain launches: the next op's descriptor prefetched (TQ_S2_SEQPF, default 1)
  static bool s2_seq_prefetch() {
    static const bool v = [] {
      const char* e = getenv("TQ_S2_SEQPF");
      return !(e && e[0] == '0');
    }();
    return v;
  }
  // chain launches on (TQ_S2_SEQ, default 1; tq_plan_set "sweep_chain" per plan)
  static bool s2_seq_enabled() {
    static const bool v = [] {
      const char* e = getenv("TQ_S2_SEQ");
      return !(e && e[0] == '0');
    }();
    return v;
  }

 private:
  int note_extent(int m, int64_t e) {
    auto it = ext_.find(m);
    if (it == ext_.end()) { ext_[m] = e; return TQ_OK; }
    if (it->second != e) {
      set_error("invalid argument: mode " + std::to_string(m) + " has inconsistent extents");
      return TQ_ERR_INVALID;
    }
    return TQ_OK;
  }

  int region() const { return br_ == 1 ? 1 : 0; }
  BufRef new_buf(int64_t numel, int64_t* off_out) {
    const int64_t off = arenas_[region()].alloc(numel * (int64_t)P_.esz);
    *off_out = off;
    BufRef b;
    b.kind = BUF_ARENA;
    b.off = off / (int64_t)P_.esz;
    b.region = region();
    return b;
  }
  void release(const Live& L) {
    if (L.owned && L.buf.kind == BUF_ARENA) arenas_[L.buf.region].release(L.buf.off * (int64_t)P_.esz);
  }
  // the step result's buffer: pinned results live in the separate pinned region
  BufRef new_result_buf(int64_t numel, int64_t* off_out) {
    if (!pin_next_) return new_buf(numel, off_out);
    const int64_t off = pinned_arenas_[region()].alloc(numel * (int64_t)P_.esz);
    *off_out = off;
    BufRef b;
    b.kind = BUF_PINNED;
    b.off = off / (int64_t)P_.esz;
    b.region = region();
    return b;
  }

  // permute X into contiguous `order` (+ broadcast modes `bcast` with stride 0) at dst
  int emit_permute(const Live& X, const std::vector<int>& order, const std::map<int, int64_t>& bcast,
                   BufRef dst, bool to_output, int step, const std::string& why) {
    std::vector<int64_t> shape, sst;
    for (int m : order) {
      const int p = X.pos(m);
      if (p >= 0) { shape.push_back(X.ext[p]); sst.push_back(X.stride[p]); }
      else {
        auto it = bcast.find(m);
        if (it == bcast.end()) { set_error("internal: permute mode missing"); return TQ_ERR_INVALID; }
        shape.push_back(it->second); sst.push_back(0);
      }
    }
    PermPlan pp;
    TQ_TRY(build_perm_plan(P_.dtype, (int)shape.size(), shape.data(), sst.data(), &pp));
    Op op;
    op.kind = OP_PERMUTE;
    op.a = X.buf;
    op.c = dst;
    op.writes_output = to_output;
    op.perm = (int)P_.perms.size();
    op.step = step;
    const int64_t n = prod(shape);
    op.na = X.numel();
    op.nc = n;
    op.bytes = 2.0 * n * P_.esz;
    std::ostringstream o;
    o << "step " << step << " PERMUTE " << why << " " << modes_str(X.modes) << "->" << modes_str(order)
      << " n=" << n << " [" << perm_plan_kind(pp) << "]" << (to_output ? " ->OUT" : "");
    op.note = o.str();
    P_.perms.push_back(std::move(pp));
    P_.ops.push_back(op);
    return TQ_OK;
  }

  static bool runs_equal(const std::vector<int>& modes, const std::vector<std::vector<int>>& runs) {
    size_t k = 0;
    for (auto& r : runs)
      for (int m : r) {
        if (k >= modes.size() || modes[k] != m) return false;
        ++k;
      }
    return k == modes.size();
  }

  std::vector<int> filter(const std::vector<int>& modes, const std::set<int>& s) {
    std::vector<int> r;
    for (int m : modes) if (s.count(m)) r.push_back(m);
    return r;
  }

  int64_t ext_of(const std::vector<int>& ms) {
    int64_t p = 1;
    for (int m : ms) p *= ext_[m];
    return p;
  }

  int step(int s, Live A0, Live B0, bool final, Live& res) {
    for (int m : A0.modes) cnt_[m]--;
    for (int m : B0.modes) cnt_[m]--;
    std::set<int> inA(A0.modes.begin(), A0.modes.end()), inB(B0.modes.begin(), B0.modes.end());
    std::set<int> batch, contr, freeA, freeB, sumA, sumB;
    for (int m : A0.modes) {
      const bool need = cnt_[m] > 0;
      if (inB.count(m)) (need ? batch : contr).insert(m);
      else (need ? freeA : sumA).insert(m);
    }
    for (int m : B0.modes) if (!inA.count(m)) (cnt_[m] > 0 ? freeB : sumB).insert(m);
    const bool dep = A0.dep || B0.dep;
    const int nid = n_inputs_ + s;

    ApplyDesc d;
    const bool can_apply = apply_desc(A0, B0, batch, contr, sumA, sumB, d);
    // ---- fused sweep chains: an APPLY whose big operand is the open chain's result extends it
    if (chain_.active) {
      const bool pendA = A0.buf.kind == BUF_PENDING, pendB = B0.buf.kind == BUF_PENDING;
      bool extended = false;
      if (can_apply && (d.a_big ? pendA : pendB) && !(d.a_big ? pendB : pendA) && dep == chain_.dep &&
          br_ == chain_.br) {
        Chain::Gate g = make_gate(s, d, d.a_big ? B0 : A0, d.a_big ? A0 : B0, dep);
        chain_.gates.push_back(g);
        ChainShape sh;
        if (sweeps_enabled() && chain_shape(chain_, d.order, sh)) {
          chain_.out_modes = d.order;
          chain_.id = nid;
          extended = true;
        } else {
          chain_.gates.pop_back();
        }
      }
      if (!extended) {
        TQ_TRY(flush_chain(false));
        // the flushed result now has a real buffer: refresh this step's copies
        if (A0.buf.kind == BUF_PENDING) A0 = live_[chain_.flushed_id];
        if (B0.buf.kind == BUF_PENDING) B0 = live_[chain_.flushed_id];
      } else {
        res.modes = d.order;
        for (int m : d.order) res.ext.push_back(ext_[m]);
        res.stride = contig_strides(res.ext);
        res.buf = BufRef{BUF_PENDING, nid, 0};
        res.owned = true;
        res.dep = dep;
        for (int m : res.modes) cnt_[m]++;
        if (final) {
          live_.push_back(res);  // flush patches live_[id]; the caller's push is replaced below
          TQ_TRY(flush_chain(true));
          res = live_.back();
          live_.pop_back();
        }
        return TQ_OK;
      }
    }
    const size_t first_op = P_.ops.size();
    if (can_apply && !final && sweeps_enabled() && A0.buf.kind != BUF_PENDING &&
        B0.buf.kind != BUF_PENDING) {
      // open a chain with this gate (emitted at flush: as APPLY if it stays a single gate)
      chain_ = Chain{};
      chain_.active = true;
      chain_.dep = dep;
      chain_.br = br_;
      chain_.X0 = d.a_big ? A0 : B0;
      chain_.release_X0 = !(dep && !chain_.X0.dep);
      chain_.gates.push_back(make_gate(s, d, d.a_big ? B0 : A0, d.a_big ? A0 : B0, dep));
      chain_.out_modes = d.order;
      chain_.id = nid;
      ChainShape sh;
      if (chain_shape(chain_, d.order, sh)) {
        res.modes = d.order;
        for (int m : d.order) res.ext.push_back(ext_[m]);
        res.stride = contig_strides(res.ext);
        res.buf = BufRef{BUF_PENDING, nid, 0};
        res.owned = true;
        res.dep = dep;
        for (int m : res.modes) cnt_[m]++;
        return TQ_OK;
      }
      chain_ = Chain{};  // does not fit a sweep tile: plain APPLY below
    }
    if (can_apply) {
      TQ_TRY(emit_apply(s, d, final, A0, B0, res));
    } else {
      TQ_TRY(gemm_step(s, A0, B0, final, batch, contr, freeA, freeB, sumA, sumB, res));
    }
    for (int m : res.modes) cnt_[m]++;
    // slice-invariant hoisting: a step that reads no sliced input runs once per execute; its
    // result is pinned in the arena when a slice-dependent step consumes it
    res.dep = dep;
    for (size_t k = first_op; k < P_.ops.size(); ++k) {
      P_.ops[k].invariant = !res.dep;
      P_.ops[k].branch = br_;
    }
    if (!(res.dep && !A0.dep)) release(A0);
    if (!(res.dep && !B0.dep)) release(B0);
    return TQ_OK;
  }

  // write the step result either straight into the output (final step, matching order)
  // or into a fresh arena buffer (then permuted to the output if final).
  BufRef result_target(bool final, const std::vector<int>& order, int64_t numel, bool* direct,
                       int64_t* off) {
    *direct = final && order == P_.out_modes;
    if (*direct) { *off = -1; return BufRef{BUF_OUTPUT, 0, 0}; }
    return new_result_buf(numel, off);
  }

  // ---- APPLY lowering: big operand S = [O][K1][M][K2][I] (contracted modes in <= 2 runs),
  // small operand G[K][N] read through a gather table, C = [O][N][M][I]
  struct ApplyDesc {
    bool a_big = true;
    std::vector<int> korder, nfree, order;
    int64_t O = 1, K1 = 1, M = 1, K2 = 1, I = 1, K = 1, N = 1;
    std::vector<int32_t> gtab;   // empty: small operand already contiguous in [K][N] order
  };

  bool apply_desc(const Live& A0, const Live& B0, const std::set<int>& batch,
                  const std::set<int>& contr, const std::set<int>& sumA, const std::set<int>& sumB,
                  ApplyDesc& d) {
    if (!batch.empty() || !sumA.empty() || !sumB.empty() || contr.empty()) return false;
    d.a_big = A0.numel() >= B0.numel();
    const Live& Bg = d.a_big ? A0 : B0;
    const Live& Sm = d.a_big ? B0 : A0;
    if (Bg.buf.kind != BUF_PENDING && !Bg.contiguous()) return false;
    d.K = ext_of(std::vector<int>(contr.begin(), contr.end()));
    d.N = Sm.numel() / d.K;
    if (Sm.numel() > 1024 || d.K > 32 || d.N > 32) return false;
    std::vector<std::pair<int, int>> runs;  // (start, length)
    for (int i = 0; i < (int)Bg.modes.size(); ++i) {
      if (!contr.count(Bg.modes[i])) continue;
      if (!runs.empty() && runs.back().first + runs.back().second == i) runs.back().second++;
      else runs.push_back({i, 1});
    }
    if (runs.empty() || runs.size() > 2) return false;
    const int p1 = runs[0].first, c1 = runs[0].second;
    const int p2 = runs.size() == 2 ? runs[1].first : p1 + c1;
    const int c2 = runs.size() == 2 ? runs[1].second : 0;
    d.korder.assign(Bg.modes.begin() + p1, Bg.modes.begin() + p1 + c1);
    d.korder.insert(d.korder.end(), Bg.modes.begin() + p2, Bg.modes.begin() + p2 + c2);
    for (int m : Sm.modes) if (!contr.count(m)) d.nfree.push_back(m);
    std::vector<int> gorder = d.korder;
    gorder.insert(gorder.end(), d.nfree.begin(), d.nfree.end());
    if (!(Sm.contiguous() && Sm.modes == gorder)) {
      std::vector<int64_t> gext, gst;
      for (int m : gorder) {
        const int p = Sm.pos(m);
        gext.push_back(Sm.ext[p]);
        gst.push_back(Sm.stride[p]);
      }
      const int64_t n = prod(gext);
      d.gtab.resize(n);
      for (int64_t t = 0; t < n; ++t) {
        int64_t rem = t, off = 0;
        for (int q = (int)gext.size() - 1; q >= 0; --q) { off += (rem % gext[q]) * gst[q]; rem /= gext[q]; }
        d.gtab[t] = (int32_t)off;
      }
    }
    d.order.assign(Bg.modes.begin(), Bg.modes.begin() + p1);
    d.order.insert(d.order.end(), d.nfree.begin(), d.nfree.end());
    d.order.insert(d.order.end(), Bg.modes.begin() + p1 + c1, Bg.modes.begin() + p2);
    d.order.insert(d.order.end(), Bg.modes.begin() + p2 + c2, Bg.modes.end());
    for (int i = 0; i < p1; ++i) d.O *= Bg.ext[i];
    for (int i = p1; i < p1 + c1; ++i) d.K1 *= Bg.ext[i];
    for (int i = p1 + c1; i < p2; ++i) d.M *= Bg.ext[i];
    for (int i = p2; i < p2 + c2; ++i) d.K2 *= Bg.ext[i];
    for (size_t i = p2 + c2; i < Bg.modes.size(); ++i) d.I *= Bg.ext[i];
    return true;
  }

  int add_gtab(const std::vector<int32_t>& t) {
    if (t.empty()) return -1;
    P_.gtabs.push_back(t);
    return (int)P_.gtabs.size() - 1;
  }

  int emit_apply(int s, const ApplyDesc& d, bool final, const Live& A0, const Live& B0, Live& res) {
    const Live& Bg = d.a_big ? A0 : B0;
    const Live& Sm = d.a_big ? B0 : A0;
    const int64_t outn = d.O * d.N * d.M * d.I;
    bool direct;
    int64_t roff;
    BufRef tgt = result_target(final, d.order, outn, &direct, &roff);
    Op op;
    op.kind = OP_APPLY;
    op.a = Bg.buf;
    op.b = Sm.buf;
    op.gtab = add_gtab(d.gtab);
    op.c = tgt;
    op.writes_output = direct;
    op.O = d.O; op.K = d.K1; op.M = d.M; op.K2 = d.K2; op.N = d.N; op.I = d.I;
    op.na = d.O * d.K1 * d.M * d.K2 * d.I;
    op.nb = Sm.numel();
    op.nc = outn;
    op.step = s;
    op.flops = (double)d.O * d.M * d.I * d.K * d.N * (cplx_ ? 8.0 : 2.0);
    op.bytes = (double)(d.O * d.K * d.M * d.I + outn + d.K * d.N) * P_.esz;
    std::ostringstream o;
    o << "step " << s << " APPLY O=" << d.O << " K1=" << d.K1 << " M=" << d.M << " K2=" << d.K2
      << " I=" << d.I << " N=" << d.N << (direct ? " ->OUT" : "");
    op.note = o.str();
    P_.ops.push_back(op);
    res.modes = d.order;
    res.ext.clear();
    for (int m : d.order) res.ext.push_back(ext_[m]);
    res.stride = contig_strides(res.ext);
    res.buf = tgt;
    res.owned = !direct;
    if (final && !direct)
      TQ_TRY(emit_permute(res, P_.out_modes, {}, BufRef{BUF_OUTPUT, 0, 0}, true, s, "result->out"));
    return TQ_OK;
  }

  // ---- sweep chains ------------------------------------------------------------------------
  struct Chain {
    struct Gate {
      Live Sm;
      bool release = true;
      int step = -1;
      ApplyDesc d;
    };
    bool active = false;
    bool dep = false;
    int br = 0;           // branch of its steps
    int id = -1;          // SSA id of the (pending) chain result
    int flushed_id = -1;
    Live X0;
    bool release_X0 = true;
    std::vector<Gate> gates;
    std::vector<int> out_modes;
  };
  struct ChainShape {
    bool s2 = false;      // fits the in-place butterfly sweep (tq_sweep2.hip)
    std::vector<int> tin, tout, outer;
    std::vector<std::vector<int>> W;   // working-set mode lists after each gate (W[q-1] = tout)
    int64_t tin_n = 1, tout_n = 1, wmax = 1;
  };

  static bool sweeps_enabled() {
    static const int v = [] {
      const char* e = getenv("TQ_SWEEP");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    return v != 0;
  }

  Chain::Gate make_gate(int s, const ApplyDesc& d, const Live& Sm, const Live& Bg, bool dep) {
    Chain::Gate g;
    g.Sm = Sm;
    g.step = s;
    g.d = d;
    (void)Bg;
    g.release = !(dep && !Sm.dep);
    return g;
  }

  int64_t count_of(const std::vector<int>& ms) { return ext_of(ms); }

  // tile modes / working sets of a chain; false if it does not fit the sweep kernel's limits
  bool chain_shape(const Chain& c, const std::vector<int>& out_modes, ChainShape& sh) {
    if ((int)c.gates.size() > std::max(kSweepMaxGates, kS2MaxGates)) return false;
    std::set<int> contracted;
    for (auto& g : c.gates) {
      if (g.d.K * g.d.N > kSweepMaxKN) return false;
      contracted.insert(g.d.korder.begin(), g.d.korder.end());
    }
    for (int m : c.X0.modes) (contracted.count(m) ? sh.tin : sh.outer).push_back(m);
    std::vector<int> w = sh.tin;
    sh.W.clear();
    for (size_t j = 0; j < c.gates.size(); ++j) {
      const auto& g = c.gates[j];
      std::vector<int> nw;
      for (int m : w) if (std::find(g.d.korder.begin(), g.d.korder.end(), m) == g.d.korder.end()) nw.push_back(m);
      for (int m : g.d.korder)
        if (std::find(w.begin(), w.end(), m) == w.end()) return false;  // contracts an outer mode
      nw.insert(nw.end(), g.d.nfree.begin(), g.d.nfree.end());
      w = nw;
      sh.W.push_back(w);
      sh.wmax = std::max(sh.wmax, count_of(w));
    }
    std::set<int> wset(w.begin(), w.end());
    for (int m : out_modes) if (wset.count(m)) sh.tout.push_back(m);
    if (sh.tout.size() != w.size()) return false;
    sh.W.back() = sh.tout;
    // untouched modes keep their relative order (APPLY preserves it)
    std::vector<int> outer_y;
    for (int m : out_modes) if (!wset.count(m)) outer_y.push_back(m);
    if (outer_y != sh.outer) return false;
    sh.tin_n = count_of(sh.tin);
    sh.tout_n = count_of(sh.tout);
    sh.wmax = std::max({sh.wmax, sh.tin_n, sh.tout_n});
    int64_t tab = 0;
    for (size_t j = 0; j < c.gates.size(); ++j) tab += count_of(sh.W[j]) * (c.gates[j].d.K + 1);
    const bool old_ok = (int)c.gates.size() <= kSweepMaxGates && sh.wmax <= sweep_wmax((int)P_.esz) &&
                        tab <= kSweepTabMax;
    {
      S2Desc scratch;  // the full layout (every limit checked), so flush_chain cannot fail on it
      sh.s2 = s2_layout(c, sh, out_modes, &scratch);
    }
    return old_ok || sh.s2;
  }

  static int ilog2(int64_t v) {
    if (v <= 0 || (v & (v - 1))) return -1;
    int l = 0;
    while ((int64_t(1) << l) < v) ++l;
    return l;
  }
  static int64_t s2_small_elems() {
    static const int64_t v = [] {
      const char* e = getenv("TQ_S2_SMALL");
      return e ? (int64_t)atoll(e) : (int64_t(1) << 22);
    }();
    return v;
  }
  // chunks a big sweep2 op is split into at least (TQ_S2_MINCHUNKS): 128 since r05 (the deferred
  // C4 path's 2^19-element levels, two halves per launch: 0.766 -> 0.747 ms per block, two blocks
  // in flight 0.565 -> 0.520; C2 / C3 +-0; 64 / 512: 0.80 / 0.88, profiles/knobs_r05.txt)
  static int s2_min_chunks() {
    static const int v = [] {
      const char* e = getenv("TQ_S2_MINCHUNKS");
      return e ? atoi(e) : 128;
    }();
    return v;
  }
  // slices per batch when the per-slice working set is small (TQ_SLICE_LANES, default 32; 1 = off;
  // C3 with the capped sweep2 launches: 1.27 ms per step at 8 lanes, 1.18 at 16; r04 with 32-op
  // sweep2 launches: 0.778 -> 0.726 ms at 32 (two launches per per-slice level, half the GEMM /
  // reduce / permute batches), profiles/knobs_r04.jsonl)
  // arena the lane copies may add in total (TQ_LANE_ARENA_MB, default 6 GiB of the 288 GB):
  // C3's 6-MiB per-slice part gets 16 lanes, C4's 1.1 GiB gets 4 (measured: 16.4 -> 15.9 ms/step)
  static size_t lane_arena_budget() {
    static const size_t v = [] {
      const char* e = getenv("TQ_LANE_ARENA_MB");
      return (size_t)(e ? std::max(0, atoi(e)) : 6144) << 20;
    }();
    return v;
  }
  static int slice_lanes() {
    static const int v = [] {
      const char* e = getenv("TQ_SLICE_LANES");
      return e ? std::max(1, std::min(64, atoi(e))) : 32;
    }();
    return v;
  }
  // narrowest chunk (log2 columns) of the small-tensor rule (TQ_S2_MINLC; 1 since r04: with the
  // 32-lane batches and 4096-element register-block tiles C2 0.399 -> 0.365 ms, C3 0.786 ->
  // 0.700, C4 N = 8 rank 2.21 -> 2.12, profiles/knobs_r04.jsonl; r03 measured 2 better alone)
  // TQ_S2_SWZ=0: sweep2 tiles keep the r04 column-only swizzle instead of the modeled one
  static bool s2_swz_model() {
    static const bool v = [] {
      const char* e = getenv("TQ_S2_SWZ");
      return !(e && atoi(e) == 0);
    }();
    return v;
  }
  // TQ_S2_LANEBLK=1: register blocks of 6 positions over 4 lanes (lane blocks; off by default:
  // 28 % fewer passes on C4's big sweep ops, the same time -- DESIGN.md §3.3)
  static bool s2_lane_blocks() {
    static const bool v = [] {
      const char* e = getenv("TQ_S2_LANEBLK");
      return e && atoi(e) != 0;
    }();
    return v;
  }
  // TQ_S2_WAVELOCAL=0: a workgroup barrier between every two sweep2 passes
  static bool s2_wave_local() {
    static const bool v = [] {
      const char* e = getenv("TQ_S2_WAVELOCAL");
      return !(e && atoi(e) == 0);
    }();
    return v;
  }
  static int s2_min_logc() {
    static const int v = [] {
      const char* e = getenv("TQ_S2_MINLC");
      return e ? std::max(0, std::min(5, atoi(e))) : 1;
    }();
    return v;
  }
  // ... for tiles of >= 2^9 positions (TQ_S2_MINLC_BIG, default 0: one column): such a chunk
  // holds >= 512 elements per column, so a narrower chunk halves a workgroup's gate-pass VALU
  // (passes are VALU-issue bound, probes/pass_probe.hip) and doubles the workgroups.  Measured
  // r04 (C2: 26 levels of 1024-position tiles, 2 -> 1 column, 4 -> 8 chunks): 0.323 -> 0.303 ms;
  // applied to every small tensor it left C3 / the C4 N = 8 rank +-0.4 % (not kept there)
  static int s2_min_logc_big() {
    static const int v = [] {
      const char* e = getenv("TQ_S2_MINLC_BIG");
      return e ? std::max(0, std::min(5, atoi(e))) : 0;
    }();
    return v;
  }
  // narrowest chunk (log2 columns) of a sweep2 op before the tile / min-chunk caps (TQ_S2_LC):
  // 7 since r03 (C3's per-slice ops, 128-element tiles: 32 -> 128 columns per chunk, 1.16 ->
  // 1.04 ms per step with the capped launches; C4 and C2 +-0; 8-10 no better)
  static int s2_base_logc() {
    static const int v = [] {
      const char* e = getenv("TQ_S2_LC");
      return e ? std::max(0, std::min(10, atoi(e))) : 7;
    }();
    return v;
  }
  static bool s2_blocks_enabled() {
    static const int v = [] {
      const char* e = getenv("TQ_S2_BLOCKS");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    return v != 0;
  }
  static bool s2_epi_enabled() {
    static const int v = [] {
      const char* e = getenv("TQ_S2_EPI");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    return v != 0;
  }
  static bool s2_enabled() {
    static const int v = [] {
      const char* e = getenv("TQ_SWEEP2");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    return v != 0;
  }
  // the pre-split boundary GEMM (TQ_GEMM_PLANES=0: the GEMM-side split kernel instead)
  static bool planes_enabled() {
    static const int v = [] {
      const char* e = getenv("TQ_GEMM_PLANES");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    return v != 0;
  }
  static bool s2_dense_enabled() {
    static const int v = [] {
      const char* e = getenv("TQ_S2_DENSE");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    return v != 0;
  }
  // Dense form of a sweep chain (tq_sweepd.hip): complex64, a small input tile (tin <= 16), an
  // output tile of <= 256, a big tensor (>= 2^20 output elements), and the six lowest column bits
  // memory-fastest and contiguous in X and Y (a wave's 64 lanes = 64 consecutive elements).
  bool s2_dense_layout(const Chain& c, const ChainShape& sh, const std::vector<int>& out_modes, S2Dense* dd) {
    if (!s2_dense_enabled() || P_.dtype != TQ_C64 || !c.X0.contiguous()) return false;
    // whole 32-output MFMA tiles (tq_sweepd.hip)
    if (sh.tin_n < 2 || sh.tin_n > kS2DMaxTin || sh.tout_n < 32 || sh.tout_n > kS2DMaxTout || sh.tout_n % 32)
      return false;
    if (ilog2(sh.tin_n) < 0 || ilog2(sh.tout_n) < 0) return false;
    std::map<int, int64_t> sx, sy;
    {
      auto cs = contig_strides(c.X0.ext);
      for (size_t q = 0; q < c.X0.modes.size(); ++q) sx[c.X0.modes[q]] = cs[q];
      std::vector<int64_t> ye;
      for (int m : out_modes) ye.push_back(ext_[m]);
      auto cy = contig_strides(ye);
      for (size_t q = 0; q < out_modes.size(); ++q) sy[out_modes[q]] = cy[q];
    }
    std::vector<std::pair<int64_t, int64_t>> cb;
    for (int m : sh.outer) {
      const int nb = ilog2(ext_[m]);
      if (nb < 0) return false;
      for (int i = 0; i < nb; ++i) cb.push_back({sx[m] << i, sy.at(m) << i});
    }
    std::sort(cb.begin(), cb.end());
    if (cb.size() < 6 || (int)cb.size() > kS2MaxColBits) return false;
    for (int b = 0; b < 6; ++b)
      if (cb[b].first != (int64_t(1) << b) || cb[b].second != (int64_t(1) << b)) return false;
    const int64_t ncols = int64_t(1) << cb.size();
    if (ncols * sh.tout_n < (int64_t(1) << 20)) return false;
    dd->ncols = ncols;
    dd->colbits = (int)cb.size();
    dd->tin = (int)sh.tin_n;
    dd->tout = (int)sh.tout_n;
    for (size_t b = 0; b < cb.size(); ++b) { dd->w_in[b] = cb[b].first; dd->w_out[b] = cb[b].second; }
    std::map<int, int64_t> dig;
    for (int64_t t = 0; t < sh.tin_n; ++t) {
      digits(t, sh.tin, dig);
      int64_t o = 0;
      for (int m : sh.tin) o += dig[m] * sx[m];
      if (o >= (int64_t(1) << 31)) return false;   // staged as int32 by the kernel
      dd->in_off[t] = o;
    }
    for (int64_t t = 0; t < sh.tout_n; ++t) {
      digits(t, sh.tout, dig);
      int64_t o = 0;
      for (int m : sh.tout) o += dig[m] * sy.at(m);
      if (o >= (int64_t(1) << 31)) return false;   // the kernel stages them as int32
      dd->out_off[t] = o;
    }
    return true;
  }

  // GF(2) rank of a few small bit vectors
  static int gf2_rank(std::vector<int> v) {
    int r = 0;
    for (int bit = 31; bit >= 0; --bit) {
      int piv = -1;
      for (size_t i = r; i < v.size(); ++i) if ((v[i] >> bit) & 1) { piv = (int)i; break; }
      if (piv < 0) continue;
      std::swap(v[r], v[piv]);
      for (size_t i = 0; i < v.size(); ++i) if ((int)i != r && ((v[i] >> bit) & 1)) v[i] ^= v[r];
      ++r;
    }
    return r;
  }

  // TQ_S2_REORDER (default 1): commute a chain's square gates into fuller register blocks
  static bool s2_reorder_on() {
    static const bool v = [] {
      const char* e = getenv("TQ_S2_REORDER");
      return !(e && e[0] == '0');
    }();
    return v;
  }

  // Register blocks take CONSECUTIVE square gates whose positions fit B bits (s2_layout
  // block_span).  A brick-wall chain lists a layer's gates before the next layer's, so the greedy
  // run closes a block at every layer's edge: (0,1)(2,3) | (4,5)(6,7) | (1,2)(3,4) ...  Square gates
  // on disjoint positions commute (a square gate's outputs take its inputs' positions), so within
  // each maximal run of square gates the gates are re-listed block by block: a block starts at
  // the first unscheduled gate and takes every later gate whose overlapping predecessors (in the
  // chain's order) are already scheduled or in the block, while the block's positions fit B bits.
  // The result is a linear extension of the overlap order: per amplitude the same products,
  // summed in another order of commuting factors (the rounding differs, the value does not).
  // Non-square gates (expanding / contracting the working set) stay where they are.  False if
  // the order is unchanged.
  bool s2_reorder_squares(const Chain& c, Chain& out, int B) {
    const int ng = (int)c.gates.size();
    if (ng < 3) return false;
    auto nbits = [&](int m) { return ilog2(ext_[m]); };
    std::map<std::pair<int, int>, int> slot;   // (mode, bit) -> slot: s2_layout's positions, relabelled
    int next = 0;
    for (int m : c.X0.modes) for (int i = 0; i < nbits(m); ++i) slot[{m, i}] = next++;
    std::vector<std::vector<int>> sl(ng);
    std::vector<char> sq(ng, 0);
    for (int j = 0; j < ng; ++j) {
      const auto& g = c.gates[j];
      std::vector<int> freed;
      for (auto it = g.d.korder.rbegin(); it != g.d.korder.rend(); ++it)
        for (int i = 0; i < nbits(*it); ++i) {
          auto f = slot.find({*it, i});
          if (f == slot.end()) return false;
          freed.push_back(f->second);
          slot.erase(f);
        }
      size_t fi = 0, nout = 0;
      sl[j] = freed;
      for (auto it = g.d.nfree.rbegin(); it != g.d.nfree.rend(); ++it)
        for (int i = 0; i < nbits(*it); ++i, ++nout) {
          const int s = fi < freed.size() ? freed[fi++] : next++;
          slot[{*it, i}] = s;
          if (nout >= freed.size()) sl[j].push_back(s);
        }
      sq[j] = g.d.K == g.d.N && (g.d.K == 2 || g.d.K == 4) && nout == freed.size();
    }
    auto overlap = [&](int a, int b) {
      for (int x : sl[a]) for (int y : sl[b]) if (x == y) return true;
      return false;
    };
    std::vector<int> order;
    std::vector<char> done(ng, 0), inblk(ng, 0);
    for (int j = 0; j < ng;) {
      if (!sq[j]) { order.push_back(j++); continue; }
      int e = j;
      while (e < ng && sq[e]) ++e;
      std::vector<int> rem;
      for (int q = j; q < e; ++q) rem.push_back(q);
      while (!rem.empty()) {
        std::vector<int> blk{rem[0]}, U = sl[rem[0]];
        inblk[rem[0]] = 1;
        for (size_t t = 1; t < rem.size() && (int)blk.size() < kS2BlkMaxGates; ++t) {
          const int g = rem[t];
          bool ready = true;
          for (int h = j; h < g && ready; ++h) if (!done[h] && !inblk[h] && overlap(h, g)) ready = false;
          if (!ready) continue;
          std::vector<int> u2 = U;
          for (int x : sl[g]) if (std::find(u2.begin(), u2.end(), x) == u2.end()) u2.push_back(x);
          if ((int)u2.size() > B) continue;
          U = u2;
          blk.push_back(g);
          inblk[g] = 1;
        }
        for (int g : blk) {
          done[g] = 1;
          inblk[g] = 0;
          order.push_back(g);
          rem.erase(std::find(rem.begin(), rem.end(), g));
        }
      }
      j = e;
    }
    bool same = true;
    for (int j = 0; j < ng; ++j) same = same && order[j] == j;
    if (same) return false;
    out = c;
    for (int j = 0; j < ng; ++j) out.gates[j] = c.gates[order[j]];
    return true;
  }

  // Layout of an in-place butterfly sweep (tq_sweep2.hip): every mode bit of the working set
  // gets a tile position (input tile bits memory-fastest first; a gate's outputs reuse the
  // positions it frees), the columns are the untouched mode bits ordered by stride, and a
  // per-position XOR swizzle keeps the half-wave LDS accesses of the load / store phases
  // conflict-free.  False if the chain does not fit (non power-of-two extents, K or N > 8,
  // more than s2_max_pos live bits).
  bool s2_layout(const Chain& c, const ChainShape& sh, const std::vector<int>& out_modes,
                 S2Desc* out) {
    if (!s2_enabled() || c.gates.empty() || (int)c.gates.size() > kS2MaxGates) return false;
    // tiles beyond 2^(chunk bits - 5) positions leave fewer than 32 columns per chunk and the
    // gate passes 2- to 4-way LDS bank conflicts: only small (latency-bound) tensors use them,
    // where the longer chains save launches
    int maxpos = s2_max_pos((int)P_.esz);
    {
      int64_t nx = 1, ny = 1;
      for (int m : c.X0.modes) nx *= ext_[m];
      for (int m : out_modes) ny *= ext_[m];
      if (std::max(nx, ny) > s2_small_elems()) maxpos = std::min(maxpos, s2_chunk_bits((int)P_.esz) - 5);
    }
    auto nbits = [&](int m) { return ilog2(ext_[m]); };
    for (int m : c.X0.modes) if (nbits(m) < 0) return false;
    if (!c.X0.contiguous()) return false;
    for (auto& g : c.gates) {
      if (g.d.K > kS2MaxK || g.d.N > kS2MaxKN) return false;
      for (int m : g.d.nfree) if (nbits(m) < 0) return false;
    }
    std::map<int, int64_t> sx, sy;
    {
      auto cs = contig_strides(c.X0.ext);
      for (size_t q = 0; q < c.X0.modes.size(); ++q) sx[c.X0.modes[q]] = cs[q];
      std::vector<int64_t> ye;
      for (int m : out_modes) ye.push_back(ext_[m]);
      auto cy = contig_strides(ye);
      for (size_t q = 0; q < out_modes.size(); ++q) sy[out_modes[q]] = cy[q];
    }
    typedef std::pair<int, int> MB;  // (mode, bit of its index)
    std::map<MB, int> pos;
    std::vector<std::pair<int64_t, MB>> tb;
    for (int m : sh.tin) for (int i = 0; i < nbits(m); ++i) tb.push_back({sx[m] << i, {m, i}});
    std::sort(tb.begin(), tb.end());
    uint32_t live = 0;
    int used = 0;
    for (auto& t : tb) {
      if (used >= maxpos) return false;
      pos[t.second] = used;
      live |= 1u << used;
      ++used;
    }
    const std::map<MB, int> pos_in = pos;
    S2Desc d;
    d.ngates = (int)c.gates.size();
    std::vector<std::vector<int>> kdep(c.gates.size()), ndep(c.gates.size());
    std::vector<int> last_np;   // output positions of the last gate, index bit order
    int last_nk = 0;            // its input index bits (they are the first output bits)
    for (size_t j = 0; j < c.gates.size(); ++j) {
      const auto& g = c.gates[j];
      std::vector<MB> kb, nb;   // index bits, least significant first
      for (auto it = g.d.korder.rbegin(); it != g.d.korder.rend(); ++it)
        for (int i = 0; i < nbits(*it); ++i) kb.push_back({*it, i});
      for (auto it = g.d.nfree.rbegin(); it != g.d.nfree.rend(); ++it)
        for (int i = 0; i < nbits(*it); ++i) nb.push_back({*it, i});
      if ((int64_t(1) << kb.size()) != g.d.K || (int64_t(1) << nb.size()) != g.d.N) return false;
      uint32_t kmask = 0;
      std::vector<int> freed, kp;
      for (auto& b : kb) {
        auto f = pos.find(b);
        if (f == pos.end()) return false;
        kmask |= 1u << f->second;
        freed.push_back(f->second);
        kp.push_back(f->second);
        pos.erase(f);
      }
      S2Gate& G = d.gate[j];
      G.K = (int)g.d.K;
      G.N = (int)g.d.N;
      G.pass_mask = live & ~kmask;
      live &= ~kmask;
      std::vector<int> np;
      size_t fi = 0;
      for (auto& b : nb) {
        int p;
        if (fi < freed.size()) p = freed[fi++];
        else {
          p = 0;
          while (p < maxpos && ((live >> p) & 1)) ++p;
          if (p >= maxpos) return false;
        }
        pos[b] = p;
        live |= 1u << p;
        np.push_back(p);
        used = std::max(used, p + 1);
      }
      if (j + 1 == c.gates.size()) { last_np = np; last_nk = (int)kp.size(); }
      for (int k = 0; k < G.K; ++k) {
        int v = 0;
        for (size_t t = 0; t < kp.size(); ++t) if ((k >> t) & 1) v |= 1 << kp[t];
        kdep[j].push_back(v);
      }
      for (int n = 0; n < G.N; ++n) {
        int v = 0;
        for (size_t t = 0; t < np.size(); ++t) if ((n >> t) & 1) v |= 1 << np[t];
        ndep[j].push_back(v);
      }
      for (int t = 0; t < G.K * G.N; ++t) {
        G.gidx[t] = g.d.gtab.empty() ? t : g.d.gtab[t];
        if (G.gidx[t] >= kS2GateRaw) return false;   // the kernel stages kS2GateRaw elements per gate
        d.cgidx[j][t] = (uint8_t)G.gidx[t];
      }
    }
    // the final working set must be the output tile
    {
      std::set<MB> want;
      for (int m : sh.tout) for (int i = 0; i < nbits(m); ++i) want.insert({m, i});
      std::set<MB> have;
      for (auto& kv : pos) have.insert(kv.first);
      if (want != have) return false;
    }
    if (!out) return true;
    // columns: untouched mode bits by increasing stride
    std::vector<std::pair<int64_t, int64_t>> cb;  // (stride in X, stride in Y)
    for (int m : sh.outer) for (int i = 0; i < nbits(m); ++i) cb.push_back({sx[m] << i, sy.at(m) << i});
    std::sort(cb.begin(), cb.end());
    if ((int)cb.size() > kS2MaxColBits) return false;
    d.colbits = (int)cb.size();
    d.ncols = int64_t(1) << d.colbits;
    for (size_t j = 0; j < cb.size(); ++j) { d.k.w_in[j] = cb[j].first; d.k.w_out[j] = cb[j].second; }
    const int lc_cap = s2_chunk_bits((int)P_.esz) - used;
    if (lc_cap < 0) return false;
    int lc = std::max(s2_base_logc(), d.colbits - 10);
    lc = std::min(lc, lc_cap);
    lc = std::min(lc, d.colbits);
    // small tensors: narrower chunks, so that the op still spreads over >= s2_min_chunks()
    // workgroups (a 2^19-element tensor with a 256-element tile has only 64 chunks of 32 columns)
    if (const int mc = std::max(1, (min_chunks_ > 0 ? min_chunks_ : s2_min_chunks()) /
                                       (group_hint_ * ((c.dep && lanes_hint_ > 1) ? lanes_hint_ : 1)));
        mc > 1) {
      int lg = 0;
      while ((2 << lg) <= mc) ++lg;
      const int minlc = used >= 9 ? std::min(s2_min_logc(), s2_min_logc_big()) : s2_min_logc();
      lc = std::min(lc, std::max(std::min(minlc, d.colbits), d.colbits - lg));
    }
    if (one_chunk_) lc = std::min(lc_cap, d.colbits);   // the chain-launch form (Op::stab1)
    d.logC = lc;
    d.nchunks = int64_t(1) << (d.colbits - lc);
    // load / store enumerations: chunk bits by increasing memory stride
    struct CBit { int64_t w; int col; int pos; };  // col >= 0: column bit, else tile position
    std::vector<CBit> ld, st;
    for (int j = 0; j < lc; ++j) { ld.push_back({cb[j].first, j, -1}); st.push_back({cb[j].second, j, -1}); }
    for (auto& kv : pos_in) ld.push_back({sx[kv.first.first] << kv.first.second, -1, kv.second});
    for (auto& kv : pos) st.push_back({sy.at(kv.first.first) << kv.first.second, -1, kv.second});
    auto by_w = [](const CBit& a, const CBit& b) { return a.w < b.w; };
    std::sort(ld.begin(), ld.end(), by_w);
    std::sort(st.begin(), st.end(), by_w);
    // Store-phase epilogue: the last gate (K <= N, its inputs on the first output positions) is
    // applied in registers while the tile leaves LDS -- one LDS write + read of the largest
    // working set and one barrier less per chunk.  Its output position bits move to the lowest
    // register-slot bits of the store enumeration (the lane bits keep the smallest strides);
    // the positions it adds are not live before it, so input k sits in slot r0 + k.
    // register blocks of consecutive square gates (S2Desc::pmeta): the pass starting at gate j
    // ends before block_span(j, ng); bm = its block positions, live = the live positions
    // TQ_S2_B4MIN: the smallest tile (elements) that gets 16-element register blocks (default
    // 4096 since r04: a 4096-element tile then leaves half the threads idle in its block passes,
    // but needs fewer passes -- C2 0.386 -> 0.370 ms, C4 N = 8 rank -0.3 %; 8192 before)
    static const int64_t b4min = [] {
      const char* e = getenv("TQ_S2_B4MIN");
      return e ? (int64_t)atoll(e) : (int64_t)4096;
    }();
    const int64_t tile_elems = int64_t(1) << (lc + used);
    const int B = (P_.esz <= 8 && tile_elems >= b4min) ? 4 : s2_block_bits((int)P_.esz, tile_elems);
    auto kmask_of = [&](int j) {
      uint32_t m = 0;
      for (int k = 0; k < d.gate[j].K; ++k) m |= (uint32_t)kdep[j][k];
      return m;
    };
    auto square = [&](int j) {
      const S2Gate& G = d.gate[j];
      if (G.K != G.N || (G.K != 2 && G.K != 4)) return false;
      for (int k = 0; k < G.K; ++k) if (kdep[j][k] != ndep[j][k]) return false;
      return true;
    };
    const bool blocks = s2_blocks_enabled();
    auto block_span = [&](int j, int ng, uint32_t* bm_out, uint32_t* live_out) {
      int e = j + 1;
      uint32_t bm = 0, live = 0;
      if (blocks && square(j)) {
        bm = kmask_of(j);
        live = d.gate[j].pass_mask | bm;
        while (e < ng && e - j < kS2BlkMaxGates && square(e) &&
               __builtin_popcount(bm | kmask_of(e)) <= B)
          bm |= kmask_of(e), ++e;
      }
      if (e - j >= 2) {
        // pad the block with untouched live positions up to B bits (fewer, larger groups)
        for (int q = 0; q < kS2MaxPos && __builtin_popcount(bm) < B; ++q)
          if (((live >> q) & 1) && !((bm >> q) & 1)) bm |= 1u << q;
        if (__builtin_popcount(bm) != B) e = j + 1;
      }
      *bm_out = bm;
      *live_out = live;
      return e;
    };
    // Lane blocks (TQ_S2_LANEBLK): a register block over 6 positions, 4 in a thread's registers
    // and 2 on its lane bits 4 and 5 (group-index bits 4 and 5: the other 3 threads of the block
    // are lanes l ^ 16, l ^ 32, l ^ 48 of the same wave).  A gate whose position sits on a lane
    // bit first trades it with a register bit the gate does not use (a swap: v_permlane16 /
    // 32_swap, 2 instructions per element pair and dword; the register position evicted is the
    // one used again latest).  C4's light-cone staircases hold 3 gates in 4 positions and 5 in 6:
    // about 40 % fewer LDS passes on its big sweep ops for ~0.3 swaps per gate (r06 model).
    struct PPlan {
      int first = 0, end = 0;          // gates [first, end)
      bool block = false, lanes = false;
      uint32_t bm = 0, mask = 0;       // block positions (plain: B of them; lane: the 4 start
                                       // registers), group positions (pass mask)
      int reg0[4] = {}, reg1[4] = {};  // lane block: register bits' positions at start / end
      int ln0[2] = {}, ln1[2] = {};    // lane bits 4 / 5: positions at start / end
      std::vector<std::array<int, 3>> ops;   // lane block: {gate, slot i, slot j (-1: 2x2)} or {-1, lane bit, slot}
      std::vector<int> order;          // group-index bits (after the columns) -> position
    };
    const bool lane_ok = s2_lane_blocks() && blocks && B == 4 && d.logC <= 4;
    auto ascending = [](uint32_t m) {
      std::vector<int> v;
      for (; m; m &= m - 1) v.push_back(__builtin_ctz(m));
      return v;
    };
    auto lane_span = [&](int j, int ng, int e4, PPlan& lp) {
      if (!lane_ok || !square(j)) return false;
      const uint32_t live = d.gate[j].pass_mask | kmask_of(j);
      int e = j + 1;
      uint32_t u = kmask_of(j);
      while (e < ng && e - j < kS2BlkMaxGates && square(e) && __builtin_popcount(u | kmask_of(e)) <= 6)
        u |= kmask_of(e), ++e;
      for (; e > e4 && e - j >= 2; --e) {
        // positions in order of first use, then untouched live positions (they stay on the lanes)
        std::vector<int> first_use;
        for (int q = j; q < e; ++q)
          for (int p : ascending(kmask_of(q)))
            if (std::find(first_use.begin(), first_use.end(), p) == first_use.end()) first_use.push_back(p);
        if (first_use.size() <= 4 || first_use.size() > 6) continue;
        uint32_t padded = 0;
        for (int p : first_use) padded |= 1u << p;
        for (int p : ascending(live & ~padded)) {
          if (first_use.size() >= 6) break;
          first_use.push_back(p);
          padded |= 1u << p;
        }
        if (first_use.size() != 6) return false;
        const std::vector<int> oth = ascending(live & ~padded);
        if ((int)oth.size() < 4 - d.logC) return false;
        int reg[4], ln[2];
        for (int b = 0; b < 4; ++b) reg[b] = first_use[b];
        ln[0] = first_use[4];
        ln[1] = first_use[5];
        PPlan r;
        r.first = j;
        r.end = e;
        r.block = r.lanes = true;
        std::copy(reg, reg + 4, r.reg0);
        std::copy(ln, ln + 2, r.ln0);
        auto slot = [&](int p) {
          for (int b = 0; b < 4; ++b) if (reg[b] == p) return b;
          return -1;
        };
        for (int q = j; q < e; ++q) {
          const std::vector<int> gp = ascending(kmask_of(q));
          for (int p : gp) {
            if (slot(p) >= 0) continue;
            const int l = ln[0] == p ? 0 : 1;
            // evict the register position (not this gate's) whose next use is latest
            int best = -1, best_next = -1;
            for (int b = 0; b < 4; ++b) {
              if (std::find(gp.begin(), gp.end(), reg[b]) != gp.end()) continue;
              int nx = 1 << 20;
              for (int t = q + 1; t < e; ++t)
                if ((kmask_of(t) >> reg[b]) & 1) { nx = t; break; }
              if (nx > best_next) best_next = nx, best = b;
            }
            r.ops.push_back({-1, l, best});
            std::swap(reg[best], ln[l]);
          }
          // index bit t of the gate <-> position of input k = 1 << t
          const int i0 = slot(__builtin_ctz((uint32_t)kdep[q][1]));
          const int j0 = d.gate[q].K == 4 ? slot(__builtin_ctz((uint32_t)kdep[q][2])) : -1;
          r.ops.push_back({q, i0, j0});
        }
        if ((int)r.ops.size() > kS2BlkMaxGates) continue;
        std::copy(reg, reg + 4, r.reg1);
        std::copy(ln, ln + 2, r.ln1);
        for (int b = 0; b < 4; ++b) r.bm |= 1u << r.reg0[b];
        r.mask = live & ~r.bm;
        // lane bits 4 / 5 are group-index bits 4 / 5: the lane positions at order 4 - logC, 5 - logC
        r.order.assign(oth.begin(), oth.begin() + (4 - d.logC));
        r.order.push_back(r.ln0[0]);
        r.order.push_back(r.ln0[1]);
        r.order.insert(r.order.end(), oth.begin() + (4 - d.logC), oth.end());
        lp = r;
        return true;
      }
      return false;
    };
    auto plan_passes = [&](int ng) {
      std::vector<PPlan> v;
      for (int j = 0; j < ng;) {
        uint32_t bm = 0, lv = 0;
        const int e = block_span(j, ng, &bm, &lv);
        PPlan pp;
        if (lane_span(j, ng, e, pp)) {
          v.push_back(pp);
          j = pp.end;
          continue;
        }
        pp.first = j;
        pp.end = e;
        pp.block = e - j >= 2;
        pp.bm = pp.block ? bm : 0;
        pp.mask = pp.block ? (lv & ~bm) : d.gate[j].pass_mask;
        pp.order = ascending(pp.mask);
        v.push_back(pp);
        j = e;
      }
      return v;
    };
    // a last gate inside a register block costs no pass of its own: no epilogue then
    bool last_alone = true;
    {
      const std::vector<PPlan> pl = plan_passes((int)c.gates.size());
      if (!pl.empty()) last_alone = pl.back().end - pl.back().first == 1;
    }
    d.epi = 0;
    if (s2_epi_enabled() && last_alone && !last_np.empty()) {
      const S2Gate& G = d.gate[c.gates.size() - 1];
      const int nn = (int)last_np.size();
      bool ok = G.K <= G.N && G.K * G.N <= 16 && G.N >= 2 && last_nk <= nn &&
                (int)st.size() >= kS2LogThreads + nn && (int)st.size() <= kS2LogThreads + 4;
      std::vector<CBit> rest, moved(nn);
      for (size_t t = 0; ok && t < st.size(); ++t) {
        const auto it = std::find(last_np.begin(), last_np.end(), st[t].pos);
        if (st[t].col >= 0 || it == last_np.end()) { rest.push_back(st[t]); continue; }
        if (t < 5) ok = false;   // keep the coalesced 32-lane runs
        moved[it - last_np.begin()] = st[t];
      }
      if (ok) {
        st.assign(rest.begin(), rest.begin() + kS2LogThreads);
        st.insert(st.end(), moved.begin(), moved.end());
        st.insert(st.end(), rest.begin() + kS2LogThreads, rest.end());
        d.epi = (int)c.gates.size();
      }
    }
    // swizzle vectors: the first 4 / 5 chunk bits of each enumeration (one 16- / 32-lane group)
    // must map to independent bank slots (mod 16 / mod 32)
    int vsw[kS2MaxPos];
    for (int& v : vsw) v = -1;
    auto choose = [&](const std::vector<CBit>& e) {
      std::vector<int> vec;
      for (size_t t = 0; t < e.size() && t < 5; ++t) {
        if (e[t].col >= 0) { vec.push_back(e[t].col < 5 ? (1 << e[t].col) : 0); continue; }
        int& v = vsw[e[t].pos];
        if (v < 0) {
          static const int order[] = {1, 2, 4, 8, 16, 3, 5, 6, 9, 10, 12, 17, 18, 20, 24, 7, 11, 13,
                                      14, 19, 21, 22, 25, 26, 28, 15, 23, 27, 29, 30, 31};
          v = 0;
          for (int cand : order) {
            std::vector<int> a = vec, b;
            a.push_back(cand);
            for (size_t q = 0; q < a.size() && q < 4; ++q) b.push_back(a[q] & 15);
            if (gf2_rank(a) == (int)a.size() && gf2_rank(b) == (int)b.size()) { v = cand; break; }
          }
        }
        vec.push_back(v);
      }
    };
    choose(ld);
    choose(st);
    // ---- LDS bank model.  The tile image of (position set p, column c) is
    //   ((p << logC) | c) ^ S(p),  S(p) = XOR of vsw[q] over the positions q in p,
    // vsw[q] a 5-bit vector: only address bits below 5 are XOR-ed, so the map is a bijection of
    // the tile when the images of the address bits below 5 stay independent (columns j: 1 << j,
    // positions q with q + logC < 5: (1 << (q + logC)) ^ vsw[q]; s2_swz_valid).
    // A wave's LDS access is served in lane groups (MI355X_MICROARCH.md §LDS; 8-byte elements:
    // ds_read_b64 2 x 32 lanes on element mod 32, ds_write_b64 4 x 16 lanes on element mod 16);
    // every access of the kernel is XOR-linear in its lane bits, so a group of 2^k lanes whose
    // address differences span k directions with bank effects of rank r is 2^(k - r)-way.  The
    // lane directions: the load (LDS writes) and store (reads) enumerations, and for every pass
    // the columns then the pass positions (tq_sweep2.hip gate_pass_u / block_pass group index).
    // Chunks of fewer than 32 columns put pass positions into the lane groups, which a swizzle
    // of the column bits alone (r04) could not separate: the r04 PMC's 0.9 conflict cycles per
    // sweep2 LDS instruction on C4's 8-column slice ops.  The vectors: the enumerations' choice,
    // then a coordinate descent on the modeled cost (0 on every sweep op of C2 / C3 / C4).
    int swl[kS2MaxPos], rl, rm, wl, wm;   // log2 lanes per group / log2 bank modulus (elements)
    if (P_.esz <= 4) rl = rm = wl = wm = 5;
    else if (P_.esz == 8) { rl = rm = 5; wl = wm = 4; }
    else { rl = rm = 4; wl = wm = 3; }
    {
      struct Pat { std::vector<int> dirs; double rd, wr; };   // column j -> -(j + 1), position q -> q
      std::vector<Pat> pats;
      auto enum_dirs = [&](const std::vector<CBit>& e) {
        std::vector<int> v;
        for (size_t t = 0; t < e.size() && t < 5; ++t) v.push_back(e[t].col >= 0 ? -(e[t].col + 1) : e[t].pos);
        return v;
      };
      pats.push_back({enum_dirs(ld), 0.0, double(int64_t(1) << d.nld)});
      pats.push_back({enum_dirs(st), double(int64_t(1) << d.nst), 0.0});
      // as the pass loop below (the lane bits of a lane block: its start layout)
      for (const PPlan& pp : plan_passes((int)c.gates.size() - (d.epi ? 1 : 0))) {
        double rd, wr;
        if (!pp.block) rd = d.gate[pp.first].K, wr = d.gate[pp.first].N;
        else rd = wr = double(1 << B);
        std::vector<int> v;
        for (int q = 0; q < d.logC && v.size() < 5; ++q) v.push_back(-(q + 1));
        for (size_t t = 0; t < pp.order.size() && v.size() < 5; ++t) v.push_back(pp.order[t]);
        const double groups = double(int64_t(1) << (d.logC + __builtin_popcount(pp.mask)));
        pats.push_back({v, groups * rd, groups * wr});
      }
      double ideal = 0;
      for (auto& pt : pats) ideal += pt.rd / double(1 << rl) + pt.wr / double(1 << wl);
      auto cost = [&](const int* w) {   // modeled extra LDS cycles per chunk
        double x = 0;
        for (auto& pt : pats)
          for (int side = 0; side < 2; ++side) {
            const double n = side ? pt.wr : pt.rd;
            const int lg = side ? wl : rl, mb = (1 << (side ? wm : rm)) - 1;
            if (n <= 0) continue;
            std::vector<int> eff;
            for (int t = 0; t < (int)pt.dirs.size() && t < lg; ++t) {
              const int dd = pt.dirs[t];
              eff.push_back((dd < 0 ? (1 << (-dd - 1)) : ((1 << (dd + d.logC)) ^ w[dd])) & mb);
            }
            const int k = (int)eff.size();
            x += n * double((1 << (k - gf2_rank(eff))) - 1) / double(1 << lg);
          }
        return x;
      };
      const int cm = (1 << d.logC) - 1;
      for (int q = 0; q < kS2MaxPos; ++q) swl[q] = (vsw[q] < 0 ? 0 : vsw[q]) & cm;   // the r04 layout
      d.lds_model[0] = (float)(ideal > 0 ? cost(swl) / ideal : 0.0);
      // start from the enumerations' choice, then coordinate descent over the eligible positions'
      // vectors (strict improvements only: a conflict-free r04 layout stays as it was)
      // positions that reach a lane group: the only ones whose vector matters
      uint32_t rel = 0;
      for (auto& pt : pats)
        for (int dd : pt.dirs)
          if (dd >= 0 && dd < used) rel |= 1u << dd;
      const int lowb = std::min(5, d.logC + used);   // address bits the swizzle may write
      auto valid = [&](const int* w) {
        std::vector<int> im;
        for (int b = 0; b < lowb; ++b) im.push_back(b < d.logC ? 1 << b : (1 << b) ^ w[b - d.logC]);
        return gf2_rank(im) == lowb;
      };
      auto descend = [&](int* w) {
        double b = cost(w);
        for (int it = 0; it < 6 && b > 0; ++it) {
          bool moved = false;
          for (int q = 0; q < kS2MaxPos; ++q) {
            if (!((rel >> q) & 1)) continue;
            int bv = w[q];
            for (int v = 0; v < (1 << lowb); ++v) {
              if (v == bv) continue;
              w[q] = v;
              if (q + d.logC < 5 && !valid(w)) continue;
              const double x = cost(w);
              if (x < b - 1e-9) b = x, bv = v, moved = true;
            }
            w[q] = bv;
          }
          if (!moved) break;
        }
        return b;
      };
      double best;
      if (!s2_swz_model()) {   // TQ_S2_SWZ=0: the r04 column-only swizzle (A/B)
        best = cost(swl);
      } else {
        for (int q = 0; q < kS2MaxPos; ++q) swl[q] = (vsw[q] < 0 || q + d.logC < 5) ? 0 : vsw[q];
        best = descend(swl);
      }
      d.lds_model[1] = (float)(ideal > 0 ? best / ideal : 0.0);
    }
    for (int p = 0; p < kS2MaxPos; ++p) d.vsw[p] = swl[p];
    auto code = [&](const CBit& b) {
      if (b.col >= 0) return 1 << b.col;
      return ((1 << b.pos) << kS2CodeP) | (d.vsw[b.pos] << kS2CodeS);
    };
    d.nld = (int)ld.size();
    d.nst = (int)st.size();
    if (d.nld > 16 || d.nst > 16) return false;
    // the kernel carries the lane part of a load / store offset (the low kS2LogThreads chunk
    // bits) as a 32-bit byte offset: chains on high-order legs of huge tensors do not fit
    for (size_t t = 0; t < ld.size(); ++t) { d.ld_w[t] = ld[t].w; d.ld_code[t] = code(ld[t]); }
    for (size_t t = 0; t < st.size(); ++t) { d.st_w[t] = st[t].w; d.st_code[t] = code(st[t]); }
    if (!s2_lane_offsets_fit(d.ld_w, d.nld, d.st_w, d.nst, (int64_t)P_.esz)) return false;
    // LDS element address of a code: ((p << logC) | c) ^ s -- XOR-linear in the code
    auto lds_addr = [&](int cd) {
      const int p = (cd >> kS2CodeP) & ((1 << kS2MaxPos) - 1), cc = cd & ((1 << kS2CodeP) - 1),
                sv = (cd >> kS2CodeS) & 31;
      return ((p << d.logC) | cc) ^ sv;
    };
    for (int t = 0; t < d.nld; ++t) d.ld_a[t] = lds_addr(d.ld_code[t]);
    for (int t = 0; t < d.nst; ++t) d.st_a[t] = lds_addr(d.st_code[t]);
    const int rin = std::max(1, (1 << d.nld) >> kS2LogThreads), rout = std::max(1, (1 << d.nst) >> kS2LogThreads);
    for (int r = 0; r < kS2MaxSlots; ++r) {
      const int ri = r % rin, ro = r % rout;
      for (int b = kS2LogThreads; b < d.nld; ++b)
        if ((ri >> (b - kS2LogThreads)) & 1) { d.k.ld_hm[r] += d.ld_w[b]; d.ld_hc[r] ^= d.ld_code[b]; }
      for (int b = kS2LogThreads; b < d.nst; ++b)
        if ((ro >> (b - kS2LogThreads)) & 1) { d.k.st_hm[r] += d.st_w[b]; d.st_hc[r] ^= d.st_code[b]; }
      d.k.ld_ha[r] = lds_addr(d.ld_hc[r]);
      d.k.st_ha[r] = lds_addr(d.st_hc[r]);
    }
    auto swz = [&](int bits) {
      int v = 0;
      for (int p = 0; p < kS2MaxPos; ++p) if ((bits >> p) & 1) v ^= d.vsw[p];
      return v;
    };
    for (size_t j = 0; j < c.gates.size(); ++j) {
      S2Gate& G = d.gate[j];
      for (int k = 0; k < G.K; ++k) {
        G.kdep[k] = kdep[j][k];
        G.ksw[k] = swz(kdep[j][k]);
        G.kaddr[k] = (G.kdep[k] << d.logC) ^ G.ksw[k];
      }
      for (int n = 0; n < G.N; ++n) {
        G.ndep[n] = ndep[j][n];
        G.nsw[n] = swz(ndep[j][n]);
        G.naddr[n] = (G.ndep[n] << d.logC) ^ G.nsw[n];
      }
    }
    // gate fields and group tables (what the kernel used to build per workgroup)
    for (size_t j = 0; j < c.gates.size(); ++j) {
      const S2Gate& G = d.gate[j];
      int32_t* gm = d.k.gmeta[j];
      gm[kS2GmK] = G.K;
      gm[kS2GmN] = G.N;
      gm[kS2GmPass] = (int32_t)G.pass_mask;
      for (int k = 0; k < kS2MaxK; ++k) gm[kS2GmKaddr + k] = k < G.K ? G.kaddr[k] : 0;
      for (int n = 0; n < kS2MaxKN; ++n) gm[kS2GmNaddr + n] = n < G.N ? G.naddr[n] : 0;
      for (int jj = 0; jj < 64; ++jj) {
        const int half = jj >> 5, v = jj & 31;
        uint32_t m = G.pass_mask;
        int base = 0, sw = 0;
        for (int t = 0; m; ++t) {
          const int lo = __builtin_ctz(m);
          m &= m - 1;
          if (half == 0 && t < 5 && ((v >> t) & 1)) { base |= 1 << lo; sw ^= d.vsw[lo]; }
          if (half == 1 && t >= 5 && ((v >> (t - 5)) & 1)) { base |= 1 << lo; sw ^= d.vsw[lo]; }
        }
        d.k.lut[j][jj] = ((base << d.logC) ^ sw) * (int32_t)P_.esz;   // bytes
      }
    }
    // passes: register blocks of consecutive square gates (S2Desc::pmeta) -- plain, or lane
    // blocks (plan_passes) -- single gates otherwise
    {
      const int ng = (int)c.gates.size() - (d.epi ? 1 : 0);   // the epilogue gate is no pass
      // group table of a pass: group-index bits (after the columns) -> positions, in `order`
      auto group_lut = [&](const std::vector<int>& order, int32_t* lut) {
        for (int jj = 0; jj < 64; ++jj) {
          const int half = jj >> 5, v = jj & 31;
          int base = 0, sw = 0;
          for (int t = 0; t < (int)order.size(); ++t) {
            const int lo = order[t];
            if (half == 0 && t < 5 && ((v >> t) & 1)) { base |= 1 << lo; sw ^= d.vsw[lo]; }
            if (half == 1 && t >= 5 && ((v >> (t - 5)) & 1)) { base |= 1 << lo; sw ^= d.vsw[lo]; }
          }
          lut[jj] = ((base << d.logC) ^ sw) * (int32_t)P_.esz;   // bytes
        }
      };
      auto addr = [&](int pos) { return ((1 << pos) << d.logC) ^ d.vsw[pos]; };   // elements
      // a gate's block code from its register slots; canonical placement I < J: swap the gate's
      // two legs -- input / output index bits 0 and 1 of every coefficient (a square gate: its
      // outputs sit on its inputs' positions).  The kernel then needs 6 (B = 4) / 3 (B = 3)
      // block-gate bodies instead of 12 / 6 (instruction-cache footprint, tq_sweep2.hip blk_gate)
      auto gate_code = [&](int q, int i0, int j0) {
        if (d.gate[q].K != 4) return i0;
        if (i0 > j0) {
          uint8_t cg[16];
          auto sw = [](int v) { return ((v & 1) << 1) | ((v >> 1) & 1); };
          for (int k = 0; k < 4; ++k)
            for (int n = 0; n < 4; ++n) cg[sw(k) * 4 + sw(n)] = d.cgidx[q][k * 4 + n];
          for (int t = 0; t < 16; ++t) d.cgidx[q][t] = cg[t];
          std::swap(i0, j0);
        }
        return i0 | (j0 << 2) | 16;
      };
      const std::vector<PPlan> plan = plan_passes(ng);
      if ((int)plan.size() > kS2MaxGates) return false;
      d.npass = 0;
      for (const PPlan& pp : plan) {
        const int j = pp.first;
        int32_t* pm = d.k.pmeta[d.npass++];
        pm[kS2PmFirst] = j;
        if (!pp.block) {
          // a single-gate pass carries the gate's fields itself (S2Keep::pmeta): the kernel
          // reads a pass's whole head in one batch, ahead of the pass
          const S2Gate& G = d.gate[j];
          pm[kS2PmCount] = 1 | ((G.K * 16 + G.N) << 8);
          pm[kS2PmB] = 0;
          pm[kS2PmPass] = (int32_t)G.pass_mask;
          for (int k = 0; k < kS2MaxK; ++k) pm[kS2PmAddr + k] = k < G.K ? G.kaddr[k] : 0;
          for (int n = 0; n < kS2MaxKN; ++n) pm[kS2PmCode + n] = n < G.N ? G.naddr[n] : 0;
          group_lut(pp.order, d.k.lut[j]);
          continue;
        }
        pm[kS2PmPass] = (int32_t)pp.mask;
        if (pp.lanes) {
          pm[kS2PmCount] = (int)pp.ops.size();
          pm[kS2PmB] = 4 | kS2PmLanes;
          for (int b = 0; b < 4; ++b) {
            pm[kS2PmAddr + b] = addr(pp.reg0[b]);
            pm[kS2PmAddrEnd + b] = addr(pp.reg1[b]);
          }
          pm[kS2PmLaneDelta] = addr(pp.ln0[0]) ^ addr(pp.ln1[0]);
          pm[kS2PmLaneDelta + 1] = addr(pp.ln0[1]) ^ addr(pp.ln1[1]);
          for (size_t t = 0; t < pp.ops.size(); ++t) {
            const auto& o = pp.ops[t];
            pm[kS2PmCode + (int)t] = o[0] < 0 ? (kS2SwapCode | (o[1] << 2) | o[2]) : gate_code(o[0], o[1], o[2]);
          }
        } else {
          pm[kS2PmCount] = pp.end - pp.first;
          pm[kS2PmB] = B;
          int bp[4], nb = 0;
          for (int q = 0; q < kS2MaxPos; ++q)
            if ((pp.bm >> q) & 1) bp[nb++] = q;
          for (int b = 0; b < B; ++b) pm[kS2PmAddr + b] = pm[kS2PmAddrEnd + b] = addr(bp[b]);
          pm[kS2PmLaneDelta] = pm[kS2PmLaneDelta + 1] = 0;
          auto local = [&](int pos) {
            for (int b = 0; b < B; ++b) if (bp[b] == pos) return b;
            return -1;
          };
          for (int q = pp.first; q < pp.end; ++q) {
            // index bit t of the gate <-> position of input k = 1 << t
            const int i0 = local(__builtin_ctz((uint32_t)kdep[q][1]));
            const int j0 = d.gate[q].K == 4 ? local(__builtin_ctz((uint32_t)kdep[q][2])) : -1;
            pm[kS2PmCode + (q - pp.first)] = gate_code(q, i0, j0);
          }
        }
        group_lut(pp.order, d.k.lut[j]);
      }
      if (getenv("TQ_S2_DUMP") && out) {
        fprintf(stderr, "s2 op: %d gates, %d passes, logC %d, used %d:", d.ngates, d.npass, d.logC, used);
        for (const PPlan& pp : plan) {
          fprintf(stderr, " |%s", pp.lanes ? "L" : "");
          auto gate_pos = [&](int g) {
            uint32_t m = 0;
            for (int k = 0; k < d.gate[g].K; ++k) m |= (uint32_t)kdep[g][k];
            for (int k = 0; k < d.gate[g].N; ++k) m |= (uint32_t)ndep[g][k];
            fprintf(stderr, " %dx%d:", d.gate[g].K, d.gate[g].N);
            for (int b = 0; b < 16; ++b) if ((m >> b) & 1) fprintf(stderr, "%d", b);
          };
          if (pp.lanes) {
            for (const auto& o : pp.ops) {
              if (o[0] < 0) fprintf(stderr, " s%d%d", o[1] + 4, o[2]);
              else gate_pos(o[0]);
            }
          } else {
            for (int g = pp.first; g < pp.end; ++g) gate_pos(g);
          }
        }
        fprintf(stderr, "\n");
      }
      // group tables by pass (row p = the table of pass p's first gate): the kernel reads a
      // pass's row without first reading which gate starts it
      for (int q = 0; q < d.npass; ++q) {
        const int g = d.k.pmeta[q][kS2PmFirst];
        if (g != q) std::copy(d.k.lut[g], d.k.lut[g] + 64, d.k.lut[q]);
      }
      // Barriers between passes (kS2PmSync, bit 16 of a pass's count word: the workgroup barrier
      // before that pass).  Thread t of the 512 takes the groups gi = t (mod 512) in every pass
      // (tq_sweep2.hip gate_pass_u / block_pass), so wave w owns the groups whose gi bits 6..8
      // (kS2WaveBits .. kS2LogThreads - 1, asserted in the kernel) are
      // w, i.e. the elements whose address bits behind those group bits (columns below logC, then
      // the pass's group positions in its order) are w.  Two consecutive passes with the same
      // wave-select address bits leave every element with one wave: no barrier between them (LDS
      // accesses of one wave complete in order; a lane block's swaps stay inside the wave: its
      // lane bits are group bits 4 and 5).
      auto wave_sig = [&](int q) {
        const std::vector<int>& order = plan[q].order;
        const int lg = d.logC + (int)order.size();   // log2 groups
        std::vector<int> sig;
        for (int b = kS2WaveBits; b < kS2LogThreads && b < lg; ++b)
          sig.push_back(b < d.logC ? -1 - b : order[b - d.logC]);
        return sig;
      };
      d.nsync = 0;
      for (int q = 0; q < d.npass; ++q) {
        const bool sync = q == 0 || !s2_wave_local() || wave_sig(q) != wave_sig(q - 1);
        if (sync) d.k.pmeta[q][kS2PmCount] |= kS2PmSync;
        d.nsync += sync;
      }
    }
    if (getenv("TQ_DEBUG_S2")) {
      fprintf(stderr, "S2 cols=2^%d logC=%d used=%d epi=%d ld:", d.colbits, d.logC, used, d.epi);
      for (int t = 0; t < d.nld; ++t) fprintf(stderr, " %lld/%x", (long long)d.ld_w[t], d.ld_code[t]);
      fprintf(stderr, " | st:");
      for (int t = 0; t < d.nst; ++t) fprintf(stderr, " %lld/%x", (long long)d.st_w[t], d.st_code[t]);
      fprintf(stderr, " | vsw:");
      for (int p = 0; p < kS2MaxPos; ++p) fprintf(stderr, " %d", d.vsw[p]);
      fprintf(stderr, " | gates:");
      for (size_t j = 0; j < c.gates.size(); ++j)
      {
        uint32_t km = 0, nm = 0;
        for (int k = 0; k < d.gate[j].K; ++k) km |= (uint32_t)kdep[j][k];
        for (int n = 0; n < d.gate[j].N; ++n) nm |= (uint32_t)ndep[j][n];
        fprintf(stderr, " [K%d N%d pass%x in%x out%x]", d.gate[j].K, d.gate[j].N, d.gate[j].pass_mask, km, nm);
      }
      fprintf(stderr, "\n");
    }
    *out = d;
    return true;
  }

  // mixed-radix digits of index t over `modes` (last fastest)
  void digits(int64_t t, const std::vector<int>& modes, std::map<int, int64_t>& dig) {
    for (int q = (int)modes.size() - 1; q >= 0; --q) {
      const int64_t e = ext_[modes[q]];
      dig[modes[q]] = t % e;
      t /= e;
    }
  }
  int64_t index_of(const std::vector<int>& modes, const std::map<int, int64_t>& dig) {
    int64_t t = 0;
    for (int m : modes) t = t * ext_[m] + dig.at(m);
    return t;
  }

  // one OP_SWEEP2 op: chain c (shape sh, layout d) from src (n0 elements) into tgt (nq)
  void emit_s2(const Chain& c, const ChainShape& sh, const S2Desc& d, BufRef src, int64_t n0, BufRef tgt,
               int64_t nq, bool direct, const char* what, const S2Desc* d1 = nullptr) {
    Op op;
    op.kind = OP_SWEEP2;
    op.a = src;
    op.c = tgt;
    op.writes_output = direct;
    int step0 = c.gates.front().step;   // a re-listed chain (s2_reorder_squares): first / last path step
    op.step = step0;
    for (auto& g : c.gates) step0 = std::min(step0, g.step), op.step = std::max(op.step, g.step);
    op.tin = (int)sh.tin_n;
    op.tout = (int)sh.tout_n;
    op.ncols = d.ncols;
    op.s2_nchunks = d.nchunks;
    op.na = src.kind == BUF_TABLE ? 0 : n0;
    op.nc = nq;
    double flops = 0;
    for (size_t j = 0; j < c.gates.size(); ++j) {
      SweepGate sg;
      sg.g = c.gates[j].Sm.buf;
      sg.K = (int)c.gates[j].d.K;
      sg.N = (int)c.gates[j].d.N;
      sg.n = c.gates[j].Sm.numel();
      op.sgates.push_back(sg);
      flops += (double)d.ncols * count_of(sh.W[j]) * sg.K * (cplx_ ? 8.0 : 2.0);
    }
    op.stab = (int)P_.stabs.size();
    P_.stabs.push_back(s2_blob(d, P_.esz));
    if (d.nchunks == 1) {
      op.stab1 = op.stab;
    } else if (d1) {
      op.stab1 = (int)P_.stabs.size();
      P_.stabs.push_back(s2_blob(*d1, P_.esz));
    }
    op.flops = flops;
    op.bytes = (double)(n0 + nq) * P_.esz;
    std::ostringstream o;
    o << "step " << step0 << ".." << op.step << " SWEEP2 " << what << "gates=" << c.gates.size()
      << " tin=" << op.tin << " tout=" << op.tout << " cols=" << op.ncols << " C=" << (1 << d.logC)
      << " chunks=" << d.nchunks << (direct ? " ->OUT" : "") << " KxN=";
    for (int j = 0; j < d.ngates; ++j) o << (j ? "," : "") << d.gate[j].K << "x" << d.gate[j].N;
    o << " passes=" << d.npass;
    {
      int nl = 0;
      for (int q = 0; q < d.npass; ++q) nl += (d.k.pmeta[q][kS2PmB] & kS2PmLanes) != 0;
      if (nl) o << " lanes=" << nl;
    }
    if (d.epi) o << " epi";
    {
      char b[48];
      snprintf(b, sizeof b, " ldsx=%.2f->%.2f syncs=%d/%d", d.lds_model[0], d.lds_model[1], d.nsync, d.npass);
      o << b;
    }
    op.note = o.str();
    P_.ops.push_back(op);
  }

  int flush_chain(bool final) {
    if (!chain_.active) return TQ_OK;
    Chain c = chain_;
    chain_ = Chain{};
    chain_.flushed_id = c.id;
    const size_t first_op = P_.ops.size();
    Live res;
    const bool saved_pin = pin_next_;
    const int saved_br = br_;
    pin_next_ = pinned_[c.id];
    br_ = c.br;
    ChainShape sh0;
    const bool shape_ok = chain_shape(c, c.out_modes, sh0);
    if (c.gates.size() == 1 && !(shape_ok && sh0.s2)) {
      const auto& g = c.gates[0];
      const Live& A0 = g.d.a_big ? c.X0 : g.Sm;
      const Live& B0 = g.d.a_big ? g.Sm : c.X0;
      TQ_TRY(emit_apply(g.step, g.d, final, A0, B0, res));
    } else if (shape_ok && sh0.s2) {
      const int64_t n0 = c.X0.numel();
      const int64_t nq = n0 / sh0.tin_n * sh0.tout_n;
      S2Dense dd;
      const bool dense = s2_dense_layout(c, sh0, c.out_modes, &dd);
      // dense: the chain composed on the identity first (a tiny sweep2 op into an arena matrix)
      int64_t moff = -1;
      BufRef mbuf;
      if (dense) {
        const int vm = 1 << 30;   // a column mode of its own: the basis vector index
        ext_[vm] = sh0.tin_n;
        Chain c2 = c;
        c2.X0 = Live{};
        c2.X0.modes = sh0.tin;
        c2.X0.modes.push_back(vm);
        for (int m : c2.X0.modes) c2.X0.ext.push_back(ext_[m]);
        c2.X0.stride = contig_strides(c2.X0.ext);
        std::vector<char> ident((size_t)(sh0.tin_n * sh0.tin_n) * P_.esz, 0);
        for (int64_t k = 0; k < sh0.tin_n; ++k) {
          const float one = 1.0f;
          std::memcpy(ident.data() + (size_t)(k * sh0.tin_n + k) * P_.esz, &one, sizeof(float));
        }
        c2.X0.buf = BufRef{BUF_TABLE, (int64_t)P_.stabs.size(), 0, 0};
        P_.stabs.push_back(std::move(ident));
        std::vector<int> out2 = sh0.tout;
        out2.push_back(vm);
        ChainShape sh2;
        S2Desc d2;
        if (!chain_shape(c2, out2, sh2) || !sh2.s2 || !s2_layout(c2, sh2, out2, &d2)) {
          ext_.erase(vm);
          set_error("internal: sweep2 compose layout");
          return TQ_ERR_INVALID;
        }
        ext_.erase(vm);
        mbuf = new_buf(sh0.tin_n * sh0.tout_n, &moff);
        emit_s2(c2, sh2, d2, c2.X0.buf, sh0.tin_n * sh0.tin_n, mbuf, sh0.tin_n * sh0.tout_n, false, "compose ");
      }
      bool direct;
      int64_t roff;
      BufRef tgt = result_target(final, c.out_modes, nq, &direct, &roff);
      if (dense) {
        Op op;
        op.kind = OP_SWEEP2;
        op.s2_dense = true;
        op.a = c.X0.buf;
        op.b = mbuf;
        op.c = tgt;
        op.writes_output = direct;
        op.step = c.gates.back().step;
        op.tin = (int)sh0.tin_n;
        op.tout = (int)sh0.tout_n;
        op.ncols = dd.ncols;
        op.na = n0;
        op.nb = sh0.tin_n * sh0.tout_n;
        op.nc = nq;
        std::vector<char> blob(sizeof(S2Dense));
        std::memcpy(blob.data(), &dd, sizeof(S2Dense));
        op.stab = (int)P_.stabs.size();
        P_.stabs.push_back(std::move(blob));
        op.flops = (double)nq * sh0.tin_n * 8.0;
        op.bytes = (double)(n0 + nq) * P_.esz;
        std::ostringstream o;
        o << "step " << c.gates.front().step << ".." << op.step << " SWEEP2 DENSE gates=" << c.gates.size()
          << " tin=" << op.tin << " tout=" << op.tout << " cols=" << op.ncols << (direct ? " ->OUT" : "");
        op.note = o.str();
        P_.ops.push_back(op);
        arenas_[region()].release(moff);
      } else {
        S2Desc d;
        if (!s2_layout(c, sh0, c.out_modes, &d)) { set_error("internal: sweep2 layout"); return TQ_ERR_INVALID; }
        // the square gates re-listed into fuller register blocks, when that saves passes
        Chain cr;
        if (s2_reorder_on() && d.npass > 1 && s2_reorder_squares(c, cr, 4)) {
          ChainShape shr;
          S2Desc dr;
          if (chain_shape(cr, cr.out_modes, shr) && shr.s2 && shr.tin_n == sh0.tin_n && shr.tout_n == sh0.tout_n &&
              s2_layout(cr, shr, cr.out_modes, &dr) && dr.npass < d.npass) {
            c = cr;
            sh0 = shr;
            d = dr;
          }
        }
        // a small tensor split into chunks for parallelism: also its one-chunk form, which a
        // chain launch (one workgroup running consecutive dependent ops) uses
        S2Desc d1;
        bool has1 = false;
        if (d.nchunks > 1 && d.nchunks <= s2_seq_max_chunks() &&
            (d.ncols * (int64_t)sh0.tout_n) <= (int64_t(1) << s2_chunk_bits((int)P_.esz))) {
          one_chunk_ = true;
          has1 = s2_layout(c, sh0, c.out_modes, &d1) && d1.nchunks == 1;
          one_chunk_ = false;
        }
        emit_s2(c, sh0, d, c.X0.buf, n0, tgt, nq, direct, "", has1 ? &d1 : nullptr);
      }
      res.modes = c.out_modes;
      for (int m : c.out_modes) res.ext.push_back(ext_[m]);
      res.stride = contig_strides(res.ext);
      res.buf = tgt;
      res.owned = !direct;
      if (final && !direct)
        TQ_TRY(emit_permute(res, P_.out_modes, {}, BufRef{BUF_OUTPUT, 0, 0}, true, c.gates.back().step,
                            "result->out"));
    } else {
      ChainShape sh = sh0;
      if (!shape_ok) { set_error("internal: chain shape"); return TQ_ERR_INVALID; }
      const int64_t n0 = c.X0.numel();
      const int64_t nq = n0 / sh.tin_n * sh.tout_n;
      bool direct;
      int64_t roff;
      BufRef tgt = result_target(final, c.out_modes, nq, &direct, &roff);
      Op op;
      op.kind = OP_SWEEP;
      op.a = c.X0.buf;
      op.c = tgt;
      op.writes_output = direct;
      op.step = c.gates.back().step;
      op.tin = (int)sh.tin_n;
      op.tout = (int)sh.tout_n;
      op.ncols = n0 / sh.tin_n;
      // strides of X0 (contiguous, its own order) and of Y (contiguous, out order)
      std::map<int, int64_t> sx, sy;
      {
        auto cs = contig_strides(c.X0.ext);
        for (size_t q = 0; q < c.X0.modes.size(); ++q) sx[c.X0.modes[q]] = cs[q];
        std::vector<int64_t> ye;
        for (int m : c.out_modes) ye.push_back(ext_[m]);
        auto cy = contig_strides(ye);
        for (size_t q = 0; q < c.out_modes.size(); ++q) sy[c.out_modes[q]] = cy[q];
      }
      // outer runs (merge neighbours contiguous in both X and Y), innermost first
      std::vector<std::array<int64_t, 3>> runs;  // ext, in stride, out stride (outer->inner)
      for (int m : sh.outer) {
        const int64_t e = ext_[m];
        if (e == 1) continue;
        if (!runs.empty() && runs.back()[1] == sx[m] * e && runs.back()[2] == sy[m] * e) {
          runs.back()[0] *= e;
          runs.back()[1] = sx[m];
          runs.back()[2] = sy[m];
        } else {
          runs.push_back({e, sx[m], sy[m]});
        }
      }
      if (runs.size() > (size_t)kSweepMaxRuns) { set_error("internal: sweep runs"); return TQ_ERR_INVALID; }
      std::reverse(runs.begin(), runs.end());
      op.nruns = (int)runs.size();
      for (size_t r = 0; r < runs.size(); ++r) {
        op.run_ext[r] = runs[r][0]; op.run_in[r] = runs[r][1]; op.run_out[r] = runs[r][2];
      }
      // tables: tin_off (int64) | tout_off (int64) | per gate [W][K+1] int16
      std::vector<char> blob;
      auto put64 = [&](int64_t v) { const char* p = (const char*)&v; blob.insert(blob.end(), p, p + 8); };
      std::map<int, int64_t> dig;
      for (int64_t t = 0; t < sh.tin_n; ++t) {
        digits(t, sh.tin, dig);
        int64_t o = 0;
        for (int m : sh.tin) o += dig[m] * sx[m];
        put64(o);
      }
      op.tout_off_at = blob.size();
      for (int64_t t = 0; t < sh.tout_n; ++t) {
        digits(t, sh.tout, dig);
        int64_t o = 0;
        for (int m : sh.tout) o += dig[m] * sy[m];
        put64(o);
      }
      std::vector<int> prev = sh.tin;
      double flops = 0;
      op.tabs_at = blob.size();
      size_t entries = 0;
      for (size_t j = 0; j < c.gates.size(); ++j) {
        const auto& g = c.gates[j];
        const std::vector<int>& w = sh.W[j];
        SweepGate sg;
        sg.g = g.Sm.buf;
        sg.gtab = add_gtab(g.d.gtab);
        sg.K = (int)g.d.K;
        sg.N = (int)g.d.N;
        sg.n = g.Sm.numel();
        sg.W = (int)count_of(w);
        sg.tab_off = entries;
        for (int64_t e = 0; e < sg.W; ++e) {
          std::map<int, int64_t> de;
          digits(e, w, de);
          std::map<int, int64_t> dn;
          for (int m : g.d.nfree) dn[m] = de[m];
          const int64_t n = index_of(g.d.nfree, dn);
          for (int64_t k = 0; k < sg.K; ++k) {
            std::map<int, int64_t> dk = de;
            std::map<int, int64_t> kd;
            digits(k, g.d.korder, kd);
            for (auto& kv : kd) dk[kv.first] = kv.second;
            const int32_t v = (int32_t)index_of(prev, dk);
            blob.insert(blob.end(), (const char*)&v, (const char*)&v + 4);
          }
          const int32_t nv = (int32_t)n;
          blob.insert(blob.end(), (const char*)&nv, (const char*)&nv + 4);
          entries += sg.K + 1;
        }
        flops += (double)op.ncols * sg.W * sg.K * (cplx_ ? 8.0 : 2.0);
        op.sgates.push_back(sg);
        prev = w;
      }
      op.tab_len = (int)entries;
      op.stab = (int)P_.stabs.size();
      P_.stabs.push_back(std::move(blob));
      // coalescing: walk columns fastest when the innermost outer run is unit-stride
      op.load_colfast = (op.nruns > 0 && op.run_in[0] == 1 && op.run_ext[0] >= 16) ? 1 : 0;
      op.store_colfast = (op.nruns > 0 && op.run_out[0] == 1 && op.run_ext[0] >= 16) ? 1 : 0;
      op.flops = flops;
      op.bytes = (double)(n0 + nq) * P_.esz;
      op.na = n0;
      op.nc = nq;
      std::ostringstream o;
      o << "step " << c.gates.front().step << ".." << op.step << " SWEEP gates=" << c.gates.size()
        << " tin=" << op.tin << " tout=" << op.tout << " cols=" << op.ncols << " runs=" << op.nruns
        << (direct ? " ->OUT" : "");
      op.note = o.str();
      P_.ops.push_back(op);
      res.modes = c.out_modes;
      for (int m : c.out_modes) res.ext.push_back(ext_[m]);
      res.stride = contig_strides(res.ext);
      res.buf = tgt;
      res.owned = !direct;
      if (final && !direct)
        TQ_TRY(emit_permute(res, P_.out_modes, {}, BufRef{BUF_OUTPUT, 0, 0}, true, op.step, "result->out"));
    }
    for (size_t k = first_op; k < P_.ops.size(); ++k) {
      P_.ops[k].invariant = !c.dep;
      P_.ops[k].branch = c.br;
    }
    res.dep = c.dep;
    // the pending result gets its real buffer
    Live& L = live_[c.id];
    L.buf = res.buf;
    L.owned = res.owned;
    L.modes = res.modes;
    L.ext = res.ext;
    L.stride = res.stride;
    L.dep = c.dep;
    // operands are released only now, after the result buffer was placed
    if (c.release_X0) release(c.X0);
    for (auto& g : c.gates) if (g.release) release(g.Sm);
    pin_next_ = saved_pin;
    br_ = saved_br;
    return TQ_OK;
  }

  // A GEMM step whose output is tiny (M * N <= 16, no batch modes, no single-side sums) and whose
  // operands would need a permute: one strided skinny op reads both in place (bit weights from the
  // operands' own strides; every M / N / K mode a power of two).  true: emitted (*rc its status)
  static bool skinny_strided_enabled() {
    static const int v = [] {
      const char* e = getenv("TQ_SKINNY_STRIDED");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    return v != 0;
  }
  bool skinny_step(int s, const Live* A, const Live* B, const std::set<int>& sA, const std::set<int>& sB,
                   const std::vector<int>& bord, const std::vector<int>& mord, const std::vector<int>& nord,
                   const std::vector<int>& kord, bool final, Live& res, int* rc) {
    if (!skinny_strided_enabled() || !bord.empty() || !sA.empty() || !sB.empty()) return false;
    const int64_t M = ext_of(mord), N = ext_of(nord), K = ext_of(kord);
    auto p2 = [](int64_t v) { return v >= 1 && (v & (v - 1)) == 0; };
    if (!p2(M) || !p2(N) || M * N > 16 || !p2(K) || K < 256 || K > (int64_t(1) << kSkMaxKBits)) return false;
    for (const auto* ord : {&mord, &nord, &kord})
      for (int m : *ord) if (!p2(ext_[m])) return false;
    if (A->buf.kind == BUF_PENDING || B->buf.kind == BUF_PENDING) return false;
    // bit weights, least significant bit first (row-major index: the last mode is fastest)
    auto weights = [&](const Live& X, const std::vector<int>& ord, int64_t* w, int cap) {
      int nb = 0;
      for (auto it = ord.rbegin(); it != ord.rend(); ++it) {
        const int pos = X.pos(*it);
        int e = 0;
        while ((int64_t(1) << e) < ext_[*it]) ++e;
        for (int b = 0; b < e; ++b) {
          if (nb >= cap) return -1;
          w[nb++] = X.stride[pos] << b;
        }
      }
      return nb;
    };
    SkinnyArgs sk;
    sk.K = K;
    sk.M = (int)M;
    sk.N = (int)N;
    if (weights(*A, mord, sk.wam, 4) < 0 || weights(*B, nord, sk.wbn, 4) < 0) return false;
    const int nka = weights(*A, kord, sk.wak, kSkMaxKBits), nkb = weights(*B, kord, sk.wbk, kSkMaxKBits);
    if (nka < 0 || nkb < 0 || nka != nkb) return false;
    sk.nkb = nka;
    std::vector<int> rord = mord;
    rord.insert(rord.end(), nord.begin(), nord.end());
    bool direct;
    int64_t roff;
    BufRef tgt = result_target(final, rord, M * N, &direct, &roff);
    Op op;
    op.kind = OP_GEMM;
    op.skinny = true;
    op.sk = sk;
    op.a = A->buf; op.b = B->buf; op.c = tgt;
    op.writes_output = direct;
    op.M = M; op.N = N; op.K = K; op.batch = 1;
    const int P = skinny_blocks(K);
    op.ws_bytes = P > 1 ? (size_t)P * M * N * P_.esz : 0;
    op.na = A->numel();
    op.nb = B->numel();
    op.nc = M * N;
    op.nws = (int64_t)((op.ws_bytes + P_.esz - 1) / P_.esz);
    int64_t wsoff = -1;
    if (op.ws_bytes) {
      wsoff = arenas_[region()].alloc((int64_t)op.ws_bytes);
      op.ws = BufRef{BUF_ARENA, 0, wsoff / (int64_t)P_.esz, region()};
    }
    op.step = s;
    op.flops = (double)M * N * K * (cplx_ ? 8.0 : 2.0);
    op.bytes = (double)(M * K + K * N + M * N) * P_.esz;
    std::ostringstream o;
    o << "step " << s << " SKINNY M=" << M << " N=" << N << " K=" << K << " (strided, no permutes)"
      << (direct ? " ->OUT" : "");
    op.note = o.str();
    P_.ops.push_back(op);
    if (wsoff >= 0) arenas_[region()].release(wsoff);
    res.modes = rord;
    res.ext.clear();
    for (int m : rord) res.ext.push_back(ext_[m]);
    res.stride = contig_strides(res.ext);
    res.buf = tgt;
    res.owned = !direct;
    *rc = TQ_OK;
    if (final && !direct)
      *rc = emit_permute(res, P_.out_modes, {}, BufRef{BUF_OUTPUT, 0, 0}, true, s, "result->out");
    return true;
  }

  struct GemmChoice {
    bool swap = false;          // roles: A = second operand
    int korder_from = 0;        // 0: A's order, 1: B's order
    double cost = 1e300;
  };

  int gemm_step(int s, const Live& X, const Live& Y, bool final, const std::set<int>& batch,
                const std::set<int>& contr, const std::set<int>& freeX, const std::set<int>& freeY,
                const std::set<int>& sumX, const std::set<int>& sumY, Live& res) {
    // Evaluate role assignments and the source of the (batch, K) order.
    struct Cand {
      const Live* A; const Live* B;
      std::set<int> fA, fB, sA, sB;
      std::vector<int> bord, kord, mord, nord;
      bool a_ok = false, b_ok = false; int ta = 0, tb = 0;
      double cost = 0;
    };
    std::vector<Cand> cands;
    for (int swap = 0; swap < 2; ++swap)
      for (int from = 0; from < 2; ++from) {
        Cand c;
        c.A = swap ? &Y : &X; c.B = swap ? &X : &Y;
        c.fA = swap ? freeY : freeX; c.fB = swap ? freeX : freeY;
        c.sA = swap ? sumY : sumX; c.sB = swap ? sumX : sumY;
        std::set<int> kset = contr;
        kset.insert(c.sA.begin(), c.sA.end());
        kset.insert(c.sB.begin(), c.sB.end());
        const Live& src = from == 0 ? *c.A : *c.B;
        c.bord = filter(src.modes, batch);
        c.kord = filter(src.modes, kset);
        // sum modes absent from src go last in K
        for (int m : (from == 0 ? c.sB : c.sA)) c.kord.push_back(m);
        c.mord = filter(c.A->modes, c.fA);
        c.nord = filter(c.B->modes, c.fB);
        // A layouts: [b][M][K] (ta=0) or [b][K][M] (ta=1)
        if (c.A->contiguous() && c.sB.empty()) {
          if (runs_equal(c.A->modes, {c.bord, c.mord, c.kord})) { c.a_ok = true; c.ta = 0; }
          else if (runs_equal(c.A->modes, {c.bord, c.kord, c.mord})) { c.a_ok = true; c.ta = 1; }
        }
        if (c.B->contiguous() && c.sA.empty()) {
          if (runs_equal(c.B->modes, {c.bord, c.kord, c.nord})) { c.b_ok = true; c.tb = 0; }
          else if (runs_equal(c.B->modes, {c.bord, c.nord, c.kord})) { c.b_ok = true; c.tb = 1; }
        }
        const int64_t bsz = ext_of(c.bord), msz = ext_of(c.mord), nsz = ext_of(c.nord),
                      ksz = ext_of(c.kord);
        if (!c.a_ok) c.cost += 2.0 * bsz * msz * ksz;
        if (!c.b_ok) c.cost += 2.0 * bsz * ksz * nsz;
        std::vector<int> rord = c.bord;
        rord.insert(rord.end(), c.mord.begin(), c.mord.end());
        rord.insert(rord.end(), c.nord.begin(), c.nord.end());
        if (final && rord != P_.out_modes) c.cost += 2.0 * bsz * msz * nsz;
        // mild preference for the larger operand as A with M >= N (taller tiles)
        c.cost += 1e-3 * (double)(swap);
        cands.push_back(c);
      }
    auto best = std::min_element(cands.begin(), cands.end(),
                                 [](const Cand& a, const Cand& b) { return a.cost < b.cost; });
    Cand c = *best;
    const int64_t bsz = ext_of(c.bord), M = ext_of(c.mord), N = ext_of(c.nord),
                  K = ext_of(c.kord);
    if (!(c.a_ok && c.b_ok)) {
      int rc = 0;
      if (skinny_step(s, c.A, c.B, c.sA, c.sB, c.bord, c.mord, c.nord, c.kord, final, res, &rc)) return rc;
    }
    // materialise operands
    BufRef abuf = c.A->buf, bbuf = c.B->buf;
    int64_t aoff = -1, boff = -1;
    if (!c.a_ok) {
      std::vector<int> ord = c.bord;
      ord.insert(ord.end(), c.mord.begin(), c.mord.end());
      ord.insert(ord.end(), c.kord.begin(), c.kord.end());
      std::map<int, int64_t> bc;
      for (int m : c.sB) bc[m] = ext_[m];
      abuf = new_buf(bsz * M * K, &aoff);
      TQ_TRY(emit_permute(*c.A, ord, bc, abuf, false, s, "A->[b][M][K]"));
      c.ta = 0;
    }
    if (!c.b_ok) {
      std::vector<int> ord = c.bord;
      ord.insert(ord.end(), c.kord.begin(), c.kord.end());
      ord.insert(ord.end(), c.nord.begin(), c.nord.end());
      std::map<int, int64_t> bc;
      for (int m : c.sA) bc[m] = ext_[m];
      bbuf = new_buf(bsz * K * N, &boff);
      TQ_TRY(emit_permute(*c.B, ord, bc, bbuf, false, s, "B->[b][K][N]"));
      c.tb = 0;
    }
    std::vector<int> rord = c.bord;
    rord.insert(rord.end(), c.mord.begin(), c.mord.end());
    rord.insert(rord.end(), c.nord.begin(), c.nord.end());
    bool direct;
    int64_t roff;
    BufRef tgt = result_target(final, rord, bsz * M * N, &direct, &roff);
    Op op;
    op.kind = OP_GEMM;
    op.a = abuf; op.b = bbuf; op.c = tgt;
    op.writes_output = direct;
    op.transA = c.ta; op.transB = c.tb;
    op.M = M; op.N = N; op.K = K; op.batch = bsz;
    op.lda = c.ta ? M : K; op.sA = M * K;
    op.ldb = c.tb ? K : N; op.sB = K * N;
    op.ldc = N; op.sC = M * N;
    op.ws_bytes = gemm_workspace(P_.dtype, M, N, K, bsz);
    op.na = bsz * M * K;
    op.nb = bsz * K * N;
    op.nc = bsz * M * N;
    op.nws = (int64_t)((op.ws_bytes + P_.esz - 1) / P_.esz);
    int64_t wsoff = -1;
    if (op.ws_bytes) {
      wsoff = arenas_[region()].alloc((int64_t)op.ws_bytes);
      op.ws = BufRef{BUF_ARENA, 0, wsoff / (int64_t)P_.esz, region()};
    }
    op.step = s;
    op.flops = (double)bsz * M * N * K * (cplx_ ? 8.0 : 2.0);
    op.bytes = (double)bsz * (M * K + K * N + M * N) * P_.esz;
    std::ostringstream o;
    o << "step " << s << " GEMM b=" << bsz << " M=" << M << " N=" << N << " K=" << K
      << " tA=" << c.ta << " tB=" << c.tb << (c.a_ok ? "" : " permA") << (c.b_ok ? "" : " permB")
      << (direct ? " ->OUT" : "");
    op.note = o.str();
    P_.ops.push_back(op);
    if (wsoff >= 0) arenas_[region()].release(wsoff);
    if (aoff >= 0) arenas_[region()].release(aoff);
    if (boff >= 0) arenas_[region()].release(boff);
    res.modes = rord;
    for (int m : rord) res.ext.push_back(ext_[m]);
    res.stride = contig_strides(res.ext);
    res.buf = tgt;
    res.owned = !direct;
    if (final && !direct)
      TQ_TRY(emit_permute(res, P_.out_modes, {}, BufRef{BUF_OUTPUT, 0, 0}, true, s, "result->out"));
    return TQ_OK;
  }

  Plan& P_;
  int lanes_hint_ = 1;
  int group_hint_ = 1;
  int min_chunks_ = 0;
  bool one_chunk_ = false;   // s2_layout: one chunk of the whole tensor when it fits the tile
  bool cplx_ = false;
  int n_inputs_ = 0;
  Chain chain_;
  std::vector<Live> live_;
  std::map<int, int64_t> ext_;
  std::map<int, int> cnt_;
  Arena arenas_[2];          // per branch, so the two subtrees can run concurrently
  Arena pinned_arenas_[2];
  int br_ = 0;               // branch of the step being compiled (0, 1, 2 = join)
  std::vector<int> step_branch_;
  std::vector<char> pinned_;
  bool pin_next_ = false;
};

}  // namespace

int plan_compile(Plan& P, int dtype, int n_inputs, const int32_t* in_ranks, const int32_t* in_modes,
                 const int64_t* in_extents, const int64_t* in_strides, int out_rank,
                 const int32_t* out_modes, int n_steps, const int32_t* path, int n_sliced,
                 const int32_t* sliced_modes, int group_hint, int min_chunks) {
  TQ_CHECK_ARG(dtype_valid(dtype), "dtype");
  TQ_CHECK_ARG(group_hint >= 1, "group_hint");
  TQ_CHECK_ARG(min_chunks >= 0, "min_chunks");
  TQ_CHECK_ARG(n_inputs >= 1, "need at least one input");
  TQ_CHECK_ARG(n_steps == n_inputs - 1, "a pairwise path has n_inputs - 1 steps");
  TQ_CHECK_ARG(out_rank >= 0 && out_rank <= TQ_MAX_RANK, "output rank");
  TQ_CHECK_ARG(n_sliced >= 0 && n_sliced <= 62, "n_sliced");
  P = Plan{};
  P.dtype = dtype;
  Compiler c(P, 1, group_hint, min_chunks);
  TQ_TRY(c.run(n_inputs, in_ranks, in_modes, in_extents, in_strides, out_rank, out_modes, n_steps,
               path, n_sliced, sliced_modes));
  if (P.lanes > 1) {
    // slice lanes: compile again with wider chunks for the slice-dependent sweeps (the lanes of
    // a batch share their launches); kept if the second plan runs with the same lanes
    Plan Q{};
    Q.dtype = dtype;
    Compiler c2(Q, P.lanes, group_hint, min_chunks);
    if (c2.run(n_inputs, in_ranks, in_modes, in_extents, in_strides, out_rank, out_modes, n_steps,
               path, n_sliced, sliced_modes) == TQ_OK && Q.lanes == P.lanes)
      P = std::move(Q);
  }
  plan_planes_layout(P);   // sizes known at compile time (queries, CPU tests); allocated at materialize
  // the compile arguments, kept for a recompile with another group hint (plan_recompile)
  CompileArgs& a = P.args;
  int nm = 0;
  for (int i = 0; i < n_inputs; ++i) nm += in_ranks[i];
  a.in_ranks.assign(in_ranks, in_ranks + n_inputs);
  a.in_modes.assign(in_modes, in_modes + nm);
  a.in_extents.assign(in_extents, in_extents + nm);
  a.in_strides.clear();
  if (in_strides) a.in_strides.assign(in_strides, in_strides + nm);
  a.out_modes.assign(out_modes, out_modes + out_rank);
  a.path.assign(path, path + 2 * n_steps);
  a.sliced.assign(sliced_modes, sliced_modes + n_sliced);
  P.group_hint = group_hint;
  P.min_chunks = min_chunks;
  return TQ_OK;
}

int plan_recompile(Plan& P, int group_hint, int min_chunks) {
  TQ_CHECK_ARG(P.d_arena == nullptr && P.d_tables == nullptr, "a plan is recompiled before its first execute only");
  TQ_CHECK_ARG(!P.args.in_ranks.empty(), "plan has no compile arguments");
  if (group_hint == P.group_hint && min_chunks == P.min_chunks) return TQ_OK;
  const CompileArgs a = P.args;
  const bool seq = P.use_seq, coop = P.use_coop, planes = P.use_planes, graph = P.use_graph;
  Plan Q;
  TQ_TRY(plan_compile(Q, P.dtype, (int)a.in_ranks.size(), a.in_ranks.data(), a.in_modes.data(),
                      a.in_extents.data(), a.in_strides.empty() ? nullptr : a.in_strides.data(),
                      (int)a.out_modes.size(), a.out_modes.data(), (int)a.path.size() / 2, a.path.data(),
                      (int)a.sliced.size(), a.sliced.data(), group_hint, min_chunks));
  Q.use_seq = seq;
  Q.use_coop = coop;
  Q.use_planes = planes;
  Q.use_graph = graph;
  P = std::move(Q);
  return TQ_OK;
}

void plan_clone_compiled(const Plan& src, Plan& dst) {
  dst = src;
  dst.d_arena = dst.d_tables = dst.d_planes = nullptr;
  dst.owns_device = false;
  dst.device = -1;
  dst.serial = 0;
  dst.h_bad = nullptr;
  dst.profile = 0;
  dst.ev_used.clear();
  dst.ev_free.clear();
  dst.graphs.clear();
  dst.graph_clock = 0;
  dst.cap_stream = nullptr;
  dst.side_streams.clear();
  dst.side_events.clear();
  dst.graph_builds = dst.graph_launches = 0;
  dst.ps_fallbacks = 0;
  dst.run_mode = 0;
}

void plan_planes_layout(Plan& P) {
  if (P.planes_gemm < 0) return;
  const Op& g = P.ops[P.planes_gemm];
  const size_t lanes = (size_t)std::max(1, P.lanes);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  P.planes_lane_bytes = al((size_t)12 * (size_t)(P.planes_n[0] + P.planes_n[1]));
  P.planes_ws_off = lanes * P.planes_lane_bytes;
  // every lane-batch size up to the lane count: a partial batch may pick more K splits (r05c)
  P.planes_sc_off = P.planes_ws_off + al(planes_gemm_workspace(g.M, g.N, g.K, (int64_t)lanes));
  P.planes_bytes = P.planes_sc_off + al(lanes * 2 * sizeof(int32_t));
}

uint64_t next_plan_serial();

int plan_materialize(Plan& P, void* arena, void* tables, hipStream_t stream) {
  TQ_HIP(hipGetDevice(&P.device));
  P.serial = next_plan_serial();
  if (arena || tables) {
    P.d_arena = arena;
    P.d_tables = tables;
    P.owns_device = false;
  } else {
    P.owns_device = true;
    if (P.arena_bytes) TQ_HIP(hipMalloc(&P.d_arena, P.arena_bytes));
    if (P.table_bytes) TQ_HIP(hipMalloc(&P.d_tables, P.table_bytes));
  }
  if (P.table_bytes) {
    std::vector<char> host(P.table_bytes, 0);
    for (size_t i = 0; i < P.perms.size(); ++i)
      if (perm_plan_table_bytes(P.perms[i])) perm_plan_pack_table(P.perms[i], host.data() + P.perm_tab_off[i]);
    for (size_t i = 0; i < P.gtabs.size(); ++i)
      std::memcpy(host.data() + P.gtab_off[i], P.gtabs[i].data(), P.gtabs[i].size() * sizeof(int32_t));
    for (size_t i = 0; i < P.stabs.size(); ++i)
      std::memcpy(host.data() + P.stab_off[i], P.stabs[i].data(), P.stabs[i].size());
    TQ_HIP(hipMemcpyAsync(P.d_tables, host.data(), P.table_bytes, hipMemcpyHostToDevice, stream));
    TQ_HIP(hipStreamSynchronize(stream));
  }
  if (P.n_ps && !P.h_bad) TQ_HIP(hipHostMalloc((void**)&P.h_bad, P.n_slices * sizeof(uint32_t), hipHostMallocDefault));
  // the pre-split boundary GEMM's planes, partials and scale words (plan-owned plans only)
  if (P.planes_gemm >= 0 && P.owns_device && !P.d_planes) {
    plan_planes_layout(P);
    if (hipMalloc(&P.d_planes, P.planes_bytes) != hipSuccess) {
      (void)hipGetLastError();
      P.d_planes = nullptr;   // no room: the GEMM-side split path runs instead
    }
  }
  return TQ_OK;
}

int plan_profile_read(Plan& P, int kind, double* ms, int64_t* launches, double* flops,
                      double* bytes) {
  double t = 0, f = 0, b = 0;
  int64_t n = 0;
  for (auto& ev : P.ev_used) {
    if (kind >= 0 && ev.kind != kind) continue;
    TQ_HIP(hipEventSynchronize(ev.b));
    float e = 0;
    TQ_HIP(hipEventElapsedTime(&e, ev.a, ev.b));
    t += e; f += ev.flops; b += ev.bytes; ++n;
  }
  if (ms) *ms = t;
  if (launches) *launches = n;
  if (flops) *flops = f;
  if (bytes) *bytes = b;
  return TQ_OK;
}

bool sweeps_enabled_global() {
  const char* e = getenv("TQ_SWEEP");
  return !(e && e[0] == '0');
}

namespace {

bool graphs_disabled() {
  static const int v = [] {
    const char* e = getenv("TQ_GRAPH");
    return (e && e[0] == '0') ? 1 : 0;
  }();
  return v != 0;
}

}  // namespace
bool graphs_enabled() { return !graphs_disabled(); }
namespace {

// HIP release calls: the first failure is recorded (tq_last_error) and reported; a resource is
// forgotten only once its release succeeded, so a release refused mid-way (e.g. by a stream
// capture elsewhere in the process: HIP refuses hipGraphExecDestroy / hipFree while any stream
// captures in global mode) can be retried later with nothing leaked or freed twice
int rel(hipError_t e, const char* what, int& rc) {
  if (e == hipSuccess) return 1;
  if (rc == TQ_OK) set_error(std::string("HIP error ") + hipGetErrorString(e) + " releasing " + what);
  rc = TQ_ERR_HIP;
  return 0;
}

int drop_graph_entry(Plan::GraphEntry& g) {
  int rc = TQ_OK;
  if (g.done && rel(hipEventSynchronize(g.done), "graph event", rc) && rel(hipEventDestroy(g.done), "graph event", rc))
    g.done = nullptr;
  if (g.exec && rel(hipGraphExecDestroy(g.exec), "graph exec", rc)) g.exec = nullptr;
  if (g.graph && rel(hipGraphDestroy(g.graph), "graph", rc)) g.graph = nullptr;
  if (rc == TQ_OK) g = Plan::GraphEntry{};
  return rc;
}

int drop_graph(Plan& P) {
  int rc = TQ_OK;
  std::vector<Plan::GraphEntry> keep;
  for (auto& g : P.graphs)
    if (drop_graph_entry(g) != TQ_OK) {
      rc = TQ_ERR_HIP;
      keep.push_back(g);
    }
  P.graphs.swap(keep);
  return rc;
}

}  // namespace

int plan_release(Plan& P) {
  int rc = drop_graph(P);
  if (P.cap_stream && rel(hipStreamDestroy(P.cap_stream), "capture stream", rc)) P.cap_stream = nullptr;
  auto drop_events = [&](std::vector<Plan::Ev>& v) {
    std::vector<Plan::Ev> keep;
    for (auto& ev : v) {
      if (ev.a && rel(hipEventDestroy(ev.a), "event", rc)) ev.a = nullptr;
      if (ev.b && rel(hipEventDestroy(ev.b), "event", rc)) ev.b = nullptr;
      if (ev.a || ev.b) keep.push_back(ev);
    }
    v.swap(keep);
  };
  drop_events(P.ev_used);
  drop_events(P.ev_free);
  {
    std::vector<hipStream_t> ks;
    for (auto s : P.side_streams)
      if (!rel(hipStreamDestroy(s), "group side stream", rc)) ks.push_back(s);
    P.side_streams.swap(ks);
    std::vector<hipEvent_t> ke;
    for (auto e : P.side_events)
      if (!rel(hipEventDestroy(e), "group event", rc)) ke.push_back(e);
    P.side_events.swap(ke);
  }
  if (P.owns_device) {
    if (P.d_arena && rel(hipFree(P.d_arena), "arena", rc)) P.d_arena = nullptr;
    if (P.d_tables && rel(hipFree(P.d_tables), "tables", rc)) P.d_tables = nullptr;
  } else {
    P.d_arena = P.d_tables = nullptr;
  }
  if (P.h_bad && rel(hipHostFree(P.h_bad), "host flag", rc)) P.h_bad = nullptr;
  if (P.d_planes && rel(hipFree(P.d_planes), "planes", rc)) P.d_planes = nullptr;
  return rc;
}


int plan_enqueue(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
                 int64_t s_step, int accumulate, hipStream_t stream);
// the pre-split boundary GEMM runs: the plan has one, its buffers exist, the plan option is on
// and the pre-split (predicted-scale) mode of the split kernel is not running
static bool planes_active(const Plan& P) {
  return P.planes_gemm >= 0 && P.d_planes != nullptr && P.use_planes && !P.run_mode;
}
int plan_launch(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
                int64_t s_step, int accumulate, hipStream_t stream);

int plan_run(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
             int64_t s_step, int accumulate, hipStream_t stream) {
  TQ_CHECK_ARG(s_step >= 1, "slice_step");
  TQ_CHECK_ARG(s_begin >= 0 && s_end <= P.n_slices, "slice range");
  TQ_CHECK_ARG(P.arena_bytes == 0 || P.d_arena, "plan not materialized");
  {
    // a plan's arena, tables and graphs live on one device; running it with another device
    // current would hand that device foreign pointers
    int cur = -1;
    TQ_HIP(hipGetDevice(&cur));
    TQ_CHECK_ARG(P.device < 0 || cur == P.device,
                 "plan was materialized on device " + std::to_string(P.device) +
                     " but device " + std::to_string(cur) + " is current");
  }
  // pre-split GEMM operands (Op::ps_cand) when every candidate still takes the f16 split path
  // under the current library switches, and the stream is not being captured by the caller
  // (the window check below synchronizes)
  P.run_mode = 0;
  if (P.n_ps && P.h_bad) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    TQ_HIP(hipStreamIsCapturing(stream, &cs));
    bool ok = cs == hipStreamCaptureStatusNone;
    for (const Op& op : P.ops)
      if (op.ps_cand && !gemm_c64_presplit_ok(op.transA, op.transB, op.M, op.N, op.K, op.batch, op.lda, op.ldb))
        ok = false;
    P.run_mode = ok ? 1 : 0;
  }
  TQ_TRY(plan_launch(P, inputs, out, s_begin, s_end, s_step, accumulate, stream));
  if (P.use_coop && !P.coop_once.empty() && P.d_tables) {
    // cooperative chain launches (opt-in) rely on their workgroups being co-resident; a wait
    // that gave up (sync[1], counted by the kernel) means the op read stale data: the execute
    // synchronizes to check (outside a caller's capture) and fails instead of returning it
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    TQ_HIP(hipStreamIsCapturing(stream, &cs));
    if (cs == hipStreamCaptureStatusNone) {
      uint32_t gaveup = 0;
      for (size_t r = 0; r < P.coop_once.size(); ++r) {
        uint32_t w = 0;
        char* slot = (char*)P.d_tables + P.sync_off + r * Plan::kSyncSlot + 4;
        TQ_HIP(hipMemcpyAsync(&w, slot, 4, hipMemcpyDeviceToHost, stream));
        TQ_HIP(hipStreamSynchronize(stream));
        if (w) TQ_HIP(hipMemsetAsync(slot, 0, 4, stream));
        gaveup += w;
      }
      if (gaveup) {
        TQ_HIP(hipStreamSynchronize(stream));
        set_error("cooperative sweep chain: " + std::to_string(gaveup) +
                  " workgroup wait(s) gave up (workgroups not co-resident); the result is invalid -- "
                  "run with sweep_coop 0");
        return TQ_ERR_HIP;
      }
    }
  }
  if (P.run_mode) {
    // slices whose operand max left its scale window produced zeros: add them on the split path
    const uint32_t* dbad = reinterpret_cast<const uint32_t*>((const char*)P.d_tables + P.bad_off);
    TQ_HIP(hipMemcpyAsync(P.h_bad, dbad, P.n_slices * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    TQ_HIP(hipStreamSynchronize(stream));
    // a lane-batched candidate GEMM flags its whole batch in the batch's first slice (the
    // other lanes' words are not written): batches are consecutive groups of `lanes` slices
    bool batched = false;
    for (const Op& op : P.ops) batched = batched || (op.ps_cand && op.lane_batch);
    std::vector<int64_t> redo, batch;
    for (int64_t sl = s_begin; sl < s_end; sl += s_step * std::max(1, P.lanes)) {
      batch.clear();
      for (int64_t q = sl; q < s_end && (int64_t)batch.size() < std::max(1, P.lanes); q += s_step) batch.push_back(q);
      for (int64_t q : batch)
        if (batched ? P.h_bad[batch[0]] != 0 : P.h_bad[q] != 0) redo.push_back(q);
    }
    P.run_mode = 0;
    for (int64_t sl : redo) TQ_TRY(plan_enqueue(P, inputs, out, sl, sl + 1, 1, 1, stream));
    P.ps_fallbacks += (int64_t)redo.size();
  }
  return TQ_OK;
}

int plan_launch(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
                int64_t s_step, int accumulate, hipStream_t stream) {
  if (P.profile || !P.use_graph || graphs_disabled())
    return plan_enqueue(P, inputs, out, s_begin, s_end, s_step, accumulate, stream);
  // a caller's stream capture (a torch.cuda.graph around the call): the launches go straight
  // into that capture -- a graph of the plan's own, built on its side stream and launched into
  // the capturing stream, ran once at capture time and was not part of the caller's replays
  {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    TQ_HIP(hipStreamIsCapturing(stream, &cs));
    if (cs != hipStreamCaptureStatusNone)
      return plan_enqueue(P, inputs, out, s_begin, s_end, s_step, accumulate, stream);
  }
  Plan::GraphKey key;
  key.inputs.assign(inputs, inputs + P.n_inputs);
  key.out = out; key.b = s_begin; key.e = s_end; key.s = s_step; key.acc = accumulate;
  key.mode = P.run_mode;
  key.planes = planes_active(P) ? 1 : 0;
  key.seq = P.use_seq;
  key.coop = P.use_coop;
  constexpr size_t kMaxGraphs = 8;
  Plan::GraphEntry* hit = nullptr;
  for (auto& g : P.graphs) if (g.key == key) hit = &g;
  if (!hit) {
    if (P.graphs.size() >= kMaxGraphs) {  // evict the least recently used (after it finished)
      auto lru = std::min_element(P.graphs.begin(), P.graphs.end(),
                                  [](const Plan::GraphEntry& a, const Plan::GraphEntry& b) { return a.used < b.used; });
      drop_graph_entry(*lru);
      P.graphs.erase(lru);
    }
    if (!P.cap_stream) TQ_HIP(hipStreamCreateWithFlags(&P.cap_stream, hipStreamNonBlocking));
    TQ_HIP(hipStreamBeginCapture(P.cap_stream, hipStreamCaptureModeThreadLocal));
    const int rc = plan_enqueue(P, inputs, out, s_begin, s_end, s_step, accumulate, P.cap_stream);
    hipGraph_t g = nullptr;
    const hipError_t ce = hipStreamEndCapture(P.cap_stream, &g);
    if (rc != TQ_OK) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    TQ_HIP(ce);
    Plan::GraphEntry e;
    e.key = key;
    e.graph = g;
    TQ_HIP(hipGraphInstantiate(&e.exec, g, nullptr, nullptr, 0));
    TQ_HIP(hipEventCreateWithFlags(&e.done, hipEventDisableTiming));
    P.graphs.push_back(e);
    hit = &P.graphs.back();
    ++P.graph_builds;
  }
  hit->used = ++P.graph_clock;
  TQ_HIP(hipGraphLaunch(hit->exec, stream));
  TQ_HIP(hipEventRecord(hit->done, stream));
  ++P.graph_launches;
  return TQ_OK;
}

// ---- executor: one plan, or a GROUP of plans compiled from the same network (blocks as lanes).
// A group executes its plans' schedules in lockstep: every sweep2 level (and dense-sweep level,
// and chain launch) of all instances is ONE launch whose op list holds every instance's ops --
// the slice-lane mechanism with an instance index -- so G amplitude blocks in flight cost the
// launches of one; the other ops (GEMM, permute, lane sum, ...) run per instance.  A group of one
// plan is exactly the single-plan executor.
namespace {

bool sweep_lanes_on();   // TQ_SWEEP_LANES (default 1): per-slice table sweeps lane-merged

struct Inst {
  Plan* P = nullptr;
  const void* const* inputs = nullptr;
  void* out = nullptr;
  std::vector<std::vector<int64_t>> lane_in_off;
  std::vector<int64_t> lane_sl;
  int cur = 0;             // lane the launches address
  double beta_out = 0.0;   // the first slice of a non-accumulating call overwrites the output
  bool first = true;
  bool lanes_summed = false;
};

class Exec {
 public:
  Exec(std::vector<Inst>& insts, hipStream_t stream) : I_(insts), st_(stream), P0_(*insts[0].P) {}

  int run(int64_t s_begin, int64_t s_end, int64_t s_step, int accumulate);

 private:
  std::vector<Inst>& I_;
  hipStream_t st_;
  Plan& P0_;
  int lane_gemm_ = 1;   // > 1: the GEMM launch below covers that many lanes

  size_t esz() const { return P0_.esz; }
  char* ptr(const Inst& x, const BufRef& b) const {
    const Plan& P = *x.P;
    switch (b.kind) {
      case BUF_INPUT: return (char*)x.inputs[b.index] + (x.lane_in_off[x.cur][b.index] + b.off) * P.esz;
      case BUF_ARENA: return (char*)P.d_arena + P.lane_phys + (size_t)x.cur * P.lane_stride + b.off * P.esz;
      case BUF_PINNED: return (char*)P.d_arena + b.off * P.esz;
      case BUF_OUTPUT: return (char*)x.out + b.off * P.esz;
      case BUF_TABLE: return (char*)P.d_tables + b.off;
    }
    return nullptr;
  }
  static void set_lane(Inst& x, int j) {
    x.cur = j;
    x.beta_out = (x.first && x.cur == 0) ? 0.0 : 1.0;
  }
  void set_lane_all(int j) {
    for (auto& x : I_) set_lane(x, j);
  }
  static uint32_t* amax_word(const Inst& x, int w) {
    return reinterpret_cast<uint32_t*>((char*)x.P->d_tables + x.P->amax_off) + w;
  }
  // lane j's copy of max word w: per-slice words have one set per lane (the pre-split mode keeps
  // one shared set: its scales are predicted per batch)
  static int lane_amax_stride(const Inst& x, int w) {
    return (w >= x.P->n_amax_once && !x.P->run_mode) ? x.P->n_amax_slice : 0;
  }
  static uint32_t* amax_lane(const Inst& x, int w, int j) { return amax_word(x, w + j * lane_amax_stride(x, w)); }
  // scale word of per-slice max word w; window flag of slice q
  static int32_t* sc_word(const Inst& x, int w) {
    return reinterpret_cast<int32_t*>((char*)x.P->d_tables + x.P->sc_off) + (w - x.P->n_amax_once);
  }
  static uint32_t* bad_word(const Inst& x, int64_t q) {
    return reinterpret_cast<uint32_t*>((char*)x.P->d_tables + x.P->bad_off) + q;
  }
  // the pre-split boundary GEMM: lane j's planes of operand r (0 = A, 1 = B) and scale words
  static _Float16* planes_ptr(const Inst& x, int j, int r) {
    const Plan& P = *x.P;
    return reinterpret_cast<_Float16*>((char*)P.d_planes + (size_t)j * P.planes_lane_bytes +
                                       (r ? (size_t)12 * P.planes_n[0] : 0));
  }
  static int32_t* planes_sc(const Inst& x, int j, int r) {
    return reinterpret_cast<int32_t*>((char*)x.P->d_planes + x.P->planes_sc_off) + 2 * j + r;
  }

  // profiling (HIP events on the stream; the group's first plan holds the records)
  Plan::Ev ev_begin(int kind) {
    Plan::Ev ev{};
    if (P0_.ev_free.empty()) {
      if (hipEventCreate(&ev.a) != hipSuccess || hipEventCreate(&ev.b) != hipSuccess) ev.kind = -1;
    } else {
      ev = P0_.ev_free.back();
      P0_.ev_free.pop_back();
    }
    if (ev.kind == -1) return ev;
    ev.kind = kind;
    ev.flops = 0;
    ev.bytes = 0;
    return ev;
  }

  int launch_one(Inst& x, const Op& op);
  int fill_s2(const Inst& x, S2Op& o, const Op& op, int stab) const;
  SweepArgs sweep_args(const Inst& x, const Op& op, double beta) const;
  int sweep_lanes_ = 0;   // > 0: the OP_SWEEP entry below runs every lane of the batch in one launch
  // per-instance work of a group: member k > 0 on side stream k - 1 (forked from and joined back
  // into the execution stream: parallel branches of the captured graph), member 0 on the stream
  hipStream_t ost_ = nullptr;   // the stream launch_one / lane sums use (st_ unless forked)
  template <typename F>
  int each_instance(F&& f);
  int launch_chain(int b, int e, int coop);
  int launch(const std::vector<int>& grp);
};

// the table-driven sweep op's launch record for instance x's current lane
SweepArgs Exec::sweep_args(const Inst& x, const Op& op, double beta) const {
  const Plan& P = *x.P;
      SweepArgs a;
      const char* blob = (const char*)P.d_tables + P.stab_off[op.stab];
      a.X = ptr(x, op.a);
      a.Y = ptr(x, op.c);
      a.ncols = op.ncols;
      auto lg = [](int64_t v) {
        if (v <= 0 || (v & (v - 1))) return -1;
        int l = 0;
        while ((int64_t(1) << l) < v) ++l;
        return l;
      };
      a.nruns = op.nruns;
      for (int r = 0; r < op.nruns; ++r) {
        a.run_ext[r] = op.run_ext[r]; a.run_in[r] = op.run_in[r]; a.run_out[r] = op.run_out[r];
        a.run_shift[r] = lg(op.run_ext[r]);
      }
      a.tin = op.tin;
      a.tout = op.tout;
      a.tin_shift = lg(op.tin);
      a.tout_shift = lg(op.tout);
      a.tabs = (const int32_t*)(blob + op.tabs_at);
      a.tab_len = op.tab_len;
      a.tin_off = (const int64_t*)blob;
      a.tout_off = (const int64_t*)(blob + op.tout_off_at);
      a.ngates = (int)op.sgates.size();
      for (int j = 0; j < a.ngates; ++j) {
        const SweepGate& g = op.sgates[j];
        a.G[j] = ptr(x, g.g);
        a.gidx[j] = g.gtab >= 0 ? (const int32_t*)((char*)P.d_tables + P.gtab_off[g.gtab]) : nullptr;
        a.K[j] = g.K; a.N[j] = g.N; a.W[j] = g.W;
        a.tab_at[j] = (int)g.tab_off;
      }
      // power-of-two outer extents: per-bit column-offset weights
      {
        bool p2 = true;
        int nb = 0;
        for (int r = 0; r < op.nruns && p2; ++r) {
          const int l = lg(op.run_ext[r]);
          if (l < 0 || nb + l > 48) { p2 = false; break; }
          for (int b = 0; b < l; ++b) {
            a.w_in[nb + b] = op.run_in[r] << b;
            a.w_out[nb + b] = op.run_out[r] << b;
          }
          nb += l;
        }
        a.colbits = p2 ? nb : -1;
      }
      a.load_colfast = op.load_colfast;
      a.store_colfast = op.store_colfast;
      a.use_beta = beta != 0.0;
      a.beta = beta;
  return a;
}

template <typename F>
int Exec::each_instance(F&& f) {
  static const bool fork = [] {
    const char* e = getenv("TQ_GROUP_FORK");
    return !(e && e[0] == '0');
  }();
  const int n = (int)I_.size();
  if (n == 1 || !fork) {
    ost_ = st_;
    for (auto& x : I_) TQ_TRY(f(x));
    return TQ_OK;
  }
  Plan& P = P0_;
  while ((int)P.side_streams.size() < n - 1) {
    hipStream_t s = nullptr;
    TQ_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    P.side_streams.push_back(s);
  }
  while ((int)P.side_events.size() < n) {
    hipEvent_t e = nullptr;
    TQ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    P.side_events.push_back(e);
  }
  TQ_HIP(hipEventRecord(P.side_events[0], st_));
  int rc = TQ_OK;
  for (int k = 1; k < n && rc == TQ_OK; ++k) {
    hipStream_t s = P.side_streams[k - 1];
    TQ_HIP(hipStreamWaitEvent(s, P.side_events[0], 0));
    ost_ = s;
    rc = f(I_[k]);
    TQ_HIP(hipEventRecord(P.side_events[k], s));
  }
  ost_ = st_;
  if (rc == TQ_OK) rc = f(I_[0]);
  for (int k = 1; k < n; ++k) TQ_HIP(hipStreamWaitEvent(st_, P.side_events[k], 0));
  return rc;
}

int Exec::launch_one(Inst& x, const Op& op) {
  Plan& P = *x.P;
  const hipStream_t st = ost_ ? ost_ : st_;
  const double beta = op.writes_output ? x.beta_out : 0.0;
  const bool planes_on = planes_active(P);
  if (planes_on && op.kind == OP_GEMM && &op == &P.ops[P.planes_gemm]) {
    // lane batch: entries = the batch's lanes (planes and scale words at their lane strides),
    // the combine sums them into lane 0's result when the plan sums the lanes (Op::lane_sum)
    const int j0 = lane_gemm_ > 1 ? 0 : x.cur;
    PlanesGemmArgs a;
    a.A = planes_ptr(x, j0, 0);
    a.B = planes_ptr(x, j0, 1);
    a.sA = a.sB = (int64_t)(P.planes_lane_bytes / 2);
    a.psA = P.planes_n[0];
    a.psB = P.planes_n[1];
    a.lda = op.lda;
    a.ldb = op.ldb;
    a.M = (int)op.M;
    a.N = (int)op.N;
    a.K = op.K;
    a.batch = lane_gemm_;
    a.W = reinterpret_cast<float*>((char*)P.d_planes + P.planes_ws_off);
    a.ws_bytes = P.planes_sc_off - P.planes_ws_off;
    PlanesCombineArgs c;
    c.sc_a = planes_sc(x, j0, 0);
    c.sc_b = planes_sc(x, j0, 1);
    c.sc_stride = 2;
    c.C = ptr(x, op.c);
    c.ldc = op.ldc;
    c.sC = (int64_t)(P.lane_stride / P.esz);
    c.lane_sum = lane_gemm_ > 1 && op.lane_sum;
    c.beta = (float)beta;
    return planes_gemm_launch(a, c, st);
  }
  switch (op.kind) {
    case OP_PERMUTE:
      TQ_TRY(perm_plan_launch(P.perms[op.perm], (char*)P.d_tables + P.perm_tab_off[op.perm], ptr(x, op.a),
                              ptr(x, op.c), beta, st));
      break;
    case OP_GEMM: {
      if (op.skinny) {
        SkinnyArgs a = op.sk;
        a.A = ptr(x, op.a);
        a.B = ptr(x, op.b);
        a.C = ptr(x, op.c);
        a.W = op.ws_bytes ? ptr(x, op.ws) : nullptr;
        a.beta = beta;
        TQ_TRY(skinny_strided_launch(P.dtype, a, st));
        break;
      }
      GemmPresplit ps;
      const bool pre = P.run_mode && op.ps_cand;
      if (pre) {
        ps.sc_a = sc_word(x, op.amax_a);
        ps.sc_b = sc_word(x, op.amax_b);
        ps.bad = bad_word(x, x.lane_sl[x.cur]);
      }
      if (lane_gemm_ > 1) {   // every lane of the batch in one launch (Op::lane_batch)
        const int64_t ls = (int64_t)(P.lane_stride / P.esz);
        // pre-split: one window flag for the batch, in its first slice's word
        TQ_TRY(gemm_launch(P.dtype, op.transA, op.transB, op.M, op.N, op.K, lane_gemm_, ptr(x, op.a), op.lda,
                           op.a.kind == BUF_ARENA ? ls : 0, ptr(x, op.b), op.ldb, op.b.kind == BUF_ARENA ? ls : 0,
                           beta, ptr(x, op.c), op.ldc, ls, (char*)P.d_arena + P.lane_ws_off, P.lane_ws_bytes, st,
                           op.amax_a >= 0 ? amax_word(x, op.amax_a) : nullptr,
                           op.amax_b >= 0 ? amax_word(x, op.amax_b) : nullptr, pre ? &ps : nullptr,
                           op.amax_a >= 0 ? lane_amax_stride(x, op.amax_a) : 0,
                           op.amax_b >= 0 ? lane_amax_stride(x, op.amax_b) : 0));
        break;
      }
      TQ_TRY(gemm_launch(P.dtype, op.transA, op.transB, op.M, op.N, op.K, op.batch, ptr(x, op.a), op.lda, op.sA,
                         ptr(x, op.b), op.ldb, op.sB, beta, ptr(x, op.c), op.ldc, op.sC,
                         op.ws_bytes ? ptr(x, op.ws) : nullptr, op.ws_bytes, st,
                         op.amax_a >= 0 ? amax_lane(x, op.amax_a, x.cur) : nullptr,
                         op.amax_b >= 0 ? amax_lane(x, op.amax_b, x.cur) : nullptr, pre ? &ps : nullptr));
      break;
    }
    case OP_APPLY:
      TQ_TRY(apply_launch(P.dtype, op.O, op.K, op.M, op.K2, op.I, op.N, ptr(x, op.a), ptr(x, op.b),
                          op.gtab >= 0 ? (const int32_t*)((char*)P.d_tables + P.gtab_off[op.gtab]) : nullptr,
                          ptr(x, op.c), beta, st));
      break;
    case OP_AXPY:
      TQ_TRY(axpy_launch(P.dtype, op.n, ptr(x, op.a), ptr(x, op.c), beta, st));
      break;
    case OP_SWEEP: {
      const SweepArgs a = sweep_args(x, op, beta);
      TQ_TRY(sweep_launch(P.dtype, a, st));
      break;
    }
    default:
      set_error("internal: op kind");
      return TQ_ERR_INVALID;
  }
  return TQ_OK;
}

// a sweep2 op's launch record from descriptor stabs[stab] (the instance's current lane)
int Exec::fill_s2(const Inst& x, S2Op& o, const Op& op, int stab) const {
  const Plan& P = *x.P;
  o.desc = (const S2Desc*)((const char*)P.d_tables + P.stab_off[stab]);
  o.X = ptr(x, op.a);
  o.Y = ptr(x, op.c);
  const S2Desc* hd = reinterpret_cast<const S2Desc*>(P.stabs[stab].data());
  for (size_t g = 0; g < op.sgates.size(); ++g) {
    o.G[g] = ptr(x, op.sgates[g].g);
    int mx = 0;
    for (int t = 0; t < hd->gate[g].K * hd->gate[g].N; ++t) mx = std::max(mx, hd->gate[g].gidx[t] + 1);
    if (mx > kS2GateRaw) {
      set_error("internal: sweep2 gate tensor too large");
      return TQ_ERR_INVALID;
    }
    o.gnum[g] = (uint8_t)mx;
  }
  o.beta = op.writes_output ? x.beta_out : 0.0;
  o.use_beta = o.beta != 0.0;
  o.amax = op.amax_word >= 0 ? amax_lane(x, op.amax_word, x.cur) : nullptr;
  o.split_sc = P.run_mode && op.ps_gemm >= 0 ? sc_word(x, op.amax_word) : nullptr;
  // host-built lane / chunk-base tables behind the descriptor (TQ_S2_HOSTTAB=0: computed in the
  // kernel, the r05 prologue)
  static const bool host_tabs = [] {
    const char* e = getenv("TQ_S2_HOSTTAB");
    return !(e && e[0] == '0');
  }();
  const char* blob = (const char*)P.d_tables + P.stab_off[stab];
  o.rows = host_tabs ? (hd->npass & 0xff) | (hd->ngates & 0xff) << 8 | (hd->colbits & 0xff) << 16 : 0;
  o.lanes = host_tabs && hd->aux_lanes ? reinterpret_cast<const uint4*>(blob + hd->aux_lanes) : nullptr;
  o.cbase = host_tabs && hd->aux_cb ? reinterpret_cast<const int64_t*>(blob + hd->aux_cb) : nullptr;
  return TQ_OK;
}

// Plan::seq_once run [b, e): its ops in order, a workgroup per (instance, stream), one launch (as
// many instances per launch as kS2SeqMaxStreams allows); or (coop >= 0) Plan::coop_once run
// `coop`: its ops in order on coop_width workgroups each, one launch per instance
int Exec::launch_chain(int b, int e, int coop) {
  const bool prof = (P0_.profile >> (int)OP_SWEEP) & 1;
  if (coop >= 0) {
    for (auto& x : I_) {
      Plan& P = *x.P;
      Plan::Ev ev{};
      if (prof) {
        ev = ev_begin((int)OP_SWEEP);
        TQ_HIP(hipEventRecord(ev.a, st_));
      }
      const int w = P.coop_width[coop];
      S2Launch L;
      L.seq = 1;
      L.sync = reinterpret_cast<uint32_t*>((char*)P.d_tables + P.sync_off + (size_t)coop * Plan::kSyncSlot);
      for (int i = b; i < e; ++i) {
        const Op& op = P.ops[P.sched_once[i][0]];
        S2Op& o = L.op[L.nops];
        TQ_TRY(fill_s2(x, o, op, op.stab));
        o.block_begin = 0;
        o.nblocks = w;
        o.lds_io = kS2Coop | (L.nops * w) << 8 | (op.lds_io & 4);   // (bit 2: set by the planner)
        ++L.nops;
        ev.flops += op.flops;
        ev.bytes += op.bytes;
      }
      L.sync_total = L.nops * w;
      TQ_TRY(sweep2_launch(P.dtype, L, st_));
      if (prof) {
        TQ_HIP(hipEventRecord(ev.b, st_));
        P0_.ev_used.push_back(ev);
      }
    }
    return TQ_OK;
  }
  int nstreams = 1, nops = 0;
  for (int i = b; i < e; ++i)
    for (int j : P0_.sched_once[i]) {
      nstreams = std::max(nstreams, P0_.seq_stream[j] + 1);
      ++nops;
    }
  const int per = std::max(1, std::min(kS2SeqMaxStreams / nstreams, kS2MaxOps / std::max(1, nops)));
  for (size_t k0 = 0; k0 < I_.size(); k0 += (size_t)per) {
    Plan::Ev ev{};
    if (prof) {
      ev = ev_begin((int)OP_SWEEP);
      TQ_HIP(hipEventRecord(ev.a, st_));
    }
    S2Launch L;
    L.seq = 1;
    for (size_t k = k0; k < std::min(I_.size(), k0 + (size_t)per); ++k) {
      const Inst& x = I_[k];
      const Plan& P = *x.P;
      for (int i = b; i < e; ++i)
        for (int j : P.sched_once[i]) {
          const Op& op = P.ops[j];
          S2Op& o = L.op[L.nops++];
          TQ_TRY(fill_s2(x, o, op, op.stab1));
          o.lds_io = op.lds_io;
          // an LDS hand-off moves the whole tensor: the kernel's first-chunk path only
          if ((o.lds_io & 3) && reinterpret_cast<const S2Desc*>(P.stabs[op.stab1].data())->nchunks != 1) {
            set_error("internal: sweep2 LDS hand-off on a multi-chunk layout");
            return TQ_ERR_INVALID;
          }
          o.block_begin = (int)(k - k0) * nstreams + P.seq_stream[j];   // the (instance, stream) workgroup
          o.nblocks = 1;
          ev.flops += op.flops;
          ev.bytes += op.bytes;
        }
    }
    TQ_TRY(sweep2_launch(P0_.dtype, L, st_));
    if (prof) {
      TQ_HIP(hipEventRecord(ev.b, st_));
      P0_.ev_used.push_back(ev);
    }
  }
  return TQ_OK;
}

// one entry of the schedule: a single op (per instance), or independent sweep2 ops of every
// instance (and, merged across the batch, of every lane) in one launch
int Exec::launch(const std::vector<int>& grp) {
  const Op& op0 = P0_.ops[grp[0]];
  const int pkind = op0.kind == OP_SWEEP2 ? (int)OP_SWEEP : op0.kind;
  const int nl = (int)I_[0].lane_sl.size();
  Plan::Ev ev{};
  const bool prof = (P0_.profile >> pkind) & 1;
  bool lanes_merge = op0.kind == OP_SWEEP2 && nl > 1 && !op0.invariant;
  for (int j : grp) lanes_merge = lanes_merge && !P0_.ops[j].writes_output;
  if (prof) {
    ev = ev_begin(pkind);
    // a lane-batched GEMM or a sweep level merged across the batch's lanes does every lane's
    // work; a group does every instance's
    const int mult = (lanes_merge ? nl : sweep_lanes_ > 1 ? sweep_lanes_ : lane_gemm_) * (int)I_.size();
    for (int j : grp) {
      ev.flops += P0_.ops[j].flops * mult;
      ev.bytes += P0_.ops[j].bytes * mult;
    }
    TQ_HIP(hipEventRecord(ev.a, st_));
  }
  if (op0.kind == OP_SWEEP2) {
    // (instance, lane, op) triples of this level: every lane's ops when the level is merged
    // across the batch, else each instance's current lane; at most kS2MaxOps per launch
    struct Item { int k, lane, q; };
    std::vector<Item> items, dense;
    for (int k = 0; k < (int)I_.size(); ++k)
      for (int j = 0; j < (lanes_merge ? nl : 1); ++j)
        for (int q : grp) (P0_.ops[q].s2_dense ? dense : items).push_back({k, lanes_merge ? j : I_[k].cur, q});
    std::vector<int> keep(I_.size());
    for (size_t k = 0; k < I_.size(); ++k) keep[k] = I_[k].cur;
    // dense ops (tq_sweepd.hip): their own launches, at most two input tile sizes each
    // (TQ_S2D_MIX=0: one)
    static const bool s2d_mix = [] {
      const char* e = getenv("TQ_S2D_MIX");
      return !(e && e[0] == '0');
    }();
    static const bool s2d_nt = [] {
      const char* e = getenv("TQ_S2D_NT");
      return e && e[0] == '1';
    }();
    while (!dense.empty()) {
      S2DLaunch L;
      const int tin = P0_.ops[dense[0].q].tin;
      int tin2 = 0;
      std::vector<Item> rest;
      int blocks = 0;
      for (auto& it : dense) {
        Inst& x = I_[it.k];
        const Plan& P = *x.P;
        const Op& op = P.ops[it.q];
        if (op.tin != tin && tin2 == 0 && s2d_mix && !s2d_nt) tin2 = op.tin;
        if ((op.tin != tin && op.tin != tin2) || L.nops == kS2MaxOps) {
          rest.push_back(it);
          continue;
        }
        set_lane(x, it.lane);
        S2DOp& o = L.op[L.nops++];
        o.desc = (const S2Dense*)((const char*)P.d_tables + P.stab_off[op.stab]);
        o.X = ptr(x, op.a);
        o.M = ptr(x, op.b);
        o.Y = ptr(x, op.c);
        o.tin = op.tin;
        o.tout = op.tout;
        o.block_begin = blocks;
        o.nblocks = s2d_blocks(op.ncols);
        o.ncols = op.ncols;
        blocks += o.nblocks;
        o.beta = op.writes_output ? x.beta_out : 0.0;
        o.use_beta = o.beta != 0.0;
        o.amax = op.amax_word >= 0 ? amax_lane(x, op.amax_word, x.cur) : nullptr;
        o.split_sc = P.run_mode && op.ps_gemm >= 0 ? sc_word(x, op.amax_word) : nullptr;
        if (planes_active(P) && op.planes_role) {
          o.planes = planes_ptr(x, x.cur, op.planes_role - 1);
          o.pstride = P.planes_n[op.planes_role - 1];
          o.amax_in = amax_lane(x, op.planes_in_amax, x.cur);
          o.sc_out = planes_sc(x, x.cur, op.planes_role - 1);
          o.amax = nullptr;
        }
      }
      TQ_TRY(sweepd_launch(P0_.dtype, L, st_));
      dense.swap(rest);
    }
    for (size_t i0 = 0; i0 < items.size(); i0 += kS2MaxOps) {
      S2Launch L;
      L.nops = (int)std::min<size_t>(kS2MaxOps, items.size() - i0);
      int blocks = 0;
      for (int q = 0; q < L.nops; ++q) {
        const Item& it = items[i0 + q];
        Inst& x = I_[it.k];
        set_lane(x, it.lane);
        const Op& op = x.P->ops[it.q];
        S2Op& o = L.op[q];
        TQ_TRY(fill_s2(x, o, op, op.stab));
        o.block_begin = blocks;
        o.nblocks = s2_blocks(op.s2_nchunks);
        blocks += o.nblocks;
      }
      TQ_TRY(sweep2_launch(P0_.dtype, L, st_));
    }
    for (size_t k = 0; k < I_.size(); ++k) set_lane(I_[k], keep[k]);
  } else if (op0.kind == OP_SWEEP && sweep_lanes_ > 1) {
    // the per-slice table sweep of every lane in one launch (grid.y = lane; SweepLanes)
    TQ_TRY(each_instance([&](Inst& x) -> int {
      const Op& op = x.P->ops[grp[0]];
      const int keep = x.cur;
      SweepLanes ls;
      ls.n = sweep_lanes_;
      for (int j = 0; j < sweep_lanes_; ++j) {
        set_lane(x, j);
        ls.X[j] = ptr(x, op.a);
        ls.Y[j] = ptr(x, op.c);
        for (size_t g = 0; g < op.sgates.size(); ++g) ls.G[j][g] = ptr(x, op.sgates[g].g);
      }
      set_lane(x, 0);
      const SweepArgs a = sweep_args(x, op, 0.0);
      set_lane(x, keep);
      return sweep_launch_lanes(x.P->dtype, a, ls, ost_ ? ost_ : st_);
    }));
  } else {
    TQ_TRY(each_instance([&](Inst& x) -> int { return launch_one(x, x.P->ops[grp[0]]); }));
  }
  if (prof) {
    TQ_HIP(hipEventRecord(ev.b, st_));
    P0_.ev_used.push_back(ev);
  }
  return TQ_OK;
}

int Exec::run(int64_t s_begin, int64_t s_end, int64_t s_step, int accumulate) {
  const int ns = (int)P0_.sliced.size();
  for (auto& x : I_) x.first = !accumulate;
  if (s_begin >= s_end) {
    for (auto& x : I_)
      if (!accumulate && x.P->out_numel) TQ_HIP(hipMemsetAsync(x.out, 0, x.P->out_numel * esz(), st_));
    return TQ_OK;
  }
  // Slices run in batches of P.lanes (slice lanes, Plan::lanes): lane j owns its own copy of the
  // per-slice arena part, the batch's sweep2 levels share launches across lanes, other ops run
  // lane by lane in lane order (so output accumulation keeps its order)
  const int64_t nlanes = std::max(1, P0_.lanes);
  std::vector<int64_t> in_off;
  for (int64_t s0 = s_begin; s0 < s_end; s0 += s_step * nlanes) {
    for (auto& x : I_) {
      const Plan& P = *x.P;
      x.lane_sl.clear();
      x.lane_in_off.clear();
      in_off.assign(P.n_inputs, 0);
      for (int64_t sl = s0; sl < s_end && (int64_t)x.lane_sl.size() < nlanes; sl += s_step) {
        // decode slice id (row-major over sliced modes) -> per-input element offsets
        std::vector<int64_t> idx(ns);
        int64_t rem = sl;
        for (int q = ns - 1; q >= 0; --q) {
          idx[q] = rem % P.sliced_ext[q];
          rem /= P.sliced_ext[q];
        }
        for (int i = 0; i < P.n_inputs; ++i) {
          int64_t o = 0;
          for (int q = 0; q < ns; ++q) o += idx[q] * P.inputs[i].slice_stride[q];
          in_off[i] = o;
        }
        x.lane_sl.push_back(sl);
        x.lane_in_off.push_back(in_off);
      }
      set_lane(x, 0);
      x.lanes_summed = false;
    }
    const int nl = (int)I_[0].lane_sl.size();
    if (s0 == s_begin) {
      for (auto& x : I_)
        if (x.P->n_amax_once) TQ_HIP(hipMemsetAsync(amax_word(x, 0), 0, x.P->n_amax_once * sizeof(uint32_t), st_));
      size_t run = 0, crun = 0;
      for (int i = 0; i < (int)P0_.sched_once.size();) {
        while (P0_.use_seq && run < P0_.seq_once.size() && P0_.seq_once[run].first < i) ++run;
        if (P0_.use_seq && run < P0_.seq_once.size() && P0_.seq_once[run].first == i) {
          TQ_TRY(launch_chain(i, P0_.seq_once[run].second, -1));
          i = P0_.seq_once[run].second;
          continue;
        }
        while (P0_.use_coop && crun < P0_.coop_once.size() && P0_.coop_once[crun].first < i) ++crun;
        if (P0_.use_coop && crun < P0_.coop_once.size() && P0_.coop_once[crun].first == i) {
          TQ_TRY(launch_chain(i, P0_.coop_once[crun].second, (int)crun));
          i = P0_.coop_once[crun].second;
          continue;
        }
        TQ_TRY(launch(P0_.sched_once[i]));
        ++i;
      }
    }
    // per-slice max words: one set per lane (pre-split mode: one set shared by the batch's
    // lanes, max-ed over all of them -- an upper bound of every lane's operand)
    for (auto& x : I_) {
      const Plan& P = *x.P;
      if (P.n_amax_slice && P.run_mode)   // scales from the previous slice's max, then max = 0
        TQ_TRY(presplit_prep_launch(amax_word(x, P.n_amax_once), sc_word(x, P.n_amax_once), P.n_amax_slice, st_));
      else if (P.n_amax_slice)
        TQ_HIP(hipMemsetAsync(amax_word(x, P.n_amax_once), 0, (size_t)P.n_amax_slice * nl * sizeof(uint32_t), st_));
    }
    for (auto& grp : P0_.sched_slice) {
      const Op& op0 = P0_.ops[grp[0]];
      bool merged = op0.kind == OP_SWEEP2;
      for (int j : grp) merged = merged && !P0_.ops[j].writes_output;
      if (merged || nl == 1) {
        set_lane_all(0);
        TQ_TRY(launch(grp));
        bool sums = false;
        for (int j : grp) sums = sums || P0_.ops[j].lane_sum;
        if (merged && nl > 1 && sums)
          TQ_TRY(each_instance([&](Inst& x) -> int {
            for (int j : grp)
              if (x.P->ops[j].lane_sum) {   // a lane-merged level whose lanes an output permute sums
                TQ_TRY(lane_sum_launch(x.P->dtype, x.P->ops[j].nc, ptr(x, x.P->ops[j].c),
                                       (int64_t)(x.P->lane_stride / esz()), nl, ost_));
                x.lanes_summed = true;
              }
            return TQ_OK;
          }));
      } else if (op0.kind == OP_GEMM && op0.lane_batch) {
        set_lane_all(0);
        lane_gemm_ = nl;
        const int rc = each_instance([&](Inst& x) -> int {
          TQ_TRY(launch_one(x, x.P->ops[grp[0]]));
          if (op0.lane_sum) {
            // (the pre-split GEMM's combine has summed the lanes already)
            if (!(planes_active(*x.P) && grp[0] == x.P->planes_gemm))
              TQ_TRY(lane_sum_launch(x.P->dtype, op0.nc, ptr(x, op0.c), (int64_t)(x.P->lane_stride / esz()), nl,
                                     ost_));
            x.lanes_summed = true;
          }
          return TQ_OK;
        });
        lane_gemm_ = 1;
        TQ_TRY(rc);
      } else if (op0.lane_once && I_[0].lanes_summed) {
        set_lane_all(0);
        TQ_TRY(launch(grp));
      } else if (op0.kind == OP_SWEEP && grp.size() == 1 && !op0.writes_output && sweep_lanes_on() &&
                 nl <= kSweepMaxLanes) {
        // a per-slice table sweep whose lanes write their own copies: one launch for the batch
        set_lane_all(0);
        sweep_lanes_ = nl;
        const int rc = launch(grp);
        sweep_lanes_ = 0;
        TQ_TRY(rc);
      } else {
        for (int j = 0; j < nl; ++j) {
          set_lane_all(j);
          TQ_TRY(launch(grp));
        }
      }
    }
    for (auto& x : I_) x.first = false;
  }
  return TQ_OK;
}

bool sweep_lanes_on() {
  static const bool v = [] {
    const char* e = getenv("TQ_SWEEP_LANES");
    return !(e && e[0] == '0');
  }();
  return v;
}

// the plans of a group are the same compiled network (identical op lists and schedules)
bool same_structure(const Plan& a, const Plan& b) {
  if (a.dtype != b.dtype || a.ops.size() != b.ops.size() || a.sched_once != b.sched_once ||
      a.sched_slice != b.sched_slice || a.lanes != b.lanes || a.n_slices != b.n_slices ||
      a.seq_once != b.seq_once || a.seq_stream != b.seq_stream || a.use_seq != b.use_seq ||
      a.use_coop != b.use_coop || a.coop_once != b.coop_once || a.n_inputs != b.n_inputs ||
      planes_active(a) != planes_active(b) || a.planes_gemm != b.planes_gemm)
    return false;
  for (size_t i = 0; i < a.ops.size(); ++i)
    if (a.ops[i].kind != b.ops[i].kind || a.ops[i].stab != b.ops[i].stab || a.ops[i].stab1 != b.ops[i].stab1 ||
        a.ops[i].invariant != b.ops[i].invariant || a.ops[i].writes_output != b.ops[i].writes_output)
      return false;
  return true;
}

}  // namespace

int plan_enqueue(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
                 int64_t s_step, int accumulate, hipStream_t stream) {
  std::vector<Inst> I(1);
  I[0].P = &P;
  I[0].inputs = inputs;
  I[0].out = out;
  Exec ex(I, stream);
  return ex.run(s_begin, s_end, s_step, accumulate);
}

int group_enqueue(Plan* const* plans, int n, const void* const* const* inputs, void* const* outs, int64_t s_begin,
                  int64_t s_end, int64_t s_step, int accumulate, hipStream_t stream) {
  std::vector<Inst> I((size_t)n);
  for (int k = 0; k < n; ++k) {
    I[k].P = plans[k];
    I[k].inputs = inputs[k];
    I[k].out = outs[k];
  }
  Exec ex(I, stream);
  return ex.run(s_begin, s_end, s_step, accumulate);
}

uint64_t next_plan_serial() {
  static std::atomic<uint64_t> c{0};
  return ++c;
}

int plan_run_group(Plan* const* plans, int n, const void* const* const* inputs, void* const* outs, int64_t s_begin,
                   int64_t s_end, int64_t s_step, int accumulate, hipStream_t stream) {
  TQ_CHECK_ARG(n >= 1 && plans && inputs && outs, "empty group");
  if (n == 1) return plan_run(*plans[0], inputs[0], outs[0], s_begin, s_end, s_step, accumulate, stream);
  Plan& P0 = *plans[0];
  TQ_CHECK_ARG(s_step >= 1, "slice_step");
  TQ_CHECK_ARG(s_begin >= 0 && s_end <= P0.n_slices, "slice range");
  int cur = -1;
  TQ_HIP(hipGetDevice(&cur));
  for (int k = 0; k < n; ++k) {
    Plan& P = *plans[k];
    TQ_CHECK_ARG(P.arena_bytes == 0 || P.d_arena, "plan not materialized");
    TQ_CHECK_ARG(P.device < 0 || cur == P.device, "a group plan was materialized on another device");
    for (int q = 0; q < k; ++q)
      TQ_CHECK_ARG(plans[q] != plans[k] && outs[q] != outs[k], "a group runs distinct plans into distinct outputs");
    P.run_mode = 0;   // no pre-split (predicted-scale) GEMM mode in a group
    TQ_CHECK_ARG(same_structure(P0, P), "the plans of a group must be compiled from the same network");
  }
  TQ_CHECK_ARG(!P0.use_coop, "cooperative chain launches do not run in a group");
  const bool eager = P0.profile || !P0.use_graph || graphs_disabled();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  TQ_HIP(hipStreamIsCapturing(stream, &cs));
  if (eager || cs != hipStreamCaptureStatusNone)
    return group_enqueue(plans, n, inputs, outs, s_begin, s_end, s_step, accumulate, stream);
  // one hipGraph of the whole group, cached in the first plan under every member's serial,
  // inputs and output (a serial is never reused, so a replay cannot address a freed plan)
  Plan::GraphKey key;
  for (int k = 0; k < n; ++k) {
    key.inputs.insert(key.inputs.end(), inputs[k], inputs[k] + plans[k]->n_inputs);
    key.group.push_back(outs[k]);
    key.group.push_back(reinterpret_cast<const void*>((uintptr_t)plans[k]->serial));
  }
  key.out = outs[0]; key.b = s_begin; key.e = s_end; key.s = s_step; key.acc = accumulate;
  key.planes = planes_active(P0) ? 1 : 0;
  key.seq = P0.use_seq;
  constexpr size_t kMaxGraphs = 8;
  Plan::GraphEntry* hit = nullptr;
  for (auto& g : P0.graphs) if (g.key == key) hit = &g;
  if (!hit) {
    if (P0.graphs.size() >= kMaxGraphs) {
      auto lru = std::min_element(P0.graphs.begin(), P0.graphs.end(),
                                  [](const Plan::GraphEntry& a, const Plan::GraphEntry& b) { return a.used < b.used; });
      drop_graph_entry(*lru);
      P0.graphs.erase(lru);
    }
    if (!P0.cap_stream) TQ_HIP(hipStreamCreateWithFlags(&P0.cap_stream, hipStreamNonBlocking));
    TQ_HIP(hipStreamBeginCapture(P0.cap_stream, hipStreamCaptureModeThreadLocal));
    const int rc = group_enqueue(plans, n, inputs, outs, s_begin, s_end, s_step, accumulate, P0.cap_stream);
    hipGraph_t g = nullptr;
    const hipError_t ce = hipStreamEndCapture(P0.cap_stream, &g);
    if (rc != TQ_OK) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    TQ_HIP(ce);
    Plan::GraphEntry e;
    e.key = key;
    e.graph = g;
    TQ_HIP(hipGraphInstantiate(&e.exec, g, nullptr, nullptr, 0));
    TQ_HIP(hipEventCreateWithFlags(&e.done, hipEventDisableTiming));
    P0.graphs.push_back(e);
    hit = &P0.graphs.back();
    ++P0.graph_builds;
  }
  hit->used = ++P0.graph_clock;
  TQ_HIP(hipGraphLaunch(hit->exec, stream));
  TQ_HIP(hipEventRecord(hit->done, stream));
  ++P0.graph_launches;
  return TQ_OK;
}

}  // namespace tq
