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

#include <algorithm>
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

class Compiler {
 public:
  Compiler(Plan& P) : P_(P) {}

  int run(int n_inputs, const int32_t* in_ranks, const int32_t* in_modes, const int64_t* in_ext,
          const int64_t* in_strides, int out_rank, const int32_t* out_modes, int n_steps,
          const int32_t* path, int n_sliced, const int32_t* sliced) {
    P_.esz = dtype_size(P_.dtype);
    cplx_ = dtype_complex(P_.dtype);
    P_.n_inputs = n_inputs;
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
      TQ_TRY(step(s, live_[x], live_[y], s == n_steps - 1, res));
      live_.push_back(res);
    }
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
    P_.pinned_base = (size_t)((arena_.peak() + kAlign - 1) / kAlign * kAlign);
    P_.arena_bytes = P_.pinned_base + (size_t)pinned_arena_.peak();
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
    P_.table_bytes = tb;
    for (auto& op : P_.ops) {
      (op.invariant ? P_.flops_once : P_.flops_slice) += op.flops;
      (op.invariant ? P_.bytes_once : P_.bytes_slice) += op.bytes;
      P_.n_gemm += op.kind == OP_GEMM;
      P_.n_apply += op.kind == OP_APPLY;
      P_.n_permute += op.kind == OP_PERMUTE;
    }
    P_.flops = P_.flops_once + P_.flops_slice * (double)P_.n_slices;
    P_.bytes = P_.bytes_once + P_.bytes_slice * (double)P_.n_slices;
    std::ostringstream d;
    for (size_t i = 0; i < P_.ops.size(); ++i)
      d << (P_.ops[i].invariant ? "[once]  " : "[slice] ") << P_.ops[i].note << "\n";
    P_.describe = d.str();
    return TQ_OK;
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

  BufRef new_buf(int64_t numel, int64_t* off_out) {
    const int64_t off = arena_.alloc(numel * (int64_t)P_.esz);
    *off_out = off;
    BufRef b;
    b.kind = BUF_ARENA;
    b.off = off / (int64_t)P_.esz;
    return b;
  }
  void release(const Live& L) {
    if (L.owned && L.buf.kind == BUF_ARENA) arena_.release(L.buf.off * (int64_t)P_.esz);
  }
  // the step result's buffer: pinned results live in the separate pinned region
  BufRef new_result_buf(int64_t numel, int64_t* off_out) {
    if (!pin_next_) return new_buf(numel, off_out);
    const int64_t off = pinned_arena_.alloc(numel * (int64_t)P_.esz);
    *off_out = off;
    BufRef b;
    b.kind = BUF_PINNED;
    b.off = off / (int64_t)P_.esz;
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
    op.bytes = 2.0 * n * P_.esz;
    std::ostringstream o;
    o << "step " << step << " PERMUTE " << why << " " << modes_str(X.modes) << "->" << modes_str(order)
      << " n=" << n << (pp.use_generic ? " [generic]" : "") << (to_output ? " ->OUT" : "");
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

    const size_t first_op = P_.ops.size();
    int rc = TQ_OK;
    const bool applied = try_apply(s, A0, B0, final, batch, contr, sumA, sumB, res, rc);
    if (rc != TQ_OK) return rc;
    if (!applied) TQ_TRY(gemm_step(s, A0, B0, final, batch, contr, freeA, freeB, sumA, sumB, res));
    for (int m : res.modes) cnt_[m]++;
    // slice-invariant hoisting: a step that reads no sliced input runs once per execute; its
    // result is pinned in the arena when a slice-dependent step consumes it
    res.dep = A0.dep || B0.dep;
    for (size_t k = first_op; k < P_.ops.size(); ++k) P_.ops[k].invariant = !res.dep;
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

  bool try_apply(int s, const Live& A0, const Live& B0, bool final, const std::set<int>& batch,
                 const std::set<int>& contr, const std::set<int>& sumA, const std::set<int>& sumB,
                 Live& res, int& rc) {
    if (!batch.empty() || !sumA.empty() || !sumB.empty() || contr.empty()) return false;
    const bool a_big = A0.numel() >= B0.numel();
    const Live& Bg = a_big ? A0 : B0;
    const Live& Sm = a_big ? B0 : A0;
    if (!Bg.contiguous()) return false;
    const int64_t K = ext_of(std::vector<int>(contr.begin(), contr.end()));
    const int64_t N = Sm.numel() / K;
    if (Sm.numel() > 1024 || K > 32 || N > 32) return false;
    // contracted modes must form at most two runs in the big operand: [O][K1][M][K2][I]
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
    std::vector<int> korder(Bg.modes.begin() + p1, Bg.modes.begin() + p1 + c1);
    korder.insert(korder.end(), Bg.modes.begin() + p2, Bg.modes.begin() + p2 + c2);
    std::vector<int> nfree;
    for (int m : Sm.modes) if (!contr.count(m)) nfree.push_back(m);
    // small operand read as G[K][N] through a gather table (any layout / strides, no launch)
    int gtab = -1;
    {
      std::vector<int> gorder = korder;
      gorder.insert(gorder.end(), nfree.begin(), nfree.end());
      if (!(Sm.contiguous() && Sm.modes == gorder)) {
        std::vector<int64_t> gext, gst;
        for (int m : gorder) {
          const int p = Sm.pos(m);
          gext.push_back(Sm.ext[p]);
          gst.push_back(Sm.stride[p]);
        }
        const int64_t n = prod(gext);
        std::vector<int32_t> tab(n);
        for (int64_t t = 0; t < n; ++t) {
          int64_t rem = t, off = 0;
          for (int d = (int)gext.size() - 1; d >= 0; --d) { off += (rem % gext[d]) * gst[d]; rem /= gext[d]; }
          tab[t] = (int32_t)off;
        }
        gtab = (int)P_.gtabs.size();
        P_.gtabs.push_back(std::move(tab));
      }
    }
    std::vector<int> order(Bg.modes.begin(), Bg.modes.begin() + p1);
    order.insert(order.end(), nfree.begin(), nfree.end());
    order.insert(order.end(), Bg.modes.begin() + p1 + c1, Bg.modes.begin() + p2);
    order.insert(order.end(), Bg.modes.begin() + p2 + c2, Bg.modes.end());
    int64_t O = 1, K1 = 1, M = 1, K2 = 1, I = 1;
    for (int i = 0; i < p1; ++i) O *= Bg.ext[i];
    for (int i = p1; i < p1 + c1; ++i) K1 *= Bg.ext[i];
    for (int i = p1 + c1; i < p2; ++i) M *= Bg.ext[i];
    for (int i = p2; i < p2 + c2; ++i) K2 *= Bg.ext[i];
    for (size_t i = p2 + c2; i < Bg.modes.size(); ++i) I *= Bg.ext[i];
    const int64_t outn = O * N * M * I;
    bool direct;
    int64_t roff;
    BufRef tgt = result_target(final, order, outn, &direct, &roff);
    Op op;
    op.kind = OP_APPLY;
    op.a = Bg.buf;
    op.b = Sm.buf;
    op.gtab = gtab;
    op.c = tgt;
    op.writes_output = direct;
    op.O = O; op.K = K1; op.M = M; op.K2 = K2; op.N = N; op.I = I;
    op.step = s;
    op.flops = (double)O * M * I * K * N * (cplx_ ? 8.0 : 2.0);
    op.bytes = (double)(O * K * M * I + outn + K * N) * P_.esz;
    std::ostringstream o;
    o << "step " << s << " APPLY O=" << O << " K1=" << K1 << " M=" << M << " K2=" << K2
      << " I=" << I << " N=" << N << (direct ? " ->OUT" : "");
    op.note = o.str();
    P_.ops.push_back(op);
    res.modes = order;
    for (int m : order) res.ext.push_back(ext_[m]);
    res.stride = contig_strides(res.ext);
    if (direct) {
      res.buf = tgt;
      res.owned = false;
    } else {
      res.buf = tgt;
      res.owned = true;
      if (final) {
        rc = emit_permute(res, P_.out_modes, {}, BufRef{BUF_OUTPUT, 0, 0}, true, s, "result->out");
        if (rc != TQ_OK) return true;
      }
    }
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
    int64_t wsoff = -1;
    if (op.ws_bytes) {
      wsoff = arena_.alloc((int64_t)op.ws_bytes);
      op.ws = BufRef{BUF_ARENA, 0, wsoff / (int64_t)P_.esz};
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
    if (wsoff >= 0) arena_.release(wsoff);
    if (aoff >= 0) arena_.release(aoff);
    if (boff >= 0) arena_.release(boff);
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
  bool cplx_ = false;
  std::vector<Live> live_;
  std::map<int, int64_t> ext_;
  std::map<int, int> cnt_;
  Arena arena_;
  Arena pinned_arena_;
  std::vector<char> pinned_;
  bool pin_next_ = false;
};

}  // namespace

int plan_compile(Plan& P, int dtype, int n_inputs, const int32_t* in_ranks, const int32_t* in_modes,
                 const int64_t* in_extents, const int64_t* in_strides, int out_rank,
                 const int32_t* out_modes, int n_steps, const int32_t* path, int n_sliced,
                 const int32_t* sliced_modes) {
  TQ_CHECK_ARG(dtype_valid(dtype), "dtype");
  TQ_CHECK_ARG(n_inputs >= 1, "need at least one input");
  TQ_CHECK_ARG(n_steps == n_inputs - 1, "a pairwise path has n_inputs - 1 steps");
  TQ_CHECK_ARG(out_rank >= 0 && out_rank <= TQ_MAX_RANK, "output rank");
  TQ_CHECK_ARG(n_sliced >= 0 && n_sliced <= 62, "n_sliced");
  P = Plan{};
  P.dtype = dtype;
  Compiler c(P);
  return c.run(n_inputs, in_ranks, in_modes, in_extents, in_strides, out_rank, out_modes, n_steps,
               path, n_sliced, sliced_modes);
}

int plan_materialize(Plan& P, void* arena, void* tables, hipStream_t stream) {
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
    TQ_HIP(hipMemcpyAsync(P.d_tables, host.data(), P.table_bytes, hipMemcpyHostToDevice, stream));
    TQ_HIP(hipStreamSynchronize(stream));
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

namespace {

bool graphs_disabled() {
  static const int v = [] {
    const char* e = getenv("TQ_GRAPH");
    return (e && e[0] == '0') ? 1 : 0;
  }();
  return v != 0;
}

void drop_graph(Plan& P) {
  if (P.graph_exec) (void)hipGraphExecDestroy(P.graph_exec);
  if (P.graph) (void)hipGraphDestroy(P.graph);
  P.graph_exec = nullptr;
  P.graph = nullptr;
  P.has_graph = false;
}

}  // namespace

void plan_release(Plan& P) {
  drop_graph(P);
  if (P.cap_stream) (void)hipStreamDestroy(P.cap_stream);
  P.cap_stream = nullptr;
  for (auto& ev : P.ev_used) { (void)hipEventDestroy(ev.a); (void)hipEventDestroy(ev.b); }
  for (auto& ev : P.ev_free) { (void)hipEventDestroy(ev.a); (void)hipEventDestroy(ev.b); }
  P.ev_used.clear();
  P.ev_free.clear();
  if (P.owns_device) {
    if (P.d_arena) (void)hipFree(P.d_arena);
    if (P.d_tables) (void)hipFree(P.d_tables);
  }
  P.d_arena = P.d_tables = nullptr;
}


int plan_enqueue(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
                 int64_t s_step, int accumulate, hipStream_t stream);

int plan_run(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
             int64_t s_step, int accumulate, hipStream_t stream) {
  TQ_CHECK_ARG(s_step >= 1, "slice_step");
  TQ_CHECK_ARG(s_begin >= 0 && s_end <= P.n_slices, "slice range");
  TQ_CHECK_ARG(P.arena_bytes == 0 || P.d_arena, "plan not materialized");
  if (P.profile || !P.use_graph || graphs_disabled())
    return plan_enqueue(P, inputs, out, s_begin, s_end, s_step, accumulate, stream);
  Plan::GraphKey key;
  key.inputs.assign(inputs, inputs + P.n_inputs);
  key.out = out; key.b = s_begin; key.e = s_end; key.s = s_step; key.acc = accumulate;
  if (!(P.has_graph && key == P.gkey)) {
    drop_graph(P);
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
    P.graph = g;
    TQ_HIP(hipGraphInstantiate(&P.graph_exec, P.graph, nullptr, nullptr, 0));
    P.gkey = key;
    P.has_graph = true;
    ++P.graph_builds;
  }
  TQ_HIP(hipGraphLaunch(P.graph_exec, stream));
  ++P.graph_launches;
  return TQ_OK;
}

int plan_enqueue(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
                 int64_t s_step, int accumulate, hipStream_t stream) {
  const size_t esz = P.esz;
  std::vector<int64_t> in_off(P.n_inputs, 0);
  const int ns = (int)P.sliced.size();
  bool first = !accumulate;
  if (s_begin >= s_end) {
    if (!accumulate && P.out_numel) TQ_HIP(hipMemsetAsync(out, 0, P.out_numel * esz, stream));
    return TQ_OK;
  }
  for (int64_t sl = s_begin; sl < s_end; sl += s_step) {
    // decode slice id (row-major over sliced modes) -> per-input element offsets
    std::vector<int64_t> idx(ns);
    int64_t rem = sl;
    for (int q = ns - 1; q >= 0; --q) { idx[q] = rem % P.sliced_ext[q]; rem /= P.sliced_ext[q]; }
    for (int i = 0; i < P.n_inputs; ++i) {
      int64_t o = 0;
      for (int q = 0; q < ns; ++q) o += idx[q] * P.inputs[i].slice_stride[q];
      in_off[i] = o;
    }
    auto ptr = [&](const BufRef& b) -> char* {
      switch (b.kind) {
        case BUF_INPUT: return (char*)inputs[b.index] + (in_off[b.index] + b.off) * esz;
        case BUF_ARENA: return (char*)P.d_arena + b.off * esz;
        case BUF_PINNED: return (char*)P.d_arena + P.pinned_base + b.off * esz;
        case BUF_OUTPUT: return (char*)out + b.off * esz;
      }
      return nullptr;
    };
    const double beta_out = first ? 0.0 : 1.0;
    for (const Op& op : P.ops) {
      if (op.invariant && sl != s_begin) continue;  // hoisted: computed in this call's first slice
      const double beta = op.writes_output ? beta_out : 0.0;
      Plan::Ev ev{};
      const bool prof = (P.profile >> op.kind) & 1;
      if (prof) {
        if (P.ev_free.empty()) {
          TQ_HIP(hipEventCreate(&ev.a));
          TQ_HIP(hipEventCreate(&ev.b));
        } else {
          ev = P.ev_free.back();
          P.ev_free.pop_back();
        }
        ev.kind = op.kind; ev.flops = op.flops; ev.bytes = op.bytes;
        TQ_HIP(hipEventRecord(ev.a, stream));
      }
      switch (op.kind) {
        case OP_PERMUTE:
          TQ_TRY(perm_plan_launch(P.perms[op.perm], (char*)P.d_tables + P.perm_tab_off[op.perm],
                                  ptr(op.a), ptr(op.c), beta, stream));
          break;
        case OP_GEMM:
          TQ_TRY(gemm_launch(P.dtype, op.transA, op.transB, op.M, op.N, op.K, op.batch, ptr(op.a),
                             op.lda, op.sA, ptr(op.b), op.ldb, op.sB, beta, ptr(op.c), op.ldc, op.sC,
                             op.ws_bytes ? ptr(op.ws) : nullptr, op.ws_bytes, stream));
          break;
        case OP_APPLY:
          TQ_TRY(apply_launch(P.dtype, op.O, op.K, op.M, op.K2, op.I, op.N, ptr(op.a), ptr(op.b),
                              op.gtab >= 0 ? (const int32_t*)((char*)P.d_tables + P.gtab_off[op.gtab]) : nullptr,
                              ptr(op.c), beta, stream));
          break;
        case OP_AXPY:
          TQ_TRY(axpy_launch(P.dtype, op.n, ptr(op.a), ptr(op.c), beta, stream));
          break;
      }
      if (prof) {
        TQ_HIP(hipEventRecord(ev.b, stream));
        P.ev_used.push_back(ev);
      }
    }
    first = false;
  }
  return TQ_OK;
}

}  // namespace tq
