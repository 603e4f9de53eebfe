// extern "C" surface of libtneqhip.so (declared in include/tneqhip.h).
#include <cstring>
#include <string>
#include <exception>
#include <new>
#include <vector>

#include "tq_common.h"
#include "tq_optim.h"
#include "tq_plan.h"

// development aid: TQ_TRACE_FILE=<path> appends a line per plan execute / destroy step (finds
// which call a native abort comes from when the test runner swallows stderr)
static void trace(const char* what, const void* p, int64_t v = 0) {
  static const char* path = getenv("TQ_TRACE_FILE");
  if (!path) return;
  if (FILE* f = fopen(path, "a")) {
    fprintf(f, "%s %p %lld\n", what, p, (long long)v);
    fclose(f);
  }
}
// ... and records the exception behind a std::terminate (an exception leaving a destructor)
static const bool g_trace_terminate = [] {
  if (!getenv("TQ_TRACE_FILE")) return false;
  static std::terminate_handler prev = std::set_terminate([] {
    const char* what = "(no exception)";
    std::string msg;
    if (auto ep = std::current_exception()) {
      try {
        std::rethrow_exception(ep);
      } catch (const std::exception& e) {
        msg = e.what();
        what = msg.c_str();
      } catch (...) {
        what = "(non-std exception)";
      }
    }
    if (FILE* f = fopen(getenv("TQ_TRACE_FILE"), "a")) {
      fprintf(f, "terminate: %s\n", what);
      fclose(f);
    }
    if (prev) prev();
    abort();
  });
  return true;
}();

namespace tq {
namespace {
thread_local std::string g_last_error;
}
void set_error(const std::string& msg) { g_last_error = msg; }
const std::string& last_error() { return g_last_error; }
}  // namespace tq

namespace tq {
bool gemm_3m();
bool gemm_bf16();
bool gemm_f16();
int gemm_f16_var();
bool gemm_presplit_enabled();
bool gemm_configure(const char* key, int64_t v);
bool graphs_enabled();
bool sweeps_enabled_global();
}

extern "C" int64_t tq_library_query(const char* key) {
  if (!key) return -1;
  const std::string k(key);
  if (k == "gemm_3m") return tq::gemm_3m() ? 1 : 0;
  if (k == "gemm_bf16") return tq::gemm_bf16() ? 1 : 0;
  if (k == "gemm_f16") return tq::gemm_f16() ? 1 : 0;
  if (k == "gemm_f16_var") return tq::gemm_f16_var();
  if (k == "gemm_presplit") return tq::gemm_presplit_enabled() ? 1 : 0;
  if (k == "graphs") return tq::graphs_enabled() ? 1 : 0;
  if (k == "sweep") return tq::sweeps_enabled_global() ? 1 : 0;

  return -1;
}

extern "C" int tq_library_set(const char* key, int64_t value) {
  if (!key) return TQ_ERR_INVALID;
  if (tq::gemm_configure(key, value)) return TQ_OK;
  tq::set_error(std::string("tq_library_set: unknown key ") + key);
  return TQ_ERR_INVALID;
}

// development only (not in the public header): drains the sweep2 phase stamps of a library
// built with -DTQ_S2_TIMING (9 x u64 per record); returns the record count (0 otherwise)
extern "C" int tq_debug_sweep2_timing(unsigned long long* out, int n) { return tq::sweep2_timing(out, n); }
// development only: in-kernel clock records of a -DTQ_KCLOCK build (tq_kclock.h), 4 x u64 each
// (s_memtime, s_memrealtime at workgroup 0's start and end); which: 0 sweep2, 1 planes GEMM,
// 2 the complex64 K-outer split GEMM.  Returns the record count (0 in the product build)
extern "C" int tq_debug_kernel_clock(int which, unsigned long long* out, int n) {
  switch (which) {
    case 0: return tq::sweep2_kclock(out, n);
    case 1: return tq::planes_gemm_kclock(out, n);
    case 2: return tq::kouter_kclock(out, n);
  }
  return -1;
}

struct tq_plan_s {
  tq::Plan plan;
  bool materialized = false;
};

#define TQ_GUARD_BEGIN try {
#define TQ_GUARD_END                                                   \
  }                                                                    \
  catch (const std::bad_alloc&) {                                      \
    tq::set_error("host allocation failed");                           \
    return TQ_ERR_ALLOC;                                               \
  }                                                                    \
  catch (const std::exception& e) {                                    \
    tq::set_error(std::string("exception: ") + e.what());              \
    return TQ_ERR_INVALID;                                             \
  }

extern "C" {

int tq_version(void) { return (0 << 16) | 1; }

int tq_last_error(char* buf, size_t n) {
  const std::string& e = tq::last_error();
  if (buf && n) {
    const size_t k = std::min(n - 1, e.size());
    std::memcpy(buf, e.data(), k);
    buf[k] = 0;
  }
  return (int)e.size();
}

int tq_device_synchronize(void) {
  TQ_HIP(hipDeviceSynchronize());
  return TQ_OK;
}

int tq_permute(int dtype, int rank, const int64_t* shape, const int64_t* src_strides,
               const void* src, void* dst, double beta, void* stream) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(rank == 0 || (shape && src_strides), "null shape/strides");
  return tq::permute_launch(dtype, rank, shape, src_strides, src, dst, beta, (hipStream_t)stream);
  TQ_GUARD_END
}

int tq_gemm_batched(int dtype, int transA, int transB, int64_t M, int64_t N, int64_t K,
                    int64_t batch, const void* A, int64_t lda, int64_t strideA, const void* B,
                    int64_t ldb, int64_t strideB, double beta, void* C, int64_t ldc,
                    int64_t strideC, void* workspace, size_t ws_bytes, void* stream) {
  TQ_GUARD_BEGIN
  return tq::gemm_launch(dtype, transA, transB, M, N, K, batch, A, lda, strideA, B, ldb, strideB,
                         beta, C, ldc, strideC, workspace, ws_bytes, (hipStream_t)stream);
  TQ_GUARD_END
}

size_t tq_planes_gemm_workspace(int64_t M, int64_t N, int64_t K, int64_t batch) {
  if (M < 1 || N < 1 || K < 1 || batch < 1) return 0;
  return tq::planes_gemm_workspace(M, N, K, batch);
}

int tq_planes_gemm_check(int64_t M, int64_t N, int64_t K, int64_t batch, int64_t lda, int64_t ldb,
                         size_t ws_bytes) {
  TQ_GUARD_BEGIN
  return tq::planes_gemm_check(M, N, K, batch, lda, ldb, ws_bytes);
  TQ_GUARD_END
}

size_t tq_gemm_workspace_size(int dtype, int64_t M, int64_t N, int64_t K, int64_t batch) {
  if (!tq::dtype_valid(dtype)) return 0;
  return tq::gemm_workspace(dtype, M, N, K, batch);
}

int tq_axpy(int dtype, int64_t n, const void* x, void* y, double beta, void* stream) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(tq::dtype_valid(dtype), "dtype");
  return tq::axpy_launch(dtype, n, x, y, beta, (hipStream_t)stream);
  TQ_GUARD_END
}

static int pair_plan(tq::Plan& P, int dtype, int rankA, const int64_t* shapeA, const int32_t* modesA,
                     int rankB, const int64_t* shapeB, const int32_t* modesB, int rankC,
                     const int32_t* modesC) {
  TQ_CHECK_ARG(rankA >= 0 && rankB >= 0 && rankC >= 0, "rank");
  std::vector<int32_t> ranks = {rankA, rankB};
  std::vector<int32_t> modes(modesA, modesA + rankA);
  modes.insert(modes.end(), modesB, modesB + rankB);
  std::vector<int64_t> ext(shapeA, shapeA + rankA);
  ext.insert(ext.end(), shapeB, shapeB + rankB);
  const int32_t path[2] = {0, 1};
  return tq::plan_compile(P, dtype, 2, ranks.data(), modes.data(), ext.data(), nullptr, rankC,
                          modesC, 1, path, 0, nullptr);
}

size_t tq_contract_pair_workspace(int dtype, int rankA, const int64_t* shapeA,
                                  const int32_t* modesA, int rankB, const int64_t* shapeB,
                                  const int32_t* modesB, int rankC, const int32_t* modesC) {
  try {
    tq::Plan P;
    if (pair_plan(P, dtype, rankA, shapeA, modesA, rankB, shapeB, modesB, rankC, modesC) != TQ_OK)
      return 0;
    return P.arena_bytes + P.table_bytes + 256;
  } catch (...) {
    return 0;
  }
}

int tq_contract_pair(int dtype, int rankA, const int64_t* shapeA, const int32_t* modesA,
                     const void* A, int rankB, const int64_t* shapeB, const int32_t* modesB,
                     const void* B, int rankC, const int32_t* modesC, void* C, void* workspace,
                     size_t ws_bytes, void* stream) {
  TQ_GUARD_BEGIN
  tq::Plan P;
  // a one-shot plan: launched eagerly (no graph capture, no capture stream), and every HIP
  // resource it holds (events, graphs, owned memory) is released on every return path
  struct Release {
    tq::Plan& p;
    ~Release() { tq::plan_release(p); }
  } release{P};
  TQ_TRY(pair_plan(P, dtype, rankA, shapeA, modesA, rankB, shapeB, modesB, rankC, modesC));
  P.use_graph = false;
  const size_t need = P.arena_bytes + P.table_bytes + 256;
  TQ_CHECK_ARG(ws_bytes >= need || (P.arena_bytes + P.table_bytes) == 0, "workspace too small");
  char* ws = (char*)workspace;
  char* arena = ws;
  char* tables = ws + (P.arena_bytes + 255) / 256 * 256;
  TQ_TRY(tq::plan_materialize(P, P.arena_bytes ? arena : nullptr,
                              P.table_bytes ? tables : nullptr, (hipStream_t)stream));
  if (!P.arena_bytes && !P.table_bytes) P.owns_device = false;
  const void* ins[2] = {A, B};
  return tq::plan_run(P, ins, C, 0, 1, 1, 0, (hipStream_t)stream);
  TQ_GUARD_END
}

int tq_plan_create(tq_plan* out, int dtype, int n_inputs, const int32_t* in_ranks,
                   const int32_t* in_modes, const int64_t* in_extents, const int64_t* in_strides,
                   int out_rank, const int32_t* out_modes, int n_steps, const int32_t* path,
                   int n_sliced, const int32_t* sliced_modes) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(out != nullptr, "null plan pointer");
  *out = nullptr;
  auto* h = new tq_plan_s();
  int rc = tq::plan_compile(h->plan, dtype, n_inputs, in_ranks, in_modes, in_extents, in_strides,
                            out_rank, out_modes, n_steps, path, n_sliced, sliced_modes);
  if (rc != TQ_OK) {
    tq::plan_release(h->plan);
    delete h;
    return rc;
  }
  *out = h;
  return TQ_OK;
  TQ_GUARD_END
}

int tq_plan_clone(tq_plan src, tq_plan* out) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(src != nullptr && out != nullptr, "null plan");
  *out = nullptr;
  auto* h = new tq_plan_s();
  tq::plan_clone_compiled(src->plan, h->plan);
  *out = h;
  return TQ_OK;
  TQ_GUARD_END
}

int tq_plan_set(tq_plan p, const char* key, int64_t value) {
  if (!p || !key) {
    tq::set_error("tq_plan_set: null argument");
    return TQ_ERR_INVALID;
  }
  const std::string k(key);
  if (k == "graph") {            // 0: launch eagerly (e.g. inside a caller's stream capture)
    p->plan.use_graph = value != 0;
    return TQ_OK;
  }
  if (k == "sweep_chain") {      // 0: the small sweep2 ops of a chain run one launch per level
    p->plan.use_seq = value != 0;
    return TQ_OK;
  }
  if (k == "gemm_planes") {      // 0: the boundary GEMM on the GEMM-side split kernel
    p->plan.use_planes = value != 0;
    return TQ_OK;
  }
  if (k == "group_hint") {       // compile again for lockstep groups of `value` plans (before the first execute)
    if (p->materialized) {
      tq::set_error("tq_plan_set: group_hint before the plan's first execute only");
      return TQ_ERR_INVALID;
    }
    TQ_GUARD_BEGIN
    return tq::plan_recompile(p->plan, (int)value, p->plan.min_chunks);
    TQ_GUARD_END
  }
  if (k == "min_chunks") {       // compile again: big sweep ops in at least `value` chunks (0: default)
    if (p->materialized) {
      tq::set_error("tq_plan_set: min_chunks before the plan's first execute only");
      return TQ_ERR_INVALID;
    }
    TQ_GUARD_BEGIN
    return tq::plan_recompile(p->plan, p->plan.group_hint, (int)value);
    TQ_GUARD_END
  }
  if (k == "sweep_coop") {       // 0: the multi-chunk sweep2 levels of a chain run one launch each
    p->plan.use_coop = value != 0;
    return TQ_OK;
  }
  tq::set_error("tq_plan_set: unknown key " + k);
  return TQ_ERR_INVALID;
}

int64_t tq_plan_query(tq_plan p, const char* key) {
  if (!p || !key) return -1;
  const tq::Plan& P = p->plan;
  const std::string k(key);
  if (k == "n_slices") return P.n_slices;
  if (k == "arena_bytes") return (int64_t)P.arena_bytes;
  if (k == "table_bytes") return (int64_t)P.table_bytes;
  if (k == "flops") return (int64_t)P.flops;
  if (k == "bytes_moved") return (int64_t)P.bytes;
  if (k == "flops_once") return (int64_t)P.flops_once;
  if (k == "flops_slice") return (int64_t)P.flops_slice;
  if (k == "bytes_once") return (int64_t)P.bytes_once;
  if (k == "bytes_slice") return (int64_t)P.bytes_slice;
  if (k == "n_ops_once") { int64_t c = 0; for (auto& o : P.ops) c += o.invariant; return c; }
  if (k == "n_kernels") return (int64_t)P.ops.size();
  if (k == "graph_builds") return P.graph_builds;
  if (k == "graph_launches") return P.graph_launches;
  if (k == "n_presplit") return P.n_ps;
  if (k == "lanes") return P.lanes;
  if (k == "group_hint") return P.group_hint;
  if (k == "min_chunks") return P.min_chunks;
  if (k == "presplit_fallbacks") return P.ps_fallbacks;
  if (k == "n_gemm") return P.n_gemm;
  if (k == "n_apply") return P.n_apply;
  if (k == "n_permute") return P.n_permute;
  if (k == "n_sweep") return P.n_sweep;
  if (k == "n_sweep_gates") return P.n_sweep_gates;
  if (k == "n_sweep2") { int64_t c = 0; for (auto& o : P.ops) c += o.kind == tq::OP_SWEEP2; return c; }
  if (k == "n_launch_once") {   // launches of the hoisted part as executed (chain launches merged)
    int64_t c = P.n_launch_once;
    if (P.use_seq) for (auto& r : P.seq_once) c -= r.second - r.first - 1;
    if (P.use_coop) for (auto& r : P.coop_once) c -= r.second - r.first - 1;
    return c;
  }
  if (k == "n_chain_launches") return P.use_seq ? (int64_t)P.seq_once.size() : 0;
  if (k == "n_coop_launches") return P.use_coop ? (int64_t)P.coop_once.size() : 0;
  if (k == "coop_timeouts") {    // waits of cooperative chain launches that gave up (expected 0)
    int64_t c = 0;
    for (size_t r = 0; r < P.coop_once.size() && P.d_tables; ++r) {
      uint32_t w = 0;
      if (hipMemcpy(&w, (const char*)P.d_tables + P.sync_off + r * tq::Plan::kSyncSlot + 4, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
      c += w;
    }
    return c;
  }
  if (k == "n_coop_ops") {
    int64_t c = 0;
    if (P.use_coop) for (auto& r : P.coop_once) c += r.second - r.first;
    return c;
  }
  if (k == "n_launch_slice") return P.n_launch_slice;
  if (k == "planes_gemm") return P.planes_gemm >= 0 ? 1 : 0;   // a pre-split boundary GEMM was planned
  if (k == "planes_active") return (P.planes_gemm >= 0 && P.use_planes && (P.d_planes || !P.d_arena)) ? 1 : 0;
  if (k == "planes_bytes") return (int64_t)P.planes_bytes;
  // the planes GEMM's shape and partials workspace (host-side layout: no GPU needed)
  if (k == "planes_ws_bytes") return P.planes_gemm >= 0 ? (int64_t)(P.planes_sc_off - P.planes_ws_off) : 0;
  if (P.planes_gemm >= 0 && k.rfind("planes_gemm_", 0) == 0) {
    const tq::Op& g = P.ops[P.planes_gemm];
    if (k == "planes_gemm_M") return g.M;
    if (k == "planes_gemm_N") return g.N;
    if (k == "planes_gemm_K") return g.K;
    if (k == "planes_gemm_lda") return g.lda;
    if (k == "planes_gemm_ldb") return g.ldb;
  }
  if (k == "out_numel") return P.out_numel;
  return -1;
}

int tq_plan_describe(tq_plan p, char* buf, size_t n) {
  if (!p) return TQ_ERR_INVALID;
  const std::string& d = p->plan.describe;
  if (buf && n) {
    const size_t k = std::min(n - 1, d.size());
    std::memcpy(buf, d.data(), k);
    buf[k] = 0;
  }
  return (int)d.size();
}

int tq_plan_execute(tq_plan p, const void* const* inputs, void* out, int64_t slice_begin,
                    int64_t slice_end, int64_t slice_step, int accumulate, void* stream) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(p != nullptr, "null plan");
  if (!p->materialized) {  // device memory is taken at first use, so plans compile without a GPU
    TQ_TRY(tq::plan_materialize(p->plan, nullptr, nullptr, (hipStream_t)stream));
    p->materialized = true;
  }
  trace("execute", p, (int64_t)(intptr_t)stream);
  const int rc = tq::plan_run(p->plan, inputs, out, slice_begin, slice_end, slice_step, accumulate,
                              (hipStream_t)stream);
  trace("executed", p, rc);
  return rc;
  TQ_GUARD_END
}

int tq_plan_execute_group(int n, const tq_plan* plans, const void* const* const* inputs, void* const* outs,
                          int64_t slice_begin, int64_t slice_end, int64_t slice_step, int accumulate,
                          void* stream) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(n >= 1 && n <= 64 && plans && inputs && outs, "group of 1..64 plans");
  std::vector<tq::Plan*> ps((size_t)n);
  for (int k = 0; k < n; ++k) {
    TQ_CHECK_ARG(plans[k] != nullptr && inputs[k] != nullptr, "null plan / inputs in a group");
    if (!plans[k]->materialized) {
      TQ_TRY(tq::plan_materialize(plans[k]->plan, nullptr, nullptr, (hipStream_t)stream));
      plans[k]->materialized = true;
    }
    ps[k] = &plans[k]->plan;
  }
  trace("execute_group", plans[0], n);
  const int rc = tq::plan_run_group(ps.data(), n, inputs, outs, slice_begin, slice_end, slice_step, accumulate,
                                    (hipStream_t)stream);
  trace("executed_group", plans[0], rc);
  return rc;
  TQ_GUARD_END
}

int tq_plan_profile(tq_plan p, int enable) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(p != nullptr, "null plan");
  tq::Plan& P = p->plan;
  for (auto& ev : P.ev_used) P.ev_free.push_back(ev);  // reset: recycle recorded events
  P.ev_used.clear();
  P.profile = (unsigned)enable;
  return TQ_OK;
  TQ_GUARD_END
}

int tq_plan_profile_read(tq_plan p, int op_kind, double* total_ms, int64_t* launches,
                         double* flops, double* bytes) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(p != nullptr, "null plan");
  return tq::plan_profile_read(p->plan, op_kind, total_ms, launches, flops, bytes);
  TQ_GUARD_END
}

int tq_hermite_features(int dtype, int64_t n_points, int K, const double* x, const double* weights,
                        void* phi, void* mx, void* stream) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(tq::dtype_valid(dtype), "dtype");
  TQ_CHECK_ARG(K >= 1 && K <= TQ_HERMITE_MAX_K, "K must be in [1, TQ_HERMITE_MAX_K]");
  TQ_CHECK_ARG(n_points >= 0, "n_points < 0");
  TQ_CHECK_ARG(weights != nullptr, "null weights");
  TQ_CHECK_ARG(n_points == 0 || x != nullptr, "null x");
  TQ_CHECK_ARG(phi != nullptr || mx != nullptr, "neither phi nor mx requested");
  return tq::hermite_launch(dtype, n_points, K, x, weights, phi, mx, (hipStream_t)stream);
  TQ_GUARD_END
}

int tq_inverse_cdf_sample(int dtype, int64_t n_rows, int64_t grid_size, const void* density,
                          int64_t ld_density, const void* grid_x, const float* u, void* samples,
                          int64_t samples_stride, void* stream) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(dtype == TQ_F32 || dtype == TQ_F64, "density must be real (TQ_F32 / TQ_F64)");
  TQ_CHECK_ARG(grid_size >= 2 && grid_size <= TQ_ICDF_MAX_GRID,
               "grid_size must be in [2, TQ_ICDF_MAX_GRID]");
  TQ_CHECK_ARG(n_rows >= 0 && n_rows <= INT32_MAX, "n_rows out of range");
  TQ_CHECK_ARG(ld_density >= grid_size, "ld_density < grid_size");
  TQ_CHECK_ARG(n_rows == 0 || (density && grid_x && u && samples), "null pointer");
  return tq::icdf_launch(dtype, n_rows, grid_size, density, ld_density, grid_x, u, samples,
                         samples_stride, (hipStream_t)stream);
  TQ_GUARD_END
}

int tq_fidelity_forward(int dtype, int64_t n, const void* t, const void* o, double* stats, void* loss,
                        void* stream) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(n >= 0, "n");
  TQ_CHECK_ARG(t && o && stats && loss, "null pointer");
  return tq::fidelity_forward_launch(dtype, n, t, o, stats, loss, (hipStream_t)stream);
  TQ_GUARD_END
}

int tq_fidelity_backward(int dtype, int64_t n, const void* t, const void* o, const double* stats,
                         const void* g, void* grad_o, void* stream) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(n >= 0, "n");
  TQ_CHECK_ARG(t && o && stats && g && grad_o, "null pointer");
  return tq::fidelity_backward_launch(dtype, n, t, o, stats, g, grad_o, (hipStream_t)stream);
  TQ_GUARD_END
}

int tq_plan_destroy(tq_plan p) {
  if (!p) return TQ_OK;
  trace("destroy", p, (int64_t)p->plan.graphs.size());
  // a refused release (e.g. a stream capture in progress elsewhere in the process) keeps the
  // plan and what it still holds: the caller retries the destroy later (the Python host defers
  // it until no capture is in progress); nothing is leaked or released twice
  const int rc = tq::plan_release(p->plan);
  trace("released", p, rc);
  if (rc != TQ_OK) return rc;
  delete p;
  trace("deleted", p);
  return TQ_OK;
}

int tq_sgdg_step(int dtype, int n, void* const* params, void* const* grads, void* const* bufs,
                 const int32_t* rows, const int32_t* cols, const int32_t* flags, double lr,
                 double momentum, double dampening, double weight_decay, int nesterov,
                 void* stream) {
  TQ_GUARD_BEGIN
  TQ_CHECK_ARG(tq::dtype_valid(dtype), "dtype");
  TQ_CHECK_ARG(n >= 0, "n");
  if (n == 0) return TQ_OK;
  TQ_CHECK_ARG(params && grads && bufs && rows && cols && flags, "null argument");
  // every descriptor is checked before anything runs (no partly applied step)
  size_t ws_total = 0;
  for (int i = 0; i < n; ++i) {
    const bool stf = flags[i] & tq::kSgdgStiefel;
    TQ_CHECK_ARG(params[i] && grads[i] && rows[i] >= 1 && cols[i] >= 1, "bad parameter descriptor");
    TQ_CHECK_ARG(bufs[i] || !(stf || momentum != 0.0), "missing momentum buffer");
    if (stf && (rows[i] > cols[i] || cols[i] > tq::kSgdgMaxDimGlobal)) {
      tq::set_error("sgdg: Stiefel parameters need rows <= cols <= " + std::to_string(tq::kSgdgMaxDimGlobal));
      return TQ_ERR_UNSUPPORTED;
    }
    if (stf && cols[i] > tq::kSgdgMaxDim) ws_total += (tq::sgdg_ws_bytes(dtype, rows[i], cols[i]) + 255) / 256 * 256;
  }
  // large Stiefel parameters: one stream-ordered scratch for the call
  char* ws = nullptr;
  if (ws_total) TQ_HIP(hipMallocAsync((void**)&ws, ws_total, (hipStream_t)stream));
  size_t ws_at = 0;
  for (int b = 0; b < n; b += tq::kSgdgMaxBatch) {
    tq::SgdgLaunch L{};
    L.n = std::min(n - b, tq::kSgdgMaxBatch);
    L.nesterov = nesterov;
    L.lr = lr;
    L.momentum = momentum;
    L.dampening = dampening;
    L.weight_decay = weight_decay;
    for (int i = 0; i < L.n; ++i) {
      void* pw = nullptr;
      if ((flags[b + i] & tq::kSgdgStiefel) && cols[b + i] > tq::kSgdgMaxDim) {
        pw = ws + ws_at;
        ws_at += (tq::sgdg_ws_bytes(dtype, rows[b + i], cols[b + i]) + 255) / 256 * 256;
      }
      L.p[i] = tq::SgdgParam{params[b + i], grads[b + i], bufs[b + i], rows[b + i], cols[b + i],
                             flags[b + i], 0, pw};
    }
    const int rc = tq::sgdg_launch(dtype, L, (hipStream_t)stream);
    if (rc != TQ_OK) {
      if (ws) (void)hipFreeAsync(ws, (hipStream_t)stream);
      return rc;
    }
  }
  if (ws) TQ_HIP(hipFreeAsync(ws, (hipStream_t)stream));
  return TQ_OK;
  TQ_GUARD_END
}

}  // extern "C"
