// Contraction-plan compiler and executor (host C++ over the HIP kernels).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "tq_common.h"
#include "tq_permute.h"

namespace tq {

// where an operand lives
enum BufKind { BUF_INPUT = 0, BUF_ARENA = 1, BUF_OUTPUT = 2, BUF_TABLE = 3 };
struct BufRef {
  int kind = BUF_ARENA;
  int64_t index = 0;  // input id for BUF_INPUT
  int64_t off = 0;    // element offset (bytes for BUF_TABLE)
};

enum OpKind { OP_PERMUTE = 0, OP_GEMM = 1, OP_APPLY = 2, OP_AXPY = 3 };

struct Op {
  int kind = OP_PERMUTE;
  BufRef a, b, c;       // permute: a -> c ; gemm: c = a*b ; apply: c = a (x) b ; axpy: c += a
  bool writes_output = false;
  // permute
  int perm = -1;        // index into Plan::perms
  // gemm
  int transA = 0, transB = 0;
  int64_t M = 0, N = 0, K = 0, batch = 1, lda = 0, ldb = 0, ldc = 0, sA = 0, sB = 0, sC = 0;
  BufRef ws;
  size_t ws_bytes = 0;
  // apply
  int64_t O = 0, I = 0;  // with K, N above
  // axpy
  int64_t n = 0;
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

struct Plan {
  int dtype = TQ_C64;
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
  size_t table_bytes = 0;
  size_t arena_bytes = 0;
  void* d_arena = nullptr;
  void* d_tables = nullptr;
  bool owns_device = false;
  double flops = 0, bytes = 0;
  int n_gemm = 0, n_apply = 0, n_permute = 0;
  std::string describe;
};

int plan_compile(Plan& P, int dtype, int n_inputs, const int32_t* in_ranks, const int32_t* in_modes,
                 const int64_t* in_extents, const int64_t* in_strides, int out_rank,
                 const int32_t* out_modes, int n_steps, const int32_t* path, int n_sliced,
                 const int32_t* sliced_modes);
// upload tables / allocate arena (owned) — or use caller memory when `arena`/`tables` are given
int plan_materialize(Plan& P, void* arena, void* tables, hipStream_t stream);
int plan_run(Plan& P, const void* const* inputs, void* out, int64_t s_begin, int64_t s_end,
             int64_t s_step, int accumulate, hipStream_t stream);
void plan_release(Plan& P);

}  // namespace tq
