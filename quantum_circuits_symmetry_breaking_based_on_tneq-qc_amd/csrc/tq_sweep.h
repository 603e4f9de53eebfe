// Fused multi-gate sweep op (tq_sweep.hip): argument block shared by the plan compiler and the
// kernel.  Limits: working set <= kSweepWMax elements, <= kSweepMaxGates gates per chain,
// K*N <= kSweepMaxKN per gate, <= kSweepMaxRuns runs of outer modes.
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace tq {

constexpr int kSweepWMax = 64;        // working-set elements (32 for complex128)
inline int sweep_wmax(int dtype_bytes) { return dtype_bytes > 8 ? 32 : 64; }
constexpr int kSweepMaxGates = 8;
constexpr int kSweepMaxKN = 64;
constexpr int kSweepMaxRuns = 8;
constexpr int kSweepTabMax = 2048;   // int16 entries of all gate tables of one op (LDS)

struct SweepArgs {
  const void* X = nullptr;  // chain input (contiguous)
  void* Y = nullptr;        // chain output (contiguous)
  int64_t ncols = 0;        // number of outer-mode assignments
  int nruns = 0;            // outer runs, innermost first: extent, stride in X, stride in Y
  int run_shift[kSweepMaxRuns] = {};   // log2(extent) or -1
  int64_t run_ext[kSweepMaxRuns] = {};
  int64_t run_in[kSweepMaxRuns] = {};
  int64_t run_out[kSweepMaxRuns] = {};
  int tin = 0, tout = 0;    // tile sizes (elements) in X / Y
  int tin_shift = -1, tout_shift = -1;  // log2 or -1
  const int64_t* tin_off = nullptr;   // device: element offset of each input-tile element in X
  const int64_t* tout_off = nullptr;  // device: element offset of each output-tile element in Y
  int ngates = 0;
  const void* G[kSweepMaxGates] = {};
  const int32_t* gidx[kSweepMaxGates] = {};  // gather table of G[k*N+n] (null: contiguous)
  int K[kSweepMaxGates] = {}, N[kSweepMaxGates] = {}, W[kSweepMaxGates] = {};
  const int32_t* tabs = nullptr;             // device: all gate tables, packed
  int tab_at[kSweepMaxGates] = {};           // entry offset of gate j's [W][K+1] table
  int tab_len = 0;                           // total int16 entries (<= kSweepTabMax)
  int load_colfast = 1, store_colfast = 1;
  // column offsets when every outer extent is a power of two: the offset is linear in the bits
  // of the column index, off(c) = sum_b bit_b(c) * w[b] (bits 0..5 -> lane part, the rest ->
  // chunk part); colbits < 0 selects the generic run decomposition
  int colbits = -1;
  int64_t w_in[48] = {}, w_out[48] = {};
  int use_beta = 0;
  double beta = 0.0;
};

// the slice lanes of one per-slice op in ONE launch (grid.y = lane): lane j reads X[j] and the
// gate tensors G[j][*] and writes Y[j]; every other field (tables, tile, column weights) is the
// SweepArgs' own, shared by the lanes (the same op on each lane's copy of the arena)
constexpr int kSweepMaxLanes = 32;
constexpr int kSweepFanKN = 16;
struct SweepLanes {
  int n = 0;
  // fan-out (set by sweep_launch_lanes when every lane reads the SAME X -- a slice-invariant input
  // of a per-slice op -- and every gate has K*N <= kSweepFanKN): X's chunk is loaded once and every
  // lane's gates run on it in turn (the per-lane grid re-read X once per lane)
  int fan = 0;
  const void* X[kSweepMaxLanes] = {};
  void* Y[kSweepMaxLanes] = {};
  const void* G[kSweepMaxLanes][kSweepMaxGates] = {};
};

int sweep_launch(int dtype, const SweepArgs& a, hipStream_t stream);
int sweep_launch_lanes(int dtype, const SweepArgs& a, const SweepLanes& l, hipStream_t stream);

}  // namespace tq
