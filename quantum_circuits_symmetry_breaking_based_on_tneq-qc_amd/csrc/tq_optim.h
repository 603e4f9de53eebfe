// One SGDG step over a group of parameters in one launch (tq_optim.hip).
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace tq {

constexpr int kSgdgStiefel = 1;   // Stiefel (Cayley) branch: rows <= cols and stiefel=True
constexpr int kSgdgBufInit = 2;   // momentum buffer already holds a previous value
constexpr int kSgdgRetract = 4;   // qr_retraction of the row-normalised parameter first
constexpr int kSgdgMaxDim = 32;   // rows <= cols <= 32: the Stiefel branch's matrices live in LDS
constexpr int kSgdgMaxDimGlobal = 2048;  // larger (cols <= 2048): the same math on a global scratch
constexpr int kSgdgMaxBatch = 48; // parameters per launch (the descriptors travel as kernel arguments)

struct SgdgParam {
  void* param;       // rows x cols, contiguous (the parameter viewed as in SGDG.step)
  void* grad;        // same shape; written back (weight decay) on the SGD branch
  void* buf;         // momentum buffer: cols x rows (Stiefel) or rows x cols (SGD)
  int rows, cols;
  int flags;
  int pad;
  void* ws;          // Stiefel with cols > kSgdgMaxDim: global scratch of sgdg_ws_bytes (else null)
};

struct SgdgLaunch {
  int n;
  int nesterov;
  double lr, momentum, dampening, weight_decay;
  SgdgParam p[kSgdgMaxBatch];
};

// one workgroup per parameter; n <= kSgdgMaxBatch.  Every descriptor is checked before anything
// is launched; Stiefel parameters with cols > kSgdgMaxDim need their `ws`.
int sgdg_launch(int dtype, const SgdgLaunch& L, hipStream_t stream);
// bytes of the Stiefel branch's matrices for a rows x cols parameter of dtype
size_t sgdg_ws_bytes(int dtype, int rows, int cols);

}  // namespace tq
