/*
 * tneqhip.h — C ABI of libtneqhip.so, the MI355X (gfx950) contraction engine that sits
 * under the tneq_qc backend / contractor plugin surface.
 *
 * Every entry point takes plain pointers and sizes (no torch types).  Device pointers are
 * caller-owned (e.g. torch.Tensor.data_ptr()); plans and their arenas are library-owned.
 * `stream` is a hipStream_t passed as void* (NULL = the default stream).
 * Return value: 0 = ok, < 0 = error (tq_last_error() has the message).  The Python host maps
 * TQ_ERR_INVALID to ValueError and everything else to RuntimeError, as the reference does
 * (SURVEY.md §8(b) "Conventions": qctn.py:826-831 ValueError, compiler.py:120-121 RuntimeError).
 *
 * Which reference interface each entry point replaces (all paths under /root/reference):
 *   tq_permute        — the strided transpose inside every pairwise step of
 *                       opt_einsum's ContractExpression (called at
 *                       tneq_qc/contractor/einsum_strategy.py:639-643 and
 *                       symmetry_breaking_quantum.py:142,154,213) and the explicit
 *                       permute(...).contiguous() at tneq_qc/distributed/engine/distributed_engine.py:1330,1635;
 *                       BackendPyTorch.permute tneq_qc/backends/backend_pytorch.py:619-621.
 *   tq_gemm_batched   — the GEMM / bmm under each tensordot (torch.tensordot -> at::mm) and the
 *                       partial bmm at distributed_engine.py:1477-1487.
 *   tq_contract_pair  — one pairwise tensordot with arbitrary output mode order
 *                       (opt_einsum pairwise step; BackendPyTorch.einsum backend_pytorch.py:623-625
 *                       for two operands; ComputeBackend.einsum backend_interface.py:495-507).
 *   tq_plan_*         — a whole ContractExpression: ComputeBackend.execute_expression
 *                       (backend_interface.py:102-114, backend_pytorch.py:99-105) over the
 *                       expression created by EinsumStrategy.create_contract_expression
 *                       (einsum_strategy.py:622-643), plus index slicing.
 *   tq_axpy           — the partial-amplitude accumulation before the slice reduce
 *                       (AllReduceGrad, tneq_qc/distributed/optim/allreduce_grad.py:13-60).
 *   tq_hermite_features — EngineSiamese.generate_data and its helpers _init_mx_weights /
 *                       _eval_hermitenorm_batch(_np) (tneq_qc/core/engine_siamese.py:59-254).
 *   tq_inverse_cdf_sample — the clamp / cumsum / normalise / search / interpolate block of
 *                       EngineSiamese.sample (tneq_qc/core/engine_siamese.py:854-905).
 *   tq_fidelity_forward / _backward — the symmetry-breaking fit's fidelity loss
 *                       (symmetry_breaking_quantum.py:220-229) and its gradient, one launch each.
 *   tq_sgdg_step       — SGDG.step, the Stiefel / Cayley optimizer of the symmetry-breaking
 *                       training loop (tneq_qc/optim/stiefel_optimizer_complex.py:77-176,
 *                       called at symmetry_breaking_quantum.py:216-230).
 */
#ifndef TNEQHIP_H
#define TNEQHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types; complex types are interleaved (re, im) like numpy / torch complex64/128 */
enum { TQ_F32 = 0, TQ_F64 = 1, TQ_C64 = 2, TQ_C128 = 3 };

enum {
  TQ_OK = 0,
  TQ_ERR_INVALID = -1,     /* bad shape / mode / argument  -> ValueError */
  TQ_ERR_HIP = -2,         /* HIP runtime error             -> RuntimeError */
  TQ_ERR_ALLOC = -3,       /* device allocation failed      -> RuntimeError (MemoryError) */
  TQ_ERR_UNSUPPORTED = -4  /* valid but not implemented     -> RuntimeError */
};

#define TQ_MAX_RANK 64

/* ---- library ---------------------------------------------------------------------- */
int tq_version(void);                      /* (major << 16) | minor */
int tq_last_error(char* buf, size_t n);    /* copies the last error of this thread; returns its length */
int tq_device_synchronize(void);
/* Library configuration: "gemm_bf16" (1: the K-outer complex64 GEMM runs on the 16-bit matrix
 * cores with f32 accuracy; env TQ_GEMM_BF16=0 selects the f32-MFMA kernel), "gemm_f16" (1, with
 * gemm_bf16: a 2-term f16 split of the power-of-two-scaled operands, 12 MFMAs per complex
 * tile-step; 0 / env TQ_GEMM_F16=0: an exact 3-term bf16 split, 24 MFMAs), "gemm_f16_var" (f16
 * tile variant: 6 (default) = 8 waves of 64x32 with Gauss's 3-multiplication product (9 MFMAs
 * per complex tile-step) and 3 staging sets, 5 = the same with 2 staging sets, 0 = the 64x32
 * tile with the 4-multiplication product, 1 = 4 waves of
 * 64x64, 2 = 4 waves of 64x64 with Gauss's product, 3 = variant 0 on a 4-slot LDS ring, one
 * barrier per two K-steps, 4 = variant 0 on v_mfma_f32_16x16x32_f16; env TQ_GEMM_F16_VAR),
 * "gemm_presplit" (0 by default, env TQ_GEMM_PRESPLIT=1, with gemm_f16_var 0: a plan's per-slice
 * sweep ops store the boundary GEMM's operands as f16 terms with a predicted scale, checked by
 * the GEMM; a slice outside the window is re-run on the split path -- the execute call then
 * synchronizes its stream), "presplit_bias" (testing: offset of the predicted scale), "gemm_3m" (1: the f32-MFMA complex64 kernel uses Gauss's 3-multiplication
 * product, env TQ_GEMM_3M=0 turns it off), "sweep" (fused multi-gate sweeps, env TQ_SWEEP),
 * "graphs" (plan execution through hipGraphs, env TQ_GRAPH).  -1 if unknown.  No reference
 * counterpart (the reference has no native layer); used for measurement reports. */
int64_t tq_library_query(const char* key);
/* Sets "gemm_bf16" / "gemm_f16" / "gemm_f16_var" / "gemm_3m" / "gemm_presplit" / "presplit_bias" at run time (launches issued afterwards; a plan replaying a
 * captured hipGraph keeps the kernels it captured).  TQ_ERR_INVALID for other keys.  No
 * reference counterpart; used by tests and A/B measurements. */
int tq_library_set(const char* key, int64_t value);

/* ---- kernels ----------------------------------------------------------------------- */

/* dst[c_0..c_{r-1}] = src[sum_d c_d * src_strides[d]] + beta * dst[...]
 * dst is contiguous in the order of `shape` (row-major, last dim fastest).
 * src_strides are in elements and may be 0 (broadcast) or describe any view (slice).  */
int tq_permute(int dtype, int rank, const int64_t* shape, const int64_t* src_strides,
               const void* src, void* dst, double beta, void* stream);

/* C_b = A_b * B_b + beta * C_b for b in [0, batch);  row-major operands:
 *   transA == 0: A_b is M x K with leading dim lda (K contiguous);  transA == 1: A_b is K x M (M contiguous)
 *   transB == 0: B_b is K x N with leading dim ldb (N contiguous);  transB == 1: B_b is N x K (K contiguous)
 *   C_b is M x N with leading dim ldc.
 * No conjugation.  `workspace` may be NULL (then no split-K is used).               */
int tq_gemm_batched(int dtype, int transA, int transB, int64_t M, int64_t N, int64_t K,
                    int64_t batch, const void* A, int64_t lda, int64_t strideA, const void* B,
                    int64_t ldb, int64_t strideB, double beta, void* C, int64_t ldc,
                    int64_t strideC, void* workspace, size_t ws_bytes, void* stream);
size_t tq_gemm_workspace_size(int dtype, int64_t M, int64_t N, int64_t K, int64_t batch);

/* The pre-split ("planes") boundary GEMM of a plan (tq_gemmp.hip; the C4g path): the f32 split-K
 * partials a launch of up to `batch` lane entries needs (the max over every batch size <= batch:
 * a partial lane batch may choose more K splits), and the launcher's argument checks without a
 * launch (TQ_OK, or TQ_ERR_INVALID when the shape is unsupported or the partials exceed
 * ws_bytes).  Host-only: CPU tests of the sizing.  Replaces nothing in the reference (a
 * workspace of this engine's GEMM behind einsum_strategy.py:622-643's tensordot). */
size_t tq_planes_gemm_workspace(int64_t M, int64_t N, int64_t K, int64_t batch);
int tq_planes_gemm_check(int64_t M, int64_t N, int64_t K, int64_t batch, int64_t lda, int64_t ldb,
                         size_t ws_bytes);

/* y = x + beta * y over n elements (used to sum partial amplitudes of slices) */
int tq_axpy(int dtype, int64_t n, const void* x, void* y, double beta, void* stream);

/* One pairwise tensordot with arbitrary output order (einsum "A,B->C" with integer modes).
 * A mode present in A and B but not C is summed; a mode present in A, B and C is a batch
 * mode; a mode present in only one operand and not in C is summed over that operand.
 * All tensors contiguous row-major.  Call tq_contract_pair_workspace() first.          */
size_t tq_contract_pair_workspace(int dtype, int rankA, const int64_t* shapeA,
                                  const int32_t* modesA, int rankB, const int64_t* shapeB,
                                  const int32_t* modesB, int rankC, const int32_t* modesC);
int tq_contract_pair(int dtype, int rankA, const int64_t* shapeA, const int32_t* modesA,
                     const void* A, int rankB, const int64_t* shapeB, const int32_t* modesB,
                     const void* B, int rankC, const int32_t* modesC, void* C,
                     void* workspace, size_t ws_bytes, void* stream);

/* ---- plans: a GPU-resident contraction tree with preallocated intermediates --------- */
typedef struct tq_plan_s* tq_plan;

/* Inputs: n_inputs tensors; tensor i has in_ranks[i] modes taken consecutively from
 * in_modes / in_extents / in_strides (strides in elements; pass NULL for contiguous).
 * path: n_steps pairs of SSA ids (inputs are 0..n_inputs-1, step s creates id n_inputs+s),
 * exactly opt_einsum's "ssa path".  The last step's result must hold exactly the out_modes.
 * sliced_modes: contracted modes that are fixed per slice; slice ids enumerate them in
 * row-major order of the given list.                                                    */
int tq_plan_create(tq_plan* plan, int dtype, int n_inputs, const int32_t* in_ranks,
                   const int32_t* in_modes, const int64_t* in_extents, const int64_t* in_strides,
                   int out_rank, const int32_t* out_modes, int n_steps, const int32_t* path,
                   int n_sliced, const int32_t* sliced_modes);

/* Queries (algorithmic counts): "n_slices", "arena_bytes", "table_bytes", "out_numel",
 * "flops" / "bytes_moved" (a whole execute over all slices), "flops_once" / "bytes_once"
 * (slice-invariant part, hoisted: run once per execute), "flops_slice" / "bytes_slice"
 * (per slice), "n_kernels", "n_ops_once", "n_gemm", "n_apply", "n_permute", "lanes" (slices
 * per batch: lane copies of the per-slice arena part within a 6-GiB budget, env TQ_SLICE_LANES /
 * TQ_LANE_ARENA_MB), "n_presplit" (pre-split GEMM candidates), "presplit_fallbacks" (slices
 * re-run on the split path so far).  -1 if unknown. */
int64_t tq_plan_query(tq_plan plan, const char* key);
/* A copy of a compiled plan (same schedule, no device state: its own arena and tables at its
 * first execute) -- one per stream / block in flight without compiling the network again. */
int tq_plan_clone(tq_plan src, tq_plan* out);

/* Plan options: "graph" = 1 (default) replays the execute's launches from a captured hipGraph,
 * 0 launches them eagerly on the stream (use when the caller captures the stream itself);
 * "sweep_chain" = 1 (default, env TQ_S2_SEQ) runs consecutive hoisted levels that are each one
 * small sweep2 op as one launch of one workgroup (query "n_chain_launches"), 0 one launch per
 * level; "gemm_planes" = 1 (default, env TQ_GEMM_PLANES) runs the plan's boundary GEMM on operands
 * its dense producers store pre-split as six f16 term planes (query "planes_gemm": planned,
 * "planes_active", "planes_bytes": the extra device memory), 0 on the GEMM-side split kernel;
 * "sweep_coop" = 0 (default, env TQ_S2_COOP) -- 1 runs consecutive hoisted levels of
 * multi-chunk sweep2 ops as one launch whose workgroups hand off through a counter barrier
 * (diagnostic: measured slower).  Its workgroups must be co-resident: a wait that gives up
 * (bounded spin) makes tq_plan_execute synchronize-check and fail with TQ_ERR_HIP ("the result
 * is invalid") instead of returning the stale result; inside a caller's capture the check is
 * skipped (query "coop_timeouts" then reports the count).  Before the first execute only
 * (the plan is compiled again): "group_hint" = G compiles for lockstep groups of G plans
 * (tq_plan_execute_group: every sweep op shares its launches, so ops take G x fewer, wider
 * chunks); "min_chunks" = n > 0 splits every big sweep op into at least n chunks (default 128,
 * env TQ_S2_MINCHUNKS; a caller with several plans in flight on other streams wants fewer). */
int tq_plan_set(tq_plan plan, const char* key, int64_t value);
/* human-readable per-step description into buf (for debugging / DESIGN evidence) */
int tq_plan_describe(tq_plan plan, char* buf, size_t n);

/* Runs slices slice_begin, slice_begin + slice_step, ... < slice_end and sums them into out
 * (out = sum + (accumulate ? out : 0)).  inputs[i] are device pointers of the FULL inputs.  */
int tq_plan_execute(tq_plan plan, const void* const* inputs, void* out, int64_t slice_begin,
                    int64_t slice_end, int64_t slice_step, int accumulate, void* stream);

/* Blocks as lanes: run n plans compiled from the SAME network (same equation, shapes, path,
 * slicing, dtype, strides; distinct plans, e.g. one per amplitude block of a sampler) in lockstep
 * on one stream, each on its own inputs[k] (n_inputs pointers) into its own outs[k], over the same
 * slice range.  Every sweep level / chain launch of all members is ONE kernel launch (their op
 * lists concatenated); the remaining ops run per member.  Results equal n tq_plan_execute calls.
 * Replaces: n concurrent executions of the reference's ContractExpression
 * (einsum_strategy.py:622-643) for n bitstring batches (SURVEY.md §8(e) "shard bitstrings").
 * Refused (TQ_ERR_INVALID): mismatched plans, repeated plans or outputs, cooperative-chain plans. */
int tq_plan_execute_group(int n, const tq_plan* plans, const void* const* const* inputs, void* const* outs,
                          int64_t slice_begin, int64_t slice_end, int64_t slice_step, int accumulate,
                          void* stream);
/* Releases the plan's graphs, events, streams and device memory.  TQ_ERR_HIP when HIP refuses a
 * release (e.g. hipGraphExecDestroy / hipFree while a stream capture is in progress in this
 * process): the plan stays valid with whatever it still holds, and a later tq_plan_destroy
 * retries; nothing is released twice.  */
int tq_plan_destroy(tq_plan plan);

/* Per-op timing with HIP events recorded on the execution stream around every kernel of the
 * plan (bench evidence for the roofline of the dominant kernel).  tq_plan_profile(plan, mask)
 * resets the records and times the op kinds whose bit (1 << kind) is set in mask (-1 = all,
 * 0 = off).  tq_plan_profile_read sums, over the launches of one
 * op kind since the reset (TQ_OP_PERMUTE / TQ_OP_GEMM / TQ_OP_APPLY, or -1 for all), the
 * elapsed milliseconds, the launch count and the algorithmic flops / bytes. */
enum { TQ_OP_PERMUTE = 0, TQ_OP_GEMM = 1, TQ_OP_APPLY = 2, TQ_OP_AXPY = 3, TQ_OP_SWEEP = 4 };
int tq_plan_profile(tq_plan plan, int enable);
int tq_plan_profile_read(tq_plan plan, int op_kind, double* total_ms, int64_t* launches,
                         double* flops, double* bytes);

/* ---- measurement data (EngineSiamese) ---------------------------------------------- */
#define TQ_HERMITE_MAX_K 128
#define TQ_ICDF_MAX_GRID 8192

/* Hermite measurement data of n_points scalar inputs x (float64, device):
 *   phi[p][k]   = (w_k * sqrt(exp(-x_p^2 / 2))) * He_k(x_p)   (k < K; probabilists' Hermite)
 *   mx[p][k][l] = conj(phi[p][k]) * phi[p][l]
 * weights: HOST array of K float64 w_k, copied into the launch arguments.  1 <= K <=
 * TQ_HERMITE_MAX_K.  A complex dtype computes in float64 and rounds once
 * (engine_siamese.py:165-207); a real dtype computes in its own precision (:212-254).
 * phi ([n_points][K]) or mx ([n_points][K][K]) may be NULL.                              */
int tq_hermite_features(int dtype, int64_t n_points, int K, const double* x, const double* weights,
                        void* phi, void* mx, void* stream);

/* One inverse-CDF draw per row of a real density (dtype TQ_F32 / TQ_F64; row s at
 * density + s * ld_density) on grid_x (grid_size points, 2 <= grid_size <= TQ_ICDF_MAX_GRID):
 * clamp at 0, inclusive prefix sum, normalise by (total + 1e-10), idx = min(#(cdf < u[s]),
 * grid_size - 2), linear interpolation between grid points idx and idx + 1 into
 * samples[s * samples_stride].  u: n_rows float32 uniforms (device).                       */
int tq_inverse_cdf_sample(int dtype, int64_t n_rows, int64_t grid_size, const void* density,
                          int64_t ld_density, const void* grid_x, const float* u, void* samples,
                          int64_t samples_stride, void* stream);

/* Fidelity loss of the symmetry-breaking fit (symmetry_breaking_quantum.py:220-229, the loss of
 * every pruning candidate; validate_target_tensor :159-166), over n complex elements (dtype
 * TQ_C64 / TQ_C128, t = target, o = the contraction's output, both device):
 *   a = <t, o> = sum conj(t_i) o_i, T = <t, t>, N = <o, o>, L = 1 - |a|^2 / max(T N, 1e-12)
 * forward: stats (device, 4 float64) = Re a, Im a, T, N; loss (device, one real of the dtype's
 * precision) = L; float64 accumulation, one workgroup.
 * backward: grad_o (device, n complex) = g * 2 dL/d(conj o) (torch's gradient of a real loss
 * w.r.t. a complex tensor), g = device pointer to the upstream gradient of L (one real):
 *   grad_o_i = 2 g (-a t_i / D + |a|^2 T o_i / D^2), D = max(T N, 1e-12), the second term only
 *   when T N >= 1e-12 (the clamp passes no gradient).                                        */
int tq_fidelity_forward(int dtype, int64_t n, const void* t, const void* o, double* stats, void* loss,
                        void* stream);
int tq_fidelity_backward(int dtype, int64_t n, const void* t, const void* o, const double* stats,
                         const void* g, void* grad_o, void* stream);

/* One SGDG optimizer step (tneq_qc/optim/stiefel_optimizer_complex.py:77-176, SGDG.step, with
 * gutils.py unit / qr_retraction / matrix_norm_one) for n parameters of one group, one workgroup
 * per parameter.  Parameter i is a rows[i] x cols[i] contiguous matrix (the parameter reshaped
 * to (prod of its leading half dims) x (rest), as SGDG.step views it) with a gradient of the
 * same shape and a momentum buffer.  flags[i]: TQ_SGDG_STIEFEL selects the Cayley branch (needs
 * rows <= cols <= TQ_SGDG_MAX_COLS; buffer cols x rows; matrices in LDS up to cols 32, on a
 * stream-ordered global scratch above), otherwise the SGD branch with weight decay /
 * momentum / dampening / nesterov (buffer rows x cols; the gradient is updated in place by
 * the weight decay, as d_p.add_ does); TQ_SGDG_BUF_INIT = the buffer holds the previous
 * momentum (else it is initialised as the reference does: zeros / a copy of d_p);
 * TQ_SGDG_RETRACT = qr_retraction of the row-normalised parameter first (the reference draws
 * this with random.randint(1, 101) == 1 on the host).  Arithmetic in the parameter's precision.
 * Every descriptor is checked before any parameter is touched: TQ_ERR_UNSUPPORTED (a Stiefel
 * parameter outside the limits) leaves the whole group unchanged. */
enum { TQ_SGDG_STIEFEL = 1, TQ_SGDG_BUF_INIT = 2, TQ_SGDG_RETRACT = 4, TQ_SGDG_MAX_COLS = 2048 };
int tq_sgdg_step(int dtype, int n, void* const* params, void* const* grads, void* const* bufs,
                 const int32_t* rows, const int32_t* cols, const int32_t* flags, double lr,
                 double momentum, double dampening, double weight_decay, int nesterov,
                 void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TNEQHIP_H */
