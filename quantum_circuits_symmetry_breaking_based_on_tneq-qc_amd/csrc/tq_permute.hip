// Strided gather / permute to a contiguous destination, LDS-tiled for gfx950.
//
// Replaces the high-rank transpose that each opt_einsum pairwise step performs before its
// GEMM (reference: tensordot inside the ContractExpression built at
// tneq_qc/contractor/einsum_strategy.py:639-643; explicit permute(...).contiguous() at
// tneq_qc/distributed/engine/distributed_engine.py:1330,1635).
//
// Design (HBM-bound; 2 * numel * sizeof bytes algorithmic):
//  * Host fuses dims that are contiguous in both views, then picks a tile made of
//      O-dims: the innermost destination dims (product >= 64)  -> coalesced stores
//      I-dims: the smallest-stride source dims (product >= 64)  -> coalesced loads
//    (dims of extent 2 — qubit legs — are packed until a run is long enough).
//  * Every tile element has a tile-relative source offset, LDS slot and destination offset
//    that do not depend on the tile: the host tabulates them once; each thread loads ITS
//    entries into registers once and then streams many tiles (persistent grid ~8 blocks/CU),
//    so no per-element index arithmetic runs in the loop.
//  * LDS holds the tile in destination order with one pad element per 32 (bank spread).
//  * Anything the tile path cannot express (ragged tile dims, rank overflow) runs a generic
//    one-element-per-thread decode kernel.
#include <algorithm>
#include <numeric>

#include "tq_common.h"
#include "tq_permute.h"

namespace tq {

namespace {

constexpr int kThreads = 256;
constexpr int kMaxTile = 4096;

__host__ __device__ inline int lds_pad(int p) { return p + (p >> 5); }

template <typename T, typename Idx, int EPT>
__global__ void __launch_bounds__(kThreads)
permute_tiled_kernel(const T* __restrict__ src, T* __restrict__ dst, const Idx* __restrict__ tab,
                     int tile_elems, PermOuter outer, int64_t n_tiles, float beta_f, double beta_d,
                     int use_beta) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* lds = reinterpret_cast<T*>(smem_raw);
  const int tid = threadIdx.x;
  Idx lsrc[EPT], llds[EPT], sdst[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int e = tid + j * kThreads;
    if (e < tile_elems) {
      lsrc[j] = tab[e];
      llds[j] = tab[tile_elems + e];
      sdst[j] = tab[2 * tile_elems + e];
    } else {
      lsrc[j] = 0; llds[j] = 0; sdst[j] = 0;
    }
  }
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    int64_t rem = tile, sbase = 0, dbase = 0;
    for (int d = outer.n - 1; d >= 0; --d) {
      const int64_t c = rem % outer.cnt[d];
      rem /= outer.cnt[d];
      sbase += c * outer.sstride[d];
      dbase += c * outer.dstride[d];
    }
    T v[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j)
      if (tid + j * kThreads < tile_elems) v[j] = src[sbase + (int64_t)lsrc[j]];
#pragma unroll
    for (int j = 0; j < EPT; ++j)
      if (tid + j * kThreads < tile_elems) lds[llds[j]] = v[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = tid + j * kThreads;
      if (e < tile_elems) {
        T w = lds[lds_pad(e)];
        T* p = dst + dbase + (int64_t)sdst[j];
        if (use_beta) {
          if constexpr (sizeof(typename Traits<T>::R) == 4) w = w + (*p) * beta_f;
          else w = w + (*p) * beta_d;
        }
        *p = w;
      }
    }
    __syncthreads();
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
permute_generic_kernel(const T* __restrict__ src, T* __restrict__ dst, PermGeneric g,
                       int64_t numel, float beta_f, double beta_d, int use_beta) {
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < numel;
       i += (int64_t)gridDim.x * kThreads) {
    int64_t rem = i, so = 0;
    for (int d = g.rank - 1; d >= 0; --d) {
      const int64_t c = rem % g.ext[d];
      rem /= g.ext[d];
      so += c * g.sstride[d];
    }
    T w = src[so];
    if (use_beta) {
      if constexpr (sizeof(typename Traits<T>::R) == 4) w = w + dst[i] * beta_f;
      else w = w + dst[i] * beta_d;
    }
    dst[i] = w;
  }
}

// pick a tile extent for dim `ext` given the current tile product `p` and a cap.
// returns 0 if the dim cannot be tiled evenly (ragged) — caller then stops adding dims.
int64_t tile_extent(int64_t ext, int64_t p, int64_t cap) {
  if (p * ext <= cap) return ext;
  int64_t room = cap / p;
  for (int64_t t = room; t >= 2; --t)
    if (ext % t == 0) return t;
  return 0;
}

}  // namespace

int build_perm_plan(int dtype, int rank, const int64_t* shape, const int64_t* sstrides,
                    PermPlan* plan) {
  PermPlan& P = *plan;
  P = PermPlan{};
  P.dtype = dtype;
  // 1) drop extent-1 dims, check extents
  std::vector<int64_t> ext, ss;
  int64_t numel = 1;
  for (int d = 0; d < rank; ++d) {
    TQ_CHECK_ARG(shape[d] >= 0, "negative extent");
    numel *= shape[d];
    if (shape[d] != 1) { ext.push_back(shape[d]); ss.push_back(sstrides[d]); }
  }
  P.numel = numel;
  if (numel == 0) return TQ_OK;
  // 2) fuse dims contiguous in source too (destination is always contiguous)
  std::vector<int64_t> fe, fs;
  for (size_t d = 0; d < ext.size(); ++d) {
    if (!fe.empty() && fs.back() == ss[d] * ext[d]) {
      fe.back() *= ext[d];
      fs.back() = ss[d];
    } else {
      fe.push_back(ext[d]);
      fs.push_back(ss[d]);
    }
  }
  if (fe.empty()) { fe.push_back(1); fs.push_back(0); }  // single element
  const int r = (int)fe.size();
  std::vector<int64_t> ds(r);
  {
    int64_t s = 1;
    for (int d = r - 1; d >= 0; --d) { ds[d] = s; s *= fe[d]; }
  }
  // generic description (fallback)
  P.generic.rank = r;
  if (r > kPermMaxRank) {
    set_error("permute: rank after fusion exceeds " + std::to_string(kPermMaxRank));
    return TQ_ERR_UNSUPPORTED;
  }
  for (int d = 0; d < r; ++d) { P.generic.ext[d] = fe[d]; P.generic.sstride[d] = fs[d]; }

  // 3) choose tile dims
  std::vector<int64_t> te(r, 0);  // tile extent per dim (0 = not in tile)
  int64_t tprod = 1;
  bool ok = true;
  // O-dims: innermost destination dims
  for (int d = r - 1; d >= 0 && tprod < 64; --d) {
    const int64_t t = tile_extent(fe[d], tprod, 256);
    if (t == 0) break;
    te[d] = t;
    tprod *= t;
    if (t < fe[d]) break;  // a split dim ends the contiguous destination run
  }
  if (te[r - 1] == 0) ok = false;  // innermost destination dim cannot be tiled evenly
  // I-dims: smallest nonzero source stride first
  if (ok) {
    std::vector<int> order(r);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
      int64_t sa = fs[a] == 0 ? INT64_MAX : fs[a], sb = fs[b] == 0 ? INT64_MAX : fs[b];
      return sa < sb;
    });
    int64_t iprod = 1;
    for (int k = 0; k < r && iprod < 64; ++k) {
      const int d = order[k];
      if (fs[d] == 0) break;
      if (te[d] != 0) { iprod *= te[d]; if (te[d] < fe[d]) break; continue; }
      int64_t t = tile_extent(fe[d], tprod, kMaxTile);
      if (t == 0) break;
      te[d] = t; tprod *= t; iprod *= t;
      if (t < fe[d]) break;
    }
  }
  // 4) outer iteration space (blocks along tile dims + all other dims)
  int n_outer = 0;
  if (ok) {
    for (int d = 0; d < r; ++d) {
      const int64_t cnt = te[d] ? fe[d] / te[d] : fe[d];
      const int64_t step = te[d] ? te[d] : 1;
      if (cnt == 1) continue;
      if (n_outer >= kPermMaxRank) { ok = false; break; }
      P.outer.cnt[n_outer] = cnt;
      P.outer.sstride[n_outer] = fs[d] * step;
      P.outer.dstride[n_outer] = ds[d] * step;
      ++n_outer;
    }
    P.outer.n = n_outer;
  }
  if (!ok || tprod > kMaxTile) {
    P.use_generic = true;
    return TQ_OK;
  }
  // 5) tables: load order (smallest source stride fastest), store order (dst order)
  std::vector<int> tdims;  // tile dims in destination order
  for (int d = 0; d < r; ++d) if (te[d]) tdims.push_back(d);
  const int nt = (int)tdims.size();
  std::vector<int64_t> lds_stride(nt);
  {
    int64_t s = 1;
    for (int k = nt - 1; k >= 0; --k) { lds_stride[k] = s; s *= te[tdims[k]]; }
  }
  std::vector<int> lorder(nt);
  std::iota(lorder.begin(), lorder.end(), 0);
  std::stable_sort(lorder.begin(), lorder.end(), [&](int a, int b) {
    int64_t sa = fs[tdims[a]] == 0 ? INT64_MAX : fs[tdims[a]];
    int64_t sb = fs[tdims[b]] == 0 ? INT64_MAX : fs[tdims[b]];
    return sa < sb;
  });
  const int T = (int)tprod;
  P.tile_elems = T;
  P.tab.assign(3 * (size_t)T, 0);
  int64_t maxoff = 0;
  for (int e = 0; e < T; ++e) {
    // load element e: decode with lorder[0] fastest
    int64_t rem = e, soff = 0, lpos = 0;
    for (int q = 0; q < nt; ++q) {
      const int k = lorder[q];
      const int d = tdims[k];
      const int64_t c = rem % te[d];
      rem /= te[d];
      soff += c * fs[d];
      lpos += c * lds_stride[k];
    }
    P.tab[e] = soff;
    P.tab[T + e] = lds_pad((int)lpos);
    // store element e (destination order within tile)
    int64_t rem2 = e, doff = 0;
    for (int k = nt - 1; k >= 0; --k) {
      const int d = tdims[k];
      const int64_t c = rem2 % te[d];
      rem2 /= te[d];
      doff += c * ds[d];
    }
    P.tab[2 * T + e] = doff;
    maxoff = std::max(maxoff, std::max(soff, doff));
  }
  P.idx64 = maxoff >= (int64_t(1) << 31);
  P.n_tiles = numel / T;
  P.use_generic = false;
  return TQ_OK;
}

size_t perm_plan_table_bytes(const PermPlan& P) {
  if (P.use_generic || P.numel == 0) return 0;
  return P.tab.size() * (P.idx64 ? 8 : 4);
}

void perm_plan_pack_table(const PermPlan& P, void* host_buf) {
  if (P.idx64) {
    int64_t* o = (int64_t*)host_buf;
    for (size_t i = 0; i < P.tab.size(); ++i) o[i] = P.tab[i];
  } else {
    int32_t* o = (int32_t*)host_buf;
    for (size_t i = 0; i < P.tab.size(); ++i) o[i] = (int32_t)P.tab[i];
  }
}

namespace {
template <typename T, typename Idx>
int launch_tiled_t(const PermPlan& P, const void* dtab, const void* src, void* dst, double beta,
                   hipStream_t stream) {
  const int T_ = P.tile_elems;
  const size_t smem = (size_t)lds_pad(T_ - 1) + 1;
  const size_t smem_bytes = smem * sizeof(T);
  const int64_t grid64 = std::min<int64_t>(P.n_tiles, 2048);
  const int grid = (int)std::max<int64_t>(grid64, 1);
  const int ept = (T_ + kThreads - 1) / kThreads;
  const int use_beta = beta != 0.0;
#define TQ_PERM_CASE(E)                                                                      \
  if (ept <= E) {                                                                            \
    hipLaunchKernelGGL((permute_tiled_kernel<T, Idx, E>), dim3(grid), dim3(kThreads),        \
                       smem_bytes, stream, (const T*)src, (T*)dst, (const Idx*)dtab, T_,     \
                       P.outer, P.n_tiles, (float)beta, beta, use_beta);                     \
    TQ_HIP(hipGetLastError());                                                               \
    return TQ_OK;                                                                            \
  }
  TQ_PERM_CASE(1)
  TQ_PERM_CASE(2)
  TQ_PERM_CASE(4)
  TQ_PERM_CASE(8)
  TQ_PERM_CASE(16)
#undef TQ_PERM_CASE
  set_error("permute: tile too large");
  return TQ_ERR_UNSUPPORTED;
}

template <typename T>
int launch_generic_t(const PermPlan& P, const void* src, void* dst, double beta,
                     hipStream_t stream) {
  const int64_t blocks = std::min<int64_t>((P.numel + kThreads - 1) / kThreads, 8192);
  hipLaunchKernelGGL((permute_generic_kernel<T>), dim3((int)blocks), dim3(kThreads), 0, stream,
                     (const T*)src, (T*)dst, P.generic, P.numel, (float)beta, beta,
                     (int)(beta != 0.0));
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

template <typename T>
int launch_t(const PermPlan& P, const void* dtab, const void* src, void* dst, double beta,
             hipStream_t stream) {
  if (P.use_generic) return launch_generic_t<T>(P, src, dst, beta, stream);
  if (P.idx64) return launch_tiled_t<T, int64_t>(P, dtab, src, dst, beta, stream);
  return launch_tiled_t<T, int32_t>(P, dtab, src, dst, beta, stream);
}
}  // namespace

int perm_plan_launch(const PermPlan& P, const void* dtab, const void* src, void* dst, double beta,
                     hipStream_t stream) {
  if (P.numel == 0) return TQ_OK;
  switch (P.dtype) {
    case TQ_F32: return launch_t<float>(P, dtab, src, dst, beta, stream);
    case TQ_F64: return launch_t<double>(P, dtab, src, dst, beta, stream);
    case TQ_C64: return launch_t<c64>(P, dtab, src, dst, beta, stream);
    case TQ_C128: return launch_t<c128>(P, dtab, src, dst, beta, stream);
  }
  set_error("permute: bad dtype");
  return TQ_ERR_INVALID;
}

// One-shot permute (standalone C-ABI call): table uploaded with stream-ordered allocation.
int permute_launch(int dtype, int rank, const int64_t* shape, const int64_t* src_strides,
                   const void* src, void* dst, double beta, hipStream_t stream) {
  TQ_CHECK_ARG(dtype_valid(dtype), "dtype");
  TQ_CHECK_ARG(rank >= 0 && rank <= TQ_MAX_RANK, "rank");
  PermPlan P;
  TQ_TRY(build_perm_plan(dtype, rank, shape, src_strides, &P));
  const size_t tb = perm_plan_table_bytes(P);
  void* dtab = nullptr;
  if (tb) {
    std::vector<char> host(tb);
    perm_plan_pack_table(P, host.data());
    TQ_HIP(hipMallocAsync(&dtab, tb, stream));
    TQ_HIP(hipMemcpyAsync(dtab, host.data(), tb, hipMemcpyHostToDevice, stream));
    // pageable source: hipMemcpyAsync stages it before returning, so `host` may die here
    TQ_HIP(hipStreamSynchronize(stream));
  }
  int rc = perm_plan_launch(P, dtab, src, dst, beta, stream);
  if (dtab) (void)hipFreeAsync(dtab, stream);
  return rc;
}

}  // namespace tq
