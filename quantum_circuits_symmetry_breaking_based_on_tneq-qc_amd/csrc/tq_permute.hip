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
#include <map>
#include <mutex>
#include <numeric>

#include "tq_common.h"
#include "tq_permute.h"

namespace tq {

namespace {

constexpr int kThreads = 256;
constexpr int kMaxTile = 4096;

__host__ __device__ inline int lds_pad(int p) { return p + (p >> 5); }

// LDS slot of destination-order tile position p (see PermSwz)
__host__ __device__ inline int lds_slot(const PermSwz& z, int p) {
  if (z.mode == 0) return lds_pad(p);
  if (z.mode == 2) return p;
  int x = p;
  for (int q = 0; q < 16; ++q)
    if ((p >> q) & 1) x ^= z.vsw[q];
  return x;
}

// tile -> (source base, destination base): mixed-radix decode of the tile index over the outer
// dims (shifts when every count is a power of two — binary qubit legs)
__device__ __forceinline__ void tile_bases(const PermOuter& outer, int64_t tile, int64_t& sb,
                                           int64_t& db) {
  int64_t rem = tile;
  sb = 0;
  db = 0;
  if (outer.all_pow2) {
    for (int d = outer.n - 1; d >= 0; --d) {
      const int64_t c = rem & ((int64_t(1) << outer.lg[d]) - 1);
      rem >>= outer.lg[d];
      sb += c * outer.sstride[d];
      db += c * outer.dstride[d];
    }
  } else {
    for (int d = outer.n - 1; d >= 0; --d) {
      const int64_t c = rem % outer.cnt[d];
      rem /= outer.cnt[d];
      sb += c * outer.sstride[d];
      db += c * outer.dstride[d];
    }
  }
}

template <typename T>
__device__ __forceinline__ T add_scaled(T w, T y, float bf, double bd) {
  if constexpr (sizeof(typename Traits<T>::R) == 4) return w + y * bf;
  else return w + y * bd;
}

// VEC naturally aligned elements moved by one lane access (16 B for VEC * sizeof(T) == 16).
// Global and LDS traffic goes through native 4/8/16-byte vector types so that one lane access is
// one instruction (a struct of two doubles otherwise ends up split or spilled).
template <typename T, int VEC>
struct alignas(VEC * sizeof(T)) Vec { T v[VEC]; };
template <int B> struct RawT;
template <> struct RawT<4> { using t = unsigned int; };
template <> struct RawT<8> { using t = unsigned int __attribute__((ext_vector_type(2))); };
template <> struct RawT<16> { using t = unsigned int __attribute__((ext_vector_type(4))); };
template <typename V>
__device__ __forceinline__ V vload(const void* p) {
  using R = typename RawT<sizeof(V)>::t;
  const R r = *reinterpret_cast<const R*>(p);
  V v;
  __builtin_memcpy(&v, &r, sizeof(V));
  return v;
}
template <typename V>
__device__ __forceinline__ void vstore(void* p, const V& v) {
  using R = typename RawT<sizeof(V)>::t;
  R r;
  __builtin_memcpy(&r, &v, sizeof(V));
  *reinterpret_cast<R*>(p) = r;
}
template <typename T>
__device__ __forceinline__ void sstore(T* p, const T& v) { vstore<T>(p, v); }

// Persistent tile loop.  Lane access g of a tile: load VEC source-adjacent elements (one global
// load), scatter them to their destination-order LDS slots (VEC ds_writes), then — after the
// barrier — read VEC destination-adjacent elements (one ds_read) and store them (one global
// store).  All offsets come from per-thread registers filled once from the host tables; the next
// tile's loads are issued before the current tile's stores, so every workgroup keeps one tile of
// loads in flight behind its stores.
template <typename T, typename Idx, int EPT, int VEC>
__global__ void __launch_bounds__(kThreads)
permute_tiled_kernel(const T* __restrict__ src, T* __restrict__ dst, const Idx* __restrict__ tab,
                     int groups, PermOuter outer, PermSwz swz, int64_t n_tiles, int64_t tile_mul,
                     float beta_f, double beta_d, int use_beta) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* lds = reinterpret_cast<T*>(smem_raw);
  using V = Vec<T, VEC>;
  const int tid = threadIdx.x;
  Idx ls[EPT], sd[EPT];
  int l0[EPT], rd[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int g = tid + j * kThreads;
    const bool in = g < groups;
    ls[j] = in ? tab[g] : 0;
    l0[j] = in ? (int)tab[groups + g] : 0;
    sd[j] = in ? tab[2 * groups + g] : 0;
    rd[j] = in ? lds_slot(swz, VEC * g) : 0;
  }
  // tile visiting order: t -> (t * tile_mul) mod n_tiles (odd tile_mul, n_tiles a power of two),
  // so the tiles in flight at once spread over the whole tensor instead of one stride family
  const int64_t tmask = tile_mul == 1 ? int64_t(-1) : n_tiles - 1;
  int64_t tile = blockIdx.x;
  if (tile >= n_tiles) return;
  int64_t sb, db;
  tile_bases(outer, (tile * tile_mul) & tmask, sb, db);
  V v[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j)
    if (tid + j * kThreads < groups) v[j] = vload<V>(src + sb + (int64_t)ls[j]);
  for (; tile < n_tiles; tile += gridDim.x) {
#pragma unroll
    for (int j = 0; j < EPT; ++j)
      if (tid + j * kThreads < groups) {
#pragma unroll
        for (int b = 0; b < VEC; ++b) {
          const int s = swz.mode == 1 ? (l0[j] ^ swz.vdelta[b]) : (l0[j] + swz.vdelta[b]);
          sstore(lds + s, v[j].v[b]);
        }
      }
    __syncthreads();
    const int64_t cur_db = db;
    if (tile + gridDim.x < n_tiles) {
      tile_bases(outer, ((tile + gridDim.x) * tile_mul) & tmask, sb, db);
#pragma unroll
      for (int j = 0; j < EPT; ++j)
        if (tid + j * kThreads < groups)
          v[j] = vload<V>(src + sb + (int64_t)ls[j]);
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      if (tid + j * kThreads < groups) {
        V w = vload<V>(lds + rd[j]);
        T* p = dst + cur_db + (int64_t)sd[j];
        if (use_beta) {
          const V y = vload<V>(p);
#pragma unroll
          for (int b = 0; b < VEC; ++b) w.v[b] = add_scaled(w.v[b], y.v[b], beta_f, beta_d);
        }
        vstore<V>(p, w);
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

// LDS addressing for one kernel configuration.  pow2: every tile extent is a power of two, so
// the load index -> destination position map is a bit permutation pi (dpos of single-bit indices)
// and an XOR swizzle can spread the ds_write groups: a group of 128 / esz consecutive lanes (the
// ds_write_b32 / b64 / b128 banking groups) covers load bits lv .. lv+bw-1; lanes whose load bit
// lands on a position bit q >= bw get vsw[q] = a not-yet-covered low bit in [lv, bw).
PermSwz make_swizzle(bool pow2, int esz, int vec, const std::vector<int64_t>& dpos,
                     int64_t inner_pos_stride) {
  PermSwz z{};
  const int T = (int)dpos.size();
  if (!pow2) {
    z.mode = vec == 1 ? 0 : 2;
    for (int b = 0; b < vec; ++b) z.vdelta[b] = (int)(b * inner_pos_stride);
    return z;
  }
  z.mode = 1;
  int t = 0;
  while ((1 << t) < T) ++t;
  int bw = 0;
  while ((1 << bw) < 128 / esz) ++bw;
  int lv = 0;
  while ((1 << lv) < vec) ++lv;
  std::vector<int> pi(t);
  for (int i = 0; i < t; ++i) {
    int q = 0;
    while ((int64_t(1) << q) < dpos[(size_t)1 << i]) ++q;
    pi[i] = q;
  }
  std::vector<bool> covered(bw + 1, false);
  for (int i = 0; i < bw && lv + i < t; ++i)
    if (pi[lv + i] < bw) covered[pi[lv + i]] = true;
  int next = lv;
  for (int i = 0; i < bw && lv + i < t; ++i) {
    const int q = pi[lv + i];
    if (q < bw || q >= 16) continue;
    while (next < bw && covered[next]) ++next;
    if (next >= bw) break;
    z.vsw[q] = 1 << next;
    covered[next] = true;
  }
  for (int b = 0; b < vec; ++b) z.vdelta[b] = lds_slot(z, (int)dpos[b]);
  return z;
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

  // 3) choose tile dims (tiles of at most 32 KiB of LDS: 4096 elements of <= 8 bytes, 2048 of
  // 16 bytes, so that 4-5 workgroups share a CU)
  const int64_t max_tile = dtype_size(dtype) > 8 ? kMaxTile / 2 : kMaxTile;
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
    // ... and keep adding source dims (longer source runs) until the tile holds max_tile
    // elements: a small tile (e.g. 512 elements when the O- and I-dims overlap) leaves too few
    // bytes in flight per workgroup and pays the per-tile barriers and decode on 4 KB
    int64_t iprod = 1;
    for (int k = 0; k < r && (iprod < 64 || tprod < max_tile); ++k) {
      const int d = order[k];
      if (fs[d] == 0) break;
      if (te[d] != 0) { iprod *= te[d]; if (te[d] < fe[d]) break; continue; }
      int64_t t = tile_extent(fe[d], tprod, max_tile);
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
    P.outer.all_pow2 = 1;
    for (int d = 0; d < n_outer; ++d) {
      const int64_t c = P.outer.cnt[d];
      if (c & (c - 1)) { P.outer.all_pow2 = 0; P.outer.lg[d] = -1; continue; }
      int l = 0;
      while ((int64_t(1) << l) < c) ++l;
      P.outer.lg[d] = l;
    }
  }
  if (!ok || tprod > max_tile) {
    P.use_generic = true;
    return TQ_OK;
  }
  // 5) per-element maps: load element e (smallest source stride fastest) -> source offset and
  //    destination-order tile position; destination position p -> destination offset
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
  std::vector<int64_t> soff(T), dpos(T), doff(T);
  int64_t maxoff = 0;
  for (int e = 0; e < T; ++e) {
    int64_t rem = e, so = 0, lp = 0;
    for (int q = 0; q < nt; ++q) {
      const int k = lorder[q];
      const int d = tdims[k];
      const int64_t c = rem % te[d];
      rem /= te[d];
      so += c * fs[d];
      lp += c * lds_stride[k];
    }
    soff[e] = so;
    dpos[e] = lp;
    int64_t rem2 = e, dof = 0;
    for (int k = nt - 1; k >= 0; --k) {
      const int d = tdims[k];
      const int64_t c = rem2 % te[d];
      rem2 /= te[d];
      dof += c * ds[d];
    }
    doff[e] = dof;
    maxoff = std::max(maxoff, std::max(so, dof));
  }
  const bool pow2 = (T & (T - 1)) == 0 && [&] {
    for (int k = 0; k < nt; ++k)
      if (te[tdims[k]] & (te[tdims[k]] - 1)) return false;
    return true;
  }();
  const int esz = (int)dtype_size(dtype);
  // 6) scalar configuration
  P.swz1 = make_swizzle(pow2, esz, 1, dpos, lds_stride[lorder[0]]);
  P.tab.assign(3 * (size_t)T, 0);
  for (int e = 0; e < T; ++e) {
    P.tab[e] = soff[e];
    P.tab[T + e] = lds_slot(P.swz1, (int)dpos[e]);
    P.tab[2 * T + e] = doff[e];
  }
  // 7) vector configuration: VEC source-adjacent elements per load, VEC destination-adjacent per
  //    store (16-B lane accesses), verified element by element against the scalar maps
  for (int vec = std::min(4, 16 / esz); vec >= 2 && !getenv("TQ_PERM_NOVEC"); vec /= 2) {
    if (T % vec) continue;
    bool ok_v = true;
    for (int d = 0; d < n_outer && ok_v; ++d)
      ok_v = P.outer.sstride[d] % vec == 0 && P.outer.dstride[d] % vec == 0;
    for (int g = 0; g < T / vec && ok_v; ++g)
      ok_v = soff[vec * g] % vec == 0 && doff[vec * g] % vec == 0;
    for (int e = 0; e < T && ok_v; ++e)
      ok_v = soff[e] == soff[e - e % vec] + e % vec && doff[e] == doff[e - e % vec] + e % vec;
    if (!ok_v) continue;
    PermSwz z = make_swizzle(pow2, esz, vec, dpos, lds_stride[lorder[0]]);
    for (int e = 0; e < T && ok_v; ++e) {
      const int s0 = lds_slot(z, (int)dpos[e - e % vec]);
      const int b = e % vec;
      const int want = z.mode == 1 ? (s0 ^ z.vdelta[b]) : (s0 + z.vdelta[b]);
      ok_v = lds_slot(z, (int)dpos[e]) == want && lds_slot(z, e) == lds_slot(z, e - b) + b;
    }
    if (!ok_v) continue;
    const int G = T / vec;
    P.tab.resize(3 * (size_t)T + 3 * (size_t)G);
    int64_t* t2 = P.tab.data() + 3 * (size_t)T;
    for (int g = 0; g < G; ++g) {
      t2[g] = soff[vec * g];
      t2[G + g] = lds_slot(z, (int)dpos[vec * g]);
      t2[2 * G + g] = doff[vec * g];
    }
    P.swzv = z;
    P.vec = vec;
    break;
  }
  P.idx64 = maxoff >= (int64_t(1) << 31);
  P.n_tiles = numel / T;
  P.tile_mul = 1;
  if ((P.n_tiles & (P.n_tiles - 1)) == 0 && P.n_tiles > 1) {
    const char* e = getenv("TQ_PERM_TILEMUL");
    P.tile_mul = e ? (atoll(e) | 1) : 1;
  }
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
// Persistent grid: exactly the workgroups that are resident at once (occupancy x CUs, as the
// tile's LDS allows), tiles spread evenly over them — a grid larger than what is resident runs
// in rounds whose last one leaves most CUs idle.
int resident_grid(const void* kernel, size_t smem, int64_t n_tiles) {
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> cache;
  int per_grid = 0;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({kernel, smem});
    if (it != cache.end()) per_grid = it->second;
  }
  if (!per_grid) {
    int dev = 0, cus = 256, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, kThreads, smem) != hipSuccess) per = 4;
    per_grid = std::max(1, std::min(per, 8)) * std::max(1, cus);
    std::lock_guard<std::mutex> g(mu);
    cache[{kernel, smem}] = per_grid;
  }
  const int64_t per_block = (n_tiles + per_grid - 1) / per_grid;
  return (int)std::max<int64_t>(1, (n_tiles + per_block - 1) / std::max<int64_t>(1, per_block));
}

template <typename T, typename Idx, int VEC>
int launch_tiled_t(const PermPlan& P, const void* dtab, const void* src, void* dst, double beta,
                   hipStream_t stream) {
  const int T_ = P.tile_elems, G = T_ / VEC;
  const PermSwz& z = VEC == 1 ? P.swz1 : P.swzv;
  const size_t smem = z.mode == 0 ? (size_t)lds_pad(T_ - 1) + 1 : (size_t)T_;
  const size_t smem_bytes = smem * sizeof(T);
  const int ept = (G + kThreads - 1) / kThreads;
  const int use_beta = beta != 0.0;
  const Idx* tab = (const Idx*)dtab + (VEC == 1 ? 0 : 3 * (size_t)T_);
#define TQ_PERM_CASE(E)                                                                        \
  if (ept <= E) {                                                                              \
    const int grid = resident_grid((const void*)permute_tiled_kernel<T, Idx, E, VEC>,          \
                                   smem_bytes, P.n_tiles);                                     \
    hipLaunchKernelGGL((permute_tiled_kernel<T, Idx, E, VEC>), dim3(grid), dim3(kThreads),     \
                       smem_bytes, stream, (const T*)src, (T*)dst, tab, G, P.outer, z,         \
                       P.n_tiles, P.tile_mul, (float)beta, beta, use_beta);                    \
    TQ_HIP(hipGetLastError());                                                                 \
    return TQ_OK;                                                                              \
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

template <typename T, typename Idx>
int launch_tiled_any(const PermPlan& P, const void* dtab, const void* src, void* dst, double beta,
                     hipStream_t stream) {
  const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
  if constexpr (sizeof(T) <= 4)
    if (P.vec == 4 && al % (4 * sizeof(T)) == 0)
      return launch_tiled_t<T, Idx, 4>(P, dtab, src, dst, beta, stream);
  if constexpr (sizeof(T) <= 8)
    if (P.vec == 2 && al % (2 * sizeof(T)) == 0)
      return launch_tiled_t<T, Idx, 2>(P, dtab, src, dst, beta, stream);
  return launch_tiled_t<T, Idx, 1>(P, dtab, src, dst, beta, stream);
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
  if (P.idx64) return launch_tiled_any<T, int64_t>(P, dtab, src, dst, beta, stream);
  return launch_tiled_any<T, int32_t>(P, dtab, src, dst, beta, stream);
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

const char* perm_plan_kind(const PermPlan& P) {
  if (P.numel == 0) return "empty";
  if (P.use_generic) return "generic";
  return P.vec == 4 ? "vec4" : P.vec == 2 ? "vec2" : "tiled";
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
