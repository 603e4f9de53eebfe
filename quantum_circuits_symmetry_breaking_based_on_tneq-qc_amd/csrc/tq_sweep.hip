// Fused multi-gate sweep: several consecutive small-operand absorptions in ONE HBM pass.
//
// In a qubit-line sweep (the contraction tree of every amplitude workload, SURVEY.md §8(a) rows
// a4/a5: each opt_einsum pairwise step at einsum_strategy.py:639-643 absorbs one (2,2,2,2) gate
// into the running tensor) consecutive steps touch a few legs each: one APPLY pass per gate
// reads and writes the whole running tensor.  A chain of q such steps is executed here as
//     Y[outer, t_out] = (G_q o ... o G_1)(X[outer, t_in])
// where the tile modes t_in (legs of X any gate of the chain contracts) and t_out (legs of Y a
// gate produced) span at most 64 elements (32 for complex128).  A workgroup owns chunks of 64
// "columns" (assignments of the untouched outer modes): the chunk's tile is staged in LDS as
// [tile element][column]; each gate is applied by waves that take one output element e of the
// new working set at a time, four at once for latency hiding — e, its K source rows and its gate
// column are wave-uniform (host-built tables in LDS, coefficients broadcast from LDS), the column
// is the lane, so a gate costs K conflict-free ds_read_b64 + one ds_write per element and lane.
// The next chunk's global loads are issued into registers before the current chunk's gates run.
// Algorithmic bytes = (numel(X) + numel(Y)) * sizeof.
#include <algorithm>

#include "tq_common.h"
#include "tq_sweep.h"

namespace tq {

namespace {

constexpr int kThreads = 1024, kWaves = 16, COLS = 64, LCOLS = 6, LD = COLS + 1;

// generic (non power-of-two extents) column offset: mixed radix over the outer runs
__device__ __forceinline__ int64_t col_offset_generic(const SweepArgs& a, int64_t c,
                                                    bool out) {
  int64_t off = 0;
  for (int r = 0; r < a.nruns; ++r) {
    const int64_t d = c % a.run_ext[r];
    c /= a.run_ext[r];
    off += d * (out ? a.run_out[r] : a.run_in[r]);
  }
  return off;
}

// chunk part of a power-of-two column offset: bits >= 6 of the column index (wave-uniform)
__device__ __forceinline__ int64_t chunk_offset(const int64_t* w, int nbits, int64_t ch) {
  int64_t off = 0;
  for (int b = LCOLS; b < nbits; ++b)
    if ((ch >> (b - LCOLS)) & 1) off += w[b];
  return off;
}

template <int KC, typename T>
__device__ __forceinline__ void gate_pass(const T* src, T* dst, const int32_t* tab, const T* g,
                                          int K, int N, int W, int wave) {
  const int KK = KC > 0 ? KC : K;
  for (int e0 = wave; e0 < W; e0 += 4 * kWaves) {
    T acc[4];
    int nn[4];
    const int32_t* row[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = min(e0 + u * kWaves, W - 1);
      row[u] = tab + e * (KK + 1);
      nn[u] = row[u][KK];
      acc[u] = tzero<T>();
    }
    if constexpr (KC > 0) {
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) cmac(acc[u], src[row[u][k] * LD], g[k * N + nn[u]]);
    } else {
      for (int k = 0; k < KK; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) cmac(acc[u], src[row[u][k] * LD], g[k * N + nn[u]]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (e0 + u * kWaves < W) dst[(e0 + u * kWaves) * LD] = acc[u];
  }
}

template <typename T, int WMAX, bool FAN>
__global__ void __launch_bounds__(kThreads) sweep_kernel(SweepArgs a, SweepLanes ls) {
  constexpr int RMAX = WMAX * COLS / kThreads;  // staged elements per thread
  // FAN: a third buffer keeps the chunk's input for every lane; the lanes' coefficients are all
  // staged once per workgroup (K*N <= kSweepFanKN each)
  __shared__ T buf[FAN ? 3 : 2][WMAX * LD];
  __shared__ T gs[FAN ? kSweepMaxLanes * kSweepMaxGates * kSweepFanKN : kSweepMaxGates * kSweepMaxKN];
  __shared__ int64_t tio[2 * WMAX];              // tin_off | tout_off
  __shared__ int64_t lo_in[COLS], lo_out[COLS];  // lane part of the column offsets
  __shared__ int32_t tabs[kSweepTabMax];         // gate tables: per output element K source rows, n

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // a lane-merged launch (SweepLanes): blockIdx.y selects the slice lane's tensors (FAN: every
  // lane in turn inside the workgroup, X shared)
  const int ln = ls.n > 0 && !FAN ? (int)blockIdx.y : -1;
  const T* __restrict__ X = reinterpret_cast<const T*>(ln >= 0 ? ls.X[ln] : FAN ? ls.X[0] : a.X);
  const bool pow2 = a.colbits >= 0;
  constexpr int GS = FAN ? kSweepFanKN : kSweepMaxKN;   // coefficient slots per gate in gs
  const int nlg = FAN ? ls.n : 1;                       // lanes whose coefficients are staged
  // ---- prologue: every table load independent of the others (one latency, not one per gate)
  for (int idx = tid; idx < nlg * a.ngates * GS; idx += kThreads) {
    const int lj = idx / GS, t = idx - lj * GS;
    const int l = lj / a.ngates, j = lj - l * a.ngates;
    if (t < a.K[j] * a.N[j]) {
      const T* G = reinterpret_cast<const T*>(FAN ? ls.G[l][j] : ln >= 0 ? ls.G[ln][j] : a.G[j]);
      gs[idx] = G[a.gidx[j] ? a.gidx[j][t] : t];
    }
  }
  for (int t = tid; t < a.tab_len; t += kThreads) tabs[t] = a.tabs[t];
  for (int t = tid; t < a.tin; t += kThreads) tio[t] = a.tin_off[t];
  for (int t = tid; t < a.tout; t += kThreads) tio[WMAX + t] = a.tout_off[t];
  if (tid < COLS && pow2) {
    int64_t oi = 0, oo = 0;
    for (int b = 0; b < LCOLS && b < a.colbits; ++b)
      if ((tid >> b) & 1) { oi += a.w_in[b]; oo += a.w_out[b]; }
    lo_in[tid] = oi;
    lo_out[tid] = oo;
  }
  __syncthreads();

  const int64_t nchunks = (a.ncols + COLS - 1) / COLS;
  const int nin = a.tin * COLS, nout = a.tout * COLS;
  const bool lcf = a.load_colfast, scf = a.store_colfast;
  T reg[RMAX];

  // element idx of a chunk -> (tile element t, column c)
  auto tc = [&](int idx, bool colfast, int tsize, int tshift, int& t, int& c) {
    if (colfast) { t = idx >> LCOLS; c = idx & (COLS - 1); }
    else if (tshift >= 0) { c = idx >> tshift; t = idx & (tsize - 1); }
    else { c = idx / tsize; t = idx - c * tsize; }
  };

  auto prefetch = [&](int64_t ch) {
    const int64_t c0 = ch * COLS;
    const int64_t hi = pow2 ? chunk_offset(a.w_in, a.colbits, ch) : 0;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int idx = tid + r * kThreads;
      reg[r] = tzero<T>();
      if (idx < nin) {
        int t, c;
        tc(idx, lcf, a.tin, a.tin_shift, t, c);
        if (c0 + c < a.ncols) {
          const int64_t co = pow2 ? hi + lo_in[c] : col_offset_generic(a, c0 + c, false);
          reg[r] = X[co + tio[t]];
        }
      }
    }
  };

  constexpr int IN = FAN ? 2 : 0;   // the buffer the chunk enters
  int64_t ch = blockIdx.x;
  if (ch < nchunks) prefetch(ch);
  for (; ch < nchunks; ch += gridDim.x) {
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int idx = tid + r * kThreads;
      if (idx < nin) {
        int t, c;
        tc(idx, lcf, a.tin, a.tin_shift, t, c);
        buf[IN][t * LD + c] = reg[r];
      }
    }
    __syncthreads();
    const int64_t nxt = ch + gridDim.x;
    if (nxt < nchunks) prefetch(nxt);  // in flight while the gates run
    for (int l = 0; l < nlg; ++l) {
      T* __restrict__ Y = reinterpret_cast<T*>(FAN ? ls.Y[l] : ln >= 0 ? ls.Y[ln] : a.Y);
      for (int j = 0; j < a.ngates; ++j) {
        // FAN: gate 0 reads the kept input, later gates ping-pong between buffers 0 and 1
        const T* src = (FAN ? (j == 0 ? buf[2] : buf[(j - 1) & 1]) : buf[j & 1]) + lane;
        T* dst = (FAN ? buf[j & 1] : buf[(j + 1) & 1]) + lane;
        const int K = a.K[j], N = a.N[j], W = a.W[j];
        const int32_t* tab = tabs + a.tab_at[j];
        const T* g = gs + (FAN ? (l * a.ngates + j) * GS : j * GS);
        switch (K) {
          case 1: gate_pass<1>(src, dst, tab, g, K, N, W, wave); break;
          case 2: gate_pass<2>(src, dst, tab, g, K, N, W, wave); break;
          case 4: gate_pass<4>(src, dst, tab, g, K, N, W, wave); break;
          default: gate_pass<0>(src, dst, tab, g, K, N, W, wave); break;
        }
        __syncthreads();
      }
      const T* res = FAN ? buf[(a.ngates - 1) & 1] : buf[a.ngates & 1];
      const int64_t c0 = ch * COLS;
      const int64_t hi = pow2 ? chunk_offset(a.w_out, a.colbits, ch) : 0;
      for (int idx = tid; idx < nout; idx += kThreads) {
        int t, c;
        tc(idx, scf, a.tout, a.tout_shift, t, c);
        if (c0 + c < a.ncols) {
          T v = res[t * LD + c];
          const int64_t co = pow2 ? hi + lo_out[c] : col_offset_generic(a, c0 + c, true);
          T* p = Y + co + tio[WMAX + t];
          if (a.use_beta) {
            if constexpr (sizeof(typename Traits<T>::R) == 4) v = v + *p * (float)a.beta;
            else v = v + *p * a.beta;
          }
          *p = v;
        }
      }
      __syncthreads();  // res / the buffers are rewritten by the next lane or chunk
    }
  }
}

template <typename T>
int sweep_t(const SweepArgs& a, const SweepLanes& ls, hipStream_t stream) {
  constexpr int WMAX = sizeof(T) > 8 ? 32 : 64;
  if (a.tin > WMAX || a.tout > WMAX) {
    set_error("sweep: tile too large for dtype");
    return TQ_ERR_UNSUPPORTED;
  }
  const int64_t nchunks = (a.ncols + COLS - 1) / COLS;
  // 16 waves per workgroup (one output element per wave and gate pass at a 64-element tile);
  // 2 workgroups per CU fit in LDS; >= 2 chunks per workgroup let the register prefetch overlap
  const int64_t cap = 256 * 2;
  int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(nchunks, nchunks >= 2 * cap ? cap : std::max<int64_t>(256, (nchunks + 1) / 2)));
  const int nl = std::max(1, ls.n);
  if constexpr (sizeof(T) <= 8) {   // (complex128: three tile buffers + the lanes' coefficients exceed LDS)
    if (ls.fan && nl > 1) {
      // X read once per chunk, every lane's gates in turn (one workgroup per CU: 3 tile buffers)
      const int64_t fb = std::max<int64_t>(1, std::min<int64_t>(nchunks, 256));
      hipLaunchKernelGGL((sweep_kernel<T, WMAX, true>), dim3((unsigned)fb), dim3(kThreads), 0, stream, a, ls);
      TQ_HIP(hipGetLastError());
      return TQ_OK;
    }
  }
  if (nl > 1) blocks = std::max<int64_t>(1, std::min<int64_t>(nchunks, (2 * cap + nl - 1) / nl));   // one round shared
  hipLaunchKernelGGL((sweep_kernel<T, WMAX, false>), dim3((unsigned)blocks, (unsigned)nl), dim3(kThreads), 0, stream, a, ls);
  TQ_HIP(hipGetLastError());
  return TQ_OK;
}

}  // namespace

int sweep_launch_lanes(int dtype, const SweepArgs& a, const SweepLanes& l0, hipStream_t stream) {
  if (a.ncols == 0) return TQ_OK;
  // fan-out when every lane reads the same X and every gate fits kSweepFanKN coefficients
  // (TQ_SWEEP_FAN=0: the per-lane grid)
  static const bool fan_on = [] {
    const char* e = getenv("TQ_SWEEP_FAN");
    return !(e && e[0] == '0');
  }();
  SweepLanes l = l0;
  l.fan = 0;
  if (fan_on && l.n > 1 && !a.use_beta && dtype != TQ_C128) {
    bool same = true;
    for (int j = 1; j < l.n; ++j) same = same && l.X[j] == l.X[0];
    for (int j = 0; j < a.ngates; ++j) same = same && a.K[j] * a.N[j] <= kSweepFanKN;
    l.fan = same ? 1 : 0;
  }
  if (a.ngates < 1 || a.ngates > kSweepMaxGates || a.nruns > kSweepMaxRuns || a.colbits > 48 ||
      a.tab_len > kSweepTabMax || l.n < 0 || l.n > kSweepMaxLanes) {
    set_error("sweep: unsupported chain shape");
    return TQ_ERR_UNSUPPORTED;
  }
  for (int j = 0; j < a.ngates; ++j)
    if (a.K[j] * a.N[j] > kSweepMaxKN || a.W[j] > kSweepWMax) {
      set_error("sweep: gate too large");
      return TQ_ERR_UNSUPPORTED;
    }
  switch (dtype) {
    case TQ_F32: return sweep_t<float>(a, l, stream);
    case TQ_F64: return sweep_t<double>(a, l, stream);
    case TQ_C64: return sweep_t<c64>(a, l, stream);
    case TQ_C128: return sweep_t<c128>(a, l, stream);
  }
  set_error("sweep: bad dtype");
  return TQ_ERR_INVALID;
}

int sweep_launch(int dtype, const SweepArgs& a, hipStream_t stream) {
  return sweep_launch_lanes(dtype, a, SweepLanes{}, stream);
}

}  // namespace tq
