// Store-pattern probe for the dense sweep's planes mode (tq_sweepd.hip emit_planes): what HBM write
// rate the output pattern alone reaches, without the products and the f16 split.
// Layout as C4's left dense op per lane: 4096 groups of 64 columns x 256 rows, rows contiguous
// (out_off = 64 r), six f16 planes 2^26 elements apart; 2 ops x 4 lanes = 8 such regions (6 GiB).
// A wave takes group g = blk * 4 + wave, stride (grid waves), and per 32-row tile rt writes each
// plane's 4 KiB (32 rows x 128 B) with 4 store instructions.
//   var 0: as the kernel: a store instruction = 32 rows x 32 B (lane = row, fk = 16-B half)
//   var 1: a store instruction = 1 KiB contiguous (lane L at 16 B x L)
//   var 2/3: vars 0/1 with non-temporal stores
//   var 4: var 1, the six planes of a tile interleaved per instruction (pl inner)
// hipcc --offload-arch=gfx950 -O3 planes_store_probe.hip -o planes_store_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;
constexpr long kPlaneElems = 1L << 26;        // f16 elements per plane (one lane of one op)
constexpr int kRegions = 8;                   // 2 ops x 4 lanes
constexpr int kGroups = 4096, kTout = 256;

template <int VAR>
__global__ void __launch_bounds__(256) store_kernel(_Float16* base, int nblocks_per_region, u32x4 v,
                                                     const uint2* __restrict__ xin) {
  const int region = blockIdx.x / nblocks_per_region, blk = blockIdx.x % nblocks_per_region;
  _Float16* P = base + (long)region * 6 * kPlaneElems;
  const int lane = threadIdx.x & 63, fr = lane & 31, fk = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = nblocks_per_region * kWaves;
  // vars 5 / 6: the kernel's input reads -- 16 x 8 B per lane and group (2 tiles x 8 k-steps),
  // used by the group's stores (5: loaded at the group's start; 6: one group ahead)
  auto xload = [&](int g) {
    unsigned acc = 0;
    if (g < kGroups) {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) acc ^= xin[((long)region * kGroups + g) * 1024 + s2 * 64 + lane].x;
    }
    return acc;
  };
  unsigned xnext = 0;
  if constexpr (VAR == 6) xnext = xload(blk * kWaves + wave);
  for (int g = blk * kWaves + wave; g < kGroups; g += nw) {
    const long gb = (long)g * 64 * kTout;
    unsigned xacc = 0;
    if constexpr (VAR == 5) xacc = xload(g);
    if constexpr (VAR == 6) {
      xacc = xnext;
      xnext = xload(g + nw);
    }
    for (int rt = 0; rt < kTout; rt += 32) {
      if constexpr (VAR == 0 || VAR == 2) {
        const long rb = gb + 64L * (rt + fr) + 8 * fk;
#pragma unroll
        for (int pl = 0; pl < 6; ++pl)
#pragma unroll
          for (int tl = 0; tl < 2; ++tl)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              u32x4* dst = reinterpret_cast<u32x4*>(P + pl * kPlaneElems + rb + 32 * tl + 16 * h);
              if constexpr (VAR == 2) __builtin_nontemporal_store(v, dst);
              else *dst = v;
            }
      } else if constexpr (VAR == 1 || VAR == 3) {
        const long tb = gb + 64L * rt + 8 * lane;
#pragma unroll
        for (int pl = 0; pl < 6; ++pl)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            u32x4* dst = reinterpret_cast<u32x4*>(P + pl * kPlaneElems + tb + 512 * i);
            if constexpr (VAR == 3) __builtin_nontemporal_store(v, dst);
            else *dst = v;
          }
      } else if constexpr (VAR == 5 || VAR == 6) {
        const long rb = gb + 64L * (rt + fr) + 8 * fk;
        u32x4 w = v;
        w.x ^= xacc;
#pragma unroll
        for (int pl = 0; pl < 6; ++pl)
#pragma unroll
          for (int tl = 0; tl < 2; ++tl)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              u32x4* dst = reinterpret_cast<u32x4*>(P + pl * kPlaneElems + rb + 32 * tl + 16 * h);
              *dst = w;
            }
      } else {
        const long tb = gb + 64L * rt + 8 * lane;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int pl = 0; pl < 6; ++pl) {
            u32x4* dst = reinterpret_cast<u32x4*>(P + pl * kPlaneElems + tb + 512 * i);
            *dst = v;
          }
      }
    }
  }
}

// var 7: the C4 launch's two op shapes -- regions 0-3 as above (tout 256, 4096 groups), regions
// 4-7 tout 128 over 8192 groups (same bytes), workgroups split bpr_a / bpr_b; loads as var 5
// GB: groups per iteration of the tout-128 regions (their loads issued together); GB = 0: no
// loads, but a vmcnt(0) wait at every group start (the drain of the wave's stores alone)
template <int GB>
__global__ void __launch_bounds__(256) store2_kernel(_Float16* base, int bpr_a, int bpr_b, u32x4 v,
                                                      const uint2* __restrict__ xin) {
  const bool isb = (int)blockIdx.x >= 4 * bpr_a;
  const int bpr = isb ? bpr_b : bpr_a;
  const int rel = isb ? blockIdx.x - 4 * bpr_a : blockIdx.x;
  const int region = (isb ? 4 : 0) + rel / bpr, blk = rel % bpr;
  const int tout = isb ? 128 : 256, ngroups = isb ? 8192 : 4096;
  _Float16* P = base + (long)region * 6 * kPlaneElems;
  const int lane = threadIdx.x & 63, fr = lane & 31, fk = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = bpr * kWaves;
  const int nld = isb ? 8 : 16;
  const int gpi = isb && GB > 0 ? GB : 1;   // groups per iteration
  for (int g0 = (blk * kWaves + wave) * gpi; g0 < ngroups; g0 += nw * gpi) {
    unsigned xacc = 0;
    if constexpr (GB == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
    for (int q = 0; q < gpi; ++q)
      for (int s2 = 0; s2 < nld && xin; ++s2) xacc ^= xin[((long)region * 8192 + g0 + q) * 512 + s2 * 32 + fr].x;
    for (int q = 0; q < gpi; ++q)
    for (int rt = 0; rt < tout; rt += 32) {
      const long gb = (long)(g0 + q) * 64 * tout;
      const long rb = gb + 64L * (rt + fr) + 8 * fk;
      u32x4 w = v;
      w.x ^= xacc;
#pragma unroll
      for (int pl = 0; pl < 6; ++pl)
#pragma unroll
        for (int tl = 0; tl < 2; ++tl)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            u32x4* dst = reinterpret_cast<u32x4*>(P + pl * kPlaneElems + rb + 32 * tl + 16 * h);
            *dst = w;
          }
    }
  }
}

// var 8: the two-shape launch with the input reads issued as LDS-DMA (global_load_lds_dwordx4 into
// a per-wave LDS scratch) and never waited for: the reads' DRAM traffic without any wave waiting
// on them
__global__ void __launch_bounds__(256) store3_kernel(_Float16* base, int bpr_a, int bpr_b, u32x4 v,
                                                      const uint2* __restrict__ xin) {
  __shared__ __attribute__((aligned(16))) unsigned char scratch[kWaves][1024];
  const bool isb = (int)blockIdx.x >= 4 * bpr_a;
  const int bpr = isb ? bpr_b : bpr_a;
  const int rel = isb ? blockIdx.x - 4 * bpr_a : blockIdx.x;
  const int region = (isb ? 4 : 0) + rel / bpr, blk = rel % bpr;
  const int tout = isb ? 128 : 256, ngroups = isb ? 8192 : 4096;
  _Float16* P = base + (long)region * 6 * kPlaneElems;
  const int lane = threadIdx.x & 63, fr = lane & 31, fk = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = bpr * kWaves;
  const int ndma = isb ? 4 : 8;   // x 1 KiB = the group's 16 x 256 B (A) / 8 x 256 B (B) of reads... x2
  const unsigned lds = (unsigned)(uintptr_t)&scratch[wave][0];
  for (int g = blk * kWaves + wave; g < ngroups; g += nw) {
    const char* src = reinterpret_cast<const char*>(xin + ((long)region * 8192 + g) * 512);
    for (int d = 0; d < ndma; ++d) {
      const char* a = src + d * 1024 + lane * 16;
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" :: "s"(lds), "v"(a) : "memory", "m0");
    }
    const long gb = (long)g * 64 * tout;
    for (int rt = 0; rt < tout; rt += 32) {
      const long rb = gb + 64L * (rt + fr) + 8 * fk;
#pragma unroll
      for (int pl = 0; pl < 6; ++pl)
#pragma unroll
        for (int tl = 0; tl < 2; ++tl)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            u32x4* dst = reinterpret_cast<u32x4*>(P + pl * kPlaneElems + rb + 32 * tl + 16 * h);
            *dst = v;
          }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// linear fill of the same bytes (the ceiling: every wave writes consecutive 1-KiB blocks)
__global__ void __launch_bounds__(256) fill_kernel(u32x4* base, long n16, u32x4 v) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256) base[i] = v;
}

template <typename F>
static double time_ms(F&& f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 2; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char** argv) {
  const int bpr = argc > 1 ? atoi(argv[1]) : 64;   // workgroups per region (C4's launch: ~64-128)
  const size_t bytes = (size_t)kRegions * 6 * kPlaneElems * 2;
  _Float16* buf = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
  const u32x4 v = {0x3c003c00u, 0x3c003c00u, 0x3c003c00u, 0x3c003c00u};
  uint2* xin = nullptr;   // inputs: 8 regions x 4096 groups x 1024 x 8 B (256 MiB; var 7: 8192 x 512)
  if (hipMalloc(&xin, (size_t)kRegions * kGroups * 1024 * 8) != hipSuccess) return 1;
  (void)hipMemset(xin, 0, (size_t)kRegions * kGroups * 1024 * 8);
  const double gb = bytes / 1e9;
  auto report = [&](const char* name, double ms) {
    printf("{\"variant\": \"%s\", \"blocks_per_region\": %d, \"ms\": %.3f, \"TBps\": %.2f}\n", name, bpr, ms, gb / ms);
  };
  const dim3 grid(kRegions * bpr);
  report("fill", time_ms([&] { hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, (u32x4*)buf, (long)(bytes / 16), v); }, 5));
  report("rows32B", time_ms([&] { hipLaunchKernelGGL(store_kernel<0>, grid, dim3(256), 0, 0, buf, bpr, v, xin); }, 5));
  report("contig1K", time_ms([&] { hipLaunchKernelGGL(store_kernel<1>, grid, dim3(256), 0, 0, buf, bpr, v, xin); }, 5));
  report("rows32B_nt", time_ms([&] { hipLaunchKernelGGL(store_kernel<2>, grid, dim3(256), 0, 0, buf, bpr, v, xin); }, 5));
  report("contig1K_nt", time_ms([&] { hipLaunchKernelGGL(store_kernel<3>, grid, dim3(256), 0, 0, buf, bpr, v, xin); }, 5));
  report("rows32B_xload", time_ms([&] { hipLaunchKernelGGL(store_kernel<5>, grid, dim3(256), 0, 0, buf, bpr, v, xin); }, 5));
  report("rows32B_xprefetch", time_ms([&] { hipLaunchKernelGGL(store_kernel<6>, grid, dim3(256), 0, 0, buf, bpr, v, xin); }, 5));
  for (int ba : {48, 64, 80}) {
    const int bb = 128 - ba;
    char name[64];
    snprintf(name, sizeof name, "twoshapes_xload_a%d_b%d", ba, bb);
    report(name, time_ms([&] { hipLaunchKernelGGL(store2_kernel<1>, dim3(4 * ba + 4 * bb), dim3(256), 0, 0, buf, ba, bb, v, xin); }, 5));
  }
  report("twoshapes_xload_b2groups", time_ms([&] { hipLaunchKernelGGL(store2_kernel<2>, dim3(4 * 64 + 4 * 64), dim3(256), 0, 0, buf, 64, 64, v, xin); }, 5));
  report("twoshapes_xload_b4groups", time_ms([&] { hipLaunchKernelGGL(store2_kernel<4>, dim3(4 * 64 + 4 * 64), dim3(256), 0, 0, buf, 64, 64, v, xin); }, 5));
  report("twoshapes_drain_only", time_ms([&] { hipLaunchKernelGGL(store2_kernel<0>, dim3(4 * 64 + 4 * 64), dim3(256), 0, 0, buf, 64, 64, v, xin); }, 5));
  report("twoshapes_dma_nowait", time_ms([&] { hipLaunchKernelGGL(store3_kernel, dim3(4 * 64 + 4 * 64), dim3(256), 0, 0, buf, 64, 64, v, xin); }, 5));
  report("twoshapes_noload", time_ms([&] { hipLaunchKernelGGL(store2_kernel<1>, dim3(4 * 64 + 4 * 64), dim3(256), 0, 0, buf, 64, 64, v, (const uint2*)nullptr); }, 5));
  report("contig1K_plinner", time_ms([&] { hipLaunchKernelGGL(store_kernel<4>, grid, dim3(256), 0, 0, buf, bpr, v, xin); }, 5));
  hipFree(buf);
  return 0;
}
