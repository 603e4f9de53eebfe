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
  uint2* xin = nullptr;   // inputs: 8 regions x 4096 groups x 1024 x 8 B (256 MiB)
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
  report("contig1K_plinner", time_ms([&] { hipLaunchKernelGGL(store_kernel<4>, grid, dim3(256), 0, 0, buf, bpr, v, xin); }, 5));
  hipFree(buf);
  return 0;
}
