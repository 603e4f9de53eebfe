// Pass-latency probe (r04): what one barriered LDS pass of the sweep2 kernel costs on gfx950 at
// 512 threads per workgroup, piece by piece.  One workgroup per CU on 256 CUs (or 1 / 2 per CU),
// P passes per launch; thread 0 of workgroup 0 reads the shader clock after each pass.
//   variant 0: barrier only
//   variant 1: one dependent LDS read per thread, then the barrier
//   variant 2: a 4x4 complex64 gate: 4 LDS reads, 16 complex MACs, 4 LDS writes, barrier
//   variant 3: variant 2 preceded by a dependent LDS read of the pass's metadata (the address
//              base), i.e. two LDS round trips per pass
//   variant 4: variant 2 with 4 groups per thread (8192-element tile instead of 2048)
//   variant 5: a 4x4 gate on a 1024-element tile: 256 groups, threads >= 256 idle
//   variant 6: the same with two threads per group (adjacent lanes), each computing 2 outputs
//   variant 7: variant 5 with the 16 coefficients read from LDS every pass (broadcast reads)
//   variant 8: variant 7 with the coefficients made wave-uniform (readfirstlane: scalar registers)
// Usage: ./pass_probe  -> one JSON line per (variant, workgroups per CU)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int NT = 512, P = 64;

struct c64 { float re, im; };

template <int V>
__global__ void __launch_bounds__(NT) probe(unsigned long long* out, int salt) {
  __shared__ c64 tile[8192];
  __shared__ int meta[64];
  const int tid = threadIdx.x;
  for (int i = tid; i < 8192; i += NT) tile[i] = c64{(float)(i ^ salt), 1.f};
  if (tid < 64) meta[tid] = (tid * 37 + salt) & 63;
  __syncthreads();
  const c64 c[4] = {{0.5f, 0.1f}, {0.2f, -0.3f}, {-0.4f, 0.2f}, {0.1f, 0.7f}};
  unsigned long long t0 = clock64();
  int m = 0;
  for (int p = 0; p < P; ++p) {
    if constexpr (V == 1) {
      m = meta[(m + tid + p) & 63];
    } else if constexpr (V == 7 || V == 8) {
      __shared__ c64 cfl[16];
      if (p == 0 && tid < 16) cfl[tid] = c64{0.1f * tid, 0.05f * tid};
      if (p == 0) __syncthreads();
      c64 cc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        cc[i] = cfl[(i + m) & 15];
        if constexpr (V == 8) {
          cc[i].re = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(cc[i].re)));
          cc[i].im = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(cc[i].im)));
        }
      }
      const int grp = tid;
      if (grp < 256) {
        const int a = grp;
        c64 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = tile[a + k * 256];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          c64 acc{0.f, 0.f};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc.re += x[k].re * cc[k * 4 + n].re - x[k].im * cc[k * 4 + n].im;
            acc.im += x[k].re * cc[k * 4 + n].im + x[k].im * cc[k * 4 + n].re;
          }
          tile[a + n * 256] = acc;
        }
      }
    } else if constexpr (V == 5 || V == 6) {
      // 1024-element tile: inputs at stride 256 (positions 8, 9)
      const int grp = V == 5 ? tid : tid >> 1;
      if (grp < 256) {
        const int a = grp;
        c64 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = tile[a + k * 256];
        constexpr int NO = V == 5 ? 4 : 2;
        const int n0 = V == 5 ? 0 : (tid & 1) * 2;
#pragma unroll
        for (int q = 0; q < NO; ++q) {
          const int n = n0 + q;
          c64 acc{0.f, 0.f};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const c64 cc = c[(k + n) & 3];
            acc.re += x[k].re * cc.re - x[k].im * cc.im;
            acc.im += x[k].re * cc.im + x[k].im * cc.re;
          }
          tile[a + n * 256] = acc;
        }
      }
    } else if constexpr (V >= 2) {
      int base = 0;
      if constexpr (V == 3) base = meta[(m + p) & 63] & 1;   // the pass's metadata first
      constexpr int G = V == 4 ? 4 : 1;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int grp = tid + g * NT;
        // 4 inputs at stride 2048 / 4 groups: positions 11, 12 of a 13-bit index
        const int a = (grp ^ base) & 2047;
        c64 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = tile[a + k * 2048];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          c64 acc{0.f, 0.f};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const c64 cc = c[(k + n) & 3];
            acc.re += x[k].re * cc.re - x[k].im * cc.im;
            acc.im += x[k].re * cc.im + x[k].im * cc.re;
          }
          tile[a + n * 2048] = acc;
        }
      }
      m += base;
    }
    __syncthreads();
    if (blockIdx.x == 0 && tid == 0 && p == P - 1) out[0] = clock64() - t0;
  }
  if (blockIdx.x == 0 && tid == 0) out[1] = (unsigned long long)m + (unsigned long long)tile[5].re;
}

template <int V>
void run(int wgs, unsigned long long* d, const char* name) {
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe<V>, dim3(wgs), dim3(NT), 0, 0, d, rep);
  hipDeviceSynchronize();
  unsigned long long h[2];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, 0);
  for (int rep = 0; rep < 20; ++rep) hipLaunchKernelGGL(probe<V>, dim3(wgs), dim3(NT), 0, 0, d, rep);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  printf("{\"variant\": %d, \"name\": \"%s\", \"workgroups\": %d, \"clocks_per_pass\": %.0f, \"us_per_launch\": %.2f}\n",
         V, name, wgs, (double)h[0] / P, ms * 1000.0 / 20);
}

int main() {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 16) != hipSuccess) return 1;
  for (int wgs : {256, 512}) {
    run<0>(wgs, d, "barrier only");
    run<1>(wgs, d, "1 dependent LDS read + barrier");
    run<2>(wgs, d, "4x4 gate, 1 group per thread");
    run<3>(wgs, d, "metadata read + 4x4 gate");
    run<4>(wgs, d, "4x4 gate, 4 groups per thread");
    run<5>(wgs, d, "4x4 gate on 1024 elements, 256 threads");
    run<6>(wgs, d, "4x4 gate on 1024 elements, 2 threads per group");
    run<7>(wgs, d, "variant 5 + coefficients from LDS each pass");
    run<8>(wgs, d, "variant 7 with scalar (readfirstlane) coefficients");
  }
  hipFree(d);
  return 0;
}
