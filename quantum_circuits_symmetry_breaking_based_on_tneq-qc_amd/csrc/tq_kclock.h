// In-kernel clock stamps (development build only: -DTQ_KCLOCK; the product library contains no
// stamp).  Workgroup 0 of a launch records s_memtime (shader clock) and s_memrealtime (100 MHz)
// at its start and end; the in-kernel clock of that launch is
// (mt1 - mt0) / (rt1 - rt0) x 100 MHz (MI355X_MICROARCH.md: the PMC estimate
// GRBM_GUI_ACTIVE / 8 / duration is not physical for short dispatches).  Read back through
// tq_debug_kernel_clock (tq_capi.cpp; scripts/kernel_clock.py).
#pragma once

#ifdef TQ_KCLOCK
constexpr int kKClockSlots = 4096;
#define TQ_KCLOCK_DEFINE(name)                                   \
  __device__ unsigned long long name[kKClockSlots][4];          \
  __device__ unsigned int name##_n;
#define TQ_KCLOCK_BEGIN()                                                         \
  unsigned long long kc_mt0_ = 0, kc_rt0_ = 0;                                    \
  const bool kc_rec_ = (blockIdx.x | blockIdx.y | blockIdx.z) == 0 && threadIdx.x == 0; \
  if (kc_rec_) {                                                                  \
    kc_mt0_ = __builtin_amdgcn_s_memtime();                                       \
    kc_rt0_ = __builtin_amdgcn_s_memrealtime();                                   \
  }
#define TQ_KCLOCK_END(name)                                                       \
  if (kc_rec_) {                                                                  \
    const unsigned long long mt1 = __builtin_amdgcn_s_memtime();                  \
    const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();              \
    const unsigned s = atomicAdd(&name##_n, 1u) % kKClockSlots;                   \
    name[s][0] = kc_mt0_;                                                         \
    name[s][1] = kc_rt0_;                                                         \
    name[s][2] = mt1;                                                             \
    name[s][3] = rt1;                                                             \
  }
// host: copy up to n records (4 x u64 each) and reset; returns the count
#define TQ_KCLOCK_READ(name, out, n)                                                               \
  [&]() -> int {                                                                                   \
    unsigned cnt = 0;                                                                              \
    if (hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(name##_n), sizeof(cnt)) != hipSuccess) return -1;     \
    const int k = (int)std::min<unsigned>(std::min<unsigned>(cnt, kKClockSlots), (unsigned)(n));   \
    if (k > 0 && hipMemcpyFromSymbol((out), HIP_SYMBOL(name), sizeof(unsigned long long) * 4 * k) != hipSuccess) \
      return -1;                                                                                   \
    const unsigned zero = 0;                                                                       \
    if (hipMemcpyToSymbol(HIP_SYMBOL(name##_n), &zero, sizeof(zero)) != hipSuccess) return -1;     \
    return k;                                                                                      \
  }()
#else
#define TQ_KCLOCK_DEFINE(name)
#define TQ_KCLOCK_BEGIN()
#define TQ_KCLOCK_END(name)
#define TQ_KCLOCK_READ(name, out, n) 0
#endif
