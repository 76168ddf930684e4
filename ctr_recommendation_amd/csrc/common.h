// Shared device helpers for the FiBiNET gfx950 kernels.
// Wave width is 64 on CDNA4; every cross-lane idiom below assumes it.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

// Every kernel of the library is launched through fbn_launch: while the host has a probe armed
// (fbn_probe_arm .. fbn_probe_disarm around one entry-point call, bench.py's roofline timings) the
// launch records the probe's start event at the first kernel's start and its stop event at every
// kernel's end (hipExtLaunchKernelGGL): the call's kernel span as rocprofv3 sees it, with no
// marker packets or dispatch gaps around it.
bool fbn_probe_take(hipEvent_t* start, hipEvent_t* stop);
template <typename F, typename... Args>
inline void fbn_launch(F kernel, const dim3& grid, const dim3& block, unsigned shmem, hipStream_t stream,
                       Args... args) {
  hipEvent_t start = nullptr, stop = nullptr;
  fbn_probe_take(&start, &stop);
  hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, start, stop, 0, args...);
}

#define FBN_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));

// Error codes shared with include/fibinet.h
enum {
  FBN_OK = 0,
  FBN_ERR_ARG = 1,
  FBN_ERR_LAUNCH = 2,
  FBN_ERR_UNSUPPORTED = 3,
};

// round-to-nearest-even f32 -> bf16 (NaN-safe through the hardware cvt at -O3)
__device__ __forceinline__ short f2bf(float x) {
  __bf16 b = (__bf16)x;
  return __builtin_bit_cast(short, b);
}
__device__ __forceinline__ float bf2f(short s) {
  return __builtin_bit_cast(float, ((uint32_t)(uint16_t)s) << 16);
}

// ---------------------------------------------------------------- wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// sum over aligned groups of G lanes (G power of two <= 64)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- Philox4x32-10
// Counter-based RNG for dropout: (seed, offset, element index) -> 4 uniforms.
// Stateless, so the backward can regenerate a mask and graph replay only needs the
// device-resident offset to advance.
struct Philox4 { uint32_t x, y, z, w; };
__device__ __forceinline__ Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += W0; k1 += W1;
  }
  return {c0, c1, c2, c3};
}
__device__ __forceinline__ float u01(uint32_t r) { return (float)(r >> 8) * (1.0f / 16777216.0f); }

// Wave priority of the main-stream step kernels (GEMMs, gathers, BN, bilinear).  The lazy
// table-Adam passes run beside them on the side stream as long-lived, VALU-heavy waves; a SIMD
// arbitrates issue by priority, then AGE, so at equal priority the older side waves win and the
// main-stream kernel that shares the SIMD takes the leftover slots.  s_setprio > 0 here makes the
// side stream the background (it keeps priority 0).  -DFBN_MAIN_PRIO_LEVEL=0: off (A/B).
#ifndef FBN_MAIN_PRIO_LEVEL
#define FBN_MAIN_PRIO_LEVEL 2
#endif
#define FBN_MAIN_PRIO()                                                   \
  do {                                                                    \
    if (FBN_MAIN_PRIO_LEVEL > 0) __builtin_amdgcn_s_setprio(FBN_MAIN_PRIO_LEVEL); \
  } while (0)

// ---------------------------------------------------------------- host helpers
#define FBN_CHECK_LAUNCH()                                       \
  do {                                                           \
    hipError_t _e = hipGetLastError();                           \
    if (_e != hipSuccess) { fbn_set_error(hipGetErrorString(_e)); return FBN_ERR_LAUNCH; } \
  } while (0)

void fbn_set_error(const char* msg);
static inline int fbn_cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
