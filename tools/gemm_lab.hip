// GEMM lab: what bounds the LDS-DMA bf16 GEMM on the C3 MLP shapes (tuning aid, not product).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/gemm_lab tools/gemm_lab.hip && tools/gemm_lab
//
// C[M][N] (f32) = A[M][K] * B[N][K]^T, both operands bf16 and K-contiguous (the forward and dgrad
// form).  The main loop is the product kernel's (ctr_recommendation_amd/csrc/gemm.hip,
// gemm_dma16_kernel: global_load_lds_dwordx4 straight into XOR-swizzled LDS images, counted vmcnt
// + raw s_barrier, S-stage ring) with ablation modes:
//   MODE 0  full
//   MODE 1  no MFMA (the feed alone: DMA + barriers + fragment reads)
//   MODE 2  no DMA inside the loop (MFMAs on the prologue's stages: LDS reads + MFMA alone)
// Every variant is timed with hipEvents over 50 launches after 5 warm-ups, on random data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>
#include <cmath>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(1))) void g_void;
typedef __attribute__((address_space(3))) void l_void;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ int xcd_tile(int bid, int nb) {
  const int q = nb / 8, r = nb % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

template <int GPW, int S>
__device__ __forceinline__ void wait_dma(int ahead) {
  if constexpr (S >= 5) {
    if (ahead >= 3) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * GPW) : "memory"); return; }
  }
  if constexpr (S >= 4) {
    if (ahead >= 2) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory"); return; }
  }
  if constexpr (S >= 3) {
    if (ahead >= 1) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory"); return; }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// wait until at most `ahead` stages (GPW DMA groups each) of this wave are outstanding
template <int GPW>
__device__ __forceinline__ void wait_dma_n(int ahead) {
  switch (ahead) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * GPW) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * GPW) : "memory"); break;
  }
}

template <int BM, int BN, int S, int WGM, int WGN, int MODE>
__global__ void __launch_bounds__(64 * WGM * WGN) lab_kernel(const short* __restrict__ A, const short* __restrict__ B,
                                                              float* __restrict__ C, int M, int N, int K, int tiles_n) {
  constexpr int NW = WGM * WGN;
  constexpr int BK = 64;
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 32, TN = WN / 32;
  constexpr int AB = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  constexpr int GPW = (BM + BN) / 8 / NW;
  static_assert(((BM + BN) / 8) % NW == 0, "groups");
  __shared__ __attribute__((aligned(1024))) char smem[S * STAGE];
  const int bid = xcd_tile(blockIdx.x, gridDim.x);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = K / BK;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave % WGM, wn = wave / WGM;
  const int lr = lane & 31, lh = lane >> 5;
  const short* src[GPW];
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int grp = wave * GPW + j;
    const bool isA = grp < BM / 8;
    const int off = (isA ? grp : grp - BM / 8) * 1024 + lane * 16;
    const int r = off >> 7, slot = (off >> 4) & 7;
    const int sw = (slot ^ ((r >> 1) & 7)) << 3;
    src[j] = (isA ? A + (size_t)(m0 + r) * K : B + (size_t)(n0 + r) * K) + sw;
  }
  auto issue = [&](int t, int buf) {
#pragma unroll
    for (int j = 0; j < GPW; ++j)
      __builtin_amdgcn_global_load_lds((g_void*)(src[j] + t * BK), (l_void*)(smem + buf * STAGE + (wave * GPW + j) * 1024),
                                       16, 0, 0);
  };
  auto frag = [&](const char* img, int r0, int s) {
    const int r = r0 + (lane & 31);
    const int co = ((2 * s + (lane >> 5)) ^ ((r >> 1) & 7)) << 4;
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + co);
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
#pragma unroll
  for (int q = 0; q < S - 1; ++q)
    if (q < nk) issue(q, q);
  for (int t = 0; t < nk; ++t) {
    if (MODE != 2) wait_dma<GPW, S>(min(S - 2, nk - 1 - t));
    else if (t == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (MODE != 2 && t + S - 1 < nk) issue(t + S - 1, (t + S - 1) % S);
    const char* SA = smem + (MODE == 2 ? (t % (S - 1)) : (t % S)) * STAGE;
    const char* SB = SA + AB;
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[0][i] = frag(SA, wm * WM + i * 32, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[0][j] = frag(SB, wn * WN + j * 32, 0);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int cb = s & 1, nb = cb ^ 1;
      if (s + 1 < BK / 16) {
#pragma unroll
        for (int i = 0; i < TM; ++i) af[nb][i] = frag(SA, wm * WM + i * 32, s + 1);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[nb][j] = frag(SB, wn * WN + j * 32, s + 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (MODE == 1) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j][0] += (float)af[cb][i][0] + (float)bfr[cb][j][1];
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cb][i], bfr[cb][j], acc[i][j], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + lr;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        C[(size_t)m * N + n] = acc[i][j][e];
      }
    }
}

// Schedule B: the barrier of k-step t sits before its LAST sub-step, once every wave has read the
// sub-step's fragments, and certifies stage t+1 (counted vmcnt leaves S-2 stages in flight): the
// first fragments of step t+1 are then read during step t's last MFMAs, so no LDS latency is exposed
// after a barrier, and the freed buffer (t % S) takes the DMA of stage t+S.  DMA = false: the same
// schedule on the prologue's stages only (MFMA + LDS alone).
template <int BM, int BN, int S, int WGM, int WGN, bool DMA>
__global__ void __launch_bounds__(64 * WGM * WGN) lab2_kernel(const short* __restrict__ A, const short* __restrict__ B,
                                                               float* __restrict__ C, int M, int N, int K, int tiles_n) {
  constexpr int NW = WGM * WGN;
  constexpr int BK = 64, SUB = BK / 16;
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 32, TN = WN / 32;
  constexpr int AB = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  constexpr int GPW = (BM + BN) / 8 / NW;
  static_assert(S >= 3, "schedule B keeps stage t+1 landed while t+2.. are in flight");
  __shared__ __attribute__((aligned(1024))) char smem[S * STAGE];
  const int bid = xcd_tile(blockIdx.x, gridDim.x);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = K / BK;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave % WGM, wn = wave / WGM;
  const int lr = lane & 31, lh = lane >> 5;
  const short* src[GPW];
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int grp = wave * GPW + j;
    const bool isA = grp < BM / 8;
    const int off = (isA ? grp : grp - BM / 8) * 1024 + lane * 16;
    const int r = off >> 7, slot = (off >> 4) & 7;
    const int sw = (slot ^ ((r >> 1) & 7)) << 3;
    src[j] = (isA ? A + (size_t)(m0 + r) * K : B + (size_t)(n0 + r) * K) + sw;
  }
  auto issue = [&](int t, int buf) {
#pragma unroll
    for (int j = 0; j < GPW; ++j)
      __builtin_amdgcn_global_load_lds((g_void*)(src[j] + t * BK), (l_void*)(smem + buf * STAGE + (wave * GPW + j) * 1024),
                                       16, 0, 0);
  };
  auto frag = [&](const char* img, int r0, int s) {
    const int r = r0 + (lane & 31);
    const int co = ((2 * s + (lane >> 5)) ^ ((r >> 1) & 7)) << 4;
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + co);
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // prologue: S stages (all buffers) with the DMA, S - 1 without
#pragma unroll
  for (int q = 0; q < (DMA ? S : S - 1); ++q)
    if (q < nk) issue(q, q);
  // stage 0 landed and visible (at most min(S, nk) - 1 stages still in flight)
  if (DMA) wait_dma_n<GPW>(min(S - 1, nk - 1));
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  bf16x8 af[2][TM], bfr[2][TN];
  {
    const char* SA = smem;
#pragma unroll
    for (int i = 0; i < TM; ++i) af[0][i] = frag(SA, wm * WM + i * 32, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[0][j] = frag(SA + AB, wn * WN + j * 32, 0);
  }
  for (int t = 0; t < nk; ++t) {
    const int cur = DMA ? t % S : t % (S - 1);
    const char* SA = smem + cur * STAGE;
#pragma unroll
    for (int s = 0; s < SUB; ++s) {
      const int cb = s & 1, nb = cb ^ 1;
      if (s + 1 < SUB) {
#pragma unroll
        for (int i = 0; i < TM; ++i) af[nb][i] = frag(SA, wm * WM + i * 32, s + 1);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[nb][j] = frag(SA + AB, wn * WN + j * 32, s + 1);
      } else if (t + 1 < nk) {
        // every wave has issued its reads of stage t (their data arrived: lgkmcnt(0)); stage t+1
        // landed (counted vmcnt) -> one barrier certifies both, then stage t+S goes into buffer t
        if (DMA) wait_dma_n<GPW>(min(S - 2, nk - 2 - t));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (DMA && t + S < nk) issue(t + S, t % S);
        const char* NA = smem + (DMA ? (t + 1) % S : (t + 1) % (S - 1)) * STAGE;
#pragma unroll
        for (int i = 0; i < TM; ++i) af[nb][i] = frag(NA, wm * WM + i * 32, 0);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[nb][j] = frag(NA + AB, wn * WN + j * 32, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cb][i], bfr[cb][j], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + lr;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        C[(size_t)m * N + n] = acc[i][j][e];
      }
    }
}

static unsigned short f2bf_host(float x) {
  unsigned u;
  std::memcpy(&u, &x, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}

struct Shape { const char* name; int M, N, K; };

template <int BM, int BN, int S, int WGM, int WGN, int MODE>
static void run(const Shape& sh, const short* A, const short* B, float* C, const std::vector<float>* ref) {
  if (sh.M % BM || sh.N % BN || sh.K % 64) return;
  const int tn = sh.N / BN, tm = sh.M / BM;
  const dim3 grid(tn * tm), blk(64 * WGM * WGN);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((lab_kernel<BM, BN, S, WGM, WGN, MODE>), grid, blk, 0, 0, A, B, C, sh.M, sh.N, sh.K, tn);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 50;
  CK(hipEventRecord(e0));
  for (int i = 0; i < R; ++i) hipLaunchKernelGGL((lab_kernel<BM, BN, S, WGM, WGN, MODE>), grid, blk, 0, 0, A, B, C, sh.M, sh.N, sh.K, tn);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / R;
  double err = -1;
  if (MODE == 0 && ref) {
    std::vector<float> h((size_t)sh.M * sh.N);
    CK(hipMemcpy(h.data(), C, h.size() * 4, hipMemcpyDeviceToHost));
    err = 0;
    double mx = 0;
    for (size_t i = 0; i < h.size(); i += 997) {
      err = fmax(err, fabs(h[i] - (*ref)[i]));
      mx = fmax(mx, fabs((*ref)[i]));
    }
    err /= mx;
  }
  printf("%-4s %5dx%4dx%4d  tile %3dx%3d S=%d waves=%2d mode=%d  %7.2f us  %6.0f TF  grid %d%s",
         sh.name, sh.M, sh.N, sh.K, BM, BN, S, WGM * WGN, MODE, us, 2.0 * sh.M * sh.N * sh.K / us / 1e6, tn * tm,
         err >= 0 ? "" : "\n");
  if (err >= 0) printf("  err %.1e\n", err);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int BM, int BN, int S, int WGM, int WGN, bool DMA>
static void run2(const Shape& sh, const short* A, const short* B, float* C, const std::vector<float>* ref) {
  if (sh.M % BM || sh.N % BN || sh.K % 64) return;
  const int tn = sh.N / BN, tm = sh.M / BM;
  const dim3 grid(tn * tm), blk(64 * WGM * WGN);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((lab2_kernel<BM, BN, S, WGM, WGN, DMA>), grid, blk, 0, 0, A, B, C, sh.M, sh.N, sh.K, tn);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 50;
  CK(hipEventRecord(e0));
  for (int i = 0; i < R; ++i) hipLaunchKernelGGL((lab2_kernel<BM, BN, S, WGM, WGN, DMA>), grid, blk, 0, 0, A, B, C, sh.M, sh.N, sh.K, tn);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / R;
  double err = -1;
  if (DMA && ref) {
    std::vector<float> h((size_t)sh.M * sh.N);
    CK(hipMemcpy(h.data(), C, h.size() * 4, hipMemcpyDeviceToHost));
    err = 0;
    double mx = 0;
    for (size_t i = 0; i < h.size(); i += 997) {
      err = fmax(err, fabs(h[i] - (*ref)[i]));
      mx = fmax(mx, fabs((*ref)[i]));
    }
    err /= mx;
  }
  printf("%-4s %5dx%4dx%4d  tile %3dx%3d S=%d waves=%2d schedB %s  %7.2f us  %6.0f TF  grid %d",
         sh.name, sh.M, sh.N, sh.K, BM, BN, S, WGM * WGN, DMA ? "full   " : "no-dma ", us,
         2.0 * sh.M * sh.N * sh.K / us / 1e6, tn * tm);
  if (err >= 0) printf("  err %.1e", err);
  printf("\n");
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int BM, int BN, int S, int WGM, int WGN>
static void modes2(const Shape& sh, const short* A, const short* B, float* C, const std::vector<float>* ref) {
  run2<BM, BN, S, WGM, WGN, true>(sh, A, B, C, ref);
  run2<BM, BN, S, WGM, WGN, false>(sh, A, B, C, nullptr);
}

template <int BM, int BN, int S, int WGM, int WGN>
static void modes(const Shape& sh, const short* A, const short* B, float* C, const std::vector<float>* ref) {
  run<BM, BN, S, WGM, WGN, 0>(sh, A, B, C, ref);
  run<BM, BN, S, WGM, WGN, 1>(sh, A, B, C, nullptr);
  run<BM, BN, S, WGM, WGN, 2>(sh, A, B, C, nullptr);
}

int main(int argc, char** argv) {
  // "wide": 128x256 / 256x128 tiles; F3h = one K-half of F3 on twice the rows, i.e. the per-workgroup
  // work of F3 split-K 2 on 256 workgroups (its split fix-up is not in the time)
  const bool wide = argc > 1 && !strcmp(argv[1], "wide");
  const Shape shapes_all[] = {{"F3", 8192, 512, 1920}, {"dc", 8192, 1920, 512}};
  const Shape shapes_wide[] = {{"F3", 8192, 512, 1920}, {"F3h", 16384, 512, 960}};
  const Shape* shapes = wide ? shapes_wide : shapes_all;
  for (int si = 0; si < 2; ++si) {
    const Shape& sh = shapes[si];
    const size_t na = (size_t)sh.M * sh.K, nbb = (size_t)sh.N * sh.K;
    std::vector<unsigned short> ha(na), hb(nbb);
    std::vector<float> fa(na), fb(nbb);
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 32768.f - 1.f; };
    for (size_t i = 0; i < na; ++i) { ha[i] = f2bf_host(rnd()); unsigned u = (unsigned)ha[i] << 16; std::memcpy(&fa[i], &u, 4); }
    for (size_t i = 0; i < nbb; ++i) { hb[i] = f2bf_host(rnd()); unsigned u = (unsigned)hb[i] << 16; std::memcpy(&fb[i], &u, 4); }
    std::vector<float> ref((size_t)sh.M * sh.N, 0.f);
    for (size_t i = 0; i < ref.size(); i += 997) {
      const size_t m = i / sh.N, n = i % sh.N;
      double acc = 0;
      for (int k = 0; k < sh.K; ++k) acc += (double)fa[m * sh.K + k] * fb[n * sh.K + k];
      ref[i] = (float)acc;
    }
    short *A, *B;
    float* C;
    CK(hipMalloc(&A, na * 2));
    CK(hipMalloc(&B, nbb * 2));
    CK(hipMalloc(&C, (size_t)sh.M * sh.N * 4));
    CK(hipMemcpy(A, ha.data(), na * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hb.data(), nbb * 2, hipMemcpyHostToDevice));
    if (wide) {
      modes<64, 128, 2, 2, 4>(sh, A, B, C, &ref);
      modes<128, 256, 2, 2, 4>(sh, A, B, C, &ref);
      modes<128, 256, 3, 2, 4>(sh, A, B, C, &ref);
      modes<128, 256, 2, 4, 4>(sh, A, B, C, &ref);
      modes<256, 128, 2, 4, 2>(sh, A, B, C, &ref);
      modes<256, 128, 2, 4, 4>(sh, A, B, C, &ref);
      CK(hipFree(A));
      CK(hipFree(B));
      CK(hipFree(C));
      continue;
    }
    modes2<128, 128, 3, 2, 2>(sh, A, B, C, &ref);
    modes2<128, 128, 4, 2, 2>(sh, A, B, C, &ref);
    modes2<128, 128, 3, 2, 4>(sh, A, B, C, &ref);
    modes2<128, 128, 4, 2, 4>(sh, A, B, C, &ref);
    modes2<64, 128, 3, 2, 4>(sh, A, B, C, &ref);
    modes2<128, 64, 3, 2, 2>(sh, A, B, C, &ref);
    modes2<128, 128, 4, 2, 2>(sh, A, B, C, &ref);
    modes<64, 128, 2, 2, 4>(sh, A, B, C, &ref);
    modes<64, 128, 3, 2, 4>(sh, A, B, C, &ref);
    modes<128, 128, 2, 2, 4>(sh, A, B, C, &ref);
    modes<128, 128, 3, 2, 4>(sh, A, B, C, &ref);
    modes<128, 128, 4, 2, 4>(sh, A, B, C, &ref);
    modes<128, 128, 4, 4, 4>(sh, A, B, C, &ref);
    modes<128, 128, 2, 2, 2>(sh, A, B, C, &ref);
    modes<128, 128, 3, 2, 2>(sh, A, B, C, &ref);
    modes<128, 128, 4, 2, 2>(sh, A, B, C, &ref);
    modes<128, 64, 3, 2, 2>(sh, A, B, C, &ref);
    modes<256, 128, 2, 2, 4>(sh, A, B, C, &ref);
    modes<256, 128, 3, 2, 4>(sh, A, B, C, &ref);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
  }
  return 0;
}
