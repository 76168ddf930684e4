// LDS-DMA feed-rate probe (tuning aid for gemm.hip): how many bytes per CU per second can
// global_load_lds_dwordx4 move from L2-resident or HBM-resident data into LDS, as a function of
// waves per workgroup, workgroups per CU and stages in flight?  No compute: each wave issues its
// share of a stage's 1-KiB DMA instructions, waits until at most (S-1) stages are outstanding
// (counted vmcnt), and a raw s_barrier closes the stage, as gemm_dma16_kernel does.
//
//   hipcc --offload-arch=gfx950 -O3 -o dma_probe tools/dma_probe.hip && ./dma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((address_space(1))) void g_void;
typedef __attribute__((address_space(3))) void l_void;

template <int NW, int S, int KB>   // waves, stages in flight + 1, KiB per stage
__global__ void __launch_bounds__(64 * NW) dma_kernel(const char* __restrict__ src, size_t region, int iters,
                                                      size_t wrap, int* sink) {
  constexpr int GPW = KB / NW;     // 1-KiB DMA instructions per wave per stage
  static_assert(KB % NW == 0, "stage / wave mismatch");
  __shared__ __attribute__((aligned(1024))) char smem[S * KB * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t base = ((size_t)blockIdx.x * region) % wrap;
  auto issue = [&](int t) {
#pragma unroll
    for (int j = 0; j < GPW; ++j) {
      const size_t off = (base + ((size_t)t * KB + wave * GPW + j) * 1024 + lane * 16) % wrap;
      __builtin_amdgcn_global_load_lds((g_void*)(src + off), (l_void*)(smem + (t % S) * KB * 1024 + (wave * GPW + j) * 1024),
                                       16, 0, 0);
    }
  };
  for (int q = 0; q < S - 1; ++q) issue(q);
  for (int t = 0; t < iters; ++t) {
    if (S >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 2) * GPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + S - 1 < iters) issue(t + S - 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && smem[lane] == 123 && smem[1000] == 45) sink[0] = 1;
}

template <int NW, int S, int KB>
static void run(const char* name, const char* src, size_t bytes, int blocks, int iters, size_t wrap, int* sink) {
  const size_t region = (size_t)iters * KB * 1024;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(a);
    for (int k = 0; k < 10; ++k)
      hipLaunchKernelGGL((dma_kernel<NW, S, KB>), dim3(blocks), dim3(64 * NW), 0, 0, src, region, iters, wrap, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
  }
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / 10;
  const double total = (double)blocks * region;
  printf("%-10s waves %2d stages %d KiB/stage %3d blocks %4d (%.2f/CU) wrap %6.1f MB: %7.1f us  %6.2f TB/s  %6.1f GB/s/CU\n",
         name, NW, S, KB, blocks, blocks / 256.0, wrap / 1e6, us, total / us / 1e6, total / us / 1e3 / 256);
  (void)bytes;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  char* src;
  int* sink;
  hipMalloc(&src, bytes);
  hipMalloc(&sink, 4);
  hipMemset(src, 1, bytes);
  const size_t L2 = (size_t)2 << 20, HBM = bytes;
  // the GEMM F3 shape moves 960 KiB per CU (128x128 tile, K = 1920): iters x KiB/stage = 960
  for (size_t wrap : {L2, HBM}) {
    const char* nm = wrap == L2 ? "L2-res" : "HBM";
    run<4, 2, 32>(nm, src, bytes, 256, 30, wrap, sink);
    run<4, 3, 32>(nm, src, bytes, 256, 30, wrap, sink);
    run<4, 4, 32>(nm, src, bytes, 256, 30, wrap, sink);
    run<8, 2, 32>(nm, src, bytes, 256, 30, wrap, sink);
    run<8, 4, 32>(nm, src, bytes, 256, 30, wrap, sink);
    run<16, 2, 32>(nm, src, bytes, 256, 30, wrap, sink);
    run<16, 4, 32>(nm, src, bytes, 256, 30, wrap, sink);
    run<8, 2, 24>(nm, src, bytes, 512, 40, wrap, sink);     // 64x128 tiles, 2 per CU
    run<8, 3, 24>(nm, src, bytes, 512, 40, wrap, sink);
    run<8, 2, 16>(nm, src, bytes, 1024, 60, wrap, sink);    // 64x64 tiles, 4 per CU
    run<4, 2, 16>(nm, src, bytes, 1024, 60, wrap, sink);
    run<8, 4, 16>(nm, src, bytes, 512, 60, wrap, sink);
  }
  hipFree(src);
  hipFree(sink);
  return 0;
}
