// Fused bilinear interaction, "all" branch, bf16 mode (model_fibinet.py:60-79,89):
// the W contraction on MFMA and the pair products in its epilogue, one launch each way.
//
//   forward:  U_f = V_f W (f = 1..5),  p_ij = V_i (.) U_j (1 <= i < j <= 5)  -> c[:, 5d:] (bf16)
//   backward: dU_j = sum_{i<j} dp_ij (.) V_i
//             dV_i = dc_{V_i} + sum_{j>i} dp_ij (.) U_j + dU_i W^T             -> dV (f32), dU (bf16)
//
// The unfused path (gemm U = V W -> pairs_fwd; pairs_bwd -> gemm dV += dU W^T) writes U and
// re-reads it, and reads / writes dV twice: 4 launches and ~110 MB more HBM traffic per step at C3.
// Here U never leaves the chip: the backward recomputes it (1.3 GFLOP of MFMA) instead of storing
// 21 MB and reading it back.
//
// Tile: 16 samples per workgroup (512 workgroups at B = 8192: two per CU, so one block's loads
// overlap the other's MFMAs), D/32 waves.  The MFMA runs TRANSPOSED -- U^T[n][s] =
// sum_k W^T[n][k] V[s][k] with v_mfma_f32_16x16x32_bf16 (A = W^T rows, B = the V tile's rows) --
// so a lane's accumulator holds, for its sample s = lane & 15, 4 consecutive n (rows
// 4(lane>>4) + i of the 16x16 block): every pair product is a 4-wide vector and every store 8
// (bf16) or 16 (f32) bytes, four lanes covering 16 contiguous n of a row.  Wave w owns n in
// [32w, 32w+32) (two 16-row blocks) for all 5 fields.  (A 32-sample tile on 32x32x16 MFMAs gave
// 256 workgroups, one wave per SIMD: 14 / 52 us fwd / bwd against 21 / 35 unfused.)
// LDS: the V tile [5 fields x 16 samples][D] and one weight image [D][D], bf16, rows of D/8 16-B
// chunks XOR-swizzled by the row (chunk c of row r at c ^ (r % (D/8))) so the 16-lane groups of a
// fragment read hit distinct bank quads.  In the backward, dU is written over the V tile (each
// lane overwrites exactly the elements it alone read) and becomes the second MFMA's B operand;
// that MFMA (A = W rows, K = n) accumulates straight onto the elementwise part of dV.
#include "common.h"
#include <algorithm>

namespace {

constexpr int TS = 16;   // samples per workgroup

template <int D>
__device__ __forceinline__ int swz(int r, int k) {   // element offset of (row r, k) in a swizzled image
  constexpr int CH = D / 8;
  return r * D + ((((k >> 3) ^ (r % CH))) << 3) + (k & 7);
}

// threads per workgroup and 16-row blocks of n per wave: D/32 waves of two blocks each; at D = 16
// one wave with one block
template <int D> constexpr int nthreads() { return D >= 32 ? 2 * D : 64; }
template <int D> constexpr int row_blocks() { return D >= 32 ? 2 : 1; }

// 16-B chunk loads of a [D][D] bf16 image into the swizzled LDS image.  Every load of a thread is
// issued before any LDS store (register-staged batch): one HBM/L2 round trip per stage, not one
// per chunk.
template <int D, int NT>
struct WStage {
  static constexpr int CH = D / 8, TOT = D * CH, N = (TOT + NT - 1) / NT;
  bf16x8 v[N];
  __device__ __forceinline__ void load(const short* __restrict__ src, int tid) {
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (TOT % NT == 0 || tid + j * NT < TOT) v[j] = *reinterpret_cast<const bf16x8*>(src + (size_t)(tid + j * NT) * 8);
  }
  __device__ __forceinline__ void store(short* __restrict__ img, int tid) const {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int i = tid + j * NT, r = i / CH, c = i % CH;
      if (TOT % NT == 0 || i < TOT) *reinterpret_cast<bf16x8*>(img + swz<D>(r, c * 8)) = v[j];
    }
  }
};
template <int D, int NT>
__device__ __forceinline__ void stage_w(short* __restrict__ img, const short* __restrict__ src, int tid) {
  WStage<D, NT> w;
  w.load(src, tid);
  w.store(img, tid);
}

// the V tile: LDS row f*32 + s <- V16[b0 + s][f] (memory order s*5 + f: one contiguous block)
template <int D, int NT>
__device__ __forceinline__ void stage_v(short* __restrict__ img, const short* __restrict__ V16, int b0, int ns,
                                        int tid) {
  constexpr int CH = D / 8, TOT = TS * 5 * CH, N = (TOT + NT - 1) / NT;
  const short* src = V16 + (size_t)b0 * 5 * D;
  bf16x8 v[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int i = tid + j * NT, m = i / CH;          // m = s*5 + f
    v[j] = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    if ((TOT % NT == 0 || i < TOT) && m / 5 < ns) v[j] = *reinterpret_cast<const bf16x8*>(src + (size_t)i * 8);
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int i = tid + j * NT, m = i / CH, c = i % CH;
    if (TOT % NT == 0 || i < TOT) *reinterpret_cast<bf16x8*>(img + swz<D>((m % 5) * TS + m / 5, c * 8)) = v[j];
  }
}

template <int D>
__device__ __forceinline__ bf16x8 frag(const short* img, int row, int k) {
  return *reinterpret_cast<const bf16x8*>(img + swz<D>(row, k));
}

// acc[rb][f][i] += sum_k A[n][k] * Bt[f*16 + s][k], n = 32w + 16rb + 4(lane>>4) + i, s = lane & 15
// (D = 16: K = 16, one v_mfma_f32_16x16x16_bf16 per field, 4 k per lane)
template <int D>
__device__ __forceinline__ void mfma_5(f32x4 (&acc)[row_blocks<D>()][5], const short* A, const short* Bt, int w,
                                       int lane) {
  const int lr = lane & 15, lq = lane >> 4;
  if constexpr (D == 16) {
    const bf16x4 a = *reinterpret_cast<const bf16x4*>(A + swz<D>(lr, 4 * lq));
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      const bf16x4 b = *reinterpret_cast<const bf16x4*>(Bt + swz<D>(f * TS + lr, 4 * lq));
      acc[0][f] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, acc[0][f], 0, 0, 0);
    }
    return;
  }
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    bf16x8 b[5];
#pragma unroll
    for (int f = 0; f < 5; ++f) b[f] = frag<D>(Bt, f * TS + lr, 32 * ks + 8 * lq);
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const bf16x8 a = frag<D>(A, 32 * w + 16 * rb + lr, 32 * ks + 8 * lq);
#pragma unroll
      for (int f = 0; f < 5; ++f) acc[rb][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[f], acc[rb][f], 0, 0, 0);
    }
  }
}

__device__ __forceinline__ f32x4 ld_bf4(const short* p) {
  const bf16x4 t = *reinterpret_cast<const bf16x4*>(p);
  return (f32x4){bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3])};
}
__device__ __forceinline__ bf16x4 to_bf4(const f32x4& v) { return (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])}; }

constexpr int PI[10] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
constexpr int PJ[10] = {1, 2, 3, 4, 2, 3, 4, 3, 4, 4};

template <int D>
__global__ void __launch_bounds__(nthreads<D>()) bilinear_fwd_kernel(const short* __restrict__ V16,
                                                                    const short* __restrict__ WT16,
                                                                    short* __restrict__ c, int B, int ldc) {
  FBN_MAIN_PRIO();
  constexpr int NT = nthreads<D>(), RB = row_blocks<D>();
  __shared__ __attribute__((aligned(16))) short sV[5 * TS * D];
  __shared__ __attribute__((aligned(16))) short sW[D * D];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = blockIdx.x * TS, ns = min(TS, B - b0);
  stage_v<D, NT>(sV, V16, b0, ns, tid);
  stage_w<D, NT>(sW, WT16, tid);
  __syncthreads();
  f32x4 acc[RB][5];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int f = 0; f < 5; ++f) acc[rb][f] = (f32x4){0.f, 0.f, 0.f, 0.f};
  mfma_5<D>(acc, sW, sV, w, lane);          // acc[rb][f] = U_f^T[n0..n0+3][s]
  const int s = lane & 15, lq = lane >> 4;
  if (s >= ns) return;
  short* crow = c + (size_t)(b0 + s) * ldc + 5 * D;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int n0 = 32 * w + 16 * rb + 4 * lq;
    f32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = ld_bf4(sV + swz<D>(i * TS + s, n0));
#pragma unroll
    for (int k = 0; k < 10; ++k) *reinterpret_cast<bf16x4*>(crow + k * D + n0) = to_bf4(v[PI[k]] * acc[rb][PJ[k]]);
  }
}

// dc row segment (4 consecutive values) as f32: DC16 = dc is bf16 (fbn_gemm_bf16out) or f32
template <bool DC16>
__device__ __forceinline__ f32x4 ld_dc4(const void* __restrict__ row, int off) {
  if constexpr (DC16) return ld_bf4(reinterpret_cast<const short*>(row) + off);
  else return *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(row) + off);
}

template <int D, bool DC16>
__global__ void __launch_bounds__(nthreads<D>(), 2) bilinear_bwd_kernel(const void* __restrict__ dc, int ldc,
                                                                       const short* __restrict__ V16,
                                                                       const short* __restrict__ WT16,
                                                                       const short* __restrict__ W16,
                                                                       float* __restrict__ dV,
                                                                       short* __restrict__ dU16, int B) {
  FBN_MAIN_PRIO();
  constexpr int NT = nthreads<D>(), RB = row_blocks<D>();
  __shared__ __attribute__((aligned(16))) short sV[5 * TS * D];   // V tile, then dU tile
  __shared__ __attribute__((aligned(16))) short sW[D * D];        // W^T image, then W image
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = blockIdx.x * TS, ns = min(TS, B - b0);
  stage_v<D, NT>(sV, V16, b0, ns, tid);
  stage_w<D, NT>(sW, WT16, tid);
  __syncthreads();
  WStage<D, NT> wnext;
  wnext.load(W16, tid);                     // the W image for dV += dU W^T: in flight meanwhile
  f32x4 acc[RB][5];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int f = 0; f < 5; ++f) acc[rb][f] = (f32x4){0.f, 0.f, 0.f, 0.f};
  mfma_5<D>(acc, sW, sV, w, lane);          // acc = U^T (recomputed: never stored)
  __syncthreads();                          // no wave still reads the V tile: dU may overwrite it
  const int s = lane & 15, lq = lane >> 4;
  const bool live = s < ns;
  const char* dcr = reinterpret_cast<const char*>(dc) + (size_t)(b0 + (live ? s : 0)) * ldc * (DC16 ? 2 : 4);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int n0 = 32 * w + 16 * rb + 4 * lq;
    f32x4 v[5], gv[5], gu[5];
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      v[f] = ld_bf4(sV + swz<D>(f * TS + s, n0));
      gv[f] = live ? ld_dc4<DC16>(dcr, f * D + n0) : (f32x4){0.f, 0.f, 0.f, 0.f};
      gu[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const f32x4 gp = live ? ld_dc4<DC16>(dcr, (5 + k) * D + n0) : (f32x4){0.f, 0.f, 0.f, 0.f};
      gv[PI[k]] += gp * acc[rb][PJ[k]];
      gu[PJ[k]] += gp * v[PI[k]];
    }
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      const bf16x4 t = to_bf4(gu[f]);
      // this lane alone read V at these (f, s, n0..n0+3): overwrite them with dU (the B operand)
      *reinterpret_cast<bf16x4*>(sV + swz<D>(f * TS + s, n0)) = t;
      if (live) *reinterpret_cast<bf16x4*>(dU16 + ((size_t)(b0 + s) * 5 + f) * D + n0) = t;
    }
#pragma unroll
    for (int f = 0; f < 5; ++f) acc[rb][f] = gv[f];
  }
  __syncthreads();                          // every wave is done with the W^T image and the dU tile is whole
  wnext.store(sW, tid);
  __syncthreads();
  mfma_5<D>(acc, sW, sV, w, lane);          // acc = dV^T = elementwise part + W dU^T
  if (!live) return;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int k0 = 32 * w + 16 * rb + 4 * lq;
#pragma unroll
    for (int f = 0; f < 5; ++f) *reinterpret_cast<f32x4*>(dV + ((size_t)(b0 + s) * 5 + f) * D + k0) = acc[rb][f];
  }
}

}  // namespace

extern "C" int fbn_bilinear_supported(int D) { return D == 16 || D == 32 || D == 64 || D == 128; }

extern "C" int fbn_bilinear_fwd(const short* V16, const short* WT16, short* c, int B, int D, int ldc, void* stream) {
  if (B <= 0) return FBN_OK;
  if (!V16 || !WT16 || !c || (ldc & 3) || ((uintptr_t)V16 & 15) || ((uintptr_t)WT16 & 15) || ((uintptr_t)c & 7)) {
    fbn_set_error("fbn_bilinear_fwd: bf16 V, W^T, c required; 16-B aligned V / W^T, 8-B aligned c, ldc % 4 == 0");
    return FBN_ERR_ARG;
  }
  const dim3 grid((unsigned)((B + TS - 1) / TS));
  hipStream_t st = (hipStream_t)stream;
  switch (D) {
    case 128: fbn_launch(bilinear_fwd_kernel<128>, grid, dim3(256), 0, st, V16, WT16, c, B, ldc); break;
    case 64: fbn_launch(bilinear_fwd_kernel<64>, grid, dim3(128), 0, st, V16, WT16, c, B, ldc); break;
    case 32: fbn_launch(bilinear_fwd_kernel<32>, grid, dim3(64), 0, st, V16, WT16, c, B, ldc); break;
    case 16: fbn_launch(bilinear_fwd_kernel<16>, grid, dim3(64), 0, st, V16, WT16, c, B, ldc); break;
    default: fbn_set_error("fbn_bilinear_fwd: D must be 16, 32, 64 or 128"); return FBN_ERR_UNSUPPORTED;
  }
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_bilinear_bwd(const void* dc, int ldc, int dc_bf16, const short* V16, const short* WT16,
                                const short* W16, float* dV, short* dU16, int B, int D, void* stream) {
  if (B <= 0) return FBN_OK;
  if (!dc || !V16 || !WT16 || !W16 || !dV || !dU16 || (ldc & 3) || ((uintptr_t)dc & 7) || ((uintptr_t)dV & 15) ||
      ((uintptr_t)V16 & 15) || ((uintptr_t)WT16 & 15) || ((uintptr_t)W16 & 15) || ((uintptr_t)dU16 & 7)) {
    fbn_set_error("fbn_bilinear_bwd: all operands required and aligned (16 B; dc, dU16 8 B), ldc % 4 == 0");
    return FBN_ERR_ARG;
  }
  const dim3 grid((unsigned)((B + TS - 1) / TS));
  hipStream_t st = (hipStream_t)stream;
  if (!dc_bf16 && ((uintptr_t)dc & 15)) { fbn_set_error("fbn_bilinear_bwd: f32 dc must be 16-B aligned"); return FBN_ERR_ARG; }
#define FBN_BILINEAR_BWD(DD, NTH)                                                                              \
  if (dc_bf16)                                                                                               \
    fbn_launch((bilinear_bwd_kernel<DD, true>), grid, dim3(NTH), 0, st, dc, ldc, V16, WT16, W16, dV, dU16, B); \
  else                                                                                                       \
    fbn_launch((bilinear_bwd_kernel<DD, false>), grid, dim3(NTH), 0, st, dc, ldc, V16, WT16, W16, dV, dU16, B)
  switch (D) {
    case 128: FBN_BILINEAR_BWD(128, 256); break;
    case 64: FBN_BILINEAR_BWD(64, 128); break;
    case 32: FBN_BILINEAR_BWD(32, 64); break;
    case 16: FBN_BILINEAR_BWD(16, 64); break;
    default: fbn_set_error("fbn_bilinear_bwd: D must be 16, 32, 64 or 128"); return FBN_ERR_UNSUPPORTED;
  }
#undef FBN_BILINEAR_BWD
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}
