// MFMA GEMM for the FiBiNET dense layers (gfx950 / CDNA4).
//
//   C[m][rC(n)] = sum_k A(m,k) * B(k,n) + bias[n] + beta * C[m][rC(n)]
//
// A is M x K, stored row-major ("N": A[m*lda+k]) or as its transpose ("T": A[k*lda+m]).
// B is K x N, stored as B^T ("T": B[n*ldb + rB(k)], a torch Linear weight) or plainly
// ("N": B[k*ldb + rB(n)]).  rB / rC are two-segment index remaps
// (i -> i + (i < seg ? off0 : off1)) used to skip the structurally-zero MLP input
// columns of FiBiNET (user field V_0 and the five pairs (0,j): DESIGN.md "zero columns")
// without materialising a compacted weight.
//
// Tiles: 256 threads = 4 waves in 2x2, each wave (BM/2)x(BN/2) made of 32x32 MFMA tiles.
//   fp32 path: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate), BK = 16.
//   bf16 path: v_mfma_f32_32x32x16_bf16 (operands rounded to bf16 on the LDS store,
//              f32 accumulate), BK = 32.
// LDS holds both operands K-contiguous ([row][k], rows padded to 80 B), double-buffered;
// global tiles are register-staged with 16-B loads (one barrier per K tile).
// Split-K (gridDim.z > 1) writes f32 partial slabs that gemm_splitk_reduce sums in slab
// order (deterministic).
#include "common.h"

struct Remap {
  int seg, off0, off1;
};
__device__ __forceinline__ int remap(const Remap& r, int i) { return i + (i < r.seg ? r.off0 : r.off1); }

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  int M, N, K, lda, ldb, ldc;
  Remap rB, rC;
  float beta;
  int kchunk;   // K range per split (multiple of BK)
  float* ws;    // split-K slabs [split][M][N]
};

template <bool BF16> struct GemmTraits;
template <> struct GemmTraits<false> { static constexpr int BK = 16; static constexpr int LDK = 20; typedef float T; };
template <> struct GemmTraits<true>  { static constexpr int BK = 32; static constexpr int LDK = 40; typedef short T; };

// Stage one (rows x BK) operand tile from global into registers.
// KC (K-contiguous): element (r,k) at P[(row0+r)*ld + map(k0+k)];  otherwise at P[(k0+k)*ld + map(row0+r)].
template <int ROWS, int BK, bool KC, bool MAPK>
struct TileLoader {
  static constexpr int CHUNKS = ROWS * BK / 4;
  static constexpr int PER_T = CHUNKS / 256;
  static_assert(CHUNKS % 256 == 0, "tile too small for 256 threads");
  f32x4 v[PER_T];

  __device__ __forceinline__ void load(const float* __restrict__ P, int ld, int row0, int nrows, int k0,
                                       int kend, const Remap& rm) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + 256 * i;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (KC) {
        const int r = c / (BK / 4), kk = (c % (BK / 4)) * 4;
        const int row = row0 + r, k = k0 + kk;
        if (row < nrows) {
          if (k + 3 < kend) {
            const int kg = MAPK ? remap(rm, k) : k;
            x = *reinterpret_cast<const f32x4*>(P + (size_t)row * ld + kg);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (k + e < kend) x[e] = P[(size_t)row * ld + (MAPK ? remap(rm, k + e) : k + e)];
          }
        }
      } else {
        const int kk = c / (ROWS / 4), r = (c % (ROWS / 4)) * 4;
        const int k = k0 + kk, row = row0 + r;
        if (k < kend) {
          if (row + 3 < nrows) {
            const int rg = MAPK ? remap(rm, row) : row;
            x = *reinterpret_cast<const f32x4*>(P + (size_t)k * ld + rg);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (row + e < nrows) x[e] = P[(size_t)k * ld + (MAPK ? remap(rm, row + e) : row + e)];
          }
        }
      }
      v[i] = x;
    }
  }

  template <typename T, int LDK>
  __device__ __forceinline__ void store(T* __restrict__ S) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (KC) {
        const int r = c / (BK / 4), kk = (c % (BK / 4)) * 4;
        if constexpr (sizeof(T) == 4) {
          *reinterpret_cast<f32x4*>(S + r * LDK + kk) = v[i];
        } else {
          bf16x4 b = {f2bf(v[i][0]), f2bf(v[i][1]), f2bf(v[i][2]), f2bf(v[i][3])};
          *reinterpret_cast<bf16x4*>(S + r * LDK + kk) = b;
        }
      } else {
        const int kk = c / (ROWS / 4), r = (c % (ROWS / 4)) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (sizeof(T) == 4) S[(r + e) * LDK + kk] = v[i][e];
          else S[(r + e) * LDK + kk] = f2bf(v[i][e]);
        }
      }
    }
  }
};

template <int BM, int BN, bool TA, bool TB, bool BF16>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs g) {
  typedef GemmTraits<BF16> Tr;
  typedef typename Tr::T T;
  constexpr int BK = Tr::BK, LDK = Tr::LDK;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  __shared__ __attribute__((aligned(16))) T sA[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) T sB[2][BN * LDK];

  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int kbeg = blockIdx.z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int ntiles = (kend - kbeg + BK - 1) / BK;
  const Remap none = {0x7fffffff, 0, 0};

  TileLoader<BM, BK, !TA, false> la;
  TileLoader<BN, BK, TB, true> lb;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave & 1, wn = wave >> 1;
  const int lr = lane & 31, lh = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  if (ntiles > 0) {
    la.load(g.A, g.lda, m0, g.M, kbeg, kend, none);
    lb.load(g.B, g.ldb, n0, g.N, kbeg, kend, g.rB);
    la.template store<T, LDK>(sA[0]);
    lb.template store<T, LDK>(sB[0]);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const bool more = (t + 1) < ntiles;
    if (more) {
      const int k0 = kbeg + (t + 1) * BK;
      la.load(g.A, g.lda, m0, g.M, k0, kend, none);
      lb.load(g.B, g.ldb, n0, g.N, k0, kend, g.rB);
    }
    const T* A_ = sA[buf];
    const T* B_ = sB[buf];
    if constexpr (!BF16) {
      // k permutation: lane half h covers k in [8h, 8h+8); step s uses k = 8h + s for A and B.
      f32x4 af[TM][2], bfr[TN][2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* p = A_ + (wm * WM + i * 32 + lr) * LDK + lh * 8;
        af[i][0] = *reinterpret_cast<const f32x4*>(p);
        af[i][1] = *reinterpret_cast<const f32x4*>(p + 4);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* p = B_ + (wn * WN + j * 32 + lr) * LDK + lh * 8;
        bfr[j][0] = *reinterpret_cast<const f32x4*>(p);
        bfr[j][1] = *reinterpret_cast<const f32x4*>(p + 4);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s >> 2][s & 3], bfr[j][s >> 2][s & 3],
                                                             acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(A_ + (wm * WM + i * 32 + lr) * LDK + s * 16 + lh * 8);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(B_ + (wn * WN + j * 32 + lr) * LDK + s * 16 + lh * 8);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) {
      la.template store<T, LDK>(sA[buf ^ 1]);
      lb.template store<T, LDK>(sB[buf ^ 1]);
    }
    __syncthreads();
  }

  // epilogue: C/D map of the 32x32 MFMA tile: col = lane&31, row = (e&3) + 8*(e>>2) + 4*(lane>>5)
  const bool split = gridDim.z > 1;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + lr;
      if (n >= g.N) continue;
      const float bv = (!split && g.bias) ? g.bias[n] : 0.f;
      const int nc = remap(g.rC, n);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (m >= g.M) continue;
        if (split) {
          g.ws[((size_t)blockIdx.z * g.M + m) * g.N + n] = acc[i][j][e];
        } else {
          float* cp = g.C + (size_t)m * g.ldc + nc;
          float v = acc[i][j][e] + bv;
          if (g.beta != 0.f) v += g.beta * *cp;
          *cp = v;
        }
      }
    }
}

__global__ void gemm_splitk_reduce(GemmArgs g, int nsplit) {
  const size_t total = (size_t)g.M * g.N;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(idx / g.N), n = (int)(idx % g.N);
    float s = 0.f;
    for (int z = 0; z < nsplit; ++z) s += g.ws[(size_t)z * total + idx];
    if (g.bias) s += g.bias[n];
    float* cp = g.C + (size_t)m * g.ldc + remap(g.rC, n);
    if (g.beta != 0.f) s += g.beta * *cp;
    *cp = s;
  }
}

template <int BM, int BN, bool TA, bool TB, bool BF16>
static void launch_tile(const GemmArgs& g, int nsplit, hipStream_t st) {
  dim3 grid(fbn_cdiv(g.N, BN), fbn_cdiv(g.M, BM), nsplit);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, TA, TB, BF16>), grid, dim3(256), 0, st, g);
}

template <bool TA, bool TB, bool BF16>
static void launch_sel(const GemmArgs& g, int nsplit, hipStream_t st) {
  if (g.N <= 64 || g.M <= 64) launch_tile<64, 64, TA, TB, BF16>(g, nsplit, st);
  else launch_tile<128, 128, TA, TB, BF16>(g, nsplit, st);
}

// Host-side split-K choice: fill ~2 waves of the 256-CU chip for reduction-heavy (wgrad) shapes.
static int choose_split(int M, int N, int K, int bk) {
  const int bm = (N <= 64 || M <= 64) ? 64 : 128;
  const int tiles = fbn_cdiv(M, bm) * fbn_cdiv(N, bm);
  int s = 1;
  while (tiles * s < 512 && K / (s * 2) >= 8 * bk && s < 64) s *= 2;
  return s;
}

extern "C" size_t fbn_gemm_workspace_size(int M, int N, int K, int bf16) {
  const int bk = bf16 ? 32 : 16;
  const int s = choose_split(M, N, K, bk);
  return s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
}

extern "C" int fbn_gemm(const float* A, const float* B, float* C, const float* bias, int M, int N, int K,
                        int lda, int ldb, int ldc, int transA, int transB, int rB_seg, int rB_off0,
                        int rB_off1, int rC_seg, int rC_off0, int rC_off1, float beta, int bf16,
                        float* ws, size_t ws_bytes, void* stream) {
  if (M <= 0 || N <= 0) return FBN_OK;
  if (!A || !B || !C) { fbn_set_error("fbn_gemm: null operand"); return FBN_ERR_ARG; }
  // 16-B vector loads along the contiguous dimension of every operand
  if ((lda & 3) || (ldb & 3) || ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || (rB_off0 & 3) || (rB_off1 & 3) ||
      (rB_seg != 0x7fffffff && (rB_seg & 3))) {
    fbn_set_error("fbn_gemm: operands must be 16-byte aligned with ld % 4 == 0");
    return FBN_ERR_ARG;
  }
  GemmArgs g;
  g.A = A; g.B = B; g.C = C; g.bias = bias;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.rB = {rB_seg, rB_off0, rB_off1};
  g.rC = {rC_seg, rC_off0, rC_off1};
  g.beta = beta;
  const int bk = bf16 ? 32 : 16;
  int nsplit = choose_split(M, N, K, bk);
  if (nsplit > 1 && (!ws || ws_bytes < (size_t)nsplit * M * N * sizeof(float))) nsplit = 1;
  int per = fbn_cdiv(K, nsplit);
  per = fbn_cdiv(per, bk) * bk;
  nsplit = K > 0 ? fbn_cdiv(K, per) : 1;
  g.kchunk = K > 0 ? per : 0;
  g.ws = ws;
  hipStream_t st = (hipStream_t)stream;
  const int key = (transA ? 4 : 0) | (transB ? 2 : 0) | (bf16 ? 1 : 0);
  switch (key) {
    case 0: launch_sel<false, false, false>(g, nsplit, st); break;
    case 1: launch_sel<false, false, true>(g, nsplit, st); break;
    case 2: launch_sel<false, true, false>(g, nsplit, st); break;
    case 3: launch_sel<false, true, true>(g, nsplit, st); break;
    case 4: launch_sel<true, false, false>(g, nsplit, st); break;
    case 5: launch_sel<true, false, true>(g, nsplit, st); break;
    case 6: launch_sel<true, true, false>(g, nsplit, st); break;
    default: launch_sel<true, true, true>(g, nsplit, st); break;
  }
  FBN_CHECK_LAUNCH();
  if (nsplit > 1) {
    const size_t total = (size_t)M * N;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, st, g, nsplit);
    FBN_CHECK_LAUNCH();
  }
  return FBN_OK;
}
