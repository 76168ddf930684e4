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
//   fp32 path: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate), BK = 32.
//   bf16 path: v_mfma_f32_32x32x16_bf16 (operands rounded to bf16 on the LDS store,
//              f32 accumulate), BK = 64.
// LDS holds both operands K-contiguous ([row][k], rows padded to 144 B so the 16-lane
// groups of ds_read_b128 hit 16 distinct bank quads), double-buffered; global tiles are
// register-staged with 16-B loads one tile ahead (one barrier per K tile).  Operands whose
// contiguous dimension is M or N (the wgrad "T" A operand and the "N" B operand) are
// loaded as 4x4 micro-blocks and transposed in registers, so every LDS store is a
// 4-element k-run (ds_write_b64 / b128).
// The host picks the tile (64x64 .. 128x128) and a split-K factor so that a launch has
// >= 4 workgroups per CU: these GEMMs are short (K <= 2688 or M,N <= 512) and a single
// workgroup per CU cannot hide the global-load latency behind its MFMAs.
// Workgroups are remapped so that consecutive tiles (which share an A row panel) run on
// one XCD and hit its L2 (MI355X: round-robin dispatch over 8 XCDs).
// Split-K (gridDim.z > 1) writes f32 partial slabs that gemm_splitk_reduce sums in slab
// order (deterministic).
#include "common.h"
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <cstdio>

#ifndef FBN_DMA_STAGES
#define FBN_DMA_STAGES 2
#endif

struct Remap {
  int seg, off0, off1;
};
__device__ __forceinline__ int remap(const Remap& r, int i) { return i + (i < r.seg ? r.off0 : r.off1); }

struct GemmArgs {
  const void* A;   // float or bf16 (see a16 / b16)
  const void* B;
  float* C;
  const float* bias;
  int M, N, K, lda, ldb, ldc;
  Remap rB, rC;
  float beta;
  int kchunk;   // K range per split (multiple of BK)
  float* ws;    // split-K slabs [split][M][N]
  float* stats; // optional [ceil(M/BM)][N][2]: per-tile column (sum, M2 about the tile mean) of C
  // split operands (LDS-DMA kernel only): a k-contiguous A is [A | A2] along K (A(m,k) for k >= kseg
  // at A2[m*lda2 + k - kseg]); a k-major B is [B | B2] along N (B(k,n) for n >= nseg at
  // B2[k*ldb2 + n - nseg]).  kseg / nseg are multiples of the tile and BK; INT_MAX = unused.
  const void* A2;
  const void* B2;
  int lda2, kseg, ldb2, nseg;
  // split-bf16 x3 (LDS-DMA kernel, S3 instantiations): K = 3 s3k0 in three K-segments; segment s of A
  // reads its hi image (s < 2) or its lo image (s == 2, s3_loa elements past hi), of B hi (s != 1)
  // or lo (s == 1, s3_lob past hi): C = A_hi B_hi + A_hi B_lo + A_lo B_hi from two images each
  int s3k0;
  long long s3_loa, s3_lob;
  int c16;      // C is bf16 (short*, ldc in elements): split == 1, no stats / beta (fbn_gemm_bf16out)
  // BatchNorm backward first pass fused into a dgrad epilogue (fbn_gemm_bn_bwd_part): C is the
  // gradient G wrt the BN output's activation; per row chunk of bnb_rpc rows (one wave's rows) and
  // column: part[chunk][0][n] = sum dy, [1][n] = sum (x - mean) dy, [2][n] = 0, dy = (act > 0) * G * scale
  const short* bnb_hact16;   // [M][N] bf16 activation image (its sign is the ReLU / dropout mask)
  const float* bnb_xpre;     // [M][N] BN input
  const float* bnb_mean;     // [N]
  float bnb_scale;
  double* bnb_part;          // null = off
  int bnb_rpc;
};

template <bool BF16> struct GemmTraits;
template <> struct GemmTraits<false> { static constexpr int BK = 32; static constexpr int LDK = 36; typedef float T; };
template <> struct GemmTraits<true>  { static constexpr int BK = 64; static constexpr int LDK = 72; typedef short T; };

template <typename T>
__device__ __forceinline__ void st4(T* dst, float a, float b, float c, float d) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<f32x4*>(dst) = (f32x4){a, b, c, d};
  } else {
    *reinterpret_cast<bf16x4*>(dst) = (bf16x4){f2bf(a), f2bf(b), f2bf(c), f2bf(d)};
  }
}

// Stage one (ROWS x BK) operand tile from global into registers.
// KC (K-contiguous): element (r,k) at P[(row0+r)*ld + map(k0+k)]; chunks of 4 k per lane.
// !KC: element (r,k) at P[(k0+k)*ld + map(row0+r)]; 4x4 micro-blocks (4 k x 4 rows) per lane.
// MAP: apply the remap to the contiguous index (k for KC, the row index otherwise).
template <int ROWS, int BK, bool KC, bool MAP>
struct TileLoader {
  static constexpr int UNITS = KC ? ROWS * BK / 4 : ROWS * BK / 16;
  static constexpr int PER_T = (UNITS + 255) / 256;     // UNITS < 256: some lanes idle
  static constexpr int NV = KC ? PER_T : PER_T * 4;
  static_assert(UNITS % 256 == 0 || UNITS < 256, "tile / thread mismatch");
  f32x4 v[NV];

  __device__ __forceinline__ f32x4 ld4(const float* __restrict__ P, int ld, int row, int nrows, int k, int kend,
                                       const Remap& rm) const {
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (KC) {
      if (row < nrows) {
        if (k + 3 < kend) {
          x = *reinterpret_cast<const f32x4*>(P + (size_t)row * ld + (MAP ? remap(rm, k) : k));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (k + e < kend) x[e] = P[(size_t)row * ld + (MAP ? remap(rm, k + e) : k + e)];
        }
      }
    } else {
      if (k < kend) {
        if (row + 3 < nrows) {
          x = *reinterpret_cast<const f32x4*>(P + (size_t)k * ld + (MAP ? remap(rm, row) : row));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (row + e < nrows) x[e] = P[(size_t)k * ld + (MAP ? remap(rm, row + e) : row + e)];
        }
      }
    }
    return x;
  }

  __device__ __forceinline__ void load(const float* __restrict__ P, int ld, int row0, int nrows, int k0, int kend,
                                       const Remap& rm) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (UNITS < 256 && c >= UNITS) continue;
      if (KC) {
        const int r = c / (BK / 4), kk = (c % (BK / 4)) * 4;
        v[i] = ld4(P, ld, row0 + r, nrows, k0 + kk, kend, rm);
      } else {
        const int r = (c % (ROWS / 4)) * 4, kk = (c / (ROWS / 4)) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i * 4 + j] = ld4(P, ld, row0 + r, nrows, k0 + kk + j, kend, rm);
      }
    }
  }

  template <typename T, int LDK>
  __device__ __forceinline__ void store(T* __restrict__ S) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (UNITS < 256 && c >= UNITS) continue;
      if (KC) {
        const int r = c / (BK / 4), kk = (c % (BK / 4)) * 4;
        st4<T>(S + r * LDK + kk, v[i][0], v[i][1], v[i][2], v[i][3]);
      } else {
        const int r = (c % (ROWS / 4)) * 4, kk = (c / (ROWS / 4)) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e)   // row r+e gets the 4-k run (kk..kk+3): register transpose
          st4<T>(S + (r + e) * LDK + kk, v[i * 4 + 0][e], v[i * 4 + 1][e], v[i * 4 + 2][e], v[i * 4 + 3][e]);
      }
    }
  }

  // split-bf16: x = hi + lo with hi = bf16(x), lo = bf16(x - hi); the hi tile at S, the lo tile at
  // S + PLANE (fp32 operands of the split-bf16 x3 GEMM)
  template <int LDK, int PLANE>
  __device__ __forceinline__ void store_split(short* __restrict__ S) const {
    auto put = [&](short* dst, float a, float b, float c, float d) {
      const short ha = f2bf(a), hb = f2bf(b), hc = f2bf(c), hd = f2bf(d);
      *reinterpret_cast<bf16x4*>(dst) = (bf16x4){ha, hb, hc, hd};
      *reinterpret_cast<bf16x4*>(dst + PLANE) =
          (bf16x4){f2bf(a - bf2f(ha)), f2bf(b - bf2f(hb)), f2bf(c - bf2f(hc)), f2bf(d - bf2f(hd))};
    };
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (UNITS < 256 && c >= UNITS) continue;
      if (KC) {
        const int r = c / (BK / 4), kk = (c % (BK / 4)) * 4;
        put(S + r * LDK + kk, v[i][0], v[i][1], v[i][2], v[i][3]);
      } else {
        const int r = (c % (ROWS / 4)) * 4, kk = (c / (ROWS / 4)) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          put(S + (r + e) * LDK + kk, v[i * 4 + 0][e], v[i * 4 + 1][e], v[i * 4 + 2][e], v[i * 4 + 3][e]);
      }
    }
  }
};

// bf16-source variant (bf16 compute only; no remap: the host passes compacted operands).
// KC: one 16-B load = 8 consecutive k of one row.  !KC: 8x8 micro-block (8 rows x 8 k) from 8
// loads of 16 B at k..k+7, transposed in registers -> 8 row stores of 8 k (16 B each).
template <int ROWS, int BK, bool KC>
struct TileLoaderBf16 {
  static constexpr int UNITS = KC ? ROWS * BK / 8 : ROWS * BK / 64;
  static constexpr int PER_T = (UNITS + 255) / 256;
  static constexpr int NV = KC ? PER_T : PER_T * 8;
  static_assert(UNITS % 256 == 0 || UNITS < 256, "tile / thread mismatch");
  bf16x8 v[NV];

  __device__ __forceinline__ bf16x8 ld8(const short* __restrict__ P, int ld, int row, int nrows, int k, int kend) const {
    bf16x8 x = {0, 0, 0, 0, 0, 0, 0, 0};
    if (KC) {
      if (row < nrows) {
        if (k + 7 < kend) {
          x = *reinterpret_cast<const bf16x8*>(P + (size_t)row * ld + k);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (k + e < kend) x[e] = P[(size_t)row * ld + k + e];
        }
      }
    } else {
      if (k < kend) {
        if (row + 7 < nrows) {
          x = *reinterpret_cast<const bf16x8*>(P + (size_t)k * ld + row);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (row + e < nrows) x[e] = P[(size_t)k * ld + row + e];
        }
      }
    }
    return x;
  }

  __device__ __forceinline__ void load(const short* __restrict__ P, int ld, int row0, int nrows, int k0, int kend) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (UNITS < 256 && c >= UNITS) continue;
      if (KC) {
        const int r = c / (BK / 8), kk = (c % (BK / 8)) * 8;
        v[i] = ld8(P, ld, row0 + r, nrows, k0 + kk, kend);
      } else {
        const int r = (c % (ROWS / 8)) * 8, kk = (c / (ROWS / 8)) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i * 8 + j] = ld8(P, ld, row0 + r, nrows, k0 + kk + j, kend);
      }
    }
  }

  template <int LDK>
  __device__ __forceinline__ void store(short* __restrict__ S) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (UNITS < 256 && c >= UNITS) continue;
      if (KC) {
        const int r = c / (BK / 8), kk = (c % (BK / 8)) * 8;
        *reinterpret_cast<bf16x8*>(S + r * LDK + kk) = v[i];
      } else {
        const int r = (c % (ROWS / 8)) * 8, kk = (c / (ROWS / 8)) * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          bf16x8 t;
#pragma unroll
          for (int j = 0; j < 8; ++j) t[j] = v[i * 8 + j][e];
          *reinterpret_cast<bf16x8*>(S + (r + e) * LDK + kk) = t;
        }
      }
    }
  }
};

// Operand loader selector: SRC16 = the operand is bf16 in memory (bf16 compute only).
template <int ROWS, int BK, bool KC, bool MAP, bool SRC16> struct OpLoader;
template <int ROWS, int BK, bool KC, bool MAP> struct OpLoader<ROWS, BK, KC, MAP, false> {
  TileLoader<ROWS, BK, KC, MAP> t;
  __device__ __forceinline__ void load(const void* P, int ld, int row0, int nrows, int k0, int kend, const Remap& rm) {
    t.load(reinterpret_cast<const float*>(P), ld, row0, nrows, k0, kend, rm);
  }
  template <typename T, int LDK> __device__ __forceinline__ void store(T* S) const { t.template store<T, LDK>(S); }
  template <int LDK, int PLANE> __device__ __forceinline__ void store_split(short* S) const {
    t.template store_split<LDK, PLANE>(S);
  }
};
template <int ROWS, int BK, bool KC, bool MAP> struct OpLoader<ROWS, BK, KC, MAP, true> {
  TileLoaderBf16<ROWS, BK, KC> t;
  __device__ __forceinline__ void load(const void* P, int ld, int row0, int nrows, int k0, int kend, const Remap&) {
    t.load(reinterpret_cast<const short*>(P), ld, row0, nrows, k0, kend);
  }
  template <typename T, int LDK> __device__ __forceinline__ void store(T* S) const {
    t.template store<LDK>(reinterpret_cast<short*>(S));
  }
};

// Shared epilogue: bias / beta / remapped C stores or split-K slabs, and the optional fused
// BatchNorm statistics.  Waves form a WGM x WGN grid over the tile (wave (wm, wn) owns rows
// wm*BM/WGM.. and columns wn*BN/WGN..).  Statistics are per 64-row tile of C: a wave's rows lie
// in one such tile (BM/WGM divides 64).  red: LDS scratch of >= WGM*BN floats, free (all waves
// past the main loop).
template <int BM, int BN, int WGM, int WGN, int TM, int TN>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, f32x16 (&acc)[TM][TN], int m0, int n0, int wm,
                                              int wn, int lr, int lh, float* red, bool split, int z) {
  constexpr int WM = BM / WGM, WN = BN / WGN;
  // C/D map of the 32x32 MFMA tile: col = lane&31, row = (e&3) + 8*(e>>2) + 4*(lane>>5)
  // split: this workgroup's K range z is one slab of ws (split-K), not C
  // common case, decided per workgroup (uniform): a whole tile of an unremapped f32 or bf16 C with no
  // beta -- straight-line stores from one row base per (i, j), 32-bit offsets, no per-element tests
  const bool fast = !split && g.beta == 0.f && g.rC.seg == 0x7fffffff && g.rC.off0 == 0 && m0 + BM <= g.M &&
                    n0 + BN <= g.N;
  if (fast) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + lr;
      const float bv = g.bias ? g.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r0 = m0 + wm * WM + i * 32 + 4 * lh;
        if (g.c16) {
          short* base = reinterpret_cast<short*>(g.C) + (size_t)r0 * g.ldc + n;
#pragma unroll
          for (int e = 0; e < 16; ++e) base[((e & 3) + 8 * (e >> 2)) * g.ldc] = f2bf(acc[i][j][e] + bv);
        } else {
          float* base = g.C + (size_t)r0 * g.ldc + n;
#pragma unroll
          for (int e = 0; e < 16; ++e) base[((e & 3) + 8 * (e >> 2)) * g.ldc] = acc[i][j][e] + bv;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TM && !fast; ++i)
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
          g.ws[((size_t)z * g.M + m) * g.N + n] = acc[i][j][e];
        } else if (g.c16) {
          reinterpret_cast<short*>(g.C)[(size_t)m * g.ldc + nc] = f2bf(acc[i][j][e] + bv);
        } else {
          float* cp = g.C + (size_t)m * g.ldc + nc;
          float v = acc[i][j][e] + bv;
          if (g.beta != 0.f) v += g.beta * *cp;
          *cp = v;
        }
      }
    }
  if (g.bnb_part && !split) {
    // BatchNorm backward first pass (bn_bwd_partial4_kernel's sums) from the accumulators: this
    // wave's WM (= 32, TM = 1) rows are one row chunk (bnb_rpc 32) or two (bnb_rpc 16: rows 0-15 of
    // the 32x32 tile are its elements e < 8, rows 16-31 e >= 8); the host checks the plan
    const int chunk = (m0 + wm * WM) / g.bnb_rpc;
    const bool two = g.bnb_rpc == 16;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + lr;
      const bool nok = n < g.N;
      const float mu = nok ? g.bnb_mean[n] : 0.f;
      double s0[2] = {0.0, 0.0}, s1[2] = {0.0, 0.0};
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
          if (nok && m < g.M) {
            const size_t idx = (size_t)m * g.N + n;
            const float dy = g.bnb_hact16[idx] > 0 ? acc[i][j][e] * g.bnb_scale : 0.f;
            const int h = (two && e >= 8) ? 1 : 0;
            s0[h] += dy;
            s1[h] += (double)((g.bnb_xpre[idx] - mu) * dy);
          }
        }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        s0[h] += __shfl_xor(s0[h], 32, 64);
        s1[h] += __shfl_xor(s1[h], 32, 64);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (lh == 0 && nok && (h == 0 || two)) {
          double* pp = g.bnb_part + (size_t)(chunk + h) * 3 * g.N;
          pp[n] = s0[h];
          pp[g.N + n] = s1[h];
          pp[2 * (size_t)g.N + n] = 0.0;
        }
    }
  }
  if (g.stats && !split) {
    // BatchNorm fusion: exact two-pass (sum, M2) of each 64-row tile's column values from
    // registers; the BN finalize merges tiles in f64 (Chan) -- no extra pass over C.
    static_assert(64 % WM == 0, "a wave's rows must lie in one 64-row statistics tile");
    constexpr int WPG = 64 / WM;                      // waves (along M) per statistics tile
    const int grp = (wm * WM) / 64;                   // this wave's statistics tile inside the block
    const int rows = min(64, g.M - (m0 + grp * 64));
    float bvj[TN], mean[TN], ps[TN], sum0[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + lr;
      bvj[j] = (g.bias && n < g.N) ? g.bias[n] : 0.f;
      mean[j] = 0.f;
      sum0[j] = 0.f;
    }
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
            const float v = acc[i][j][e] + bvj[j];
            const float t = pass == 0 ? v : (v - mean[j]) * (v - mean[j]);
            s += m < g.M ? t : 0.f;
          }
        s += __shfl_xor(s, 32, 64);
        ps[j] = s;
      }
      if (lh == 0)
#pragma unroll
        for (int j = 0; j < TN; ++j) red[wm * BN + wn * WN + j * 32 + lr] = ps[j];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int c = wn * WN + j * 32 + lr;
        float tot = 0.f;
#pragma unroll
        for (int k = 0; k < WPG; ++k) tot += red[(grp * WPG + k) * BN + c];
        if (pass == 0) {
          sum0[j] = tot;
          mean[j] = rows > 0 ? tot / (float)rows : 0.f;
        } else if (wm % WPG == 0 && lh == 0 && n0 + c < g.N && rows > 0) {
          float* o = g.stats + ((size_t)(m0 / 64 + grp) * g.N + n0 + c) * 2;
          o[0] = sum0[j];
          o[1] = tot;
        }
      }
      __syncthreads();
    }
  }
}

// SPLIT (BF16, fp32 operands in memory): split-bf16 x3 -- each operand tile is staged in LDS as a hi
// and a lo bf16 plane (x = hi + lo to ~16 mantissa bits) and C += Ahi Bhi + Ahi Blo + Alo Bhi on the
// bf16 MFMA with fp32 accumulation: the fp32 GEMMs of the bf16-forward / fp32-backward mode at
// three bf16 MFMA passes instead of the 8x slower fp32 MFMA (the dropped Alo Blo term is 2^-16
// relative).
template <int BM, int BN, bool TA, bool TB, bool BF16, bool A16, bool B16, bool SPLIT = false>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs g, int tiles_n, int remap_xcd) {
  FBN_MAIN_PRIO();
  typedef GemmTraits<BF16> Tr;
  typedef typename Tr::T T;
  static_assert(!SPLIT || (BF16 && !A16 && !B16), "split-bf16 stages fp32 operands");
  // split: K tiles of 32 (two LDS planes per operand at half the depth: the LDS of a plain bf16 tile)
  constexpr int BK = SPLIT ? 32 : Tr::BK, LDK = SPLIT ? 40 : Tr::LDK;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  constexpr int PL = SPLIT ? 2 : 1;                 // LDS planes per operand tile (hi, lo)
  __shared__ __attribute__((aligned(16))) T sA[2][PL * BM * LDK];
  __shared__ __attribute__((aligned(16))) T sB[2][PL * BN * LDK];

  // XCD-aware tile order: dispatch deals blocks round-robin over 8 XCDs, so block b runs on
  // XCD b % 8; give each XCD a contiguous run of tiles (neighbours share the A row panel).
  int bid = blockIdx.x;
  const int nb = gridDim.x;
  if (remap_xcd) bid = (bid % 8) * (nb / 8) + bid / 8;
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int n0 = tn * BN, m0 = tm * BM;
  const int kbeg = blockIdx.z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int ntiles = (kend - kbeg + BK - 1) / BK;
  const Remap none = {0x7fffffff, 0, 0};

  OpLoader<BM, BK, !TA, false, A16> la;
  OpLoader<BN, BK, TB, true, B16> lb;

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

  auto stage = [&](int b) {
    if constexpr (SPLIT) {
      la.template store_split<LDK, BM * LDK>(reinterpret_cast<short*>(sA[b]));
      lb.template store_split<LDK, BN * LDK>(reinterpret_cast<short*>(sB[b]));
    } else {
      la.template store<T, LDK>(sA[b]);
      lb.template store<T, LDK>(sB[b]);
    }
  };
  if (ntiles > 0) {
    la.load(g.A, g.lda, m0, g.M, kbeg, kend, none);
    lb.load(g.B, g.ldb, n0, g.N, kbeg, kend, g.rB);
    stage(0);
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
      // k permutation: lane half h covers k in [16h, 16h+16); step s uses k = 16h + s for A and B.
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const f32x4*>(A_ + (wm * WM + i * 32 + lr) * LDK + lh * 16 + q * 4);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const f32x4*>(B_ + (wn * WN + j * 32 + lr) * LDK + lh * 16 + q * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
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
        if constexpr (SPLIT) {
          bf16x8 al[TM], bl[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i)
            al[i] = *reinterpret_cast<const bf16x8*>(A_ + BM * LDK + (wm * WM + i * 32 + lr) * LDK + s * 16 + lh * 8);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            bl[j] = *reinterpret_cast<const bf16x8*>(B_ + BN * LDK + (wn * WN + j * 32 + lr) * LDK + s * 16 + lh * 8);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bl[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
      }
    }
    if (more) stage(buf ^ 1);
    __syncthreads();
  }

  gemm_epilogue<BM, BN, 2, 2>(g, acc, m0, n0, wm, wn, lr, lh, reinterpret_cast<float*>(&sA[0][0]), gridDim.z > 1,
                              blockIdx.z);
}

__global__ void gemm_splitk_reduce(GemmArgs g, int nsplit) {
  FBN_MAIN_PRIO();
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

// ------------------------------------------------------------------ bf16 LDS-DMA kernel
// Both operands bf16 in memory, K % 64 == 0 per split, no B remap.  Each operand is either
//   KC (k-contiguous: A[m*lda+k] / B[n*ldb+k]; the forward and dgrad GEMMs), or
//   KM (k-major:      A[k*lda+m] / B[k*ldb+n]; the wgrad GEMMs, batch = k).
// Staging: global_load_lds_dwordx4 straight into LDS (no VGPR round trip, no ds_write); one
// DMA wave-instruction writes 1 KiB contiguously (lane L -> bytes 16L..16L+15), so images are
// unpadded and bank conflicts are removed by XOR-permuting 16-B chunks: the permutation is
// applied to each lane's SOURCE address and undone on the read (the same involution).
//   KC image [rows][64 k], 128-B rows; chunk c of row r in slot c ^ ((r >> 1) & 7).  MFMA
//      fragments by ds_read_b128 (16 lanes = 16 consecutive rows: all 16 bank quads).
//   KM image [64 k][ROWS], rows of 2*ROWS bytes; chunk c of row k in slot c ^ f(k) with
//      f = 4*((k>>1)&1) (128-B rows) or 4*(k&3) (256-B rows).  Fragments by two
//      ds_read_b64_tr_b16 (each 16-lane group reads 4 k-rows x 16 columns and receives them
//      column-major = the MFMA lane layout); a 32-lane half then covers 16 bank quads.
// One barrier per K-step: at the top of step t every wave has finished reading stage t-1, so
// the DMA of stage t+1 into that buffer is issued right after the barrier and lands while the
// MFMAs of stage t run.
typedef __attribute__((address_space(1))) void g_void;
typedef __attribute__((address_space(3))) void l_void;
typedef short v4s __attribute__((ext_vector_type(4)));

template <int ROWS>
__device__ __forceinline__ int km_off(int k, int m) {   // byte offset of (k, m) in a KM image
  constexpr int RB = ROWS * 2;
  const int f = RB == 128 ? (((k >> 1) & 1) << 2) : ((k & 3) << 2);
  return k * RB + ((((m >> 3) ^ f)) << 4) + (m & 7) * 2;
}

// MFMA 32x32x16 fragment (lane l: row l&31, k = 8*(l>>5) + j) of a 32-row slab starting at
// row r0, k-step s, from a KC or KM image.
template <int ROWS, bool KM>
__device__ __forceinline__ bf16x8 frag(const char* img, int r0, int s, int lane) {
  if constexpr (!KM) {
    const int r = r0 + (lane & 31);
    const int co = ((2 * s + (lane >> 5)) ^ ((r >> 1) & 7)) << 4;
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + co);
  } else {
    const int i16 = lane & 15, G = lane >> 4;
    const int m = r0 + 16 * (G & 1) + 4 * (i16 & 3);
    const int k = 16 * s + 8 * (G >> 1) + (i16 >> 2);
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + km_off<ROWS>(k, m)));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + km_off<ROWS>(k + 4, m)));
    return (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

// wait until at most n of this wave's DMA groups are outstanding (n: compile-time multiple of GPW)
template <int GPW, int S>
__device__ __forceinline__ void wait_dma(int ahead) {   // ahead = stages allowed to stay in flight (0 .. S-2)
  if constexpr (S >= 4) {
    if (ahead >= 2) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory"); return; }
  }
  if constexpr (S >= 3) {
    if (ahead >= 1) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory"); return; }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// XCD-aware, bijective block -> tile order: blocks b and b+8 share an XCD (round-robin
// dispatch); give each XCD a contiguous run of tile ids so neighbouring tiles (which share an A
// row panel) hit one L2.  Bijective for any grid size (remainder blocks spread over the first
// nb % 8 XCD slots).
__device__ __forceinline__ int xcd_tile(int bid, int nb) {
  const int q = nb / 8, r = nb % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// WGM x WGN waves (64 * WGM * WGN threads); wave (wm, wn) owns a (BM/WGM) x (BN/WGN) sub-tile
// of 32x32 MFMA blocks.  8 waves on a 128x128 tile: two waves per SIMD, each with 2 MFMAs per
// 3 fragment reads (4 waves on 64x64 tiles: 1 MFMA per 2 reads).
template <int BM, int BN, bool AKM, bool BKM, int S, int WGM = 2, int WGN = 2, bool S3 = false>
__device__ __forceinline__ void gemm_dma16_tile(const GemmArgs& g, int m0, int n0, int z, bool split) {
  constexpr int NW = WGM * WGN;
  constexpr int BK = 64;
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 32, TN = WN / 32;
  constexpr int AB = BM * BK * 2, STAGE = (BM + BN) * BK * 2;   // A image bytes, stage bytes
  constexpr int GPW = (BM + BN) / 8 / NW;                         // 1-KiB DMA groups per wave per stage
  static_assert(((BM + BN) / 8) % NW == 0 && BM % 16 == 0 && WM % 32 == 0 && WN % 32 == 0, "tile / wave mismatch");
  static_assert(S >= 2 && S <= 4, "stages");
  __shared__ __attribute__((aligned(1024))) char smem[S * STAGE];

  const int kbeg = z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave % WGM, wn = wave / WGM;
  const int lr = lane & 31, lh = lane >> 5;

  // this lane's source for each of its wave's DMA groups, and the per-stage source advance
  // (rows / columns past M or N are clamped to valid memory: their products land only in C
  // entries that are not stored)
  const short* src[GPW];
  const short* src2[GPW];   // split A ([A | A2] along K): the same lane's chunk in A2, k rebased to kseg
  long long adv[GPW];
  long long loff[GPW];      // S3: the lo image's offset, read in K-segment sel[j]
  int sel[GPW];
  const int t2 = kbeg < g.kseg ? (g.kseg - kbeg) / BK : 0;   // first K-step read from A2
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int grp = wave * GPW + j;
    const bool isA = grp < BM / 8;
    const int off = (isA ? grp : grp - BM / 8) * 1024 + lane * 16;   // byte offset inside the operand image
    const short* P = reinterpret_cast<const short*>(isA ? g.A : g.B);
    int ld = isA ? g.lda : g.ldb, lim = isA ? g.M : g.N, base = isA ? m0 : n0;
    const bool km = isA ? AKM : BKM;
    const int rows = isA ? BM : BN;
    src2[j] = nullptr;
    loff[j] = isA ? g.s3_loa : g.s3_lob;
    sel[j] = isA ? 2 : 1;
    if (!km) {
      const int r = off >> 7, slot = (off >> 4) & 7;
      const int row = min(base + r, lim - 1);
      const int sw = (slot ^ ((r >> 1) & 7)) << 3;
      if constexpr (S3) {   // k = 0 of the hi image; per element of k
        src[j] = P + (size_t)row * ld + sw;
        adv[j] = 1;
        continue;
      }
      src[j] = P + (size_t)row * ld + kbeg + sw;
      if (isA && g.A2) src2[j] = reinterpret_cast<const short*>(g.A2) + (size_t)row * g.lda2 + (kbeg - g.kseg) + sw;
      adv[j] = BK;
    } else {
      if (!isA && g.B2 && n0 >= g.nseg) {   // this tile's columns lie in B2 (nseg is a multiple of BN)
        P = reinterpret_cast<const short*>(g.B2);
        ld = g.ldb2;
        lim -= g.nseg;
        base -= g.nseg;
      }
      const int RB = rows * 2;
      const int k = off / RB, slot = (off % RB) >> 4;
      const int f = RB == 128 ? (((k >> 1) & 1) << 2) : ((k & 3) << 2);
      int col = base + ((slot ^ f) << 3);
      if (col + 8 > lim) col = 0;
      if constexpr (S3) {
        src[j] = P + (size_t)k * ld + col;
        adv[j] = ld;
        continue;
      }
      src[j] = P + (size_t)(kbeg + k) * ld + col;
      adv[j] = (long long)BK * ld;
    }
  }
  auto issue = [&](int t, int buf) {
    if constexpr (S3) {
      // K-step t reads k' = kbeg + t BK in segment s = k' / s3k0 (BK never straddles one)
      const int kk = kbeg + t * BK, s = kk / g.s3k0, kl = kk - s * g.s3k0;
#pragma unroll
      for (int j = 0; j < GPW; ++j) {
        const short* s0 = src[j] + (s == sel[j] ? loff[j] : 0) + (long long)kl * adv[j];
        __builtin_amdgcn_global_load_lds((g_void*)s0, (l_void*)(smem + buf * STAGE + (wave * GPW + j) * 1024), 16, 0,
                                         0);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < GPW; ++j) {
      const short* s0 = (src2[j] && t >= t2) ? src2[j] : src[j];
      __builtin_amdgcn_global_load_lds((g_void*)(s0 + t * adv[j]), (l_void*)(smem + buf * STAGE + (wave * GPW + j) * 1024),
                                       16, 0, 0);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // S-stage ring: stages t+1 .. t+S-2 stay in flight across the barrier of step t (counted
  // vmcnt + raw s_barrier; __syncthreads() would drain every DMA with vmcnt(0)).  The barrier
  // also certifies that every wave finished step t-1, whose buffer the DMA of stage t+S-1
  // overwrites.
#pragma unroll
  for (int q = 0; q < S - 1; ++q)
    if (q < nk) issue(q, q);
  for (int t = 0; t < nk; ++t) {
    wait_dma<GPW, S>(min(S - 2, nk - 1 - t));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + S - 1 < nk) issue(t + S - 1, (t + S - 1) % S);
    const char* SA = smem + (t % S) * STAGE;
    const char* SB = SA + AB;
    // fragments double-buffered in registers: the LDS reads of sub-step s+1 are in flight while
    // the MFMAs of sub-step s run (one wave per SIMD at 128x128 tiles cannot hide them otherwise)
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[0][i] = frag<BM, AKM>(SA, wm * WM + i * 32, 0, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[0][j] = frag<BN, BKM>(SB, wn * WN + j * 32, 0, lane);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int cb = s & 1, nb = cb ^ 1;
      if (s + 1 < BK / 16) {
#pragma unroll
        for (int i = 0; i < TM; ++i) af[nb][i] = frag<BM, AKM>(SA, wm * WM + i * 32, s + 1, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[nb][j] = frag<BN, BKM>(SB, wn * WN + j * 32, s + 1, lane);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of this sub-step's MFMAs
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cb][i], bfr[cb][j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();   // the stats epilogue reuses the staging LDS
  gemm_epilogue<BM, BN, WGM, WGN>(g, acc, m0, n0, wm, wn, lr, lh, reinterpret_cast<float*>(smem), split, z);
}

template <int BM, int BN, bool AKM, bool BKM, int S, int WGM = 2, int WGN = 2, bool S3 = false>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_dma16_kernel(GemmArgs g, int tiles_n, int remap_xcd) {
  FBN_MAIN_PRIO();
  int bid = blockIdx.x;
  const int nb = gridDim.x;
  if (remap_xcd) bid = xcd_tile(bid, nb);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  gemm_dma16_tile<BM, BN, AKM, BKM, S, WGM, WGN, S3>(g, tm * BM, tn * BN, blockIdx.z, gridDim.z > 1);
}

// Several slab-mode GEMMs (fbn_gemm_slabs_group: the step's weight gradients) in ONE launch: the
// flat block index runs over problem p's tiles x K-slabs in [start[p], start[p+1]), slab-major
// (the order of a separate launch's (x, z) grid).  Every problem writes its K-slabs into its own
// ws exactly as a separate fbn_gemm_slabs launch would: each output element's K-chunk is summed by
// the same 32x32x16 MFMA sequence whatever the tile shape, so the slabs are bit-identical.
#define FBN_GEMM_GROUP_MAX 6
struct GemmGroup {
  GemmArgs g[FBN_GEMM_GROUP_MAX];
  int tiles_n[FBN_GEMM_GROUP_MAX], tiles[FBN_GEMM_GROUP_MAX], start[FBN_GEMM_GROUP_MAX + 1];
  int n;
  int remap;   // XCD-aware block order (FBN_GROUP_XCD=0: dispatch order, A/B)
};
template <int BM, int BN, bool AKM, bool BKM, int S, int WGM, int WGN, bool S3 = false>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_dma16_group_kernel(GemmGroup G) {
  FBN_MAIN_PRIO();
  // XCD-aware order over the whole flat grid: each XCD runs a contiguous run of (problem, slab,
  // tile), so workgroups that share an operand panel of one K-slab meet in one L2: the launch's L2
  // fills 251 -> 115 MB for ~77 MB of operands (profiles/r03x_pmc_traffic.json); the time is
  // unchanged (0.4285 vs 0.4289 ms/step) -- the re-reads were served by the MALL
  const int b = G.remap ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
  int p = 0;
#pragma unroll
  for (int q = 1; q < FBN_GEMM_GROUP_MAX; ++q)
    if (q < G.n && b >= G.start[q]) p = q;
  const int local = b - G.start[p];
  const int z = local / G.tiles[p], t = local - z * G.tiles[p];
  const int tm = t / G.tiles_n[p], tn = t - tm * G.tiles_n[p];
  gemm_dma16_tile<BM, BN, AKM, BKM, S, WGM, WGN, S3>(G.g[p], tm * BM, tn * BN, z, true);
}

// vectorised split-K reduce: 4 consecutive columns per thread (N, ldc and the C remap in
// multiples of 4, C 16-B aligned); same slab order as gemm_splitk_reduce (bit-identical)
__global__ void gemm_splitk_reduce4(GemmArgs g, int nsplit) {
  FBN_MAIN_PRIO();
  const int N4 = g.N >> 2;
  const size_t total4 = (size_t)g.M * N4, total = (size_t)g.M * g.N;
  for (size_t i4 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i4 < total4; i4 += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(i4 / N4), n = (int)(i4 - (size_t)m * N4) * 4;
    const size_t idx = (size_t)m * g.N + n;
    f32x4 s = *reinterpret_cast<const f32x4*>(g.ws + idx);
    for (int z = 1; z < nsplit; ++z) s += *reinterpret_cast<const f32x4*>(g.ws + (size_t)z * total + idx);
    if (g.bias) s += *reinterpret_cast<const f32x4*>(g.bias + n);
    float* cp = g.C + (size_t)m * g.ldc + remap(g.rC, n);
    if (g.beta != 0.f) s += g.beta * *reinterpret_cast<const f32x4*>(cp);
    *reinterpret_cast<f32x4*>(cp) = s;
  }
}

// wide split-K reduce for many slabs over a small C (the wgrad GEMMs with K = 5B or B): block =
// 16 column quads x 16 slab groups; slab group zg sums slabs zg, zg+16, ...; the 16 partials are
// combined in a fixed order (deterministic)
__global__ void __launch_bounds__(256) gemm_splitk_reduce4_wide(GemmArgs g, int nsplit) {
  FBN_MAIN_PRIO();
  __shared__ f32x4 red[16][16];
  const int qd = threadIdx.x & 15, zg = threadIdx.x >> 4;
  const int N4 = g.N >> 2;
  const size_t total4 = (size_t)g.M * N4, total = (size_t)g.M * g.N;
  const size_t i4 = (size_t)blockIdx.x * 16 + qd;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  size_t idx = 0;
  if (i4 < total4) {
    const int m = (int)(i4 / N4), n = (int)(i4 - (size_t)m * N4) * 4;
    idx = (size_t)m * g.N + n;
    for (int z = zg; z < nsplit; z += 16) acc += *reinterpret_cast<const f32x4*>(g.ws + (size_t)z * total + idx);
  }
  red[zg][qd] = acc;
  __syncthreads();
  if (zg == 0 && i4 < total4) {
    f32x4 s = red[0][qd];
#pragma unroll
    for (int k = 1; k < 16; ++k) s += red[k][qd];
    const int m = (int)(i4 / N4), n = (int)(i4 - (size_t)m * N4) * 4;
    if (g.bias) s += *reinterpret_cast<const f32x4*>(g.bias + n);
    float* cp = g.C + (size_t)m * g.ldc + remap(g.rC, n);
    if (g.beta != 0.f) s += g.beta * *reinterpret_cast<const f32x4*>(cp);
    *reinterpret_cast<f32x4*>(cp) = s;
  }
}

// split-K reduce with the BatchNorm statistics epilogue: one workgroup per 64x64 tile of C;
// thread (col = tid & 63, rows 16*(tid >> 6) .. +15) -> coalesced slab reads along n.  Sums the
// K-slabs in the same order as gemm_splitk_reduce (so C is bit-identical with or without stats),
// then (sum, M2 about the tile mean) of each column from registers.
__global__ __launch_bounds__(256) void gemm_splitk_reduce_stats(GemmArgs g, int nsplit) {
  FBN_MAIN_PRIO();
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c, m0 = blockIdx.y * 64;
  const int rows = min(64, g.M - m0);
  const size_t total = (size_t)g.M * g.N;
  const bool nok = n < g.N;
  const float bv = (nok && g.bias) ? g.bias[n] : 0.f;
  const int nc = nok ? remap(g.rC, n) : 0;
  float v[16];
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + rg * 16 + r;
    v[r] = 0.f;
    if (nok && m < g.M) {
      const size_t idx = (size_t)m * g.N + n;
      float a = 0.f;
      for (int z = 0; z < nsplit; ++z) a += g.ws[(size_t)z * total + idx];
      a += bv;
      float* cp = g.C + (size_t)m * g.ldc + nc;
      if (g.beta != 0.f) a += g.beta * *cp;
      *cp = a;
      v[r] = a;
      s += a;
    }
  }
  red[rg][c] = s;
  __syncthreads();
  const float sum0 = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  const float mean = rows > 0 ? sum0 / (float)rows : 0.f;
  __syncthreads();
  float q = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + rg * 16 + r;
    const float t = v[r] - mean;
    q += m < g.M ? t * t : 0.f;
  }
  red[rg][c] = q;
  __syncthreads();
  if (rg == 0 && nok) {
    float* o = g.stats + ((size_t)blockIdx.y * g.N + n) * 2;
    o[0] = sum0;
    o[1] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// ------------------------------------------------------------------ host-side planning
struct GemmPlan {
  int bm, bn, split;
  int waves = 4;   // LDS-DMA kernel: 4 (2x2) or 8 (2 along M x 4 along N)
  int stages = 0;  // LDS-DMA ring depth (0 = FBN_DMA_STAGES)
};

static GemmPlan plan_gemm(int M, int N, int K, int bk) {
  // Prefer the biggest tile that still yields >= 1024 workgroups (4 per CU); otherwise the
  // smallest tile, then split K until ~1024 workgroups or K per split drops to 4 tiles.
  const int cand[4][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}};
  GemmPlan p = {64, 64, 1};
  for (int c = 0; c < 4; ++c) {
    const int bm = cand[c][0], bn = cand[c][1];
    if ((bm == 128 && M < 256) || (bn == 128 && N < 256)) continue;   // mostly-empty tiles
    const long long tiles = (long long)fbn_cdiv(M, bm) * fbn_cdiv(N, bn);
    if (tiles >= 1024) { p = {bm, bn, 1}; return p; }
  }
  const long long tiles = (long long)fbn_cdiv(M, 64) * fbn_cdiv(N, 64);
  int s = 1;
  while (tiles * s < 1024 && K / (s * 2) >= 4 * bk && s < 64) s *= 2;
  p.split = s;
  return p;
}

// LDS-DMA kernel plan (tools/gemm_sweep.py on the C3 shapes, MI355X, profiles/r02_gemm_sweep.log):
// * large outputs (>= 512 64x64 tiles, no split): 8 waves on 64x128 tiles (each wave 32x32 of a
//   2x4 wave grid), or 128x128 tiles when N >= 1024 and they still give >= 256 workgroups -- 8
//   waves (two per SIMD) keep the MFMA pipe busy while the partner wave waits on its LDS reads;
//   F3 30.9 -> 26.8 us, dc 36.2 -> 32.5 us, U 11.4 -> 9.4 us;
// * small outputs (the wgrad GEMMs, K = batch): split K to ~512 workgroups; M, N >= 512 take
//   128x128 tiles with 8 waves (dWa 42.5 -> 35.1 us), else 64x64 with 4 waves.
static GemmPlan plan_dma16(int M, int N, int K) {
  const long long t64 = (long long)fbn_cdiv(M, 64) * fbn_cdiv(N, 64);
  if (t64 >= 512) {
    if (const char* e = getenv("FBN_DMA_BIG_TILE")) {   // tuning knob: "bm,bn" for large outputs
      int a = 64, b = 64;
      if (sscanf(e, "%d,%d", &a, &b) == 2) return {a, b, 1};
    }
    if (N >= 1024 && (long long)fbn_cdiv(M, 128) * fbn_cdiv(N, 128) >= 256) return {128, 128, 1, 8};
    // tuning knob: "bm,bn,waves" for an output whose 64x128 tiles leave fewer than two workgroups
    // per CU (C3: MLP layer 2, 8192 x 256)
    const char* mt = getenv("FBN_DMA_MID_TILE");
    if (mt && (long long)fbn_cdiv(M, 64) * fbn_cdiv(N, 128) < 512) {
      int a = 64, b = 128, w = 8;
      if (sscanf(mt, "%d,%d,%d", &a, &b, &w) == 3) return {a, b, 1, w};
    }
    if (N >= 128) return {64, 128, 1, 8};
    return {64, 64, 1};
  }
  GemmPlan p = (M >= 512 && N >= 512) ? GemmPlan{128, 128, 1, 8} : GemmPlan{64, 64, 1};
  const long long tiles = (long long)fbn_cdiv(M, p.bm) * fbn_cdiv(N, p.bn);
  const long long target = p.bm == 128 ? 512 : 256;
  // a tiny output (the d x d / d x 128 weight gradients: 4 tiles) is latency-bound, not feed-bound:
  // split K down to 2 K-steps per workgroup and keep a 4-deep ring (FBN_GEMM_TINY=0: the old rule)
  const char* te = getenv("FBN_GEMM_TINY");
  const bool tiny = tiles <= 16 && !(te && atoi(te) == 0);
  const int min_k = tiny ? 128 : 256;
  while (p.split < 64 && tiles * p.split * 2 <= target && K / (p.split * 2) >= min_k) p.split *= 2;
  if (tiny) p.stages = 4;
  return p;
}

// K-slabs of the LDS-DMA plan after the K-per-split rounding gemm_impl applies (slab mode)
static int slab_split(int M, int N, int K) {
  const GemmPlan p = plan_dma16(M, N, K);
  int per = fbn_cdiv(K, p.split);
  per = fbn_cdiv(per, 64) * 64;
  return K > 0 ? fbn_cdiv(K, per) : 1;
}

template <int BM, int BN, bool TA, bool TB, bool BF16, bool A16, bool B16, bool SPLIT = false>
static void launch_tile(const GemmArgs& g, int nsplit, hipStream_t st) {
  const int tn = fbn_cdiv(g.N, BN), tm = fbn_cdiv(g.M, BM);
  const int nb = tn * tm;
  dim3 grid(nb, 1, nsplit);
  fbn_launch((gemm_kernel<BM, BN, TA, TB, BF16, A16, B16, SPLIT>), grid, dim3(256), 0, st, g, tn,
                     (nb % 8 == 0) ? 1 : 0);
}

template <int BM, int BN, bool AKM, bool BKM, int WGM, int WGN>
static void launch_dma16(const GemmArgs& g, const GemmPlan& p, hipStream_t st) {
  const int tn = fbn_cdiv(g.N, BN), tm = fbn_cdiv(g.M, BM);
  const int nb = tn * tm;
  const int rx = nb >= 8 ? 1 : 0;
  const char* e = getenv("FBN_GEMM_STAGES");   // tuning knob
  const int S = e ? atoi(e) : (p.stages ? p.stages : FBN_DMA_STAGES);
  const dim3 grid(nb, 1, p.split), blk(64 * WGM * WGN);
  if (g.s3k0) {   // split-bf16 x3 over two images per operand (two-stage ring only)
    fbn_launch((gemm_dma16_kernel<BM, BN, AKM, BKM, 2, WGM, WGN, true>), grid, blk, 0, st, g, tn, rx);
    return;
  }
  if (S <= 2)
    fbn_launch((gemm_dma16_kernel<BM, BN, AKM, BKM, 2, WGM, WGN>), grid, blk, 0, st, g, tn, rx);
  else if (S == 3)
    fbn_launch((gemm_dma16_kernel<BM, BN, AKM, BKM, 3, WGM, WGN>), grid, blk, 0, st, g, tn, rx);
  else
    fbn_launch((gemm_dma16_kernel<BM, BN, AKM, BKM, 4, WGM, WGN>), grid, blk, 0, st, g, tn, rx);
}

template <bool AKM, bool BKM>
static void launch_dma16_sel(const GemmArgs& g, const GemmPlan& p, hipStream_t st) {
  if (p.waves == 8) {
    if (p.bm == 128 && p.bn == 128) launch_dma16<128, 128, AKM, BKM, 2, 4>(g, p, st);
    else if (p.bm == 128) launch_dma16<128, 64, AKM, BKM, 4, 2>(g, p, st);
    else if (p.bn == 128) launch_dma16<64, 128, AKM, BKM, 2, 4>(g, p, st);
    else launch_dma16<64, 64, AKM, BKM, 2, 2>(g, p, st);
    return;
  }
  if (p.bm == 128 && p.bn == 128) launch_dma16<128, 128, AKM, BKM, 2, 2>(g, p, st);
  else if (p.bm == 128) launch_dma16<128, 64, AKM, BKM, 2, 2>(g, p, st);
  else if (p.bn == 128) launch_dma16<64, 128, AKM, BKM, 2, 2>(g, p, st);
  else launch_dma16<64, 64, AKM, BKM, 2, 2>(g, p, st);
}

template <bool TA, bool TB, bool BF16, bool A16, bool B16>
static void launch_sel(const GemmArgs& g, const GemmPlan& p, hipStream_t st) {
  if (p.bm == 128 && p.bn == 128) launch_tile<128, 128, TA, TB, BF16, A16, B16>(g, p.split, st);
  else if (p.bm == 128) launch_tile<128, 64, TA, TB, BF16, A16, B16>(g, p.split, st);
  else if (p.bn == 128) launch_tile<64, 128, TA, TB, BF16, A16, B16>(g, p.split, st);
  else launch_tile<64, 64, TA, TB, BF16, A16, B16>(g, p.split, st);
}

template <bool TA, bool TB>
static void launch_split(const GemmArgs& g, const GemmPlan& p, hipStream_t st) {
  if (p.bm == 128 && p.bn == 128) launch_tile<128, 128, TA, TB, true, false, false, true>(g, p.split, st);
  else if (p.bm == 128) launch_tile<128, 64, TA, TB, true, false, false, true>(g, p.split, st);
  else if (p.bn == 128) launch_tile<64, 128, TA, TB, true, false, false, true>(g, p.split, st);
  else launch_tile<64, 64, TA, TB, true, false, false, true>(g, p.split, st);
}

template <bool TA, bool TB>
static void launch_types(const GemmArgs& g, const GemmPlan& p, int bf16, int a16, int b16, hipStream_t st) {
  if (bf16 == 2) launch_split<TA, TB>(g, p, st);
  else if (!bf16) launch_sel<TA, TB, false, false, false>(g, p, st);
  else if (a16 && b16) launch_sel<TA, TB, true, true, true>(g, p, st);
  else if (a16) launch_sel<TA, TB, true, true, false>(g, p, st);
  else if (b16) launch_sel<TA, TB, true, false, true>(g, p, st);
  else launch_sel<TA, TB, true, false, false>(g, p, st);
}

// upper bound over both kernels' plans (the caller does not say whether the DMA path applies)
extern "C" size_t fbn_gemm_workspace_size(int M, int N, int K, int bf16) {
  GemmPlan p = plan_gemm(M, N, K, bf16 == 1 ? 64 : 32);
  if (bf16) {
    const GemmPlan q = plan_dma16(M, N, K);
    if (q.split > p.split) p = q;
  }
  return p.split > 1 ? (size_t)p.split * M * N * sizeof(float) : 0;
}

// a16 / b16: the A / B operand is bf16 in memory (requires bf16 = 1, ld % 8 == 0 and no rB remap)
// stats: optional [ceil(M/64)][N][2] per-64-row-tile column (sum, M2) of C, from the MFMA epilogue (split == 1,
//        64-row tiles) or the split-K reduce; C is bit-identical with or without stats
static int gemm_impl(const void* A, const void* B, float* C, const float* bias, int M, int N, int K, int lda,
                     int ldb, int ldc, int transA, int transB, int rB_seg, int rB_off0, int rB_off1, int rC_seg,
                     int rC_off0, int rC_off1, float beta, int bf16, int a16, int b16, float* stats, float* ws,
                     size_t ws_bytes, const void* A2, int lda2, int kseg, const void* B2, int ldb2, int nseg,
                     void* stream, int c16 = 0, const GemmArgs* bnb = nullptr, int* slabs = nullptr,
                     const long long* s3 = nullptr);

extern "C" int fbn_gemm(const void* A, const void* B, float* C, const float* bias, int M, int N, int K, int lda,
                        int ldb, int ldc, int transA, int transB, int rB_seg, int rB_off0, int rB_off1, int rC_seg,
                        int rC_off0, int rC_off1, float beta, int bf16, int a16, int b16, float* stats, float* ws,
                        size_t ws_bytes, void* stream) {
  return gemm_impl(A, B, C, bias, M, N, K, lda, ldb, ldc, transA, transB, rB_seg, rB_off0, rB_off1, rC_seg, rC_off0,
                   rC_off1, beta, bf16, a16, b16, stats, ws, ws_bytes, nullptr, 0, 0x7fffffff, nullptr, 0, 0x7fffffff,
                   stream);
}

// Split operands (bf16 LDS-DMA path only): A2/kseg for a k-contiguous A = [A | A2] along K,
// B2/nseg for a k-major B = [B | B2] along N; kseg, nseg multiples of 128, ld2 % 8 == 0.
extern "C" int fbn_gemm_split(const void* A, const void* B, float* C, const float* bias, int M, int N, int K, int lda,
                              int ldb, int ldc, int transA, int transB, int rC_seg, int rC_off0, int rC_off1,
                              float beta, float* stats, float* ws, size_t ws_bytes, const void* A2, int lda2,
                              int kseg, const void* B2, int ldb2, int nseg, void* stream) {
  if ((A2 && (transA || (kseg & 127) || (lda2 & 7) || ((uintptr_t)A2 & 15))) ||
      (B2 && (transB || (nseg & 127) || (ldb2 & 7) || ((uintptr_t)B2 & 15)))) {
    fbn_set_error("fbn_gemm_split: A2 needs a k-contiguous A, B2 a k-major B; segments % 128, ld % 8, 16-B aligned");
    return FBN_ERR_ARG;
  }
  return gemm_impl(A, B, C, bias, M, N, K, lda, ldb, ldc, transA, transB, 0x7fffffff, 0, 0, rC_seg, rC_off0, rC_off1,
                   beta, 1, 1, 1, stats, ws, ws_bytes, A2, lda2, A2 ? kseg : 0x7fffffff, B2, ldb2,
                   B2 ? nseg : 0x7fffffff, stream);
}

// bf16 operands, bf16 C (rounded once from the f32 accumulators; C[m * ldc + n]); no bias, beta,
// remap or statistics, never split along K.  The bf16-mode dgrad of the MLP input (dc), whose only
// reader (fbn_bilinear_bwd) takes it in bf16: half the bytes written and read.
extern "C" int fbn_gemm_bf16out(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                                int transA, int transB, void* stream) {
  return gemm_impl(A, B, reinterpret_cast<float*>(C), nullptr, M, N, K, lda, ldb, ldc, transA, transB, 0x7fffffff, 0, 0,
                   0x7fffffff, 0, 0, 0.f, 1, 1, 1, nullptr, nullptr, 0, nullptr, 0, 0x7fffffff, nullptr, 0, 0x7fffffff,
                   stream, 1);
}

// Split-bf16 x3 (the bf16_fwd backward): C = beta C + A_hi B_hi + A_hi B_lo + A_lo B_hi, as ONE bf16
// GEMM over K = 3 K0 on the LDS-DMA path; A / B point at the hi image, their lo image lies lo_a /
// lo_b elements further (same layout): hi + lo carry 16 significant bits of each fp32 operand.
extern "C" int fbn_gemm_s3(const void* A, const void* B, float* C, int M, int N, int K0, int lda, int ldb, int ldc,
                           int transA, int transB, long long lo_a, long long lo_b, float beta, float* ws,
                           size_t ws_bytes, void* stream) {
  const long long s3[3] = {K0, lo_a, lo_b};
  return gemm_impl(A, B, C, nullptr, M, N, 3 * K0, lda, ldb, ldc, transA, transB, 0x7fffffff, 0, 0, 0x7fffffff, 0, 0,
                   beta, 1, 1, 1, nullptr, ws, ws_bytes, nullptr, 0, 0x7fffffff, nullptr, 0, 0x7fffffff, stream, 0,
                   nullptr, nullptr, s3);
}

// Slab mode (bf16 LDS-DMA path; the wgrad GEMMs of the trainer): op(A) op(B) with the split-K
// partial products left in ws as nsplit slabs [nsplit][M][N] (f32) -- no reduce launch; the
// caller sums them in the step's fbn_sum_jobs2 launch with the other deferred reductions (slab
// order, deterministic).  A2/kseg, B2/nseg as fbn_gemm_split.  Returns FBN_OK and *nsplit.
extern "C" size_t fbn_gemm_slabs_size(int M, int N, int K) {
  return (M > 0 && N > 0) ? (size_t)slab_split(M, N, K) * M * N * sizeof(float) : 0;
}
extern "C" int fbn_gemm_slabs(const void* A, const void* B, int M, int N, int K, int lda, int ldb, int transA,
                              int transB, float* ws, size_t ws_bytes, const void* A2, int lda2, int kseg,
                              const void* B2, int ldb2, int nseg, int* nsplit, void* stream) {
  if (!nsplit) { fbn_set_error("fbn_gemm_slabs: null nsplit"); return FBN_ERR_ARG; }
  if ((A2 && (transA || (kseg & 127) || (lda2 & 7) || ((uintptr_t)A2 & 15))) ||
      (B2 && (transB || (nseg & 127) || (ldb2 & 7) || ((uintptr_t)B2 & 15)))) {
    fbn_set_error("fbn_gemm_slabs: A2 needs a k-contiguous A, B2 a k-major B; segments % 128, ld % 8, 16-B aligned");
    return FBN_ERR_ARG;
  }
  return gemm_impl(A, B, ws, nullptr, M, N, K, lda, ldb, N, transA, transB, 0x7fffffff, 0, 0, 0x7fffffff, 0, 0, 0.f,
                   1, 1, 1, nullptr, ws, ws_bytes, A2, lda2, A2 ? kseg : 0x7fffffff, B2, ldb2,
                   B2 ? nseg : 0x7fffffff, stream, 0, nullptr, nsplit);
}

extern "C" int fbn_gemm_slabs_split(int M, int N, int K) { return (M > 0 && N > 0) ? slab_split(M, N, K) : 0; }

// K-slabs of a problem inside fbn_gemm_slabs_group: three quarters of fbn_gemm_slabs_split's
// (rounded) -- the grouped problems fill the chip together, so each needs fewer workgroups and
// fewer slabs are written and summed, but the launch wants two of its 64-KB workgroups on every CU:
// C3's four problems give 672 workgroups at fbn_gemm_slabs's partition, 497 at 3/4 and 336 at 1/2
// (round 3's default, which left most CUs one workgroup): 0.4099 vs 0.4178 ms/step over 5
// interleaved rounds on two boxes, C2 0.2028 vs 0.2052 (profiles/r06_wgrad_split_ab.txt; a quarter:
// 0.44).  FBN_GROUP_SPLIT_DIV overrides the divisor, fractional allowed (1: fbn_gemm_slabs's own
// partition, whose sums the group then reproduces bit for bit;
// tests/test_gpu_trainer.py::test_wgrad_group_bit_identical).
#define FBN_GROUP_SPLIT_DIV_DEFAULT (4.0 / 3.0)
static bool group_w4() {
  const char* e = getenv("FBN_GROUP_W4");   // read per call
  return e && atoi(e) != 0;
}
static int group_split(int M, int N, int K) {
  int s = slab_split(M, N, K);
  const char* e = getenv("FBN_GROUP_SPLIT_DIV");   // slabs = s / div (integral div) or round(s / div)
  const double div = e ? atof(e) : FBN_GROUP_SPLIT_DIV_DEFAULT;
  if (div > 1.0) {
    s = std::max(1, div == (double)(int)div ? s / (int)div : (int)std::lround(s / div));
    const int per = fbn_cdiv(fbn_cdiv(K, s), 64) * 64;
    s = fbn_cdiv(K, per);
  }
  return s;
}
extern "C" int fbn_gemm_slabs_group_split(int M, int N, int K) {
  return (M > 0 && N > 0 && K > 0) ? group_split(M, N, K) : 0;
}

// n <= FBN_GEMM_GROUP_MAX slab-mode GEMMs (each what fbn_gemm_slabs(d[i]...) computes, into d[i].ws
// as fbn_gemm_slabs_group_split(M, N, K) K-slabs) in one launch, on the tile shape the largest
// problem's own plan takes.  Every problem: k-major A and B (transA = 1, transB = 0, the
// weight-gradient form), bf16, K % 64 == 0.
struct FbnSlabGemm {   // one record of fbn_gemm_slabs_group (include/fibinet.h)
  const void* A;
  const void* B;
  float* ws;
  size_t ws_bytes;
  const void* A2;
  const void* B2;
  int M, N, K, lda, ldb, transA, transB, lda2, kseg, ldb2, nseg, s3k0;
  long long lo_a, lo_b;   // s3k0 > 0: split-bf16 x3 (GemmArgs::s3k0), K = 3 s3k0
};
extern "C" int fbn_gemm_slabs_group(const void* descs, int n, void* stream) {
  const FbnSlabGemm* d = static_cast<const FbnSlabGemm*>(descs);
  if (n <= 0) return FBN_OK;
  if (!d || n > FBN_GEMM_GROUP_MAX) { fbn_set_error("fbn_gemm_slabs_group: 1 <= n <= 6 descriptors"); return FBN_ERR_ARG; }
  GemmGroup G;
  G.n = n;
  const char* xe = getenv("FBN_GROUP_XCD");
  G.remap = !(xe && atoi(xe) == 0);
  int big = 0;
  double fl = -1.0;
  for (int i = 0; i < n; ++i) {
    const FbnSlabGemm& x = d[i];
    const bool ok = x.A && x.B && x.ws && x.M > 0 && x.N > 0 && x.K > 0 && x.transA && !x.transB && x.K % 64 == 0 &&
                    !(x.lda & 7) && !(x.ldb & 7) && !(x.M & 7) && !(x.N & 7) && !((uintptr_t)x.A & 15) &&
                    !((uintptr_t)x.B & 15) && !x.A2 &&
                    (!x.B2 || (!(x.nseg & 127) && !(x.ldb2 & 7) && !((uintptr_t)x.B2 & 15))) &&
                    x.ws_bytes >= (size_t)group_split(x.M, x.N, x.K) * x.M * x.N * sizeof(float) &&
                    (x.s3k0 == 0 || (!(x.s3k0 & 63) && x.K == 3 * x.s3k0 && !x.B2 && !(x.lo_a & 7) && !(x.lo_b & 7))) &&
                    (x.s3k0 > 0) == (d[0].s3k0 > 0);
    if (!ok) {
      fbn_set_error("fbn_gemm_slabs_group: each problem needs transA = 1, transB = 0, K % 64 == 0, M, N, ld % 8 == 0, "
                    "16-B aligned operands, no A2, ws >= fbn_gemm_slabs_size; split-bf16 x3 (s3k0 > 0) on every "
                    "problem or none, K = 3 s3k0, s3k0 % 64 == 0, no B2");
      return FBN_ERR_ARG;
    }
    const double f = (double)x.M * x.N * x.K;
    if (f > fl) { fl = f; big = i; }
  }
  const GemmPlan bp = plan_dma16(d[big].M, d[big].N, d[big].K);
  const bool wide = bp.waves == 8 && bp.bm == 128 && bp.bn == 128;
  const int BM = wide ? 128 : 64, BN = wide ? 128 : 64;
  long long total = 0;
  for (int i = 0; i < n; ++i) {
    const FbnSlabGemm& x = d[i];
    GemmArgs& g = G.g[i];
    g = GemmArgs{};
    g.A = x.A; g.B = x.B; g.C = x.ws; g.bias = nullptr;
    g.M = x.M; g.N = x.N; g.K = x.K; g.lda = x.lda; g.ldb = x.ldb; g.ldc = x.N;
    g.rB = {0x7fffffff, 0, 0};
    g.rC = {0x7fffffff, 0, 0};
    g.beta = 0.f;
    g.A2 = nullptr; g.lda2 = 0; g.kseg = 0x7fffffff;
    g.B2 = x.B2; g.ldb2 = x.ldb2; g.nseg = x.B2 ? x.nseg : 0x7fffffff;
    g.s3k0 = x.s3k0; g.s3_loa = x.lo_a; g.s3_lob = x.lo_b;
    g.c16 = 0;
    g.bnb_hact16 = nullptr; g.bnb_xpre = nullptr; g.bnb_mean = nullptr; g.bnb_scale = 1.f; g.bnb_part = nullptr;
    g.bnb_rpc = 1;
    g.stats = nullptr;
    g.ws = x.ws;
    const int split = group_split(x.M, x.N, x.K);
    g.kchunk = fbn_cdiv(fbn_cdiv(x.K, split), 64) * 64;
    G.tiles_n[i] = fbn_cdiv(x.N, BN);
    G.tiles[i] = G.tiles_n[i] * fbn_cdiv(x.M, BM);
    G.start[i] = (int)total;
    total += (long long)G.tiles[i] * split;
  }
  G.start[n] = (int)total;
  hipStream_t st = (hipStream_t)stream;
  const char* se = getenv("FBN_GROUP_STAGES");   // A/B knob: LDS-DMA ring depth of the group (2 or 3)
  if (d[0].s3k0 && wide)
    fbn_launch((gemm_dma16_group_kernel<128, 128, true, true, 2, 2, 4, true>), dim3((unsigned)total), dim3(512), 0,
                       st, G);
  else if (d[0].s3k0)
    fbn_launch((gemm_dma16_group_kernel<64, 64, true, true, 2, 2, 2, true>), dim3((unsigned)total), dim3(256), 0,
                       st, G);
  else if (wide && group_w4())   // A/B knob: 4 waves of 64x64 (fewer LDS fragment reads per MFMA)
    fbn_launch((gemm_dma16_group_kernel<128, 128, true, true, 2, 2, 2>), dim3((unsigned)total), dim3(256), 0,
                       st, G);
  else if (wide && se && atoi(se) == 4)
    fbn_launch((gemm_dma16_group_kernel<128, 128, true, true, 4, 2, 4>), dim3((unsigned)total), dim3(512), 0,
                       st, G);
  else if (wide && se && atoi(se) == 3)
    fbn_launch((gemm_dma16_group_kernel<128, 128, true, true, 3, 2, 4>), dim3((unsigned)total), dim3(512), 0,
                       st, G);
  else if (wide)
    fbn_launch((gemm_dma16_group_kernel<128, 128, true, true, 2, 2, 4>), dim3((unsigned)total), dim3(512), 0,
                       st, G);
  else
    fbn_launch((gemm_dma16_group_kernel<64, 64, true, true, 2, 2, 2>), dim3((unsigned)total), dim3(256), 0,
                       st, G);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

static int gemm_impl(const void* A, const void* B, float* C, const float* bias, int M, int N, int K, int lda,
                     int ldb, int ldc, int transA, int transB, int rB_seg, int rB_off0, int rB_off1, int rC_seg,
                     int rC_off0, int rC_off1, float beta, int bf16, int a16, int b16, float* stats, float* ws,
                     size_t ws_bytes, const void* A2, int lda2, int kseg, const void* B2, int ldb2, int nseg,
                     void* stream, int c16, const GemmArgs* bnb, int* slabs, const long long* s3) {
  if (slabs) *slabs = 0;
  if (M <= 0 || N <= 0) return FBN_OK;
  if (!A || !B || !C) { fbn_set_error("fbn_gemm: null operand"); return FBN_ERR_ARG; }
  // 16-B vector loads along the contiguous dimension of every operand
  if ((lda & 3) || (ldb & 3) || ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || (rB_off0 & 3) || (rB_off1 & 3) ||
      (rB_seg != 0x7fffffff && (rB_seg & 3))) {
    fbn_set_error("fbn_gemm: operands must be 16-byte aligned with ld % 4 == 0");
    return FBN_ERR_ARG;
  }
  if ((a16 || b16) && (!bf16 || (a16 && (lda & 7)) || (b16 && (ldb & 7)) || (b16 && rB_seg != 0x7fffffff))) {
    fbn_set_error("fbn_gemm: bf16 operands need bf16 compute, ld % 8 == 0 and no B remap");
    return FBN_ERR_ARG;
  }
  if (bf16 == 2 && (a16 || b16 || A2 || B2 || c16 || bnb)) {
    fbn_set_error("fbn_gemm: split-bf16 (bf16 = 2) takes fp32 operands only");
    return FBN_ERR_ARG;
  }
  GemmArgs g;
  g.A = A; g.B = B; g.C = C; g.bias = bias;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.rB = {rB_seg, rB_off0, rB_off1};
  g.rC = {rC_seg, rC_off0, rC_off1};
  g.beta = beta;
  g.A2 = A2; g.lda2 = lda2; g.kseg = kseg;
  g.B2 = B2; g.ldb2 = ldb2; g.nseg = nseg;
  g.s3k0 = s3 ? (int)s3[0] : 0;
  g.s3_loa = s3 ? s3[1] : 0;
  g.s3_lob = s3 ? s3[2] : 0;
  g.c16 = c16;
  g.bnb_hact16 = bnb ? bnb->bnb_hact16 : nullptr;
  g.bnb_xpre = bnb ? bnb->bnb_xpre : nullptr;
  g.bnb_mean = bnb ? bnb->bnb_mean : nullptr;
  g.bnb_scale = bnb ? bnb->bnb_scale : 1.f;
  g.bnb_part = bnb ? bnb->bnb_part : nullptr;
  g.bnb_rpc = bnb ? bnb->bnb_rpc : 1;
  const int bk = bf16 == 1 ? 64 : 32;     // fp32 and split-bf16 (bf16 = 2) tiles are 32 deep
  // LDS-DMA path: bf16 operands, K % 64 == 0, 16-B rows; k-major operands need their
  // M / N extent in whole 8-element chunks
  const bool dma16 = bf16 && a16 && b16 && rB_seg == 0x7fffffff && K % 64 == 0 && !(lda & 7) && !(ldb & 7) &&
                     (!transA ? true : !(M & 7)) && (transB ? true : !(N & 7)) && !getenv("FBN_GEMM_NO_DMA16");
  if ((A2 || B2) && !dma16) {
    fbn_set_error("fbn_gemm_split: split operands need the bf16 LDS-DMA path (K % 64 == 0, bf16 operands)");
    return FBN_ERR_ARG;
  }
  if (s3 && (!dma16 || A2 || B2 || c16 || bnb || stats || (s3[0] & 63) || K != 3 * s3[0] || (s3[1] & 7) ||
             (s3[2] & 7))) {
    fbn_set_error("fbn_gemm_s3: needs the bf16 LDS-DMA path (K0 % 64 == 0, ld % 8, k-major extents % 8), image "
                  "offsets % 8, no split operands / stats");
    return FBN_ERR_ARG;
  }
  GemmPlan p = dma16 ? plan_dma16(M, N, K) : plan_gemm(M, N, K, bk);
  if (slabs) {
    // slab mode (fbn_gemm_slabs): the K-slabs stay in ws for a later fbn_sum_jobs2 launch; a plan
    // with one split writes its single slab there too
    if (!dma16 || bias || stats || c16 || bnb || beta != 0.f || !ws ||
        ws_bytes < (size_t)slab_split(M, N, K) * M * N * sizeof(float)) {
      fbn_set_error("fbn_gemm_slabs: needs the bf16 LDS-DMA path, no bias / beta / stats, ws >= fbn_gemm_slabs_size");
      return FBN_ERR_ARG;
    }
    p.split = slab_split(M, N, K);
  } else if (const char* f = getenv("FBN_GEMM_FORCE")) {   // tuning sweeps only: "bm,bn,split[,waves[,stages]]"
    int a = 0, b = 0, c = 0, w = 4, sg = 0;
    if (sscanf(f, "%d,%d,%d,%d,%d", &a, &b, &c, &w, &sg) >= 3) p = {a, b, c, w, sg};
  }
  g.stats = stats;
  if (p.split > 1 && (c16 || !ws || ws_bytes < (size_t)p.split * M * N * sizeof(float))) p.split = 1;
  int per = fbn_cdiv(K, p.split);
  per = fbn_cdiv(per, bk) * bk;
  p.split = K > 0 ? fbn_cdiv(K, per) : 1;
  // stats: 64-row tiles from the MFMA epilogue (split == 1; a wave's rows inside one 64-row
  // tile) or from the split-K reduce
  if (stats && p.split == 1 && !(dma16 && p.waves == 8 && p.bm == 128)) p.bm = 64;
  g.kchunk = K > 0 ? per : 0;
  g.ws = ws;
  if (slabs && p.split == 1) {   // one slab: the kernel's plain C store into ws
    g.C = ws; g.ldc = N;
    g.rC = {0x7fffffff, 0, 0};
  }
  hipStream_t st = (hipStream_t)stream;
  const int key = (transA ? 2 : 0) | (transB ? 1 : 0);
  if (dma16) {
    switch (key) {
      case 0: launch_dma16_sel<false, true>(g, p, st); break;
      case 1: launch_dma16_sel<false, false>(g, p, st); break;
      case 2: launch_dma16_sel<true, true>(g, p, st); break;
      default: launch_dma16_sel<true, false>(g, p, st); break;
    }
  } else switch (key) {
    case 0: launch_types<false, false>(g, p, bf16, a16, b16, st); break;
    case 1: launch_types<false, true>(g, p, bf16, a16, b16, st); break;
    case 2: launch_types<true, false>(g, p, bf16, a16, b16, st); break;
    default: launch_types<true, true>(g, p, bf16, a16, b16, st); break;
  }
  FBN_CHECK_LAUNCH();
  if (slabs) {
    *slabs = p.split;
    return FBN_OK;
  }
  if (p.split > 1 && stats) {
    fbn_launch(gemm_splitk_reduce_stats, dim3(fbn_cdiv(N, 64), fbn_cdiv(M, 64)), dim3(256), 0, st, g,
                       p.split);
    FBN_CHECK_LAUNCH();
  } else if (p.split > 1) {
    const bool v4 = !(N & 3) && !(ldc & 3) && !((uintptr_t)C & 15) && (!bias || !((uintptr_t)bias & 15)) &&
                    (rC_seg == 0x7fffffff || !(rC_seg & 3)) && !(rC_off0 & 3) && !(rC_off1 & 3);
    const size_t total = v4 ? (size_t)M * N / 4 : (size_t)M * N;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    if (v4 && p.split >= 16 && total < (size_t)65536)
      fbn_launch(gemm_splitk_reduce4_wide, dim3((unsigned)((total + 15) / 16)), dim3(256), 0, st, g, p.split);
    else if (v4) fbn_launch(gemm_splitk_reduce4, dim3(blocks), dim3(256), 0, st, g, p.split);
    else fbn_launch(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, st, g, p.split);
    FBN_CHECK_LAUNCH();
  }
  return FBN_OK;
}

// The BatchNorm backward's first pass fused into its dgrad GEMM (bf16 mode, one process): C = op(A)
// op(B) (bf16 operands, f32 C, no bias) and, from the accumulators, part = the column partials of
// fbn_bn_bwd_fused ([fbn_bn_bwd_chunks(M, N)][3][N] doubles) for the matrix source G = C, the
// activation's bf16 image `hact16` (mask = its sign), the BN input `xpre` and mean -- pass part to
// fbn_bn_bwd_fused as part_pre.  Needs the plan whose waves cover exactly one row chunk each:
// fbn_gemm_bn_bwd_part_supported(M, N, K, lda, ldb, transA, transB) says whether it applies.
extern "C" int fbn_bn_bwd_chunks(int B, int C);
extern "C" int fbn_gemm_bn_bwd_part_supported(int M, int N, int K, int lda, int ldb, int transA, int transB) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || (lda & 7) || (ldb & 7) || (transA && (M & 7)) || (!transB && (N & 7)))
    return 0;
  const GemmPlan p = plan_dma16(M, N, K);
  if (p.split != 1 || p.waves != 8 || p.bm != 64 || p.bn != 128) return 0;   // 2 x 4 waves: 32 rows each
  const int nch = fbn_bn_bwd_chunks(M, N);
  // one row chunk per wave (32 rows) or two (16 rows each)
  return (N % 4 == 0 && M % 32 == 0 && (M / 32 == nch || M / 16 == nch)) ? 1 : 0;
}

extern "C" int fbn_gemm_bn_bwd_part(const void* A, const void* B, float* C, int M, int N, int K, int lda, int ldb,
                                    int ldc, int transA, int transB, const short* hact16, const float* xpre,
                                    const float* mean, float scale, double* part, void* stream) {
  if (!fbn_gemm_bn_bwd_part_supported(M, N, K, lda, ldb, transA, transB)) {
    fbn_set_error("fbn_gemm_bn_bwd_part: no plan with one row chunk per wave for this shape");
    return FBN_ERR_UNSUPPORTED;
  }
  if (!hact16 || !xpre || !mean || !part || ldc != N) {
    fbn_set_error("fbn_gemm_bn_bwd_part: hact16, xpre, mean and part are required, ldc == N");
    return FBN_ERR_ARG;
  }
  GemmArgs x;
  x.bnb_hact16 = hact16;
  x.bnb_xpre = xpre;
  x.bnb_mean = mean;
  x.bnb_scale = scale;
  x.bnb_part = part;
  x.bnb_rpc = M / fbn_bn_bwd_chunks(M, N);     // 32 or 16 (fbn_gemm_bn_bwd_part_supported)
  return gemm_impl(A, B, C, nullptr, M, N, K, lda, ldb, ldc, transA, transB, 0x7fffffff, 0, 0, 0x7fffffff, 0, 0, 0.f,
                   1, 1, 1, nullptr, nullptr, 0, nullptr, 0, 0x7fffffff, nullptr, 0, 0x7fffffff, stream, 0, &x);
}
