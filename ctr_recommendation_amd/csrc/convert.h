// bf16 images of fp32 matrices (the GEMM weight operands, the batch's item_emb_d128): the tile
// body shared by fbn_convert_bf16 (mlp.hip) and the step-head launch that runs it beside the row
// claims (fbn_adam_claim_catchup_conv, optim.hip).
#pragma once
#include "common.h"

// part: 0 = the value rounded to bf16 ("hi"), 1 = the rounding residual x - hi rounded to bf16 ("lo"):
// hi + lo carries 16 significant bits of x (the split-bf16 images of the bf16_fwd backward GEMMs);
// 2 = both images from one read, lo pst elements past hi (the operands of fbn_gemm_s3 and the
// split-bf16 x3 slab GEMMs, which read A_hi B_hi + A_hi B_lo + A_lo B_hi from them);
// dld: the destination's row stride in elements (0 = cols), so images can be laid side by side
__device__ __forceinline__ short conv_bf(float x, int part) {
  const short h = f2bf(x);
  return part ? f2bf(x - bf2f(h)) : h;
}
struct ConvJob {
  const float* src;
  short* dst;
  int rows, cols, ld, trans, seg, off0, off1, part, dld, pst;
};
// the images of four consecutive outputs: one 8-B store each (vec) or element stores
__device__ __forceinline__ void conv_store4(short* d, const f32x4& x, int part, int pst, int n, bool vec) {
  if (part < 2) {
    if (vec) {
      *reinterpret_cast<bf16x4*>(d) = (bf16x4){conv_bf(x[0], part), conv_bf(x[1], part), conv_bf(x[2], part),
                                               conv_bf(x[3], part)};
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (e < n) d[e] = conv_bf(x[e], part);
    }
    return;
  }
  bf16x4 hi, lo;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hi[e] = f2bf(x[e]);
    lo[e] = f2bf(x[e] - bf2f(hi[e]));
  }
  if (vec) {
    *reinterpret_cast<bf16x4*>(d) = hi;
    *reinterpret_cast<bf16x4*>(d + pst) = lo;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (e < n) {
        d[e] = hi[e];
        d[e + pst] = lo[e];
      }
  }
}
#define FBN_CONV_MAX 16
struct ConvJobs {
  ConvJob j[FBN_CONV_MAX];
  int tile0[FBN_CONV_MAX + 1];   // first 64x64 output tile of each job (prefix sum)
};
// One 64x64 output tile per workgroup, four consecutive outputs per thread (one 8-B bf16x4 store):
// a plain job reads four source columns at once (16-B load when they are contiguous and aligned:
// the remap offsets and seg are multiples of 4); a transposed job reads its source tile along the
// source's contiguous dimension into LDS (coalesced) and writes the output rows from LDS.
__device__ __forceinline__ void convert_tile(const ConvJobs& jobs, int njobs, int blk) {
  __shared__ float tile[64][65];
  int jb = 0;
  while (jb + 1 < njobs && blk >= jobs.tile0[jb + 1]) ++jb;
  const ConvJob J = jobs.j[jb];
  const int t = blk - jobs.tile0[jb];
  const int tcols = (J.cols + 63) / 64;
  const int i0 = (t / tcols) * 64, j0 = (t % tcols) * 64;
  const int tq = threadIdx.x & 15, tr = threadIdx.x >> 4;   // column quad, row of 16
  if (!J.trans) {
    const int j = j0 + 4 * tq;
    if (j >= J.cols) return;
    const int dld = J.dld ? J.dld : J.cols;
    const bool full = j + 4 <= J.cols;
    const int b = j + (j < J.seg ? J.off0 : J.off1);
    const bool vec = full && !(J.ld & 3) && !(b & 3) && (J.seg == 0x7fffffff || !(J.seg & 3) || j + 4 <= J.seg ||
                                                         j >= J.seg);
    f32x4 val[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {   // all loads in flight before the first store
      const int i = i0 + tr + 16 * k;
      if (i >= J.rows) { val[k] = (f32x4){0.f, 0.f, 0.f, 0.f}; continue; }
      if (vec) {
        val[k] = *reinterpret_cast<const f32x4*>(J.src + (size_t)i * J.ld + b);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int jj = j + e;
          val[k][e] = jj < J.cols ? J.src[(size_t)i * J.ld + jj + (jj < J.seg ? J.off0 : J.off1)] : 0.f;
        }
      }
    }
    const bool vst = full && !(dld & 3) && !(J.pst & 3);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = i0 + tr + 16 * k;
      if (i >= J.rows) continue;
      conv_store4(J.dst + (size_t)i * dld + j, val[k], J.part, J.pst, J.cols - j, vst);
    }
    return;
  }
  // out[i][j] = src[j][rm(i)]: lanes run along i, the source's contiguous dimension
  {
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int i = i0 + tx;
    const int b = i + (i < J.seg ? J.off0 : J.off1);
#pragma unroll
    for (int r = ty; r < 64; r += 4) {
      const int j = j0 + r;
      tile[r][tx] = (i < J.rows && j < J.cols) ? J.src[(size_t)j * J.ld + b] : 0.f;
    }
  }
  __syncthreads();
  const int j = j0 + 4 * tq;
  if (j >= J.cols) return;
  const int dld = J.dld ? J.dld : J.cols;
  const bool vst = j + 4 <= J.cols && !(dld & 3) && !(J.pst & 3);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = tr + 16 * k, i = i0 + r;
    if (i >= J.rows) continue;
    const f32x4 x = {tile[4 * tq][r], tile[4 * tq + 1][r], tile[4 * tq + 2][r], tile[4 * tq + 3][r]};
    conv_store4(J.dst + (size_t)i * dld + j, x, J.part, J.pst, J.cols - j, vst);
  }
}


// host: pack n <= FBN_CONV_MAX ConvJob records into the kernel argument; returns the 64 x 64 tile count
static inline int conv_jobs_pack(const void* jobs, int n, ConvJobs& J) {
  J.tile0[0] = 0;
  for (int i = 0; i < FBN_CONV_MAX; ++i) {
    J.j[i] = ((const ConvJob*)jobs)[i < n ? i : 0];
    J.tile0[i + 1] = J.tile0[i] + (i < n ? fbn_cdiv(J.j[i].rows, 64) * fbn_cdiv(J.j[i].cols, 64) : 0);
  }
  return J.tile0[n];
}
