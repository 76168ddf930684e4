#include <cstdlib>
// K5 epilogue / K6 / K7: bilinear pair products, BatchNorm(+ReLU+dropout), sigmoid + BCE head.
//
// Bilinear "all" (model_fibinet.py:69-79): U_f = V_f W (an MFMA GEMM, gemm.hip), then
// p_ij = V_i (.) U_j for 1 <= i < j <= 5 written straight into the compact MLP input
// c = [V_1..V_5 | p_12 .. p_45].  Pairs (0, j) are identically zero because V_0 == 0
// (:152) and their weight columns are skipped by the GEMM remap (DESIGN.md "zero columns").
// Bilinear "each" (:81-86, opt-in): p_ij = (V_i W_i) (.) V_j, U_i = V_i W_i.
//
// BatchNorm follows ATen's CPU formulas so the fp32 path matches to rounding:
//   train: two-pass mean / biased var in double, y = x * (invstd*g) + (b - mean*invstd*g),
//          running stats with momentum and unbiased var;
//   bwd:   dotp = sum (x-mean) dy, dx = (dy - sum(dy)/N - (x-mean) * dotp*invstd^2/N) * invstd * g.
// ReLU and dropout are fused into the same elementwise pass.  Dropout keep-masks come from a
// Philox4x32-10 stream keyed by (seed, offset) so the backward never stores them: the
// backward factor is recovered from the stored activation (h_act > 0 <=> kept and positive).
#include "common.h"
#include "convert.h"

// ------------------------------------------------------------------ bilinear pairs
// pair index k enumerates (i,j), 1<=i<j<=5 lexicographically: (1,2)(1,3)(1,4)(1,5)(2,3)...(4,5)
// constexpr (not __constant__) so that fully unrolled loops index register arrays with
// compile-time constants -- a runtime index would spill the arrays to scratch
__device__ constexpr int c_pi[10] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
__device__ constexpr int c_pj[10] = {1, 2, 3, 4, 2, 3, 4, 3, 4, 4};

// mode 0 ("all"): p = V_i * U_j ; mode 1 ("each"): p = U_i * V_j   (field indices 0..4 = fields 1..5)
// OutT = float, or short (bf16: the MLP input feeding bf16 GEMMs directly)
__device__ __forceinline__ void store4(float* p, const f32x4& v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void store4(short* p, const f32x4& v) {
  *reinterpret_cast<bf16x4*>(p) = (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
}
// split-bf16 images (bf16_fwd training, fbn_gemm_s3 operands): hi = bf16(x) at p, lo = bf16(x - hi)
// lo_off elements further
__device__ __forceinline__ void store_img4(short* p, long long lo_off, const f32x4& v) {
  bf16x4 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = f2bf(v[e]);
    l[e] = f2bf(v[e] - bf2f(h[e]));
  }
  *reinterpret_cast<bf16x4*>(p) = h;
  *reinterpret_cast<bf16x4*>(p + lo_off) = l;
}
// the lo image alone (its hi image written elsewhere)
__device__ __forceinline__ void store_lo4(short* p, const f32x4& v) {
  bf16x4 l;
#pragma unroll
  for (int e = 0; e < 4; ++e) l[e] = f2bf(v[e] - bf2f(f2bf(v[e])));
  *reinterpret_cast<bf16x4*>(p) = l;
}
// V from the fp32 fields (fp32 mode) or from their bf16 copy (bf16 mode: the fp32 copy is not
// written at all; U = V W is computed from the same bf16 V by the GEMM)
__device__ __forceinline__ f32x4 load_v4(const float* __restrict__ V, const short* __restrict__ V16, size_t off) {
  if (V16) {
    const bf16x4 t = *reinterpret_cast<const bf16x4*>(V16 + off);
    return (f32x4){bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3])};
  }
  return *reinterpret_cast<const f32x4*>(V + off);
}

template <typename OutT>
__global__ void pairs_fwd_kernel(const float* __restrict__ Vc, const short* __restrict__ Vc16,
                                 const float* __restrict__ U, OutT* __restrict__ c, int B, int D, int ldc, int mode) {
  const int q4 = D / 4;
  const size_t total = (size_t)B * q4;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(idx / q4), col = (int)(idx % q4) * 4;
    f32x4 v[5], u[5];
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      v[f] = load_v4(Vc, Vc16, ((size_t)b * 5 + f) * D + col);
      u[f] = *reinterpret_cast<const f32x4*>(U + ((size_t)b * 5 + f) * D + col);
    }
    OutT* out = c + (size_t)b * ldc + 5 * D + col;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const f32x4 pr = mode == 0 ? v[c_pi[k]] * u[c_pj[k]] : u[c_pi[k]] * v[c_pj[k]];
      store4(out + k * D, pr);
    }
  }
}

// bf16_fwd training, bilinear "all": the MLP input c = [V | pairs] written only as split images
// (c: [B][ldc] hi + lo B ldc further) -- the layer-1 GEMM reads c's hi image, the backward's
// split-bf16 x3 GEMMs both -- and the lo image of the fields V (vi: [B][5][D] hi, written by the
// gather as its bf16 copy; lo 5 B D further, written here)
// eight columns per thread: 16-byte image stores (half the store instructions of four)
__device__ __forceinline__ void store_img8(short* p, long long lo_off, const f32x4& a, const f32x4& b) {
  bf16x8 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = f2bf(a[e]);
    h[e + 4] = f2bf(b[e]);
    l[e] = f2bf(a[e] - bf2f(h[e]));
    l[e + 4] = f2bf(b[e] - bf2f(h[e + 4]));
  }
  *reinterpret_cast<bf16x8*>(p) = h;
  if (lo_off >= 0) *reinterpret_cast<bf16x8*>(p + lo_off) = l;
}
__global__ void pairs_fwd_img_kernel(const float* __restrict__ Vc, const float* __restrict__ U, short* __restrict__ ci,
                                     short* __restrict__ vi, int B, int D, int ldc) {
  const int q8 = D / 8;
  const size_t total = (size_t)B * q8;
  const long long clo = (long long)B * ldc, vlo = 5LL * B * D;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(idx / q8), col = (int)(idx % q8) * 8;
    f32x4 v[5][2], u[5][2];
#pragma unroll
    for (int f = 0; f < 5; ++f)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        v[f][h] = *reinterpret_cast<const f32x4*>(Vc + ((size_t)b * 5 + f) * D + col + 4 * h);
        u[f][h] = *reinterpret_cast<const f32x4*>(U + ((size_t)b * 5 + f) * D + col + 4 * h);
      }
    short* out = ci + (size_t)b * ldc + col;
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      store_img8(out + f * D, clo, v[f][0], v[f][1]);
      if (vi) {   // V's lo image only (its hi image is the gather's bf16 copy)
        bf16x8 l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = v[f][e >> 2][e & 3];
          l[e] = f2bf(x - bf2f(f2bf(x)));
        }
        *reinterpret_cast<bf16x8*>(vi + vlo + ((size_t)b * 5 + f) * D + col) = l;
      }
    }
#pragma unroll
    for (int k = 0; k < 10; ++k)
      store_img8(out + (5 + k) * D, clo, v[c_pi[k]][0] * u[c_pj[k]][0], v[c_pi[k]][1] * u[c_pj[k]][1]);
  }
}

// dV (out) = dc_V + sum of pair-grad terms that land on V ; dU (out) = pair-grad terms that land on U
// MODE (bilinear "all" = 0 / "each" = 1) is a template parameter and the pair loop is unrolled
// with compile-time indices: with runtime indices the five-field register arrays go to scratch.
template <int MODE>
__global__ void __launch_bounds__(256) pairs_bwd_kernel(const float* __restrict__ dc, const float* __restrict__ Vc,
                                                        const short* __restrict__ Vc16,
                                                        const float* __restrict__ U, float* __restrict__ dV,
                                                        float* __restrict__ dU, short* __restrict__ dU16, int B, int D,
                                                        int ldc, short* __restrict__ dUi) {
  const int q4 = D / 4;
  const size_t total = (size_t)B * q4;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(idx / q4), col = (int)(idx % q4) * 4;
    f32x4 v[5], u[5], gv[5], gu[5];
    const float* dcb = dc + (size_t)b * ldc + col;
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      v[f] = load_v4(Vc, Vc16, ((size_t)b * 5 + f) * D + col);
      u[f] = *reinterpret_cast<const f32x4*>(U + ((size_t)b * 5 + f) * D + col);
      gv[f] = *reinterpret_cast<const f32x4*>(dcb + f * D);
      gu[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    constexpr int PI[10] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
    constexpr int PJ[10] = {1, 2, 3, 4, 2, 3, 4, 3, 4, 4};
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const f32x4 g = *reinterpret_cast<const f32x4*>(dcb + (5 + k) * D);
      if constexpr (MODE == 0) { gv[PI[k]] += g * u[PJ[k]]; gu[PJ[k]] += g * v[PI[k]]; }
      else { gu[PI[k]] += g * v[PJ[k]]; gv[PJ[k]] += g * u[PI[k]]; }
    }
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      *reinterpret_cast<f32x4*>(dV + ((size_t)b * 5 + f) * D + col) = gv[f];
      if (dU) *reinterpret_cast<f32x4*>(dU + ((size_t)b * 5 + f) * D + col) = gu[f];
      if (dU16) store4(dU16 + ((size_t)b * 5 + f) * D + col, gu[f]);
      if (dUi) store_img4(dUi + ((size_t)b * 5 + f) * D + col, 5LL * B * D, gu[f]);   // split images (bf16_fwd)
    }
  }
}

// ------------------------------------------------------------------ column statistics
// Partial column sums over a chunk of rows: part[chunk][c] (double).  mode 0: sum x ;
// mode 1: sum (x - mean[c])^2.  Block = 256 threads covering 64 columns x 4 row lanes.
__global__ void colstat_partial_kernel(const float* __restrict__ X, int B, int C, int ldx, int rows_per_chunk,
                                       const double* __restrict__ mean, double* __restrict__ part, int mode) {
  __shared__ double red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(B, r0 + rows_per_chunk);
  double s = 0.0;
  if (col < C) {
    const double mu = mode ? mean[col] : 0.0;
    for (int r = r0 + rl; r < r1; r += 4) {
      const double x = (double)X[(size_t)r * ldx + col];
      s += mode ? (x - mu) * (x - mu) : x;
    }
  }
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && col < C)
    part[(size_t)blockIdx.y * C + col] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// out[c] = sum_k part[k][c]: one wave per column, lanes stride the chunks, fixed shuffle tree
// (deterministic; the chunk loads are independent instead of a serial dependent chain)
__global__ void chunk_reduce_kernel(const double* part, int nchunk, int C, double* out) {
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  double s = 0.0;
  for (int k = lane; k < nchunk; k += 64) s += part[(size_t)k * C + c];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[c] = s;
}

__global__ void bn_mean_kernel(const double* sum, double ntot, int C, double* mean) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) mean[c] = sum[c] / ntot;
}

// finalize BN train stats from the (global) sum of squared deviations: invstd, float mean,
// running-stat update (momentum, unbiased var)
__global__ void bn_finalize_kernel(const double* m2, const double* mean_d, double ntot, int C, float* mean,
                                   float* invstd, float* run_mean, float* run_var, float momentum, float eps,
                                   int update_running) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double s = m2[c];
  const float var_b = (float)(s / ntot);
  mean[c] = (float)mean_d[c];
  invstd[c] = 1.f / sqrtf(var_b + eps);
  if (update_running) {
    const float unb = ntot > 1.0 ? (float)(s / (ntot - 1.0)) : var_b;
    run_mean[c] = momentum * (float)mean_d[c] + (1.f - momentum) * run_mean[c];
    run_var[c] = momentum * unb + (1.f - momentum) * run_var[c];
  }
}

__global__ void bn_eval_params_kernel(const float* run_mean, const float* run_var, float* mean, float* invstd,
                                      int C, float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = run_mean[c];
  invstd[c] = 1.f / sqrtf(run_var[c] + eps);
}

// y = relu(x*alpha + beta'), alpha = invstd*g, beta' = b - mean*alpha ; then dropout (train)
__global__ void bn_act_fwd_kernel(const float* __restrict__ X, float* __restrict__ Y, int B, int C,
                                  const float* __restrict__ mean, const float* __restrict__ invstd,
                                  const float* __restrict__ g, const float* __restrict__ bta, float p_drop,
                                  const unsigned long long* __restrict__ rng, unsigned stream_id,
                                  unsigned char* __restrict__ mask_out, const unsigned char* __restrict__ mask_in,
                                  short* __restrict__ Y16) {
  const size_t total4 = (size_t)B * C / 4;
  const float keep = 1.f - p_drop;
  const float scale = p_drop > 0.f ? 1.0f / keep : 1.f;
  uint32_t k0 = 0, k1 = 0, off = 0;
  if (rng) { k0 = (uint32_t)rng[0]; k1 = (uint32_t)(rng[0] >> 32); off = (uint32_t)rng[1]; }
  for (size_t i4 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i4 < total4; i4 += (size_t)gridDim.x * blockDim.x) {
    const size_t i = i4 * 4;
    const int col = (int)(i % C);
    f32x4 x = *reinterpret_cast<const f32x4*>(X + i);
    f32x4 y;
    float um[4] = {1.f, 1.f, 1.f, 1.f};
    if (p_drop > 0.f && !mask_in) {
      const Philox4 r = philox4x32_10((uint32_t)i4, (uint32_t)(i4 >> 32), stream_id, off, k0, k1);
      um[0] = u01(r.x); um[1] = u01(r.y); um[2] = u01(r.z); um[3] = u01(r.w);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float alpha = invstd[col + e] * g[col + e];
      const float bp = bta[col + e] - mean[col + e] * alpha;
      float v = fmaxf(x[e] * alpha + bp, 0.f);
      if (p_drop > 0.f) {
        const bool kept = mask_in ? mask_in[i + e] != 0 : um[e] < keep;
        v = kept ? v * scale : 0.f;
        if (mask_out) mask_out[i + e] = kept ? 1 : 0;
      }
      y[e] = v;
    }
    *reinterpret_cast<f32x4*>(Y + i) = y;
    if (Y16) store4(Y16 + i, y);
  }
}

struct HeadArgs {
  const float* w; const float* bias;
  float* logits; float* probs; const float* labels; float* loss_terms; float* gout;
  float denom;
};
// Linear(C,1) + sigmoid + BCE terms + dL/dlogit of one row from the wave's lane partials
// (lane q holds columns 4q..4q+3): shared by head_fwd_kernel and the fused BN2 + head kernel
// The row's outputs from its summed dot product s (one lane)
__device__ __forceinline__ float head_lane(float s, int row, const HeadArgs& h) {
  float go = 0.f;
  const float o = s + h.bias[0];
  const float pr = 1.f / (1.f + expf(-o));
  if (h.logits) h.logits[row] = o;
  if (h.probs) h.probs[row] = pr;
  if (h.labels) {
    const float t = h.labels[row];
    const float lp = fmaxf(logf(pr), -100.f), l1p = fmaxf(logf(1.f - pr), -100.f);
    if (h.loss_terms) h.loss_terms[row] = -(t * lp + (1.f - t) * l1p);
    if (h.gout) {
      const float gp = ((pr - t) / fmaxf((1.f - pr) * pr, 1e-12f)) / h.denom;
      go = gp * (1.f - pr) * pr;
      h.gout[row] = go;
    }
  }
  return go;
}
__device__ __forceinline__ float head_row(float s, int row, int lane, const HeadArgs& h) {
  s = wave_sum(s);
  return lane == 0 ? head_lane(s, row, h) : 0.f;   // dL/dlogit of the row on lane 0
}

// Column-blocked form: block = 64 column quads (256 columns) x 4 row lanes over a chunk of rows,
// the per-column affine (alpha, beta') computed once per thread, no index division.  Same
// Philox counter (flat quad index) and arithmetic as bn_act_fwd_kernel.
// HEAD (C == 256, one column block): each wave holds whole rows, so the head Linear(256,1) +
// sigmoid + BCE of src/model_fibinet.py:134,136 runs on the activations still in registers
// (the same lane partials and reduction as head_fwd_kernel: bit-identical, one launch fewer).
// BWD (HEAD, 1024 threads, one row per wave): the BN2 backward's column partials of the rank-1
// source (fbn_bn_bwd_fused's first pass, bn_bwd_partial4) from the row's dL/dlogit, activation
// and input while they are in registers: bpart[chunk][3][C] = {sum dy, sum (x-mean) dy,
// sum gout*h}, dy = gout*w*(h > 0)*bscale, the same float products and f64 sums; waves folded in
// a fixed order (deterministic).
template <bool HEAD, int NT = 256, bool BWD = false>
__global__ void __launch_bounds__(NT) bn_act_fwd2_kernel(const float* __restrict__ X, float* __restrict__ Y, int B,
                                                         int C, int rows_per_chunk, const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ g, const float* __restrict__ bta,
                                                         float p_drop, const unsigned long long* __restrict__ rng,
                                                         unsigned stream_id, unsigned char* __restrict__ mask_out,
                                                         const unsigned char* __restrict__ mask_in,
                                                         short* __restrict__ Y16, HeadArgs head,
                                                         double* __restrict__ bpart = nullptr, float bscale = 1.f,
                                                         long long y16_lo = 0) {
  FBN_MAIN_PRIO();
  constexpr int NWV = NT / 64;
  const int q = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + q * 4;
  if (c >= C) return;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(B, r0 + rows_per_chunk);
  const float keep = 1.f - p_drop;
  const float scale = p_drop > 0.f ? 1.0f / keep : 1.f;
  uint32_t k0 = 0, k1 = 0, off = 0;
  if (rng) { k0 = (uint32_t)rng[0]; k1 = (uint32_t)(rng[0] >> 32); off = (uint32_t)rng[1]; }
  float alpha[4], bp[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    alpha[e] = invstd[c + e] * g[c + e];
    bp[e] = bta[c + e] - mean[c + e] * alpha[e];
  }
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  for (int r = r0 + rl; r < r1; r += NWV) {
    const size_t i = (size_t)r * C + c, i4 = i >> 2;
    const f32x4 x = *reinterpret_cast<const f32x4*>(X + i);
    float um[4] = {1.f, 1.f, 1.f, 1.f};
    if (p_drop > 0.f && !mask_in) {
      const Philox4 rr = philox4x32_10((uint32_t)i4, (uint32_t)(i4 >> 32), stream_id, off, k0, k1);
      um[0] = u01(rr.x); um[1] = u01(rr.y); um[2] = u01(rr.z); um[3] = u01(rr.w);
    }
    f32x4 y;
    unsigned mk = 0u;   // the four mask bytes, one 32-bit store
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = fmaxf(x[e] * alpha[e] + bp[e], 0.f);
      if (p_drop > 0.f) {
        const bool kept = mask_in ? mask_in[i + e] != 0 : um[e] < keep;
        v = kept ? v * scale : 0.f;
        mk |= (kept ? 1u : 0u) << (8 * e);
      }
      y[e] = v;
    }
    if (p_drop > 0.f && mask_out) *reinterpret_cast<unsigned*>(mask_out + i) = mk;
    if (Y) *reinterpret_cast<f32x4*>(Y + i) = y;
    if (Y16) {
      if (y16_lo) store_img4(Y16 + i, y16_lo, y);   // split images (bf16_fwd): hi here, lo y16_lo further
      else store4(Y16 + i, y);
    }
    if (HEAD) {
      const f32x4 ww = *reinterpret_cast<const f32x4*>(head.w + c);
      const float go = head_row(y[0] * ww[0] + y[1] * ww[1] + y[2] * ww[2] + y[3] * ww[3], r, q, head);
      if (BWD) {
        const float gv = __shfl(go, 0, 64);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = gv * ww[e];
          const float dy = y[e] > 0.f ? d * bscale : 0.f;
          s0[e] += dy;
          s1[e] += (double)((x[e] - mean[c + e]) * dy);
          s2[e] += (double)(gv * y[e]);
        }
      }
    }
  }
  if (BWD) {
    // C == 256: lane q holds columns 4q..4q+3; fold the NWV waves per quantity through LDS
    __shared__ double red[NWV][256];
    double* pp = bpart + (size_t)blockIdx.y * 3 * C;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double* sk = k == 0 ? s0 : (k == 1 ? s1 : s2);
#pragma unroll
      for (int e = 0; e < 4; ++e) red[rl][q * 4 + e] = sk[e];
      __syncthreads();
      if (threadIdx.x < 256) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NWV; ++w) t += red[w][threadIdx.x];
        pp[(size_t)k * C + threadIdx.x] = t;
      }
      __syncthreads();
    }
  }
}

// bn_act_fwd2_kernel<false> with FOUR rows per wave and iteration (rows r0 + rl + 4j of a 16-row
// chunk): the four rows' loads are issued before any row's arithmetic.  Same operations per
// element, same outputs.
__global__ void __launch_bounds__(256) bn_act_fwd4r_kernel(const float* __restrict__ X, float* __restrict__ Y, int B,
                                                           int C, int rows_per_chunk, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ g, const float* __restrict__ bta,
                                                           float p_drop, const unsigned long long* __restrict__ rng,
                                                           unsigned stream_id, unsigned char* __restrict__ mask_out,
                                                           const unsigned char* __restrict__ mask_in,
                                                           short* __restrict__ Y16, long long y16_lo) {
  FBN_MAIN_PRIO();
  const int q = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + q * 4;
  if (c >= C) return;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(B, r0 + rows_per_chunk);
  const float keep = 1.f - p_drop;
  const float scale = p_drop > 0.f ? 1.0f / keep : 1.f;
  uint32_t k0 = 0, k1 = 0, off = 0;
  if (rng) { k0 = (uint32_t)rng[0]; k1 = (uint32_t)(rng[0] >> 32); off = (uint32_t)rng[1]; }
  float alpha[4], bp[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    alpha[e] = invstd[c + e] * g[c + e];
    bp[e] = bta[c + e] - mean[c + e] * alpha[e];
  }
  for (int rb = r0 + rl; rb < r1; rb += 16) {
    f32x4 x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = rb + 4 * j;
      x[j] = r < r1 ? *reinterpret_cast<const f32x4*>(X + (size_t)r * C + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = rb + 4 * j;
      if (r >= r1) break;
      const size_t i = (size_t)r * C + c, i4 = i >> 2;
      float um[4] = {1.f, 1.f, 1.f, 1.f};
      if (p_drop > 0.f && !mask_in) {
        const Philox4 rr = philox4x32_10((uint32_t)i4, (uint32_t)(i4 >> 32), stream_id, off, k0, k1);
        um[0] = u01(rr.x); um[1] = u01(rr.y); um[2] = u01(rr.z); um[3] = u01(rr.w);
      }
      f32x4 y;
      unsigned mk = 0u;   // the four mask bytes, one 32-bit store
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = fmaxf(x[j][e] * alpha[e] + bp[e], 0.f);
        if (p_drop > 0.f) {
          const bool kept = mask_in ? mask_in[i + e] != 0 : um[e] < keep;
          v = kept ? v * scale : 0.f;
          mk |= (kept ? 1u : 0u) << (8 * e);
        }
        y[e] = v;
      }
      if (p_drop > 0.f && mask_out) *reinterpret_cast<unsigned*>(mask_out + i) = mk;
      if (Y) *reinterpret_cast<f32x4*>(Y + i) = y;
      if (Y16) {
        if (y16_lo) store_img4(Y16 + i, y16_lo, y);
        else store4(Y16 + i, y);
      }
    }
  }
}

// The same fused BN2 + ReLU + dropout + head + BN2-backward first pass (C == 256) with FOUR rows
// per wave: 4 waves per row chunk, wave rl takes rows r0 + rl + 4k in order (bn_bwd_partial4's
// rows and accumulation order, so its partials equal that kernel's bit for bit).  The four rows'
// loads and Philox draws are independent, their dot products are reduced side by side with
// wave_sum's butterfly (the same order per row), and lanes 0..3 finish rows 0..3 at once
// (head_lane, the same operations as head_row's lane 0) -- one latency chain per four rows
// instead of one per row, and one LDS fold of 4 waves per chunk instead of 3 of 16.
__global__ void __launch_bounds__(256) bn_act_head_bwd4_kernel(
    const float* __restrict__ X, float* __restrict__ Y, int B, int C, int rows_per_chunk,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ g,
    const float* __restrict__ bta, float p_drop, const unsigned long long* __restrict__ rng, unsigned stream_id,
    unsigned char* __restrict__ mask_out, const unsigned char* __restrict__ mask_in, HeadArgs head,
    double* __restrict__ bpart, float bscale) {
  FBN_MAIN_PRIO();
  __shared__ double red[3][4][256];
  const int q = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = q * 4;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(B, r0 + rows_per_chunk);
  const float keep = 1.f - p_drop;
  const float scale = p_drop > 0.f ? 1.0f / keep : 1.f;
  uint32_t k0 = 0, k1 = 0, off = 0;
  if (rng) { k0 = (uint32_t)rng[0]; k1 = (uint32_t)(rng[0] >> 32); off = (uint32_t)rng[1]; }
  float alpha[4], bp[4], mu[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    alpha[e] = invstd[c + e] * g[c + e];
    bp[e] = bta[c + e] - mean[c + e] * alpha[e];
    mu[e] = mean[c + e];
  }
  const f32x4 ww = *reinterpret_cast<const f32x4*>(head.w + c);
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  for (int rb = r0 + rl; rb < r1; rb += 16) {   // wave-uniform bound
    f32x4 x[4], y[4];
    float sp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = rb + 4 * j;
      x[j] = r < r1 ? *reinterpret_cast<const f32x4*>(X + (size_t)r * C + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = rb + 4 * j;
      const bool ok = r < r1;
      const size_t i = (size_t)r * C + c, i4 = i >> 2;
      float um[4] = {1.f, 1.f, 1.f, 1.f};
      if (p_drop > 0.f && !mask_in) {
        const Philox4 rr = philox4x32_10((uint32_t)i4, (uint32_t)(i4 >> 32), stream_id, off, k0, k1);
        um[0] = u01(rr.x); um[1] = u01(rr.y); um[2] = u01(rr.z); um[3] = u01(rr.w);
      }
      unsigned mk = 0u;   // the four mask bytes, one 32-bit store
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = fmaxf(x[j][e] * alpha[e] + bp[e], 0.f);
        if (p_drop > 0.f) {
          const bool kept = mask_in ? (ok && mask_in[i + e] != 0) : um[e] < keep;
          v = kept ? v * scale : 0.f;
          mk |= (kept ? 1u : 0u) << (8 * e);
        }
        y[j][e] = v;
      }
      if (p_drop > 0.f && mask_out && ok) *reinterpret_cast<unsigned*>(mask_out + i) = mk;
      if (Y && ok) *reinterpret_cast<f32x4*>(Y + i) = y[j];
      sp[j] = y[j][0] * ww[0] + y[j][1] * ww[1] + y[j][2] * ww[2] + y[j][3] * ww[3];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) sp[j] += __shfl_xor(sp[j], o, 64);
    }
    float go = 0.f;
    if (q < 4) {
      const float sq = q == 0 ? sp[0] : (q == 1 ? sp[1] : (q == 2 ? sp[2] : sp[3]));
      const int row = rb + 4 * q;
      if (row < r1) go = head_lane(sq, row, head);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gv = __shfl(go, j, 64);
      if (rb + 4 * j < r1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = gv * ww[e];
          const float dy = y[j][e] > 0.f ? d * bscale : 0.f;
          s0[e] += dy;
          s1[e] += (double)((x[j][e] - mu[e]) * dy);
          s2[e] += (double)(gv * y[j][e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][rl][c + e] = s0[e];
    red[1][rl][c + e] = s1[e];
    red[2][rl][c + e] = s2[e];
  }
  __syncthreads();
  double* pp = bpart + (size_t)blockIdx.y * 3 * C;
#pragma unroll
  for (int k = 0; k < 3; ++k)
    pp[(size_t)k * C + threadIdx.x] =
        red[k][0][threadIdx.x] + red[k][1][threadIdx.x] + red[k][2][threadIdx.x] + red[k][3][threadIdx.x];
}

// ------------------------------------------------------------------ BN backward
// dy[b][c] = G[b][c] * fac(hact)  (matrix source)  or  gvec[b] * w[c] * fac(hact)  (rank-1 head source)
// fac = scale if hact > 0 else 0  (ReLU-after-BN + dropout recovered from the stored activation)
struct BnBwdSrc {
  const float* G;      // [B][C] or null
  const float* gvec;   // [B] (rank-1 source)
  const float* w;      // [C]
  const float* hact;   // [B][C]
  float scale;
  const short* hact16; // [B][C] bf16 image of the activation, read instead of hact when hact is null
                       // (matrix source only: the mask needs just the sign, bf16 keeps it)
  long long dx16_lo;   // > 0: the bf16 output is split images (hi, lo this many elements further)
};
// the activation's "> 0" test on 4 columns, from the f32 activation or its bf16 image (a bf16
// bit pattern read as a signed short is > 0 exactly when the value is > +0)
__device__ __forceinline__ f32x4 bn_act4(const BnBwdSrc& s, size_t i) {
  if (s.hact) return *reinterpret_cast<const f32x4*>(s.hact + i);
  const uint2 u = *reinterpret_cast<const uint2*>(s.hact16 + i);
  return (f32x4){(short)(u.x & 0xffffu) > 0 ? 1.f : 0.f, (short)(u.x >> 16) > 0 ? 1.f : 0.f,
                 (short)(u.y & 0xffffu) > 0 ? 1.f : 0.f, (short)(u.y >> 16) > 0 ? 1.f : 0.f};
}
__device__ __forceinline__ float bn_dy(const BnBwdSrc& s, int b, int c, int C) {
  const size_t i = (size_t)b * C + c;
  const float d = s.G ? s.G[i] : s.gvec[b] * s.w[c];
  return s.hact[i] > 0.f ? d * s.scale : 0.f;
}

// partials over row chunks: part0 = sum dy, part1 = sum (x-mean)*dy, part2 (rank-1 only) = sum gvec*hact
__global__ void bn_bwd_partial_kernel(BnBwdSrc s, const float* __restrict__ Xpre, const float* __restrict__ mean,
                                      int B, int C, int rows_per_chunk, double* part) {
  __shared__ double red[3][4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(B, r0 + rows_per_chunk);
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const float mu = mean[c];
    for (int r = r0 + rl; r < r1; r += 4) {
      const float dy = bn_dy(s, r, c, C);
      s0 += dy;
      s1 += (double)((Xpre[(size_t)r * C + c] - mu) * dy);
      if (!s.G) s2 += (double)(s.gvec[r] * s.hact[(size_t)r * C + c]);
    }
  }
  red[0][rl][threadIdx.x & 63] = s0;
  red[1][rl][threadIdx.x & 63] = s1;
  red[2][rl][threadIdx.x & 63] = s2;
  __syncthreads();
  if (rl == 0 && c < C) {
    const int t = threadIdx.x;
    double* pp = part + (size_t)blockIdx.y * 3 * C;
    pp[c] = red[0][0][t] + red[0][1][t] + red[0][2][t] + red[0][3][t];
    pp[C + c] = red[1][0][t] + red[1][1][t] + red[1][2][t] + red[1][3][t];
    pp[2 * C + c] = red[2][0][t] + red[2][1][t] + red[2][2][t] + red[2][3][t];
  }
}

// Vectorised partials for the fused backward: 4 columns per lane (256 columns per block), the
// block's 4 waves take rows r0+w, r0+w+4, ...; f64 accumulation; part[chunk][3][C].
__global__ void __launch_bounds__(256) bn_bwd_partial4_kernel(BnBwdSrc s, const float* __restrict__ Xpre,
                                                              const float* __restrict__ mean, int B, int C,
                                                              int rows_per_chunk, double* __restrict__ part) {
  FBN_MAIN_PRIO();
  __shared__ double red[3][4][256];
  const int q = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + q * 4;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(B, r0 + rows_per_chunk);
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (c < C) {
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + c);
    const f32x4 ww = s.G ? (f32x4){0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(s.w + c);
#pragma unroll 4
    for (int r = r0 + rl; r < r1; r += 4) {
      const size_t i = (size_t)r * C + c;
      const f32x4 h = bn_act4(s, i);
      const f32x4 x = *reinterpret_cast<const f32x4*>(Xpre + i);
      f32x4 d;
      float gv = 0.f;
      if (s.G) d = *reinterpret_cast<const f32x4*>(s.G + i);
      else { gv = s.gvec[r]; d = (f32x4){gv * ww[0], gv * ww[1], gv * ww[2], gv * ww[3]}; }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dy = h[e] > 0.f ? d[e] * s.scale : 0.f;
        s0[e] += dy;
        s1[e] += (double)((x[e] - mu[e]) * dy);
        if (!s.G) s2[e] += (double)(gv * h[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][rl][q * 4 + e] = s0[e];
    red[1][rl][q * 4 + e] = s1[e];
    red[2][rl][q * 4 + e] = s2[e];
  }
  __syncthreads();
  // 768 outputs per block: thread t writes entries t, t+256, t+512 of {sum dy | sum (x-mu)dy | sum gvec*hact}
  double* pp = part + (size_t)blockIdx.y * 3 * C;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int cc = blockIdx.x * 256 + threadIdx.x;
    if (cc < C)
      pp[(size_t)k * C + cc] = red[k][0][threadIdx.x] + red[k][1][threadIdx.x] + red[k][2][threadIdx.x] +
                               red[k][3][threadIdx.x];
  }
}

// red = {sum dy, sum (x-mean) dy, sum gvec*hact} (global sums, [3][C]).
// coef[c] = {gm = sum dy / N, k = dotp * invstd^2 / N}; dgamma = dotp*invstd, dbeta = sum dy; dw = sum gvec*hact
__global__ void bn_bwd_finalize_kernel(const double* red, int C, double ntot, const float* invstd, float* coef,
                                       float* dgamma, float* dbeta, float* dw) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = invstd[c];
  const float sdy = (float)red[c], dotp = (float)red[C + c];
  coef[c] = sdy / (float)ntot;
  coef[C + c] = dotp * is * is / (float)ntot;
  if (dgamma) dgamma[c] = dotp * is;
  if (dbeta) dbeta[c] = sdy;
  if (dw) dw[c] = (float)red[2 * C + c];
}

__global__ void bn_bwd_apply_kernel(BnBwdSrc s, const float* __restrict__ Xpre, const float* __restrict__ mean,
                                    const float* __restrict__ invstd, const float* __restrict__ g,
                                    const float* __restrict__ coef, float* __restrict__ dX, short* __restrict__ dX16,
                                    int B, int C) {
  const size_t total = (size_t)B * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / C), c = (int)(i % C);
    const float dy = bn_dy(s, b, c, C);
    const float v = (dy - coef[c] - (Xpre[i] - mean[c]) * coef[C + c]) * invstd[c] * g[c];
    dX[i] = v;
    if (dX16) dX16[i] = f2bf(v);
  }
}

// ------------------------------------------------------------------ column sums (bias grads)
__global__ void colsum_partial_kernel(const float* __restrict__ X, int B, int C, int ldx, int rows_per_chunk,
                                      float* __restrict__ part) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(B, r0 + rows_per_chunk);
  float s = 0.f;
  if (c < C)
    for (int r = r0 + rl; r < r1; r += 4) s += X[(size_t)r * ldx + c];
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < C)
    part[(size_t)blockIdx.y * C + c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}
__global__ void colsum_final_kernel(const float* part, int nchunk, int C, float* out, float beta) {
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  float s = 0.f;
  for (int k = lane; k < nchunk; k += 64) s += part[(size_t)k * C + c];
  s = wave_sum(s);
  if (lane == 0) out[c] = beta != 0.f ? out[c] * beta + s : s;
}

// ------------------------------------------------------------------ single-process BN fusions
// Forward statistics from the GEMM's per-64-row-tile (sum, M2) partials in ONE launch: per
// column one wave sums the tile sums (-> mean), then Chan's merge of the tile M2s about that
// mean, then the finalize.  Same f64 operations in the same order as fbn_bn_tile_stats x2 +
// fbn_bn_mean + fbn_bn_finalize (the multi-rank path, which all-reduces in between).
__global__ void bn_tile_finalize_kernel(const float* __restrict__ part, int T, int C, int M, int tile_rows,
                                        double ntot, float* mean, float* invstd, float* run_mean, float* run_var,
                                        float momentum, float eps, int update_running) {
  FBN_MAIN_PRIO();
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  double s = 0.0, q = 0.0, mu;
  if (T <= 256) {
    // one round trip: every (sum, M2) pair of this lane's tiles loaded at once and kept in
    // registers for both passes (same operations, same order as the loop below)
    float2 sm[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = lane + 64 * j;
      sm[j] = t < T ? *reinterpret_cast<const float2*>(part + ((size_t)t * C + c) * 2) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (lane + 64 * j < T) s += (double)sm[j].x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    mu = s / ntot;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = lane + 64 * j;
      if (t < T) {
        const int nt = min(tile_rows, M - t * tile_rows);
        const double dm = (double)sm[j].x / nt - mu;
        q += (double)sm[j].y + nt * dm * dm;
      }
    }
  } else {
    for (int t = lane; t < T; t += 64) s += (double)part[((size_t)t * C + c) * 2];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    mu = s / ntot;
    for (int t = lane; t < T; t += 64) {
      const float S = part[((size_t)t * C + c) * 2], M2 = part[((size_t)t * C + c) * 2 + 1];
      const int nt = min(tile_rows, M - t * tile_rows);
      const double dm = (double)S / nt - mu;
      q += (double)M2 + nt * dm * dm;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  if (lane == 0) {
    const float var_b = (float)(q / ntot);
    mean[c] = (float)mu;
    invstd[c] = 1.f / sqrtf(var_b + eps);
    if (update_running) {
      const float unb = ntot > 1.0 ? (float)(q / (ntot - 1.0)) : var_b;
      run_mean[c] = momentum * (float)mu + (1.f - momentum) * run_mean[c];
      run_var[c] = momentum * unb + (1.f - momentum) * run_var[c];
    }
  }
}

// SyncBN (multi-GPU) forward statistics with ONE all-reduce per layer: each rank turns its
// tile partials into raw f64 moments {sum x, sum x^2} (sum x^2 = sum_t M2_t + S_t^2 / n_t);
// after the all-reduce, M2 = sum x^2 - sum x * mean in f64 (relative error ~1e-16 * mean^2/var).
__global__ void bn_tile_moments_kernel(const float* __restrict__ part, int T, int C, int M, int tile_rows,
                                       double* __restrict__ out) {
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  double s1 = 0.0, s2 = 0.0;
  for (int t = lane; t < T; t += 64) {
    const double S = part[((size_t)t * C + c) * 2], M2 = part[((size_t)t * C + c) * 2 + 1];
    const int nt = min(tile_rows, M - t * tile_rows);
    s1 += S;
    s2 += M2 + S * S / nt;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if (lane == 0) { out[c] = s1; out[C + c] = s2; }
}

__global__ void bn_moments_finalize_kernel(const double* __restrict__ mom, double ntot, int C, float* mean,
                                           float* invstd, float* run_mean, float* run_var, float momentum, float eps,
                                           int update_running) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double mu = mom[c] / ntot;
  double q = mom[C + c] - mom[c] * mu;
  if (q < 0.0) q = 0.0;
  const float var_b = (float)(q / ntot);
  mean[c] = (float)mu;
  invstd[c] = 1.f / sqrtf(var_b + eps);
  if (update_running) {
    const float unb = ntot > 1.0 ? (float)(q / (ntot - 1.0)) : var_b;
    run_mean[c] = momentum * (float)mu + (1.f - momentum) * run_mean[c];
    run_var[c] = momentum * unb + (1.f - momentum) * run_var[c];
  }
}

// Backward: chunk reduce of the three partial sums + the finalize of bn_bwd_finalize_kernel,
// one wave per column (chunk_reduce_kernel's order).
// 64 columns per 1024-thread block: lanes run along the columns (coalesced rows of the partial
// slab), the 16 waves stride over the chunks, then a fixed-order fold across the waves
// (deterministic) and the finalize.
__global__ void __launch_bounds__(1024) bn_bwd_reduce_finalize_kernel(const double* __restrict__ part, int nchunk,
                                                                      int C, double ntot,
                                                                      const float* __restrict__ invstd, float* coef,
                                                                      float* dgamma, float* dbeta, float* dw) {
  __shared__ double red[16][3][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double r0 = 0.0, r1 = 0.0, r2 = 0.0;
  if (c < C) {
    for (int k = w; k < nchunk; k += 16) {
      const double* pk = part + (size_t)k * 3 * C + c;
      r0 += pk[0];
      r1 += pk[C];
      r2 += pk[2 * C];
    }
  }
  red[w][0][lane] = r0;
  red[w][1][lane] = r1;
  red[w][2][lane] = r2;
  __syncthreads();
  if (w == 0 && c < C) {
    double r[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 3; ++q)
      for (int k = 0; k < 16; ++k) r[q] += red[k][q][lane];
    const float is = invstd[c];
    const float sdy = (float)r[0], dotp = (float)r[1];
    coef[c] = sdy / (float)ntot;
    coef[C + c] = dotp * is * is / (float)ntot;
    if (dgamma) dgamma[c] = dotp * is;
    if (dbeta) dbeta[c] = sdy;
    if (dw) dw[c] = (float)r[2];
  }
}

// Same reduction on NC columns per block (C / NC workgroups instead of C / 64): 64 chunk streams
// per column, NC lanes reading one row segment of the slab; then 48 NC threads fold the 64
// streams of one (quantity, column) in fixed order (deterministic) and NC finalize.  The fold's
// order does not depend on NC, so every NC gives the same bits (NC = 16 by default; FBN_BN_REDUCE_NC
// = 4 / 8: more, smaller workgroups -- A/B knob).
template <int NC>
__global__ void __launch_bounds__(64 * NC) bn_bwd_reduce_finalize16_kernel(const double* __restrict__ part, int nchunk,
                                                                           int C, double ntot,
                                                                           const float* __restrict__ invstd,
                                                                           float* coef, float* dgamma, float* dbeta,
                                                                           float* dw) {
  FBN_MAIN_PRIO();
  __shared__ double red[64][3][NC];
  __shared__ double red2[16][3][NC];
  __shared__ double tot[3][NC];
  const int col = threadIdx.x % NC, str = threadIdx.x / NC;
  const int c = blockIdx.x * NC + col;
  double r0 = 0.0, r1 = 0.0, r2 = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int k = str; k < nchunk; k += 64) {
      const double* pk = part + (size_t)k * 3 * C + c;
      r0 += pk[0];
      r1 += pk[C];
      r2 += pk[2 * C];
    }
  }
  red[str][0][col] = r0;
  red[str][1][col] = r1;
  red[str][2][col] = r2;
  __syncthreads();
  // fixed-order two-level fold of the 64 chunk-stride partials: 16 groups of 4, then the 16
  if (threadIdx.x < 48 * NC) {
    const int j = threadIdx.x / (3 * NC), qc = threadIdx.x % (3 * NC), q = qc / NC, cc = qc % NC;
    red2[j][q][cc] = ((red[4 * j][q][cc] + red[4 * j + 1][q][cc]) + red[4 * j + 2][q][cc]) + red[4 * j + 3][q][cc];
  }
  __syncthreads();
  if (threadIdx.x < 3 * NC) {
    const int q = threadIdx.x / NC, cc = threadIdx.x % NC;
    double r = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) r += red2[k][q][cc];
    tot[q][cc] = r;
  }
  __syncthreads();
  if (threadIdx.x < NC && c < C) {
    const float is = invstd[c];
    const float sdy = (float)tot[0][col], dotp = (float)tot[1][col];
    coef[c] = sdy / (float)ntot;
    coef[C + c] = dotp * is * is / (float)ntot;
    if (dgamma) dgamma[c] = dotp * is;
    if (dbeta) dbeta[c] = sdy;
    if (dw) dw[c] = (float)tot[2][col];
  }
}

// Vectorised apply (4 columns per thread, 256 columns x 4 row lanes per block, one row chunk
// per blockIdx.y) with the column partial sums of dX (the pre-BN Linear's bias gradient) in
// the same pass: colpart[chunk][c] (null: skipped).
__global__ void __launch_bounds__(256) bn_bwd_apply4_kernel(BnBwdSrc s, const float* __restrict__ Xpre,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            const float* __restrict__ g,
                                                            const float* __restrict__ coef, float* __restrict__ dX,
                                                            short* __restrict__ dX16, int B, int C,
                                                            int rows_per_chunk, float* __restrict__ colpart) {
  FBN_MAIN_PRIO();
  __shared__ f32x4 red[4][64];
  const int q = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + q * 4;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(B, r0 + rows_per_chunk);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + c);
    const f32x4 is = *reinterpret_cast<const f32x4*>(invstd + c);
    const f32x4 gg = *reinterpret_cast<const f32x4*>(g + c);
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(coef + c);
    const f32x4 c1 = *reinterpret_cast<const f32x4*>(coef + C + c);
    const f32x4 ww = s.G ? (f32x4){0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(s.w + c);
    for (int r = r0 + rl; r < r1; r += 4) {
      const size_t i = (size_t)r * C + c;
      const f32x4 h = bn_act4(s, i);
      const f32x4 x = *reinterpret_cast<const f32x4*>(Xpre + i);
      f32x4 d;
      if (s.G) d = *reinterpret_cast<const f32x4*>(s.G + i);
      else { const float gv = s.gvec[r]; d = (f32x4){gv * ww[0], gv * ww[1], gv * ww[2], gv * ww[3]}; }
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dy = h[e] > 0.f ? d[e] * s.scale : 0.f;
        v[e] = (dy - c0[e] - (x[e] - mu[e]) * c1[e]) * is[e] * gg[e];
      }
      if (dX) *reinterpret_cast<f32x4*>(dX + i) = v;
      if (dX16) {
        if (s.dx16_lo) store_img4(dX16 + i, s.dx16_lo, v);
        else store4(dX16 + i, v);
      }
      acc += v;
    }
  }
  if (!colpart) return;
  red[rl][q] = acc;
  __syncthreads();
  if (rl == 0 && c < C)
    *reinterpret_cast<f32x4*>(colpart + (size_t)blockIdx.y * C + c) = red[0][q] + red[1][q] + red[2][q] + red[3][q];
}

// Deferred sums, one launch for all of a step's small reductions (bias gradients from column
// partials, the head-bias gradient and the loss from [B] vectors):
//   out[c] = beta * out[c] + scale * sum_{k < nch} part[k * C + c]
// one 256-thread block per output column, fixed-order tree (deterministic).
//   (ld = row stride of part; 0 = C)
// and, in the same launch (fbn_sum_jobs2), the split-K slabs of the step's weight-gradient GEMMs
// (fbn_gemm_slabs): out[m * ldc + rm(n)] = beta * out + sum_{z < nsplit} ws[z][m][n] (slab groups
// then a fixed-order fold: deterministic), rm(n) = n + (n < seg ? off0 : off1).
struct SumJob {
  const float* part;
  float* out;
  int nch, C;
  float scale, beta;
  int ld;
  int pad_;
};
struct SlabJob {
  const float* ws;
  float* out;
  int M, N, ldc, nsplit, seg, off0, off1;
  float beta;
};
#define FBN_MAX_SUM_JOBS 16
#define FBN_SUM_WIDE 32        // jobs with at least this many columns take 16 columns per block
#define FBN_MAX_SLAB_JOBS 8
#define FBN_SLAB_GROUPS 4      // slab groups per output quad (256 threads = 64 quads x 4 groups)
struct SumJobs {
  SumJob j[FBN_MAX_SUM_JOBS];
  int col0[FBN_MAX_SUM_JOBS + 1];
  int n;
  SlabJob s[FBN_MAX_SLAB_JOBS];
  int blk0[FBN_MAX_SLAB_JOBS + 1];   // first block of each slab job (after the column blocks)
  int ns;
  int direct;                        // slab jobs of <= FBN_SLAB_DIRECT slabs: slab_direct
};
// slab jobs of at most FBN_SLAB_DIRECT slabs: one output quad per thread, every slab's load in
// flight at once, summed in slab order (no LDS fold; a quarter of the blocks)
#define FBN_SLAB_DIRECT 8
__device__ __forceinline__ void slab_direct(const SlabJob& sj, int lb) {
  const size_t total = (size_t)sj.M * sj.N;
  const size_t i4 = (size_t)lb * 256 + threadIdx.x;
  if (i4 >= total / 4) return;
  const float* src = sj.ws + i4 * 4;
  f32x4 x[FBN_SLAB_DIRECT];
#pragma unroll
  for (int z = 0; z < FBN_SLAB_DIRECT; ++z)
    if (z < sj.nsplit) x[z] = *reinterpret_cast<const f32x4*>(src + (size_t)z * total);
  f32x4 t = x[0];
#pragma unroll
  for (int z = 1; z < FBN_SLAB_DIRECT; ++z)
    if (z < sj.nsplit) t += x[z];
  const int m = (int)(i4 * 4 / sj.N), n = (int)(i4 * 4 - (size_t)m * sj.N);
  float* cp = sj.out + (size_t)m * sj.ldc + n + (n < sj.seg ? sj.off0 : sj.off1);
  if (sj.beta != 0.f) t += sj.beta * *reinterpret_cast<const f32x4*>(cp);
  *reinterpret_cast<f32x4*>(cp) = t;
}
__device__ __forceinline__ void slab_block(const SumJobs& J, int gb) {
  __shared__ f32x4 red[FBN_SLAB_GROUPS][64];
  int u = 0;
  while (u + 1 < J.ns && gb >= J.blk0[u + 1]) ++u;
  const SlabJob sj = J.s[u];
  if (J.direct && sj.nsplit <= FBN_SLAB_DIRECT) {
    slab_direct(sj, gb - J.blk0[u]);
    return;
  }
  const int qd = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const size_t total = (size_t)sj.M * sj.N;
  const size_t i4 = (size_t)(gb - J.blk0[u]) * 64 + qd;   // output quad
  const bool ok = i4 < total / 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
    const float* src = sj.ws + i4 * 4;
    int z = grp;
    for (; z + 3 * FBN_SLAB_GROUPS < sj.nsplit; z += 4 * FBN_SLAB_GROUPS) {   // 4 slabs in flight
      const f32x4 a = *reinterpret_cast<const f32x4*>(src + (size_t)z * total);
      const f32x4 b = *reinterpret_cast<const f32x4*>(src + (size_t)(z + FBN_SLAB_GROUPS) * total);
      const f32x4 c = *reinterpret_cast<const f32x4*>(src + (size_t)(z + 2 * FBN_SLAB_GROUPS) * total);
      const f32x4 d = *reinterpret_cast<const f32x4*>(src + (size_t)(z + 3 * FBN_SLAB_GROUPS) * total);
      acc += a; acc += b; acc += c; acc += d;
    }
    for (; z < sj.nsplit; z += FBN_SLAB_GROUPS) acc += *reinterpret_cast<const f32x4*>(src + (size_t)z * total);
  }
  red[grp][qd] = acc;
  __syncthreads();
  if (grp == 0 && ok) {
    f32x4 t = red[0][qd];
#pragma unroll
    for (int k = 1; k < FBN_SLAB_GROUPS; ++k) t += red[k][qd];
    const int m = (int)(i4 * 4 / sj.N), n = (int)(i4 * 4 - (size_t)m * sj.N);
    float* cp = sj.out + (size_t)m * sj.ldc + n + (n < sj.seg ? sj.off0 : sj.off1);
    if (sj.beta != 0.f) t += sj.beta * *reinterpret_cast<const f32x4*>(cp);
    *reinterpret_cast<f32x4*>(cp) = t;
  }
}
// wide jobs (C >= FBN_SUM_WIDE): a block takes 16 consecutive columns and 16 row streams (16 lanes
// read one 64-B run of a row: coalesced; every row stream has nch/16 rows), then a fixed-order fold
// of the 16 streams
__device__ __forceinline__ void sum_wide_block(const SumJob& jb, int c0) {
  __shared__ float red[16][17];
  const int col = threadIdx.x & 15, str = threadIdx.x >> 4, c = c0 + col;
  const size_t ld = jb.ld > 0 ? jb.ld : jb.C;
  float a0 = 0.f, a1 = 0.f;
  if (c < jb.C) {
    int k = str;
    for (; k + 16 < jb.nch; k += 32) {
      a0 += jb.part[(size_t)k * ld + c];
      a1 += jb.part[(size_t)(k + 16) * ld + c];
    }
    for (; k < jb.nch; k += 16) a0 += jb.part[(size_t)k * ld + c];
  }
  red[str][col] = a0 + a1;
  __syncthreads();
  if (str == 0 && c < jb.C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][col];
    t *= jb.scale;
    jb.out[c] = jb.beta != 0.f ? jb.beta * jb.out[c] + t : t;
  }
}
__global__ void __launch_bounds__(256) sum_jobs_kernel(SumJobs J) {
  __shared__ float red[4];
  const int gc = blockIdx.x;
  if (gc >= J.col0[J.n]) {
    slab_block(J, gc - J.col0[J.n]);
    return;
  }
  int u = 0;
  while (u + 1 < J.n && gc >= J.col0[u + 1]) ++u;
  const SumJob jb = J.j[u];
  if (jb.C >= FBN_SUM_WIDE) {
    sum_wide_block(jb, (gc - J.col0[u]) * 16);
    return;
  }
  const int c = gc - J.col0[u];
  const size_t ld = jb.ld > 0 ? jb.ld : jb.C;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int k = threadIdx.x;
  for (; k + 768 < jb.nch; k += 1024) {
    a0 += jb.part[(size_t)k * ld + c];
    a1 += jb.part[(size_t)(k + 256) * ld + c];
    a2 += jb.part[(size_t)(k + 512) * ld + c];
    a3 += jb.part[(size_t)(k + 768) * ld + c];
  }
  for (; k < jb.nch; k += 256) a0 += jb.part[(size_t)k * ld + c];
  float v = wave_sum((a0 + a1) + (a2 + a3));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = jb.scale * ((red[0] + red[1]) + (red[2] + red[3]));
    jb.out[c] = jb.beta != 0.f ? jb.beta * jb.out[c] + t : t;
  }
}

// ------------------------------------------------------------------ head: o = h.w + b, p = sigmoid(o), BCE
// one wave per row.  gout[b] = dL/do when labels are given (mean BCE over `denom` samples),
// using ATen's BCE backward ((p-t)/max((1-p)p, 1e-12)/N) followed by sigmoid backward (g(1-p)p).
__global__ void head_fwd_kernel(const float* __restrict__ H, const float* __restrict__ w, const float* __restrict__ bias,
                                int B, int C, float* __restrict__ logits, float* __restrict__ probs,
                                const float* __restrict__ labels, float* __restrict__ loss_terms,
                                float* __restrict__ gout, float denom) {
  const int lane = threadIdx.x & 63;
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= B) return;
  float s = 0.f;
  for (int c = lane * 4; c < C; c += 256) {
    const f32x4 h = *reinterpret_cast<const f32x4*>(H + (size_t)row * C + c);
    const f32x4 ww = *reinterpret_cast<const f32x4*>(w + c);
    s += h[0] * ww[0] + h[1] * ww[1] + h[2] * ww[2] + h[3] * ww[3];
  }
  head_row(s, row, lane, HeadArgs{w, bias, logits, probs, labels, loss_terms, gout, denom});
}

// sigmoid backward only (drop-in mode: torch computes BCE and hands us dL/dp)
__global__ void sigmoid_bwd_kernel(const float* gp, const float* probs, float* gout, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) gout[i] = gp[i] * (1.f - probs[i]) * probs[i];
}

// dH[b][c] = g[b] * w[c]   (rank-1; used by the drop-in backward)
__global__ void outer_kernel(const float* g, const float* w, float* out, int B, int C) {
  const size_t total = (size_t)B * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
    out[i] = g[i / C] * w[i % C];
}

// out = scale * sum(x): one 1024-thread block, 4 independent accumulators per thread, wave
// shuffles + 16-entry LDS stage (fixed order: deterministic)
__global__ void __launch_bounds__(1024) sum_kernel(const float* x, int n, float* out, float scale) {
  __shared__ float red[16];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int i = threadIdx.x;
  for (; i + 3 * 1024 < n; i += 4 * 1024) {
    s0 += x[i]; s1 += x[i + 1024]; s2 += x[i + 2048]; s3 += x[i + 3072];
  }
  for (; i < n; i += 1024) s0 += x[i];
  float s = wave_sum((s0 + s1) + (s2 + s3));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = threadIdx.x < 16 ? red[threadIdx.x] : 0.f;
    t = wave_sum(t);
    if (threadIdx.x == 0) out[0] = t * scale;
  }
}

// ------------------------------------------------------------------ C ABI
static int ew_grid(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}
static int row_chunks(int B) {
  int ch = (B + 127) / 128;
  return ch < 1 ? 1 : (ch > 256 ? 256 : ch);
}
// row chunks of the fused BN backward (partial + apply): >= 512 workgroups of 256 columns x
// rows_per_chunk, at least 16 rows per chunk
static int bn_bwd_chunks(int B, int C) {
  const int cg = (C + 255) / 256;
  int ch = (512 + cg - 1) / cg;
  const int cap = (B + 15) / 16;
  if (ch > cap) ch = cap;
  if (ch > 1024) ch = 1024;
  return ch < 1 ? 1 : ch;
}

// c_bf16: c is a bf16 [B][ldc] buffer (bf16 GEMM mode) instead of float
extern "C" int fbn_pairs_fwd(const float* Vc, const short* Vc16, const float* U, void* c, int B, int D, int ldc,
                             int mode, int c_bf16, void* stream) {
  if (B <= 0) return FBN_OK;
  if ((D & 3) || (ldc & 3)) { fbn_set_error("pairs: D and ldc must be multiples of 4"); return FBN_ERR_ARG; }
  if (c_bf16)
    fbn_launch(pairs_fwd_kernel<short>, dim3(ew_grid((size_t)B * D / 4)), dim3(256), 0, (hipStream_t)stream,
                       Vc, Vc16, U, (short*)c, B, D, ldc, mode);
  else
    fbn_launch(pairs_fwd_kernel<float>, dim3(ew_grid((size_t)B * D / 4)), dim3(256), 0, (hipStream_t)stream,
                       Vc, Vc16, U, (float*)c, B, D, ldc, mode);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_pairs_fwd_img(const float* Vc, const float* U, void* c_img, void* vc_img, int B, int D, int ldc,
                                 void* stream) {
  if (B <= 0) return FBN_OK;
  if ((D & 7) || (ldc & 7) || ldc < 15 * D || !Vc || !U || !c_img) {
    fbn_set_error("fbn_pairs_fwd_img: Vc, U, c_img; D, ldc multiples of 8, ldc >= 15 D");
    return FBN_ERR_ARG;
  }
  fbn_launch(pairs_fwd_img_kernel, dim3(ew_grid((size_t)B * D / 8)), dim3(256), 0, (hipStream_t)stream, Vc, U,
             (short*)c_img, (short*)vc_img, B, D, ldc);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_pairs_bwd_img(const float* dc, const float* Vc, const float* U, float* dV, void* dU_img, int B,
                                 int D, int ldc, void* stream) {
  if (B <= 0) return FBN_OK;
  if ((D & 3) || (ldc & 3) || !dc || !Vc || !U || !dV || !dU_img) {
    fbn_set_error("fbn_pairs_bwd_img: dc, Vc, U, dV, dU_img; D, ldc multiples of 4");
    return FBN_ERR_ARG;
  }
  fbn_launch(pairs_bwd_kernel<0>, dim3(ew_grid((size_t)B * D / 4)), dim3(256), 0, (hipStream_t)stream, dc, Vc,
             (const short*)nullptr, U, dV, (float*)nullptr, (short*)nullptr, B, D, ldc, (short*)dU_img);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_pairs_bwd(const float* dc, const float* Vc, const short* Vc16, const float* U, float* dV,
                             float* dU, short* dU16, int B, int D, int ldc, int mode, void* stream) {
  if (B <= 0) return FBN_OK;
  if (mode == 0)
    fbn_launch(pairs_bwd_kernel<0>, dim3(ew_grid((size_t)B * D / 4)), dim3(256), 0, (hipStream_t)stream, dc, Vc,
                       Vc16, U, dV, dU, dU16, B, D, ldc, (short*)nullptr);
  else
    fbn_launch(pairs_bwd_kernel<1>, dim3(ew_grid((size_t)B * D / 4)), dim3(256), 0, (hipStream_t)stream, dc, Vc,
                       Vc16, U, dV, dU, dU16, B, D, ldc, (short*)nullptr);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// workspace for the BN entry points: chunk partials [nchunk][3][C] doubles + 4*C doubles of scratch
extern "C" size_t fbn_bn_workspace_size(int B, int C) {
  const int nch = row_chunks(B) > bn_bwd_chunks(B, C) ? row_chunks(B) : bn_bwd_chunks(B, C);
  return ((size_t)nch * 3 * C + 4 * (size_t)C) * sizeof(double);
}
extern "C" int fbn_bn_bwd_chunks(int B, int C) { return bn_bwd_chunks(B, C); }

// Local column pass over this rank's rows: out_d[c] = sum_b X[b][c]  (mean_d == null)
//                                       or  out_d[c] = sum_b (X[b][c] - mean_d[c])^2
extern "C" int fbn_bn_stats_pass(const float* X, int B, int C, const double* mean_d, double* out_d, void* ws,
                                 void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int nch = row_chunks(B), rpc = B > 0 ? (B + nch - 1) / nch : 1;
  double* part = (double*)ws;
  fbn_launch(colstat_partial_kernel, dim3(fbn_cdiv(C, 64), nch), dim3(256), 0, st, X, B, C, C, rpc, mean_d,
                     part, mean_d ? 1 : 0);
  fbn_launch(chunk_reduce_kernel, dim3(fbn_cdiv(C, 4)), dim3(256), 0, st, part, nch, C, out_d);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_bn_mean(const double* sum_d, double ntot, int C, double* mean_d, void* stream) {
  fbn_launch(bn_mean_kernel, dim3(fbn_cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, sum_d, ntot, C, mean_d);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_bn_finalize(const double* m2_d, const double* mean_d, double ntot, int C, float* mean,
                               float* invstd, float* run_mean, float* run_var, float momentum, float eps,
                               int update_running, void* stream) {
  fbn_launch(bn_finalize_kernel, dim3(fbn_cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, m2_d, mean_d, ntot,
                     C, mean, invstd, run_mean, run_var, momentum, eps, update_running);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// single-process convenience: both passes + finalize (ws >= fbn_bn_workspace_size)
extern "C" int fbn_bn_stats(const float* X, int B, int C, float* mean, float* invstd, float* run_mean, float* run_var,
                            float momentum, float eps, int update_running, void* ws, void* stream) {
  if (B <= 0) return FBN_OK;
  double* scratch = (double*)ws + (size_t)row_chunks(B) * 3 * C;
  double* sum_d = scratch;
  double* mean_d = scratch + C;
  int rc = fbn_bn_stats_pass(X, B, C, nullptr, sum_d, ws, stream);
  if (!rc) rc = fbn_bn_mean(sum_d, (double)B, C, mean_d, stream);
  if (!rc) rc = fbn_bn_stats_pass(X, B, C, mean_d, sum_d, ws, stream);
  if (!rc) rc = fbn_bn_finalize(sum_d, mean_d, (double)B, C, mean, invstd, run_mean, run_var, momentum, eps,
                                update_running, stream);
  return rc;
}

extern "C" int fbn_bn_eval_params(const float* run_mean, const float* run_var, float* mean, float* invstd, int C,
                                  float eps, void* stream) {
  fbn_launch(bn_eval_params_kernel, dim3(fbn_cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, run_mean,
                     run_var, mean, invstd, C, eps);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// Rows per workgroup of the BN-apply kernels: 4 = one row per wave, so every row of the batch is
// in flight at once (the fused head reduces a whole row per wave and then runs a serial sigmoid /
// BCE tail: with 16 rows per workgroup each wave walked 4 rows one after the other).
// A/B knob: bn_act_fwd4r_kernel (four rows per wave, 16-row chunks) for the plain BN + ReLU + dropout
static bool bn_act_rows4() {
  const char* e = getenv("FBN_BN_ACT_R4");   // read per call
  return e && atoi(e) != 0;
}
static int bn_act_rows_per_chunk() {
  const char* e = getenv("FBN_BN_ACT_RPC");   // A/B knob, read per call
  const int v = e ? atoi(e) : 4;
  const int rpc = v >= 4 && v % 4 == 0 ? v : 4;
  return rpc;
}

// rng: device [seed, offset] (uint64 x2) or null; mask_out (optional, u8 [B][C]) receives the keep-mask;
// mask_in (optional, u8 [B][C]) replaces the RNG (parity tests against injected masks)
extern "C" int fbn_bn_act_fwd(const float* X, float* Y, int B, int C, const float* mean, const float* invstd,
                              const float* g, const float* b, float p_drop, const unsigned long long* rng,
                              unsigned stream_id, unsigned char* mask_out, const unsigned char* mask_in,
                              short* Y16, void* stream) {
  if (B <= 0) return FBN_OK;
  if (C & 3) { fbn_set_error("bn_act: C % 4"); return FBN_ERR_ARG; }
  if (p_drop > 0.f && !rng && !mask_in) { fbn_set_error("bn_act: dropout needs an rng state or a mask"); return FBN_ERR_ARG; }
  if (!Y && !Y16) { fbn_set_error("bn_act: no output"); return FBN_ERR_ARG; }
  if (bn_act_rows4()) {
    fbn_launch(bn_act_fwd4r_kernel, dim3(fbn_cdiv(C, 256), fbn_cdiv(B, 16)), dim3(256), 0, (hipStream_t)stream, X, Y,
               B, C, 16, mean, invstd, g, b, p_drop, rng, stream_id, mask_out, mask_in, Y16, 0LL);
    FBN_CHECK_LAUNCH();
    return FBN_OK;
  }
  const int rpc = bn_act_rows_per_chunk();
  fbn_launch(bn_act_fwd2_kernel<false>, dim3(fbn_cdiv(C, 256), fbn_cdiv(B, rpc)), dim3(256), 0,
                     (hipStream_t)stream, X, Y, B, C, rpc, mean, invstd, g, b, p_drop, rng, stream_id, mask_out, mask_in,
                     Y16, HeadArgs{}, nullptr, 1.f, 0LL);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// fbn_bn_act_fwd with the bf16 output as split images: Y_img = hi (the layer-2 GEMM operand), lo =
// bf16(y - hi) B*C elements further (the bf16_fwd backward's split-bf16 x3 weight gradient)
extern "C" int fbn_bn_act_fwd_img(const float* X, float* Y, int B, int C, const float* mean, const float* invstd,
                                  const float* g, const float* b, float p_drop, const unsigned long long* rng,
                                  unsigned stream_id, unsigned char* mask_out, const unsigned char* mask_in,
                                  void* Y_img, void* stream) {
  if (B <= 0) return FBN_OK;
  if ((C & 3) || !Y_img) { fbn_set_error("bn_act_img: C % 4, Y_img"); return FBN_ERR_ARG; }
  if (p_drop > 0.f && !rng && !mask_in) { fbn_set_error("bn_act: dropout needs an rng state or a mask"); return FBN_ERR_ARG; }
  if (bn_act_rows4()) {
    fbn_launch(bn_act_fwd4r_kernel, dim3(fbn_cdiv(C, 256), fbn_cdiv(B, 16)), dim3(256), 0, (hipStream_t)stream, X, Y,
               B, C, 16, mean, invstd, g, b, p_drop, rng, stream_id, mask_out, mask_in, (short*)Y_img,
               (long long)B * C);
    FBN_CHECK_LAUNCH();
    return FBN_OK;
  }
  const int rpc = bn_act_rows_per_chunk();
  fbn_launch(bn_act_fwd2_kernel<false>, dim3(fbn_cdiv(C, 256), fbn_cdiv(B, rpc)), dim3(256), 0,
                     (hipStream_t)stream, X, Y, B, C, rpc, mean, invstd, g, b, p_drop, rng, stream_id, mask_out, mask_in,
                     (short*)Y_img, HeadArgs{}, nullptr, 1.f, (long long)B * C);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// BN + ReLU + dropout of the last hidden layer (C = 256) fused with the head (fbn_head_fwd's outputs)
extern "C" int fbn_bn_act_head_fwd(const float* X, float* Y, int B, int C, const float* mean, const float* invstd,
                                   const float* g, const float* b, float p_drop, const unsigned long long* rng,
                                   unsigned stream_id, unsigned char* mask_out, const unsigned char* mask_in,
                                   const float* hw, const float* hbias, float* logits, float* probs,
                                   const float* labels, float* loss_terms, float* gout, float denom,
                                   double* bwd_part, float bwd_scale, void* stream) {
  if (B <= 0) return FBN_OK;
  if (C != 256) { fbn_set_error("bn_act_head: the fused head needs C == 256"); return FBN_ERR_UNSUPPORTED; }
  if (p_drop > 0.f && !rng && !mask_in) { fbn_set_error("bn_act: dropout needs an rng state or a mask"); return FBN_ERR_ARG; }
  if (bwd_part && !gout) { fbn_set_error("bn_act_head: backward partials need labels / gout"); return FBN_ERR_ARG; }
  if (bwd_part) {
    // the row chunks of fbn_bn_bwd_fused, so its reduce reads these partials as its own
    const int nch = bn_bwd_chunks(B, C), rpc = (B + nch - 1) / nch;
    static const bool one_row = getenv("FBN_HEAD_ONE_ROW") != nullptr;   // A/B knob: one row per wave
    if (!one_row) {
      fbn_launch(bn_act_head_bwd4_kernel, dim3(1, fbn_cdiv(B, rpc)), dim3(256), 0, (hipStream_t)stream, X, Y, B,
                 C, rpc, mean, invstd, g, b, p_drop, rng, stream_id, mask_out, mask_in,
                 HeadArgs{hw, hbias, logits, probs, labels, loss_terms, gout, denom}, bwd_part, bwd_scale);
      FBN_CHECK_LAUNCH();
      return FBN_OK;
    }
    fbn_launch((bn_act_fwd2_kernel<true, 1024, true>), dim3(1, fbn_cdiv(B, rpc)), dim3(1024), 0,
                       (hipStream_t)stream, X, Y, B, C, rpc, mean, invstd, g, b, p_drop, rng, stream_id, mask_out,
                       mask_in, nullptr, HeadArgs{hw, hbias, logits, probs, labels, loss_terms, gout, denom}, bwd_part,
                       bwd_scale, 0LL);
    FBN_CHECK_LAUNCH();
    return FBN_OK;
  }
  const int rpc = bn_act_rows_per_chunk();
  fbn_launch(bn_act_fwd2_kernel<true>, dim3(1, fbn_cdiv(B, rpc)), dim3(256), 0, (hipStream_t)stream, X, Y, B,
                     C, rpc, mean, invstd, g, b, p_drop, rng, stream_id, mask_out, mask_in, (short*)nullptr,
                     HeadArgs{hw, hbias, logits, probs, labels, loss_terms, gout, denom}, nullptr, 1.f, 0LL);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// BN(+ReLU+dropout) backward, stage 1: local sums red_d[3][C] = {sum dy, sum (x-mean) dy, sum gvec*hact}.
// Source of dL/d(act): G (matrix) or gvec (x) w (rank-1 head).
extern "C" int fbn_bn_bwd_reduce(const float* G, const float* gvec, const float* w, const float* hact, float scale,
                                 const float* Xpre, const float* mean, int B, int C, double* red_d, void* ws,
                                 void* stream) {
  hipStream_t st = (hipStream_t)stream;
  BnBwdSrc s{G, gvec, w, hact, scale, nullptr};
  const int nch = row_chunks(B), rpc = B > 0 ? (B + nch - 1) / nch : 1;
  double* part = (double*)ws;
  fbn_launch(bn_bwd_partial_kernel, dim3(fbn_cdiv(C, 64), nch), dim3(256), 0, st, s, Xpre, mean, B, C, rpc, part);
  fbn_launch(chunk_reduce_kernel, dim3(fbn_cdiv(3 * C, 4)), dim3(256), 0, st, part, nch, 3 * C, red_d);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// stage 2 (after an optional all-reduce of red_d): dXpre, dgamma, dbeta, dw (rank-1 only)
extern "C" int fbn_bn_bwd_apply(const float* G, const float* gvec, const float* w, const float* hact, float scale,
                                const float* Xpre, const float* mean, const float* invstd, const float* gamma, int B,
                                int C, const double* red_d, double ntot, float* dXpre, short* dXpre16, float* dgamma,
                                float* dbeta, float* dw, void* ws, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  BnBwdSrc s{G, gvec, w, hact, scale, nullptr};
  float* coef = (float*)((double*)ws + (size_t)row_chunks(B) * 3 * C + 3 * (size_t)C);
  fbn_launch(bn_bwd_finalize_kernel, dim3(fbn_cdiv(C, 256)), dim3(256), 0, st, red_d, C, ntot, invstd, coef,
                     dgamma, dbeta, G ? nullptr : dw);
  if (B > 0 && !(C & 3)) {
    const int nch = row_chunks(B), rpc = (B + nch - 1) / nch;
    fbn_launch(bn_bwd_apply4_kernel, dim3(fbn_cdiv(C, 256), nch), dim3(256), 0, st, s, Xpre, mean, invstd,
                       gamma, coef, dXpre, dXpre16, B, C, rpc, nullptr);
  } else if (B > 0) {
    fbn_launch(bn_bwd_apply_kernel, dim3(ew_grid((size_t)B * C)), dim3(256), 0, st, s, Xpre, mean, invstd,
                       gamma, coef, dXpre, dXpre16, B, C);
  }
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_bn_bwd(const float* G, const float* gvec, const float* w, const float* hact, float scale,
                          const float* Xpre, const float* mean, const float* invstd, const float* gamma, int B, int C,
                          float* dXpre, float* dgamma, float* dbeta, float* dw, void* ws, void* stream) {
  if (B <= 0) return FBN_OK;
  double* red = (double*)ws + (size_t)row_chunks(B) * 3 * C;   // 3*C doubles
  int rc = fbn_bn_bwd_reduce(G, gvec, w, hact, scale, Xpre, mean, B, C, red, ws, stream);
  if (!rc) rc = fbn_bn_bwd_apply(G, gvec, w, hact, scale, Xpre, mean, invstd, gamma, B, C, red, (double)B, dXpre,
                                 nullptr, dgamma, dbeta, dw, ws, stream);
  return rc;
}

extern "C" size_t fbn_colsum_workspace_size(int B, int C) { return (size_t)row_chunks(B) * C * sizeof(float); }

// out[c] = beta*out[c] + sum_b X[b][c]
extern "C" int fbn_colsum(const float* X, int B, int C, int ldx, float* out, float beta, void* ws, void* stream) {
  if (B <= 0) return FBN_OK;
  hipStream_t st = (hipStream_t)stream;
  const int nch = row_chunks(B), rpc = (B + nch - 1) / nch;
  fbn_launch(colsum_partial_kernel, dim3(fbn_cdiv(C, 64), nch), dim3(256), 0, st, X, B, C, ldx, rpc, (float*)ws);
  fbn_launch(colsum_final_kernel, dim3(fbn_cdiv(C, 4)), dim3(256), 0, st, (const float*)ws, nch, C, out, beta);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_head_fwd(const float* H, const float* w, const float* bias, int B, int C, float* logits,
                            float* probs, const float* labels, float* loss_terms, float* gout, float denom,
                            void* stream) {
  if (B <= 0) return FBN_OK;
  if (C & 3) { fbn_set_error("head: C % 4"); return FBN_ERR_ARG; }
  fbn_launch(head_fwd_kernel, dim3(fbn_cdiv((long long)B * 64, 256)), dim3(256), 0, (hipStream_t)stream, H, w,
                     bias, B, C, logits, probs, labels, loss_terms, gout, denom);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_sigmoid_bwd(const float* gp, const float* probs, float* gout, int B, void* stream) {
  if (B <= 0) return FBN_OK;
  fbn_launch(sigmoid_bwd_kernel, dim3(fbn_cdiv(B, 256)), dim3(256), 0, (hipStream_t)stream, gp, probs, gout, B);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_outer(const float* g, const float* w, float* out, int B, int C, void* stream) {
  if (B <= 0) return FBN_OK;
  fbn_launch(outer_kernel, dim3(ew_grid((size_t)B * C)), dim3(256), 0, (hipStream_t)stream, g, w, out, B, C);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_sum(const float* x, int n, float* out, float scale, void* stream) {
  fbn_launch(sum_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, x, n, out, scale);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// ------------------------------------------------------------------ bf16 weight copies
// out[i*dld + j] = bf16( T ? src[j*ld + rm(i)] : src[i*ld + rm(j)] ) (or its rounding residual, part 1),
// i < rows, j < cols, rm(x) = x + (x < seg ? off0 : off1).  Up to 16 jobs per launch: the compacted /
// transposed bf16 weight images the bf16 GEMMs read (made once per step), the split-bf16 operand images.
__global__ void __launch_bounds__(256) convert_bf16_kernel(ConvJobs jobs, int njobs) {
  convert_tile(jobs, njobs, blockIdx.x);
}

// jobs: host array of n (<= 16) ConvJob records {src, dst, rows, cols, ld, trans, seg, off0, off1, part, dld}
extern "C" int fbn_convert_bf16(const void* jobs, int n, void* stream) {
  if (n <= 0) return FBN_OK;
  if (n > FBN_CONV_MAX) { fbn_set_error("convert_bf16: at most 16 jobs"); return FBN_ERR_ARG; }
  ConvJobs J;
  const int tiles = conv_jobs_pack(jobs, n, J);
  if (tiles <= 0) return FBN_OK;
  fbn_launch(convert_bf16_kernel, dim3(tiles), dim3(256), 0, (hipStream_t)stream, J, n);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// ------------------------------------------------------------------ BN stats from GEMM tile partials
// part[t][c] = (sum, M2 about the tile mean) over the rows of 64-row tile t (fbn_gemm stats).
// mean_d == null: out[c] = sum_t S_t ;  else out[c] = sum_t (M2_t + n_t (S_t/n_t - mean)^2)
// (Chan's parallel merge, f64; one wave per column, fixed order).
__global__ void bn_tile_stats_kernel(const float* __restrict__ part, int T, int C, int M, int tile_rows,
                                     const double* __restrict__ mean_d, double* __restrict__ out) {
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  double s = 0.0;
  const double mu = mean_d ? mean_d[c] : 0.0;
  for (int t = lane; t < T; t += 64) {
    const float S = part[((size_t)t * C + c) * 2], M2 = part[((size_t)t * C + c) * 2 + 1];
    if (!mean_d) {
      s += (double)S;
    } else {
      const int nt = min(tile_rows, M - t * tile_rows);
      const double dm = (double)S / nt - mu;
      s += (double)M2 + nt * dm * dm;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[c] = s;
}

extern "C" int fbn_bn_tile_stats(const float* part, int M, int C, const double* mean_d, double* out_d, void* stream) {
  const int T = (M + 63) / 64;
  fbn_launch(bn_tile_stats_kernel, dim3(fbn_cdiv(C, 4)), dim3(256), 0, (hipStream_t)stream, part, T, C, M, 64,
                     mean_d, out_d);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// ------------------------------------------------------------------ single-process BN fusions (C ABI)
extern "C" int fbn_bn_tile_finalize(const float* part, int M, int C, double ntot, float* mean, float* invstd,
                                    float* run_mean, float* run_var, float momentum, float eps, int update_running,
                                    void* stream) {
  if (M <= 0) return FBN_OK;
  fbn_launch(bn_tile_finalize_kernel, dim3(fbn_cdiv(C, 4)), dim3(256), 0, (hipStream_t)stream, part,
                     (M + 63) / 64, C, M, 64, ntot, mean, invstd, run_mean, run_var, momentum, eps, update_running);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" size_t fbn_bn_colpart_size(int B, int C) { return (size_t)bn_bwd_chunks(B, C) * C * sizeof(float); }

static int bn_bwd_fused_impl(const float* G, const float* gvec, const float* w, const float* hact,
                             const short* hact16, float scale, const float* Xpre, const float* mean,
                             const float* invstd, const float* gamma, int B, int C, double ntot, float* dXpre,
                             short* dXpre16, float* dgamma, float* dbeta, float* dw, float* colpart,
                             const double* part_pre, void* ws, void* stream, long long img_lo);
extern "C" int fbn_bn_bwd_fused(const float* G, const float* gvec, const float* w, const float* hact,
                                const short* hact16, float scale, const float* Xpre, const float* mean,
                                const float* invstd, const float* gamma, int B, int C, double ntot, float* dXpre,
                                short* dXpre16, float* dgamma, float* dbeta, float* dw, float* colpart,
                                const double* part_pre, void* ws, void* stream) {
  return bn_bwd_fused_impl(G, gvec, w, hact, hact16, scale, Xpre, mean, invstd, gamma, B, C, ntot, dXpre, dXpre16,
                           dgamma, dbeta, dw, colpart, part_pre, ws, stream, 0);
}
// fbn_bn_bwd_fused with dXpre_img = split images of dXpre (hi, lo B*C elements further; bf16_fwd)
extern "C" int fbn_bn_bwd_fused_img(const float* G, const float* gvec, const float* w, const float* hact,
                                    const short* hact16, float scale, const float* Xpre, const float* mean,
                                    const float* invstd, const float* gamma, int B, int C, double ntot, float* dXpre,
                                    void* dXpre_img, float* dgamma, float* dbeta, float* dw, float* colpart,
                                    const double* part_pre, void* ws, void* stream) {
  if (!dXpre_img) { fbn_set_error("fbn_bn_bwd_fused_img: dXpre_img"); return FBN_ERR_ARG; }
  return bn_bwd_fused_impl(G, gvec, w, hact, hact16, scale, Xpre, mean, invstd, gamma, B, C, ntot, dXpre,
                           (short*)dXpre_img, dgamma, dbeta, dw, colpart, part_pre, ws, stream, (long long)B * C);
}
static int bn_bwd_fused_impl(const float* G, const float* gvec, const float* w, const float* hact,
                             const short* hact16, float scale, const float* Xpre, const float* mean,
                             const float* invstd, const float* gamma, int B, int C, double ntot, float* dXpre,
                             short* dXpre16, float* dgamma, float* dbeta, float* dw, float* colpart,
                             const double* part_pre, void* ws, void* stream, long long img_lo) {
  if (B <= 0) return FBN_OK;
  if (C & 3) { fbn_set_error("fbn_bn_bwd_fused: C % 4"); return FBN_ERR_ARG; }
  if (!hact && !(hact16 && G)) {
    fbn_set_error("fbn_bn_bwd_fused: the bf16 activation image stands in only for a matrix source");
    return FBN_ERR_ARG;
  }
  if (!dXpre && !dXpre16) { fbn_set_error("fbn_bn_bwd_fused: no output"); return FBN_ERR_ARG; }
  hipStream_t st = (hipStream_t)stream;
  BnBwdSrc s{G, gvec, w, hact, scale, hact16, img_lo};
  const int nch = bn_bwd_chunks(B, C), rpc = (B + nch - 1) / nch;
  double* part = (double*)ws;
  float* coef = (float*)((double*)ws + (size_t)nch * 3 * C + 3 * (size_t)C);
  if (part_pre)   // the first pass already ran inside the forward (fbn_bn_act_head_fwd's bwd_part)
    part = const_cast<double*>(part_pre);
  else
    fbn_launch(bn_bwd_partial4_kernel, dim3(fbn_cdiv(C, 256), nch), dim3(256), 0, st, s, Xpre, mean, B, C, rpc,
                       part);
  static const bool wide = !getenv("FBN_BN_REDUCE64");   // A/B knob: 64 columns per workgroup
  const char* nce = getenv("FBN_BN_REDUCE_NC");   // A/B knob, read per call: columns per workgroup
  const int nc = nce ? atoi(nce) : 16;
  if (wide && nc == 4)
    fbn_launch(bn_bwd_reduce_finalize16_kernel<4>, dim3(fbn_cdiv(C, 4)), dim3(256), 0, st, part, nch, C, ntot,
               invstd, coef, dgamma, dbeta, dw);
  else if (wide && nc == 8)
    fbn_launch(bn_bwd_reduce_finalize16_kernel<8>, dim3(fbn_cdiv(C, 8)), dim3(512), 0, st, part, nch, C, ntot,
               invstd, coef, dgamma, dbeta, dw);
  else if (wide)
    fbn_launch(bn_bwd_reduce_finalize16_kernel<16>, dim3(fbn_cdiv(C, 16)), dim3(1024), 0, st, part, nch, C, ntot,
                       invstd, coef, dgamma, dbeta, dw);
  else
    fbn_launch(bn_bwd_reduce_finalize_kernel, dim3(fbn_cdiv(C, 64)), dim3(1024), 0, st, part, nch, C, ntot,
                       invstd, coef, dgamma, dbeta, dw);
  fbn_launch(bn_bwd_apply4_kernel, dim3(fbn_cdiv(C, 256), nch), dim3(256), 0, st, s, Xpre, mean, invstd, gamma,
                     coef, dXpre, dXpre16, B, C, rpc, colpart);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_colsum_partial(const float* X, int B, int C, int ldx, float* part, void* stream) {
  if (B <= 0) return FBN_OK;
  const int nch = row_chunks(B), rpc = (B + nch - 1) / nch;
  fbn_launch(colsum_partial_kernel, dim3(fbn_cdiv(C, 64), nch), dim3(256), 0, (hipStream_t)stream, X, B, C,
                     ldx, rpc, part);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_row_chunks(int B) { return row_chunks(B); }

// jobs: host array of n (<= 16) {part, out, nch, C, scale, beta, ld, pad} (copied into the kernel
// argument); slabs: host array of ns (<= 8) {ws, out, M, N, ldc, nsplit, seg, off0, off1, beta}
// (N, ldc, seg, off0, off1 multiples of 4; out 16-B aligned).  One launch for both.
extern "C" int fbn_sum_jobs2(const SumJob* jobs, int n, const SlabJob* slabs, int ns, void* stream) {
  if (n < 0 || ns < 0 || n > FBN_MAX_SUM_JOBS || ns > FBN_MAX_SLAB_JOBS) {
    fbn_set_error("fbn_sum_jobs2: too many jobs");
    return FBN_ERR_ARG;
  }
  SumJobs J;
  J.n = n;
  J.col0[0] = 0;
  for (int i = 0; i < n; ++i) {
    J.j[i] = jobs[i];
    // blocks of job i: one per column, or one per 64 columns for a wide job
    J.col0[i + 1] = J.col0[i] + (jobs[i].C >= FBN_SUM_WIDE ? fbn_cdiv(jobs[i].C, 16) : jobs[i].C);
  }
  J.ns = ns;
  const char* de = getenv("FBN_SLAB_DIRECT");   // A/B knob (0: the 4-group LDS fold for every slab job)
  J.direct = !(de && atoi(de) == 0);
  J.blk0[0] = 0;
  for (int i = 0; i < ns; ++i) {
    const SlabJob& sj = slabs[i];
    if ((sj.N & 3) || (sj.ldc & 3) || (sj.off0 & 3) || (sj.off1 & 3) || (sj.seg != 0x7fffffff && (sj.seg & 3)) ||
        ((uintptr_t)sj.out & 15) || ((uintptr_t)sj.ws & 15) || sj.nsplit < 1) {
      fbn_set_error("fbn_sum_jobs2: slab job needs N, ldc, remap % 4, 16-B aligned buffers, nsplit >= 1");
      return FBN_ERR_ARG;
    }
    J.s[i] = sj;
    const int qpb = (J.direct && sj.nsplit <= FBN_SLAB_DIRECT) ? 256 : 64;   // output quads per block
    J.blk0[i + 1] = J.blk0[i] + (int)fbn_cdiv((long long)sj.M * sj.N / 4, qpb);
  }
  const int blocks = J.col0[n] + J.blk0[ns];
  if (blocks <= 0) return FBN_OK;
  fbn_launch(sum_jobs_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, J);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_sum_jobs(const SumJob* jobs, int n, void* stream) {
  if (n <= 0) return FBN_OK;
  return fbn_sum_jobs2(jobs, n, nullptr, 0, stream);
}

extern "C" int fbn_bn_tile_moments(const float* part, int M, int C, double* out_d, void* stream) {
  if (M <= 0) { (void)hipMemsetAsync(out_d, 0, 2 * sizeof(double) * C, (hipStream_t)stream); return FBN_OK; }
  fbn_launch(bn_tile_moments_kernel, dim3(fbn_cdiv(C, 4)), dim3(256), 0, (hipStream_t)stream, part,
                     (M + 63) / 64, C, M, 64, out_d);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_bn_moments_finalize(const double* mom_d, double ntot, int C, float* mean, float* invstd,
                                       float* run_mean, float* run_var, float momentum, float eps, int update_running,
                                       void* stream) {
  fbn_launch(bn_moments_finalize_kernel, dim3(fbn_cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, mom_d, ntot,
                     C, mean, invstd, run_mean, run_var, momentum, eps, update_running);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}
