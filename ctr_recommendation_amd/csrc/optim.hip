// K8 / K9: global-norm gradient clipping + Adam (coupled L2) for the FiBiNET trainer.
//
// Semantics of train_fibinet.py:78,119,121-122 with torch's single-tensor Adam:
//   g  <- g * min(1, max_norm / (||g||_2 + 1e-6))          (clip_grad_norm_, all params)
//   g  <- g + wd * p                                        (coupled weight decay)
//   m  <- m + (1-b1) * (g - m)                              (lerp, weight < 0.5 branch)
//   v  <- v * b2 + ((1-b2) * g) * g                         (mul_ + addcmul_)
//   p  <- p + (-lr/bc1 * m) / (sqrt(v) / sqrt(bc2) + eps)   (addcdiv_)
// The per-step scalars (1-b1, -lr/bc1, sqrt(bc2)) come from a host-built schedule table
// (OneCycleLR with beta1 cycling, double precision like torch) indexed by a device-resident
// step counter, so a whole training step can be captured in a hipGraph and replayed.
//
// Table parameter: the gradient of E is non-zero only on the rows the batch touched.  The
// dense pass reads w, m, v (24 B/element, the HBM floor for exact dense-Adam semantics) and
// the gradient only through the row->slot map (4 B/row); untouched rows get g = 0 + wd*p.
// The map entries of touched rows are reset in the same pass.
#include "common.h"

#pragma clang fp contract(off)

struct AdamConsts {
  float w1;     // 1 - beta1 (as float)
  float nss;    // -lr / bias_correction1 (as float)
  float bc2s;   // sqrt(bias_correction2) (as float)
  float pad;
};

// ------------------------------------------------------------------ squared norm partials
// out slot += sum x^2 over n elements (double atomics on one slot per call; few blocks)
__global__ void sumsq_kernel(const float* __restrict__ x, long long n, const int* __restrict__ n_rows, int row_len,
                             double* __restrict__ out) {
  __shared__ double red[256];
  long long lim = n_rows ? (long long)(*n_rows) * row_len : n;
  double s = 0.0;
  const long long n4 = lim / 4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + 4 * i);
    s += (double)(v[0] * v[0]) + (double)(v[1] * v[1]) + (double)(v[2] * v[2]) + (double)(v[3] * v[3]);
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += (long long)gridDim.x * blockDim.x)
    s += (double)(x[i] * x[i]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(out, red[0]);
}

// coef = min(1, max_norm / (sqrt(total) + 1e-6)); also exposes the norm
__global__ void clip_coef_kernel(const double* sumsq, float max_norm, float* coef_out, float* norm_out) {
  const float total = sqrtf((float)sumsq[0]);
  float c = max_norm / (total + 1e-6f);
  coef_out[0] = c < 1.f ? c : 1.f;
  if (norm_out) norm_out[0] = total;
}

__device__ __forceinline__ float adam_elem(float& p, float& m, float& v, float g, float coef, float wd, float b2,
                                           float omb2, float eps, const AdamConsts& k) {
  g = g * coef;
  g = g + wd * p;
  m = m + k.w1 * (g - m);
  v = v * b2;
  v = v + (omb2 * g) * g;
  const float denom = sqrtf(v) / k.bc2s + eps;
  p = p + (k.nss * m) / denom;
  return p;
}

__global__ void adam_dense_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                  float* __restrict__ v, long long n, const float* __restrict__ coef_ptr,
                                  const AdamConsts* __restrict__ table, const int* __restrict__ step_ptr, float wd,
                                  float b2, float omb2, float eps) {
  const AdamConsts k = table[*step_ptr];
  const float coef = coef_ptr ? *coef_ptr : 1.f;
  const long long n4 = n / 4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    f32x4 pp = *reinterpret_cast<f32x4*>(p + 4 * i);
    f32x4 mm = *reinterpret_cast<f32x4*>(m + 4 * i);
    f32x4 vv = *reinterpret_cast<f32x4*>(v + 4 * i);
    const f32x4 gg = *reinterpret_cast<const f32x4*>(g + 4 * i);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pp[e], me = mm[e], ve = vv[e];
      adam_elem(pe, me, ve, gg[e], coef, wd, b2, omb2, eps, k);
      pp[e] = pe; mm[e] = me; vv[e] = ve;
    }
    *reinterpret_cast<f32x4*>(p + 4 * i) = pp;
    *reinterpret_cast<f32x4*>(m + 4 * i) = mm;
    *reinterpret_cast<f32x4*>(v + 4 * i) = vv;
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_elem(pp, mm, vv, g[i], coef, wd, b2, omb2, eps, k);
    p[i] = pp; m[i] = mm; v[i] = vv;
  }
}

// One group of D/4 lanes per row; rows_per_wave = 256/D.  map[r] = slot of r in gU or -1.
template <int D>
__global__ void __launch_bounds__(256) adam_table_kernel(float* __restrict__ p, float* __restrict__ m,
                                                         float* __restrict__ v, long long nrows, int* __restrict__ map,
                                                         const float* __restrict__ gU, const float* __restrict__ coef_ptr,
                                                         const AdamConsts* __restrict__ table,
                                                         const int* __restrict__ step_ptr, float wd, float b2, float omb2,
                                                         float eps) {
  constexpr int G = D / 4;
  constexpr int RPW = 64 / G;
  const AdamConsts k = table[*step_ptr];
  const float coef = coef_ptr ? *coef_ptr : 1.f;
  const int lane = threadIdx.x & 63, q = lane % G;
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long r0 = gw * RPW; r0 < nrows; r0 += nw * RPW) {
    const long long r = r0 + lane / G;
    if (r >= nrows) continue;
    const int u = map[r];
    const size_t off = (size_t)r * D + 4 * q;
    f32x4 pp = *reinterpret_cast<f32x4*>(p + off);
    f32x4 mm = *reinterpret_cast<f32x4*>(m + off);
    f32x4 vv = *reinterpret_cast<f32x4*>(v + off);
    f32x4 gg = {0.f, 0.f, 0.f, 0.f};
    if (u >= 0) gg = *reinterpret_cast<const f32x4*>(gU + (size_t)u * D + 4 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pp[e], me = mm[e], ve = vv[e];
      adam_elem(pe, me, ve, gg[e], coef, wd, b2, omb2, eps, k);
      pp[e] = pe; mm[e] = me; vv[e] = ve;
    }
    *reinterpret_cast<f32x4*>(p + off) = pp;
    *reinterpret_cast<f32x4*>(m + off) = mm;
    *reinterpret_cast<f32x4*>(v + off) = vv;
    if (u >= 0 && q == 0) map[r] = -1;
  }
}

// end of step: advance Adam step + dropout RNG offset, clear sparse-grad bookkeeping
__global__ void step_end_kernel(int* step, unsigned long long* rng, int* n_uniq, double* sumsq) {
  step[0] += 1;
  if (rng) rng[1] += 1;
  if (n_uniq) n_uniq[0] = 0;
  if (sumsq) sumsq[0] = 0.0;
}

// gU rows [0, n_uniq) zero-fill (the next step's scatter target)
__global__ void zero_rows_kernel(float* gU, const int* n_uniq, int D) {
  const long long lim = (long long)(*n_uniq) * D;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += (long long)gridDim.x * blockDim.x)
    gU[i] = 0.f;
}

// ------------------------------------------------------------------ C ABI
extern "C" int fbn_sumsq(const float* x, long long n, const int* n_rows, int row_len, double* out, void* stream) {
  if (n <= 0 && !n_rows) return FBN_OK;
  hipLaunchKernelGGL(sumsq_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, x, n, n_rows, row_len, out);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_clip_coef(const double* sumsq, float max_norm, float* coef, float* norm, void* stream) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, sumsq, max_norm, coef, norm);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_adam_dense(float* p, const float* g, float* m, float* v, long long n, const float* coef,
                              const void* consts_table, const int* step, float wd, float beta2, float eps,
                              void* stream) {
  if (n <= 0) return FBN_OK;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) {
    fbn_set_error("adam_dense: 16-byte alignment required");
    return FBN_ERR_ARG;
  }
  long long blocks = (n / 4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_dense_kernel, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, coef,
                     (const AdamConsts*)consts_table, step, wd, beta2, (float)(1.0 - (double)beta2), eps);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_adam_table(float* p, float* m, float* v, long long nrows, int D, int* map, const float* gU,
                              const float* coef, const void* consts_table, const int* step, float wd, float beta2,
                              float eps, void* stream) {
  if (nrows <= 0) return FBN_OK;
  const int rpw = 256 / D;
  long long waves = (nrows + rpw - 1) / rpw;
  long long blocks = (waves + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  hipStream_t st = (hipStream_t)stream;
  const float omb2 = (float)(1.0 - (double)beta2);
  const AdamConsts* t = (const AdamConsts*)consts_table;
  switch (D) {
    case 16: hipLaunchKernelGGL((adam_table_kernel<16>), dim3((int)blocks), dim3(256), 0, st, p, m, v, nrows, map, gU, coef, t, step, wd, beta2, omb2, eps); break;
    case 32: hipLaunchKernelGGL((adam_table_kernel<32>), dim3((int)blocks), dim3(256), 0, st, p, m, v, nrows, map, gU, coef, t, step, wd, beta2, omb2, eps); break;
    case 64: hipLaunchKernelGGL((adam_table_kernel<64>), dim3((int)blocks), dim3(256), 0, st, p, m, v, nrows, map, gU, coef, t, step, wd, beta2, omb2, eps); break;
    case 128: hipLaunchKernelGGL((adam_table_kernel<128>), dim3((int)blocks), dim3(256), 0, st, p, m, v, nrows, map, gU, coef, t, step, wd, beta2, omb2, eps); break;
    case 256: hipLaunchKernelGGL((adam_table_kernel<256>), dim3((int)blocks), dim3(256), 0, st, p, m, v, nrows, map, gU, coef, t, step, wd, beta2, omb2, eps); break;
    default: fbn_set_error("adam_table: D must be 16/32/64/128/256"); return FBN_ERR_UNSUPPORTED;
  }
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_step_end(int* step, unsigned long long* rng, int* n_uniq, double* sumsq, void* stream) {
  hipLaunchKernelGGL(step_end_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step, rng, n_uniq, sumsq);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_zero_rows(float* gU, const int* n_uniq, int D, void* stream) {
  hipLaunchKernelGGL(zero_rows_kernel, dim3(1024), dim3(256), 0, (hipStream_t)stream, gU, n_uniq, D);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}
