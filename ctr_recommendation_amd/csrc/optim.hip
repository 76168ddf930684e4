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
#include <cstdlib>

#pragma clang fp contract(off)

// squared-norm accumulators: FBN_SUMSQ_SLOTS doubles, block b adds into slot b % SLOTS (one
// address per block would serialise the returning-free f64 atomics of thousands of blocks)
#define FBN_SUMSQ_SLOTS 64

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
  if (threadIdx.x == 0) atomicAdd(out + (blockIdx.x & (FBN_SUMSQ_SLOTS - 1)), red[0]);
}

// coef = min(1, max_norm / (sqrt(total) + 1e-6)); also exposes the norm
__global__ void clip_coef_kernel(const double* sumsq, float max_norm, float* coef_out, float* norm_out) {
  double s = 0.0;
  for (int i = 0; i < FBN_SUMSQ_SLOTS; ++i) s += sumsq[i];
  const float total = sqrtf((float)s);
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

// clip coefficient of clip_grad_norm_ from the sumsq slots (same sequential order as
// clip_coef_kernel, so the value is bit-identical)
__device__ __forceinline__ float clip_from_slots(const double* sumsq, float max_norm, float* total_out) {
  double s = 0.0;
  for (int i = 0; i < FBN_SUMSQ_SLOTS; ++i) s += sumsq[i];
  const float total = sqrtf((float)s);
  const float c = max_norm / (total + 1e-6f);
  *total_out = total;
  return c < 1.f ? c : 1.f;
}

// sumsq != null: the clip coefficient is computed here (every block, thread 0) and block 0
// publishes it (coef_out, norm_out) for the table passes that follow -- no clip_coef launch.
__global__ void adam_dense_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                  float* __restrict__ v, long long n, const float* __restrict__ coef_ptr,
                                  const AdamConsts* __restrict__ table, const int* __restrict__ step_ptr, float wd,
                                  float b2, float omb2, float eps, const double* __restrict__ sumsq, float max_norm,
                                  float* coef_out, float* norm_out) {
  const AdamConsts k = table[*step_ptr];
  float coef;
  if (sumsq) {
    __shared__ float sc;
    if (threadIdx.x == 0) {
      float total;
      sc = clip_from_slots(sumsq, max_norm, &total);
      if (blockIdx.x == 0) {
        if (coef_out) *coef_out = sc;
        if (norm_out) *norm_out = total;
      }
    }
    __syncthreads();
    coef = sc;
  } else {
    coef = coef_ptr ? *coef_ptr : 1.f;
  }
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

// ------------------------------------------------------------------ sparse table gradient
// Slots are entry indices.  Single GPU: entry e = b*(L+1)+t (t = 0 item, t >= 1 history), its
// gradient vector is gvec[b][t ? 1 : 0] (the backward stores 2 vectors per sample); a row hit
// by several entries keeps them in `extra` (slot of the claiming entry; FLAG in slot_row).
// Multi-GPU owner: entry = received row i, its gradient is rows[i] (Lp1 = 1), duplicates are
// added into the claimer's own row.
#define FBN_SLOT_FLAG 0x40000000
struct GradSrc {
  const float* vec;     // Lp1 > 1: [B][2][D] per-sample vectors;  Lp1 == 1: [n][D] per-entry rows
  float* extra;         // [n][D] duplicate accumulation (single GPU) or null
  int* slot_row;        // [n] claimed row | FLAG, or -1
  int Lp1;
};
template <int D>
__device__ __forceinline__ const float* grad_base(const GradSrc& s, int e) {
  if (s.Lp1 == 1) return s.vec + (size_t)e * D;
  const int b = e / s.Lp1, t = e - b * s.Lp1;
  return s.vec + ((size_t)b * 2 + (t ? 1 : 0)) * D;
}

// duplicates of a claimed row: single GPU -> extra[claimer] += vec(e) (and flag the claimer);
// owner mode -> rows[claimer] += rows[e].  One G-lane group per entry, contiguous atomics.
template <int D>
__global__ void __launch_bounds__(256) sparse_fixup_kernel(const int64_t* __restrict__ item,
                                                           const int64_t* __restrict__ seq, const int* __restrict__ ids,
                                                           int n, int L, long long V, int rank,
                                                           const int* __restrict__ map, GradSrc s) {
  constexpr int G = D / 4, RPW = 64 / G;
  const int lane = threadIdx.x & 63, q = lane % G;
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long e0 = gw * RPW; e0 < n; e0 += nw * RPW) {
    const long long e = e0 + lane / G;
    if (e >= n) continue;
    long long r;
    if (ids) {
      r = ids[e];
      if (rank == 0 && r == 0) continue;
    } else {
      const long long b = e / (L + 1), t = e - b * (L + 1);
      r = t == 0 ? item[b] : seq[b * L + (t - 1)];
      if (r <= 0 || r >= V) continue;
    }
    const int u = map[r];
    if (u == (int)e || u < 0) continue;
    const float* src = grad_base<D>(s, (int)e);
    float* dst;
    if (s.extra) {
      if (q == 0) atomicOr(&s.slot_row[u], FBN_SLOT_FLAG);
      dst = s.extra + (size_t)u * D;
    } else {
      dst = const_cast<float*>(s.vec) + (size_t)u * D;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(dst + k * G + q, src[k * G + q]);
  }
}

// Row claiming for the sparse gradient (single GPU): entry e = b*(L+1)+t claims row r if it is
// the first to touch it.  Run as the first kernel of a step so the untouched-row Adam can start
// on the side stream before the forward's GEMMs.
// dup (optional): dup[e] = the entry that claimed e's row when that is not e itself, else -1
// (a claim never changes within a step, so the value a failed claim observes is final); the
// fix-up then reads dup coalesced instead of re-resolving every id through the map.
__global__ void claim_rows_kernel(const int64_t* __restrict__ item, const int64_t* __restrict__ seq, int B, int L,
                                  long long V, int* __restrict__ map, int* __restrict__ slot_row, int* __restrict__ dup) {
  const long long n = (long long)B * (L + 1);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long b = e / (L + 1), t = e - b * (L + 1);
    const long long r = t == 0 ? item[b] : seq[b * L + (t - 1)];
    int owner = -1;
    if (r > 0 && r < V) {
      owner = __hip_atomic_load(map + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (owner == -1) {
        int expected = -1;
        if (__hip_atomic_compare_exchange_strong(map + r, &expected, (int)e, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
          slot_row[e] = (int)r;
        else
          owner = expected;
      }
    }
    if (dup) dup[e] = owner;
  }
}

// duplicates resolved at claim time (single GPU): extra[dup[e]] += vec(e), claimer flagged
template <int D>
__global__ void __launch_bounds__(256) sparse_fixup_dup_kernel(const int* __restrict__ dup, int n, GradSrc s) {
  constexpr int G = D / 4, RPW = 64 / G;
  const int lane = threadIdx.x & 63, q = lane % G;
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long e0 = gw * RPW; e0 < n; e0 += nw * RPW) {
    const long long e = e0 + lane / G;
    const int u = e < n ? dup[e] : -1;
    if (u < 0) continue;
    const float* src = grad_base<D>(s, (int)e);
    if (q == 0) atomicOr(&s.slot_row[u], FBN_SLOT_FLAG);
    float* dst = s.extra + (size_t)u * D;
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(dst + k * G + q, src[k * G + q]);
  }
}

// sum of squares of the table gradient from per-sample vector norms (fbn_fields_bwd's gnorm
// [B][2]): a claiming entry without duplicates adds its vector's norm; one with duplicates
// (FLAG) sums vector + extra explicitly.  One thread per entry, coalesced slot_row reads.
template <int D>
__global__ void __launch_bounds__(256) sumsq_norms_kernel(GradSrc s, const double* __restrict__ gnorm, int n,
                                                          double* __restrict__ out) {
  __shared__ double red[4];
  double acc = 0.0;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int sr = s.slot_row[e];
    if (sr == -1) continue;
    const int b = (int)(e / s.Lp1), t = (int)(e - (long long)b * s.Lp1);
    if (!(sr & FBN_SLOT_FLAG)) {
      acc += gnorm[(size_t)b * 2 + (t ? 1 : 0)];
    } else {
      const float* v = grad_base<D>(s, (int)e);
      const float* x = s.extra + (size_t)e * D;
      for (int k = 0; k < D; ++k) {
        const float y = v[k] + x[k];
        acc += (double)(y * y);
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out + (blockIdx.x & (FBN_SUMSQ_SLOTS - 1)), (red[0] + red[1]) + (red[2] + red[3]));
}

// sum of squares of the clipped-to-be table gradient, over claiming entries only
template <int D>
__global__ void __launch_bounds__(256) sumsq_sparse_kernel(GradSrc s, int n, double* __restrict__ out) {
  constexpr int G = D / 4, RPW = 64 / G;
  __shared__ double red[256];
  const int lane = threadIdx.x & 63, q = lane % G;
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  double acc = 0.0;
  for (long long e0 = gw * RPW; e0 < n; e0 += nw * RPW) {
    const long long e = e0 + lane / G;
    if (e >= n) continue;
    const int sr = s.slot_row[e];
    if (sr == -1) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(grad_base<D>(s, (int)e) + 4 * q);
    if (sr & FBN_SLOT_FLAG) v += *reinterpret_cast<const f32x4*>(s.extra + (size_t)e * D + 4 * q);
    acc += (double)(v[0] * v[0]) + (double)(v[1] * v[1]) + (double)(v[2] * v[2]) + (double)(v[3] * v[3]);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(out + (blockIdx.x & (FBN_SUMSQ_SLOTS - 1)), red[0]);
}

// One group of D/4 lanes per row; rows_per_wave = 256/D.  map[r] = claiming entry or -1.
// UNTOUCHED_ONLY: update only rows the batch did not touch (map[r] == -1).  Their gradient is
// exactly 0, so the update (g = 0*coef + wd*p) does not depend on the backward or the clip
// coefficient and runs on a side stream concurrently with the whole backward; the touched
// rows are updated afterwards by adam_touched_kernel.  Otherwise: every row, reading the
// gradient of touched rows through the map.
template <int D, bool UNTOUCHED_ONLY>
__device__ __forceinline__ void adam_table_body(float* __restrict__ p, float* __restrict__ m,
                                                         float* __restrict__ v, long long nrows, int* __restrict__ map,
                                                         GradSrc gs, const float* __restrict__ coef_ptr,
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
    if (UNTOUCHED_ONLY && u >= 0) continue;
    const size_t off = (size_t)r * D + 4 * q;
    f32x4 pp = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(p + off));
    f32x4 mm = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(m + off));
    f32x4 vv = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(v + off));
    f32x4 gg = {0.f, 0.f, 0.f, 0.f};
    if (!UNTOUCHED_ONLY && u >= 0) {
      gg = *reinterpret_cast<const f32x4*>(grad_base<D>(gs, u) + 4 * q);
      if (gs.extra && (gs.slot_row[u] & FBN_SLOT_FLAG)) {
        float* ex = gs.extra + (size_t)u * D + 4 * q;
        gg += *reinterpret_cast<const f32x4*>(ex);
        *reinterpret_cast<f32x4*>(ex) = (f32x4){0.f, 0.f, 0.f, 0.f};   // keep `extra` all-zero
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pp[e], me = mm[e], ve = vv[e];
      adam_elem(pe, me, ve, gg[e], coef, wd, b2, omb2, eps, k);
      pp[e] = pe; mm[e] = me; vv[e] = ve;
    }
    __builtin_nontemporal_store(pp, reinterpret_cast<f32x4*>(p + off));
    __builtin_nontemporal_store(mm, reinterpret_cast<f32x4*>(m + off));
    __builtin_nontemporal_store(vv, reinterpret_cast<f32x4*>(v + off));
    if (!UNTOUCHED_ONLY && u >= 0 && q == 0) map[r] = -1;
  }
}

#define FBN_ADAM_TABLE_ARGS                                                                                  \
  float *p, float *m, float *v, long long nrows, int *map, GradSrc gs, const float *coef, const AdamConsts *t,   \
      const int *step, float wd, float b2, float omb2, float eps
template <int D>
__global__ void __launch_bounds__(256) adam_table_all(FBN_ADAM_TABLE_ARGS) {
  adam_table_body<D, false>(p, m, v, nrows, map, gs, coef, t, step, wd, b2, omb2, eps);
}

// Untouched rows, as a low-footprint streaming kernel: it runs beside the backward on a side
// stream, so it must not take the CUs' wave slots from the backward's kernels.  Launched with
// <= 2 workgroups per CU; each lane keeps UNR rows (3 x 16 B each) in flight so the few waves
// still stream HBM near its rate (Little: ~12 MB in flight chip-wide).
template <int D>
__global__ void __launch_bounds__(256) adam_table_untouched(FBN_ADAM_TABLE_ARGS) {
  constexpr int G = D / 4, RPW = 64 / G, UNR = 4;
  const AdamConsts k = t[*step];
  const int lane = threadIdx.x & 63, q = lane % G;
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long r0 = gw * RPW * UNR; r0 < nrows; r0 += nw * RPW * UNR) {
    f32x4 pp[UNR], mm[UNR], vv[UNR];
    bool act[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long r = r0 + u * RPW + lane / G;
      act[u] = r < nrows && map[r] < 0;
      if (act[u]) {
        const size_t off = (size_t)r * D + 4 * q;
        pp[u] = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(p + off));
        mm[u] = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(m + off));
        vv[u] = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(v + off));
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (!act[u]) continue;
      const long long r = r0 + u * RPW + lane / G;
      const size_t off = (size_t)r * D + 4 * q;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = pp[u][e], me = mm[u][e], ve = vv[u][e];
        adam_elem(pe, me, ve, 0.f, 1.f, wd, b2, omb2, eps, k);
        pp[u][e] = pe; mm[u][e] = me; vv[u][e] = ve;
      }
      __builtin_nontemporal_store(pp[u], reinterpret_cast<f32x4*>(p + off));
      __builtin_nontemporal_store(mm[u], reinterpret_cast<f32x4*>(m + off));
      __builtin_nontemporal_store(vv[u], reinterpret_cast<f32x4*>(v + off));
    }
  }
}

// ------------------------------------------------------------------ lazy table Adam (exact)
// A row whose loss gradient is zero at step s still gets torch's coupled-L2 Adam update
// (g = 0 * coef + wd * p, then m, v, p).  That update depends only on the row and on step s's
// schedule constants, so it can be REPLAYED later with the same float operations in the same
// order: bit-identical to stepping it eagerly.  last[r] = number of Adam steps applied to row r.
// Each step, before the gather reads the table, fbn_adam_catchup brings every row the batch
// claimed, plus a rolling window of nrows/F rows (window (step mod F)), up to `step`; the rolling
// window bounds every row's lag by F steps.  fbn_adam_touched then applies the step with the real
// gradient (last = step + 1).  fbn_adam_flush brings the whole table up to date (checkpoint,
// evaluation).  The schedule constants of the last W <= FBN_LAZY_MAX_LAG steps sit in LDS.
#define FBN_LAZY_MAX_LAG 512

template <int D>
__device__ __forceinline__ void replay_rows(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                            long long r, int q, int k0, int t, const AdamConsts* __restrict__ win,
                                            int w0, const AdamConsts* __restrict__ table, float wd, float b2,
                                            float omb2, float eps) {
  const size_t off = (size_t)r * D + 4 * q;
  f32x4 pp = *reinterpret_cast<f32x4*>(p + off);
  f32x4 mm = *reinterpret_cast<f32x4*>(m + off);
  f32x4 vv = *reinterpret_cast<f32x4*>(v + off);
  for (int s = k0; s < t; ++s) {
    // the rolling window keeps every row within F <= FBN_LAZY_MAX_LAG steps, so the constants of
    // steps k0 .. t-1 are all in the LDS window (a global fallback would turn this into flat loads)
    const AdamConsts k = win[s - w0];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pp[e], me = mm[e], ve = vv[e];
      adam_elem(pe, me, ve, 0.f, 1.f, wd, b2, omb2, eps, k);
      pp[e] = pe; mm[e] = me; vv[e] = ve;
    }
  }
  *reinterpret_cast<f32x4*>(p + off) = pp;
  *reinterpret_cast<f32x4*>(m + off) = mm;
  *reinterpret_cast<f32x4*>(v + off) = vv;
}

// items [0, n_ent): claiming entries (slot_row != -1); items [n_ent, n_ent + chunk): rows of the
// rolling window not claimed this step.  nrows_total / F / chunk describe the window.
template <int D>
__global__ void __launch_bounds__(256) adam_catchup_kernel(float* __restrict__ p, float* __restrict__ m,
                                                           float* __restrict__ v, const int* __restrict__ slot_row,
                                                           int n_ent, const int* __restrict__ map, long long nrows,
                                                           int F, long long chunk, int parts, int* __restrict__ last,
                                                           const AdamConsts* __restrict__ table,
                                                           const int* __restrict__ step, float wd, float b2,
                                                           float omb2, float eps) {
  constexpr int G = D / 4, RPW = 64 / G;
  __shared__ AdamConsts win[FBN_LAZY_MAX_LAG];
  const int t = *step;
  const int w0 = t > FBN_LAZY_MAX_LAG ? t - FBN_LAZY_MAX_LAG : 0;
  for (int i = threadIdx.x; i < t - w0; i += blockDim.x) win[i] = table[w0 + i];
  __syncthreads();
  const long long roll0 = (long long)(t % F) * chunk;
  const long long nroll = (parts & 2) && roll0 < nrows ? min(chunk, nrows - roll0) : 0;
  if (!(parts & 1)) n_ent = 0;
  const long long n = n_ent + nroll;
  const int lane = threadIdx.x & 63, q = lane % G;
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long i0 = gw * RPW; i0 < n; i0 += nw * RPW) {
    const long long i = i0 + lane / G;
    if (i >= n) continue;
    long long r;
    if (i < n_ent) {
      const int sr = slot_row[i];
      if (sr == -1) continue;
      r = sr & ~FBN_SLOT_FLAG;
    } else {
      r = roll0 + (i - n_ent);
      if (map && map[r] != -1) continue;   // claimed this step: its claiming entry replays it
    }
    const int k0 = last[r];
    if (k0 >= t) continue;
    replay_rows<D>(p, m, v, r, q, k0, t, win, w0, table, wd, b2, omb2, eps);
    if (q == 0) last[r] = t;
  }
}

// every row up to `step` (checkpoint / evaluation)
template <int D>
__global__ void __launch_bounds__(256) adam_flush_kernel(float* __restrict__ p, float* __restrict__ m,
                                                         float* __restrict__ v, long long nrows, int* __restrict__ last,
                                                         const AdamConsts* __restrict__ table,
                                                         const int* __restrict__ step, float wd, float b2, float omb2,
                                                         float eps) {
  constexpr int G = D / 4, RPW = 64 / G;
  __shared__ AdamConsts win[FBN_LAZY_MAX_LAG];
  const int t = *step;
  const int w0 = t > FBN_LAZY_MAX_LAG ? t - FBN_LAZY_MAX_LAG : 0;
  for (int i = threadIdx.x; i < t - w0; i += blockDim.x) win[i] = table[w0 + i];
  __syncthreads();
  const int lane = threadIdx.x & 63, q = lane % G;
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long r0 = gw * RPW; r0 < nrows; r0 += nw * RPW) {
    const long long r = r0 + lane / G;
    if (r >= nrows) continue;
    const int k0 = last[r];
    if (k0 >= t) continue;
    replay_rows<D>(p, m, v, r, q, k0, t, win, w0, table, wd, b2, omb2, eps);
    if (q == 0) last[r] = t;
  }
}

// Touched rows: one group per claiming entry e (slot_row[e] = row | FLAG); gradient =
// gvec-slot(e) (+ extra[e]); Adam with the clip coefficient; the row's map entry is reset.
template <int D>
__global__ void __launch_bounds__(256) adam_touched_kernel(float* __restrict__ p, float* __restrict__ m,
                                                           float* __restrict__ v, int* __restrict__ map, GradSrc gs,
                                                           int n, const float* __restrict__ coef_ptr,
                                                           const AdamConsts* __restrict__ table,
                                                           const int* __restrict__ step_ptr, float wd, float b2,
                                                           float omb2, float eps, int* __restrict__ last) {
  constexpr int G = D / 4, RPW = 64 / G;
  const AdamConsts k = table[*step_ptr];
  const float coef = coef_ptr ? *coef_ptr : 1.f;
  const int lane = threadIdx.x & 63, q = lane % G;
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long e0 = gw * RPW; e0 < n; e0 += nw * RPW) {
    const long long e = e0 + lane / G;
    if (e >= n) continue;
    const int sr = gs.slot_row[e];
    if (sr == -1) continue;
    const long long r = sr & ~FBN_SLOT_FLAG;
    f32x4 gg = *reinterpret_cast<const f32x4*>(grad_base<D>(gs, (int)e) + 4 * q);
    if (sr & FBN_SLOT_FLAG) {
      float* ex = gs.extra + (size_t)e * D + 4 * q;
      gg += *reinterpret_cast<const f32x4*>(ex);
      *reinterpret_cast<f32x4*>(ex) = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    const size_t off = (size_t)r * D + 4 * q;
    f32x4 pp = *reinterpret_cast<f32x4*>(p + off);
    f32x4 mm = *reinterpret_cast<f32x4*>(m + off);
    f32x4 vv = *reinterpret_cast<f32x4*>(v + off);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float pe = pp[c], me = mm[c], ve = vv[c];
      adam_elem(pe, me, ve, gg[c], coef, wd, b2, omb2, eps, k);
      pp[c] = pe; mm[c] = me; vv[c] = ve;
    }
    *reinterpret_cast<f32x4*>(p + off) = pp;
    *reinterpret_cast<f32x4*>(m + off) = mm;
    *reinterpret_cast<f32x4*>(v + off) = vv;
    if (q == 0) {
      map[r] = -1;
      if (last) last[r] = *step_ptr + 1;
    }
  }
}

// end of step: advance Adam step + dropout RNG offset, clear the norm accumulator
__global__ void step_end_kernel(int* step, unsigned long long* rng, double* sumsq, long long* nbt0, long long* nbt1) {
  step[0] += 1;
  if (rng) rng[1] += 1;
  if (nbt0) nbt0[0] += 1;   // BatchNorm num_batches_tracked
  if (nbt1) nbt1[0] += 1;
  if (sumsq)
    for (int i = 0; i < FBN_SUMSQ_SLOTS; ++i) sumsq[i] = 0.0;
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
                              const double* sumsq, float max_norm, float* coef_out, float* norm_out, void* stream) {
  if (n <= 0) return FBN_OK;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) {
    fbn_set_error("adam_dense: 16-byte alignment required");
    return FBN_ERR_ARG;
  }
  long long blocks = (n / 4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_dense_kernel, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, coef,
                     (const AdamConsts*)consts_table, step, wd, beta2, (float)(1.0 - (double)beta2), eps, sumsq,
                     max_norm, coef_out, norm_out);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

#define FBN_DISPATCH_D(KERNEL, D, GRID, ...)                                                         \
  switch (D) {                                                                                      \
    case 16: hipLaunchKernelGGL((KERNEL<16>), GRID, dim3(256), 0, st, __VA_ARGS__); break;          \
    case 32: hipLaunchKernelGGL((KERNEL<32>), GRID, dim3(256), 0, st, __VA_ARGS__); break;          \
    case 64: hipLaunchKernelGGL((KERNEL<64>), GRID, dim3(256), 0, st, __VA_ARGS__); break;          \
    case 128: hipLaunchKernelGGL((KERNEL<128>), GRID, dim3(256), 0, st, __VA_ARGS__); break;        \
    case 256: hipLaunchKernelGGL((KERNEL<256>), GRID, dim3(256), 0, st, __VA_ARGS__); break;        \
    default: fbn_set_error("D must be 16/32/64/128/256"); return FBN_ERR_UNSUPPORTED;              \
  }

static dim3 group_grid(long long n, int D, long long cap) {
  const int rpw = 256 / D;
  long long blocks = ((n + rpw - 1) / rpw + 3) / 4;
  if (blocks < 1) blocks = 1;
  if (blocks > cap) blocks = cap;
  return dim3((unsigned)blocks);
}

// gvec: single GPU per-sample vectors [B][2][D] (Lp1 = L+1) or owner per-entry rows [n][D] (Lp1 = 1)
extern "C" int fbn_sparse_fixup(const int64_t* item, const int64_t* seq, const int* ids, int n, int L, long long V,
                                int rank, const int* map, const float* gvec, float* extra, int* slot_row, int Lp1,
                                int D, void* stream) {
  if (n <= 0) return FBN_OK;
  hipStream_t st = (hipStream_t)stream;
  GradSrc s{gvec, extra, slot_row, Lp1};
  FBN_DISPATCH_D(sparse_fixup_kernel, D, group_grid(n, D, 8192), item, L > 0 ? seq : nullptr, ids, n, L, V, rank,
                 map, s);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// single GPU: the fix-up from claim-time duplicates (fbn_claim_rows' dup), then the table
// gradient's sum of squares from fbn_fields_bwd's per-sample norms
extern "C" int fbn_sparse_fixup_dup(const int* dup, int n, const float* gvec, float* extra, int* slot_row, int Lp1,
                                    int D, void* stream) {
  if (n <= 0) return FBN_OK;
  if (!dup || !extra) { fbn_set_error("fbn_sparse_fixup_dup: dup and extra are required"); return FBN_ERR_ARG; }
  hipStream_t st = (hipStream_t)stream;
  GradSrc s{gvec, extra, slot_row, Lp1};
  FBN_DISPATCH_D(sparse_fixup_dup_kernel, D, group_grid(n, D, 4096), dup, n, s);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_sumsq_sparse_norms(const double* gnorm, const float* gvec, float* extra, int* slot_row, int Lp1,
                                      int n, int D, double* out, void* stream) {
  if (n <= 0) return FBN_OK;
  if (Lp1 < 2) { fbn_set_error("fbn_sumsq_sparse_norms: per-sample vectors only (Lp1 >= 2)"); return FBN_ERR_ARG; }
  hipStream_t st = (hipStream_t)stream;
  GradSrc s{gvec, extra, slot_row, Lp1};
  int blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  FBN_DISPATCH_D(sumsq_norms_kernel, D, dim3(blocks), s, gnorm, n, out);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_sumsq_sparse(const float* gvec, float* extra, int* slot_row, int Lp1, int n, int D, double* out,
                                void* stream) {
  if (n <= 0) return FBN_OK;
  hipStream_t st = (hipStream_t)stream;
  GradSrc s{gvec, extra, slot_row, Lp1};
  FBN_DISPATCH_D(sumsq_sparse_kernel, D, group_grid(n, D, 4096), s, n, out);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// mode 0: every row (touched rows read their gradient through the map and are reset);
// mode 1: untouched rows only (g = 0, coefficient-independent; run it concurrently with the
// backward, then fbn_adam_touched once the clip coefficient is known), throttled to 512
// workgroups so it leaves CUs to the backward; mode 2: as mode 1 on the full grid (serial use)
extern "C" int fbn_adam_table(float* p, float* m, float* v, long long nrows, int D, int* map, const float* gvec,
                              float* extra, int* slot_row, int Lp1, const float* coef, const void* consts_table,
                              const int* step, float wd, float beta2, float eps, int mode, void* stream) {
  if (nrows <= 0) return FBN_OK;
  hipStream_t st = (hipStream_t)stream;
  const float omb2 = (float)(1.0 - (double)beta2);
  const AdamConsts* t = (const AdamConsts*)consts_table;
  GradSrc s{gvec, extra, slot_row, Lp1};
  static const int throttle = getenv("FBN_ADAM_BLOCKS") ? atoi(getenv("FBN_ADAM_BLOCKS")) : 512;   // tuning knob
  const dim3 grid = mode == 1 ? dim3(throttle) : group_grid(nrows, D, 16384);
  if (mode == 1 || mode == 2) {
    FBN_DISPATCH_D(adam_table_untouched, D, grid, p, m, v, nrows, map, s, coef, t, step, wd, beta2, omb2, eps);
  } else {
    FBN_DISPATCH_D(adam_table_all, D, grid, p, m, v, nrows, map, s, coef, t, step, wd, beta2, omb2, eps);
  }
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_adam_touched(float* p, float* m, float* v, int D, int* map, const float* gvec, float* extra,
                                int* slot_row, int Lp1, int n, const float* coef, const void* consts_table,
                                const int* step, float wd, float beta2, float eps, int* last, void* stream) {
  if (n <= 0) return FBN_OK;
  hipStream_t st = (hipStream_t)stream;
  const float omb2 = (float)(1.0 - (double)beta2);
  const AdamConsts* t = (const AdamConsts*)consts_table;
  GradSrc s{gvec, extra, slot_row, Lp1};
  FBN_DISPATCH_D(adam_touched_kernel, D, group_grid(n, D, 8192), p, m, v, map, s, n, coef, t, step, wd, beta2,
                 omb2, eps, last);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_claim_rows(const int64_t* item, const int64_t* seq, int B, int L, long long V, int* map,
                              int* slot_row, int* dup, void* stream) {
  const long long n = (long long)B * (L + 1);
  if (n <= 0) return FBN_OK;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(claim_rows_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, item, L > 0 ? seq : nullptr,
                     B, L, V, map, slot_row, dup);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_step_end(int* step, unsigned long long* rng, double* sumsq, long long* nbt0, long long* nbt1,
                            void* stream) {
  hipLaunchKernelGGL(step_end_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step, rng, sumsq, nbt0, nbt1);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}


// lazy table Adam: replay the zero-loss-gradient steps of the claimed rows and of rolling window
// (step mod F) (chunk = ceil(nrows / F) rows) up to `step`; last: [nrows] steps applied per row
// parts: 1 = the claimed rows (must precede the gather), 2 = the rolling window (unclaimed rows:
// nothing else reads them this step -> may run on a side stream), 3 = both
extern "C" int fbn_adam_catchup(float* p, float* m, float* v, long long nrows, int D, const int* slot_row, int n_ent,
                                const int* map, int F, int parts, int* last, const void* consts_table, const int* step,
                                float wd, float beta2, float eps, void* stream) {
  if (nrows <= 0) return FBN_OK;
  if (F < 1 || F > FBN_LAZY_MAX_LAG) { fbn_set_error("fbn_adam_catchup: 1 <= F <= 512"); return FBN_ERR_ARG; }
  hipStream_t st = (hipStream_t)stream;
  const float omb2 = (float)(1.0 - (double)beta2);
  const long long chunk = (nrows + F - 1) / F;
  const long long items = ((parts & 1) ? n_ent : 0) + ((parts & 2) ? chunk : 0);
  if (items <= 0) return FBN_OK;
  // the window-only pass runs beside the step: a few workgroups per CU leave the CUs' wave
  // slots to the main stream while its four-chain replay keeps the VALU busy
  static const int wcap = getenv("FBN_WINDOW_BLOCKS") ? atoi(getenv("FBN_WINDOW_BLOCKS")) : 256;   // tools/window_sweep.sh
  const long long cap = parts == 2 ? wcap : 8192;
  FBN_DISPATCH_D(adam_catchup_kernel, D, group_grid(items, D, cap), p, m, v, slot_row, n_ent, map, nrows, F, chunk,
                 parts, last, (const AdamConsts*)consts_table, step, wd, beta2, omb2, eps);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_adam_flush(float* p, float* m, float* v, long long nrows, int D, int* last, const void* consts_table,
                              const int* step, float wd, float beta2, float eps, void* stream) {
  if (nrows <= 0) return FBN_OK;
  hipStream_t st = (hipStream_t)stream;
  const float omb2 = (float)(1.0 - (double)beta2);
  FBN_DISPATCH_D(adam_flush_kernel, D, group_grid(nrows, D, 16384), p, m, v, nrows, last,
                 (const AdamConsts*)consts_table, step, wd, beta2, omb2, eps);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// Multi-GPU: the loss and this rank's table-gradient sum of squares ride in the dense-gradient
// all-reduce (two floats appended to it): pack before, unpack after (sumsq += all ranks' table
// norms; the loss becomes the global mean).  One thread each.
__global__ void pack_extras_kernel(const float* loss, double* tab_slots, float* out) {
  double s = 0.0;
  for (int i = 0; i < FBN_SUMSQ_SLOTS; ++i) {
    s += tab_slots[i];
    tab_slots[i] = 0.0;
  }
  out[0] = *loss;
  out[1] = (float)s;
}
__global__ void unpack_extras_kernel(const float* in, float* loss, double* sumsq) {
  *loss = in[0];
  sumsq[0] += (double)in[1];
}
extern "C" int fbn_pack_extras(const float* loss, double* tab_slots, float* out, void* stream) {
  hipLaunchKernelGGL(pack_extras_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, loss, tab_slots, out);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}
extern "C" int fbn_unpack_extras(const float* in, float* loss, double* sumsq, void* stream) {
  hipLaunchKernelGGL(unpack_extras_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, in, loss, sumsq);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}
