#include <cstdlib>
// K1 / K2 / K4: FiBiNET field construction, SENET and the embedding scatter-add gradient.
//
// Forward (one "sample group" of D/4 lanes per sample, each lane owning 4 contiguous
// columns, so a D=128 fp32 row is one 512-B coalesced read by 32 lanes):
//   X1 = C[likes], X2 = C[views], X3 = E[item_id], X4 = ReLU(LN(h_mm)),
//   X5 = sum_{t: s_t != 0} E[s_t] / max(1, #nonzero)         (model_fibinet.py:152-176)
//   z_f = mean_d X_f ; a = sigmoid(W2 relu(W1 z + b1) + b2) ; V_f = X_f * a_f   (:24-35)
// All 21 table rows of a sample are issued before any is consumed (21 x 16 B in flight per
// lane); the (B,20,d) history tensor of the reference is never materialised.
// V_0 == 0 (the user field is all zeros, :152), so only fields 1..5 are stored.
//
// Backward: SENET + mean + LayerNorm + ReLU backward per sample, then the embedding
// gradient: E rows get dX3 (item) and dX5/count (each non-padding history slot); row 0 is
// never written (padding_idx=0, :100).  The table gradient is accumulated either into a
// dense V x d buffer (torch drop-in semantics) or into a compact per-unique-row buffer
// addressed through a row->slot map (the native trainer: see DESIGN.md "sparse table grad").
// Small parameter gradients (SENET, LN, cate table) are reduced per block in LDS and
// written as per-block partial slabs summed by fbn_reduce_partials (deterministic).
#include "common.h"

#define FBN_MAXR 8   // max SENET reduced width supported (reference: 3)
#define FBN_MAX_L 32 // max history length (the reference keeps the last 20)
#ifndef FBN_HCH
// default history rows in flight per sample before they are summed (FBN_FIELDS_HCH: 5 / 10 / 20;
// the sum runs in slot order whatever the chunk, so every choice gives the same bits): 10 -- round 3
// measured 5 best beside the side-stream passes (0.4184 vs 0.4203 (10) vs 0.4212 ms/step (20),
// profiles/r03s2_group_knobs_ab.txt); on round 6's step the two tie on time (0.4027 / 0.4136 vs
// 0.4035 / 0.4141 ms/step, two boxes) and 10 runs the gather itself faster inside the step (in-step
// fraction of the HBM roofline 0.52-0.61 vs 0.37-0.51; profiles/r06_knob_resweep_ab.txt)
#define FBN_HCH 10
#endif

struct FieldArgs {
  const int64_t* item_id;   // [B]
  const int64_t* item_seq;  // [B][L] or null (L = 0)
  const int64_t* likes;     // [B]
  const int64_t* views;     // [B]
  const float* hmm;         // [B][D] pre-LayerNorm mm projection (bias included)
  const float* ln_g;        // [D]
  const float* ln_b;        // [D]
  const float* cate;        // [n_cate][D]
  const float* table;       // mode 0: [V][D] rows; mode 1: exchanged row buffer
  const int* pos;           // mode 1: [B][L+1] row index into `table` (-1 = none)
  const float* w1; const float* b1; const float* w2; const float* b2;  // SENET [R][6],[R],[6][R],[6]
  float* X;                 // [B][2][D] fields 3 and 5 (item row, history mean); the backward
                            // recomputes fields 1, 2 (cate rows) and 4 (LN of hmm) bit-identically
  float* Vc;                // [B][5][D] fields 1..5 (post-SENET)
  short* Vc16;              // optional bf16 copy of Vc (GEMM operand of the bilinear U = V W and its wgrad)
  void* c;                  // [B][ldc] float or bf16 (c16); cols [0,5D) <- Vc (MLP input, compact layout);
                            // null: not written (the bf16 GEMMs read those columns from Vc16)
  float* a_out;             // [B][6]
  float* cnt_out;           // [B]
  int* err;                 // id range violations (sticky flag)
  int* map;                 // sparse-grad map [V]: row -> claiming entry (-1 = untouched) or null
  int* slot_row;            // [B*(L+1)]: entry -> row it claimed, -1 otherwise (pre-filled with -1)
  long long V;              // rows of the table (mode 0)
  int B, L, ldc, R, n_cate, c16;
  float ln_eps;
  const int* hot;           // optional hot-row list (fbn_hot_rows) staged in LDS: [H] row ids
  const int* hot_n;         // its length (entries past H ignored)
  int H;
  int abl;                  // measurement only (FBN_FIELDS_ABL, tools/time_fields.py): 1 = no history
                            // loads, 2 = no field stores, 4 = no item / cate / mm loads; 0 = the real kernel
};

// hot-row staging (fbn_fields_fwd_hot, an A/B variant of the gather): up to FBN_HOT_ROWS(D) rows
// (32 KB of f32) sit in LDS, found through an open-addressed id table of twice that size
#define FBN_HOT_ROWS(D) ((8192 / (D)) < 256 ? (8192 / (D)) : 256)
__device__ __forceinline__ unsigned hot_hash(int r) { return (unsigned)r * 0x9E3779B1u; }

// Sparse-gradient registration: the first entry e = b*(L+1)+t that touches row r claims it
// (map[r] = e, slot_row[e] = r).  Slots are entry indices, so no shared counter is needed:
// a global "next free slot" atomic serialises on one address (~12 ns per wave-level atomic).
__device__ __forceinline__ void map_claim(int* map, int* slot_row, int r, int e) {
  if (__hip_atomic_load(map + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != -1) return;
  int expected = -1;
  if (__hip_atomic_compare_exchange_strong(map + r, &expected, e, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT))
    slot_row[e] = r;
}

// field 4 = ReLU(LayerNorm(h)) for this lane's 4 columns; shared by the forward and the
// backward's recompute so both run the same operations (bit-identical)
template <int G>
__device__ __forceinline__ f32x4 ln_relu(const f32x4& h, const float* ln_g, const float* ln_b, float eps, int q) {
  constexpr int D = 4 * G;
  const float s1 = group_sum<G>(h[0] + h[1] + h[2] + h[3]);
  const float mean = s1 / (float)D;
  const f32x4 dh = h - mean;
  const float s2 = group_sum<G>(dh[0] * dh[0] + dh[1] * dh[1] + dh[2] * dh[2] + dh[3] * dh[3]);
  const float rstd = 1.f / sqrtf(s2 / (float)D + eps);
  const f32x4 g4 = *reinterpret_cast<const f32x4*>(ln_g + 4 * q);
  const f32x4 bb4 = *reinterpret_cast<const f32x4*>(ln_b + 4 * q);
  f32x4 x4;
#pragma unroll
  for (int e = 0; e < 4; ++e) x4[e] = fmaxf(dh[e] * rstd * g4[e] + bb4[e], 0.f);
  return x4;
}

template <int D>
__device__ __forceinline__ void senet_excite(const float (&z)[6], const float* w1, const float* b1,
                                             const float* w2, const float* b2, int R, float (&q)[FBN_MAXR],
                                             float (&a)[6]) {
  for (int j = 0; j < R; ++j) {
    float s = b1[j];
#pragma unroll
    for (int f = 0; f < 6; ++f) s += w1[j * 6 + f] * z[f];
    q[j] = s;
  }
#pragma unroll
  for (int f = 0; f < 6; ++f) {
    float s = b2[f];
    for (int j = 0; j < R; ++j) s += w2[f * R + j] * fmaxf(q[j], 0.f);
    a[f] = 1.f / (1.f + __expf(-s));
  }
}

// row r of the exchanged row buffer (MODE 1: f32 rows; MODE 2: bf16 rows, the bf16 mode's wire format)
template <int D, int MODE>
__device__ __forceinline__ f32x4 load_row(const FieldArgs& p, size_t r, int q) {
  if constexpr (MODE == 2) {
    const bf16x4 h = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const short*>(p.table) + r * D + 4 * q);
    return (f32x4){bf2f(h[0]), bf2f(h[1]), bf2f(h[2]), bf2f(h[3])};
  } else {
    return *reinterpret_cast<const f32x4*>(p.table + r * D + 4 * q);
  }
}

// BUF (MODE 0, tables under 4 GB): the history rows are read through a buffer resource over the
// table, and a padding / past-L slot's load gets an out-of-range offset -- the buffer unit returns
// zeros without a memory request, so dead slots stay off the fetch path (the global-load form
// reads row 0 for them: an L2 hit, but L2 bandwidth and TA cycles all the same)
#define FBN_BUF_FLAGS 0x00020000   // gfx9 buffer descriptor word 3 (raw, 32-bit dwords)
// CMP: the sample's live history slots are compacted first (ballot + mbcnt; their rows staged in a
// per-sample LDS list in slot order), so a chunk of HCH loads carries only live rows and a sample
// takes ceil(n_live / HCH) rounds instead of L / HCH; summed in slot order like the plain form --
// the skipped padding slots added +0.0 there, so the two are bit-identical.
template <int D, int MODE, int HCH, bool BUF = false, bool HOT = false, bool CMP = false>
__global__ void __launch_bounds__(256) fields_fwd_kernel(FieldArgs p) {
  FBN_MAIN_PRIO();
  // (unused, and dropped, unless BUF)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.table), 0, (int)((unsigned long long)p.V * D * 4), FBN_BUF_FLAGS);
  constexpr int HR = HOT ? FBN_HOT_ROWS(D) : 1, HT = 2 * HR;   // staged rows, id-table slots
  __shared__ f32x4 hrow[HOT ? HR * (D / 4) : 1];
  __shared__ int hkey[HOT ? HT : 1];   // staged row id (-1 = empty)
  __shared__ int hval[HOT ? HT : 1];   // its index in hrow
  int nh = 0;
  if constexpr (HOT) {
    nh = min(*p.hot_n, min(p.H, HR));
    for (int i = threadIdx.x; i < HT; i += blockDim.x) hkey[i] = -1;
    __syncthreads();
    for (int i = threadIdx.x; i < nh; i += blockDim.x) {   // insert (linear probing, CAS in LDS)
      const int r = p.hot[i];
      unsigned h = hot_hash(r) >> (32 - __builtin_ctz(HT));
      for (int k = 0; k < HT; ++k, h = (h + 1) & (HT - 1))
        if (atomicCAS(&hkey[h], -1, r) == -1) {
          hval[h] = i;
          break;
        }
    }
    for (int i = threadIdx.x; i < nh * (D / 4); i += blockDim.x) {
      const int j = i / (D / 4), c = i - j * (D / 4);
      hrow[i] = *reinterpret_cast<const f32x4*>(p.table + (size_t)p.hot[j] * D + 4 * c);
    }
    __syncthreads();
  }
  constexpr int G = D / 4;                  // lanes per sample
  constexpr int SPW = 64 / G;               // samples per wave
  const int lane = threadIdx.x & 63;
  const int q = lane % G;
  const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int L = p.L;

  for (int b0 = gw * SPW; b0 < p.B; b0 += nwaves * SPW) {
    const int b = b0 + lane / G;
    if (b >= p.B) continue;
    // ---------------- ids + validation
    long long item = p.item_id[b];
    long long lk = p.likes[b], vw = p.views[b];
    bool bad = false;
    if (lk < 0 || lk >= p.n_cate) { bad = true; lk = 0; }
    if (vw < 0 || vw >= p.n_cate) { bad = true; vw = 0; }
    // history rows are issued in chunks of HCH slots (all loads of a chunk in flight before
    // any is consumed) and summed in slot order like the reference's sum over dim 1
    // independent loads first (they overlap the row gather below)
    const bool ld3 = !(p.abl & 4);
    const f32x4 c1 = ld3 ? *reinterpret_cast<const f32x4*>(p.cate + lk * D + 4 * q) : (f32x4){0.f, 0.f, 0.f, 0.f};
    const f32x4 c2 = ld3 ? *reinterpret_cast<const f32x4*>(p.cate + vw * D + 4 * q) : (f32x4){0.f, 0.f, 0.f, 0.f};
    const f32x4 h = ld3 ? *reinterpret_cast<const f32x4*>(p.hmm + (size_t)b * D + 4 * q) : (f32x4){1.f, 2.f, 3.f, 4.f};
    f32x4 rit = {0.f, 0.f, 0.f, 0.f};
    f32x4 hs = {0.f, 0.f, 0.f, 0.f};
    int nnz = 0;
    const int* pb = MODE >= 1 ? p.pos + (size_t)b * (L + 1) : nullptr;
    if (MODE == 0) {
      if (item < 0 || item >= p.V) { bad = true; item = -1; }
      if (item >= 0 && ld3) rit = *reinterpret_cast<const f32x4*>(p.table + item * D + 4 * q);
    } else {
      const int pi = pb[0];
      if (pi >= 0) rit = load_row<D, MODE>(p, pi, q);
    }
    // all history ids in ONE round (lane q of the group holds slots q, q+G, ...), broadcast by
    // shuffles, then every row load is issued before any is consumed (two dependent round trips
    // per sample instead of one per chunk); summed in slot order like the reference
    constexpr int IPL = (FBN_MAX_L + G - 1) / G;      // ids per lane
    int sid[IPL];
#pragma unroll
    for (int j = 0; j < IPL; ++j) {
      const int t = q + j * G;
      int r = -1;
      if (t < L) {
        if (MODE == 0) {
          long long s = p.item_seq[(size_t)b * L + t];
          if (s < 0 || s >= p.V) { bad = true; s = 0; }
          r = s != 0 ? (int)s : -1;
        } else {
          r = pb[t + 1];
        }
      }
      sid[j] = r;
    }
    const int gbase = lane - q;
    if constexpr (CMP) {
      constexpr int SPB = 4 * SPW;                     // samples per 256-thread block
      __shared__ int lid[SPB][FBN_MAX_L];
      int* mine = lid[(threadIdx.x >> 6) * SPW + lane / G];
      const unsigned long long gmask = (G == 64 ? ~0ull : ((1ull << G) - 1)) << gbase;
      int nl = 0;
#pragma unroll
      for (int j = 0; j < IPL; ++j) {
        const unsigned long long mk = __ballot(sid[j] >= 0) & gmask;
        const int below = __popcll(mk & ((1ull << lane) - 1));
        if (sid[j] >= 0) mine[nl + below] = sid[j];
        nl += __popcll(mk);
      }
      __builtin_amdgcn_wave_barrier();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);         // the list is read back by the group's lanes
      int nch = (nl + HCH - 1) / HCH;                  // wave-uniform bound: the wave's largest
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) nch = max(nch, __shfl_xor(nch, o, 64));
      for (int c = 0; c < nch; ++c) {
        f32x4 hist[HCH];
        bool live[HCH];
#pragma unroll
        for (int u = 0; u < HCH; ++u) {
          const int k = c * HCH + u;
          live[u] = k < nl;
          const int r = mine[live[u] ? k : 0];
          if constexpr (BUF) {
            const unsigned off = live[u] ? ((unsigned)r * D + 4 * q) * 4u : 0xFFFFFFF0u;
            hist[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
          } else {
            hist[u] = load_row<D, MODE>(p, live[u] ? r : 0, q);
          }
        }
#pragma unroll
        for (int u = 0; u < HCH; ++u) hs += live[u] ? hist[u] : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      nnz = nl;
      __builtin_amdgcn_wave_barrier();                 // the next sample's list overwrites this one
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
    for (int t0 = 0; t0 < ((CMP || (p.abl & 1)) ? 0 : L); t0 += HCH) {
      // branch-free: every slot of the chunk issues its load (a padding or past-L slot reads row
      // 0, an L2-resident line, and contributes +0 by a select) -- a load under a branch makes
      // hipcc drain vmcnt(0) before the next, which serialised the chunk's round trips
      f32x4 hist[HCH];
      bool live[HCH];
#pragma unroll
      for (int u = 0; u < HCH; ++u) {
        const int t = t0 + u;
        int r = -1;
#pragma unroll
        for (int j = 0; j < IPL; ++j)
          if ((t / G) == j) r = __shfl(sid[j], gbase + (t % G), 64);
        live[u] = t < L && r >= 0;
        if constexpr (HOT) {
          // two probes of the id table (slot -> list index): a staged row is read from LDS and
          // its global load is sent out of range (no fetch)
          int hi = -1;
          if (live[u] && nh > 0) {
            const unsigned h = hot_hash(r) >> (32 - __builtin_ctz(HT));
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              const unsigned hk = (h + k) & (HT - 1);
              if (hi < 0 && hkey[hk] == r) hi = hval[hk];
            }
          }
          const unsigned off = (live[u] && hi < 0) ? ((unsigned)r * D + 4 * q) * 4u : 0xFFFFFFF0u;
          hist[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
          if (hi >= 0) hist[u] = hrow[hi * (D / 4) + q];
        } else if constexpr (BUF) {
          const unsigned off = live[u] ? ((unsigned)r * D + 4 * q) * 4u : 0xFFFFFFF0u;
          hist[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        } else {
          hist[u] = load_row<D, MODE>(p, live[u] ? r : 0, q);
        }
      }
#pragma unroll
      for (int u = 0; u < HCH; ++u) {
        hs += live[u] ? hist[u] : (f32x4){0.f, 0.f, 0.f, 0.f};
        nnz += live[u] ? 1 : 0;
      }
    }
    if (bad) atomicOr(p.err, 1);        // any lane: history ids are validated by the lane holding them

    // ---------------- history masked mean
    const float cnt = fmaxf((float)nnz, 1.f);
    f32x4 x5 = hs / cnt;

    // ---------------- mm field: LayerNorm(eps) + ReLU
    const f32x4 x4 = ln_relu<G>(h, p.ln_g, p.ln_b, p.ln_eps, q);

    // ---------------- SENET
    const f32x4 xs[5] = {c1, c2, rit, x4, x5};
    float z[6];
    z[0] = 0.f;
#pragma unroll
    for (int f = 0; f < 5; ++f) z[f + 1] = group_sum<G>(xs[f][0] + xs[f][1] + xs[f][2] + xs[f][3]) / (float)D;
    float qv[FBN_MAXR], a[6];
    senet_excite<D>(z, p.w1, p.b1, p.w2, p.b2, p.R, qv, a);

    // ---------------- stores
    float* Xb = p.X + (size_t)b * 2 * D + 4 * q;
    if (!(p.abl & 2)) {
      *reinterpret_cast<f32x4*>(Xb) = rit;
      *reinterpret_cast<f32x4*>(Xb + D) = x5;
    }
    float* Vb = p.Vc ? p.Vc + (size_t)b * 5 * D + 4 * q : nullptr;
    float* cb = (p.c && !p.c16) ? (float*)p.c + (size_t)b * p.ldc + 4 * q : nullptr;
    short* cb16 = (p.c && p.c16) ? (short*)p.c + (size_t)b * p.ldc + 4 * q : nullptr;
#pragma unroll
    for (int f = 0; f < 5 && !(p.abl & 2); ++f) {
      const f32x4 v = xs[f] * a[f + 1];
      if (p.Vc) *reinterpret_cast<f32x4*>(Vb + f * D) = v;   // bf16 mode: only the bf16 copies
      const bf16x4 v16 = (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
      if (cb16) *reinterpret_cast<bf16x4*>(cb16 + f * D) = v16;
      else if (cb) *reinterpret_cast<f32x4*>(cb + f * D) = v;
      if (p.Vc16) *reinterpret_cast<bf16x4*>(p.Vc16 + ((size_t)b * 5 + f) * D + 4 * q) = v16;
    }
#pragma unroll
    for (int f = 0; f < 6; ++f)
      if (f % G == q) p.a_out[(size_t)b * 6 + f] = a[f];   // G may be < 6 (D = 16)
    if (q == 0) p.cnt_out[b] = cnt;

    // ---------------- sparse-grad map insert (rows that will receive a gradient)
    if (MODE == 0 && p.map) {
      for (int t = q; t <= L; t += G) {
        long long r = (t == 0) ? item : p.item_seq[(size_t)b * L + (t - 1)];
        if (r > 0 && r < p.V) map_claim(p.map, p.slot_row, (int)r, b * (L + 1) + t);
      }
    }
  }
}

// ------------------------------------------------------------------------------ backward
struct FieldBwdArgs {
  const int64_t* item_id; const int64_t* item_seq; const int64_t* likes; const int64_t* views;
  const float* hmm; const float* ln_g;
  const float* w1; const float* b1; const float* w2;
  const float* X;      // [B][2][D] fields 3, 5 (fields 1, 2, 4 are recomputed)
  const float* cate;   // [n_cate][D] (field 1, 2 recompute)
  const float* ln_b;   // [D] (field 4 recompute)
  const float* a;      // [B][6]
  const float* cnt;    // [B]
  const float* dV;     // [B][5][D] total gradient wrt V_1..V_5
  float* dhmm;         // [B][D] gradient wrt the pre-LN projection
  short* dhmm16;       // optional bf16 copy (operand of the mm_proj weight-gradient GEMM)
  long long dhmm16_lo; // > 0: dhmm16 is split images (hi, lo this many elements further; bf16_fwd)
  float* partials;     // [gridDim.x][P]; P = 6R + R + 6R + 6 + 2D + n_cate*D
  // table gradient, mode 0: dense gtab[V][D] (atomics) if gvec == null; otherwise the two
  // per-sample vectors gvec[b][0] = dX3 (item row), gvec[b][1] = dX5/count (each history row)
  float* gtab; float* gvec;
  double* gnorm;       // optional with gvec: [B][2] sums of squares of the two vectors (clip norm)
  // mode 1: rows written to sendbuf at pos[b][t] (f32); mode 2: the same in bf16 (bf16 mode's wire)
  const int* pos; void* sendbuf;
  long long V;
  int B, L, R, n_cate;
  float ln_eps;
};

// Column-transposed copy of a group's row vector for coalesced atomics: lane q of a G-lane
// group holds columns 4q..4q+3; after the transpose, t[e] is column e*G + q, so atomic
// instruction e of the group covers one contiguous G*4-byte run of the row (full-rate
// global_atomic_add_f32 shape) instead of four 16-B-strided runs.
template <int G>
__device__ __forceinline__ f32x4 transpose_cols(const f32x4& v, int lane) {
  const int base = lane - lane % G, q = lane % G;
  f32x4 t;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int src = base + e * (G / 4) + q / 4;
    const float x0 = __shfl(v[0], src, 64), x1 = __shfl(v[1], src, 64);
    const float x2 = __shfl(v[2], src, 64), x3 = __shfl(v[3], src, 64);
    const int c = q & 3;
    t[e] = c == 0 ? x0 : (c == 1 ? x1 : (c == 2 ? x2 : x3));
  }
  return t;
}
template <int G>
__device__ __forceinline__ void atomic_add_row_t(float* row, const f32x4& t, int q) {
  atomicAdd(row + q, t[0]); atomicAdd(row + G + q, t[1]); atomicAdd(row + 2 * G + q, t[2]);
  atomicAdd(row + 3 * G + q, t[3]);
}

// Backward of the fields.  No LDS atomics (they serialised on the few hot addresses every
// sample adds into -- the LN columns, 11 cate rows, the SENET weights -- and cost ~25 LDS cycles
// each): the LN and SENET parameter gradients accumulate in registers (SENET's group-uniform
// entries spread over the group's lanes: entry k in lane k mod G), the cate rows by plain
// read-modify-write into a per-wave LDS slice with the wave's sample groups taking turns; each
// wave folds its groups with shuffles into its slice, and the block sums its 4 slices into its
// partial row (same layout as before).
template <int D, int MODE, int RMAX>
__global__ void __launch_bounds__(256) fields_bwd_kernel(FieldBwdArgs p) {
  FBN_MAIN_PRIO();
  constexpr int G = D / 4;
  constexpr int SPW = 64 / G;
  constexpr int NPMAX = 13 * RMAX + 6;
  constexpr int SJ = (NPMAX + G - 1) / G;          // SENET entries per lane
  extern __shared__ __attribute__((aligned(16))) float sp[];   // 4 wave slices of P floats + SENET staging
  const int R = p.R;
  const int NP = 13 * R + 6;
  const int P = NP + 3 * D + p.n_cate * D;      // ... | cate rows | mm_proj bias (column sums of dhmm)
  const int wave = threadIdx.x >> 6;
  float* ws = sp + wave * P;                       // this wave's slice
  // per group: {ds[6], z[6], dq[R], rj[R]} staged for the lanes that own SENET entries
  float* sv = sp + 4 * P + (wave * SPW + (threadIdx.x & 63) / G) * (12 + 2 * RMAX);
  for (int i = threadIdx.x; i < 4 * P; i += blockDim.x) sp[i] = 0.f;
  __syncthreads();
  float* w_lg = ws + NP;
  float* w_ct = w_lg + 2 * D;
  float* w_hb = w_ct + p.n_cate * D;

  const int lane = threadIdx.x & 63;
  const int q = lane % G, grp = lane / G;
  const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int L = p.L;
  f32x4 acc_lg = {0.f, 0.f, 0.f, 0.f}, acc_lb = {0.f, 0.f, 0.f, 0.f}, acc_hb = {0.f, 0.f, 0.f, 0.f};
  float acc_se[SJ];
#pragma unroll
  for (int j = 0; j < SJ; ++j) acc_se[j] = 0.f;

  for (int b0 = gw * SPW; b0 < p.B; b0 += nwaves * SPW) {
    const int b = b0 + grp;
    const bool live = b < p.B;
    f32x4 dx0 = {0.f, 0.f, 0.f, 0.f}, dx1 = {0.f, 0.f, 0.f, 0.f};
    long long lk = -1, vw = -1;
    if (live) {
      const float* Xb = p.X + (size_t)b * 2 * D + 4 * q;
      const float* dVb = p.dV + (size_t)b * 5 * D + 4 * q;
      f32x4 x[5], dv[5];
      lk = p.likes[b];
      vw = p.views[b];
      // fields 1, 2 as the forward read them (an out-of-range id read row 0 and raised the flag)
      const long long lkc = (lk >= 0 && lk < p.n_cate) ? lk : 0, vwc = (vw >= 0 && vw < p.n_cate) ? vw : 0;
      x[0] = *reinterpret_cast<const f32x4*>(p.cate + lkc * D + 4 * q);
      x[1] = *reinterpret_cast<const f32x4*>(p.cate + vwc * D + 4 * q);
      x[2] = *reinterpret_cast<const f32x4*>(Xb);
      x[4] = *reinterpret_cast<const f32x4*>(Xb + D);
#pragma unroll
      for (int f = 0; f < 5; ++f) dv[f] = *reinterpret_cast<const f32x4*>(dVb + f * D);
      const f32x4 h = *reinterpret_cast<const f32x4*>(p.hmm + (size_t)b * D + 4 * q);
      x[3] = ln_relu<G>(h, p.ln_g, p.ln_b, p.ln_eps, q);
      float a[6];
#pragma unroll
      for (int f = 0; f < 6; ++f) a[f] = p.a[(size_t)b * 6 + f];
      // recompute squeeze + hidden exactly as the forward did
      float z[6];
      z[0] = 0.f;
#pragma unroll
      for (int f = 0; f < 5; ++f) z[f + 1] = group_sum<G>(x[f][0] + x[f][1] + x[f][2] + x[f][3]) / (float)D;
      float qv[RMAX], rj[RMAX], dq[RMAX];
#pragma unroll
      for (int j = 0; j < RMAX; ++j) {
        float s = 0.f;
        if (j < R) {
          s = p.b1[j];
#pragma unroll
          for (int f = 0; f < 6; ++f) s += p.w1[j * 6 + f] * z[f];
        }
        qv[j] = s;
        rj[j] = fmaxf(s, 0.f);
      }
      // excitation backward
      float ds[6];
      ds[0] = 0.f;   // da_0 = sum(dV_0 * X_0) = 0 since X_0 == 0
#pragma unroll
      for (int f = 0; f < 5; ++f) {
        const float da = group_sum<G>(dv[f][0] * x[f][0] + dv[f][1] * x[f][1] + dv[f][2] * x[f][2] + dv[f][3] * x[f][3]);
        ds[f + 1] = da * (1.f - a[f + 1]) * a[f + 1];
      }
      float dz[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < RMAX; ++j) {
        float dr = 0.f;
        if (j < R) {
#pragma unroll
          for (int f = 0; f < 6; ++f) dr += p.w2[f * R + j] * ds[f];
        }
        dq[j] = (j < R && qv[j] > 0.f) ? dr : 0.f;
        if (j < R) {
#pragma unroll
          for (int f = 0; f < 6; ++f) dz[f] += p.w1[j * 6 + f] * dq[j];
        }
      }
      // SENET parameter-gradient entries (group-uniform): lane q owns entries q, q+G, ... of the
      // flattened [w1 R*6 | b1 R | w2 6*R | b2 6]; the values come through LDS (runtime indices
      // into registers would go to scratch)
      if (q == 0) {
#pragma unroll
        for (int f = 0; f < 6; ++f) { sv[f] = ds[f]; sv[6 + f] = z[f]; }
#pragma unroll
        for (int jj = 0; jj < RMAX; ++jj) { sv[12 + jj] = dq[jj]; sv[12 + RMAX + jj] = rj[jj]; }
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < SJ; ++j) {
        const int k = q + j * G;
        float v = 0.f;
        if (k < 6 * R) v = sv[12 + k / 6] * sv[6 + k % 6];                                  // dq_j * z_f
        else if (k < 7 * R) v = sv[12 + (k - 6 * R)];                                        // dq_j
        else if (k < 13 * R) v = sv[(k - 7 * R) / R] * sv[12 + RMAX + (k - 7 * R) % R];      // ds_f * r_j
        else if (k < NP) v = sv[k - 13 * R];                                                 // ds_f
        acc_se[j] += v;
      }
      __builtin_amdgcn_wave_barrier();
      f32x4 dx[5];
#pragma unroll
      for (int f = 0; f < 5; ++f) dx[f] = dv[f] * a[f + 1] + dz[f + 1] / (float)D;
      dx0 = dx[0];
      dx1 = dx[1];

      // field 4: ReLU + LayerNorm backward -> d(h_mm)
      {
        const float mean = group_sum<G>(h[0] + h[1] + h[2] + h[3]) / (float)D;
        const f32x4 dh = h - mean;
        const float s2 = group_sum<G>(dh[0] * dh[0] + dh[1] * dh[1] + dh[2] * dh[2] + dh[3] * dh[3]);
        const float rstd = 1.f / sqrtf(s2 / (float)D + p.ln_eps);
        const f32x4 gam = *reinterpret_cast<const f32x4*>(p.ln_g + 4 * q);
        f32x4 gl, xh, gx;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gl[e] = x[3][e] > 0.f ? dx[3][e] : 0.f;
          xh[e] = dh[e] * rstd;
          gx[e] = gl[e] * gam[e];
          acc_lg[e] += gl[e] * xh[e];
          acc_lb[e] += gl[e];
        }
        const float m1 = group_sum<G>(gx[0] + gx[1] + gx[2] + gx[3]) / (float)D;
        const float m2 = group_sum<G>(gx[0] * xh[0] + gx[1] * xh[1] + gx[2] * xh[2] + gx[3] * xh[3]) / (float)D;
        f32x4 out;
#pragma unroll
        for (int e = 0; e < 4; ++e) out[e] = rstd * (gx[e] - m1 - xh[e] * m2);
        *reinterpret_cast<f32x4*>(p.dhmm + (size_t)b * D + 4 * q) = out;
        acc_hb += out;                              // mm_proj.0.bias gradient (sum over the batch)
        if (p.dhmm16) {
          const bf16x4 hi = (bf16x4){f2bf(out[0]), f2bf(out[1]), f2bf(out[2]), f2bf(out[3])};
          *reinterpret_cast<bf16x4*>(p.dhmm16 + (size_t)b * D + 4 * q) = hi;
          if (p.dhmm16_lo)
            *reinterpret_cast<bf16x4*>(p.dhmm16 + p.dhmm16_lo + (size_t)b * D + 4 * q) =
                (bf16x4){f2bf(out[0] - bf2f(hi[0])), f2bf(out[1] - bf2f(hi[1])), f2bf(out[2] - bf2f(hi[2])),
                         f2bf(out[3] - bf2f(hi[3]))};
        }
      }
      // item table: dX3 -> row item_id, dX5 / count -> each non-padding history row
      const f32x4 gh = dx[4] / p.cnt[b];
      if (MODE == 0 && p.gvec) {
        // sparse mode: plain stores; rows are resolved later through map / slot_row
        *reinterpret_cast<f32x4*>(p.gvec + (size_t)b * 2 * D + 4 * q) = dx[2];
        *reinterpret_cast<f32x4*>(p.gvec + ((size_t)b * 2 + 1) * D + 4 * q) = gh;
        if (p.gnorm) {
          double si = 0.0, sh = 0.0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            si += (double)(dx[2][e] * dx[2][e]);
            sh += (double)(gh[e] * gh[e]);
          }
#pragma unroll
          for (int o = G / 2; o > 0; o >>= 1) {
            si += __shfl_xor(si, o, 64);
            sh += __shfl_xor(sh, o, 64);
          }
          if (q == 0) {
            p.gnorm[(size_t)b * 2] = si;
            p.gnorm[(size_t)b * 2 + 1] = sh;
          }
        }
      } else if (MODE == 0) {
        const f32x4 ti = transpose_cols<G>(dx[2], lane);
        const f32x4 th = transpose_cols<G>(gh, lane);
        const long long item = p.item_id[b];
        if (item > 0 && item < p.V) atomic_add_row_t<G>(p.gtab + item * D, ti, q);
        for (int t = 0; t < L; ++t) {
          const long long s = p.item_seq[(size_t)b * L + t];
          if (s > 0 && s < p.V) atomic_add_row_t<G>(p.gtab + s * D, th, q);
        }
      } else {
        const int* pb = p.pos + (size_t)b * (L + 1);
        auto put = [&](int row, const f32x4& x) {
          if constexpr (MODE == 2) {
            *reinterpret_cast<bf16x4*>(reinterpret_cast<short*>(p.sendbuf) + (size_t)row * D + 4 * q) =
                (bf16x4){f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
          } else {
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.sendbuf) + (size_t)row * D + 4 * q) = x;
          }
        };
        if (pb[0] >= 0) put(pb[0], dx[2]);
        for (int t = 0; t < L; ++t)
          if (pb[t + 1] >= 0) put(pb[t + 1], gh);
      }
    }
    // cate table (likes, views share one table): the wave's groups take turns on its slice
#pragma unroll
    for (int gi = 0; gi < SPW; ++gi) {
      if (grp == gi && live) {
        if (lk >= 0 && lk < p.n_cate) {
          f32x4* c = reinterpret_cast<f32x4*>(w_ct + lk * D + 4 * q);
          *c = *c + dx0;
        }
        if (vw >= 0 && vw < p.n_cate) {
          f32x4* c = reinterpret_cast<f32x4*>(w_ct + vw * D + 4 * q);
          *c = *c + dx1;
        }
      }
    }
  }
  // fold the wave's groups (lanes q, q+G, ... hold the same entries / columns) into group 0
#pragma unroll
  for (int o = G; o < 64; o <<= 1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc_lg[e] += __shfl_xor(acc_lg[e], o, 64);
      acc_lb[e] += __shfl_xor(acc_lb[e], o, 64);
      acc_hb[e] += __shfl_xor(acc_hb[e], o, 64);
    }
#pragma unroll
    for (int j = 0; j < SJ; ++j) acc_se[j] += __shfl_xor(acc_se[j], o, 64);
  }
  if (grp == 0) {
    *reinterpret_cast<f32x4*>(w_lg + 4 * q) = acc_lg;
    *reinterpret_cast<f32x4*>(w_lg + D + 4 * q) = acc_lb;
    *reinterpret_cast<f32x4*>(w_hb + 4 * q) = acc_hb;
#pragma unroll
    for (int j = 0; j < SJ; ++j) {
      const int k = q + j * G;
      if (k < NP) ws[k] = acc_se[j];
    }
  }
  __syncthreads();
  float* out = p.partials + (size_t)blockIdx.x * P;
  for (int i = threadIdx.x; i < P; i += blockDim.x) out[i] = (sp[i] + sp[P + i]) + (sp[2 * P + i] + sp[3 * P + i]);
}

// destinations of the 8 parameter-gradient segments (w1, b1, w2, b2, ln_g, ln_b, cate, mm_proj bias)
struct GradOuts {
  float* p[8];
  int off[9];
};
// One launch: 64 columns per 1024-thread block, the 16 waves stride over the partial rows, a
// fixed-order fold across the waves (deterministic), then each column to its destination.
__global__ void __launch_bounds__(1024) reduce_partials_one(const float* __restrict__ part, int nblk, int P, GradOuts o) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (i < P)
    for (int r = w; r < nblk; r += 16) s += part[(size_t)r * P + i];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && i < P) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][lane];
    int seg = 0;
#pragma unroll
    for (int j = 1; j < 8; ++j) seg += (i >= o.off[j]) ? 1 : 0;
    if (o.p[seg]) o.p[seg][i - o.off[seg]] = t;
  }
}

// Same reduction on 16 columns per block (P / 16 workgroups): 64 partial-row streams per column,
// 16 lanes reading one 64-B segment, then a fixed-order fold over the 64 streams (deterministic).
__global__ void __launch_bounds__(1024) reduce_partials_one16(const float* __restrict__ part, int nblk, int P, GradOuts o) {
  __shared__ float red[64][16];
  const int col = threadIdx.x & 15, str = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + col;
  float s = 0.f;
  if (i < P)
    for (int r = str; r < nblk; r += 64) s += part[(size_t)r * P + i];
  red[str][col] = s;
  __syncthreads();
  if (threadIdx.x < 16 && i < P) {
    float t = 0.f;
    for (int k = 0; k < 64; ++k) t += red[k][col];
    int seg = 0;
#pragma unroll
    for (int j = 1; j < 8; ++j) seg += (i >= o.off[j]) ? 1 : 0;
    if (o.p[seg]) o.p[seg][i - o.off[seg]] = t;
  }
}


// ------------------------------------------------------------------------------ C ABI
#ifndef FBN_FB_MAXBLK
#define FBN_FB_MAXBLK 512    // backward: partial rows to reduce vs samples in flight (tools/time_fields.py)
#endif
static int fields_grid(int B, int D, int cap = 1024) {
  const int spw = 64 / (D / 4);
  const int waves = (B + spw - 1) / spw;
  int blocks = (waves + 3) / 4;
  return blocks < 1 ? 1 : (blocks > cap ? cap : blocks);
}

// history rows per chunk: every row of a chunk is in flight at once (branch-free issue); more rows
// per chunk = fewer dependent round trips but more registers (fewer waves resident)
template <int MODE, int HCH, bool BUF, bool HOT = false, bool CMP = false>
static int launch_fields_fwd_hb(const FieldArgs& a, int D, hipStream_t st) {
  // hot staging: fewer, longer-lived workgroups (each stages the hot rows once)
  const int grid = fields_grid(a.B, D, HOT ? 256 : 1024);
  switch (D) {
    case 16: fbn_launch((fields_fwd_kernel<16, MODE, HCH, BUF, HOT, CMP>), dim3(grid), dim3(256), 0, st, a); break;
    case 32: fbn_launch((fields_fwd_kernel<32, MODE, HCH, BUF, HOT, CMP>), dim3(grid), dim3(256), 0, st, a); break;
    case 64: fbn_launch((fields_fwd_kernel<64, MODE, HCH, BUF, HOT, CMP>), dim3(grid), dim3(256), 0, st, a); break;
    case 128: fbn_launch((fields_fwd_kernel<128, MODE, HCH, BUF, HOT, CMP>), dim3(grid), dim3(256), 0, st, a); break;
    case 256: fbn_launch((fields_fwd_kernel<256, MODE, HCH, BUF, HOT, CMP>), dim3(grid), dim3(256), 0, st, a); break;
    default: fbn_set_error("fields: embedding_dim must be one of 16,32,64,128,256"); return FBN_ERR_UNSUPPORTED;
  }
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

template <int MODE, int HCH, bool CMP>
static int launch_fields_fwd_h(const FieldArgs& a, int D, hipStream_t st) {
  if constexpr (MODE == 0) {
    if (a.hot) return launch_fields_fwd_hb<0, HCH, true, true>(a, D, st);
    // buffer-resource history loads while the table's byte extent fits the descriptor's 32 bits
    static const bool nobuf = getenv("FBN_FIELDS_NOBUF") != nullptr;   // A/B knob
    if (!nobuf && (unsigned long long)a.V * D * 4 < 0xFFFFFF00ull)
      return launch_fields_fwd_hb<0, HCH, true, false, CMP>(a, D, st);
  }
  return launch_fields_fwd_hb<MODE, HCH, false, false, CMP>(a, D, st);
}

template <int MODE>
static int launch_fields_fwd(const FieldArgs& a, int D, hipStream_t st) {
  const char* he = getenv("FBN_FIELDS_HCH");   // A/B knob, read per call
  const int hch = he ? atoi(he) : FBN_HCH;
  // FBN_FIELDS_CMP=1: the live history slots compacted first (A/B knob, read per call)
  const char* ce = getenv("FBN_FIELDS_CMP");
  if (ce && atoi(ce) == 1) {
    if (hch == 10) return launch_fields_fwd_h<MODE, 10, true>(a, D, st);
    if (hch == 8) return launch_fields_fwd_h<MODE, 8, true>(a, D, st);
    return launch_fields_fwd_h<MODE, 5, true>(a, D, st);
  }
  if (hch == 20) return launch_fields_fwd_h<MODE, 20, false>(a, D, st);
  if (hch == 5) return launch_fields_fwd_h<MODE, 5, false>(a, D, st);
  return launch_fields_fwd_h<MODE, 10, false>(a, D, st);
}

static int fields_fwd_impl(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes,
                           const int64_t* views, const float* hmm, const float* ln_g, const float* ln_b,
                           float ln_eps, const float* cate, int n_cate, const float* table, long long V,
                           const int* pos, const float* w1, const float* b1, const float* w2,
                           const float* b2, int R, float* X, float* Vc, short* Vc16, void* c, int ldc, int c_bf16,
                           float* a_out, float* cnt_out, int* err, int* map, int* slot_row, int B, int L,
                           int D, int rows_bf16, const int* hot, const int* hot_n, int H, void* stream);

extern "C" int fbn_fields_fwd(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes,
                              const int64_t* views, const float* hmm, const float* ln_g, const float* ln_b,
                              float ln_eps, const float* cate, int n_cate, const float* table, long long V,
                              const int* pos, const float* w1, const float* b1, const float* w2,
                              const float* b2, int R, float* X, float* Vc, short* Vc16, void* c, int ldc, int c_bf16,
                              float* a_out,
                              float* cnt_out, int* err, int* map, int* slot_row, int B, int L,
                              int D, int rows_bf16, void* stream) {
  return fields_fwd_impl(item_id, item_seq, likes, views, hmm, ln_g, ln_b, ln_eps, cate, n_cate, table, V, pos, w1,
                         b1, w2, b2, R, X, Vc, Vc16, c, ldc, c_bf16, a_out, cnt_out, err, map, slot_row, B, L, D,
                         rows_bf16, nullptr, nullptr, 0, stream);
}

// the gather with the batch's hot rows (fbn_hot_rows) staged in LDS (single GPU, f32 table < 4 GB)
extern "C" int fbn_fields_fwd_hot(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes,
                                  const int64_t* views, const float* hmm, const float* ln_g, const float* ln_b,
                                  float ln_eps, const float* cate, int n_cate, const float* table, long long V,
                                  const float* w1, const float* b1, const float* w2, const float* b2, int R, float* X,
                                  float* Vc, short* Vc16, void* c, int ldc, int c_bf16, float* a_out, float* cnt_out,
                                  int* err, int* map, int* slot_row, int B, int L, int D, const int* hot,
                                  const int* hot_n, int H, void* stream) {
  if (!hot || !hot_n || (unsigned long long)V * D * 4 >= 0xFFFFFF00ull) {
    fbn_set_error("fbn_fields_fwd_hot: needs the hot list and a table under 4 GB");
    return FBN_ERR_ARG;
  }
  return fields_fwd_impl(item_id, item_seq, likes, views, hmm, ln_g, ln_b, ln_eps, cate, n_cate, table, V, nullptr,
                         w1, b1, w2, b2, R, X, Vc, Vc16, c, ldc, c_bf16, a_out, cnt_out, err, map, slot_row, B, L, D, 0,
                         hot, hot_n, H, stream);
}

// Hot rows of a batch (clear = 0): every entry counts its row (cnt [V] int32, zero on entry); the
// entry that brings a row's count to tau appends it to hot[] (hot_n: length, may exceed H).
// clear = 1: the same entries zero their counts and hot_n (after the gather has read the list).
__global__ void hot_rows_kernel(const int64_t* __restrict__ item, const int64_t* __restrict__ seq, int B, int L,
                                long long V, int* __restrict__ cnt, int* __restrict__ hot, int* __restrict__ hot_n,
                                int H, int tau, int clear) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (clear && i == 0) *hot_n = 0;
  if (i >= (long long)B * (L + 1)) return;
  const long long b = i / (L + 1), t = i - b * (L + 1);
  const long long id = t == 0 ? item[b] : seq[b * L + (t - 1)];
  if (id <= 0 || id >= V) return;
  if (clear) {
    cnt[id] = 0;
    return;
  }
  if (atomicAdd(cnt + id, 1) == tau - 1) {
    const int s = atomicAdd(hot_n, 1);
    if (s < H) hot[s] = (int)id;
  }
}

extern "C" int fbn_hot_rows(const int64_t* item, const int64_t* seq, int B, int L, long long V, int* cnt, int* hot,
                            int* hot_n, int H, int tau, int clear, void* stream) {
  const long long n = (long long)B * (L + 1);
  if (n <= 0) return FBN_OK;
  fbn_launch(hot_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, item,
                     L > 0 ? seq : nullptr, B, L, V, cnt, hot, hot_n, H, tau < 1 ? 1 : tau, clear);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

static int fields_fwd_impl(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes,
                           const int64_t* views, const float* hmm, const float* ln_g, const float* ln_b,
                           float ln_eps, const float* cate, int n_cate, const float* table, long long V,
                           const int* pos, const float* w1, const float* b1, const float* w2,
                           const float* b2, int R, float* X, float* Vc, short* Vc16, void* c, int ldc, int c_bf16,
                           float* a_out, float* cnt_out, int* err, int* map, int* slot_row, int B, int L,
                           int D, int rows_bf16, const int* hot, const int* hot_n, int H, void* stream) {
  if (B <= 0) return FBN_OK;
  if (L < 0 || L > 32 || R < 1 || R > FBN_MAXR || (ldc & 3)) {
    fbn_set_error("fbn_fields_fwd: need 0 <= L <= 32, 1 <= R <= 8, ldc % 4 == 0");
    return FBN_ERR_ARG;
  }
  FieldArgs a;
  a.item_id = item_id; a.item_seq = L > 0 ? item_seq : nullptr; a.likes = likes; a.views = views;
  a.hmm = hmm; a.ln_g = ln_g; a.ln_b = ln_b; a.cate = cate; a.table = table; a.pos = pos;
  a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2;
  a.X = X; a.Vc = Vc; a.Vc16 = Vc16; a.c = c; a.a_out = a_out; a.cnt_out = cnt_out; a.err = err;
  a.map = map; a.slot_row = slot_row;
  a.V = V; a.B = B; a.L = L; a.ldc = ldc; a.R = R; a.n_cate = n_cate; a.ln_eps = ln_eps; a.c16 = c_bf16;
  a.hot = hot; a.hot_n = hot_n; a.H = H;
  const char* ae = getenv("FBN_FIELDS_ABL");   // measurement only (NOT a valid forward when set)
  a.abl = ae ? atoi(ae) : 0;
  if (pos && rows_bf16) return launch_fields_fwd<2>(a, D, (hipStream_t)stream);
  if (pos) return launch_fields_fwd<1>(a, D, (hipStream_t)stream);
  return launch_fields_fwd<0>(a, D, (hipStream_t)stream);
}

extern "C" int fbn_fields_bwd_partials_size(int D, int R, int n_cate) { return 13 * R + 6 + 3 * D + n_cate * D; }
// rows of the `partials` scratch the caller allocates: one per block
extern "C" int fbn_fields_bwd_grid(int B, int D) { return fields_grid(B, D, FBN_FB_MAXBLK); }

template <int MODE, int RMAX>
static int launch_fields_bwd_r(const FieldBwdArgs& a, int D, hipStream_t st) {
  const int grid = fields_grid(a.B, D, FBN_FB_MAXBLK);
  const size_t lds = (4 * (size_t)(13 * a.R + 6 + 3 * D + a.n_cate * D) + 4 * (64 / (D / 4)) * (12 + 2 * RMAX)) *
                     sizeof(float);   // 4 wave slices + SENET staging
  switch (D) {
    case 16: fbn_launch((fields_bwd_kernel<16, MODE, RMAX>), dim3(grid), dim3(256), lds, st, a); break;
    case 32: fbn_launch((fields_bwd_kernel<32, MODE, RMAX>), dim3(grid), dim3(256), lds, st, a); break;
    case 64: fbn_launch((fields_bwd_kernel<64, MODE, RMAX>), dim3(grid), dim3(256), lds, st, a); break;
    case 128: fbn_launch((fields_bwd_kernel<128, MODE, RMAX>), dim3(grid), dim3(256), lds, st, a); break;
    case 256: fbn_launch((fields_bwd_kernel<256, MODE, RMAX>), dim3(grid), dim3(256), lds, st, a); break;
    default: fbn_set_error("fields: embedding_dim must be one of 16,32,64,128,256"); return FBN_ERR_UNSUPPORTED;
  }
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// the reference's SENET width is 3 (reduction ratio 3 over 6 fields): register arrays sized 3
template <int MODE>
static int launch_fields_bwd(const FieldBwdArgs& a, int D, hipStream_t st) {
  return a.R <= 3 ? launch_fields_bwd_r<MODE, 3>(a, D, st) : launch_fields_bwd_r<MODE, FBN_MAXR>(a, D, st);
}

// partials: [fbn_fields_bwd_grid(B,D)][P] scratch (P = fbn_fields_bwd_partials_size(D,R,n_cate));
// param_grads: host array of 8 device pointers receiving the gradients of w1, b1, w2, b2, ln_g,
// ln_b, cate, mm_proj bias (segments of 6R, R, 6R, 6, D, D, n_cate*D, D columns of a partial row),
// or NULL: the partial rows are left for the caller to sum (the trainer's one fbn_sum_jobs2 launch).
static int fields_bwd_impl(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes,
                           const int64_t* views, const float* hmm, const float* ln_g, const float* ln_b,
                           float ln_eps, const float* w1, const float* b1, const float* w2, int R, int n_cate,
                           const float* cate, const float* X, const float* a, const float* cnt, const float* dV,
                           float* dhmm, short* dhmm16, float* partials, float* const* param_grads, float* gtab,
                           float* gvec, double* gnorm, long long V, const int* pos, void* sendbuf, int send_bf16,
                           int B, int L, int D, void* stream, long long dhmm16_lo);
extern "C" int fbn_fields_bwd(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes,
                              const int64_t* views, const float* hmm, const float* ln_g, const float* ln_b,
                              float ln_eps, const float* w1, const float* b1, const float* w2, int R, int n_cate,
                              const float* cate, const float* X, const float* a, const float* cnt, const float* dV, float* dhmm,
                              short* dhmm16, float* partials, float* const* param_grads, float* gtab, float* gvec,
                              double* gnorm, long long V, const int* pos, void* sendbuf, int send_bf16, int B,
                              int L, int D, void* stream) {
  return fields_bwd_impl(item_id, item_seq, likes, views, hmm, ln_g, ln_b, ln_eps, w1, b1, w2, R, n_cate, cate, X, a,
                         cnt, dV, dhmm, dhmm16, partials, param_grads, gtab, gvec, gnorm, V, pos, sendbuf, send_bf16, B,
                         L, D, stream, 0);
}
// fbn_fields_bwd with dhmm_img = split images of dhmm (hi, lo B*D elements further; bf16_fwd training)
extern "C" int fbn_fields_bwd_img(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes,
                                  const int64_t* views, const float* hmm, const float* ln_g, const float* ln_b,
                                  float ln_eps, const float* w1, const float* b1, const float* w2, int R, int n_cate,
                                  const float* cate, const float* X, const float* a, const float* cnt, const float* dV,
                                  float* dhmm, void* dhmm_img, float* partials, float* const* param_grads,
                                  float* gtab, float* gvec, double* gnorm, long long V, const int* pos, void* sendbuf,
                                  int send_bf16, int B, int L, int D, void* stream) {
  if (!dhmm_img) { fbn_set_error("fbn_fields_bwd_img: dhmm_img"); return FBN_ERR_ARG; }
  return fields_bwd_impl(item_id, item_seq, likes, views, hmm, ln_g, ln_b, ln_eps, w1, b1, w2, R, n_cate, cate, X, a,
                         cnt, dV, dhmm, (short*)dhmm_img, partials, param_grads, gtab, gvec, gnorm, V, pos, sendbuf,
                         send_bf16, B, L, D, stream, (long long)B * D);
}
static int fields_bwd_impl(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes,
                           const int64_t* views, const float* hmm, const float* ln_g, const float* ln_b,
                           float ln_eps, const float* w1, const float* b1, const float* w2, int R, int n_cate,
                           const float* cate, const float* X, const float* a, const float* cnt, const float* dV,
                           float* dhmm, short* dhmm16, float* partials, float* const* param_grads, float* gtab,
                           float* gvec, double* gnorm, long long V, const int* pos, void* sendbuf, int send_bf16,
                           int B, int L, int D, void* stream, long long dhmm16_lo) {
  if (B <= 0) return FBN_OK;
  if (L < 0 || L > 32 || R < 1 || R > FBN_MAXR) { fbn_set_error("fbn_fields_bwd: bad L/R"); return FBN_ERR_ARG; }
  FieldBwdArgs p;
  p.item_id = item_id; p.item_seq = L > 0 ? item_seq : nullptr; p.likes = likes; p.views = views;
  p.hmm = hmm; p.ln_g = ln_g; p.ln_b = ln_b; p.w1 = w1; p.b1 = b1; p.w2 = w2; p.cate = cate;
  p.X = X; p.a = a; p.cnt = cnt; p.dV = dV; p.dhmm = dhmm; p.dhmm16 = dhmm16; p.partials = partials;
  p.dhmm16_lo = dhmm16_lo;
  p.gtab = gtab; p.gvec = gvec; p.gnorm = gvec ? gnorm : nullptr; p.pos = pos; p.sendbuf = sendbuf;
  p.V = V; p.B = B; p.L = L; p.R = R; p.n_cate = n_cate; p.ln_eps = ln_eps;
  hipStream_t st = (hipStream_t)stream;
  int rc = !pos ? launch_fields_bwd<0>(p, D, st) : send_bf16 ? launch_fields_bwd<2>(p, D, st)
                                                               : launch_fields_bwd<1>(p, D, st);
  if (rc) return rc;
  if (!param_grads) return FBN_OK;   // deferred: the caller sums the partial rows (fbn_sum_jobs2, ld = P)
  const int P = 13 * R + 6 + 3 * D + n_cate * D;
  const int nblk = fields_grid(B, D, FBN_FB_MAXBLK);

  GradOuts o;
  const int sizes[8] = {6 * R, R, 6 * R, 6, D, D, n_cate * D, D};
  o.off[0] = 0;
  for (int j = 0; j < 8; ++j) {
    if (j < 7 && !param_grads[j]) {
      fbn_set_error("fbn_fields_bwd: null parameter-gradient destination");
      return FBN_ERR_ARG;
    }
    o.p[j] = param_grads[j];   // [7] (mm_proj bias) may be null: not written
    o.off[j + 1] = o.off[j] + sizes[j];
  }
  static const bool narrow = getenv("FBN_PARTIALS64") != nullptr;   // A/B knob: 64 columns per workgroup
  if (narrow)
    fbn_launch(reduce_partials_one, dim3(fbn_cdiv(P, 64)), dim3(1024), 0, st, (const float*)partials, nblk, P, o);
  else
    fbn_launch(reduce_partials_one16, dim3(fbn_cdiv(P, 16)), dim3(1024), 0, st, (const float*)partials, nblk, P,
                       o);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}
