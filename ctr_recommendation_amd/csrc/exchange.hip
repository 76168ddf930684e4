// Row-sharded embedding exchange (multi-GPU, one process per GPU, RCCL all-to-all between).
//
// The item table E (V x D) is split into N contiguous row blocks of Vl = ceil(V/N) rows:
// owner(id) = id / Vl, local row = id - owner*Vl.  Per step:
//   requester: route_count  -> counts[o]       (entries per owner: item slot + non-padding history slots)
//              route_fill   -> send_ids[...]   (local row ids grouped by owner), pos[b][t] (entry position);
//                              positions are handed out per 256-entry round (one atomic per owner)
//   [all_to_all_single of counts, then ids]
//   owner:     owner_gather -> reply rows (E_local[id]); registers the rows in the sparse-grad map
//   [all_to_all_single of rows back]
//   requester: fields_fwd MODE 1 reads rows at pos[b][t]  (fields.hip)
// Backward mirrors it: fields_bwd MODE 1 writes one gradient row per entry at pos[b][t],
// all_to_all back to the owners: the received rows ARE the owner's sparse gradient (slot =
// received entry), and fbn_sparse_fixup folds duplicates of a row into the entry that claimed
// it (the sparse reduce-scatter).  Ids stay int64 until routed; routed ids are int32 local rows.
#include "common.h"

// entry (b, t): t = 0 item id (always routed, even id 0 -> owner 0, row 0), t >= 1 history slot
// t-1 (routed only if non-zero).  Invalid ids set *err and are not routed (pos = -1).
__device__ __forceinline__ long long entry_id(const int64_t* item, const int64_t* seq, int L, int b, int t) {
  return t == 0 ? item[b] : seq[(size_t)b * L + (t - 1)];
}

__global__ void route_count_kernel(const int64_t* __restrict__ item, const int64_t* __restrict__ seq, int B, int L,
                                   long long V, long long Vl, int nranks, int* __restrict__ counts, int* err) {
  __shared__ int hist[64];
  for (int i = threadIdx.x; i < 64; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const long long total = (long long)B * (L + 1);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(e / (L + 1)), t = (int)(e % (L + 1));
    const long long id = entry_id(item, seq, L, b, t);
    if (id < 0 || id >= V) { atomicOr(err, 1); continue; }
    if (t > 0 && id == 0) continue;
    atomicAdd(&hist[(int)(id / Vl)], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nranks; i += blockDim.x)
    if (hist[i]) atomicAdd(&counts[i], hist[i]);
}

// offsets = exclusive scan of counts (N <= 64, one thread); cursor zeroed
__global__ void route_scan_kernel(const int* counts, int nranks, int* offsets, int* cursor) {
  int s = 0;
  for (int i = 0; i < nranks; ++i) { offsets[i] = s; s += counts[i]; cursor[i] = 0; }
  offsets[nranks] = s;
}

// One round = 256 consecutive entries per workgroup.  Positions inside an owner's segment are
// handed out per round, not per entry: each wave ranks its lanes per owner by ballot, the round's
// per-owner totals take ONE global atomic each (a per-entry atomicAdd on cursor[o] serialised all
// B*(L+1) entries of a step on nranks counters: ~1 ms per step at N = 1, ~0.25 ms at N = 8).
// Order inside a round is deterministic (wave, lane); rounds of different workgroups race.
// FC (the fixed-capacity exchange, fbn_route_fc): owner o's segment is block o of cap + 1 slots
// (position o * (cap + 1) + k); an entry past k = cap - 1 is not routed (pos -1) and flags the
// routing as overflowed -- *ovf = 1 and every block's last slot = -2 (the flag travels in-band
// with the ids, so every owner learns that some requester overflowed)
template <bool FC>
__global__ void __launch_bounds__(256) route_fill_kernel(const int64_t* __restrict__ item,
                                                         const int64_t* __restrict__ seq, int B, int L, long long V,
                                                         long long Vl, int nranks, const int* __restrict__ offsets,
                                                         int* __restrict__ cursor, int* __restrict__ send_ids,
                                                         int* __restrict__ pos, int cap, int* __restrict__ ovf,
                                                         int* __restrict__ err) {
  __shared__ int wc[4][64];     // per wave, per owner: entries this round
  __shared__ int gb[4][64];     // per wave, per owner: first position
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long total = (long long)B * (L + 1);
  for (long long r0 = (long long)blockIdx.x * 256; r0 < total; r0 += (long long)gridDim.x * 256) {
    for (int i = threadIdx.x; i < 4 * 64; i += 256) (&wc[0][0])[i] = 0;
    const long long e = r0 + threadIdx.x;
    int o = -1, lid = 0;
    if (e < total) {
      const int b = (int)(e / (L + 1)), t = (int)(e % (L + 1));
      const long long id = entry_id(item, seq, L, b, t);
      if (id >= 0 && id < V && !(t > 0 && id == 0)) {
        o = (int)(id / Vl);
        lid = (int)(id - (long long)o * Vl);
      } else if (FC && (id < 0 || id >= V)) {
        atomicOr(err, 1);                            // (the count pass flags them in the other form)
      }
    }
    __syncthreads();
    int rank = 0;
    unsigned long long todo = __ballot(o >= 0);
    while (todo) {                                   // one pass per distinct owner in the wave
      const int ow = __shfl(o, __ffsll((long long)todo) - 1, 64);
      const unsigned long long m = __ballot(o == ow);
      if (o == ow) rank = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      if (lane == 0) wc[wave][ow] = __popcll(m);
      todo &= ~m;
    }
    __syncthreads();
    if (threadIdx.x < nranks) {
      const int q = threadIdx.x;
      const int n = wc[0][q] + wc[1][q] + wc[2][q] + wc[3][q];
      int base = n ? (FC ? 0 : offsets[q]) + atomicAdd(&cursor[q], n) : 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) { gb[w][q] = base; base += wc[w][q]; }
    }
    __syncthreads();
    if (e < total) {
      int p = -1;
      if (o >= 0) {
        p = gb[wave][o] + rank;
        if (FC) {
          if (p >= cap) {
            p = -1;
            atomicOr(ovf, 1);
            for (int k = 0; k < nranks; ++k) send_ids[(size_t)k * (cap + 1) + cap] = -2;
          } else {
            p += o * (cap + 1);
          }
        }
        if (p >= 0) send_ids[p] = lid;
      }
      pos[e] = p;
    }
    __syncthreads();                                 // wc / gb are rewritten by the next round
  }
}

// the fixed-capacity routing's initial state: every slot "no row" (-1), counters and flag zero
__global__ void route_fc_init_kernel(int* __restrict__ send_ids, long long n, int* __restrict__ stat, int nstat) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    send_ids[i] = -1;
  if (blockIdx.x == 0 && threadIdx.x < nstat) stat[threadIdx.x] = 0;
}

// owner side of a fixed-capacity routing: stat[0] |= "some requester overflowed" (a block whose
// last slot is -2) -- the same value on every rank, so all of them agree on a fallback.  self_send
// (an all-to-all that skipped the caller's own block): that block is copied from the caller's
// send_ids first (its flag slot included).
__global__ void __launch_bounds__(256) route_fc_status_kernel(const int* __restrict__ self_send,
                                                              int* __restrict__ recv_ids, int world, int rank, int cap,
                                                              int* __restrict__ stat) {
  const size_t o = (size_t)rank * (cap + 1);
  if (self_send)
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i <= cap; i += (long long)gridDim.x * blockDim.x)
      reinterpret_cast<int*>(recv_ids)[o + i] = self_send[o + i];
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    const int r = threadIdx.x;
    // (the own block's flag read at its source: the copy above may not have reached it yet)
    const int* blk = (self_send && r == rank) ? self_send : recv_ids;
    const bool f = r < world && blk[(size_t)r * (cap + 1) + cap] == -2;
    if (__ballot(f) != 0ull && r == 0) stat[0] = 1;
  }
}

// owner side: out[i] = E_local[ids[i]]; G = D/4 lanes per row.  Received entry i claims its
// row for the sparse gradient (map[r] = i, slot_row[i] = r) unless another entry did first.
// Rows with global id 0 (rank 0, local row 0) are padding: gathered (the item lookup of id 0
// reads row 0) but never registered for a gradient.
// (self_out: entries [self_lo, self_lo + self_n) -- the caller's own requests in the fixed-capacity
// exchange -- are written there instead, at the same index: the requester's row buffer itself)
template <int D>
__global__ void __launch_bounds__(256) owner_gather_kernel(const int* __restrict__ ids, int n, const float* __restrict__ E,
                                                           float* __restrict__ out, int* map, int* slot_row, int rank,
                                                           int out_bf16, float* __restrict__ self_out, int self_lo,
                                                           int self_n) {
  constexpr int G = D / 4, RPW = 64 / G;
  const int lane = threadIdx.x & 63, q = lane % G;
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long i0 = gw * RPW; i0 < n; i0 += nw * RPW) {
    const long long i = i0 + lane / G;
    if (i >= n) continue;
    const int r = ids[i];
    if (r < 0) continue;   // a fixed-capacity block's empty slot: nothing requested
    const f32x4 row = *reinterpret_cast<const f32x4*>(E + (size_t)r * D + 4 * q);
    float* dst = (self_out && i >= self_lo && i < self_lo + self_n) ? self_out : out;
    if (out_bf16)   // bf16 mode: the rows cross the wire as bf16 (half the all-to-all bytes)
      *reinterpret_cast<bf16x4*>(reinterpret_cast<short*>(dst) + i * D + 4 * q) =
          (bf16x4){f2bf(row[0]), f2bf(row[1]), f2bf(row[2]), f2bf(row[3])};
    else
      *reinterpret_cast<f32x4*>(dst + i * D + 4 * q) = row;
    if (map && q == 0 && !(rank == 0 && r == 0) &&
        __hip_atomic_load(map + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == -1) {
      int expected = -1;
      if (__hip_atomic_compare_exchange_strong(map + r, &expected, (int)i, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT))
        slot_row[i] = r;
    }
  }
}

// Registration only (the lazy table Adam must replay the claimed rows BEFORE they are
// gathered): same claims as owner_gather_kernel's map path.
__global__ void owner_claim_kernel(const int* __restrict__ ids, int n, int* map, int* slot_row, int rank) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = ids[i];
    if (r < 0 || (rank == 0 && r == 0)) continue;
    if (__hip_atomic_load(map + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != -1) continue;
    int expected = -1;
    if (__hip_atomic_compare_exchange_strong(map + r, &expected, i, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      slot_row[i] = r;
  }
}

// ------------------------------------------------------------------ C ABI
extern "C" int fbn_owner_claim(const int* ids, int n, int* map, int* slot_row, int rank, void* stream) {
  if (n <= 0) return FBN_OK;
  int blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  fbn_launch(owner_claim_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, ids, n, map, slot_row, rank);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_route(const int64_t* item, const int64_t* seq, int B, int L, long long V, long long Vl, int nranks,
                         int* counts, int* offsets, int* cursor, int* send_ids, int* pos, int* err, void* stream) {
  if (nranks < 1 || nranks > 64) { fbn_set_error("route: 1 <= nranks <= 64"); return FBN_ERR_ARG; }
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(counts, 0, sizeof(int) * nranks, st);
  const long long total = (long long)B * (L + 1);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  // the count's per-workgroup histograms meet in one global atomic per (workgroup, owner): keep
  // the workgroups few (grid-stride) so the nranks counters see <= 256 atomics each
  fbn_launch(route_count_kernel, dim3(std::min(blocks, 256)), dim3(256), 0, st, item, L > 0 ? seq : nullptr,
                     B, L, V, Vl, nranks, counts, err);
  fbn_launch(route_scan_kernel, dim3(1), dim3(1), 0, st, counts, nranks, offsets, cursor);
  fbn_launch(route_fill_kernel<false>, dim3(blocks), dim3(256), 0, st, item, L > 0 ? seq : nullptr, B, L, V, Vl,
                     nranks, offsets, cursor, send_ids, pos, 0, nullptr, nullptr);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// The fixed-capacity routing: entry positions o * (cap + 1) + k in owner o's block, blocks
// pre-filled with -1, stat = [overflow flag, entries requested from owner 0 .. nranks-1] (the
// requested counts include entries past cap).  No count pass and no host-side counts: the ids,
// looked-up rows and gradient rows all cross as equal-split all-to-alls of cap + 1 slots.
extern "C" int fbn_route_fc(const int64_t* item, const int64_t* seq, int B, int L, long long V, long long Vl, int nranks,
                            int cap, int* send_ids, int* pos, int* stat, int* err, void* stream) {
  if (nranks < 1 || nranks > 64 || cap < 1) { fbn_set_error("fbn_route_fc: 1 <= nranks <= 64, cap >= 1"); return FBN_ERR_ARG; }
  if (!item || !send_ids || !pos || !stat || !err || (L > 0 && !seq)) { fbn_set_error("fbn_route_fc: null buffer"); return FBN_ERR_ARG; }
  hipStream_t st = (hipStream_t)stream;
  const long long nslots = (long long)nranks * (cap + 1);
  long long iblocks = (nslots + 255) / 256;
  if (iblocks > 1024) iblocks = 1024;
  fbn_launch(route_fc_init_kernel, dim3((unsigned)iblocks), dim3(256), 0, st, send_ids, nslots, stat, nranks + 1);
  const long long total = (long long)B * (L + 1);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  fbn_launch(route_fill_kernel<true>, dim3(blocks), dim3(256), 0, st, item, L > 0 ? seq : nullptr, B, L, V, Vl,
             nranks, nullptr, stat + 1, send_ids, pos, cap, stat, err);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// After the ids all-to-all of a fixed-capacity routing: stat[0] becomes the GLOBAL overflow flag
// (this rank's, or any requester's in-band flag), then stat[0 .. nranks] is copied to `host`
// (pinned) on the stream -- the host reads it once the stream got there and, if set, every rank
// exchanges that step with host-side split sizes instead (RowExchange).
extern "C" int fbn_route_fc_status(const int* send_ids, int* recv_ids, int nranks, int rank, int cap, int* stat,
                                   int* host, void* stream) {
  if (nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks || cap < 1 || !recv_ids || !stat) {
    fbn_set_error("fbn_route_fc_status: 1 <= nranks <= 64, 0 <= rank < nranks, cap >= 1, buffers");
    return FBN_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  long long blocks = send_ids ? ((long long)cap + 1 + 255) / 256 : 1;
  if (blocks > 1024) blocks = 1024;
  fbn_launch(route_fc_status_kernel, dim3((unsigned)blocks), dim3(256), 0, st, send_ids, recv_ids, nranks, rank, cap,
             stat);
  FBN_CHECK_LAUNCH();
  if (host && hipMemcpyAsync(host, stat, sizeof(int) * (nranks + 1), hipMemcpyDeviceToHost, st) != hipSuccess) {
    fbn_set_error("fbn_route_fc_status: hipMemcpyAsync failed");
    return FBN_ERR_LAUNCH;
  }
  return FBN_OK;
}

#define FBN_DISPATCH_D(KERNEL, D, GRID, ...)                                                         \
  switch (D) {                                                                                      \
    case 16: fbn_launch((KERNEL<16>), GRID, dim3(256), 0, st, __VA_ARGS__); break;          \
    case 32: fbn_launch((KERNEL<32>), GRID, dim3(256), 0, st, __VA_ARGS__); break;          \
    case 64: fbn_launch((KERNEL<64>), GRID, dim3(256), 0, st, __VA_ARGS__); break;          \
    case 128: fbn_launch((KERNEL<128>), GRID, dim3(256), 0, st, __VA_ARGS__); break;        \
    case 256: fbn_launch((KERNEL<256>), GRID, dim3(256), 0, st, __VA_ARGS__); break;        \
    default: fbn_set_error("exchange: D must be 16/32/64/128/256"); return FBN_ERR_UNSUPPORTED;      \
  }

static dim3 rows_grid(long long n, int D) {
  const int rpw = 256 / D;
  long long blocks = ((n + rpw - 1) / rpw + 3) / 4;
  if (blocks < 1) blocks = 1;
  if (blocks > 8192) blocks = 8192;
  return dim3((unsigned)blocks);
}

extern "C" int fbn_owner_gather(const int* ids, int n, const float* E, void* out, int* map, int* slot_row, int rank,
                                int D, int out_bf16, void* stream) {
  if (n <= 0) return FBN_OK;
  hipStream_t st = (hipStream_t)stream;
  FBN_DISPATCH_D(owner_gather_kernel, D, rows_grid(n, D), ids, n, E, (float*)out, map, slot_row, rank, out_bf16,
                 nullptr, 0, 0);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_owner_gather_self(const int* ids, int n, const float* E, void* out, int* map, int* slot_row,
                                     int rank, int D, int out_bf16, void* self_out, int self_lo, int self_n,
                                     void* stream) {
  if (n <= 0) return FBN_OK;
  if (self_n < 0 || self_lo < 0 || (self_n > 0 && !self_out)) {
    fbn_set_error("fbn_owner_gather_self: self block");
    return FBN_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  FBN_DISPATCH_D(owner_gather_kernel, D, rows_grid(n, D), ids, n, E, (float*)out, map, slot_row, rank, out_bf16,
                 (float*)self_out, self_lo, self_n);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// bf16 -> f32, 8 elements per thread (the owner's received bf16 gradient rows, before the sparse
// fold and the table Adam read them as f32)
__global__ void __launch_bounds__(256) widen_bf16_kernel(const short* __restrict__ in, float* __restrict__ out,
                                                         long long n8) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(in + 8 * i);
    f32x4 a, b;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] = __uint_as_float((unsigned)(unsigned short)v[k] << 16);
      b[k] = __uint_as_float((unsigned)(unsigned short)v[k + 4] << 16);
    }
    *reinterpret_cast<f32x4*>(out + 8 * i) = a;
    *reinterpret_cast<f32x4*>(out + 8 * i + 4) = b;
  }
}

extern "C" int fbn_widen_bf16(const void* in, float* out, long long n, void* stream) {
  if (n <= 0) return FBN_OK;
  if ((n & 7) || ((uintptr_t)in & 15) || ((uintptr_t)out & 15)) {
    fbn_set_error("fbn_widen_bf16: n % 8 == 0 and 16-B aligned buffers");
    return FBN_ERR_ARG;
  }
  const long long n8 = n / 8;
  long long blocks = (n8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  fbn_launch(widen_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const short*>(in), out, n8);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// Padded copy of a routing: out[o][j] = the j-th id routed to owner o (send_ids[offsets[o] + j]) for
// j < counts[o], else -1 -- an all-to-all with equal splits of `cap` then needs no host-side counts
// (RowExchange.prepare: the next step's requests reach their owners during this step)
// The next step's routing as ONE equal-split all-to-all (RowExchange.prepare): destination o
// gets a block of cap + 1 ints -- its routed local rows padded with -1 to cap, then -2 - count in
// the last slot.  Negative slots read as "no row" (fbn_adam_prefetch_rows takes the received
// blocks as they are); fbn_compact_routes recovers the counts and the packed ids at the owner,
// so the next forward needs neither a counts nor an ids all-to-all.
__global__ void pad_routes_kernel(const int* __restrict__ send_ids, const int* __restrict__ offsets,
                                  const int* __restrict__ counts, int world, int cap, int* __restrict__ out) {
  const int cap1 = cap + 1;
  const long long total = (long long)world * cap1;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int o = (int)(i / cap1), j = (int)(i - (long long)o * cap1);
    const int c = counts[o];
    out[i] = j == cap ? -2 - c : (j < c ? send_ids[offsets[o] + j] : -1);
  }
}

extern "C" int fbn_pad_routes(const int* send_ids, const int* offsets, const int* counts, int world, int cap, int* out,
                              void* stream) {
  if (world <= 0 || cap <= 0) return FBN_OK;
  if (!send_ids || !offsets || !counts || !out) { fbn_set_error("fbn_pad_routes: null buffer"); return FBN_ERR_ARG; }
  long long blocks = ((long long)world * (cap + 1) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  fbn_launch(pad_routes_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, send_ids, offsets,
                     counts, world, cap, out);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// owner side of the padded exchange: counts[r] = entries requested by rank r, ids = the requests
// packed in rank order (what the host-split ids all-to-all would have delivered)
__global__ void compact_routes_kernel(const int* __restrict__ padded, int world, int cap, int* __restrict__ ids,
                                      int* __restrict__ counts) {
  __shared__ int cnt[64], off[64];
  const int cap1 = cap + 1;
  if (threadIdx.x < world) cnt[threadIdx.x] = -2 - padded[(long long)threadIdx.x * cap1 + cap];
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int r = 0; r < world; ++r) { off[r] = s; s += cnt[r]; }
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < world) counts[threadIdx.x] = cnt[threadIdx.x];
  const long long total = (long long)world * cap1;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cap1), j = (int)(i - (long long)r * cap1);
    if (j < cnt[r]) ids[off[r] + j] = padded[i];
  }
}

extern "C" int fbn_compact_routes(const int* padded, int world, int cap, int* ids, int* counts, void* stream) {
  if (world < 1 || world > 64 || cap <= 0) { fbn_set_error("fbn_compact_routes: 1 <= world <= 64, cap > 0"); return FBN_ERR_ARG; }
  if (!padded || !ids || !counts) { fbn_set_error("fbn_compact_routes: null buffer"); return FBN_ERR_ARG; }
  long long blocks = ((long long)world * (cap + 1) + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  fbn_launch(compact_routes_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, padded, world,
                     cap, ids, counts);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

// ------------------------------------------------------------------ step inputs -> static buffers
// Up to 8 device-to-device copies in ONE launch (16-B granules; sizes and pointers 16-B aligned):
// the batch fields, labels and pos of a step copied into the addresses the trainer's captured
// compute segments read (each copy_ alone is a ~5 us blit launch).
struct CopyJobs {
  const int4* src[8];
  int4* dst[8];
  long long n16[8];
  long long first[9];   // first granule of each job (prefix sum)
};
__global__ void __launch_bounds__(256) copy_jobs_kernel(CopyJobs J, int njobs) {
  const long long total = J.first[njobs];
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (long long)gridDim.x * blockDim.x) {
    int j = 0;
    while (j + 1 < njobs && g >= J.first[j + 1]) ++j;
    const long long k = g - J.first[j];
    J.dst[j][k] = J.src[j][k];
  }
}

extern "C" int fbn_copy_jobs(const void* const* src, void* const* dst, const long long* bytes, int n, void* stream) {
  if (n <= 0) return FBN_OK;
  if (n > 8) { fbn_set_error("fbn_copy_jobs: at most 8 copies"); return FBN_ERR_ARG; }
  CopyJobs J;
  J.first[0] = 0;
  for (int i = 0; i < 8; ++i) {
    const int k = i < n ? i : 0;
    if (i < n && ((bytes[i] & 15) || (((uintptr_t)src[i] | (uintptr_t)dst[i]) & 15))) {
      fbn_set_error("fbn_copy_jobs: sizes and addresses must be 16-byte multiples");
      return FBN_ERR_ARG;
    }
    J.src[i] = (const int4*)src[k];
    J.dst[i] = (int4*)dst[k];
    J.n16[i] = i < n ? bytes[i] / 16 : 0;
    J.first[i + 1] = J.first[i] + J.n16[i];
  }
  if (J.first[n] <= 0) return FBN_OK;
  long long blocks = (J.first[n] + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  fbn_launch(copy_jobs_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, J, n);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}
