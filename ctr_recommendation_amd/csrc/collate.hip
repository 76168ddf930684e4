// Device collator: the batch_dict of BatchCollator.__call__
// (src/dataloader.py:69-121) and InferenceCollator.__call__ (src/Prediction.py:28-52), assembled
// in HBM by one launch from a dataset held column-wise in HBM (MicroLens train: 3.6 M rows,
// ~0.7 GB -- nothing next to 288 GB) and an item_info table resident in HBM.
//
// The reference builds each batch on the host: default_collate of the rows of one float64
// column_stack (src/dataloader.py:48), a pandas .loc of item_emb_d128 by item_id (:91-95), the
// last-max_len truncation of item_seq (:111-116) and pageable H2D copies (src/train_fibinet.py:
// 109-111); that path tops out near 1e6 samples/s.  Here one wave per sample copies
// its row of every column (the permutation gives the dataset row) and gathers its 128-float
// item_info row: coalesced 512-B row reads, like the table gather of fields_fwd.
//
// Unknown item ids (no item_info row): the training collator raises KeyError (.loc,
// src/dataloader.py:104-106) -- here the row is zero-filled and *missing is set, and the host
// raises KeyError when it checks; the inference collator (src/Prediction.py:37-42) uses
// reindex().fillna(0), and np.stack of a batch that mixes 128-lists with the scalar fill raises,
// so its except branch zeroes the WHOLE batch's mm vectors -- fbn_collate_zero_if reproduces that
// with a per-batch flag, without a host round trip.
#include "common.h"
#include <algorithm>

struct CollateArgs {
  const int64_t* perm;        // [B] dataset row of each batch row
  int B;
  const int64_t* item;        // [N]
  const int64_t* seq;         // [N][Ls] or null
  int Ls, L, seq_off;         // output keeps columns [seq_off, seq_off + L) (= the last L when seq_off = Ls - L)
  const int64_t* likes;       // [N] (null: skipped)
  const int64_t* views;
  const int64_t* user;
  const float* label;         // [N] or null
  const int* slot_of_id;      // [n_ids] row of emb, -1 = no item_info row (dense index by id), or
                              // with sorted_ids: [n_ids] row of emb of the k-th sorted id
  long long n_ids;
  const int64_t* sorted_ids;  // null: dense index; else [n_ids] ascending ids (sparse / hashed ids)
  const float* emb;           // [rows][E] or null
  int E;                      // multiple of 4
  int64_t* o_item;
  int64_t* o_seq;
  int64_t* o_likes;
  int64_t* o_views;
  int64_t* o_user;
  float* o_label;
  float* o_emb;
  int* missing;               // set to 1 when an item_id has no item_info row
};

__global__ void __launch_bounds__(256) collate_kernel(CollateArgs a) {
  const int lane = threadIdx.x & 63;
  const long long w = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long b = w; b < a.B; b += nw) {
    const long long r = a.perm[b];
    const int64_t id = a.item[r];
    if (lane == 0) {
      a.o_item[b] = id;
      if (a.likes) a.o_likes[b] = a.likes[r];
      if (a.views) a.o_views[b] = a.views[r];
      if (a.user) a.o_user[b] = a.user[r];
      if (a.label) a.o_label[b] = a.label[r];
    }
    if (a.seq)
      for (int t = lane; t < a.L; t += 64) a.o_seq[b * a.L + t] = a.seq[r * a.Ls + a.seq_off + t];
    if (a.emb) {
      int row = -1;
      if (!a.sorted_ids) {
        row = (id >= 0 && id < a.n_ids) ? a.slot_of_id[id] : -1;
      } else {   // lower bound over the sorted ids (wave-uniform: every lane takes the same path)
        long long lo = 0, hi = a.n_ids;
        while (lo < hi) {
          const long long mid = (lo + hi) >> 1;
          if (a.sorted_ids[mid] < id) lo = mid + 1; else hi = mid;
        }
        row = (lo < a.n_ids && a.sorted_ids[lo] == id) ? a.slot_of_id[lo] : -1;
      }
      if (row < 0 && lane == 0) *a.missing = 1;
      for (int c = lane * 4; c < a.E; c += 256) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (row >= 0) v = *reinterpret_cast<const f32x4*>(a.emb + (size_t)row * a.E + c);
        *reinterpret_cast<f32x4*>(a.o_emb + (size_t)b * a.E + c) = v;
      }
    }
  }
}

__global__ void zero_if_kernel(float* x, long long n, const int* flag) {
  if (*flag == 0) return;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] = 0.f;
}

extern "C" int fbn_collate(const int64_t* perm, int B, const int64_t* item, const int64_t* seq, int Ls, int L,
                           const int64_t* likes, const int64_t* views, const int64_t* user, const float* label,
                           const int* slot_of_id, long long n_ids, const int64_t* sorted_ids, const float* emb,
                           int E, int64_t* o_item,
                           int64_t* o_seq, int64_t* o_likes, int64_t* o_views, int64_t* o_user, float* o_label,
                           float* o_emb, int* missing, void* stream) {
  if (B <= 0) return FBN_OK;
  if (!perm || !item || !o_item) { fbn_set_error("fbn_collate: perm, item and o_item are required"); return FBN_ERR_ARG; }
  if (seq && (L < 0 || L > Ls || !o_seq)) { fbn_set_error("fbn_collate: need 0 <= L <= Ls and o_seq"); return FBN_ERR_ARG; }
  if (emb && (!slot_of_id || !o_emb || !missing || (E & 3) || ((uintptr_t)emb & 15) || ((uintptr_t)o_emb & 15))) {
    fbn_set_error("fbn_collate: emb needs slot_of_id, o_emb, missing, E % 4 == 0 and 16-B alignment");
    return FBN_ERR_ARG;
  }
  if ((likes && !o_likes) || (views && !o_views) || (user && !o_user) || (label && !o_label)) {
    fbn_set_error("fbn_collate: every input column needs its output");
    return FBN_ERR_ARG;
  }
  CollateArgs a{perm, B, item, seq, Ls, L, Ls - L, likes, views, user, label, slot_of_id, n_ids, sorted_ids, emb, E,
                o_item, o_seq, o_likes, o_views, o_user, o_label, o_emb, missing};
  const int blocks = (int)std::min<long long>(2048, ((long long)B + 3) / 4);
  fbn_launch(collate_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}

extern "C" int fbn_collate_zero_if(float* x, long long n, const int* flag, void* stream) {
  if (n <= 0) return FBN_OK;
  if (!x || !flag) { fbn_set_error("fbn_collate_zero_if: x and flag are required"); return FBN_ERR_ARG; }
  const int blocks = (int)std::min<long long>(1024, (n + 255) / 256);
  fbn_launch(zero_if_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, n, flag);
  FBN_CHECK_LAUNCH();
  return FBN_OK;
}
