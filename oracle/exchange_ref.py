"""CPU restatement of the row-shard exchange kernels (exchange.hip) -- TEST INFRASTRUCTURE ONLY.

Lets tests/test_exchange_gloo.py run the real ``RowExchange`` protocol (routing, split
bookkeeping, all_to_all_single over gloo, sparse reduce-scatter) on CPU ranks.  The
semantics restated here are the product's own contract for the sharded path (the reference
has no sharding; it replicates the table with DataParallel, src/train_fibinet.py:69-70):
owner = id // Vl; item slot always routed; history slot routed iff id != 0; padding row
(global id 0) gathered but never updated.
"""
from __future__ import annotations

import torch


class CpuExchangeKernels:
    def route(self, item, seq, B, L, V, Vl, world, counts, offsets, cursor, send_ids, pos, err):
        ids = item.view(B, 1) if seq is None or L == 0 else torch.cat([item.view(B, 1), seq.view(B, L)], dim=1)
        valid = (ids >= 0) & (ids < V)
        if not bool(valid.all()):
            err.fill_(1)
        routed = valid.clone()
        routed[:, 1:] &= ids[:, 1:] != 0
        owner = torch.where(routed, ids // Vl, torch.zeros_like(ids))
        counts.zero_()
        for o in range(world):
            counts[o] = int(((owner == o) & routed).sum())
        offs = torch.zeros(world + 1, dtype=torch.int64)
        offs[1:] = torch.cumsum(counts.to(torch.int64), 0)
        offsets.copy_(offs.to(offsets.dtype))
        cursor.zero_()
        pos.fill_(-1)
        cur = offs[:-1].clone()
        for b in range(B):
            for t in range(ids.shape[1]):
                if routed[b, t]:
                    o = int(owner[b, t])
                    p = int(cur[o])
                    cur[o] += 1
                    send_ids[p] = int(ids[b, t] - o * Vl)
                    pos[b, t] = p

    def route_fc(self, item, seq, B, L, V, Vl, world, cap, send_ids, pos, stat, err):
        """Restates fbn_route_fc: owner o's block is slots [o * (cap + 1), o * (cap + 1) + cap), its
        last slot -1 (or -2 in every block once any entry overflowed); pos = the entry's slot or -1;
        stat = [overflow, entries requested per owner].  (The kernel's order inside a block depends
        on workgroup timing; this one is entry order -- the tests compare sets, not orders.)"""
        ids = item.view(B, 1) if seq is None or L == 0 else torch.cat([item.view(B, 1), seq.view(B, L)], dim=1)
        valid = (ids >= 0) & (ids < V)
        if not bool(valid.all()):
            err.fill_(1)
        send_ids.fill_(-1)
        pos.fill_(-1)
        cnt = [0] * world
        ovf = 0
        for b in range(B):
            for t in range(ids.shape[1]):
                i = int(ids[b, t])
                if not (0 <= i < V) or (t > 0 and i == 0):
                    continue
                o = i // Vl
                k = cnt[o]
                cnt[o] += 1
                if k >= cap:
                    ovf = 1
                    continue
                send_ids[o * (cap + 1) + k] = i - o * Vl
                pos[b, t] = o * (cap + 1) + k
        if ovf:
            for o in range(world):
                send_ids[o * (cap + 1) + cap] = -2
        stat[0] = ovf
        stat[1:1 + world] = torch.tensor(cnt, dtype=stat.dtype)

    def route_fc_status(self, send_ids, recv_ids, world, rank, cap, stat, host):
        """Restates fbn_route_fc_status: (send_ids given: the own block copied first, the all-to-all
        skipped it) stat[0] |= any requester's in-band flag; host <- stat."""
        if send_ids is not None:
            o = rank * (cap + 1)
            recv_ids[o:o + cap + 1] = send_ids[o:o + cap + 1]
        if any(int(recv_ids[r * (cap + 1) + cap]) == -2 for r in range(world)):
            stat[0] = 1
        host[:world + 1] = stat[:world + 1]

    def owner_claim(self, ids, map_, slot_row, rank):
        """Restates fbn_owner_claim: first entry referencing a row claims it (padding row and empty
        fixed-capacity slots excluded)."""
        for i, r in enumerate(ids.tolist()):
            if r >= 0 and not (rank == 0 and r == 0) and int(map_[r]) == -1:
                map_[r] = i
                slot_row[i] = r

    def owner_gather(self, ids, E, out, map_, slot_row, rank, d):
        for i, r in enumerate(ids.tolist()):
            if r < 0:
                continue                      # an empty fixed-capacity slot
            out[i] = E[r]                     # a bf16 `out` (the bf16 mode's wire rows) rounds here
            if map_ is not None and not (rank == 0 and r == 0) and int(map_[r]) == -1:
                map_[r] = i
                slot_row[i] = r

    def pad_routes(self, send_ids, offsets, counts, world, cap, out):
        """Restates fbn_pad_routes: owner o's routed ids padded with -1 to cap, then -2 - count."""
        out.fill_(-1)
        for o in range(world):
            c, off = int(counts[o]), int(offsets[o])
            out[o * (cap + 1):o * (cap + 1) + c] = send_ids[off:off + c]
            out[o * (cap + 1) + cap] = -2 - c

    def compact_routes(self, padded, world, cap, ids, counts):
        """Restates fbn_compact_routes: counts from the last slot of each block, ids packed in rank order."""
        s = 0
        for r in range(world):
            c = -2 - int(padded[r * (cap + 1) + cap])
            counts[r] = c
            ids[s:s + c] = padded[r * (cap + 1):r * (cap + 1) + c]
            s += c

    def widen(self, inp, out):
        """Restates fbn_widen_bf16: the owner's bf16 wire gradient rows to f32 (exact)."""
        out.copy_(inp.float())

    @staticmethod
    def sparse_fixup_owner(ids, grows, map_, rank):
        """Restates fbn_sparse_fixup's owner mode: fold duplicates into the claiming entry."""
        for i, r in enumerate(ids.tolist()):
            if r < 0 or (rank == 0 and r == 0):
                continue
            u = int(map_[r])
            if u != i:
                grows[u] += grows[i]
