"""Row-sharded exchange protocol on 2, 3 and 4 gloo CPU ranks -- covers the N > 1 host path.

Runs the product's RowExchange (routing bookkeeping, split sizes, all_to_all_single, owner
gather, sparse reduce-scatter) with the CPU restatement of its kernels
(oracle/exchange_ref.py), and checks that
  * every requester receives exactly E[id] at pos[b][t] (item slot and non-padding history),
  * the owners' compact gradient rows equal the dense scatter-add of all ranks' gradients
    over the global table, padding row 0 excluded,
  * DistCollective sums over ranks (SyncBN / dense-grad all-reduce hook).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, V, d, B, L, q, hook=False, bf16=False, padded=False, fc=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ctr_recommendation_amd.exchange import DistCollective, RowExchange
        from oracle.exchange_ref import CpuExchangeKernels
        g = torch.Generator().manual_seed(0)
        E_full = torch.randn((V, d), generator=g)
        E_full[0] = 0
        # per-rank batches (different per rank), with padding and repeats
        gb = torch.Generator().manual_seed(100 + rank)
        item = torch.randint(0, V, (B,), generator=gb)
        seq = torch.randint(0, V, (B, L), generator=gb)
        seq[0] = 0
        seq[1, :3] = 5
        if fc == "one" and rank != 0:
            seq.zero_()          # items only: at most B entries per block -- these ranks' blocks all fit
        xg = RowExchange(rank, world, V, d, B, L, torch.device("cpu"), kernels=CpuExchangeKernels(), rows_bf16=bf16)
        lo, n_local = xg.rows_lo, xg.rows_local
        E_local = E_full[lo:lo + n_local].clone()
        cap = world * (B * (L + 1) + 1)          # (>= the fixed form's world * (cap + 1) slots)
        sparse = {"map": torch.full((n_local,), -1, dtype=torch.int32),
                  "slot_row": torch.full((cap,), -1, dtype=torch.int32)}
        err = torch.zeros(1, dtype=torch.int32)
        seen = {}

        def before_gather(n_recv):
            # the lazy table Adam's slot: every requested non-padding row is claimed by now
            # and nothing has been gathered yet -> shift the claimed rows; requesters must see it
            sr = sparse["slot_row"][:n_recv]
            claimed = sr[sr >= 0].long()
            seen["n"] = int(claimed.numel())
            E_local[claimed] += 1000.0

        if fc is not None:
            # the fixed-capacity form: blocks of cap + 1 slots, routed by prepare() (inline on CPU);
            # "tiny" overflows on every rank's batch -> all ranks read the flag and fall back together;
            # "one": cap B, only rank 0's batch (full histories) overflows -- the others learn it from
            # the in-band flag in rank 0's blocks alone
            xg.enable_fixed({"fit": B * (L + 1), "tiny": 2, "one": B}[fc])
            xg.prepare(item, seq, err)
        rows = xg.forward(item, seq, E_local, sparse, err, before_gather=before_gather if hook else None)
        pos = xg.cur_pos
        fc_state = (xg.fc_active, xg.fc_fallbacks)
        ok_pad = True
        if padded:
            # the routed-ahead form of the same requests (RowExchange.prepare on a GPU): every
            # destination's ids padded to cap with -1 and its count in the last slot, ONE
            # equal-split all-to-all, the owner packs them -> the inline path's counts and ids
            st = xg.sets[xg.cur]
            cap = B * (L + 1)
            pad = torch.empty(world * (cap + 1), dtype=torch.int32)
            xg.k.pad_routes(st["send_ids"], st["offsets"], st["counts"], world, cap, pad)
            recv = torch.empty_like(pad)
            dist.all_to_all_single(recv, pad)
            ids2 = torch.empty(world * cap, dtype=torch.int32)
            cnt2 = torch.zeros(world, dtype=torch.int32)
            xg.k.compact_routes(recv, world, cap, ids2, cnt2)
            n_recv = sum(xg.recv_counts)
            ok_pad = cnt2.tolist() == list(xg.recv_counts) and torch.equal(ids2[:n_recv], xg.recv_ids)
        ids = torch.cat([item.view(B, 1), seq], dim=1)
        ok_fwd = True
        for b in range(B):
            for t in range(L + 1):
                p = int(pos[b, t])
                if t > 0 and int(ids[b, t]) == 0:
                    ok_fwd &= p == -1
                    continue
                want = E_full[int(ids[b, t])] + (1000.0 if hook and int(ids[b, t]) != 0 else 0.0)
                ok_fwd &= p >= 0 and torch.equal(rows[p], want.to(rows.dtype))
        # backward: one random gradient row per routed entry
        sendbuf = xg.make_sendbuf()
        sendbuf.copy_(torch.randn(sendbuf.shape, generator=gb))
        grows = xg.backward(sendbuf).float()        # (the fixed form hands back the wire rows)
        CpuExchangeKernels.sparse_fixup_owner(xg.recv_ids, grows, sparse["map"], rank)
        # dense reference: all ranks' scatter over the global table
        dense = torch.zeros((V, d), dtype=torch.float64)
        for b in range(B):
            for t in range(L + 1):
                p = int(pos[b, t])
                if p >= 0 and int(ids[b, t]) != 0:
                    dense[int(ids[b, t])] += sendbuf[p].double()
        dist.all_reduce(dense)
        got = torch.zeros((n_local, d), dtype=torch.float64)
        nu = 0
        for i in range(grows.shape[0]):
            r = int(sparse["slot_row"][i])
            if r >= 0:
                assert int(sparse["map"][r]) == i
                got[r] = grows[i].double()
                nu += 1
        bwd_err = float((got - dense[lo:lo + n_local]).abs().max())
        touched = (dense[lo:lo + n_local].abs().sum(1) > 0).sum().item()
        c = DistCollective(world)
        t = torch.full((3,), float(rank + 1), dtype=torch.float64)
        c.allreduce_(t)
        own_ovf = None
        if fc is not None:
            # did THIS rank's own routing overflow? (stat[0] before the status kernel ORs the peers' flags)
            st = {}
            xg.k.route_fc(item, seq, B, L, V, xg.Vl, world, xg.cap, torch.empty(world * (xg.cap + 1), dtype=torch.int32),
                          torch.empty((B, L + 1), dtype=torch.int32), st.setdefault("stat", torch.zeros(world + 1,
                                                                                                     dtype=torch.int32)),
                          torch.zeros(1, dtype=torch.int32))
            own_ovf = int(st["stat"][0])
        q.put((rank, bool(ok_fwd and ok_pad), bwd_err, nu, touched, t.tolist(), int(err[0]),
               (fc_state, own_ovf) if fc is not None else None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,hook,bf16,padded,fc", [(2, False, False, False, None), (3, False, False, False, None),
                                                       (2, True, False, False, None), (4, False, False, True, None),
                                                       (4, True, False, False, None), (4, False, True, True, None),
                                                       (8, True, True, True, None),
                                                       (2, True, False, False, "fit"), (3, False, True, False, "fit"),
                                                       (4, True, True, False, "fit"), (3, True, False, False, "tiny"),
                                                       (8, True, True, False, "fit"), (3, True, False, False, "one"),
                                                       (4, False, True, False, "one")])
def test_row_exchange_protocol(world, hook, bf16, padded, fc):
    """hook: the owner-side claim -> before_gather -> gather split used by the lazy table Adam.
    bf16: the bf16 mode's wire rows (each delivered row == E[id] rounded to bf16).  padded: the
    routed-ahead padded blocks deliver the same counts and ids.  world 8: C4's split (eight
    owners, blocks of B * (L + 1) + 1 ints per destination), bf16 rows, history length 20.
    fc: the fixed-capacity form (equal-split all-to-alls of cap + 1 slots, empty slots negative):
    "fit" -- every block fits, the step exchanges in that form; "tiny" -- cap 2 overflows, every rank
    sees the in-band flag and the step falls back to host split sizes on all ranks together; "one" --
    only rank 0's batch overflows: the ranks whose own routing fit must still fall back, from the flag
    in rank 0's blocks (a rank that missed it would run the equal-split all-to-all against the others'
    host-split one and deadlock)."""
    V, d, B, L = (101, 8, 12, 6) if world < 8 else (1001, 8, 12, 20)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, V, d, B, L, q, hook, bf16, padded, fc))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tot = sum(range(1, world + 1))
    for rank, ok_fwd, bwd_err, nu, touched, red, err, fc_state in res:
        if fc is not None:
            fc_state, own_ovf = fc_state
            assert fc_state == ((True, 0) if fc == "fit" else (False, 1)), (rank, fc_state)
            if fc == "one":
                assert own_ovf == (1 if rank == 0 else 0), (rank, own_ovf)
        assert ok_fwd, f"rank {rank}: wrong rows delivered"
        assert bwd_err < 1e-5, f"rank {rank}: sparse reduce-scatter error {bwd_err}"
        assert nu >= touched
        assert red == [float(tot)] * 3
        assert err == 0


def _check_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ctr_recommendation_amd.loader import DeviceLoader
        dl = DeviceLoader.__new__(DeviceLoader)          # only the sticky flag matters to check()
        dl.missing = torch.tensor([1 if rank == world - 1 else 0], dtype=torch.int32)
        try:
            dl.check(world=world)
            q.put((rank, "no raise"))
        except KeyError:
            q.put((rank, "raised"))
    finally:
        dist.destroy_process_group()


def test_loader_check_raises_on_every_rank():
    """An item id without item_info on ONE rank's batch: DeviceLoader.check(world=N) all-reduces the
    flag first, so every rank raises the collator's KeyError at the same step (src/dataloader.py:104-106)
    instead of the others blocking in the next step's collectives."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_check_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == [(r, "raised") for r in range(world)], res


def _agree_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        # all ranks equal -> valid, no differing step
        a = bench._ab_agree(True, -1, "cpu")
        # rank 1 saw its losses part at step 5, rank 2 only a final-state difference (no loss step)
        b = bench._ab_agree(rank not in (1, 2), 5 if rank == 1 else -1, "cpu")
        # two ranks with differing first steps: the earliest wins
        c = bench._ab_agree(rank == 0, {1: 9, 2: 4}.get(rank, -1), "cpu")
        q.put((rank, a, b, c))
    finally:
        dist.destroy_process_group()


def test_bench_native_ab_agreement():
    """bench.py's lockstep A/B of the native-RCCL path against torch.distributed (native_ab) decides on
    EVERY rank together: the native path is validated only if every rank saw bitwise-equal runs, and
    the first differing step reported is the earliest over the ranks -- so all ranks time the same
    path (a rank timing the other one would deadlock the collectives)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, a, b, c in res:
        assert a == (True, -1), (rank, a)
        assert b == (False, 5), (rank, b)
        assert c == (False, 4), (rank, c)


def _det_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ctr_recommendation_amd.exchange import DistCollective
        gens = [torch.Generator().manual_seed(40 + r) for r in range(world)]
        # values spanning many magnitudes: a different summation order would change the bits
        vals = [torch.randn(4099, generator=g) * torch.exp(torch.randn(4099, generator=g) * 6) for g in gens]
        vals64 = [v.double() * 1e-3 for v in vals]
        want = vals[0].clone()
        want64 = vals64[0].clone()
        for r in range(1, world):
            want += vals[r]
            want64 += vals64[r]
        c = DistCollective(world, det=True)
        t, t64 = vals[rank].clone(), vals64[rank].clone()
        c.allreduce_(t)
        c.allreduce_(t64)
        q.put((rank, bool(torch.equal(t, want)), bool(torch.equal(t64, want64))))
    finally:
        dist.destroy_process_group()


def test_deterministic_allreduce_rank_order():
    """Deterministic mode's all-reduce (DistCollective(det=True): all-gather, then the ranks' slices
    added in rank order) gives exactly the rank-ordered sum on every rank, f32 and f64 -- whatever
    order a reduction algorithm would have used (the same rule the native path runs as
    fbn_comm_allgather + fbn_sum_slices)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_det_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(r, True, True) for r in range(world)], res
