"""The row-sharded (N > 1) trainer over RCCL, as a one-rank job on one MI355X.

RCCL refuses two ranks on one device, so the multi-rank rehearsals (test_gpu_multirank.py)
run their collectives over gloo.  This test runs the sharded code path itself -- RowExchange's
all-to-alls with host split lists, the route-ahead communicator and its side-stream
all-to-all (prepare), the owner-side prefetch, deferred gradient rows in a ring slot, the
packed dense all-reduce -- over the "nccl" backend (RCCL) with world = 1, both with RCCL called
on the step's own stream (csrc/comm.cpp, the default) and through torch.distributed's process
group (FiBiNETTrainer
shard=True), in a child process, and checks it against the single-GPU trainer on the same
batches: fp32 losses within 1e-5 (relative), the table within 1e-5 after the flush and the dense
parameters within 1e-3 of their displacement (norm; as test_gpu_trainer.py); with the bf16 wire
format (rows and gradient rows as bf16) the losses agree within 5e-3 over the 6 steps.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from tests._spawn import spawn_and_wait

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, store=dist.HashStore())
    try:
        from ctr_recommendation_amd.data import make_batch
        from ctr_recommendation_amd.trainer import FiBiNETTrainer
        from oracle.fibinet_oracle import build_model
        V, B, steps = 60000, 1024, 6
        out = {}
        for dtype in ("fp32", "bf16"):
            cfg = {"embedding_dim": 128, "vocab_size": V, "honour_config": True, "net_dropout": 0.0,
                   "compute_dtype": dtype}
            torch.manual_seed(0)
            init = build_model(None, cfg, honour_config=True).state_dict()
            bs = [make_batch(500 + s, B, V, device=dev) for s in range(steps + 1)]
            res = []
            # (shard, early): the single GPU; the sharded step with RCCL on the step's stream (the
            # default, exchange.NativeComm); torch.distributed's collectives with the early
            # (asynchronous) gradient all-to-all issued after the fields backward
            # (and the early gradient exchange with native RCCL on the exchange's own stream)
            for shard, early, native in ((False, False, True), (True, False, True), (True, True, False),
                                         (True, True, True)):
                os.environ["FBN_NATIVE_COMM"] = "1" if native else "0"
                tr = FiBiNETTrainer(cfg, total_steps=20, batch_size=B, device=dev, init_state=
                                    {k: v.clone() for k, v in init.items()}, shard=shard)
                tr.early_grad_xchg = early
                assert (tr.xchg is not None) == shard
                assert (tr.native_comm is not None) == (shard and native)
                assert tr._early_grad_xchg() == early
                p_init = tr.flat_p.cpu().clone()
                if shard:
                    assert tr.xchg.side is not None and tr.prefetch_owner and tr.deferred
                losses = [tr.step(bs[s][0], bs[s][1], next_batch=bs[s + 1][0]).item() for s in range(steps)]
                tr.flush()
                tr.check_ids()
                res.append((losses, tr.E.cpu().clone(), tr.flat_p.cpu().clone(), p_init))
                tr.close()                       # the communicators and their proxy threads
                tr.close()                       # idempotent
                assert tr.native_comm is None
            (l0, e0, p0, q0), (l1, e1, p1, _), (l2, e2, p2, _), (l3, e3, p3, _) = res
            # dense parameters: the difference relative to the 6 steps' displacement (Adam's
            # normalised step turns last-bit gradient differences into small absolute ones)
            out[dtype] = (l0, l1, float((e0 - e1).abs().max()), float((p0 - p1).norm() / (p0 - q0).norm()),
                          float(e0.abs().max()))
            # the early (asynchronous) gradient all-to-all: the same bars against the single GPU (the
            # duplicate fold's float atomics make two sharded runs differ in the last bits anyway)
            out[dtype + "_early"] = (l0, l2, float((e0 - e2).abs().max()), float((p0 - p2).norm() / (p0 - q0).norm()),
                                     float(e0.abs().max()))
            out[dtype + "_early_native"] = (l0, l3, float((e0 - e3).abs().max()),
                                            float((p0 - p3).norm() / (p0 - q0).norm()), float(e0.abs().max()))
        q.put(("ok", out))
    except Exception as e:   # report, then re-raise in the child
        q.put((repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def test_sharded_path_over_rccl_matches_single_gpu(hip_device):
    status, out = spawn_and_wait(_worker, (_port(),), timeout=300)
    assert status == "ok", status
    l0, l1, de, dp, e_max = out["fp32"]
    for a, b in zip(l0, l1):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (l0, l1)
    assert de <= 1e-5 * max(1.0, e_max) and dp <= 1e-3, (de, dp)
    for key in ("fp32_early", "fp32_early_native"):
        l0, l1, de, dp, e_max = out[key]
        for a, b in zip(l0, l1):
            assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (key, l0, l1)
        assert de <= 1e-5 * max(1.0, e_max) and dp <= 1e-3, (key, de, dp)
    for key in ("bf16", "bf16_early", "bf16_early_native"):
        l0, l1, de, dp, _ = out[key]
        # bf16 wire: the looked-up rows are rounded to bf16 before the fields kernel (the single-GPU
        # bf16 path reads f32 rows), so the two agree to bf16 rounding, not bit for bit
        for a, b in zip(l0, l1):
            assert abs(a - b) <= 5e-3, (key, l0, l1)


def _det_worker(port, q, steps=8):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FBN_NATIVE_COMM="1")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, store=dist.HashStore())
    try:
        from ctr_recommendation_amd.data import make_batch
        from ctr_recommendation_amd.trainer import FiBiNETTrainer
        from oracle.fibinet_oracle import build_model
        V, B = 60000, 1024
        cfg = {"embedding_dim": 128, "vocab_size": V, "honour_config": True, "net_dropout": 0.0,
               "compute_dtype": "fp32"}
        torch.manual_seed(0)
        init = build_model(None, cfg, honour_config=True).state_dict()
        bs = [make_batch(900 + s, B, V, device=dev) for s in range(steps + 1)]
        res = []
        for shard in (False, True):
            tr = FiBiNETTrainer(cfg, total_steps=max(20, steps + 4), batch_size=B, device=dev, deterministic=True,
                                init_state={k: v.clone() for k, v in init.items()}, shard=shard)
            assert tr.deterministic and (tr.native_comm is not None) == shard
            losses = [tr.step(bs[s][0], bs[s][1], next_batch=bs[s + 1][0]).item() for s in range(steps)]
            norms = float(tr.norm.item())
            tr.flush()
            tr.check_ids()
            res.append((losses, {n: getattr(tr, n).cpu().clone() for n in ("E", "Em", "Ev", "flat_p", "flat_m",
                                                                            "flat_v")}, norms,
                        tr.xchg.fc_active if shard else None))
            tr.close()
        (l0, t0, n0, _), (l1, t1, n1, fc) = res
        out = {"losses": (l0, l1), "norm": (n0, n1), "fc": fc,
               "equal": {k: bool(torch.equal(t0[k], t1[k])) for k in t0},
               "maxdiff": {k: float((t0[k] - t1[k]).abs().max()) for k in t0}}
        q.put(("ok", out))
    except Exception as e:
        q.put((repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def test_sharded_deterministic_matches_single_gpu_bitwise(hip_device):
    """Deterministic mode (src/utils.py:15-16), fp32: the one-rank sharded step over RCCL
    (route, owner claims and catch-up, exchange, per-entry gradient rows, the fixed-point owner fold,
    deferred ring slots, the packed all-reduce; through the exchange's calibration steps and the switch
    to the fixed-capacity form) against the single-GPU trainer's deterministic step on the same batches:
    every loss and the table, its Adam moments, the dense parameters and moments BIT-IDENTICAL (the
    fold's integer total is the same whichever entries carry the row, and the rest is the same
    kernels on the same values).  Only the clip norm is summed in another order (per-sample vector
    norms vs the rows' squares); it enters the update only when the clip engages, which it does not at
    max_norm 10 here -- both norms are reported."""
    status, out = spawn_and_wait(_det_worker, (_port(),), timeout=300)
    assert status == "ok", status
    print(f"det one-rank sharded vs single GPU: equal {out['equal']}, max |diff| {out['maxdiff']}, "
          f"norms {out['norm']}, fc {out['fc']}")
    assert out["fc"], "the sharded trainer never switched to the fixed-capacity exchange"
    assert max(out["norm"]) < 10.0, out["norm"]          # the clip did not engage (see docstring)
    l0, l1 = out["losses"]
    assert l0 == l1, (l0, l1)
    assert all(out["equal"].values()), (out["equal"], out["maxdiff"])


def _det_worker_steps(port, steps, q):
    _det_worker(port, q, steps)


def test_sharded_deterministic_matches_single_gpu_bitwise_long(hip_device):
    """The same bitwise comparison over 140 steps: past the deferred-gradient ring's wrap-around
    (F + 1 = 129 slots at d = 128) on both paths, with rows the rolling window replays over full
    128-step lags.  The clip must stay disengaged (both norms reported) for the bits to match."""
    status, out = spawn_and_wait(_det_worker_steps, (_port(), 140), timeout=600)
    assert status == "ok", status
    print(f"det one-rank sharded vs single GPU, 140 steps: equal {out['equal']}, max |diff| {out['maxdiff']}, "
          f"norms {out['norm']}, fc {out['fc']}")
    assert out["fc"]
    assert max(out["norm"]) < 10.0, out["norm"]
    l0, l1 = out["losses"]
    assert l0 == l1
    assert all(out["equal"].values()), (out["equal"], out["maxdiff"])


def _ab_worker(port, dtype, q):
    import argparse
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, store=dist.HashStore())
    try:
        import bench
        args = argparse.Namespace(dim=128, batch=1024, rows_per_gpu=60000, dtype=dtype, zipf=0.0, bn="local")
        q.put(("ok", bench.native_ab(args, 1, 0, dev)))
    except Exception as e:
        q.put((repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_bench_native_ab_one_rank(hip_device, dtype):
    """bench.py's A/B of the two collective paths (native_ab) as a one-rank RCCL job: native RCCL +
    step programs (calibration, recording pass, replay passes, the watchdog armed) against
    torch.distributed's eager steps, deterministic: validated -- every loss and the final table,
    moments and dense state bitwise equal -- with the native run really in programs over the
    fixed-capacity exchange."""
    status, ab = spawn_and_wait(_ab_worker, (_port(), dtype,), timeout=300)
    assert status == "ok", status
    print(f"native_ab[{dtype}]: {ab}")
    assert ab["native_healthy"] and not ab["watchdog_fired"], ab
    assert ab["native"]["programs"] == ab["batches"] and ab["native"]["fc_active"], ab
    assert ab["native"]["collectives"] == "native" and ab["torch"]["collectives"] == "torch", ab
    assert ab["validated"] and ab["first_diff_step"] == -1, ab


def _ring_worker(port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FBN_NATIVE_COMM="1")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, store=dist.HashStore())
    try:
        from ctr_recommendation_amd import trainer as trmod
        from ctr_recommendation_amd.data import make_batch
        from oracle.fibinet_oracle import build_model
        V, B, steps = 60000, 1024, 10
        cfg = {"embedding_dim": 128, "vocab_size": V, "honour_config": True, "net_dropout": 0.0,
               "compute_dtype": "bf16"}
        torch.manual_seed(0)
        init = build_model(None, cfg, honour_config=True).state_dict()
        bs = [make_batch(300 + s, B, V, device=dev) for s in range(steps + 1)]
        res = []
        for ring16 in (True, False):
            trmod._RING_BF16 = ring16
            tr = trmod.FiBiNETTrainer(cfg, total_steps=20, batch_size=B, device=dev, deterministic=True,
                                      init_state={k: v.clone() for k, v in init.items()}, shard=True)
            assert tr.ring_bf16 == ring16 and tr.ring.dtype == (torch.bfloat16 if ring16 else torch.float32)
            losses = [tr.step(bs[s][0], bs[s][1], next_batch=bs[s + 1][0]).item() for s in range(steps)]
            tr.flush()
            tr.check_ids()
            res.append((losses, {n: getattr(tr, n).cpu().clone() for n in ("E", "Em", "Ev", "flat_p", "flat_m")},
                        tr.xchg.fc_active))
            tr.close()
        (l0, t0, f0), (l1, t1, f1) = res
        q.put(("ok", {"losses": (l0, l1), "fc": (f0, f1), "equal": {k: bool(torch.equal(t0[k], t1[k])) for k in t0}}))
    except Exception as e:
        q.put((repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def test_bf16_ring_bit_identical_to_f32_ring(hip_device):
    """bf16 mode, sharded: the owner's deferred-gradient ring in bf16 (the wire's gradient rows kept as
    they arrived; widened on every read) against the f32 ring (widened once on arrival) -- the same
    f32 values reach every Adam step, so losses and the final table, moments and dense state are
    bitwise equal (deterministic mode, through the calibration steps' host-split exchange and the
    fixed-capacity form)."""
    status, out = spawn_and_wait(_ring_worker, (_port(),), timeout=300)
    assert status == "ok", status
    assert all(out["fc"]), out["fc"]
    l0, l1 = out["losses"]
    assert l0 == l1, (l0, l1)
    assert all(out["equal"].values()), out["equal"]
