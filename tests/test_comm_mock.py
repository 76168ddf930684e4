"""The native RCCL communicators (csrc/comm.cpp, exchange.NativeComm) at world > 1, on CPU.

RCCL refuses two ranks on one device and no multi-GPU box is available, so the world > 1
bookkeeping of fbn_comm_alltoallv / fbn_comm_alltoall / fbn_comm_allreduce -- per-peer send and
receive offsets, zero and uneven counts, row sizes -- is exercised against a host-memory stand-in
for the RCCL entry points (tests/mock_rccl.cpp, built here with g++): the ranks are threads of one
child process, the buffers host memory, the streams ignored.  What this cannot show (real xGMI
transport, two communicators' kernels running side by side) is left to a multi-GPU run.
"""
import os
import subprocess
import sys
import textwrap

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

CHILD = textwrap.dedent(r'''
import ctypes, sys, threading
import numpy as np
sys.path.insert(0, sys.argv[2])
from ctr_recommendation_amd import _lib
lib = _lib.lib()
assert lib.fbn_comm_load(sys.argv[1].encode()) == 0, lib.fbn_last_error()
nid = lib.fbn_comm_id_bytes()
errors = []

def run(world, seed):
    uid = (ctypes.c_char * nid)()
    assert lib.fbn_comm_unique_id(uid) == 0
    rng = np.random.default_rng(seed)
    row = 12                                                    # bytes per row (3 x f32)
    counts = rng.integers(0, 5, size=(world, world))            # counts[src][dst] rows, zeros included
    counts[0, :] = 0                                            # rank 0 sends nothing
    counts[:, world - 1] = 0                                    # the last rank receives nothing
    counts[1 % world, 0] = 7
    send = [np.arange(counts[r].sum() * 3, dtype=np.float32) + 1000 * r for r in range(world)]
    recv = [np.full(counts[:, r].sum() * 3 + 3, -1.0, dtype=np.float32) for r in range(world)]
    eq = [np.arange(world * 5, dtype=np.int32) + 100 * r for r in range(world)]
    eq_out = [np.zeros(world * 5, dtype=np.int32) for r in range(world)]
    ar32 = [np.full(6, r + 1.5, dtype=np.float32) for r in range(world)]
    ar64 = [np.full(4, (r + 1) * 0.25, dtype=np.float64) for r in range(world)]
    ari = [np.arange(5, dtype=np.int32) * (r + 1) for r in range(world)]
    pe_out = [np.full(world * 5, -7, dtype=np.int32) for r in range(world)]   # peers-only: own block untouched
    ag_out = [np.full(world * 3, -1.0, dtype=np.float64) for r in range(world)]   # all-gather, rank order

    def rank(r):
        try:
            h = ctypes.c_void_p()
            assert lib.fbn_comm_init(ctypes.byref(h), uid, world, r) == 0
            sc = (ctypes.c_int * world)(*[int(x) for x in counts[r]])
            rc = (ctypes.c_int * world)(*[int(x) for x in counts[:, r]])
            rc_ = lib.fbn_comm_alltoallv(h, send[r].ctypes.data_as(ctypes.c_void_p), sc,
                                         recv[r].ctypes.data_as(ctypes.c_void_p), rc, ctypes.c_longlong(row), None)
            assert rc_ == 0, lib.fbn_last_error()
            rc_ = lib.fbn_comm_alltoall(h, eq[r].ctypes.data_as(ctypes.c_void_p),
                                        eq_out[r].ctypes.data_as(ctypes.c_void_p), ctypes.c_longlong(5 * 4), None)
            assert rc_ == 0, lib.fbn_last_error()
            rc_ = lib.fbn_comm_alltoall_peers(h, eq[r].ctypes.data_as(ctypes.c_void_p),
                                              pe_out[r].ctypes.data_as(ctypes.c_void_p), ctypes.c_longlong(5 * 4), None)
            assert rc_ == 0, lib.fbn_last_error()
            rc_ = lib.fbn_comm_allgather(h, ar64[r].ctypes.data_as(ctypes.c_void_p),
                                         ag_out[r].ctypes.data_as(ctypes.c_void_p), ctypes.c_longlong(3 * 8), None)
            assert rc_ == 0, lib.fbn_last_error()
            for buf, code in ((ar32[r], 0), (ar64[r], 1), (ari[r], 2)):
                rc_ = lib.fbn_comm_allreduce(h, buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_longlong(buf.size),
                                             code, None)
                assert rc_ == 0, lib.fbn_last_error()
            assert lib.fbn_comm_destroy(h) == 0
        except Exception as e:
            errors.append(repr(e))
    ts = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join(60) for t in ts]
    assert not errors, errors
    for r in range(world):
        # rank r receives, in source-rank order, counts[src][r] rows from each source, taken at the
        # source's send offset of destination r
        want = []
        for src in range(world):
            off = int(counts[src, :r].sum()) * 3
            want.append(send[src][off:off + int(counts[src, r]) * 3])
        want = np.concatenate(want) if want else np.zeros(0, np.float32)
        got = recv[r]
        assert np.array_equal(got[:want.size], want), (world, r, got, want)
        assert np.all(got[want.size:] == -1.0)                  # nothing written past the received rows
        assert np.array_equal(eq_out[r], np.concatenate([eq[s][5 * r:5 * r + 5] for s in range(world)]))
        want_pe = np.concatenate([eq[s][5 * r:5 * r + 5] if s != r else np.full(5, -7, np.int32) for s in range(world)])
        assert np.array_equal(pe_out[r], want_pe), (world, r, pe_out[r], want_pe)
        assert np.array_equal(ag_out[r], np.concatenate([np.full(3, (q + 1) * 0.25) for q in range(world)]))
        assert np.allclose(ar32[r], sum(q + 1.5 for q in range(world)))
        assert np.allclose(ar64[r], sum((q + 1) * 0.25 for q in range(world)))
        assert np.array_equal(ari[r], np.arange(5) * sum(q + 1 for q in range(world)))

for world, seed in ((2, 0), (3, 1), (4, 2), (8, 3)):
    run(world, seed)
print("ok")
''')


def test_native_comm_multi_rank_bookkeeping(tmp_path):
    so = str(tmp_path / "libmock_rccl.so")
    r = subprocess.run(["g++", "-O1", "-shared", "-fPIC", "-std=c++17", "-o", so, os.path.join(HERE, "mock_rccl.cpp"),
                        "-lpthread"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    # a child process: fbn_comm_load binds one RCCL per process, the mock here
    p = subprocess.run([sys.executable, str(script), so, os.path.dirname(HERE)], capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), (p.stdout[-2000:], p.stderr[-3000:])


WATCHDOG_CHILD = textwrap.dedent(r"""
import ctypes, sys, threading, time
import numpy as np
sys.path.insert(0, sys.argv[2])
from ctr_recommendation_amd import _lib
lib = _lib.lib()
assert lib.fbn_comm_load(sys.argv[1].encode()) == 0, lib.fbn_last_error()
uid = (ctypes.c_char * lib.fbn_comm_id_bytes())()
assert lib.fbn_comm_unique_id(uid) == 0
world = 3
hs = [ctypes.c_void_p() for _ in range(world)]
for r in range(world):
    assert lib.fbn_comm_init(ctypes.byref(hs[r]), uid, world, r) == 0
assert lib.fbn_comm_watchdog_fired(None) == 0
assert lib.fbn_comm_watch(ctypes.c_longlong(700)) == 0
assert lib.fbn_comm_heartbeat(None) == 0          # a step began (no stream: the beat alone)
res = {}
eq = [np.arange(world * 4, dtype=np.int32) for _ in range(world)]
out = [np.zeros(world * 4, dtype=np.int32) for _ in range(world)]

def rank(r):
    # rank 2 never posts: ranks 0 and 1 wait for its blocks
    t0 = time.perf_counter()
    rc = lib.fbn_comm_alltoall_peers(hs[r], eq[r].ctypes.data_as(ctypes.c_void_p), out[r].ctypes.data_as(ctypes.c_void_p),
                                     ctypes.c_longlong(16), None)
    res[r] = (rc, time.perf_counter() - t0, lib.fbn_last_error().decode())

ts = [threading.Thread(target=rank, args=(r,)) for r in (0, 1)]
[t.start() for t in ts]
[t.join(30) for t in ts]
for r in (0, 1):
    rc, dt, msg = res[r]
    assert rc != 0 and dt < 10.0, (r, rc, dt, msg)       # released by the watchdog, not the mock's 20 s
    assert "watchdog" in msg, msg
assert lib.fbn_comm_watchdog_fired(None) == 1
assert all(lib.fbn_comm_watchdog_fired(h) == 1 for h in hs)
# every later call fails at once with the watchdog's message
rc = lib.fbn_comm_allreduce(hs[2], eq[2].ctypes.data_as(ctypes.c_void_p), ctypes.c_longlong(4), 2, None)
assert rc == 3 and "aborted by the watchdog" in lib.fbn_last_error().decode(), lib.fbn_last_error()
for h in hs:
    assert lib.fbn_comm_destroy(h) == 0
print("ok")
""")


def test_native_comm_watchdog_aborts_a_hung_exchange(tmp_path):
    """The watchdog of the native communicators (they bypass torch's collective timeout):
    three ranks, rank 2 never posts its all-to-all blocks; ranks 0 and 1 block in the exchange.  With
    fbn_comm_watch(700 ms) and a heartbeat at the step's start, the monitor aborts every communicator
    after ~0.7 s: both blocked calls return an error naming the watchdog (well before the stand-in's own
    20 s receive timeout), fbn_comm_watchdog_fired reports it, and any later call fails at once."""
    so = str(tmp_path / "libmock_rccl.so")
    r = subprocess.run(["g++", "-O1", "-shared", "-fPIC", "-std=c++17", "-o", so, os.path.join(HERE, "mock_rccl.cpp"),
                        "-lpthread"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    script = tmp_path / "watch.py"
    script.write_text(WATCHDOG_CHILD)
    p = subprocess.run([sys.executable, str(script), so, os.path.dirname(HERE)], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), (p.stdout[-2000:], p.stderr[-3000:])
