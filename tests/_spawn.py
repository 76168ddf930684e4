"""Test helper: run a worker in a spawned child process and wait for its (status, result) on a queue
without hanging when the child dies first (a failed process-group init, a crash): the wait polls the
child and fails at once with its exit code instead of blocking until the queue timeout."""
import queue
import time

import torch.multiprocessing as mp


def spawn_and_wait(target, args=(), timeout=300.0, nprocs=1, rank_args=False):
    """Start nprocs children running target(*args, q) (rank_args: target(rank, *args, q)); return the
    list of their queue items (one per child; a single item when nprocs == 1)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=((r,) if rank_args else ()) + tuple(args) + (q,)) for r in range(nprocs)]
    for p in procs:
        p.start()
    out, deadline = [], time.time() + timeout
    try:
        while len(out) < nprocs:
            try:
                out.append(q.get(timeout=5))
                continue
            except queue.Empty:
                pass
            dead = [p for p in procs if not p.is_alive() and p.exitcode not in (0, None)]
            if dead:
                raise AssertionError(f"child process exited with code {dead[0].exitcode} before reporting")
            if time.time() > deadline:
                raise AssertionError(f"no result from the child processes within {timeout} s")
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return out[0] if nprocs == 1 else out
