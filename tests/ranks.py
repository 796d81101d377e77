"""Multi-process test harness (gloo ranks on the CPU, or ranks sharing the test box's GPU).

run_ranks spawns one process per rank as target(rank, world, port, *args, queue). Each rank puts one
item on the queue, and run_ranks returns the items in arrival order. Every child is joined and must
exit with status 0. The cleanup runs on every path: a child still alive after a timeout or a failed
assertion is terminated through its own handle, and the queue's feeder thread is closed. So no rank
and no thread outlives the test, and none is alive at interpreter exit.
"""
import socket

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_ranks(target, world, args=(), timeout=300, join_timeout=120):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    try:
        for p in procs:
            p.start()
        items = [q.get(timeout=timeout) for _ in range(world)]
        for p in procs:
            p.join(timeout=join_timeout)
            assert p.exitcode == 0, f"a rank exited with status {p.exitcode}"
        return items
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
        q.close()
        q.join_thread()
