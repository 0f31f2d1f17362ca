"""The N>1 bench path (replicas: barrier + max-over-ranks timer, no data-path collective),
rehearsed with world_size-2 gloo on CPU."""
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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    import time

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    ws, r, local = bench.dist_env()
    assert (ws, r, local) == (world, rank, rank)
    barrier, reduce_max = bench.make_collectives(torch, dist, torch.device("cpu"))
    # rank 1 is slower: the reported time must be the max over ranks
    dt = bench.timed_region(lambda: time.sleep(0.05 + 0.1 * rank), barrier, lambda: None, reduce_max)
    q.put((rank, dt))
    dist.destroy_process_group()


def test_timed_region_reports_max_over_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res = dict(q.get() for _ in range(2))
    assert res[0] == res[1]            # every rank reports the same (max) time
    assert 0.15 <= res[0] < 1.0        # the slow rank's 0.15 s dominates


def test_single_process_collectives_are_identity():
    import bench

    barrier, reduce_max = bench.make_collectives(torch, None, torch.device("cpu"))
    barrier()
    assert reduce_max(1.5) == 1.5


def test_work_accounting():
    import bench

    assert bench.call_flops(1, 4, 1024, 1024) == 1073741824
    assert bench.call_bytes(1, 4, 1024, 1024) == 2097152
    assert bench.call_bytes(1, 4, 1024, 1024, out_bytes=4) == 2621440
