"""World-size-2 rehearsal of bench.py's multi-GPU path on CPU (gloo).

bench.py shards queries across ranks with no data-path collective; the
only cross-rank traffic is the barrier and the (max time, sum of pops) reduction.  This
runs exactly those helpers in two gloo processes.
"""
import os
import socket
import sys
from pathlib import Path

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    ids = bench.shard_query_ids(rank, world, 5)
    elapsed = 1.0 + rank          # rank 1 is the slow one
    pops = 100 * (rank + 1)
    dist.barrier()
    t, p = bench.reduce_over_ranks(dist, elapsed, pops, "cpu")
    q.put((rank, ids, t, p))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_sharding_and_reduction():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    ids = [o[1] for o in out]
    assert ids[0] == list(range(0, 5)) and ids[1] == list(range(5, 10))   # disjoint, weak scaling
    for _, _, t, p in out:
        assert t == 2.0 and p == 300.0                                     # max time, total pops


def test_single_rank_identity():
    sys.path.insert(0, str(ROOT))
    import bench
    assert bench.reduce_over_ranks(None, 1.5, 7, "cpu") == (1.5, 7.0)
    assert bench.shard_query_ids(0, 1, 3) == [0, 1, 2]
