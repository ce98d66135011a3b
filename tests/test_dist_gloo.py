"""The N>1 path on CPU: the node-range sharded round protocol (emit ->
exchange by owner shard -> merge) with 2 gloo ranks reproduces the
unsharded oracle exactly.  The GPU engine runs the same protocol (virtual
shards: tests/test_gpu_parity.py::test_shard_count_invariance; RCCL ranks:
bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    import torch.distributed as dist

    import _scenarios as S
    from _oracle import Oracle, ShardedOracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard, sst = S.churn_partition(lambda cfg: ShardedOracle(cfg), n=n, rounds=110)
        full, fst = S.churn_partition(Oracle, n=n, rounds=110)
        S.compare_stats(sst, fst)
        lo, hi = shard.lo, shard.hi
        S.compare_nodes(shard.nodes(lo, hi - lo), full.nodes(lo, hi - lo))
        q.put((rank, "ok"))
    except Exception as e:  # report, then fail in the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_protocol_matches_unsharded(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 1024, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res
