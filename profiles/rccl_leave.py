"""Two RCCL ranks of a SCAMP v2 handle (two devices: RCCL refuses two ranks
on one, see rccl_pair.py) with leave/1 calls
whose actor and target sit on different ranks (the stop lists all-gathered
after the round, psim_engine.hip), against a one-shard run of the same
schedule: per-round stats and every node's strategy row, bit for bit.
Usage: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 profiles/rccl_leave.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import torch.distributed as dist

import _scenarios as S
from partisan_amd import Simulator
from partisan_amd.sim import comm_id

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
obj = [comm_id() if rank == 0 else None]
dist.broadcast_object_list(obj, src=0)


def ranked(cfg):
    cfg.device = 0
    cfg.shard_world, cfg.shard_rank = world, rank
    return Simulator(cfg, comm=obj[0])


n, seed, rounds, at = 4096, 21, 70, 40
# the pairs from the one-shard run (every rank computes the same ones)
ref, rst, actors, targets = S.pl_leave_remote(lambda c: Simulator(c), n, seed, rounds, strategy=2, leave_at=at, k=32)
per = (n + world - 1) // world
cross = int(np.sum(actors // per != targets // per))
assert cross > 0, "no actor/target pair spans two ranks"
gs, gst = S.pl_leave_fixed(ranked, n, seed, rounds, 2, at, actors, targets)
S.compare_stats(gst, rst)
lo = rank * per
c = min(per, n - lo)
S.compare_nodes(gs.strategy_nodes(lo, c), ref.strategy_nodes(lo, c))
up = int(rst["nodes_up"][-1])
assert up <= n - len(targets), up                 # the targets stopped
print(f"rank {rank}: RCCL {world}-rank leave/1 run == 1-shard run ({len(actors)} leaves, {cross} across ranks, "
      f"{up} nodes up at the end)", flush=True)
dist.destroy_process_group()
