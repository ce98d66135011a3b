"""Two RCCL ranks of the simulator (diagnostic: the RCCL exchange path of
psim_engine.hip).  Needs two devices: RCCL 7.2 refuses two ranks on one
("Duplicate GPU detected", ncclInvalidUsage, measured on the one-GPU box),
so set HIP_VISIBLE_DEVICES per rank or run it on a node with two GPUs.
Compares the 2-rank run with a 1-shard run on the same device, bit for bit.
Usage: torchrun --nproc-per-node 2 profiles/rccl_pair.py"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")]
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


n = 4096
gs, gst = S.churn_partition(ranked, n=n, rounds=80)
ref, rst = S.churn_partition(lambda c: Simulator(c), n=n, rounds=80)
S.compare_stats(gst, rst)
per = (n + world - 1) // world
lo = rank * per
S.compare_nodes(gs.nodes(lo, min(per, n - lo)), ref.nodes(lo, min(per, n - lo)))
print(f"rank {rank}: RCCL {world}-rank run == 1-shard run, {int(gst['emitted'].sum())} msgs", flush=True)
dist.destroy_process_group()
