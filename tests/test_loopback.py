"""The engine's multi-rank code path (one shard per rank, DESIGN.md section
7) executed on one GPU: W loopback ranks (psim_loopback_comm_id, the test
vehicle of partisan_amd/csrc/psim_comm.h -- device copies and a host barrier
where RCCL ranks use ncclAllToAll / grouped ncclSend-ncclRecv / ncclAllReduce
/ ncclAllGather) against the CPU oracle, bit for bit: the owner partition and
its offsets, the count all-to-all and its one host read, the record exchange
with the self-copy, the receive grouping, the stats all-reduce, the leave/1
stop-list all-gather and the overlay statistics' gathers.  RCCL itself stays
the only product backend (bench.py --gpus N)."""
import numpy as np
import pytest

import _scenarios as S
from _loopback import LoopbackRanks
from _oracle import Oracle

pytestmark = pytest.mark.gpu


def _ranks(world):
    return lambda cfg: LoopbackRanks(cfg, world)


@pytest.mark.parametrize("world", [2, 4])
def test_loopback_churn_partition_parity(world):
    """churn (20 %, restarts and rejoins) + a half/half partition + a
    broadcast every 10 rounds, 2048 nodes; then the overlay statistics."""
    gs, gst = S.churn_partition(_ranks(world), n=2048)
    os_, ost = S.churn_partition(Oracle, n=2048)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    gh, oh = gs.histograms(), os_.histograms()
    for k in oh:
        assert np.array_equal(np.asarray(gh[k]), np.asarray(oh[k])), k
    have, rnd, hop = gs.delivery()
    ohave, ornd, ohop = os_.delivery()
    assert np.array_equal(have, ohave) and np.array_equal(hop, ohop)
    gs.close()


@pytest.mark.parametrize("world", [2, 3])
def test_loopback_multistep_parity(world):
    """rounds several at a time: batches of fixed-size exchanges on every
    rank, stopping together at the round any rank overflowed"""
    gs, gst = S.multistep(_ranks(world))
    os_, ost = S.multistep(Oracle)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    gs.close()


def test_loopback_e_miniature_parity():
    """bench.py's sharding-check schedule (config E in miniature, 2^14 nodes)
    over 3 ranks: uneven shards (2^14 / 3)."""
    gs, gst = S.e_miniature(_ranks(3))
    os_, ost = S.e_miniature(Oracle)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    gs.close()


@pytest.mark.parametrize("strategy,world", [(1, 2), (2, 2), (2, 4)])
def test_loopback_remote_leave_parity(strategy, world):
    """leave/1 (psim_leave_node) on SCAMP v1 / v2 handles: a stop reported by
    the target's rank reaches every rank through the stop-list all-gather
    (padded to the longest list), the next round's crash events."""
    o, ost, actors, targets = S.pl_leave_remote(Oracle, 1024, 7, 80, strategy)
    g, gst = S.pl_leave_fixed(_ranks(world), 1024, 7, 80, strategy, 40, actors, targets)
    assert int(ost["nodes_up"][-1]) < int(ost["nodes_up"][39])      # someone stopped
    S.compare_stats(gst, ost)
    S.compare_nodes(g.strategy_nodes(), o.strategy_nodes())
    g.close()


def test_loopback_bucket_table_parity():
    """the sets v1 bucket table (App. A Q1) on every rank, 2 ranks"""
    gs, gst = S.churn_partition(S.with_buckets(_ranks(2), 21), n=1024, rounds=100)
    os_, ost = S.churn_partition(S.with_buckets(Oracle, 21), n=1024, rounds=100)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    gs.close()
