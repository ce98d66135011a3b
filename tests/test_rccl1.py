"""The RCCL rank path executed by the real library on one GPU (DESIGN.md
section 7): a handle with shard_world = 1 and a communicator id from
ncclGetUniqueId runs the multi-rank round -- the owner partition and its
offsets, ncclAllToAll of the per-owner counts, the records through a grouped
ncclSend / ncclRecv pair to itself, the device-side ncclAllReduce of the
round's stats on the shard's stream, the leave/1 stop list and the overlay
statistics through ncclAllGather / ncclAllReduce -- on RCCL's own stream
semantics (the loopback vehicle of tests/test_loopback.py synchronises around
every collective).  Each run is compared with the CPU oracle bit for bit.
Reference role: the TCP delivery these collectives replace
(src/partisan_peer_service_client.erl:210-226)."""
import numpy as np
import pytest

import _scenarios as S
from _oracle import Oracle

pytestmark = pytest.mark.gpu


def _rccl1(cfg):
    from partisan_amd import Simulator
    from partisan_amd.sim import comm_id

    c = type(cfg).from_buffer_copy(cfg)
    c.shard_world, c.shard_rank, c.n_shards = 1, 0, 1
    return Simulator(c, comm=comm_id())


def test_rccl1_churn_partition_parity():
    """churn (20 %, restarts and rejoins) + a half/half partition + a
    broadcast every 10 rounds, 2048 nodes; the overlay statistics (the
    in-degree all-reduce and the active-row all-gathers) and deliveries"""
    gs, gst = S.churn_partition(_rccl1, n=2048)
    os_, ost = S.churn_partition(Oracle, n=2048)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    gh, oh = gs.histograms(), os_.histograms()
    for k in oh:
        assert np.array_equal(np.asarray(gh[k]), np.asarray(oh[k])), k
    have, rnd, hop = gs.delivery()
    ohave, ornd, ohop = os_.delivery()
    assert np.array_equal(have, ohave) and np.array_equal(rnd, ornd) and np.array_equal(hop, ohop)
    gs.close()


def test_rccl1_multistep_parity():
    """rounds several at a time (the rank path's batches of fixed-size
    exchanges, run_batch_ranked), with the steps in traffic that overflow a
    batch's capacities and make it redo a round exactly"""
    gs, gst = S.multistep(_rccl1)
    os_, ost = S.multistep(Oracle)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    gs.close()


def test_rccl1_e_miniature_parity():
    """bench.py's sharding-check schedule (config E in miniature, 2^14 nodes)"""
    gs, gst = S.e_miniature(_rccl1)
    os_, ost = S.e_miniature(Oracle)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    gs.close()


@pytest.mark.parametrize("strategy", [1, 2])
def test_rccl1_remote_leave_parity(strategy):
    """leave/1 on SCAMP v1 / v2: the stop list goes through the two
    ncclAllGathers (counts, then the padded lists) before the next round"""
    o, ost, actors, targets = S.pl_leave_remote(Oracle, 1024, 7, 80, strategy)
    g, gst = S.pl_leave_fixed(_rccl1, 1024, 7, 80, strategy, 40, actors, targets)
    assert int(ost["nodes_up"][-1]) < int(ost["nodes_up"][39])      # someone stopped
    S.compare_stats(gst, ost)
    S.compare_nodes(g.strategy_nodes(), o.strategy_nodes())
    g.close()


def test_rccl1_full_strategy_parity():
    """the full strategy (payload arena, fanout 5) through the rank path"""
    g, gst = S.pl_doubling(_rccl1, 1024, 3, 60, 0, fanout=5, crash_at=30, part_at=40)
    o, ost = S.pl_doubling(Oracle, 1024, 3, 60, 0, fanout=5, crash_at=30, part_at=40)
    S.compare_stats(gst, ost)
    S.compare_strategy(g, o, full_bits=[0, 1, 17, 500, 1023])
    g.close()


def test_rccl1_bucket_table_parity():
    """a non-murmur view-order table through the rank path"""
    gs, gst = S.churn_partition(S.with_buckets(_rccl1, 21), n=1024, rounds=100)
    os_, ost = S.churn_partition(S.with_buckets(Oracle, 21), n=1024, rounds=100)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    gs.close()
