"""SCAMP v1 memberships past 80 ids on the GPU: the
OTP sets v1 linear-hash order (sv1:45-279) driven by a
random 32-bit erlang:phash(NodeSpec, 2^32) table (psim_set_phash_table),
GPU == oracle bit for bit -- every round's stats and digest, node 0's view
size and active slot count every round (expansions to 22 slots, the
contractions back to 16 under leave/1's sets:del_element/2), every node's
strategy row at the end.  The oracle's set order is pinned against a
bucket-level model of stdlib sets.erl by tests/test_sets_v1.py."""
import pytest

import _scenarios as S
from _oracle import Oracle

pytestmark = pytest.mark.gpu


def _gpu(cfg):
    from partisan_amd import Simulator
    return Simulator(cfg)


def _vshards(g):
    def mk(cfg):
        from partisan_amd import Simulator
        c = type(cfg).from_buffer_copy(cfg)
        c.n_shards = g
        return Simulator(c)
    return mk


def _loop(world):
    def mk(cfg):
        from _loopback import LoopbackRanks
        return LoopbackRanks(cfg, world)
    return mk


@pytest.mark.parametrize("make,n,per_round", [(_gpu, 180, 20), (_gpu, 200, 10), (_vshards(3), 180, 20),
                                              (_loop(2), 180, 20)],
                         ids=["gpu-180", "gpu-200", "3-shards", "loopback-2"])
def test_scamp_v1_large_view_parity(make, n, per_round):
    o, ost, otr = S.pl_v1_large_view(S.with_phash(Oracle, 3), n=n, per_round=per_round)
    g, gst, gtr = S.pl_v1_large_view(S.with_phash(make, 3), n=n, per_round=per_round)
    assert max(x[0] for x in otr) > 100 and max(x[1] for x in otr) >= 22     # past 80: expanded
    assert otr[-1][1] <= 17 and int(ost["overflow"].sum()) == 0              # contracted again
    S.compare_stats(gst, ost)
    assert gtr == otr
    S.compare_nodes(g.strategy_nodes(), o.strategy_nodes())
    g.close()
