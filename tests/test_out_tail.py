"""The Plumtree outstanding table past one 64-lane register (PSIM_PT_OUT_CAP
128: entries 64.. live in the extension row's tail, psim_device.h OUT_HEAD)
on the CPU oracle: the out_tail scenario really fills tables past 64 (so the
GPU parity test in test_gpu_parity.py exercises the tail's add, ack,
neighbors_down and lazy-tick paths), with period=1 up to the cap, and every
table stays an orddict (sorted, unique keys, zeros past out_n)."""
import numpy as np

import _scenarios as S
from _oracle import Oracle
from partisan_amd import _abi

OVF_PT_OUT = 1


def _keys(v):
    return (v["pt_out_peer"].astype(np.uint64) << 32) | (v["pt_out_msg"].astype(np.uint64) << 16) \
        | (v["pt_out_round"].astype(np.uint64) & 0xFFFF)


def _check_tables(views):
    k = _keys(views)
    for i in np.nonzero(views["pt_out_n"] > 0)[0]:
        n = int(views["pt_out_n"][i])
        row = k[i]
        assert np.all(row[1:n] > row[:n - 1]), i
        assert not np.any(views["pt_out_peer"][i][n:]), i


def test_out_tail_fills_past_one_register():
    sim, st, snaps = S.out_tail(Oracle)
    assert _abi.PT_OUT_CAP == 128
    big = int(snaps[79]["pt_out_n"].max())
    assert 64 < big <= 128
    assert int((snaps[79]["pt_out_n"] > 64).sum()) >= 4
    assert int(st["overflow_by"][:, OVF_PT_OUT].sum()) == 0
    for v in snaps.values():
        _check_tables(v)
    # the heal acks the tables down again
    assert int(sim.nodes()["pt_out_n"].max()) < 16


def test_out_tail_at_cap_drops():
    sim, st, snaps = S.out_tail(Oracle, period=1, snap_at=(79,))
    assert int(snaps[79]["pt_out_n"].max()) == _abi.PT_OUT_CAP
    assert int(st["overflow_by"][:, OVF_PT_OUT].sum()) > 0
    _check_tables(snaps[79])

