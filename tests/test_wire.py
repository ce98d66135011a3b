"""The wire format (psim_wire_encode / psim_wire_decode):
{packet, 4} frames around partisan_util:term_to_iolist/1 (util:235-297) of
the reference handlers' messages -- what the connection's send path writes
(peer_service_client:95, :130, :275).  Pinned three ways:
  * tests/_etf.py (an independent encoder of the published external term
    format, and of term_to_iolist's own rules above it) against known
    term_to_binary/1 outputs of OTP 19-22 and term_to_iolist outputs;
  * every message type's frame, byte for byte, against that encoder applied
    to the tuple the reference handler builds (cited per type);
  * decode(encode(r)) == r for each of them and over every record of real
    oracle runs (HyParView + Plumtree under churn and a partition, X-BOT).
Pure host code of the product library: no GPU needed."""
import numpy as np
import pytest

import _scenarios as S
from _etf import Atom as A
from _etf import packet4, term_to_binary, term_to_iolist
from _oracle import Oracle
from partisan_amd import wire

NM = wire.names(prefix="n", host="127.0.0.1", ip_base=(10 << 24), port=9090)
U = A("undefined")


def test_etf_known_answers():
    """term_to_binary/1 outputs of OTP 19-22 (erts external term format)."""
    assert term_to_binary(A("ok")) == bytes([131, 100, 0, 2, 111, 107])
    assert term_to_binary(1) == bytes([131, 97, 1])
    assert term_to_binary(256) == bytes([131, 98, 0, 0, 1, 0])
    assert term_to_binary(-1) == bytes([131, 98, 255, 255, 255, 255])
    assert term_to_binary((A("a"), 1)) == bytes([131, 104, 2, 100, 0, 1, 97, 97, 1])
    assert term_to_binary([]) == bytes([131, 106])
    assert term_to_binary([A("a")]) == bytes([131, 108, 0, 0, 0, 1, 100, 0, 1, 97, 106])
    assert term_to_binary([1, 2, 3]) == bytes([131, 107, 0, 3, 1, 2, 3])
    assert term_to_binary({A("a"): 1}) == bytes([131, 116, 0, 0, 0, 1, 100, 0, 1, 97, 97, 1])
    # flatmap keys in term order
    assert term_to_binary({A("b"): 2, A("a"): 1}) == term_to_binary({A("a"): 1, A("b"): 2})


def test_iolist_known_answers():
    """partisan_util:term_to_iolist/1 (util:235-297): small atoms above the
    maps, term_to_binary/1 inside them and for integers."""
    assert term_to_iolist(A("ok")) == bytes([131, 115, 2, 111, 107])
    assert term_to_iolist((A("a"), 1)) == bytes([131, 104, 2, 115, 1, 97, 97, 1])
    assert term_to_iolist([A("a")]) == bytes([131, 108, 0, 0, 0, 1, 115, 1, 97, 106])
    assert term_to_iolist([]) == bytes([131, 106])
    assert term_to_iolist([1, 2]) == bytes([131, 107, 0, 2, 1, 2])
    assert term_to_iolist(256) == term_to_binary(256)
    assert term_to_iolist({A("a"): [A("b")]}) == term_to_binary({A("a"): [A("b")]})
    assert term_to_iolist((A("x"), {A("a"): 1})) == bytes([131, 104, 2, 115, 1, 120]) + term_to_binary({A("a"): 1})[1:]


def name(i):
    return A(f"n{i}@127.0.0.1")


def spec(i):
    """partisan_peer_service_manager:myself/0 (:71-76) of node i"""
    ip = (10 << 24) + i
    return {A("name"): name(i), A("listen_addrs"): [{A("ip"): (ip >> 24, (ip >> 16) & 255, (ip >> 8) & 255, ip & 255),
                                                     A("port"): 9090}],
            A("channels"): [U], A("parallelism"): 1}


def rec(dst, src, t, ttl=0, a=(0, 0, 0, 0), ex=()):
    r = np.zeros(16, np.uint32)
    r[0], r[1], r[2] = dst, src, t | (ttl << 8) | (len(ex) << 16)
    r[4:8] = a
    r[8:8 + len(ex)] = ex
    return r


EX = (3, 17, 9)
M = 0x80000000
CASES = [
    # (record, the reference's term)
    (rec(1, 2, 0, a=(7, 0, 0, 0)), (A("join"), spec(2), U, 7)),                                   # hv:506-510
    (rec(1, 2, 1, ttl=4, a=(5, 3, 0, 0)), (A("forward_join"), spec(5), U, 3, 4, spec(2))),          # hv:906-910
    (rec(1, 2, 2, a=((1 << 20) | 3, 0, 0, 0)), (A("neighbor"), spec(2), U, (1, 3), spec(1))),      # hv:728-731
    (rec(1, 2, 3, a=((2 << 20) | 9, 0, 0, 0)), (A("disconnect"), spec(2), (2, 9))),                # hv:1493-1495
    (rec(1, 2, 4, a=(1 << 20, 0, 0, 0), ex=EX),
     (A("neighbor_request"), spec(2), A("high"), U, (1, 0), [spec(e) for e in EX])),               # hv:1700-1706
    (rec(1, 2, 5, a=((1 << 20) | 1, 0, 0, 0), ex=EX),
     (A("neighbor_accepted"), spec(2), U, (1, 1), [spec(e) for e in EX])),                         # hv:1008-1012
    (rec(1, 2, 6, ex=EX), (A("neighbor_rejected"), spec(2), [spec(e) for e in EX])),                # hv:1041-1043
    (rec(1, 2, 7, ttl=5, ex=EX), (A("shuffle"), [spec(e) for e in EX], 5, spec(2))),                # hv:594-597
    (rec(1, 2, 8, ex=EX), (A("shuffle_reply"), [spec(e) for e in EX], spec(2))),                    # hv:1127-1131
    (rec(1, 2, 8), (A("shuffle_reply"), [], spec(2))),
]
PT = A("partisan_plumtree_broadcast")
MOD = A("partisan_plumtree_backend")


def fwd(msg):
    # send/3 (pt:633-638) -> cast_message/3 wraps {'$gen_cast', Msg} (hv:147-154)
    # -> forward_message (hv:441-460)
    return (A("forward_message"), PT, (A("$gen_cast"), msg))


CASES += [
    (rec(1, 2, 9, a=(300, 4, 6 | M, 0)),
     fwd((A("broadcast"), (name(6), 300), (name(6), 300), MOD, 4, spec(6), spec(2)))),              # pt:398, :431
    (rec(1, 2, 10, a=(0, 0, 6 | M, 0)), fwd((A("prune"), spec(6), spec(2)))),                       # pt:372
    (rec(1, 2, 11, a=(5, 2, 6 | M, 0)), fwd((A("i_have"), (name(6), 5), MOD, 2, spec(6), spec(2)))),  # pt:453
    (rec(1, 2, 12, a=(5, 2, 6 | M, 0)), fwd((A("ignored_i_have"), (name(6), 5), MOD, 2, spec(6), spec(2)))),
    (rec(1, 2, 13, a=(5, 2, 6 | M, 0)), fwd((A("graft"), (name(6), 5), MOD, 2, spec(6), spec(2)))),
    (rec(1, 2, 10, a=(0, 0, 6, 0)), fwd((A("prune"), name(6), spec(2)))),                          # atom root (Q6)
]
NONE = 0xFFFFFFFF
CASES += [
    (rec(9, 5, 16, a=(4, 5, 9, NONE)), (A("optimization"), U, spec(4), spec(5), spec(9), U)),       # xbot:711
    (rec(5, 9, 17, ttl=1, a=(4, 5, 9, NONE)), (A("optimization_reply"), A("true"), spec(4), spec(5), spec(9), U)),
    (rec(7, 9, 18, a=(4, 5, 9, 7)), (A("replace"), U, spec(4), spec(5), spec(9), spec(7))),         # xbot:1221
    (rec(9, 7, 19, ttl=0, a=(4, 5, 9, 7)), (A("replace_reply"), A("false"), spec(4), spec(5), spec(9), spec(7))),
    (rec(4, 7, 20, a=(4, 5, 9, 7)), (A("switch"), U, spec(4), spec(5), spec(9), spec(7))),           # xbot:1264
    (rec(7, 4, 21, ttl=1, a=(4, 5, 9, 7)), (A("switch_reply"), A("true"), spec(4), spec(5), spec(9), spec(7))),
    (rec(5, 9, 17, ttl=1, a=(4, 5, 9, 7)), (A("optimization_reply"), A("true"), spec(4), spec(5), spec(9), spec(7))),
]


@pytest.mark.parametrize("k", range(len(CASES)))
def test_frame_matches_reference_term(k):
    r, term = CASES[k]
    assert wire.encode(r, NM) == packet4(term_to_iolist(term))


@pytest.mark.parametrize("k", range(len(CASES)))
def test_decode_inverts_encode(k):
    r, _ = CASES[k]
    got, used = wire.decode(wire.encode(r, NM), NM, int(r[0]))
    assert np.array_equal(got, r) and used == len(wire.encode(r, NM))


def test_stream_of_frames_and_partial_reads():
    frames = [wire.encode(r, NM) for r, _ in CASES]
    buf = b"".join(frames)
    out = []
    while buf:
        assert wire.decode(buf[:3], NM, 0) is None                # a length prefix not complete
        got = wire.decode(buf[:len(frames[len(out)]) - 1], NM, int(CASES[len(out)][0][0]))
        assert got is None                                         # a body not complete
        r, used = wire.decode(buf, NM, int(CASES[len(out)][0][0]))
        out.append(r)
        buf = buf[used:]
    assert all(np.array_equal(a, b) for a, (b, _) in zip(out, CASES))


def test_decoder_accepts_other_term_encodings():
    """binary_to_term/1 takes any form: UTF-8 / small atoms, INTEGER_EXT for a
    small integer -- so must the decoder (a newer OTP writes ATOM_UTF8_EXT;
    a plain term_to_binary/1 frame writes ATOM_EXT everywhere)."""
    r, term = CASES[3]
    b = term_to_binary(term)
    # every ATOM_EXT (100, len16) -> SMALL_ATOM_UTF8_EXT (119, len8)
    out, i = bytearray([131]), 1
    while i < len(b):
        t = b[i]
        if t == 100:
            n = (b[i + 1] << 8) | b[i + 2]
            out += bytes([119, n]) + b[i + 3:i + 3 + n]
            i += 3 + n
        elif t == 97:
            out += bytes([98, 0, 0, 0, b[i + 1]])
            i += 2
        elif t in (104,):
            out += b[i:i + 2]
            i += 2
        elif t in (108, 116):
            out += b[i:i + 5]
            i += 5
        else:
            out += b[i:i + 1]
            i += 1
    got, _ = wire.decode(packet4(bytes(out)), NM, 1)
    assert np.array_equal(got, r)


def test_rejects_unknown_terms():
    no_cast = (A("forward_message"), PT, (A("prune"), spec(6), spec(2)))          # (no gen_cast wrapper)
    for term in [A("ok"), (A("join"), spec(2), U), (A("hello"), name(1)), (A("neighbor"), spec(2), U, (1, 3), spec(5)),
                 no_cast]:
        with pytest.raises(wire.WireError):
            wire.decode(packet4(term_to_binary(term)), NM, 1)
    with pytest.raises(wire.WireError):
        wire.decode(packet4(bytes([130, 97, 1])), NM, 1)             # wrong version byte
    with pytest.raises(wire.WireError):
        wire.encode(rec(1, 2, 11, a=(5, 2, NONE, 0)), NM)             # IHAVE of a retired id: no root


def _outbox_round_trip(sim, rounds):
    n = 0
    for _ in range(rounds):
        sim.step(1)
        box = sim.inbox()                                             # [dst, src, seq, tt, a0..a3, ex]
        for m in box:
            r = np.zeros(16, np.uint32)
            r[0], r[1], r[2] = m[0], m[1], m[3]
            r[4:8], r[8:] = m[4:8], m[8:]
            if (r[2] & 0xFF) == 11 and r[6] == NONE:
                continue
            got, _ = wire.decode(wire.encode(r, NM), NM, int(r[0]))
            assert np.array_equal(got, r), (r, got)
            n += 1
    return n


def test_round_trip_real_traffic():
    sim, _ = S.churn_partition(Oracle, n=512, rounds=60)
    sim.broadcast(3, 77)
    assert _outbox_round_trip(sim, 8) > 1000


def test_round_trip_xbot_traffic():
    sim, _ = S.churn_partition(Oracle, n=512, rounds=60, manager=2, xbot_period=5)
    assert _outbox_round_trip(sim, 12) > 500
