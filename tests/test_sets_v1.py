"""OTP `sets` v1 order past 80 elements: the oracle's
incremental restatement (oracle/psim_oracle.c set_add / set_del_slots: one
list in to_list order, re-slotted stably when the linear hash opens or
closes a slot) against a bucket-level model of stdlib's sets.erl written
here from its published algorithm -- #set{size, n, maxn, bso, exp_size,
con_size, segs}, get_slot/2, add_element/2 + maybe_expand/2 (rehash of the
buddy bucket), del_element/2 + maybe_contract/2 (B1 ++ B2), to_list/1 as the
fold over slots n..1.  No OTP is present here, so the model is a
restatement, not a pin: parity of this order with the reference is
unpinned.  The phash tables are random 32-bit values,
as erlang:phash(NodeSpec, 2^32) - 1 would be."""
import ctypes as C

import numpy as np
import pytest

import _oracle


class OtpSetsV1:
    """stdlib sets.erl (v1) over integer elements with hash table `ph`
    (ph[e] = erlang:phash(E, 2^32) - 1, so phash(E, R) = ph[e] mod R + 1)."""
    SEG, EXPAND, CONTRACT = 16, 5, 3

    def __init__(self, ph):
        self.ph = ph
        self.size, self.n, self.maxn, self.bso = 0, 16, 16, 8
        self.exp_size, self.con_size = 16 * 5, 16 * 3
        self.bkt = {i: [] for i in range(1, 17)}        # slot -> bucket, head = newest

    def phash(self, e, r):
        return int(self.ph[e]) % r + 1

    def get_slot(self, e):
        h = self.phash(e, self.maxn)
        return h - self.bso if h > self.n else h

    def add_element(self, e):
        b = self.bkt[self.get_slot(e)]
        ic = 0 if e in b else 1
        if ic:
            b.insert(0, e)
        self.maybe_expand(ic)

    def maybe_expand(self, ic):
        if self.size + ic > self.exp_size:
            if self.n == self.maxn:                     # maybe_expand_segs/1
                self.maxn, self.bso = 2 * self.maxn, 2 * self.bso
                for i in range(self.n + 1, self.maxn + 1):
                    self.bkt.setdefault(i, [])
            N = self.n + 1
            s1, s2 = N - self.bso, N
            b = self.bkt[s1]
            b1 = [e for e in b if self.phash(e, self.maxn) == s1]       # rehash/4, order kept
            b2 = [e for e in b if self.phash(e, self.maxn) == s2]
            assert len(b1) + len(b2) == len(b)
            self.bkt[s1], self.bkt[s2] = b1, b2
            self.size += ic
            self.n, self.exp_size, self.con_size = N, N * self.EXPAND, N * self.CONTRACT
        else:
            self.size += ic

    def del_element(self, e):
        b = self.bkt[self.get_slot(e)]
        dc = 1 if e in b else 0
        if dc:
            b.remove(e)
        self.maybe_contract(dc)

    def maybe_contract(self, dc):
        if self.size - dc < self.con_size and self.n > self.SEG:
            N = self.n
            s1, s2 = N - self.bso, N
            self.bkt[s1] = self.bkt[s1] + self.bkt[s2]          # put_bucket_s(Segs0, Slot1, B1 ++ B2)
            self.bkt[s2] = []
            n1 = N - 1
            self.size -= dc
            self.n, self.exp_size, self.con_size = n1, n1 * self.EXPAND, n1 * self.CONTRACT
            if self.n == self.bso:                              # maybe_contract_segs/1
                self.maxn, self.bso = self.maxn // 2, self.bso // 2
        else:
            self.size -= dc

    def to_list(self):
        out = []
        for s in range(self.n, 0, -1):          # fold: slot n..1, bucket head first, prepending
            for e in self.bkt[s]:
                out.insert(0, e)
        return out


def _oracle_run(ph, ops):
    lib = _oracle.load()
    f = lib.orc_sets_run
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                  C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    ph = np.ascontiguousarray(ph, np.uint32)
    ops = np.ascontiguousarray(ops, np.uint32)
    out = np.zeros(len(ops) + 1, np.uint32)
    k, slots = C.c_uint32(), C.c_uint32()
    rc = f(ph.ctypes.data, ph.size, ops.ctypes.data, ops.size, out.ctypes.data, out.size,
           C.byref(k), C.byref(slots))
    assert rc == 0
    return out[: k.value].tolist(), slots.value


def _model_run(ph, ops):
    s = OtpSetsV1(ph)
    for o in ops:
        o = int(o)
        if o >> 31:
            s.del_element(~o & 0xFFFFFFFF)
        else:
            s.add_element(o)
    return s.to_list(), s.n


def _ops(rng, n_elems, grow, shrink, rounds):
    """grow to `grow` elements, shrink to `shrink`, `rounds` times, with
    repeats (adds of members, deletes of non-members) mixed in"""
    ops, live = [], []
    for _ in range(rounds):
        while len(live) < grow:
            e = int(rng.integers(0, n_elems))
            ops.append(e)
            if e not in live:
                live.append(e)
        while len(live) > shrink:
            if rng.random() < 0.1:                      # a non-member: Dc = 0
                e = int(rng.integers(0, n_elems))
                if e not in live:
                    ops.append(~e & 0xFFFFFFFF)
                    continue
            e = live.pop(int(rng.integers(0, len(live))))
            ops.append(~e & 0xFFFFFFFF)
    return ops


@pytest.mark.parametrize("seed", range(6))
def test_sets_v1_order_past_80(seed):
    rng = np.random.Generator(np.random.PCG64([seed, 0x5E7]))
    n_elems = 4096
    ph = rng.integers(0, 1 << 32, n_elems, dtype=np.uint64).astype(np.uint32)
    # through the first expansions (81, 86, ... up to 128: 26 slots, MaxN 32),
    # the contractions back below 3 n, and again
    ops = _ops(rng, n_elems, 128, 40, 3)
    got, got_slots = _oracle_run(ph, ops)
    want, want_slots = _model_run(ph, ops)
    assert got_slots == want_slots
    assert got == want


def test_sets_v1_small_is_16_buckets():
    """<= 80 elements: 16 buckets (the engine's HyParView order)"""
    rng = np.random.Generator(np.random.PCG64([9, 0x5E7]))
    ph = rng.integers(0, 1 << 32, 512, dtype=np.uint64).astype(np.uint32)
    ops = _ops(rng, 512, 80, 10, 4)
    got, slots = _oracle_run(ph, ops)
    want, _ = _model_run(ph, ops)
    assert slots == 16 and got == want
    # bucket16 order: sorted by phash(E, 16), stable
    assert [int(ph[e]) & 15 for e in got] == sorted(int(ph[e]) & 15 for e in got)


def test_sets_v1_expansion_points():
    """n grows by one each time the size passes 5 n, MaxN doubles past 16
    slots; n shrinks below 3 n"""
    ph = (np.arange(1024, dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
    for size, slots in [(80, 16), (81, 17), (85, 17), (86, 18), (126, 26)]:
        _, s = _oracle_run(ph, list(range(size)))
        assert s == slots, (size, s)
    ops = list(range(81)) + [~i & 0xFFFFFFFF for i in range(31)]   # 50 left: < 3 * 17
    _, s = _oracle_run(ph, ops)
    assert s == 16
    ops = list(range(81)) + [~i & 0xFFFFFFFF for i in range(30)]   # 51 left
    _, s = _oracle_run(ph, ops)
    assert s == 17


def test_sets_v1_contract_merges_b1_then_b2():
    """A fixed expand-then-contract sequence worked by hand from sets.erl:
    a1, b1, a2, b2 share 16-slot bucket 1 (phash(E, 16) = 1); the 81st add
    opens slot 17 and rehash/4 moves b1, b2 there (phash(E, 32) = 17).  Then
    31 deletes take the size below 3 * 17: maybe_contract/2 stores slot 1 as
    B1 ++ B2 = [a2, a1] ++ [b2, b1] (buckets newest first), which to_list/1's
    reversing fold yields as b1, b2, a1, a2."""
    a1, b1, a2, b2 = 0, 1, 2, 3
    ph = np.zeros(128, np.uint32)
    ph[a1], ph[a2] = 0 + 32 * 5, 0 + 32 * 9            # low 5 bits 0: slot 1 at MaxN 16 and 32
    ph[b1], ph[b2] = 16 + 32 * 3, 16 + 32 * 7          # low 5 bits 16: slot 1, then slot 17
    fill = list(range(4, 81))
    for i in fill:
        ph[i] = (i % 15) + 1 + 32 * i                 # never bucket 1
    ops = [a1, b1, a2, b2] + fill
    got, slots = _oracle_run(ph, ops)
    assert slots == 17 and got[:2] == [a1, a2] and got[-2:] == [b1, b2]
    ops += [~i & 0xFFFFFFFF for i in fill[:31]]
    got, slots = _oracle_run(ph, ops)
    assert slots == 16
    assert got[:4] == [b1, b2, a1, a2]
    want, _ = _model_run(ph, ops)
    assert got == want
