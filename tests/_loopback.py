"""W loopback ranks driven like one simulator (test infrastructure).

Each rank is a Simulator handle with shard_world = W and the same loopback
id (psim_loopback_comm_id, partisan_amd/csrc/psim_comm.h): the engine's
multi-rank code path -- owner partition, count all-to-all and its host read,
record exchange, stats all-reduce, leave/1 stop-list all-gather, overlay
gathers -- with device copies and a host barrier in place of RCCL, all on
one GPU.  Every rank gets the same event calls (as RCCL ranks do); the
collective calls (step, histograms) run on one thread per rank."""
import threading

import numpy as np

from partisan_amd.sim import _Driver, loopback_comm_id


class LoopbackRanks:
    def __init__(self, cfg, world, device=0):
        from partisan_amd import Simulator

        self.world, self.n = world, cfg.n_nodes
        self.cfg = cfg
        self.per = (cfg.n_nodes + world - 1) // world
        cid = loopback_comm_id()
        self.ranks = []
        for r in range(world):
            c = type(cfg).from_buffer_copy(cfg)
            c.shard_world, c.shard_rank, c.n_shards, c.device = world, r, 1, device
            self.ranks.append(Simulator(c, comm=cid))

    def _all(self, name, *a):
        out = [getattr(s, name)(*a) for s in self.ranks]
        return out[0]

    def _threads(self, name, *a):
        out, err = [None] * self.world, [None] * self.world

        def run(i):
            try:
                out[i] = getattr(self.ranks[i], name)(*a)
            except BaseException as e:      # (reported below, after every thread has ended)
                err[i] = e
        ts = [threading.Thread(target=run, args=(i,)) for i in range(self.world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=600)
        for e in err:
            if e is not None:
                raise e
        return out

    # ---- events: every rank makes the same call
    def join(self, nodes, contacts): self._all("join", nodes, contacts)
    def crash(self, nodes): self._all("crash", nodes)
    def revive(self, nodes): self._all("revive", nodes)
    def leave(self, nodes): self._all("leave", nodes)
    def leave_node(self, actors, targets): self._all("leave_node", actors, targets)
    def set_partition(self, group): self._all("set_partition", group)
    def clear_partition(self): self._all("clear_partition")
    def broadcast(self, root, msg_id): self._all("broadcast", root, msg_id)
    def set_bucket_table(self, buckets): self._all("set_bucket_table", buckets)
    def set_phash_table(self, phash): self._all("set_phash_table", phash)

    # ---- collectives: one thread per rank; every rank's stats are the
    # all-reduced ones
    def step(self, n_rounds=1):
        sts = self._threads("step", n_rounds)
        for st in sts[1:]:
            assert st.tobytes() == sts[0].tobytes(), "ranks disagree on the all-reduced stats"
        return sts[0]

    def histograms(self):
        hs = self._threads("histograms")
        for h in hs[1:]:
            assert all(np.array_equal(h[k], hs[0][k]) for k in h), "ranks disagree on the overlay statistics"
        return hs[0]

    @property
    def round(self):
        return self.ranks[0].round

    run_schedule = _Driver.run_schedule

    # ---- inspection: each rank answers for the ids it owns
    def _owned(self, name, first, count):
        count = self.n - first if count is None else count
        parts, at = [], first
        while at < first + count:
            r = at // self.per
            k = min(first + count, (r + 1) * self.per) - at
            parts.append(getattr(self.ranks[r], name)(at, k))
            at += k
        return parts

    def nodes(self, first=0, count=None):
        return np.concatenate(self._owned("nodes", first, count))

    def strategy_nodes(self, first=0, count=None):
        return np.concatenate(self._owned("strategy_nodes", first, count))

    def delivery(self, first=0, count=None):
        p = self._owned("delivery", first, count)
        return tuple(np.concatenate([x[i] for x in p]) for i in range(3))

    def close(self):
        for s in self.ranks:
            s.close()
