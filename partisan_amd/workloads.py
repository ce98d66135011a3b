"""Synthetic workloads for BASELINE.json configs A-E.

Every schedule is a pure function of (N, seed) drawn from numpy's PCG64, so the
GPU engine and the CPU oracle receive identical event streams.
"""
import numpy as np

NONE = 0xFFFFFFFF


def _rng(seed, salt):
    return np.random.Generator(np.random.PCG64([int(seed) & 0xFFFFFFFFFFFFFFFF, salt]))


def sequential_join(n_nodes):
    """Config A topology (test/partisan_SUITE.erl:1591-1601, partisan_support
    :377-388): node 0 is the server, node i joins node 0 at round i."""
    sched = [(0, np.array([0], np.uint32), np.array([NONE], np.uint32))]
    for i in range(1, n_nodes):
        sched.append((i, np.array([i], np.uint32), np.array([0], np.uint32)))
    return sched


MAX_JOINS_PER_ROUND = 1 << 23


def doubling_join(n_nodes, seed, max_per_round=MAX_JOINS_PER_ROUND):
    """Bootstrap ramp for large overlays: round 0 starts node 0; round r >= 1
    starts ids [2^(r-1), 2^r) and each joins a uniformly drawn node among the
    ids started earlier (so every live node receives ~1 JOIN per round).
    Past max_per_round joiners a round the ramp goes on linearly (overlays
    above 2^24 nodes: the JOIN flood of one doubling round -- ~9 records per
    joiner -- would not fit one GPU's route buffers next to 2^26 nodes)."""
    rng = _rng(seed, 1)
    sched = [(0, np.array([0], np.uint32), np.array([NONE], np.uint32))]
    lo, r = 1, 1
    while lo < n_nodes:
        hi = min(2 * lo, lo + max_per_round, n_nodes)
        ids = np.arange(lo, hi, dtype=np.uint32)
        contacts = rng.integers(0, lo, size=hi - lo, dtype=np.uint64).astype(np.uint32)
        sched.append((r, ids, contacts))
        lo, r = hi, r + 1
    return sched


SURVEY_RAMP = 64


def survey_join(n_nodes, seed, ramp=SURVEY_RAMP):
    """Config C's bootstrap as SURVEY.md section 8(d) defines it: node i
    joins at round floor(ramp * i / N) a uniformly drawn already-joined
    node: one among those started in an earlier round.  Round 0 has no
    earlier round: node 0 is the seed and node i of round 0's batch joins a
    uniformly drawn node of [0, i) (all started in round 0, up when the JOIN
    arrives) -- a random recursive tree (~ln(N/ramp) JOINs at node 0) rather
    than a star of N/ramp JOINs at node 0, which would overrun node 0's
    disconnect-id maps and connection table (the caps) on the
    first round.  Start rounds -- and so the shuffle and promotion timer
    phases -- spread evenly over the ramp, unlike the doubling ramp, which
    starts half the overlay in its last round."""
    rng = _rng(seed, 3)
    ids = np.arange(n_nodes, dtype=np.uint64)
    rnd = (ids * ramp // n_nodes).astype(np.int64)
    sched = [(0, np.array([0], np.uint32), np.array([NONE], np.uint32))]
    for r in range(ramp):
        lo = int(np.searchsorted(rnd, r, "left"))
        hi = int(np.searchsorted(rnd, r, "right"))
        if r == 0:
            lo = 1
        if hi <= lo:
            continue
        batch = np.arange(lo, hi, dtype=np.uint32)
        first = int(np.searchsorted(rnd, r, "left"))
        if r == 0:                            # node i: uniform over [0, i)
            contacts = np.floor(rng.random(hi - lo) * batch).astype(np.uint32)
        else:
            contacts = rng.integers(0, first, size=hi - lo, dtype=np.uint64).astype(np.uint32)
        sched.append((r, batch, contacts))
    return sched


def star_join(n_nodes, at_round=1):
    """Hot-spot case: every node joins node 0 in the same round."""
    ids = np.arange(1, n_nodes, dtype=np.uint32)
    return [(0, np.array([0], np.uint32), np.array([NONE], np.uint32)),
            (at_round, ids, np.zeros(n_nodes - 1, np.uint32))]


def churn_schedule(n_nodes, seed, frac, first_round, n_rounds, protect=(0,)):
    """Config E churn: frac*N crashes spread uniformly over n_rounds starting
    at first_round; each crashed node restarts the next round and rejoins a
    uniformly drawn node that is up when the JOIN is sent and when it arrives
    (crashes "replaced by as many fresh joins"): not
    one of the restarting nodes, nor one crashing in the round the JOIN is
    sent (k + 1) or delivered (k + 2) -- a JOIN that meets a crashed contact
    is dropped and HyParView never retries it (hv:500-515), which left each
    such rejoiner isolated until round 4.  The contacts of round k's victims
    are used at round k + 1."""
    rng = _rng(seed, 2)
    total = int(frac * n_nodes)
    cand = np.setdiff1d(np.arange(n_nodes, dtype=np.uint32), np.array(protect, np.uint32))
    victims = rng.choice(cand, size=min(total, cand.size), replace=False).astype(np.uint32)
    per = np.array_split(victims, n_rounds)
    out = []
    for k, v in enumerate(per):
        down = np.concatenate([v] + [per[j] for j in (k + 1, k + 2) if j < len(per)])
        contacts = rng.integers(0, n_nodes, size=v.size, dtype=np.uint64).astype(np.uint32)
        bad = np.isin(contacts, down)
        while bad.any():                      # redraw (uniform over the nodes up)
            contacts[bad] = rng.integers(0, n_nodes, size=int(bad.sum()), dtype=np.uint64).astype(np.uint32)
            bad = np.isin(contacts, down)
        out.append((first_round + k, v, contacts))
    return out


def half_partition(n_nodes):
    g = np.zeros(n_nodes, np.uint8)
    g[n_nodes // 2:] = 1
    return g


class BenchSchedule:
    """The event schedule of bench.py's config C and E lines -- one source for
    the bench, the bench-scale parity fixtures (tests/golden/gen_bench_fixtures.py)
    and their GPU test.

    C, schedule "survey" (SURVEY.md 8(d)): survey_join's 64-round ramp and
    SURVEY_WARM warm-up rounds, then `warmup` rounds, then the timed window,
    whose first round carries the one broadcast from node 0.
    C / E, schedule "doubling": doubling_join, `settle` rounds, STEADY_ROUNDS
    untimed broadcast rounds, `warmup` rounds, the window; a broadcast from
    node 0 every BCAST_PERIOD rounds throughout.  E adds 0.2 N crashes over
    100 rounds from STEADY_ROUNDS (each victim restarts and rejoins the next
    round) and the half/half partition for rounds 20-39 of the window: in the
    middle of the churn (round 3's E line).
    E, schedule "survey": the same bootstrap, broadcasts and churn, and the
    partition where SURVEY 8(d) E puts it -- 20 rounds from phase round
    E_PARTITION (150), ten rounds after the last churn rejoin (round 140),
    whatever the window.
    Phase-round i counts from the end of the bootstrap; the window starts at
    i = t_start."""
    STEADY_ROUNDS = 40
    BCAST_PERIOD = 10
    SURVEY_WARM = 100
    E_PARTITION = 150

    def __init__(self, workload, schedule, n, seed, warmup, settle=60):
        self.workload, self.n, self.seed = workload, n, seed
        self.survey = workload == "C" and schedule == "survey"
        self.settle = settle
        self.t_start = warmup if self.survey else self.STEADY_ROUNDS + warmup
        self.k = 0
        self.last_bcast = None
        self.churn = {}
        if workload == "E":
            for r, v, c in churn_schedule(n, seed, 0.2, self.STEADY_ROUNDS, 100):
                self.churn[r] = (v, c)
            self.part = half_partition(n)
            if schedule == "survey":
                self.p_on, self.p_off = self.E_PARTITION, self.E_PARTITION + 20
            else:
                self.p_on, self.p_off = self.t_start + 20, self.t_start + 40

    def bootstrap(self):
        """(join schedule, the round run_schedule runs to)"""
        if self.survey:
            return survey_join(self.n, self.seed), SURVEY_RAMP + self.SURVEY_WARM
        boot = doubling_join(self.n, self.seed)
        return boot, boot[-1][0] + 1 + self.settle

    def bcast_round(self, i):
        return i == self.t_start if self.survey else i % self.BCAST_PERIOD == 0

    def has_events(self, i):
        return self.bcast_round(i) or (self.workload == "E" and (i in self.churn or i - 1 in self.churn or
                                                                 i in (self.p_on, self.p_off)))

    def apply(self, sim, i):
        """the events of phase-round i, before it runs"""
        if self.bcast_round(i):
            sim.broadcast(0, self.k % 0x10000)
            self.k += 1
            self.last_bcast = i
        if self.workload == "E":
            if i in self.churn:
                sim.crash(self.churn[i][0])
            if i - 1 in self.churn:
                sim.join(self.churn[i - 1][0], self.churn[i - 1][1])
            if i == self.p_on:
                sim.set_partition(self.part)
            if i == self.p_off:
                sim.clear_partition()
