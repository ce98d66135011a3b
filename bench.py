"""Benchmark: config C of BASELINE.json on MI355X.

A step is one BSP round of the hot path (HyParView handlers + timers,
Plumtree broadcast, message route) over every node of a 2^20-node overlay
per GPU.  The default schedule is SURVEY 8(d)'s: joins spread over a
64-round ramp, 100 warm-up rounds, --warmup rounds, then one broadcast from
node 0 at the first timed round, whose propagation the window measures
(--schedule doubling keeps round 2's line: doubling bootstrap, a broadcast
every 10 rounds).  Prints ONE JSON line (rank 0).  See DESIGN.md section 5.

  python bench.py                      1 GPU (config C)
  python bench.py --gpus N             N GPUs: N ranks are started here, one
                                       per GPU, node-range sharded over RCCL
  torchrun --nproc-per-node N bench.py --gpus N   the same, ranks by torchrun
  python bench.py --rank-path          1 GPU through the RCCL rank path (a
                                       one-rank communicator; diagnostic)

Every run first checks the sharded round against the one-shard engine on a
small churn + partition scenario (digest of every emitted record, every
round; node rows; overlay statistics): N RCCL ranks against one GPU, or, on
one GPU, two virtual shards against one.  A mismatch fails the run.
"""
import argparse
import contextlib
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BCAST_PERIOD = 10               # broadcast_heartbeat_interval cadence (rounds)
STEADY_ROUNDS = 40              # untimed broadcast rounds before the warmup (any --warmup)
OVERLAY_DRAIN = 40              # untimed rounds before the overlay statistics (at least)
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md)
S_NODE = 416                    # algorithmic state bytes per processed node
S_MSG = 64                      # message record bytes
CHECK_NODES = 1 << 14           # the built-in sharding check
CHECK_ROUNDS = 90
SCHEDULE_VERSION = 4            # bumps when the event schedule of a run changes (PMC keys)
OVF_KINDS = ("idmap", "pt_outstanding", "pt_sets_roots_msgs", "strategy", "conn")   # PSIM_OVF_*
ALG_FORMULA = ("B = N_run * 2 * 416 + M_in * 64 + M_out * 68 per round, N_run = nodes the phase kernels "
               "run (stats state_bytes / 832; nodes_processed less the quiet lazy ticks k_node_prep counts "
               "without running the node), M_in / M_out = delivered / emitted records.  Departs from "
               "SURVEY 8(d) (every node's 416 B read, touched nodes' written, 32-B Plumtree records): "
               "idle nodes are not read by the kernels and are not counted; every record is the "
               "64-B record the engine moves, plus its 4-B route key")



@contextlib.contextmanager
def c_stdout_to_stderr():
    """C-level writes to stdout (RCCL prints its version banner there as a
    communicator starts) go to stderr meanwhile: rank 0's stdout carries the
    one JSON line only"""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)

def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--nodes", type=int, default=1 << 20, help="nodes per GPU (weak scaling)")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--settle", type=int, default=60, help="untimed rounds after bootstrap")
    p.add_argument("--cpu-sample-nodes", type=int, default=1 << 17)
    p.add_argument("--cpu-sample-rounds", type=int, default=40)
    p.add_argument("--cpu-workers", type=int, default=16,
                   help="processes of the all-cores CPU baseline (the GPU box's CPU share is 16)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-baseline-only", action="store_true",
                   help="print the cpu_baseline object alone (no GPU): e.g. a 2^20 sample with "
                        "--cpu-sample-nodes 1048576, which takes minutes of bootstrap")
    p.add_argument("--no-check", action="store_true", help="skip the built-in sharding check")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher test on CPU: the ranks rendezvous (gloo), time a host loop with the "
                        "same barriers and max-over-ranks, and rank 0 prints the line; no GPU")
    p.add_argument("--vshards", type=int, default=1,
                   help="diagnostic: G virtual shards of --nodes each on this one GPU (the sharded "
                        "partition / exchange / receive path with device copies instead of RCCL)")
    p.add_argument("--kernel-counts", action="store_true",
                   help="diagnostic (profiles/run_pmc.sh): one round per step call, and each node-round kernel's "
                        "nodes, deliveries and emissions (psim_debug_kernel_counts) -> per_kernel_alg")
    p.add_argument("--strict", action="store_true",
                   help="cfg.strict = 1: a fixed-table overflow fails the round (PSIM_ECAPACITY) and the run")
    p.add_argument("--rank-path", action="store_true",
                   help="diagnostic at --gpus 1: run the RCCL rank path with a one-rank communicator "
                        "(owner partition, ncclAllToAll of the counts, grouped self ncclSend/ncclRecv of "
                        "the records, the stats ncclAllReduce, the overlay ncclAllGathers)")
    p.add_argument("--schedule", default="survey", choices=["survey", "doubling"],
                   help="the event schedule.  C, survey (default): SURVEY 8(d) -- joins spread "
                        "over a 64-round ramp, 100 warm-up rounds, then ONE broadcast from node 0 at the "
                        "first timed round; doubling: the round-2 line -- doubling bootstrap, --settle "
                        "rounds, a broadcast from node 0 every 10 rounds throughout.  E, survey "
                        "(default): the half/half partition at phase rounds 150-169, after the churn "
                        "(SURVEY 8(d) E); doubling: round 3's E line, the partition at window rounds "
                        "20-39, inside the churn")
    p.add_argument("--workload", default="C", choices=["C", "B", "D", "E"],
                   help="C (default, the headline line): HyParView+Plumtree; "
                        "B: full-membership strategy, fanout 5; D: SCAMP v2 (c=5); "
                        "E: C with 20%% churn over 100 rounds + a half/half partition")
    return p.parse_args()


def device_mem_used_gb():
    """hipMemGetInfo of this process's device: used = total - free (GB)."""
    import ctypes as C
    try:
        hip = C.CDLL("libamdhip64.so")
        free, tot = C.c_size_t(), C.c_size_t()
        if hip.hipMemGetInfo(C.byref(free), C.byref(tot)) != 0:
            return None
        return (tot.value - free.value) / 1e9
    except OSError:
        return None


# ------------------------------------------------------------ launcher --
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """--gpus N without a launcher: start N ranks of this script (one per
    GPU) before anything here touches a GPU, and exit with their status."""
    import torch                # device_count() does not initialise the GPU on this image

    have = torch.cuda.device_count()
    if have < args.gpus and not args.dry_run:
        print(f"bench: --gpus {args.gpus} needs {args.gpus} GPUs, this machine shows {have}",
              file=sys.stderr, flush=True)
        return 2
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in alive:          # one rank failed: the others would wait in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


# -------------------------------------------------------- CPU baseline --
SURVEY_WARM = 100               # warm-up rounds after the 64-round join ramp


def _cpu_sample(n, seed, rounds, schedule, barrier=None, progress=True):
    """The CPU oracle (a port of the reference handlers, 1 thread) on a
    bounded sample of the workload: same bootstrap, same broadcast schedule.
    Returns (node-rounds, msgs, seconds)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import Oracle
    from partisan_amd import workloads as W
    from partisan_amd.sim import default_config

    o = Oracle(default_config(n_nodes=n, seed=seed))
    # (a progress line every 32 bootstrap rounds on stderr from the 1-thread
    # sample and the first worker at 2^19 nodes and more: minutes of CPU work
    # print nothing else)
    tick = (lambda r: r % 32 or print(f"cpu_baseline: bootstrap round {r}", file=sys.stderr, flush=True)) \
        if progress and n >= (1 << 19) else None
    if schedule == "survey":
        o.run_schedule(W.survey_join(n, seed), W.SURVEY_RAMP + SURVEY_WARM, extra=tick)
    else:
        o.run_schedule(W.doubling_join(n, seed), 40, extra=tick)
    k, msgs = 0, 0
    if barrier is not None:                   # all workers time their rounds together
        barrier.wait()
    t0 = time.perf_counter()
    for r in range(rounds):
        if (r == 0) if schedule == "survey" else (r % BCAST_PERIOD == 0):
            o.broadcast(0, k)
            k += 1
        msgs += int(o.step(1)["emitted"].sum())
    return n * rounds, msgs, time.perf_counter() - t0


def _cpu_worker(a, barrier, q, progress):
    q.put(_cpu_sample(*a, barrier=barrier, progress=progress))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def reference_probe():
    """the reference Erlang path is timed only where an
    Erlang VM exists on this box (`command -v erl`)."""
    import shutil
    erl = shutil.which("erl")
    if erl is None:
        return {"available": False, "erl": None,
                "note": "unavailable: no erl on this box (no Erlang VM); the CPU baseline is the port"}
    try:
        otp = subprocess.run([erl, "-noshell", "-eval",
                              "io:format(\"~s\", [erlang:system_info(otp_release)]), halt()."],
                             capture_output=True, text=True, timeout=60).stdout.strip()
    except (OSError, subprocess.SubprocessError):
        otp = None
    return {"available": True, "erl": erl, "otp_release": otp,
            "note": "an Erlang VM exists here: erlang/harness/README.md runs config A through the "
                    "reference modules and compare_trace.py"}


def _cpu_rows():
    """the CPU restatement on configs A and B as well (1
    thread): A at its size (32 nodes, 200 bootstrap rounds + one broadcast and
    40 rounds; seeds 1-5, the survey's list), B on a bounded sample (the full
    strategy with fanout 5, gossip every round, 16384 nodes after a doubling
    bootstrap + 20 settle rounds, 20 timed rounds)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _scenarios as S
    from _oracle import Oracle
    from partisan_amd import workloads as W
    from partisan_amd.sim import default_config

    t0 = time.perf_counter()
    nr = msgs = 0
    for seed in range(1, 6):
        _, st = S.config_a(Oracle, seed=seed)
        nr += 32 * len(st)
        msgs += int(st["emitted"].sum())
    dt = time.perf_counter() - t0
    rows = {"A": {"value": nr / dt, "unit": "node-rounds/s", "cores": 1, "msgs_per_sec": msgs / dt,
                  "sample": "config A (32 nodes join node 0 one per round, 200 rounds, a broadcast, 40 rounds), "
                            "seeds 1-5, oracle, 1 thread"}}
    n, rounds = 16384, 20
    o = Oracle(default_config(n_nodes=n, seed=1, manager=1, strategy=0, fanout=5, periodic_interval=1))
    boot = W.doubling_join(n, 1)
    o.run_schedule(boot, boot[-1][0] + 1 + 20)
    t0 = time.perf_counter()
    st = o.step(rounds)
    dt = time.perf_counter() - t0
    rows["B"] = {"value": n * rounds / dt, "unit": "node-rounds/s", "cores": 1,
                 "msgs_per_sec": int(st["emitted"].sum()) / dt,
                 "sample": f"config B sample: full-membership strategy (ORSet bitsets), fanout 5, {n} nodes "
                           f"(B is 10^5), doubling bootstrap + 20 rounds, {rounds} timed rounds, oracle, 1 thread"}
    return rows


def cpu_share():
    """What bounds this process's CPUs: the cgroup quota (v2 cpu.max, v1
    cfs_quota_us / cfs_period_us), the affinity mask and the thread knobs the
    box exports (OMP_NUM_THREADS etc.; 16 on the one-GPU box)."""
    out = {"affinity_cpus": len(os.sched_getaffinity(0)), "nproc": os.cpu_count()}
    raw = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            raw = open(path).read().strip()
        except OSError:
            continue
        if path.endswith("cpu.max"):
            q, _, per = raw.partition(" ")
        else:
            try:
                per = open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()
            except OSError:
                per = ""
            q = raw
            raw = f"{q} {per}"
        out["cgroup_cpu_max"] = {"file": path, "value": raw,
                                 "quota_cpus": (int(q) / int(per)) if q.lstrip("-").isdigit() and int(q) > 0
                                 and per.isdigit() else None}
        break
    if raw is None:
        out["cgroup_cpu_max"] = None
    out["env"] = {k: os.environ[k] for k in ("OMP_NUM_THREADS", "MAX_JOBS") if k in os.environ}
    return out


CPU_FULL_SIZE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r05", "cpu20", "cpu20.json")


def _cpu_full_size(n):
    """The same oracle at the headline's full 2^20 nodes, measured once on a
    box's host by `bench.py --cpu-baseline-only --cpu-sample-nodes 1048576
    --cpu-sample-rounds 20` (its bootstrap takes minutes, so the default
    line times the bounded sample above) -- quoted from the committed record
    beside the sample, with its source, not re-measured here"""
    if n >= 1 << 20 or not os.path.exists(CPU_FULL_SIZE):
        return None
    try:
        d = json.load(open(CPU_FULL_SIZE))["cpu_baseline"]
    except (OSError, ValueError, KeyError):
        return None
    return {"value": d["value"], "unit": d["unit"], "cores": d["cores"], "all_cores_value": d["all_cores"]["value"],
            "all_cores": d["all_cores"]["cores"], "sample": d["sample"],
            "source": "profiles/r05/cpu20/cpu20.json (measured, not re-run by this command)"}


def cpu_baseline(args):
    """Run before the GPU is touched (worker processes are forked).  One
    thread, then `workers` independent oracle processes on the same sample
    with different seeds (the oracle is sequential: all-cores throughput is
    the aggregate of independent replicas)."""
    import multiprocessing as mp

    n, rounds = args.cpu_sample_nodes, args.cpu_sample_rounds
    nr, msgs, dt = _cpu_sample(n, args.seed, rounds, args.schedule)
    workers = max(1, min(args.cpu_workers, len(os.sched_getaffinity(0))))
    ctx = mp.get_context("fork")
    barrier, q = ctx.Barrier(workers), ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=((n, args.seed + i, rounds, args.schedule), barrier, q, i == 0))
             for i in range(workers)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join()
    wall = max(r[2] for r in res)
    tot = sum(r[0] for r in res)
    return {"value": nr / dt, "unit": "node-rounds/s", "cores": 1, "kind": "port",
            "msgs_per_sec": msgs / dt,
            "sample": (f"oracle/psim_oracle.c, {n} nodes, {rounds} rounds from one broadcast after the "
                       f"survey bootstrap (64-round ramp + {SURVEY_WARM} rounds), 1 thread"
                       if args.schedule == "survey" else
                       f"oracle/psim_oracle.c, {n} nodes, {rounds} steady-state rounds after a doubling "
                       f"bootstrap, broadcast every {BCAST_PERIOD} rounds, 1 thread"),
            "all_cores": {"value": tot / wall, "unit": "node-rounds/s", "cores": workers,
                          "msgs_per_sec": sum(r[1] for r in res) / wall,
                          "sample": f"{workers} oracle processes at once, each the 1-thread sample "
                                    f"with its own seed, timed rounds started together (barrier); "
                                    f"node-rounds of all / the slowest one's time"},
            "rows": _cpu_rows(),
            "full_size": _cpu_full_size(n),
            "reference": reference_probe(),
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)), "cpu_share": cpu_share()}


# --------------------------------------------------------- shard check --
STAT_FIELDS = ["emitted", "delivered", "dropped", "nodes_up", "nodes_processed", "exits",
               "send_fail", "first_deliveries", "overflow", "digest"]


def _check_schedule(sim, n, ch, r):
    """Config E in miniature (rounds of the check): churn 20% over rounds
    30-49 (crash, restart + rejoin), a half/half partition for 55-64, a
    broadcast from node 0 every 10 rounds from round 20."""
    from partisan_amd import workloads as W
    if r in ch:
        sim.crash(ch[r][0])
        sim.join(ch[r][0], ch[r][1])
    if r == 55:
        sim.set_partition(W.half_partition(n))
    if r == 65:
        sim.clear_partition()
    if r >= 20 and r % BCAST_PERIOD == 0:
        sim.broadcast(0, (r // BCAST_PERIOD) % 0x10000)


def shard_check(args, world, rank, dist, comm):
    """The sharded engine (world RCCL ranks, or 2 virtual shards on one GPU)
    against the one-shard engine on this GPU: stats + digest every round,
    this rank's node rows, the overlay statistics.  Raises on a mismatch."""
    from partisan_amd import Simulator
    from partisan_amd import workloads as W
    from partisan_amd.sim import default_config

    n, seed = CHECK_NODES, args.seed + 100
    dev = int(os.environ.get("PSIM_DEVICE", os.environ.get("LOCAL_RANK", "0")))

    ch = {r: (v, c) for r, v, c in W.churn_schedule(n, seed, 0.2, 30, 20)}

    def run(sim):
        return sim.run_schedule(W.doubling_join(n, seed), CHECK_ROUNDS,
                                extra=lambda r: _check_schedule(sim, n, ch, r))

    cfg = default_config(n_nodes=n, seed=seed, device=dev)
    # the sharded handle's route and owner partition run with 3 blocks, so
    # every block takes several consecutive source steps, as they do at full
    # size (>= 2^19 nodes per shard) -- the small check covers that path too
    os.environ["PSIM_ROUTE_BLOCKS"] = "3"
    try:
        if world > 1 or comm is not None:
            cfg.shard_world, cfg.shard_rank = world, rank
            with c_stdout_to_stderr():
                sh = Simulator(cfg, comm=comm)
            shards = world
        else:
            cfg.n_shards = 2
            sh = Simulator(cfg)
            shards = 2
    finally:
        del os.environ["PSIM_ROUTE_BLOCKS"]
    st_sh = run(sh)
    hist_sh = sh.histograms()             # a collective across ranks
    per = (n + shards - 1) // shards
    lo, cnt = (rank * per, min(n, (rank + 1) * per) - rank * per) if world > 1 else (0, n)
    nodes_sh = sh.nodes(lo, cnt)
    sh.close()
    one = Simulator(default_config(n_nodes=n, seed=seed, device=dev))
    st_one = run(one)
    hist_one = one.histograms()
    nodes_one = one.nodes(lo, cnt)
    one.close()
    bad = []
    for f in STAT_FIELDS:
        if not np.array_equal(st_sh[f], st_one[f]):
            i = np.nonzero((st_sh[f] != st_one[f]).reshape(len(st_sh), -1).any(1))[0][0]
            bad.append(f"stats.{f} differs first at round {int(st_one['round'][i])}")
    for f in nodes_one.dtype.names:
        if not np.array_equal(nodes_sh[f], nodes_one[f]):
            bad.append(f"node rows field {f} differ")
    for k, v in hist_one.items():
        if not np.array_equal(np.asarray(hist_sh[k]), np.asarray(v)):
            bad.append(f"histograms.{k} differ")
    if world > 1:                             # every rank learns whether any rank failed
        import torch
        t = torch.tensor([len(bad)], dtype=torch.int64)
        dist.all_reduce(t)
        if int(t.item()) and not bad:
            bad.append("another rank's check failed")
    if bad:
        raise SystemExit(f"bench: sharding check failed on rank {rank}: {bad[:4]}")
    return {"nodes": n, "rounds": CHECK_ROUNDS, "shards": shards,
            "rank_path": comm is not None,
            "against": "the one-shard engine on this GPU",
            "scenario": "doubling bootstrap, 20% churn rounds 30-49, half/half partition 55-64, "
                        "broadcast every 10 rounds",
            "equal": ["per-round stats and record digest", "node rows", "overlay statistics"],
            "route_blocks": 3,
            "msgs": int(st_one["emitted"].sum()),
            "symmetric_links": int(hist_one["symmetric_links"]), "components": int(hist_one["components"])}


# --------------------------------------------------------- PMC traffic --
def src_hash():
    h = hashlib.sha256()
    d = os.path.join(ROOT, "partisan_amd", "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".h")):
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    h.update(open(os.path.join(ROOT, "include", "partisan_gpu_sim.h"), "rb").read())
    return h.hexdigest()[:16]


def pmc_key(args, world, n):
    return {"workload": args.workload, "nodes": n, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "seed": args.seed, "schedule": SCHEDULE_VERSION,
            "events": args.schedule if args.workload in ("C", "E") else "doubling", "src": src_hash()}


def pmc_traffic(key):
    """HBM bytes per launch of the node-round kernels from a committed PMC
    record (profiles/pmc_records.json, written by profiles/run_pmc.sh) of
    this same command -- workload, size, GPUs, steps, warmup, seed, event
    schedule and kernel sources.  None when no record matches."""
    try:
        recs = json.load(open(os.path.join(ROOT, "profiles", "pmc_records.json")))
    except (OSError, ValueError):
        return None, None
    for r in recs:
        if r.get("key") == key:
            return r["traffic_per_launch"], r
    return None, None


# ---------------------------------------------------- pluggable (B, D) --
def main_strategy(args):
    """Configs B and D of BASELINE.json on the pluggable manager (extra
    lines, not the driver's headline): a step is one round over every node.
    B: partisan_full_membership_strategy, 100k nodes, fanout 5 (the
       extension of SURVEY App. A Q10), periodic gossip every round.
    D: partisan_scamp_v2_membership_strategy, c = 5, 2^21 nodes per GPU."""
    from partisan_amd import Simulator
    from partisan_amd import workloads as W
    from partisan_amd.sim import default_config
    if args.workload == "B":
        n = 100000 if args.nodes == 1 << 20 else args.nodes
        cfg = default_config(n_nodes=n, seed=args.seed, manager=1, strategy=0, fanout=5,
                             periodic_interval=1)
        name = "B: full-membership strategy (ORSet bitsets), fanout 5, gossip every round"
    else:
        n = (1 << 21) if args.nodes == 1 << 20 else args.nodes
        cfg = default_config(n_nodes=n, seed=args.seed, manager=1, strategy=2, scamp_c=5)
        name = "D: SCAMP v2 (c=5), doubling bootstrap, steady state"
    cfg.device = int(os.environ.get("PSIM_DEVICE", "0"))
    sim = Simulator(cfg)
    boot = W.doubling_join(n, args.seed)
    sim.run_schedule(boot, boot[-1][0] + 1 + args.settle)
    sim.step(args.warmup)
    t0 = time.perf_counter()
    st = sim.step(args.steps)
    dt = time.perf_counter() - t0
    kt = sim.kernel_times()
    msgs = int(st["emitted"].sum())
    c_ms, c_n = kt.get("consume", (0.0, 1))
    # algorithmic bytes of the consume kernel: member-row bytes it touches
    # (state_bytes, full) or the 64-B view row + header per processed node
    # (scamp), plus every message record read once and written once
    if args.workload == "B":
        state = int(st["state_bytes"].sum())
    else:
        state = int(st["nodes_processed"].sum()) * 2 * (64 + 4 * 64 * 2)
    alg = state + int(st["delivered"].sum()) * S_MSG + msgs * (S_MSG + 4)
    achieved = alg / (c_ms / 1e3) / 1e9 if c_ms > 0 else 0.0
    key = pmc_key(args, 1, n)
    traffic, trec = pmc_traffic(key)
    tsrc = trec.get("source") if trec else None
    out = {
        "metric": "simulated node-rounds/sec (+ msgs/sec), pluggable manager " + args.workload,
        "value": n * args.steps / dt, "unit": "node-rounds/s", "msgs_per_sec": msgs / dt,
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": name, "nodes": n, "seed": args.seed, "parallelism": "1 GPU"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                     "traffic_upper": trec.get("traffic_upper_per_launch") if trec else None,
                     # the counted HBM bytes over the same time: B's ORSet rows are
                     # re-read from L2 / MALL, so its algorithmic fraction is above
                     # what the memory moved (state both)
                     "traffic_frac": (traffic / (c_ms / max(1, c_n) / 1e3) / 1e9 / HBM_PEAK_GBS)
                                     if traffic and c_ms > 0 else None,
                     "kernel": "k_consume_pl",
                     "alg_bytes_per_launch": alg / max(1, c_n), "avg_launch_ms": c_ms / max(1, c_n)},
        "kernel_ms_per_step": {k: v[0] / args.steps for k, v in kt.items() if v[1]},
        "overflow": int(st["overflow"].sum()),
        "members_min": int(sim.strategy_nodes(0, min(n, 4096))["members"].min()) if args.workload == "B" else None,
        "pmc_key": key,
    }
    print(json.dumps(out), flush=True)


def dry_run(args, world, rank, dist):
    """The rank protocol of main() without a GPU: rendezvous, barrier,
    EXACTLY --steps timed steps of host work, barrier, max over ranks."""
    if os.environ.get("PSIM_BENCH_FAIL_RANK") == str(rank):
        raise SystemExit(3)                   # (test hook: a failing rank)
    x = np.arange(1 << 16, dtype=np.uint64)
    for _ in range(args.warmup):
        x = (x * 6364136223846793005 + 1442695040888963407) & 0xFFFFFFFFFFFF
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x = (x * 6364136223846793005 + 1442695040888963407) & 0xFFFFFFFFFFFF
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "dry run (launcher test)", "value": world * args.steps / dt,
                          "unit": "steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": dt / args.steps * 1e3, "dry_run": True,
                          "ranks": world, "checksum": int(x.sum() & 0xFFFF)}), flush=True)
    dist.destroy_process_group() if world > 1 else None


# ----------------------------------------------------- HyParView (C, E) --
def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU")
    if args.workload in ("B", "D"):
        if world > 1:
            raise SystemExit("bench: --workload B/D are single-GPU lines")
        return main_strategy(args)
    if world > 1 and args.vshards > 1:
        raise SystemExit("bench: --vshards is a single-GPU diagnostic")
    if args.rank_path and (world > 1 or args.vshards > 1):
        raise SystemExit("bench: --rank-path is the one-GPU diagnostic of the RCCL path (ranks > 1 use it anyway)")

    # the CPU baseline first, while no GPU has been touched (it forks)
    if args.cpu_baseline_only:
        print(json.dumps({"cpu_baseline": cpu_baseline(args), "workload": args.workload,
                          "schedule": args.schedule, "rounds": args.cpu_sample_rounds}), flush=True)
        return
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "C":
        cpu = cpu_baseline(args)

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if torch.cuda.device_count() < world and not args.dry_run:
            raise SystemExit(f"bench: {world} ranks but {torch.cuda.device_count()} GPUs: one rank per GPU")
        dist.init_process_group("gloo")
    if args.dry_run:
        return dry_run(args, world, rank, dist)

    from partisan_amd import Simulator
    from partisan_amd import workloads as W
    from partisan_amd.sim import comm_id, default_config

    def shared_comm():
        if world == 1:
            return comm_id() if args.rank_path else None
        obj = [comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return obj[0]

    check = None
    if not args.no_check:
        check = shard_check(args, world, rank, dist, shared_comm())

    # weak scaling: --nodes per GPU; the overlay spans all GPUs, node-range
    # sharded, one RCCL rank per GPU
    n = args.nodes * world * args.vshards
    cfg = default_config(n_nodes=n, seed=args.seed)
    cfg.n_shards = args.vshards
    cfg.strict = 1 if args.strict else 0
    cfg.device = int(os.environ.get("PSIM_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    comm = shared_comm()
    if world > 1:
        cfg.shard_world, cfg.shard_rank = world, rank
    with c_stdout_to_stderr():
        sim = Simulator(cfg, comm=comm)
    ovf_run = np.zeros(len(OVF_KINDS), np.uint64)          # overflows by table over every round of the run

    def step(k):
        s_ = sim.step(k)
        ovf_run[:] += s_["overflow_by"].sum(axis=0).astype(np.uint64)
        return s_

    sched = W.BenchSchedule(args.workload, args.schedule, n, args.seed, args.warmup, args.settle)
    survey = sched.survey
    boot, until = sched.bootstrap()
    ovf_run[:] += sim.run_schedule(boot, until)["overflow_by"].sum(axis=0).astype(np.uint64)
    # phase-round i counts from the end of the bootstrap; the timed window
    # starts at t_start (workloads.BenchSchedule)
    t_start = sched.t_start
    round_events = lambda i: sched.apply(sim, i)      # noqa: E731
    has_events = sched.has_events
    bcast_round = sched.bcast_round

    for i in range(t_start):
        round_events(i)
        step(1)
    if world > 1:
        dist.barrier()
    x0 = sim.exchange_stats()
    t0 = time.perf_counter()
    stats = []
    kt = {}
    i = 0
    kc = {}                                           # --kernel-counts: per kernel (nodes, in, out)
    while i < args.steps:
        # rounds up to the next one with host events run in one step call
        round_events(t_start + i)
        k = 1
        while i + k < args.steps and not has_events(t_start + i + k) and not args.kernel_counts:
            k += 1
        stats.append(step(k))
        i += k
        if args.kernel_counts:
            for name, v in sim.kernel_counts().items():
                kc[name] = tuple(a + b for a, b in zip(kc.get(name, (0, 0, 0)), v))
        for name, (ms, cnt) in sim.kernel_times().items():
            a, b = kt.get(name, (0.0, 0))
            kt[name] = (a + ms, b + cnt)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    x1 = sim.exchange_stats()
    st = np.concatenate(stats)
    dt = t1 - t0
    if world > 1:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    msgs = int(st["emitted"].sum())            # stats are global (all ranks)
    node_rounds = n * args.steps
    # roofline of the dominant kernel (the node-round phase): algorithmic
    # bytes per launch of this rank (global counters / world: equal ranges)
    per = world
    # (state_bytes: the rows of the nodes the kernels ran, 2 * S_NODE each --
    # nodes_processed also counts the quiet lazy ticks k_node_prep settles)
    proc = int(st["state_bytes"].sum()) / (2 * S_NODE) / per
    deliv = int(st["delivered"].sum()) / per
    alg_bytes = proc * 2 * S_NODE + deliv * S_MSG + msgs / per * (S_MSG + 4)
    c_ms, c_n = kt.get("consume", (0.0, 0))
    per_launch_bytes = alg_bytes / max(1, c_n)
    per_launch_s = (c_ms / 1e3) / max(1, c_n)
    achieved = per_launch_bytes / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
    # the same algorithmic bytes over the whole step (node-round phase, route,
    # gather, prepare, stats, host syncs): the whole-step roofline fraction
    step_achieved = alg_bytes / dt / 1e9 if dt > 0 else 0.0
    key = pmc_key(args, world, n)
    traffic, trec = pmc_traffic(key)
    tsrc = trec.get("source") if trec else None
    n_bc = sum(1 for j in range(t_start, t_start + args.steps) if bcast_round(j))
    out = {
        "metric": "simulated node-rounds/sec (+ msgs/sec), 1M-node HyParView+Plumtree"
                  + ("" if args.workload == "C" else " (config E: churn + partition)"),
        "value": node_rounds / dt,
        "unit": "node-rounds/s",
        "msgs_per_sec": msgs / dt,
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32", "data": "synthetic",
        "config": {"workload": ("C: HyParView+Plumtree, SURVEY 8(d) schedule: joins over a 64-round ramp "
                                "(node i at round 64*i/N, contact uniform among earlier rounds), 100 warm-up "
                                "rounds, --warmup rounds, then one broadcast from node 0 at the first timed "
                                "round; the window is that broadcast's propagation") if survey else
                               ("C: HyParView+Plumtree, doubling bootstrap, steady state, "
                                "broadcast from node 0 every 10 rounds (not SURVEY 8(d)'s schedule: the doubling "
                                "ramp starts half the overlay in one round, aligning its shuffle timers)")
                               if args.workload == "C" else
                               ("E: HyParView+Plumtree, doubling bootstrap, 20% churn over phase rounds 40-139 "
                                "(crash, restart, rejoin the next round), half/half partition for phase rounds "
                                + (f"{sched.p_on}-{sched.p_off - 1} (SURVEY 8(d) E: after the churn)"
                                   if args.schedule == "survey" else
                                   f"{sched.p_on}-{sched.p_off - 1} (window rounds 20-39, inside the churn: "
                                   "round 3's line)")
                                + ", broadcast from node 0 every 10 rounds; the window starts at phase round "
                                f"{t_start}"),
                   "nodes": n, "nodes_per_gpu": args.nodes, "seed": args.seed,
                   "schedule": args.schedule if args.workload in ("C", "E") else "doubling",
                   "untimed_broadcast_rounds": 0 if survey else STEADY_ROUNDS + args.warmup,
                   "broadcasts_before_window": 0 if survey else (t_start + BCAST_PERIOD - 1) // BCAST_PERIOD,
                   "broadcasts_in_window": n_bc,
                   "parallelism": (f"node-range sharded x{world}, RCCL all-to-all" if world > 1 else
                                   "1 GPU, the RCCL rank path with a one-rank communicator" if args.rank_path else
                                   f"1 GPU, {args.vshards} virtual shards" if args.vshards > 1 else "1 GPU")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                     "traffic_upper": trec.get("traffic_upper_per_launch") if trec else None,
                     "kernel": "k_relay + k_shuf + k_lite_half + k_consume + k_ptl + k_pt (the node-round "
                               "phase: one launch of each per round, one after another on the shard's stream, "
                               "timed by s_memrealtime stamps stored as k_relay's first block starts and as the "
                               "first kernel after k_pt starts)",
                     "alg_bytes_per_launch": per_launch_bytes,
                     "alg_bytes_formula": ALG_FORMULA,
                     "avg_launch_ms": per_launch_s * 1e3,
                     "step_achieved": step_achieved,
                     "step_frac": step_achieved / HBM_PEAK_GBS},
        "kernel_ms_per_step": {k: v[0] / args.steps for k, v in kt.items() if v[1]},
        "overflow": int(st["overflow"].sum()),
        "pmc_key": key,
    }
    if kc:
        # each node-round kernel's share of the algorithmic bytes (the formula
        # above, with the kernel's own counts: its nodes processed, records
        # delivered and emitted), per round
        # (k_node_prep's entry: quiet lazy ticks, counted without reading
        # the node -- no bytes)
        out["per_kernel_alg"] = {k: (v[0] * 2 * S_NODE + v[1] * S_MSG + v[2] * (S_MSG + 4)) / args.steps
                                 for k, v in kc.items() if k != "k_node_prep"}
        out["per_kernel_counts"] = {k: [x / args.steps for x in v] for k, v in kc.items()}
    if world > 1 or args.vshards > 1 or args.rank_path:
        # the cross-shard exchange over the window, this rank's shards: records
        # sent to another shard and their wire bytes (32 B a record, 32 more
        # for one with exchange ids; 64 B a record in memory)
        xr, xb = x1[0] - x0[0], x1[1] - x0[1]
        out["exchange"] = {"records_per_round": xr / args.steps, "wire_bytes_per_round": xb / args.steps,
                           "wire_bytes_per_record": xb / max(1, xr), "record_bytes_in_memory": 64}
    if check is not None:
        out["check"] = check
    # overlay statistics (psim_get_histograms; outside the measurement):
    # drain rounds without new broadcasts until the tracked (last) broadcast
    # has had at least its last hop + 5 rounds and OVERLAY_DRAIN rounds
    since = t_start + args.steps - sched.last_bcast
    step(OVERLAY_DRAIN)
    drained = OVERLAY_DRAIN
    while True:
        ov = sim.histograms()
        bins = np.arange(len(ov["hop"]))
        last_hop = int(bins[ov["hop"] > 0].max()) if ov["delivered"] else 0
        if since + drained >= last_hop + 5 or drained >= 400:
            break
        step(10)
        drained += 10
    nup = max(1, ov["n_up"])
    out["overlay"] = {
        "nodes_up": ov["n_up"],
        "tracked_broadcast_reliability": ov["delivered"] / nup,
        "tracked_broadcast_last_hop": last_hop if ov["delivered"] else None,
        "active_in_mean": float((ov["active_in"] * bins).sum() / nup),
        "passive_in_mean": float((ov["passive_in"] * bins).sum() / nup),
        "symmetric_active_links": ov["symmetric_links"] / max(1, ov["active_links"]),
        "active_links": ov["active_links"],
        "components": ov["components"],
        "largest_component": ov["largest_component"],
        "rounds_since_tracked_broadcast": since + drained,
        "rounds_drained": drained,
    }
    # message conservation over the window: every record emitted in round
    # r is delivered or dropped in round r + 1
    em = st["emitted"].sum(axis=1)
    got = st["delivered"].sum(axis=1) + st["dropped"]
    out["conservation"] = {"rounds_checked": int(len(st) - 1),
                           "ok": bool(np.array_equal(em[:-1], got[1:]))}
    out["device_mem_used_gb"] = device_mem_used_gb()
    out["overflow_run"] = {"rounds": sim.round, **{k: int(v) for k, v in zip(OVF_KINDS, ovf_run)},
                           "total": int(ovf_run.sum()), "strict": bool(args.strict)}
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    sim.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
