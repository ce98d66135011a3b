"""Benchmark: config C of BASELINE.json on MI355X.

A step is one BSP round of the hot path (HyParView handlers + timers,
Plumtree broadcast, message route) over every node of a 2^20-node overlay
(steady state after a doubling bootstrap; a broadcast from node 0 every 10
rounds).  Prints ONE JSON line (rank 0).  See DESIGN.md section 5.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

OVERLAY_DRAIN = 40               # untimed rounds before the overlay statistics
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md)
S_NODE = 416                    # algorithmic state bytes per processed node
S_MSG = 64                      # message record bytes


def pmc_traffic(workload):
    """HBM bytes per round of the node-round kernels (k_relay + k_consume)
    from the committed PMC passes of this same bench command
    (profiles/run_pmc.sh -> profiles/pmc_latest.txt): FETCH_SIZE doubled
    (gfx950 tallies 128-B read requests at 64 B, MI355X_MICROARCH.md HBM
    section) plus WRITE_SIZE, both in KiB per timed round.  Config C only;
    None when the file is absent."""
    if workload != "C":
        return None
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_latest.txt")
    try:
        vals = {}
        for line in open(path):
            f = line.split()
            if len(f) >= 5 and f[0] in ("FETCH_SIZE", "WRITE_SIZE") and f[3] == "per-round":
                vals[f[0]] = float(f[4])
        return (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    except (OSError, KeyError, ValueError):
        return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--nodes", type=int, default=1 << 20)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--settle", type=int, default=60, help="untimed rounds after bootstrap")
    p.add_argument("--cpu-sample-nodes", type=int, default=1 << 16)
    p.add_argument("--cpu-sample-rounds", type=int, default=40)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--vshards", type=int, default=1,
                   help="diagnostic: G virtual shards of --nodes each on this one GPU (the sharded "
                        "partition / exchange / receive path with device copies instead of RCCL)")
    p.add_argument("--workload", default="C", choices=["C", "B", "D", "E"],
                   help="C (default, the headline line): HyParView+Plumtree; "
                        "B: full-membership strategy, fanout 5; D: SCAMP v2 (c=5); "
                        "E: C with 20%% churn over 100 rounds + a half/half partition")
    return p.parse_args()


def cpu_baseline(args):
    """The CPU oracle (port of the reference handlers, 1 thread) on a bounded
    sample of the same workload: 2^16 nodes, same bootstrap, timed rounds
    with the same broadcast cadence."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import Oracle
    from partisan_amd import workloads as W
    from partisan_amd.sim import default_config

    n = args.cpu_sample_nodes
    o = Oracle(default_config(n_nodes=n, seed=args.seed))
    o.run_schedule(W.doubling_join(n, args.seed), 40)
    k = 0
    t0 = time.perf_counter()
    msgs = 0
    for r in range(args.cpu_sample_rounds):
        if r % 10 == 0:
            o.broadcast(0, k)
            k += 1
        st = o.step(1)
        msgs += int(st["emitted"].sum())
    dt = time.perf_counter() - t0
    return {"value": n * args.cpu_sample_rounds / dt, "unit": "node-rounds/s", "cores": 1,
            "kind": "port",
            "msgs_per_sec": msgs / dt,
            "sample": f"oracle/psim_oracle.c, {n} nodes, {args.cpu_sample_rounds} steady-state "
                      f"rounds after a doubling bootstrap, broadcast every 10 rounds, 1 thread"}


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
    out = {
        "metric": "simulated node-rounds/sec (+ msgs/sec), pluggable manager " + args.workload,
        "value": n * args.steps / dt, "unit": "node-rounds/s", "msgs_per_sec": msgs / dt,
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": name, "nodes": n, "seed": args.seed, "parallelism": "1 GPU"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(args.workload), "kernel": "k_consume_pl",
                     "alg_bytes_per_launch": alg / max(1, c_n), "avg_launch_ms": c_ms / max(1, c_n)},
        "kernel_ms_per_step": {k: v[0] / args.steps for k, v in kt.items() if v[1]},
        "overflow": int(st["overflow"].sum()),
        "members_min": int(sim.strategy_nodes(0, min(n, 4096))["members"].min()) if args.workload == "B" else None,
    }
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    if args.workload in ("B", "D"):
        return main_strategy(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    from partisan_amd import Simulator
    from partisan_amd import workloads as W
    from partisan_amd.sim import comm_id, default_config

    # weak scaling: --nodes per GPU; the overlay spans all GPUs, node-range
    # sharded, one RCCL rank per GPU
    n = args.nodes * world * args.vshards
    cfg = default_config(n_nodes=n, seed=args.seed)
    cfg.n_shards = args.vshards
    cfg.device = int(os.environ.get("PSIM_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    comm = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        obj = [comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = obj[0]
        cfg.shard_world, cfg.shard_rank = world, rank
    sim = Simulator(cfg, comm=comm)
    boot = W.doubling_join(n, args.seed)
    sim.run_schedule(boot, boot[-1][0] + 1 + args.settle)

    state = {"k": 0}
    churn = {}
    if args.workload == "E":
        # config E: 0.2*N crashes spread over 100 rounds, each
        # victim restarts the next round and rejoins; ids [0, N/2) | [N/2, N)
        # partitioned for 20 rounds from round 20 of the measured window
        for r, v, c in W.churn_schedule(n, args.seed, 0.2, 0, 100):
            churn[r] = (v, c)
        part = W.half_partition(n)

    def round_events(i):
        if i % 10 == 0:
            sim.broadcast(0, state["k"] % 0x10000)
            state["k"] += 1
        if args.workload == "E":
            if i in churn:
                sim.crash(churn[i][0])
            if i - 1 in churn:
                sim.join(churn[i - 1][0], churn[i - 1][1])
            if i == 20:
                sim.set_partition(part)
            if i == 40:
                sim.clear_partition()

    def has_events(i):
        return i % 10 == 0 or (args.workload == "E" and (i in churn or i - 1 in churn or i in (20, 40)))

    for i in range(args.warmup):
        round_events(i)
        sim.step(1)
    if world > 1:
        dist.barrier()
    if os.environ.get("PSIM_TRACE_GROW"):
        print("bench: timed rounds start", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    stats = []
    kt = {}
    i = 0
    while i < args.steps:
        # rounds up to the next one with host events run in one step call
        round_events(args.warmup + i)
        k = 1
        while i + k < args.steps and not has_events(args.warmup + i + k):
            k += 1
        stats.append(sim.step(k))
        i += k
        for name, (ms, cnt) in sim.kernel_times().items():
            a, b = kt.get(name, (0.0, 0))
            kt[name] = (a + ms, b + cnt)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    st = np.concatenate(stats)
    dt = t1 - t0
    if world > 1:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    msgs = int(st["emitted"].sum())            # stats are global (all ranks)
    node_rounds = n * args.steps
    # roofline of the dominant kernel (consume): algorithmic bytes per launch
    # of this rank (global counters / world: the shards are equal ranges)
    per = world                                # this process's share (its launches: c_n)
    proc = int(st["nodes_processed"].sum()) / per
    deliv = int(st["delivered"].sum()) / per
    alg_bytes = proc * 2 * S_NODE + deliv * S_MSG + msgs / per * (S_MSG + 4)
    c_ms, c_n = kt.get("consume", (0.0, 0))
    per_launch_bytes = alg_bytes / max(1, c_n)
    per_launch_s = (c_ms / 1e3) / max(1, c_n)
    achieved = per_launch_bytes / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
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
        "config": {"workload": ("C: HyParView+Plumtree, doubling bootstrap, steady state, "
                                "broadcast from node 0 every 10 rounds") if args.workload == "C" else
                               ("E: HyParView+Plumtree, 20% churn over 100 rounds (crash, restart, rejoin), "
                                "half/half partition for rounds 20-39, broadcast every 10 rounds"),
                   "nodes": n, "nodes_per_gpu": args.nodes, "seed": args.seed,
                   "parallelism": (f"node-range sharded x{world}, RCCL all-to-all" if world > 1 else
                                   f"1 GPU, {args.vshards} virtual shards" if args.vshards > 1 else "1 GPU")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(args.workload),
                     "kernel": "k_relay + k_consume (the node-round phase: one launch of each per round, "
                               "timed from k_relay's first block to k_consume's last)",
                     "alg_bytes_per_launch": per_launch_bytes,
                     "avg_launch_ms": per_launch_s * 1e3},
        "kernel_ms_per_step": {k: v[0] / args.steps for k, v in kt.items() if v[1]},
        "overflow": int(st["overflow"].sum()),
    }
    if args.workload == "E":
        lo = sim.cfg.shard_rank * args.nodes if world > 1 else 0
        v = sim.nodes(lo, min(args.nodes, 1 << 18))       # a sample of this rank's range
        # the second-to-last broadcast has had >= 10 rounds to spread
        got = (v["have"] >> ((state["k"] - 2) % 32)) & 1
        out["reliability_broadcast"] = {"msg": state["k"] - 2, "rounds": args.warmup + args.steps - 10 * (state["k"] - 2),
                                        "delivered_fraction": float(got[v["up"] == 1].mean())}
    # overlay statistics (psim_get_histograms; outside the measurement, after
    # OVERLAY_DRAIN more rounds without new broadcasts so the last one has
    # settled): the tracked broadcast's reach and hop depth, active view
    # symmetry and connectivity, mean in-degrees -- SURVEY 8(d)'s report
    sim.step(OVERLAY_DRAIN)
    ov = sim.histograms()
    bins = np.arange(len(ov["hop"]))
    nup = max(1, ov["n_up"])
    out["overlay"] = {
        "nodes_up": ov["n_up"],
        "tracked_broadcast_reliability": ov["delivered"] / nup,
        "tracked_broadcast_last_hop": int(bins[ov["hop"] > 0].max()) if ov["delivered"] else None,
        "active_in_mean": float((ov["active_in"] * bins).sum() / nup),
        "passive_in_mean": float((ov["passive_in"] * bins).sum() / nup),
        "symmetric_active_links": (ov["symmetric_links"] / max(1, ov["active_links"])
                                   if ov["symmetric_links"] != 2**64 - 1 else None),
        "components": ov["components"] if ov["components"] != 2**64 - 1 else None,
        "largest_component": ov["largest_component"] if ov["components"] != 2**64 - 1 else None,
        "rounds_since_tracked_broadcast": OVERLAY_DRAIN + (args.warmup + args.steps - 1) % 10 + 1,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "C":
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
