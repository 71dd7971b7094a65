#!/usr/bin/env python3
"""Headline benchmark: decided consensus instances/sec at n=64, f=21 (BASELINE.json configs[3]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--instances I]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (multi-GPU)

Workload: 64 replicas, f = 21, the reference's protocol exactly as it
runs (Bracha broadcast + two-phase consensus, reference quirks included), adversarial delays
(messages from/to a per-instance slow set of f replicas take D = 8 steps, all others 1),
Philox Bernoulli(1/2) proposals.  One "step" = one full pass of the hot path over the batch:
every instance simulated from its proposals until every honest replica has decided (the
reference's decide() upcall, core/byzantinerandomizedconsensus.py:94).  Instances are
independent, so ranks shard them (global Philox ids => results independent of N: weak
scaling); the only collective is one RCCL all-reduce of the statistics.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_REPLICAS, F_FAULTS, DELAY_MAX, SEED, COIN_SEED = 64, 21, 8, 0x5EED0004, 0xC017C017
SURVEY_BYTES_PER_CELL_STEP = 6 * ((N_REPLICAS + 7) // 8) + 2   # 50 B at n=64
HBM_PEAK_GBS = 8000.0                                           # MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--instances", type=int, default=1 << 20, help="instances per GPU (SURVEY §8(d) cfg4: 2^20)")
    ap.add_argument("--key-window", type=int, default=0, help="0: 4 (reference mode), 8 (spec mode)")
    ap.add_argument("--mode", choices=("reference", "spec"), default="reference",
                    help="reference: the protocol as the reference runs it (headline); spec: the intended "
                         "protocol with its common coin (SURVEY §8 F3)")
    ap.add_argument("--round-cap", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="collective backend for N > 1: nccl (= RCCL over xGMI, one GPU per rank); gloo "
                         "only rehearses the multi-rank flow with several ranks sharing one GPU")
    return ap.parse_args()


def cpu_baseline(seconds, mode="reference", window=4, round_cap=1):
    """The C oracle (a scalar port of the reference's path) on the same workload, one thread per
    core (ctypes releases the GIL inside the C run): threads take interleaved global instance ids
    from 0 and run until `seconds` have passed.  Counters only (the oracle's light mode)."""
    import concurrent.futures
    from oracle import oracle
    from tests.golden import specs as S
    threads = max(1, min(16, os.cpu_count() or 1))    # the GPU box's CPU share is 16

    def spec(g):
        if mode == "spec":
            return S.spec_cons_spec(N_REPLICAS, F_FAULTS, SEED, 2, DELAY_MAX, g, round_cap=round_cap,
                                    window=window, coin_seed=COIN_SEED)
        return S.cons_spec(N_REPLICAS, F_FAULTS, SEED, 2, DELAY_MAX, g, round_cap=round_cap)

    t0 = time.perf_counter()

    def worker(first):
        done = arrivals = count = 0
        g = first
        while time.perf_counter() - t0 < seconds:
            r = oracle.run(spec(g), light=True)
            done += r["status"] == "done"
            arrivals += r["arrivals"]
            count += 1
            g += threads
        return done, arrivals, count

    with concurrent.futures.ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(worker, range(threads)))
    dt = time.perf_counter() - t0
    done, arrivals, count = (sum(p[i] for p in parts) for i in range(3))
    return {"value": done / dt, "unit": "decided instances/s", "cores": threads, "kind": "port",
            "sample": "%d instances of the same workload (global ids 0..%d), %.1f s on %d threads, C oracle "
                      "(oracle/brc_oracle.c, event-by-event restatement); %.3g replica-message-steps/s"
                      % (count, count - 1, dt, threads, arrivals / dt)}


def load_traffic(instances, kernel_ms, mode="reference"):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json,
    written by profiles/summarize.py), used only if it was taken on this workload and size and
    its kernel time agrees with the live one within 15 % (i.e. the same kernel build)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("instances") != instances or d.get("workload") != "cfg4" or not d.get("avg_ns") or \
            d.get("mode", "reference") != mode:
        return None
    if abs(d["avg_ns"] / 1e6 - kernel_ms) > 0.15 * kernel_ms:
        return None
    return d.get("hbm_bytes_per_launch")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    coll_dev = "cuda"
    if world > 1:
        import torch
        import torch.distributed as tdist
        if args.backend == "gloo":                  # rehearsal: ranks may share a GPU
            local %= torch.cuda.device_count()
            coll_dev = "cpu"
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group("gloo")
        dist = tdist

    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd import shard
    from byzantinerandomizedconsensus_amd.engine import Engine

    per = args.instances
    spec = args.mode == "spec"
    if not args.key_window:
        args.key_window = 8 if spec else 4
    first, count = shard.shard_range(per * world, world, rank)     # global instance ids of this rank
    eng = Engine(n=N_REPLICAS, f=F_FAULTS, instances=count, protocol="consensus", seed=SEED,
                 delay_model=L.DELAY_SLOWSET, delay_max=DELAY_MAX, round_cap=args.round_cap, step_cap=4000,
                 key_window=args.key_window, variants=1, proposals=L.PROPOSALS_PHILOX,
                 instance_offset=first, device=local, mode=L.MODE_SPEC if spec else L.MODE_REFERENCE,
                 coin_seed=COIN_SEED)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    def one_step():
        eng.reset()
        eng.run()
        return eng.last_kernel_ms()

    for _ in range(args.warmup):
        one_step()
    barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        kms.append(one_step())
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(kms) / len(kms)
    # the only collective: statistics (RCCL over xGMI), max of the wall clocks
    st, hist = shard.reduce_stats(eng.stats(), dist, device=coll_dev, hist=eng.round_histogram(66))
    elapsed = shard.max_over_ranks(elapsed, dist, device=coll_dev)
    kernel_ms = shard.max_over_ranks(kernel_ms, dist, device=coll_dev)
    decided, arrivals, cell_steps = st["decided"], st["arrivals"], st["cell_steps"]
    bad = st["overflow"] + st["stepcap"] + st["running"]
    if bad:
        print("WARNING: %d instances did not finish cleanly" % bad, file=sys.stderr)
    value = decided * args.steps / elapsed
    out = None
    if rank == 0:
        achieved = SURVEY_BYTES_PER_CELL_STEP * (cell_steps / world) / (kernel_ms / 1e3) / 1e9
        traffic = load_traffic(per, kernel_ms, args.mode)
        out = {
            "metric": "decided consensus instances/sec (node) at n=64,f=21",
            "value": value,
            "unit": "instances/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (Philox4x32-10 proposals and slow sets, seed 0x5EED0004)",
            "config": {"workload": "cfg4: n=64 f=21 %s consensus to %s, slow-set delays D=8, %d instances/GPU"
                                   % ("SPEC-protocol (common coin)" if spec else "reference-protocol",
                                      "first decision" if args.round_cap == 1 else "%d decisions" % args.round_cap,
                                      per),
                       "n": N_REPLICAS, "f": F_FAULTS, "instances_per_gpu": per, "round_cap": args.round_cap,
                       "mode": args.mode, "key_window": args.key_window,
                       "parallelism": "instance-sharded x%d" % world},
            "decide_round_hist": {str(r): c for r, c in enumerate(hist) if c},
            "replica_message_steps_per_s": arrivals * args.steps / elapsed,
            "decided_fraction": decided / float(per * world),
            "kernel_ms": kernel_ms,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "note": "algorithmic = %d B (SURVEY 8(d)) x %d cell-steps per launch per GPU"
                                 % (SURVEY_BYTES_PER_CELL_STEP, cell_steps // world)},
        }
    eng.close()
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_seconds > 0:     # N = 1 only
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.mode, args.key_window, args.round_cap)
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
