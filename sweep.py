#!/usr/bin/env python3
"""Large-committee sweep (BASELINE.json configs[4]): n = 256 over f and the
network-delay distributions, with decide-round histograms all-reduced over ranks (RCCL over xGMI
with the nccl backend; one process per GPU).

    python sweep.py [--instances I] [--mode spec|reference] [--f 0,21,85] [--models const,uniform,geometric]
    python -m torch.distributed.run --nproc-per-node N ... sweep.py    (multi-GPU, weak scaling)
    python -m torch.distributed.run --nproc-per-node 1 ... sweep.py --dist   (one RCCL rank)

Every configuration is its own engine (one launch).  Instances shard across ranks by global id, so
the histograms do not depend on the rank count.  Default mode is SPEC (the intended protocol with
its common coin: the only mode with more than one round); ``--mode reference`` runs
the reference's protocol as-is (decide("-1") every round, K2 stalls under random delays).
Prints one JSON line per configuration (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N = 256
SEED, COIN_SEED = 0x5EED0005, 0xC017C017
MODELS = {"const": (0, 1), "uniform": (1, 4), "geometric": (3, 16)}   # (BRC_DELAY_*, delay_max)
BINS = 66
BYTES_PER_CELL_STEP = 6 * ((N + 7) // 8) + 2      # 194 B at n = 256 (survey_model_frac)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--instances", type=int, default=2048, help="instances per GPU per configuration")
    ap.add_argument("--mode", choices=("spec", "reference"), default="spec")
    ap.add_argument("--f", default="0,1,5,10,21,42,64,85")
    ap.add_argument("--models", default="const,uniform,geometric")
    ap.add_argument("--key-window", type=int, default=8)
    ap.add_argument("--round-cap", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group (and all-reduce the histograms) even at world size 1")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo rehearses ranks sharing one GPU")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    coll_dev = "cuda"
    if world > 1 or args.dist:
        import torch
        import torch.distributed as tdist
        if args.backend == "gloo":
            local %= torch.cuda.device_count()
            coll_dev = "cpu"
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group("gloo")
        dist = tdist
    import configs
    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd import shard
    from byzantinerandomizedconsensus_amd.engine import Engine

    mode = L.MODE_SPEC if args.mode == "spec" else L.MODE_REFERENCE
    first, count = shard.shard_range(args.instances * world, world, rank)
    fvals = [int(x) for x in args.f.split(",") if x != ""]
    for name in args.models.split(","):
        model, dmax = MODELS[name]
        for f in fvals:
            t0 = time.perf_counter()
            with Engine(n=N, f=f, instances=count, protocol="consensus", seed=SEED, delay_model=model,
                        delay_max=dmax, delay_const=1, round_cap=args.round_cap, step_cap=4000,
                        key_window=args.key_window, variants=1, proposals=L.PROPOSALS_PHILOX,
                        instance_offset=first, device=local, mode=mode, coin_seed=COIN_SEED) as eng:
                t1 = time.perf_counter()
                eng.run()
                t2 = time.perf_counter()
                kms = eng.last_kernel_ms()
                kernel = eng.last_kernel()
                st, hist = shard.reduce_stats(eng.stats(), dist, device=coll_dev, hist=eng.round_histogram(BINS))
            wall = shard.max_over_ranks(t2 - t1, dist, device=coll_dev)
            kms = shard.max_over_ranks(kms, dist, device=coll_dev)
            if rank == 0:
                decided = sum(hist[1:])
                mean_r = sum(r * c for r, c in enumerate(hist) if r) / decided if decided else None
                last = max([r for r, c in enumerate(hist) if c] or [0])
                print(json.dumps({
                    "config": "cfg5", "n": N, "f": f, "delay": name, "delay_max": dmax, "mode": args.mode,
                    "key_window": args.key_window, "instances": st["instances"], "n_gpus": world,
                    "decided": decided, "statuses": {k: st[k] for k in ("done", "quiescent", "stepcap", "overflow",
                                                                       "running")},
                    "round_hist": {str(r): c for r, c in enumerate(hist) if c}, "mean_decide_round": mean_r,
                    "max_decide_round": last, "msgs_sent": st["msgs_sent"], "arrivals": st["arrivals"],
                    "cell_steps": st["cell_steps"],
                    # the floor model bench.py and configs.py use: the cell word read + written per
                    # cell-step (16 B on the wide kernel's 8-B cells); SURVEY 8(d)'s 194 B beside it
                    "roofline": configs.roofline("cfg5-sweep", N, BYTES_PER_CELL_STEP, st["cell_steps"] / world, kms,
                                                 kernel=kernel),
                    "kernel": kernel, "collective": (dist.get_backend() + " all-reduce of the histograms")
                    if dist is not None else None,
                    "kernel_ms": kms, "wall_ms": wall * 1e3, "setup_ms": (t1 - t0) * 1e3,
                    "decided_instances_per_s": decided / wall if wall else None}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
