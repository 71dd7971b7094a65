#!/usr/bin/env python3
"""Headline benchmark: decided consensus instances/sec at n=64, f=21 (BASELINE.json configs[3]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--instances I] [--legs reference,spec]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (multi-GPU)

Workload: 64 replicas, f = 21, adversarial delays (messages from/to a
per-instance slow set of f replicas take D = 8 steps, all others 1), Philox Bernoulli(1/2)
proposals, 2^20 instances per GPU.  One "step" = one full pass of the hot path over the batch:
every instance simulated from its proposals until every honest replica has decided (the
reference's decide() upcall, core/byzantinerandomizedconsensus.py:94).  Instances are
independent, so ranks shard them (global Philox ids => results independent of N: weak
scaling); the only collective is one RCCL all-reduce of the statistics.

Legs, one JSON line (rank 0); each leg is one launch per step at 2^20 instances:
  reference  the protocol exactly as the reference runs it (quirks included) -- the headline
             `value`, on the step kernel (per-receiver cells: the general path).  Its coin branch is dead, so split proposals decide "-1" in
             round 1; `decided_value_hist` shows that share.
  spec       the protocol the reference intends, with the common coin made reachable (SURVEY §8
             F3): "many coin rounds".  Its phase window Q = 8 doubles the key slots; with 4-B cells
             2^20 instances still fit one engine (138 GB of cells).  Larger counts run as tiles of
             an engine re-keyed per tile (brc_reset_at); the statistics then come from one extra
             untimed pass.
  conn       connection-identity peers (core/brbroadcast.py:69, what the shipped reference runs;
             SURVEY §8 F1), slow-set delays: the key-lifetime kernel's two-class form.
  connu      connection peers under per-link uniform[1,2] delays: its per-link form.
  many       the reference protocol run to round cap 8 (SURVEY cfg4's "many rounds"): by round 8
             ~1,000 keys of one instance are live at once (phase leakage), more than any cell store
             holds at 2^20, so the engine runs it on the key-lifetime kernel (key window 32).
  long       the reference protocol to SURVEY cfg4's round cap 64 (key window 128: ~7,600 keys of one
             instance live at once by round 64), key-lifetime kernel, 2^20 instances in one launch.
  spec64     SPEC to round cap 64: 64 decisions per replica, coin rounds included, step kernel.
  ref2c      the reference leg's workload on the key-lifetime kernel's two-class form: under slow-set
             delays a key's honest receivers of one class evolve identically, so the kernel simulates a
             key's whole lifetime as two class states, one key per lane (csrc/brc_life.h).  Exact for
             this delay model only (the engine's default kernel for it, same results as the step kernel:
             tests/test_gpu_fullsize.py); the headline stays on the general step kernel.
  spec2c     the spec leg's workload on the same two-class form.
The legs of seconds per step (many, long, spec64) time at most LEG_STEPS of --steps / --warmup
and report the counts they timed.
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
CELL_BYTES = 4                                                  # lean kernels' compact cell (brc_internal.h C32_*)
FLOOR_BYTES_PER_CELL_STEP = 2 * CELL_BYTES                      # this layout: the cell word read + written
HBM_PEAK_GBS = 8000.0                                           # MI355X_MICROARCH.md
SPEC_TILE = 1 << 20                                             # SPEC (Q = 8) instances per engine tile
MANY_CAP = 8                                                    # the many leg's round cap
LONG_CAP = 64                                                   # SURVEY cfg4's round cap (long, spec64 legs)
# leg -> (protocol mode, peer mode, delay model, delay max, key window, kernel).  kernel: "step" pins the
# step kernel (per-receiver cells, any delay model: the general path the headline measures), "life" the
# key-lifetime kernel, None the engine's own choice (include/brc.h brc_last_kernel)
LEGS = {"reference": ("reference", "sender", "slowset", DELAY_MAX, 4, "step"),
        "spec": ("spec", "sender", "slowset", DELAY_MAX, 8, "step"),
        "conn": ("reference", "connection", "slowset", DELAY_MAX, 4, None),
        "connu": ("reference", "connection", "uniform", 2, 4, None),
        "many": ("reference", "sender", "slowset", DELAY_MAX, 32, None),
        "long": ("reference", "sender", "slowset", DELAY_MAX, 128, None),
        "spec64": ("spec", "sender", "slowset", DELAY_MAX, 8, "step"),
        "ref2c": ("reference", "sender", "slowset", DELAY_MAX, 4, "life"),
        "spec2c": ("spec", "sender", "slowset", DELAY_MAX, 8, "life")}
# legs with a round cap of their own (the others take --round-cap)
LEG_CAP = {"many": MANY_CAP, "long": LONG_CAP, "spec64": LONG_CAP}
# legs of seconds per step time at most this many (steps, warmup) of --steps / --warmup, so that the default
# run stays within minutes; every leg reports the steps it timed
LEG_STEPS = {"many": (3, 1), "long": (1, 0), "spec64": (1, 0)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--instances", type=int, default=1 << 20, help="instances per GPU (SURVEY §8(d) cfg4: 2^20)")
    ap.add_argument("--legs", default="reference,spec,conn,connu,many,long,spec64,ref2c,spec2c",
                    help="comma list of reference (the headline value), spec (SURVEY §8 F3 coin rounds), conn "
                         "(connection-identity peers, what the shipped reference runs: SURVEY §8 F1), connu (the same "
                         "under per-link uniform[1,2] delays), many (the reference protocol to round cap 8), long (the "
                         "reference protocol to SURVEY cfg4's round cap 64), spec64 (SPEC to round cap 64), ref2c / "
                         "spec2c (reference / spec on the key-lifetime kernel's two-class form)")
    ap.add_argument("--mode", choices=tuple(LEGS), default=None,
                    help="shorthand for --legs <mode> (the headline leg is the first one run)")
    ap.add_argument("--round-cap", type=int, default=1, help="round cap of every leg but many")
    ap.add_argument("--many-cap", type=int, default=MANY_CAP, help="round cap of the many leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="collective backend for N > 1: nccl (= RCCL over xGMI, one GPU per rank); gloo "
                         "only rehearses the multi-rank flow with several ranks sharing one GPU")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group (and run the statistics all-reduce) even at world size 1, "
                         "e.g. one RCCL rank under torch.distributed.run --nproc-per-node 1")
    a = ap.parse_args()
    a.legs = [a.mode] if a.mode else [x for x in a.legs.split(",") if x]
    return a


def cpu_baseline(seconds, leg="reference", round_cap=1):
    """The C oracle (a scalar port of the reference's path) on the same workload, one thread per
    core (ctypes releases the GIL inside the C run): threads take interleaved global instance ids
    from 0 and run until `seconds` have passed.  Counters only (the oracle's light mode)."""
    mode, peer, model, dmax, window, _kernel = LEGS[leg]
    import concurrent.futures
    from oracle import oracle
    from tests.golden import specs as S
    threads = max(1, min(16, os.cpu_count() or 1))    # the GPU box's CPU share is 16

    dm = {"slowset": 2, "uniform": 1}[model]

    def spec(g):
        if mode == "spec":
            return S.spec_cons_spec(N_REPLICAS, F_FAULTS, SEED, dm, dmax, g, round_cap=round_cap,
                                    window=window, coin_seed=COIN_SEED)
        return S.cons_spec(N_REPLICAS, F_FAULTS, SEED, dm, dmax, g, round_cap=round_cap, peer_mode=peer)

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


def load_profile(instances, kernel_ms, mode="reference", cell_bytes=CELL_BYTES):
    """The committed rocprofv3 summary of this leg (profiles/pmc_traffic.json for the reference leg,
    profiles/pmc_traffic_<leg>.json for the others, written by profiles/summarize.py): HBM bytes per
    launch and the instruction-issue block.  Used only if it was taken on this workload, size and
    kernel (cell_bytes: 4 for the step kernel's compact cells, 0 for the key-lifetime kernel, which
    keeps no cells) and its kernel time agrees with the live one within 15 % (the same kernel
    build); the agreement is reported beside it."""
    name = "pmc_traffic.json" if mode == "reference" else "pmc_traffic_%s.json" % mode
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("instances") != instances or d.get("workload") != "cfg4" or not d.get("avg_ns") or \
            d.get("mode", "reference") != mode or d.get("cell_bytes", 8) != cell_bytes:
        return None
    if abs(d["avg_ns"] / 1e6 - kernel_ms) > 0.15 * kernel_ms:
        return None
    return d


def make_engine(leg, count, first, device, round_cap):
    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd.engine import Engine
    mode, peer, model, dmax, window, kernel = LEGS[leg]
    spec = mode == "spec"
    old = os.environ.pop("BRC_KERNEL", None)       # read by brc_create only
    if kernel:
        os.environ["BRC_KERNEL"] = kernel
    try:
        return Engine(n=N_REPLICAS, f=F_FAULTS, instances=count, protocol="consensus", seed=SEED,
                      delay_model={"slowset": L.DELAY_SLOWSET, "uniform": L.DELAY_UNIFORM}[model], delay_max=dmax,
                      round_cap=round_cap, step_cap=4000, key_window=window, variants=1, proposals=L.PROPOSALS_PHILOX,
                      instance_offset=first, device=device, mode=L.MODE_SPEC if spec else L.MODE_REFERENCE,
                      coin_seed=COIN_SEED, peer_mode=L.PEER_CONNECTION if peer == "connection" else L.PEER_SENDER)
    finally:
        os.environ.pop("BRC_KERNEL", None)
        if old is not None:
            os.environ["BRC_KERNEL"] = old


def collect(eng):
    """This engine's statistics, round histogram and decided values (one dict)."""
    st = eng.stats()
    hist = eng.round_histogram(66)
    vals, dis = eng.decisions()
    for k, v in vals.items():
        st["dec_" + k] = v
    st["disagreements"] = dis
    return st, hist


def add_stats(a, b):
    if a is None:
        return dict(b[0]), list(b[1])
    st = {k: (max(a[0][k], v) if k == "max_t" else a[0].get(k, 0) + v) for k, v in b[0].items()}
    return st, [x + y for x, y in zip(a[1], b[1])]


def run_leg(args, mode, world, rank, local, dist, coll_dev):
    """Time one leg (K steps after W warmups, barrier + sync on both sides, max over ranks)."""
    from byzantinerandomizedconsensus_amd import shard
    per = args.instances
    first, count = shard.shard_range(per * world, world, rank)     # global instance ids of this rank
    tile = min(count, SPEC_TILE) if LEGS[mode][0] == "spec" else count
    tiles = [(first + o, min(tile, count - o)) for o in range(0, count, tile)]
    cap = args.many_cap if mode == "many" else LEG_CAP.get(mode, args.round_cap)
    eng = make_engine(mode, tiles[0][1], tiles[0][0], local, cap)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    def one_step():
        kms = 0.0
        for off, cnt in tiles:
            if cnt != tiles[0][1]:
                raise RuntimeError("uneven tiles: %d instances per GPU is not a multiple of %d" % (count, tile))
            eng.reset_at(off)
            eng.run()
            kms += eng.last_kernel_ms()
            kern.add(eng.last_kernel())
        return kms

    kern = set()

    steps, warmup = args.steps, args.warmup
    if mode in LEG_STEPS:
        steps, warmup = min(steps, LEG_STEPS[mode][0]), min(warmup, LEG_STEPS[mode][1])
    for _ in range(warmup):
        one_step()
    barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(steps):
        kms.append(one_step())
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(kms) / len(kms)          # all tiles of one step (= one launch per tile)
    if len(tiles) == 1:
        acc = collect(eng)                   # the last timed step's results
    else:                                    # one more (untimed) pass reads every tile's results
        acc = None
        for off, cnt in tiles:
            eng.reset_at(off)
            eng.run()
            acc = add_stats(acc, collect(eng))
    eng.close()
    kernel = kern.pop() if len(kern) == 1 else "mixed"
    st, hist = shard.reduce_stats(acc[0], dist, device=coll_dev, hist=acc[1])
    elapsed = shard.max_over_ranks(elapsed, dist, device=coll_dev)
    kernel_ms = shard.max_over_ranks(kernel_ms, dist, device=coll_dev)
    decided, arrivals, cell_steps = st["decided"], st["arrivals"], st["cell_steps"]
    bad = st["overflow"] + st["stepcap"] + st["running"]
    if bad:      # a leg whose instances did not all finish measures nothing: fail the run
        raise SystemExit("%s leg: %d instances did not finish cleanly (overflow %d, stepcap %d, running %d)"
                         % (mode, bad, st["overflow"], st["stepcap"], st["running"]))
    launches = len(tiles)
    cs_gpu = cell_steps / world
    secs = kernel_ms / 1e3
    if kernel not in ("step", "life"):
        raise SystemExit("%s leg: the launches ran different kernels (%s); its roofline cannot be priced" % (mode, kernel))
    prof = load_profile(per, kernel_ms, mode, CELL_BYTES if kernel == "step" else 0) if launches == 1 else None
    traffic = prof.get("hbm_bytes_per_launch") if prof else None
    if kernel == "life":
        # the key-lifetime kernel (csrc/brc_life.h) keeps a key's cells in registers for its whole
        # lifetime: no cell bytes move, HBM carries only the per-instance results.  Its roof is
        # instruction issue: frac = the busier of the two issue ports, from the same-build PMC
        iss = prof.get("issue") if prof else None
        frac = max(iss["valu_busy"], iss["salu_per_cu_cycle"]) if iss else None
        roof = {"bound": "issue", "kernel": "brc_life", "achieved": frac, "peak": 1.0,
                "unit": "issue-port fraction", "frac": frac, "traffic": traffic,
                "traffic_frac": (traffic / secs / 1e9 / HBM_PEAK_GBS) if traffic else None,
                "survey_model_gbs": SURVEY_BYTES_PER_CELL_STEP * cs_gpu / secs / 1e9,
                "cell_steps_per_s": cs_gpu / secs, "cell_bytes": 0, "units_per_launch": cs_gpu / launches,
                "note": "no HBM cell traffic (cells stay in registers for a key's lifetime), so the roof is "
                        "instruction issue: frac = max(VALU busy, SALU per CU-cycle) of the same-build rocprofv3 "
                        "PMC (roofline.profile.source): VALU busy = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x "
                        "cycles), SALU = SQ_INSTS_SALU / (256 CUs x cycles), cycles = GRBM_GUI_ACTIVE / 8 "
                        "(profiles/summarize.py issue_block); null when no profile of this build agrees with the "
                        "live kernel time; survey_model_gbs prices SURVEY 8(d)'s %d B per cell-step (bytes this "
                        "kernel never moves)" % SURVEY_BYTES_PER_CELL_STEP}
    else:
        # algorithmic bytes of THIS layout: the 4-B cell word read + written per cell-step
        achieved = FLOOR_BYTES_PER_CELL_STEP * cs_gpu / secs / 1e9
        survey = SURVEY_BYTES_PER_CELL_STEP * cs_gpu / secs / 1e9
        roof = {"bound": "hbm", "kernel": "brc_step", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "traffic_frac": (traffic / secs / 1e9 / HBM_PEAK_GBS) if traffic else None,
                "survey_model_gbs": survey, "cell_bytes": CELL_BYTES,
                "bytes_per_unit": FLOOR_BYTES_PER_CELL_STEP, "units_per_launch": cs_gpu / launches,
                "note": "achieved = %d B (the %d-B cell word read + written) x %d cell-steps per GPU per step (%d "
                        "launch%s) / kernel time; traffic = rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE per launch "
                        "(profiles/pmc_traffic*.json); survey_model_gbs prices SURVEY 8(d)'s %d B per cell-step, which "
                        "credits n-bit ECHO/READY masks this design never moves (so it can exceed the peak)"
                        % (FLOOR_BYTES_PER_CELL_STEP, CELL_BYTES, cs_gpu, launches, "" if launches == 1 else "es",
                           SURVEY_BYTES_PER_CELL_STEP)}
    if prof:
        # the same-build profile: its kernel time beside the live one, and its issue view (VALU busy,
        # SALU per CU-cycle, wave-cycle split) -- these kernels are issue- and latency-bound
        roof["profile"] = {"source": prof.get("source"), "kernel_ms": prof["avg_ns"] / 1e6,
                           "agreement": prof["avg_ns"] / 1e6 / kernel_ms}
        if prof.get("issue"):
            roof["issue"] = prof["issue"]
    leg = {
        "value": decided * steps / elapsed,
        "ms_per_step": elapsed / steps * 1e3,
        "steps": steps,
        "warmup": warmup,
        "kernel_ms": kernel_ms,
        "launches_per_step": launches,
        "decided_fraction": decided / float(per * world),
        "decide_round_hist": {str(r): c for r, c in enumerate(hist) if c},
        "decided_value_hist": {k: st["dec_" + k] for k in ("-1", "0", "1", "3", "undecided") if st["dec_" + k]},
        "agreement_violations": st["disagreements"],
        "replica_message_steps_per_s": arrivals * steps / elapsed,
        "counts": {k: st[k] for k in ("instances", "decided", "msgs_sent", "arrivals", "cell_steps", "deliveries",
                                      "decide_rounds_sum", "lane_loads", "max_t")},
        "roofline": roof,
        "kernel": kernel,
        "workload": workload_name(mode, cap, per),
        "round_cap": cap,
        "parity": parity_basis(mode),
    }
    return leg


def parity_basis(leg):
    """What the leg's results are pinned to: the reference protocol's legs to the reference
    itself (reference-harness fixtures + the C oracle pinned by them); SPEC to the oracle's restatement
    of the intended protocol only -- the reference's coin branch (core/byzantinerandomizedconsensus.py:
    89-92) is unreachable, so no reference run can produce a SPEC vector."""
    if LEGS[leg][0] == "spec":
        return ("C-oracle restatement of the intended protocol only (the reference's coin branch, "
                "core/byzantinerandomizedconsensus.py:89-92, is dead code): parity pinned by the restatement, "
                "not by reference fixtures")
    return ("reference-harness fixtures (tests/golden, the unmodified reference classes) and the C oracle they "
            "pin; 2^20 batch oracle-sampled in tests/test_gpu_fullsize.py")


def workload_name(leg, cap, per):
    proto, peer, model, dmax, window, kernel = LEGS[leg]
    form = ""
    if kernel == "step":
        form = ", step kernel (per-receiver cells: the general path, any delay model)"
    elif kernel == "life" and peer == "sender" and model == "slowset":
        form = (", key-lifetime kernel, two-class form (slow-set symmetry: a key's lifetime as two receiver-class "
                "states, exact for this delay model only)")
    if peer == "connection":
        # the key-lifetime kernel's two forms (csrc/brc_life.h): under slow-set delays the receivers of one
        # class see the same arrivals, so it counts them once per class -- exact for that model only
        form = (", two-class arrival counts (slow-set symmetry: counted once per receiver class)" if model == "slowset"
                else ", per-link arrival counts (the general form)")
    return "cfg4: n=64 f=21 %s consensus to %s, %s, %s peers%s, key window %d, %d instances/GPU" % (
        "SPEC-protocol (common coin)" if proto == "spec" else "reference-protocol",
        "first decision" if cap == 1 else "%d decisions" % cap,
        "slow-set delays D=%d" % dmax if model == "slowset" else "per-link uniform[1,%d] delays" % dmax,
        "connection-identity (core/brbroadcast.py:69)" if peer == "connection" else "sender-identity",
        form, window, per)


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
        if args.backend == "gloo":                  # rehearsal: ranks may share a GPU
            local %= torch.cuda.device_count()
            coll_dev = "cpu"
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group("gloo")
        dist = tdist

    legs = {mode: run_leg(args, mode, world, rank, local, dist, coll_dev) for mode in args.legs}
    head_mode = args.legs[0]
    head = legs[head_mode]
    out = None
    if rank == 0:
        out = {
            "metric": "decided consensus instances/sec (node) at n=64,f=21",
            "value": head["value"],
            "unit": "instances/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (Philox4x32-10 proposals and slow sets, seed 0x5EED0004)",
            "config": {"workload": head["workload"], "n": N_REPLICAS, "f": F_FAULTS,
                       "instances_per_gpu": args.instances, "round_cap": head["round_cap"],
                       "round_cap_meaning": "an instance is done when every honest replica has decided this many "
                                            "times (the run stops at that decision, not a give-up bound)",
                       "mode": head_mode,
                       "key_window": LEGS[head_mode][4],
                       "peer_mode": LEGS[head_mode][1],
                       "parallelism": "instance-sharded x%d" % world},
            "collective": (dist.get_backend() + " all-reduce of the statistics") if dist is not None else None,
        }
        for k in ("kernel", "kernel_ms", "decided_fraction", "decide_round_hist", "decided_value_hist",
                  "agreement_violations", "replica_message_steps_per_s", "counts", "roofline", "parity"):
            out[k] = head[k]
        for mode, leg in legs.items():
            if mode != head_mode:
                out[mode + "_leg"] = leg
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_seconds > 0:     # N = 1 only
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, head_mode, head["round_cap"])
    if rank == 0 and head_mode == "reference" and args.round_cap == 1:
        # the reference's own Python path cannot travel to the GPU box: its rate on this workload was
        # measured in the build container (tools/ref_cpu_rate.py) and is reported beside, not as, the baseline
        try:
            with open(os.path.join(ROOT, "profiles", "ref_cpu_rate.json")) as fh:
                r = json.load(fh)
            out["reference_python_rate"] = {
                "value": r["per_core_instances_per_s"], "unit": "decided instances/s per core",
                "cores": 1, "sample": "%d cfg4 instances, one process per core, %s CPUs, Python %s" % (
                    r["instances"], r["cpus_visible"], r["python"]),
                "source": "profiles/ref_cpu_rate.json (build container, not this host)"}
        except (OSError, ValueError, KeyError):
            pass
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
