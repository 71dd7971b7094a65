#!/usr/bin/env python3
"""Throughput of every BASELINE.json configuration that runs on the GPU (configs[1..4]), one
JSON line per workload.  bench.py stays the headline (cfg4); this measures the others with the
same clock discipline so DESIGN.md can quote all of them.

    python configs.py [--only cfg2,cfg3,...] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... configs.py
        (cfg2 / cfg3 keep their TOTAL size and shard it; cfg4 / cfg5 are per GPU)

Workloads:
  cfg2       10,000 instances n=4 f=1, honest, uniform delays [1,4], reference protocol
  cfg3       1,000,000 instances n=16 f=5, Byzantine {11..15} equivocating, uniform delays [1,4]
  cfg2-spec, cfg3-spec   the same two in SPEC mode (the reference protocol stalls on most of them)
  cfg4-ref   2^20 instances per GPU n=64 f=21, slow-set delays D=8 (the bench.py workload)
  cfg4-spec  the same in SPEC mode (common coin, phase window 8), 2^20 instances per GPU
  cfg4-conn  the same with connection-identity peers (what the shipped reference runs), 2^20
  cfg4-conn-uniform[-d2]  connection peers under per-link uniform[1,4] ([1,2]) delays, 2^20
  cfg4-beb   the reference consensus over best-effort broadcast (BRC_MODE_BEB), 2^20
  cfg4-ref-r8  the reference protocol to round cap 8 (bench.py's many leg: the key-lifetime kernel), 2^20
  cfg4-ref-r64, cfg4-spec-r64  SURVEY cfg4's round cap 64 (bench.py's long / spec64 legs), 2^20
  cfg4-conn-geometric  connection peers under geometric delays capped at 16 (64-row ring), 2^20
  cfg4-{ref,spec,beb,spec-r64}-2c  the sender-peer cfg4 rows above (which pin the step kernel) on the
             key-lifetime kernel's two-class form, the engine's default for them (slow-set symmetry)
  cfg5-*     n=256 f=85 SPEC, 6144 instances per GPU, const / uniform[1,4] / geometric<=16
  cfg5-conn-uniform  n=256 f=85, connection-identity peers (the reference as shipped), reference
             protocol, uniform[1,4] delays, 6144 instances per GPU (the wide kernel's 40-B cells)

A step is one pass of the hot path over the batch (reset + run to completion); the timed region
is K steps between barriers, max over ranks.  `roofline.achieved` = this layout's algorithmic
bytes (the cell word read + written, 2 x cell bytes per cell-step) x cell-steps per launch /
kernel time; `survey_model_gbs` prices SURVEY §8(d)'s 6*ceil(n/8)+2 B per cell-step instead;
`traffic_frac` and `issue` come from the workload's committed same-build rocprofv3 profile.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
COIN_SEED = 0xC017C017


def workloads(L):
    """name -> (instances, per_gpu, Engine kwargs)"""
    uni, slow = L.DELAY_UNIFORM, L.DELAY_SLOWSET
    base = dict(protocol="consensus", step_cap=4000, proposals=L.PROPOSALS_PHILOX, delay_const=1)
    W = {
        "cfg2": (10000, False, dict(base, n=4, f=1, seed=0x5EED0002, delay_model=uni, delay_max=4, round_cap=1,
                                    key_window=8)),
        "cfg3": (1000000, False, dict(base, n=16, f=5, seed=0x5EED0003, delay_model=uni, delay_max=4, round_cap=1,
                                      key_window=4, variants=2, byz_pattern=L.BYZ_EQUIVOCATE,
                                      byzantine=list(range(11, 16)))),
        # the reference protocol stalls on most cfg2 / cfg3 instances (an early ECHO blocks the SEND,
        # SURVEY K2); the intended protocol terminates on all of them
        "cfg2-spec": (10000, False, dict(base, n=4, f=1, seed=0x5EED0002, delay_model=uni, delay_max=4,
                                         round_cap=1, key_window=8, mode=L.MODE_SPEC, coin_seed=COIN_SEED)),
        "cfg3-spec": (1000000, False, dict(base, n=16, f=5, seed=0x5EED0003, delay_model=uni, delay_max=4,
                                           round_cap=1, key_window=4, variants=2, byz_pattern=L.BYZ_EQUIVOCATE,
                                           byzantine=list(range(11, 16)), mode=L.MODE_SPEC, coin_seed=COIN_SEED)),
        # kernel="step": the step kernel (per-receiver cells, the general path the bench headline measures);
        # the engine's default for these two-class configurations is the key-lifetime kernel (the -2c rows)
        "cfg4-ref": (1 << 20, True, dict(base, n=64, f=21, seed=0x5EED0004, delay_model=slow, delay_max=8,
                                         round_cap=1, key_window=4, kernel="step")),
        "cfg4-spec": (1 << 20, True, dict(base, n=64, f=21, seed=0x5EED0004, delay_model=slow, delay_max=8,
                                          round_cap=1, key_window=8, mode=L.MODE_SPEC, coin_seed=COIN_SEED,
                                          kernel="step")),
    }
    # cfg4 under the peer identity the shipped reference runs (core/brbroadcast.py:69: every message
    # is a new connection, no duplicate suppression; 5-word cells) and over best-effort broadcast
    W["cfg4-conn"] = (1 << 20, True, dict(base, n=64, f=21, seed=0x5EED0004, delay_model=slow, delay_max=8,
                                          round_cap=1, key_window=4, peer_mode=L.PEER_CONNECTION))
    # ... and under per-link uniform delays (the lifetime kernel's per-link form): D = 4 as cfg5's
    # uniform[1,4] (the reference protocol stalls every instance before a decision there), D = 2 (decides)
    for dmax in (4, 2):
        W["cfg4-conn-uniform" + ("" if dmax == 4 else "-d2")] = (
            1 << 20, True, dict(base, n=64, f=21, seed=0x5EED0004, delay_model=1, delay_max=dmax, round_cap=1,
                                key_window=4, peer_mode=L.PEER_CONNECTION))
    W["cfg4-beb"] = (1 << 20, True, dict(base, n=64, f=21, seed=0x5EED0004, delay_model=slow, delay_max=8,
                                         round_cap=1, key_window=8, mode=L.MODE_BEB, kernel="step"))
    # the reference protocol to round cap 8 (bench.py's many leg; the key-lifetime kernel at 2^20)
    W["cfg4-ref-r8"] = (1 << 20, True, dict(base, n=64, f=21, seed=0x5EED0004, delay_model=slow, delay_max=8,
                                            round_cap=8, key_window=32))
    # SURVEY cfg4's round cap 64 (bench.py's long and spec64 legs): the reference protocol on the key-lifetime
    # kernel (key window 128), SPEC on the step kernel (window 8), 2^20 each
    W["cfg4-ref-r64"] = (1 << 20, True, dict(base, n=64, f=21, seed=0x5EED0004, delay_model=slow, delay_max=8,
                                             round_cap=64, key_window=128))
    W["cfg4-spec-r64"] = (1 << 20, True, dict(base, n=64, f=21, seed=0x5EED0004, delay_model=slow, delay_max=8,
                                              round_cap=64, key_window=8, mode=L.MODE_SPEC, coin_seed=COIN_SEED,
                                              kernel="step"))
    # the same sender-peer cfg4 workloads on the key-lifetime kernel's two-class form (the engine's default
    # for them since round 6): a key's lifetime as two receiver-class states, exact under slow-set delays
    for nm in ("cfg4-ref", "cfg4-spec", "cfg4-beb", "cfg4-spec-r64"):
        sz, per, kw = W[nm]
        W[nm + "-2c"] = (sz, per, dict(kw, kernel="life"))
    # connection peers under cfg5's geometric delays capped at 16 (the per-link form's 64-row ring)
    W["cfg4-conn-geometric"] = (1 << 20, True, dict(base, n=64, f=21, seed=0x5EED0004, delay_model=3, delay_max=16,
                                                    round_cap=1, key_window=4, peer_mode=L.PEER_CONNECTION))
    # cfg5's committee with connection-identity peers (the reference as shipped, core/brbroadcast.py:69):
    # the wide kernel's 40-B cells (the cell + two 16-step send-count rings), reference protocol, uniform[1,4]
    W["cfg5-conn-uniform"] = (6144, True, dict(base, n=256, f=85, seed=0x5EED0005, delay_model=1, delay_max=4,
                                               round_cap=1, key_window=4, peer_mode=L.PEER_CONNECTION))
    for name, model, dmax in (("const", 0, 1), ("uniform", 1, 4), ("geometric", 3, 16)):
        # 6,144 instances per GPU: 8 waves of the 768 resident workgroups (3 per CU), so no partial last wave
        W["cfg5-" + name] = (6144, True, dict(base, n=256, f=85, seed=0x5EED0005, delay_model=model,
                                             delay_max=dmax, round_cap=1, key_window=8, mode=L.MODE_SPEC,
                                             coin_seed=COIN_SEED))
    return W


def cell_bytes(n, peer_mode=0):
    """Bytes of one (receiver, key) cell: 4 on the lean kernels (33 <= n <= 64, sender peers:
    brc_internal.h C32_*), 40 with connection peers, 8 on the others."""
    if peer_mode:
        return 40                    # connection peers: the cell + two 16-step send-count rings
    return 4 if 32 < n <= 64 else 8


# configs.py workloads that are bench.py legs: their profiles are the bench's (workload "cfg4", mode = leg)
BENCH_LEGS = {"cfg4-ref": "reference", "cfg4-spec": "spec", "cfg4-conn": "conn", "cfg4-conn-uniform-d2": "connu",
              "cfg4-ref-r8": "many", "cfg4-ref-r64": "long", "cfg4-spec-r64": "spec64", "cfg4-ref-2c": "ref2c",
              "cfg4-spec-2c": "spec2c"}


def measured_profile(name, kernel_ms):
    """The committed rocprofv3 summary of this workload (profiles/*/pmc_traffic.json, written by
    profiles/summarize.py from a configs.py --only <name> run, or the bench.py leg's for the cfg4
    workloads that are bench legs): HBM bytes per launch and the issue block, if its kernel time
    agrees with the live one within 15 % (the same kernel build).  The newest matching profile wins."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_traffic.json")),
                       key=lambda p: os.path.getmtime(p)):
        try:
            with open(path) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        mine = d.get("workload") == name or (name in BENCH_LEGS and d.get("workload") == "cfg4" and
                                               d.get("mode", "reference") == BENCH_LEGS[name] and
                                               d.get("instances") == 1 << 20)
        if not mine or not d.get("avg_ns") or not d.get("hbm_bytes_per_launch"):
            continue
        if abs(d["avg_ns"] / 1e6 - kernel_ms) <= 0.15 * kernel_ms:
            best = dict(d, path=os.path.relpath(path, ROOT))
    return best


def parity_basis(mode, L):
    """What a workload's results are pinned to.  SPEC and BEB rest on the C oracle's
    restatement alone: the reference's coin branch (core/byzantinerandomizedconsensus.py:89-92) is
    unreachable and its BEBroadcast.__init__ raises (core/bebroadcast.py), so no reference run can
    produce their vectors."""
    if mode == L.MODE_SPEC:
        return "C-oracle restatement of the intended protocol only (reference coin branch :89-92 is dead code)"
    if mode == L.MODE_BEB:
        return "C-oracle restatement only (the reference's BEBroadcast cannot be constructed)"
    return "reference-harness fixtures (tests/golden) and the C oracle they pin"


def attach_profile(out, name, kernel_ms):
    prof = measured_profile(name, kernel_ms)
    if prof:
        sec = kernel_ms / 1e3
        out["traffic"], out["traffic_source"] = prof["hbm_bytes_per_launch"], prof["path"]
        out["traffic_frac"] = prof["hbm_bytes_per_launch"] / sec / 1e9 / HBM_PEAK_GBS
        out["profile"] = {"source": prof["path"], "kernel_ms": prof["avg_ns"] / 1e6,
                          "agreement": prof["avg_ns"] / 1e6 / kernel_ms}
        if prof.get("issue"):
            out["issue"] = prof["issue"]
    return out


def roofline(name, n, bpc, cell_steps, kernel_ms, peer_mode=0, kernel="step"):
    """HBM fractions of the dominant kernel, as bench.py reports them: `frac` prices this layout's
    algorithmic bytes (the cell word read + written per cell-step), `survey_model_frac` SURVEY
    §8(d)'s n-bit-mask model, `traffic_frac` the rocprofv3 counters of a committed profile.
    kernel: Engine.last_kernel() of the run -- the key-lifetime kernel ("life") moves no cell bytes,
    so it is reported as issue-bound with no HBM fraction (bench.py does the same)."""
    sec = kernel_ms / 1e3
    if kernel not in ("step", "life"):
        raise ValueError("%s: launches ran different kernels (%r); report them apart" % (name, kernel))
    if kernel == "life":
        out = {"bound": "issue", "kernel": "brc_life", "unit": "GB/s", "peak": HBM_PEAK_GBS, "achieved": None,
               "frac": None, "survey_model_gbs": bpc * cell_steps / sec / 1e9,
               "cell_steps_per_s": cell_steps / sec, "traffic": None, "traffic_frac": None,
               "note": "key-lifetime kernel: cells stay in registers for a key's lifetime, no HBM cell traffic "
                       "(per-link form: one 8-B delivery-bitmap word per lane, key word and step in HBM), so its "
                       "roof is instruction issue: frac = max(VALU busy, SALU per CU-cycle) of the same-build "
                       "profile (bench.py); survey_model_gbs prices SURVEY 8(d)'s %d B per cell-step at n=%d" % (bpc, n)}
        out = attach_profile(out, name, kernel_ms)
        if out.get("issue"):
            out["frac"] = out["achieved"] = max(out["issue"]["valu_busy"], out["issue"]["salu_per_cu_cycle"])
            out["unit"], out["peak"] = "issue-port fraction", 1.0
        return out
    floor_b = 2 * cell_bytes(n, peer_mode)
    achieved = floor_b * cell_steps / sec / 1e9
    out = {"bound": "hbm", "kernel": "brc_step" if n <= 64 else "brc_step_wide", "unit": "GB/s", "peak": HBM_PEAK_GBS,
           "achieved": achieved,
           "frac": achieved / HBM_PEAK_GBS, "bytes_per_unit": floor_b,
           "survey_model_gbs": bpc * cell_steps / sec / 1e9, "cell_bytes": floor_b // 2,
           "traffic": None, "traffic_frac": None,
           "note": "achieved: %d B per cell-step (the %d-B cell read + written); survey_model_gbs prices SURVEY "
                   "8(d)'s %d B at n=%d, which credits n-bit sets this layout never moves (it can exceed the "
                   "peak); traffic_frac: rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE" % (floor_b, floor_b // 2, bpc, n)}
    return attach_profile(out, name, kernel_ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--instances", type=int, default=0, help="override the workloads' instance counts")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist
    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd import shard
    from byzantinerandomizedconsensus_amd.engine import Engine

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    W = workloads(L)
    names = [x for x in args.only.split(",") if x] or list(W)
    for name in names:
        size, per_gpu, kw = W[name]
        size = args.instances or size
        first, count = shard.shard_range(size * world if per_gpu else size, world, rank)
        n = kw["n"]
        bpc = 6 * ((n + 7) // 8) + 2
        kw = dict(kw)
        kernel = kw.pop("kernel", None)             # pin a kernel (BRC_KERNEL, read by brc_create)
        old = os.environ.pop("BRC_KERNEL", None)
        if kernel:
            os.environ["BRC_KERNEL"] = kernel
        try:
            eng = Engine(instances=count, instance_offset=first, device=local, **kw)
        finally:
            os.environ.pop("BRC_KERNEL", None)
            if old is not None:
                os.environ["BRC_KERNEL"] = old
        with eng:
            for _ in range(args.warmup):
                eng.reset()
                eng.run()
            barrier()
            t0 = time.perf_counter()
            kms, kern = [], set()
            for _ in range(args.steps):
                eng.reset()
                eng.run()
                kms.append(eng.last_kernel_ms())
                kern.add(eng.last_kernel())
            barrier()
            elapsed = time.perf_counter() - t0
            st, hist = shard.reduce_stats(eng.stats(), dist, device="cuda", hist=eng.round_histogram(66))
        elapsed = shard.max_over_ranks(elapsed, dist, device="cuda")
        kernel_ms = shard.max_over_ranks(sum(kms) / len(kms), dist, device="cuda")
        kname = next(iter(kern)) if len(kern) == 1 else "mixed"
        if rank == 0:
            print(json.dumps({
                "workload": name, "n": n, "f": kw["f"], "instances": st["instances"], "n_gpus": world,
                "mode": "spec" if kw.get("mode") == L.MODE_SPEC else "reference",
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                "kernel_ms": kernel_ms,
                "decided_instances_per_s": st["decided"] * args.steps / elapsed,
                "instances_per_s": st["instances"] * args.steps / elapsed,
                "replica_message_steps_per_s": st["arrivals"] * args.steps / elapsed,
                "statuses": {k: st[k] for k in ("done", "quiescent", "stepcap", "overflow", "running")},
                "decide_round_hist": {str(r): c for r, c in enumerate(hist) if c},
                "cell_steps_per_launch": st["cell_steps"], "lane_loads_per_launch": st["lane_loads"],
                "kernel": kname,
                "roofline": roofline(name, n, bpc, st["cell_steps"] / world, kernel_ms, kw.get("peer_mode", 0),
                                     kernel=kname),
                "parity": parity_basis(kw.get("mode", L.MODE_REFERENCE), L),
            }), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
