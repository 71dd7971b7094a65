#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run into committed JSON.

    python profiles/summarize.py gpurun_out/prof_<tag> profiles/<tag> [--kernel brc_step]

Writes <dest>/kernel_stats.csv (the rocprofv3 --stats table, copied), <dest>/pmc_summary.json
(per-kernel mean of every PMC counter over its dispatches) and, for the headline kernel,
profiles/pmc_traffic.json (profiles/pmc_traffic_spec.json for the SPEC leg), which bench.py
reads for roofline.traffic.

HBM bytes follow MI355X_MICROARCH.md (rocprofv3 / HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB and come from separate --pmc passes; on gfx950 FETCH_SIZE reports half the bytes of a
coalesced streaming read, so it is doubled.  The kernel's cell loads are coalesced wave
accesses of one cell per lane (8 B until r2e, 4 B since), where the doubling is checked against
SQ_INSTS_VMEM_RD x 64 x cell bytes.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def load_counters(src):
    per = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(path)):
            per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


CUS, SIMDS, XCDS = 256, 1024, 8          # MI355X_MICROARCH.md chip parameters


def issue_block(k):
    """Instruction-issue view of one kernel from its PMC means (the kernels here are issue- and
    latency-bound, not HBM-bound): VALU busy = SQ_INSTS_VALU x 2 cycles (a wave64 op on a SIMD-32)
    over SIMDs x cycles, with cycles = GRBM_GUI_ACTIVE / 8 (summed over the XCDs); SALU and branch
    instructions per CU-cycle; the wave-cycle split (SQ_WAVE_CYCLES and SQ_WAIT_* count quad-cycles)
    and the mean resident waves per SIMD."""
    need = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE")
    if not all(c in k for c in need) or not k["GRBM_GUI_ACTIVE"]:
        return None
    cyc = k["GRBM_GUI_ACTIVE"] / XCDS
    out = {"cycles": cyc, "valu_insts": k["SQ_INSTS_VALU"], "salu_insts": k["SQ_INSTS_SALU"],
           "valu_busy": k["SQ_INSTS_VALU"] * 2.0 / (SIMDS * cyc),
           "salu_per_cu_cycle": k["SQ_INSTS_SALU"] / (CUS * cyc)}
    if "SQ_INSTS_BRANCH" in k:
        out["branch_per_cu_cycle"] = k["SQ_INSTS_BRANCH"] / (CUS * cyc)
    if "SQ_INSTS_LDS" in k:
        out["lds_insts"] = k["SQ_INSTS_LDS"]
    wc = k.get("SQ_WAVE_CYCLES")
    if wc:
        out["waves_per_simd"] = wc * 4.0 / cyc / SIMDS
        for c, name in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_frac"),
                        ("SQ_ACTIVE_INST_ANY", "active_frac")):
            if c in k:
                out[name] = k[c] / wc
    return out


def kernel_avg_ns(src, kernel):
    path = os.path.join(src, "trace", "run_kernel_stats.csv")
    for r in csv.DictReader(open(path)):
        if r["Name"] == kernel:
            return float(r["AverageNs"]), int(r["Calls"])
    return None, 0


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    kernel = "brc_step"
    if "--kernel" in sys.argv:
        kernel = sys.argv[sys.argv.index("--kernel") + 1]
        args.remove(kernel)
    src, dest = args[0], args[1]
    os.makedirs(dest, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dest, "kernel_stats.csv"))
    counters = load_counters(src)
    with open(os.path.join(dest, "pmc_summary.json"), "w") as fh:
        json.dump(counters, fh, indent=1, sort_keys=True)
    bench = None
    bpath = os.path.join(src, "trace_bench.json")
    if os.path.exists(bpath):
        bench = json.loads(open(bpath).read().strip().splitlines()[-1])
        shutil.copy(bpath, os.path.join(dest, "trace_bench.json"))
    k = counters.get(kernel, {})
    avg_ns, calls = kernel_avg_ns(src, kernel)
    out = {"kernel": kernel, "avg_ns": avg_ns, "calls": calls, "source": dest, "issue": issue_block(k)}
    if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
        fetch = 2.0 * k["FETCH_SIZE"] * 1024.0
        write = k["WRITE_SIZE"] * 1024.0
        out.update({"fetch_bytes": fetch, "write_bytes": write, "hbm_bytes_per_launch": fetch + write,
                    "hbm_gbs": (fetch + write) / avg_ns if avg_ns else None})
        if "SQ_INSTS_VMEM_RD" in k:
            wave_bytes = 64.0 * (bench or {}).get("roofline", {}).get("cell_bytes", 8)   # one cell per lane
            out["vmem_rd_bytes_issued"] = k["SQ_INSTS_VMEM_RD"] * wave_bytes
            out["vmem_wr_bytes_issued"] = k.get("SQ_INSTS_VMEM_WR", 0.0) * wave_bytes
    if bench and "config" not in bench:             # a configs.py workload line
        out["workload"], out["mode"] = bench.get("workload"), bench.get("mode")
        out["instances"], out["bench_kernel_ms"] = bench.get("instances"), bench.get("kernel_ms")
        out["headline"] = False
    elif bench:
        cfg = bench.get("config", {})
        out["instances"] = cfg.get("instances_per_gpu")
        out["workload"] = cfg.get("workload", "").split(":")[0]
        out["mode"] = cfg.get("mode", "reference")
        out["bench_kernel_ms"] = bench.get("kernel_ms")
        out["cell_bytes"] = bench.get("roofline", {}).get("cell_bytes", 8)
    # the bench reads profiles/pmc_traffic.json for its reference leg, pmc_traffic_<mode>.json for the others
    paths = [os.path.join(dest, "pmc_traffic.json")]
    if out.get("headline", True):
        mode = out.get("mode", "reference")
        name = "pmc_traffic.json" if mode == "reference" else "pmc_traffic_%s.json" % mode
        paths.append(os.path.join(os.path.dirname(dest.rstrip("/")), name))
    for path in paths:
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
