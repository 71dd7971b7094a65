#!/usr/bin/env python3
"""Per kernel instantiation: VGPRs, spills, scratch bytes (compiler resource-usage metadata) and the
number of scratch_* instructions in its ISA, for every HIP unit of the build (dev tool).

    python tools/scratch_count.py [unit.hip ...] > profiles/<tag>/kres.txt
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402


def main():
    units = sys.argv[1:] or G.HIP_UNITS
    flags = [f for f in G.HIP_FLAGS_C if f != "-c"]
    print("%-58s %5s %6s %6s %8s %8s" % ("kernel", "vgpr", "vspill", "sspill", "scratchB", "scratchI"))
    for u in units:
        out = "/tmp/scratch_count.s"
        subprocess.check_call(["hipcc"] + flags + G.UNIT_FLAGS.get(u, []) + ["--cuda-device-only", "-S", "-o", out,
                                                                        os.path.join(G.CSRC, u)],
                              stderr=subprocess.DEVNULL)
        text = open(out).read()
        bodies = {}
        for m in re.finditer(r"^(_ZN3brc\w+):.*?^\s*s_endpgm", text, re.M | re.S):
            bodies[m.group(1)] = len(re.findall(r"^\s*scratch_", m.group(0), re.M))
        for m in re.finditer(r"\.name:\s+(_ZN3brc\w+)\n(.*?)\.wavefront_size", text, re.S):
            meta = m.group(2)
            get = lambda k: int(re.search(r"\." + k + r":\s+(\d+)", meta).group(1))  # noqa: E731
            name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
            name = name.replace("brc::", "").replace("(brc::Params const*)", "")
            print("%-58s %5d %6d %6d %8d %8d" % (name[:58], get("vgpr_count"), get("vgpr_spill_count"),
                                                get("sgpr_spill_count"), get("private_segment_fixed_size"),
                                                bodies.get(m.group(1), -1)))


if __name__ == "__main__":
    main()
