#!/usr/bin/env python3
"""Build an A/B variant of libbrc_hip.so with extra compile flags (dev tool, not the product build).

    python tools/variant.py <tag> [--units u1.hip,u2.hip] [-DFLAG=V ...]   ->  ab/<tag>/libbrc_hip.so

--units: compile only these translation units with the flags and link the in-tree objects
(byzantinerandomizedconsensus_amd/build/*.o, from __graft_entry__.build()) for the others.

ab/ is git-ignored but travels to the GPU box with gpurun; select a variant there with
BRC_LIB=ab/<tag>/libbrc_hip.so (byzantinerandomizedconsensus_amd/_lib.py).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402


def main():
    tag, flags = sys.argv[1], sys.argv[2:]
    units = G.HIP_UNITS
    if flags[:1] == ["--units"]:
        units, flags = flags[1].split(","), flags[2:]
    out = os.path.join(ROOT, "ab", tag)
    os.makedirs(out, exist_ok=True)
    procs, objs, mine = [], [], []
    for unit in G.HIP_UNITS:
        if unit not in units:
            objs.append(os.path.join(G.OBJ_DIR, unit.replace(".hip", ".o")))
            continue
        obj = os.path.join(out, unit.replace(".hip", ".o"))
        objs.append(obj)
        mine.append(obj)
        procs.append(subprocess.Popen(["hipcc"] + G.HIP_FLAGS_C + G.UNIT_FLAGS.get(unit, []) + flags +
                                      ["-o", obj, os.path.join(G.CSRC, unit)],
                                      cwd=ROOT))
    if any(p.wait() for p in procs):
        sys.exit("hipcc failed")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                           os.path.join(out, "libbrc_hip.so")] + objs, cwd=ROOT)
    for o in mine:
        os.remove(o)
    print(os.path.join(out, "libbrc_hip.so"))


if __name__ == "__main__":
    main()
