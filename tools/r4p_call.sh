#!/bin/bash
# round-4 final profiles, part 1: rocprofv3 trace + PMC passes of the reference and SPEC legs (same build)
set -e
mkdir -p gpurun_out/r4p
bash profiles/collect.sh r4f 1048576 reference > gpurun_out/r4p/collect_ref.log 2>&1 || { tail -20 gpurun_out/r4p/collect_ref.log; exit 1; }
tail -1 gpurun_out/r4p/collect_ref.log
bash profiles/collect.sh r4f_spec 1048576 spec > gpurun_out/r4p/collect_spec.log 2>&1 || { tail -20 gpurun_out/r4p/collect_spec.log; exit 1; }
tail -1 gpurun_out/r4p/collect_spec.log
