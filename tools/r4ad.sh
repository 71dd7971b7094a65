#!/bin/bash
# round 4 final: rocprofv3 trace + PMC of the per-link connection-peer workload at 6 waves/SIMD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 bash profiles/collect.sh r4_final_connu 0 cfg4-conn-uniform-d2 brc_life > gpurun_out/r4ad_collect.log 2>&1
