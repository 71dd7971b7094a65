#!/bin/bash
# round 4: connection-peer workloads (two-class and per-link lifetime kernel) + profile of the per-link form
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u configs.py --only cfg4-conn,cfg4-conn-uniform,cfg4-conn-uniform-d2 > gpurun_out/r4s_configs.jsonl 2> gpurun_out/r4s_configs.err && \
timeout -k 10 900 bash profiles/collect.sh r4_connu 0 cfg4-conn-uniform-d2 brc_life > gpurun_out/r4s_collect.log 2>&1
