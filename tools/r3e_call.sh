#!/bin/bash
# round-3 GPU call: wide-kernel profiles (cfg5 const / geometric) and every BASELINE workload on the final build
set -e
mkdir -p gpurun_out/r3e
bash profiles/collect.sh r3_cfg5_const 0 cfg5-const brc_step_wide > gpurun_out/r3e/collect_const.log 2>&1
tail -1 gpurun_out/r3e/collect_const.log
bash profiles/collect.sh r3_cfg5_geometric 0 cfg5-geometric brc_step_wide > gpurun_out/r3e/collect_geo.log 2>&1
tail -1 gpurun_out/r3e/collect_geo.log
timeout -k 10 600 python3 configs.py --steps 2 --warmup 1 > gpurun_out/r3e/configs.jsonl 2> gpurun_out/r3e/configs.err
