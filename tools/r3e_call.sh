#!/bin/bash
# round-3 session-3 GPU call 2: wide-kernel profiles (cfg5) and compile-variant A/B on cfg3 / cfg5
set -e
mkdir -p gpurun_out/r3e
bash profiles/collect.sh r3_cfg5_const 0 cfg5-const brc_step_wide > gpurun_out/r3e/collect_const.log 2>&1
tail -1 gpurun_out/r3e/collect_const.log
bash profiles/collect.sh r3_cfg5_geometric 0 cfg5-geometric brc_step_wide > gpurun_out/r3e/collect_geo.log 2>&1
tail -1 gpurun_out/r3e/collect_geo.log
bash tools/ab_cfg.sh "head maxilp" 2 cfg3,cfg5-const,cfg5-geometric
