#!/bin/bash
# round 4: key-lifetime kernel totals in a lane-distributed register (variant exp/vacc) -- lifetime tests on it, then A/B against HEAD
set -o pipefail
mkdir -p gpurun_out
BRC_LIB=exp/vacc/libbrc_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_life.py > gpurun_out/r4aa_tests.log 2>&1 && \
timeout -k 10 900 bash tools/ab_cfg.sh "head vacc" 3 cfg4-conn,cfg4-conn-uniform-d2 > gpurun_out/r4aa_ab.txt 2>&1
