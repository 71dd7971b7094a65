#!/bin/bash
# round 4: per-link connection-peer lifetime kernel occupancy (6 vs 7 waves/SIMD), lifetime tests on the 6-wave build
set -o pipefail
mkdir -p gpurun_out
BRC_LIB=exp/vpl6/libbrc_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_life.py > gpurun_out/r4ac_tests.log 2>&1 && \
timeout -k 10 900 bash tools/ab_cfg.sh "vpl6 vpl7" 3 cfg4-conn-uniform-d2 > gpurun_out/r4ac_ab.txt 2>&1
