#!/bin/bash
# round 4: key-lifetime kernel with lane-register step statistics and DPP sums -- tests, then A/B on the connection-peer workloads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_life.py > gpurun_out/r4y_tests.log 2>&1 && \
timeout -k 10 900 bash tools/ab_cfg.sh "head vlife2" 3 cfg4-conn,cfg4-conn-uniform-d2 > gpurun_out/r4y_ab.txt 2>&1
