#!/bin/bash
# round 4: connection-peer workloads after a lifetime-kernel change, then the lifetime tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u configs.py --only cfg4-conn,cfg4-conn-uniform,cfg4-conn-uniform-d2 > gpurun_out/r4t_configs.jsonl 2> gpurun_out/r4t_configs.err && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_life.py > gpurun_out/r4t_tests.log 2>&1
