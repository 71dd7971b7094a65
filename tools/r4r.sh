#!/bin/bash
# round 4: per-link key-lifetime kernel -- lifetime tests and the 2^20 connection-peer cases
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_life.py \
    "tests/test_gpu_fullsize.py::test_cfg4_connection_peers_2p20_sampled" > gpurun_out/r4r_tests.log 2>&1
