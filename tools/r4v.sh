#!/bin/bash
# round 4: extra-SEND records (one payload SENT by several origins) -- fixture parity, API, rejections; cfg3 timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_workloads.py tests/test_api_shim.py > gpurun_out/r4v_tests.log 2>&1 && \
timeout -k 10 300 python -u configs.py --only cfg2,cfg3 > gpurun_out/r4v_configs.jsonl 2> gpurun_out/r4v_configs.err
