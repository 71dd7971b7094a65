#!/bin/bash
# round 4: host-managed extra-SEND records -- parity / workloads / API tests, then cfg3 A/B against the value-id build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_workloads.py tests/test_api_shim.py > gpurun_out/r4w_tests.log 2>&1 && \
timeout -k 10 600 bash tools/ab_cfg.sh "head v822" 3 cfg3,cfg3-spec > gpurun_out/r4w_ab.txt 2>&1
