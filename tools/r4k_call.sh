#!/bin/bash
# round-4 GPU call k: lean GPU tests; A/B of the key-list look-ahead + tracked ring rows + busy masks +
# parallel row clears (head) vs serial row clears (noclr) vs 8d7cab7 (last); stamps
set -e
mkdir -p gpurun_out/r4k
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lean_cells.py tests/test_gpu_fullsize.py tests/test_gpu_life.py tests/test_gpu_spec.py tests/test_gpu_beb.py tests/test_gpu_workloads.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r4k/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4k/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4k/gpu_tests.log
bash tools/ab.sh "head noclr last" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head last" 1 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
BRC_LIB=exp/stamps/libbrc_hip.so timeout -k 10 120 python3 tools/stamps.py 262144 reference > gpurun_out/r4k/stamps_reference.txt 2>&1
cat gpurun_out/r4k/stamps_reference.txt
