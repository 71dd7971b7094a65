#!/bin/bash
# round-4 GPU call d: lean GPU tests on the u32 key-list build; A/B 5 vs 4 waves/SIMD vs the last measured builds
set -e
mkdir -p gpurun_out/r4d
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lean_cells.py tests/test_gpu_fullsize.py tests/test_gpu_life.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4d/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4d/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4d/gpu_tests.log
BRC_LIB=exp/w4/libbrc_hip.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lean_cells.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4d/gpu_tests_w4.log 2>&1 || { tail -30 gpurun_out/r4d/gpu_tests_w4.log; exit 1; }
tail -1 gpurun_out/r4d/gpu_tests_w4.log
bash tools/ab.sh "head w4 prev" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head w4 prev" 1 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
