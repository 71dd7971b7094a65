#!/bin/bash
# round-4 GPU call b: lean-path GPU tests on the split-bulk consensus build, A/B vs the round-3 build, stamps split
set -e
mkdir -p gpurun_out/r4b
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lean_cells.py tests/test_gpu_fullsize.py tests/test_gpu_life.py tests/test_gpu_spec.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4b/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4b/gpu_tests.log
bash tools/ab.sh "head base" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
BRC_LIB=exp/stamps/libbrc_hip.so timeout -k 10 120 python3 tools/stamps.py 262144 reference > gpurun_out/r4b/stamps_reference.txt 2>&1
cat gpurun_out/r4b/stamps_reference.txt
