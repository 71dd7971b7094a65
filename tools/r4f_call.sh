#!/bin/bash
# round-4 GPU call f: lean GPU tests; A/B without trailing refills vs a87a9b9 (prev); SPEC at 4 waves; stamps
set -e
mkdir -p gpurun_out/r4f
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lean_cells.py tests/test_gpu_fullsize.py tests/test_gpu_life.py tests/test_gpu_spec.py tests/test_gpu_beb.py tests/test_gpu_workloads.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4f/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4f/gpu_tests.log
bash tools/ab.sh "head prev" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head spec4 prev" 1 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
BRC_LIB=exp/stamps/libbrc_hip.so timeout -k 10 120 python3 tools/stamps.py 262144 reference > gpurun_out/r4f/stamps_reference.txt 2>&1
cat gpurun_out/r4f/stamps_reference.txt
