#!/bin/bash
# round-3 session-3 GPU call: parity of the candidate build (exp/sm: packed key pairs, lazy key
# metadata, SPEC word-at-once per phase index), A/B vs head, default bench line, candidate profile
set -e
mkdir -p gpurun_out/r3d
BRC_LIB=exp/sm/libbrc_hip.so timeout -k 10 540 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_lean_cells.py tests/test_gpu_spec.py tests/test_gpu_beb.py \
  tests/test_gpu_wire.py tests/test_gpu_workloads.py > gpurun_out/r3d/sm_tests.log 2>&1
tail -2 gpurun_out/r3d/sm_tests.log
bash tools/ab.sh "head pk2 sm maxilp" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head sm" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
BRC_LIB=exp/sm/libbrc_hip.so bash profiles/collect.sh r3d_sm 1048576 reference > gpurun_out/r3d/collect_sm.log 2>&1
tail -1 gpurun_out/r3d/collect_sm.log
