#!/bin/bash
# round-4 GPU call j: full GPU suite on the deferred-send build (no consensus snapshot, per-key counts);
# A/B vs 414eee0 (last) on both cfg4 legs and cfg3; stamps
set -e
mkdir -p gpurun_out/r4j
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r4j/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4j/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4j/gpu_tests.log
bash tools/ab.sh "head last" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head last" 1 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
bash tools/ab_cfg.sh "head last" 1 cfg3,cfg3-spec
BRC_LIB=exp/stamps/libbrc_hip.so timeout -k 10 120 python3 tools/stamps.py 262144 reference > gpurun_out/r4j/stamps_reference.txt 2>&1
cat gpurun_out/r4j/stamps_reference.txt
