#!/bin/bash
# round-4 GPU call g: full GPU suite (sweep through RCCL, key window 32, new fixture); A/B vs a87a9b9
# (prev); SPEC at 4 waves; stamps split
set -e
mkdir -p gpurun_out/r4g
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r4g/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4g/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4g/gpu_tests.log
bash tools/ab.sh "head lc8 prev" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head spec4 prev" 1 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
BRC_LIB=exp/stamps/libbrc_hip.so timeout -k 10 120 python3 tools/stamps.py 262144 reference > gpurun_out/r4g/stamps_reference.txt 2>&1
cat gpurun_out/r4g/stamps_reference.txt
bash tools/ab_cfg.sh "head widefull" 1 cfg5-const,cfg5-geometric
