#!/bin/bash
# round-4 GPU call a: GPU suite on the buffer/DPP build, then A/B vs the round-3 build (base) and 6 waves/SIMD
set -e
mkdir -p gpurun_out/r4a
timeout -k 10 720 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4a/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4a/gpu_tests.log
bash tools/ab.sh "head base w6" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head base" 1 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
