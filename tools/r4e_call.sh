#!/bin/bash
# round-4 GPU call e: lean GPU tests on the deferred-mark build; A/B vs delivery atomics, the u32 key-list
# build (w4) and the first round-4 commit (prev)
set -e
mkdir -p gpurun_out/r4e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lean_cells.py tests/test_gpu_fullsize.py tests/test_gpu_life.py tests/test_gpu_spec.py tests/test_gpu_beb.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4e/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4e/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4e/gpu_tests.log
bash tools/ab.sh "head nodacc w4 prev" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head prev" 1 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
