#!/bin/bash
# round-4 GPU call m: wide-kernel bit-plane matching with v_bitop3 (cfg5) and SPEC with u32 key-list entries
set -e
mkdir -p gpurun_out/r4m
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wide.py tests/test_gpu_spec.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r4m/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4m/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4m/gpu_tests.log
bash tools/ab_cfg.sh "head last" 2 cfg5-uniform,cfg5-geometric
bash tools/ab.sh "head speckl32" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
