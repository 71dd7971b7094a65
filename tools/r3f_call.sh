#!/bin/bash
# round-3 final GPU call: the in-tree build's full GPU suite, the headline profile, the default bench line
set -e
mkdir -p gpurun_out/r3f
timeout -k 10 720 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3f/gpu_tests.log 2>&1
tail -2 gpurun_out/r3f/gpu_tests.log
bash profiles/collect.sh r3f 1048576 reference > gpurun_out/r3f/collect.log 2>&1
tail -1 gpurun_out/r3f/collect.log
timeout -k 10 240 python3 bench.py > gpurun_out/r3f/bench_default.json 2> gpurun_out/r3f/bench_default.err
