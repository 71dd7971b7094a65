#!/bin/bash
# round 4 final: full GPU suite, default bench line, profile of the connection-peer leg and the per-link workload
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4z_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r4z_bench.json 2> gpurun_out/r4z_bench.err && \
timeout -k 10 600 bash profiles/collect.sh r4g_conn 1048576 conn brc_life > gpurun_out/r4z_collect1.log 2>&1 && \
timeout -k 10 600 bash profiles/collect.sh r4g_connu 0 cfg4-conn-uniform-d2 brc_life > gpurun_out/r4z_collect2.log 2>&1
