#!/bin/bash
# round 4: full GPU suite after the per-link lifetime kernel and the three-bit value ids, then the
# narrow-kernel workloads (cfg2 / cfg3) and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4u_tests.log 2>&1 && \
timeout -k 10 300 python -u configs.py --only cfg2,cfg3,cfg3-spec > gpurun_out/r4u_configs.jsonl 2> gpurun_out/r4u_configs.err && \
timeout -k 10 300 python -u bench.py > gpurun_out/r4u_bench.json 2> gpurun_out/r4u_bench.err
