#!/bin/bash
# round 4 final check: smoke(), full GPU suite and the default bench line on the final in-tree build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4ab_smoke.log 2>&1 && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4ab_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r4ab_bench.json 2> gpurun_out/r4ab_bench.err
