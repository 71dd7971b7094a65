#!/bin/bash
# round-4 final profiles, part 2: the connection-peer leg (key-lifetime kernel), every BASELINE workload, the default bench line
set -e
mkdir -p gpurun_out/r4q
bash profiles/collect.sh r4_conn 1048576 conn brc_life > gpurun_out/r4q/collect_conn.log 2>&1 || { tail -20 gpurun_out/r4q/collect_conn.log; exit 1; }
tail -1 gpurun_out/r4q/collect_conn.log
timeout -k 10 400 python3 configs.py > gpurun_out/r4q/configs.jsonl 2> gpurun_out/r4q/configs.err || { tail -20 gpurun_out/r4q/configs.err; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/r4q/bench_default.json 2> gpurun_out/r4q/bench_default.err || { tail -20 gpurun_out/r4q/bench_default.err; exit 1; }
cat gpurun_out/r4q/bench_default.json | head -c 1500
