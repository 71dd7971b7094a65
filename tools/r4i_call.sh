#!/bin/bash
# round-4 GPU call i: per-key counts A/B; stamps with the consensus split into sub-sections
set -e
mkdir -p gpurun_out/r4i
bash tools/ab.sh "head pkc" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
BRC_LIB=exp/stamps/libbrc_hip.so timeout -k 10 120 python3 tools/stamps.py 262144 reference > gpurun_out/r4i/stamps_reference.txt 2>&1
cat gpurun_out/r4i/stamps_reference.txt
