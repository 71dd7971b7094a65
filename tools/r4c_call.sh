#!/bin/bash
# round-4 GPU call c: waves-per-SIMD A/B (4 vs 5) before / after the split-bulk consensus
set -e
bash tools/ab.sh "head prev w4 prevw4 base" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
