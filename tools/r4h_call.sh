#!/bin/bash
# round-4 GPU call h: branchless pair variants vs head (LCHUNK 8) vs LCHUNK 4; SPEC head; cfg5 masked stores
set -e
mkdir -p gpurun_out/r4h
bash tools/ab.sh "head bl blne lc4" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head spec4" 1 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
bash tools/ab_cfg.sh "head widefull" 1 cfg5-const,cfg5-geometric
