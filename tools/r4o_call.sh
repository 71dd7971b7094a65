#!/bin/bash
# round-4 GPU call o: wide kernel with 8 keys per barrier (cfg5 const / uniform)
set -e
bash tools/ab_cfg.sh "head cw8" 2 cfg5-const,cfg5-uniform
