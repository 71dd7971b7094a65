#!/bin/bash
# round-4 GPU call n: geometric (DM = 16) wide kernel without spills: 2 waves/SIMD or per-word scheduling barriers
set -e
bash tools/ab_cfg.sh "head fence ww2" 2 cfg5-geometric
