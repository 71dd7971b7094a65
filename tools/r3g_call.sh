#!/bin/bash
# round-3 GPU call: waves-per-SIMD A/B of the lean kernels on the packed-pair build
set -e
bash tools/ab.sh "head w4 w6" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
bash tools/ab.sh "head w4 w6" 1 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs spec
