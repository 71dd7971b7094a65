#!/bin/bash
# round-4 GPU call l: isolate the four step-overhead changes (all off = head = 8d7cab7 behaviour)
set -e
bash tools/ab.sh "head last ahead track busyw" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
