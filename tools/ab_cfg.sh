#!/bin/bash
# Interleaved A/B of library variants on configs.py workloads (run on the GPU box from the repo root).
#   bash tools/ab_cfg.sh "<tag> ..." <rounds> <configs.py --only list>
set -u
TAGS=$1; ROUNDS=$2; ONLY=$3
mkdir -p gpurun_out/abcfg
for r in $(seq 1 $ROUNDS); do
  for t in $TAGS; do
    if [ "$t" = head ]; then lib=""; else lib=ab/$t/libbrc_hip.so; fi
    BRC_LIB=$lib timeout -k 10 300 python3 configs.py --only $ONLY --steps 2 --warmup 1 > gpurun_out/abcfg/$t.$r.jsonl 2> gpurun_out/abcfg/$t.$r.err || { echo "FAIL $t round $r"; tail -5 gpurun_out/abcfg/$t.$r.err; exit 1; }
    python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['workload'], round(d['kernel_ms'],2), d['statuses'], d['decide_round_hist'])" gpurun_out/abcfg/$t.$r.jsonl $t
  done
done
