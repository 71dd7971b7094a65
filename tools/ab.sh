#!/bin/bash
# Interleaved A/B of library variants built by tools/variant.py (run on the GPU box from the repo root).
#   bash tools/ab.sh "<tag> <tag> ..." <rounds> [bench.py args]
# tag "head" = the in-tree libbrc_hip.so.  One bench.py process per (round, variant); prints
# "tag kernel_ms value" lines and writes gpurun_out/ab/<tag>.<round>.json.
set -u
TAGS=$1; ROUNDS=$2; shift 2
ARGS=${*:-"--instances 262144 --steps 3 --warmup 1 --no-cpu --legs reference"}
mkdir -p gpurun_out/ab
for r in $(seq 1 $ROUNDS); do
  for t in $TAGS; do
    if [ "$t" = head ]; then lib=""; else lib=ab/$t/libbrc_hip.so; fi
    BRC_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab/$t.$r.json 2> gpurun_out/ab/$t.$r.err || { echo "FAIL $t round $r"; tail -5 gpurun_out/ab/$t.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['kernel_ms'],2), round(d['value']/1e6,3), d['decided_fraction'], {k[:-4]: round(v['kernel_ms'],2) for k, v in d.items() if k.endswith('_leg')})" gpurun_out/ab/$t.$r.json $t
  done
done
