#!/bin/bash
# Quick counter passes on the cfg4 bench at a reduced batch (run on the GPU box from the repo root).
#   bash tools/pmc_quick.sh <tag> [instances] [extra bench args]
# Each pass is its own rocprofv3 run (counter blocks never combined beyond one pass's budget).
set -u
TAG=$1; INST=${2:-262144}; shift; shift || true
OUT=gpurun_out/pmcq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --instances $INST --steps 1 --warmup 0 --no-cpu $*"
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc$i -o run --output-format csv -- python3 $BENCH > $OUT/pmc$i.json 2> $OUT/pmc$i.err || { echo "pmc pass $i failed"; tail -3 $OUT/pmc$i.err; exit 1; }
done
python3 - "$OUT" <<'EOF'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float)
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "brc_step" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(tot):
    print("%-24s %.4g" % (k, tot[k]))
EOF
