#!/bin/bash
# rocprofv3 collection for the headline kernel (run on the GPU box from the repo root).
#   bash profiles/collect.sh <tag> [instances] [leg] [kernel] [passes]
#     leg: a bench.py leg (reference (default), spec, conn, connu, many) -> bench.py; a configs.py
#     workload name (cfg5-const, ...) -> configs.py --only <leg> (instances ignored); kernel: brc_step
#     (default), brc_step_wide or brc_life; passes: full (default: 5 PMC passes) or light (FETCH_SIZE,
#     WRITE_SIZE and the SQ issue pass)
# 1) kernel trace + stats of bench.py (same command the numbers come from)
# 2) separate PMC passes (one counter block budget per pass, each under its own kill timeout)
set -u
TAG=${1:-r1}; INST=${2:-65536}; LEG=${3:-reference}; KERNEL=${4:-brc_step}; PASSES=${5:-full}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
case $LEG in
  cfg*) BENCH="configs.py --only $LEG --steps 2 --warmup 1" ;;
  *) BENCH="bench.py --instances $INST --steps 2 --warmup 1 --no-cpu --legs $LEG" ;;
esac
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 $BENCH > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace failed"; exit 1; }
i=0
P1="FETCH_SIZE"; P2="WRITE_SIZE"
P3="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P4="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P5="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_UNALIGNED_STALL"
if [ "$PASSES" = light ]; then PL=("$P1" "$P2" "$P3 GRBM_GUI_ACTIVE"); else PL=("$P1" "$P2" "$P3" "$P4" "$P5"); fi
for pmc in "${PL[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -T -d $OUT/pmc$i -o run --output-format csv -- python3 $BENCH > $OUT/pmc$i.json 2> $OUT/pmc$i.err || { echo "pmc pass $i failed"; exit 1; }
done
python3 profiles/summarize.py $OUT profiles/$TAG --kernel $KERNEL > $OUT/summary.json || { echo "summary failed"; exit 1; }
echo "collected $OUT"
ls -R $OUT | head -40
