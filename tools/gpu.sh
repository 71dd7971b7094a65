#!/bin/bash
# One GPU-box session of steps, each under its own time limit, chained so the first failure ends it
# (run on the GPU box from the repo root; outputs under gpurun_out/<tag>/):
#   bash tools/gpu.sh <tag> <step> [<step> ...]
# steps:
#   tests[=<pytest -k expr>]     the -m gpu suite (or a -k subset)          -> tests.log
#   smoke                         __graft_entry__.smoke()                    -> smoke.log
#   bench[=<bench.py args>]       bench.py (default args)                    -> bench.json
#   configs[=<names>]             configs.py [--only names]                  -> configs.jsonl
#   collect=<ptag>,<inst>,<leg>,<kernel>[,<passes>]   profiles/collect.sh    -> collect_<ptag>.log
#   ab=<tags>,<rounds>[,<bench args>]                 tools/ab.sh            -> ab.log
#   abcfg=<tags>,<rounds>,<configs names>             tools/ab_cfg.sh        -> abcfg.log
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  echo "== $step ($(date +%T))"
  case $name in
    tests)
      if [ -n "$arg" ]; then K=(-k "$arg"); else K=(); fi
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/tests.log 2>&1
      rc=$?; tail -3 $OUT/tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as G; G.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > $OUT/bench.json 2> $OUT/bench.err; rc=$?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['kernel_ms'], d['value'], {k: (v['kernel_ms'], v['value']) for k, v in d.items() if k.endswith('_leg')})" $OUT/bench.json ;;
    configs)
      if [ -n "$arg" ]; then O=(--only "$arg"); else O=(); fi
      timeout -k 10 900 python -u configs.py "${O[@]}" > $OUT/configs.jsonl 2> $OUT/configs.err; rc=$?; wc -l $OUT/configs.jsonl ;;
    collect)
      IFS=, read -r ptag inst leg kern passes <<< "$arg"
      timeout -k 10 900 bash profiles/collect.sh $ptag $inst $leg $kern $passes > $OUT/collect_$ptag.log 2>&1; rc=$?; tail -1 $OUT/collect_$ptag.log ;;
    ab)
      IFS=, read -r tags rounds bargs <<< "$arg"
      timeout -k 10 1200 bash tools/ab.sh "$tags" $rounds $bargs > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log ;;
    abcfg)
      IFS=, read -r tags rounds names <<< "$arg"
      names=${names//+/,}
      timeout -k 10 1200 bash tools/ab_cfg.sh "$tags" $rounds $names > $OUT/abcfg.log 2>&1; rc=$?; cat $OUT/abcfg.log ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then echo "step $step failed: rc $rc"; exit $rc; fi
done
echo "== done ($(date +%T))"
