set -o pipefail
mkdir -p gpurun_out/c19
BRC_KERNEL=life timeout -k 10 600 python -u bench.py --legs reference,spec,spec64 --steps 2 --warmup 1 --no-cpu > gpurun_out/c19/life.json 2> gpurun_out/c19/life.err; rc=$?; tail -3 gpurun_out/c19/life.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('life', round(d['kernel_ms'],2), d['decided_fraction'], {k[:-4]: (round(v['kernel_ms'],2), v.get('kernel')) for k, v in d.items() if k.endswith('_leg')}, d.get('kernel'))" gpurun_out/c19/life.json
BRC_KERNEL=life timeout -k 10 600 python -u configs.py --only cfg4-beb,cfg4-ref --steps 2 --warmup 1 > gpurun_out/c19/cfg.jsonl 2> gpurun_out/c19/cfg.err; rc=$?; tail -2 gpurun_out/c19/cfg.err; cut -c1-400 gpurun_out/c19/cfg.jsonl; exit $rc
