set -o pipefail
mkdir -p gpurun_out/c3
timeout -k 10 300 python -u bench.py --instances 1048576 --steps 1 --warmup 0 --no-cpu --legs spec64 > gpurun_out/c3/spec64.json 2> gpurun_out/c3/spec64.err; echo "spec64 rc $?"; python3 -c "import json; d=json.load(open('gpurun_out/c3/spec64.json')); print(d['kernel_ms'], d['value'], d['decide_round_hist'], d['counts'])"
timeout -k 10 400 python -u bench.py --instances 262144 --steps 1 --warmup 0 --no-cpu --legs long > gpurun_out/c3/long.json 2> gpurun_out/c3/long.err; echo "long rc $?"; python3 -c "import json; d=json.load(open('gpurun_out/c3/long.json')); print(d['kernel_ms'], d['value'], d['kernel'], d['decide_round_hist'], d['counts'])"
timeout -k 10 600 bash tools/ab.sh "head w5" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference
