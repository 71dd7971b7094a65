set -o pipefail
mkdir -p gpurun_out/c12
timeout -k 10 900 python -u -m pytest tests/test_gpu_life.py "tests/test_gpu_fullsize.py::test_cfg4_many_rounds_2p20_one_launch" "tests/test_gpu_fullsize.py::test_cfg4_round_cap_64_2p20_bench_legs[long]" "tests/test_gpu_fullsize.py::test_cfg4_long_consensus_many_rounds" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c12/tests.log 2>&1; rc=$?; tail -3 gpurun_out/c12/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu --legs many,long > gpurun_out/c12/bench.json 2> gpurun_out/c12/bench.err; rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/c12/bench.json')); print(d['kernel_ms'], d['long_leg']['kernel_ms'])"; exit $rc
