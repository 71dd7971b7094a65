set -o pipefail
mkdir -p gpurun_out/c5
timeout -k 10 900 python -u -m pytest tests/test_gpu_life.py "tests/test_gpu_fullsize.py::test_cfg4_many_rounds_2p20_one_launch" "tests/test_gpu_fullsize.py::test_cfg4_round_cap_64_2p20_bench_legs[long]" "tests/test_gpu_fullsize.py::test_cfg4_long_consensus_many_rounds" tests/test_api_shim.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c5/tests.log 2>&1; rc=$?; tail -3 gpurun_out/c5/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab.sh "head hm64" 1 --instances 1048576 --steps 2 --warmup 1 --no-cpu --legs many,conn,connu,long
