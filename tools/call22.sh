set -o pipefail
mkdir -p gpurun_out/c22
BRC_LIB=ab/qb/libbrc_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_life.py "tests/test_gpu_fullsize.py::test_cfg4_round_cap_64_2p20_bench_legs" "tests/test_gpu_fullsize.py::test_cfg4_long_consensus_many_rounds" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c22/tests.log 2>&1; rc=$?; tail -2 gpurun_out/c22/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab.sh "head qb" 2 --instances 1048576 --steps 1 --warmup 0 --no-cpu --legs long
