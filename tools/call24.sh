set -o pipefail
mkdir -p gpurun_out/c24
BRC_LIB=ab/skip/libbrc_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_life.py "tests/test_gpu_fullsize.py::test_cfg4_2p20_step_kernel_equals_lifetime_kernel" "tests/test_gpu_fullsize.py::test_cfg4_round_cap_64_2p20_bench_legs" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c24/tests.log 2>&1; rc=$?; tail -2 gpurun_out/c24/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab.sh "base skip" 2 --instances 1048576 --steps 2 --warmup 1 --no-cpu --legs ref2c,spec2c,many
