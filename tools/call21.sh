set -o pipefail
mkdir -p gpurun_out/c21
for lib in pf bstat; do
BRC_LIB=ab/$lib/libbrc_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_life.py "tests/test_gpu_fullsize.py::test_cfg4_many_rounds_2p20_one_launch" "tests/test_gpu_fullsize.py::test_cfg4_round_cap_64_2p20_bench_legs" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c21/tests_$lib.log 2>&1; rc=$?; tail -2 gpurun_out/c21/tests_$lib.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 bash tools/ab.sh "head pf bstat" 2 --instances 1048576 --steps 2 --warmup 1 --no-cpu --legs ref2c,many,long
