set -o pipefail
mkdir -p gpurun_out/c32
BRC_LIB=ab/hstat/libbrc_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_life.py "tests/test_gpu_fullsize.py::test_cfg4_2p20_step_kernel_equals_lifetime_kernel" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c32/tests.log 2>&1; rc=$?; tail -2 gpurun_out/c32/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab.sh "head hstat" 2 --instances 1048576 --steps 2 --warmup 1 --no-cpu --legs ref2c,spec2c,many,long
