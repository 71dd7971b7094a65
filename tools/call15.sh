set -o pipefail
mkdir -p gpurun_out/c15
timeout -k 10 900 python -u -m pytest tests/test_gpu_lean_cells.py tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_cfg4_2p20_step_kernel_equals_lifetime_kernel" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c15/tests.log 2>&1; rc=$?; tail -3 gpurun_out/c15/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab.sh "head f1" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference,spec
