set -o pipefail
mkdir -p gpurun_out/c6
timeout -k 10 1200 python -u -m pytest tests/test_api_shim.py tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_abi.py tests/test_gpu_life.py tests/test_gpu_lean_cells.py tests/test_gpu_wire.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c6/tests.log 2>&1; rc=$?; tail -5 gpurun_out/c6/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab_cfg.sh "head nw3" 2 cfg3,cfg3-spec,cfg2,cfg2-spec
