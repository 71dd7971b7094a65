set -o pipefail
mkdir -p gpurun_out/c28
BRC_LIB=ab/wu1/libbrc_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_wide.py "tests/test_gpu_fullsize.py::test_cfg5_n256_full_size" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c28/tests.log 2>&1; rc=$?; tail -2 gpurun_out/c28/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab_cfg.sh "head wu1" 2 cfg5-const,cfg5-uniform,cfg5-geometric,cfg5-conn-uniform
