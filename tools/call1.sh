set -o pipefail
mkdir -p gpurun_out/c1
BRC_LIB=ab/oob/libbrc_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_lean_cells.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c1/tests_oob.log 2>&1 && tail -2 gpurun_out/c1/tests_oob.log && \
timeout -k 10 1200 bash tools/ab.sh "head oob oob4" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference,spec
