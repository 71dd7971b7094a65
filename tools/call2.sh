set -o pipefail
mkdir -p gpurun_out/c2
BRC_LIB=ab/nlw/libbrc_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_workloads.py tests/test_gpu_spec.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c2/tests_nlw.log 2>&1; rc=$?; tail -3 gpurun_out/c2/tests_nlw.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 bash tools/ab.sh "head s8 c16" 2 --instances 1048576 --steps 3 --warmup 1 --no-cpu --legs reference,spec && \
timeout -k 10 1200 bash tools/ab_cfg.sh "head nlw" 2 cfg3,cfg3-spec,cfg2,cfg5-geometric,cfg5-const
