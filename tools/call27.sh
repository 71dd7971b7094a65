set -o pipefail
mkdir -p gpurun_out/c27
BRC_LIB=ab/planes/libbrc_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_life.py "tests/test_gpu_fullsize.py::test_cfg4_connection_peers_2p20_sampled" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c27/tests.log 2>&1; rc=$?; tail -2 gpurun_out/c27/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab.sh "head planes" 2 --instances 1048576 --steps 2 --warmup 1 --no-cpu --legs connu
timeout -k 10 600 bash tools/ab_cfg.sh "head planes" 1 cfg4-conn-geometric,cfg4-conn-uniform
