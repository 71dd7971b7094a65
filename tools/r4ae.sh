#!/bin/bash
# round 4: per-link pending steps from a DPP OR of the senders' delay sets (variant exp/vout): lifetime tests, A/B vs HEAD
set -o pipefail
mkdir -p gpurun_out
BRC_LIB=exp/vout/libbrc_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_life.py "tests/test_gpu_fullsize.py::test_cfg4_connection_peers_2p20_sampled" > gpurun_out/r4ae_tests.log 2>&1 && \
timeout -k 10 600 bash tools/ab_cfg.sh "head vout" 3 cfg4-conn-uniform-d2 > gpurun_out/r4ae_ab.txt 2>&1
