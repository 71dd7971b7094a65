set -o pipefail
mkdir -p gpurun_out/c16
for w in cfg4-ref-r8 cfg4-ref-r64 cfg4-conn; do
  BRC_LIB=ab/lstamp/libbrc_hip.so timeout -k 10 300 python -u tools/stamps.py 262144 $w life > gpurun_out/c16/$w.txt 2>&1; rc=$?; cat gpurun_out/c16/$w.txt; [ $rc -eq 0 ] || exit $rc
done
