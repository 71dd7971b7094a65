set -o pipefail
mkdir -p gpurun_out/c20
for w in ${WL:-cfg4-ref-2c cfg4-ref-r8 cfg4-ref-r64 cfg4-conn cfg4-spec-2c}; do
  BRC_LIB=ab/lstamp/libbrc_hip.so timeout -k 10 300 python -u tools/stamps.py 262144 $w life > gpurun_out/c20/$w.txt 2>&1; rc=$?; echo "== $w"; cat gpurun_out/c20/$w.txt; [ $rc -eq 0 ] || exit $rc
done
