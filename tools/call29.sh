set -o pipefail
mkdir -p gpurun_out/c29
timeout -k 10 1000 bash tools/ab.sh "head ilp mclause iilp" 2 --instances 1048576 --steps 2 --warmup 1 --no-cpu --legs reference,spec,ref2c,many
