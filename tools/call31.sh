set -o pipefail
mkdir -p gpurun_out/c31
timeout -k 10 900 bash tools/ab.sh "head liilp lilp" 2 --instances 1048576 --steps 2 --warmup 1 --no-cpu --legs connu,conn,ref2c,spec2c,many
timeout -k 10 400 bash tools/ab_cfg.sh "head liilp lilp" 1 cfg4-conn-geometric
