set -o pipefail
mkdir -p gpurun_out/c30
timeout -k 10 600 bash tools/ab.sh "head" 2 --instances 1048576 --steps 2 --warmup 1 --no-cpu --legs reference,spec
timeout -k 10 900 bash tools/ab_cfg.sh "head iilp16 iilp256" 2 cfg3,cfg3-spec,cfg5-const,cfg5-geometric
