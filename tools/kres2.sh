#!/bin/bash
# kres2.sh <unit.hip> [flags...]: per-kernel VGPRs / spills / scratch / occupancy (compiler resource remarks)
U=$1; shift
hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -c -Rpass-analysis=kernel-resource-usage "$U" -o /tmp/kres2.o 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' | awk -F': *' '
  /Function Name/ {name=$2} /^ *VGPRs: / {v=$2} /SGPRs Spill/ {ss=$2} /ScratchSize/ {s=$2}
  /Occupancy/ {o=$2} /VGPRs Spill/ {print name, "vgpr=" v, "sspill=" ss, "vspill=" $2, "scratch=" s, "occ=" o}'
