#!/bin/bash
# kres.sh <unit.hip>: per-kernel VGPRs / scratch / occupancy (compiler resource-usage remarks)
hipcc -O3 --offload-arch=gfx950 -std=c++17 -c -Rpass-analysis=kernel-resource-usage "$1" -o /tmp/kres.o 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' | awk -F': *' '
  /Function Name/ {name=$2} /^ *VGPRs/ {v=$2} /ScratchSize/ {s=$2} /Occupancy/ {print name, "vgpr=" v, "scratch=" s, "occ=" $2}'
