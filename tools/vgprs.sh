#!/bin/bash
# VGPRs / occupancy / LDS of the rc1pass kernel variants (make asm).
cd "$(dirname "$0")/../cpp_volume_rendering_amd/csrc" && make -s asm >/dev/null 2>&1
awk -v pat="${1:-rc1pass_tile_kernel}" '/Function Name:/{n=""; if (index($0, pat)) {n=$0; sub(/.*Function Name: /,"",n); sub(/ .*/,"",n)}} n!="" && /VGPRs: /{v=$(NF-1)} n!="" && /LDS Size/{l=$(NF-1)} n!="" && /Occupancy/{o=$(NF-1)} n!="" && /LDS Size/{print substr(n,1,70), "vgpr", v, "occ", o, "lds", l}' build/resource-usage.txt
