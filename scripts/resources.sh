#!/bin/bash
# Kernel resource usage (VGPRs, scratch, LDS, occupancy) of one source file:
#   scripts/resources.sh csrc/kmc_radix.hip [name-filter]
cd "$(dirname "$0")/../dna-kmeres-parallel_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -Icsrc ${EXTRA:-} \
  -Rpass-analysis=kernel-resource-usage -c "$1" -o /tmp/res_$$.o 2>&1 |
  awk '/Function Name/{sub(/.*Function Name: /,""); sub(/ \[-Rpass.*/,""); n=$0}
       /VGPRs:/{v=$(NF-1)} /ScratchSize/{sc=$(NF-1)} /Occupancy/{o=$(NF-1)}
       /LDS Size/{print "vgpr=" v, "scratch=" sc, "lds=" $(NF-1), "occ=" o, n}' | c++filt |
  sed -e 's/kmc::(anonymous namespace):://g' | grep -E "${2:-.}" | cut -c1-160
rm -f /tmp/res_$$.o
