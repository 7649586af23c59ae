#!/bin/bash
# Diagnostic builds of libkmc.so with compile-time knobs, for scripts/kbench.py
# A/B runs on the GPU box (KMC_LIB=...).  Usage: scripts/build_variants.sh name:"-DFLAGS" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/dna-kmeres-parallel_amd
mkdir -p $PKG/lib/variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$ROOT/include -I$PKG/csrc $flags -shared \
    -o $PKG/lib/variants/libkmc_$name.so $PKG/csrc/kmc_dense.hip $PKG/csrc/kmc_radix.hip $PKG/csrc/kmc_synth.hip $PKG/csrc/kmc_dist.hip $PKG/csrc/kmc_hash.hip $PKG/csrc/kmc_fasta_gpu.hip \
    -x none $PKG/build/kmc_common.o $PKG/build/kmc_fasta.o $PKG/build/kmc_multi.o -L/opt/rocm/lib -lrccl &
done
wait
ls $PKG/lib/variants
