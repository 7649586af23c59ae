#!/bin/bash
# Diagnostic builds of libkmc.so that recompile only one source (SRC, default
# kmc_radix) with compile-time knobs (the other objects from build/):
# lib/variants/libkmc_<name>.so
#   [SRC=kmc_hash] scripts/build_variants_one.sh name:"-DFLAGS" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/dna-kmeres-parallel_amd
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$ROOT/include -I$PKG/csrc"
SRC=${SRC:-kmc_radix}
mkdir -p $PKG/lib/variants $PKG/build/v
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( $H $flags -c $PKG/csrc/$SRC.hip -o $PKG/build/v/${SRC}_$name.o &&
    $H -shared -o $PKG/lib/variants/libkmc_$name.so $PKG/build/v/${SRC}_$name.o \
      $(ls $PKG/build/kmc_*.o | grep -v $SRC.o) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib ) &
done
wait
ls $PKG/lib/variants
