#!/bin/bash
# Diagnostic builds of libkmc.so that recompile only kmc_radix.hip with
# compile-time knobs (the other objects from build/): lib/variants/libkmc_<name>.so
#   scripts/build_radix_variants.sh name:"-DFLAGS" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/dna-kmeres-parallel_amd
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$ROOT/include -I$PKG/csrc"
mkdir -p $PKG/lib/variants $PKG/build/v
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( $H $flags -c $PKG/csrc/kmc_radix.hip -o $PKG/build/v/radix_$name.o &&
    $H -shared -o $PKG/lib/variants/libkmc_$name.so $PKG/build/v/radix_$name.o \
      $(ls $PKG/build/kmc_*.o | grep -v kmc_radix.o) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib ) &
done
wait
ls $PKG/lib/variants
