#!/bin/bash
# Variant builds of one source (SRC, default kmc_radix; kmc_hash for the canonical
# path) recompiled with compile-time knobs, every other object from build/:
# lib/variants/libkmc_<name>.so and the
# matching diagnostic library libkmc_<name>_diag.so (test hooks), so that both the
# benchmarks (KMC_LIB=...) and the parity tests (KMC_LIB + KMC_DIAG_LIB) run on the
# variant.  Usage: scripts/build_radix_variants.sh name:"-DFLAGS" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/dna-kmeres-parallel_amd
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -fvisibility=hidden -std=c++17 -I$ROOT/include -I$PKG/csrc"
L="-Wl,--version-script=$PKG/libkmc.map -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib"
mkdir -p $PKG/lib/variants $PKG/build/v
SRC=${SRC:-kmc_radix}
OTHER=$(cd $PKG/build && ls kmc_*.o | grep -v $SRC.o | sed "s|^|$PKG/build/|")
DOTHER=$(for f in $OTHER; do b=$(basename $f); if [ -f $PKG/build/diag_$b ]; then echo $PKG/build/diag_$b; else echo $f; fi; done)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( $H $flags -c $PKG/csrc/$SRC.hip -o $PKG/build/v/${SRC}_$name.o &&
    $H -shared -o $PKG/lib/variants/libkmc_$name.so $PKG/build/v/${SRC}_$name.o $OTHER $L ) &
  ( $H $flags -DKMC_DIAG_HOOKS -c $PKG/csrc/$SRC.hip -o $PKG/build/v/${SRC}_${name}_diag.o &&
    $H -shared -o $PKG/lib/variants/libkmc_${name}_diag.so $PKG/build/v/${SRC}_${name}_diag.o $DOTHER $L ) &
done
wait
ls $PKG/lib/variants
