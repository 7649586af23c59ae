#!/bin/bash
# The CPU test suite with the host C++ (libkmc.so's loader, shard planner, RCCL
# driver; the kmc driver binary) and the oracle's C restatement built with
# AddressSanitizer + UBSan.  CPU only: GPU sanitizers are not
# available on this pool.  Usage: scripts/asan_tests.sh [pytest args]
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -j8 -C dna-kmeres-parallel_amd all asan
make -s -C oracle all asan
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
# leaks: CPython and torch keep allocations until exit by design
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:print_summary=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export KMC_LIB="$PWD/dna-kmeres-parallel_amd/lib-asan/libkmc.so"
export KMC_ORACLE_LIB="$PWD/oracle/_asan/libkmc_oracle.so"
export KMC_BIN="$PWD/dna-kmeres-parallel_amd/lib-asan/kmc"
exec python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
