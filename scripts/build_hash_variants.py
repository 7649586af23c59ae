#!/usr/bin/env python3
"""DIAGNOSTIC (not product code): builds variants of the canonical-counting kernels
(csrc/kmc_hash.hip) from patched copies outside the tree (/tmp/hashvar/<tag>), linked
with the in-tree objects into dna-kmeres-parallel_amd/lib/variants/libkmc_hash_<tag>.so,
for scripts/gpu_r03y.sh: non-temporal loads of the entries K3b (fine) and K4s (sort)
read once.  All variants count correctly.  Run `make -C dna-kmeres-parallel_amd` first.
Usage: python scripts/build_hash_variants.py [tag ...]   (default: all)"""
import os
import subprocess
import sys

R = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dna-kmeres-parallel_amd")
src = open(R + "/csrc/kmc_hash.hip").read()


def variant(tag, reps):
    s = src
    for a, b in reps:
        assert a in s, (tag, a[:60])
        s = s.replace(a, b)
    d = "/tmp/hashvar/" + tag
    os.makedirs(d, exist_ok=True)
    open(d + "/kmc_hash.hip", "w").write(s)
    obj = d + "/kmc_hash.o"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                           "-I" + R + "/../include", "-I" + R + "/csrc", "-c", d + "/kmc_hash.hip", "-o", obj])
    objs = [R + "/build/" + f for f in ["kmc_dense.o", "kmc_synth.o", "kmc_dist.o", "kmc_radix.o", "kmc_fasta_gpu.o",
                                         "kmc_common.o", "kmc_fasta.o", "kmc_multi.o"]]
    out = R + "/lib/variants/libkmc_hash_%s.so" % tag
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, obj] + objs +
                          ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    print("built", out)


fine_nt = [("            xn[j] = i < a1 ? p.ent_c[i] : 0ull;",
            "            xn[j] = i < a1 ? __builtin_nontemporal_load(&p.ent_c[i]) : 0ull;")]
sort_nt = [("            kh[j] = i < n ? p.ent[b0 + i] : kEmptyH;",
            "            kh[j] = i < n ? __builtin_nontemporal_load(&p.ent[b0 + i]) : kEmptyH;")]
VARIANTS = {"fine_nt": fine_nt, "sort_nt": sort_nt, "both_nt": fine_nt + sort_nt}
if __name__ == "__main__":
    for tag in sys.argv[1:] or list(VARIANTS):
        variant(tag, VARIANTS[tag])
