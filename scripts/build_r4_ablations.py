#!/usr/bin/env python3
"""DIAGNOSTIC (not product code): builds timing-only variants of the radix R4 kernel
from patched copies of csrc/kmc_radix.hip outside the tree (/tmp/r4abl/<tag>), linked
with the in-tree objects into dna-kmeres-parallel_amd/lib/variants/libkmc_r4abl_<tag>.so,
for scripts/gpu_r03u.sh / gpu_r03v.sh / gpu_r03w.sh.  The
"noadd" and "noload" variants count wrongly by construction; "wave", "nt", "u8" and
"nt_u8" are correct alternatives, as are "exact_nt" and "place_nt" (which apply to
the shipped source: R4ABL_REV=HEAD).  The patches apply to kmc_radix.hip as of commit
3306378 (before the shipped non-temporal loads), read with `git show`.  Run
`make -C dna-kmeres-parallel_amd` first (the other objects are linked from build/).
Usage: python scripts/build_r4_ablations.py [tag ...]   (default: all)"""
import os, subprocess, sys
R = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dna-kmeres-parallel_amd")
SRC_REV = os.environ.get("R4ABL_REV", "3306378")
src = subprocess.check_output(["git", "-C", R, "show", SRC_REV + ":dna-kmeres-parallel_amd/csrc/kmc_radix.hip"], text=True)
def variant(tag, reps):
    s = src
    for a, b in reps:
        assert a in s, (tag, a[:60])
        s = s.replace(a, b)
    d = "/tmp/r4abl/" + tag
    os.makedirs(d, exist_ok=True)
    open(d + "/kmc_radix.hip", "w").write(s)
    obj = d + "/kmc_radix.o"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                           "-I" + R + "/../include", "-I" + R + "/csrc", "-c", d + "/kmc_radix.hip", "-o", obj])
    objs = [R + "/build/" + f for f in ["kmc_dense.o", "kmc_synth.o", "kmc_dist.o", "kmc_hash.o", "kmc_fasta_gpu.o",
                                         "kmc_common.o", "kmc_fasta.o", "kmc_multi.o"]]
    out = R + "/lib/variants/libkmc_r4abl_%s.so" % tag
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, obj] + objs +
                          ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    print("built", out)
noadd = [("""    if constexpr (LOW <= 15) {
        __hip_atomic_fetch_add(&h[e], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {  // two 16-bit bins per word
        __hip_atomic_fetch_add(&h[e >> 1], (e & 1u) ? 0x10000u : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }""", """    asm volatile("" ::"v"(e));"""),
         ("            if (s_sum == end - beg) {", "            if (true) {")]
noload = [("""                x[u] = v[va];""", """                x[u] = make_uint4((uint32_t)va * 2654435761u, (uint32_t)va * 40503u + 7u, j * 2246822519u,
                                  (uint32_t)(va >> 3) * 3266489917u);""")]
wave = [("""    enter(0);
    for (uint32_t j0 = threadIdx.x; j0 < V; j0 += KMC_R4_U * 1024) {""",
         """    const uint32_t wv = threadIdx.x >> 6, per = (V + 15u) / 16u, wb = wv * per, we = wb + per < V ? wb + per : V;
    {  // the last region q with vpre[q] <= wb (binary search: the regions before it are skipped at once)
        uint32_t lo = 0, hi = kMaxRegions - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (vpre[mid] <= wb) lo = mid;
            else hi = mid - 1;
        }
        r = lo;
        enter(r);
    }
    for (uint32_t j0 = wb + (threadIdx.x & 63u); j0 < we; j0 += KMC_R4_U * 64) {"""),
        ("""            const uint32_t j = j0 + 1024u * u;
            m[u] = 0u;
            if (j < V) {""", """            const uint32_t j = j0 + 64u * u;
            m[u] = 0u;
            if (j < we) {""")]
nt = [("""                x[u] = v[va];""", """                {
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(v + va));
                    x[u] = make_uint4(t[0], t[1], t[2], t[3]);
                }""")]
u8 = [("#define KMC_R4_U 4  //", "#define KMC_R4_U 8  //")]

# on the shipped source (R4ABL_REV=HEAD): the exact walk's loads and R5's stage reads non-temporal
exact_nt = [("        const auto ld = [&](uint64_t k) { return v[k]; };",
             """        const auto ld = [&](uint64_t k) {
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(v + k));
            return make_uint4(t[0], t[1], t[2], t[3]);
        };""")]
place_nt = [("            const uint4 v = *reinterpret_cast<const uint4 *>(p.stage + (s0 + r) * nbins + c0 + cc);",
             """            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 t4 = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p.stage + (s0 + r) * nbins + c0 + cc));
            const uint4 v = make_uint4(t4[0], t4[1], t4[2], t4[3]);""")]
VARIANTS = {"exact_nt": exact_nt, "place_nt": place_nt, "noadd": noadd, "noload": noload, "wave": wave, "wave_noadd": wave + noadd, "nt": nt, "u8": u8,
            "nt_u8": nt + u8}
if __name__ == "__main__":
    for tag in sys.argv[1:] or list(VARIANTS):
        variant(tag, VARIANTS[tag])
