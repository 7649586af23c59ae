"""Diagnostic (round 4): where K4s's time goes, per phase of sort_list.

Builds lib/variants/libkmc_k4sprof.so from the current kmc_hash.hip (round 5: the
direct-output instances, with the reservation + write-out tail as a phase) with clock
reads (s_memtime) patched in at the phase boundaries of sort_list (wave 0 of each
workgroup, accumulated in registers over its lists, one device add per workgroup
at the end) -- the product source carries none of it.  `--build` on the build host;
on the GPU box (no flag) it runs C4 (scripts/cbench.py's GRCh38-like genome; --c4r: C4R's) through
the variant and prints cycles per list and phase for the common and big instances.
Wave 0's phase times include its waits at the barriers that end them."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dna-kmeres-parallel_amd")
VLIB = os.path.join(PKG, "lib", "variants", "libkmc_k4sprof.so")
PH = ["load+A", "rank+B", "scan+C1C2", "scatter", "D", "pairwise", "E", "hot", "tail"]


def build():
    src = open(os.path.join(PKG, "csrc", "kmc_hash.hip")).read()

    def rep(a, b):
        nonlocal src
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    rep("template <class C, bool DIRECT>\n__device__ __forceinline__ void sort_list(",
        "__device__ unsigned long long g_k4s_prof[2][10];\n"
        "#define TS(i) do { const unsigned long long _t = __builtin_amdgcn_s_memtime(); acc[i] += _t - tp; tp = _t; } while (0)\n"
        "template <class C, bool DIRECT>\n__device__ __forceinline__ void sort_list(")
    rep("uint32_t n, const uint64_t *nxt, uint64_t &nb0, uint64_t &ne0) {",
        "uint32_t n, const uint64_t *nxt, uint64_t &nb0, uint64_t &ne0, unsigned long long (&acc)[10]) {\n"
        "    unsigned long long tp = __builtin_amdgcn_s_memtime();\n    acc[9] += 1;")
    rep("    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), gfx9 encoding\n",
        "    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), gfx9 encoding\n    TS(0);\n")
    rep("    lds_barrier();  // B: every key ranked\n", "    lds_barrier();  // B: every key ranked\n    TS(1);\n")
    rep("    lds_barrier();  // C2: slot starts\n", "    lds_barrier();  // C2: slot starts\n    TS(2);\n")
    rep("    lds_barrier();  // D: the keys of the failing slots sorted by slot\n",
        "    TS(3);\n    lds_barrier();  // D: the keys of the failing slots sorted by slot\n    TS(4);\n")
    rep("    if (nhot) lds_barrier();", "    TS(5);\n    if (nhot) lds_barrier();")
    rep("    lds_barrier();  // E: every key emitted\n",
        "    TS(7);\n    lds_barrier();  // E: every key emitted\n    TS(6);\n")
    rep("    } else {\n        if (tid == 0) p.ndist[l] = S.out;\n    }\n}",
        "        TS(8);\n    } else {\n        if (tid == 0) p.ndist[l] = S.out;\n    }\n}")
    rep("        sort_list<SortSmall, DIRECT>(p, S, l, b0, e0, n, nxt, nb0, ne0);",
        "        sort_list<SortSmall, DIRECT>(p, S, l, b0, e0, n, nxt, nb0, ne0, acc);")
    rep("    uint64_t b0 = 0, e0 = 0;  // this list's bounds (the previous one loaded them)\n",
        "    uint64_t b0 = 0, e0 = 0;  // this list's bounds (the previous one loaded them)\n    unsigned long long acc[10] = {};\n")
    rep("        b0 = nb0;\n        e0 = ne0;\n    }\n}",
        "        b0 = nb0;\n        e0 = ne0;\n    }\n"
        "    if (DIRECT && threadIdx.x == 0) for (int i = 0; i < 10; ++i) atomicAdd(&g_k4s_prof[0][i], acc[i]);\n}")
    rep("    const int64_t nl = DIRECT ? (int64_t)p.dist_off[p.l_hi] : (int64_t)*p.nbig;\n",
        "    const int64_t nl = DIRECT ? (int64_t)p.dist_off[p.l_hi] : (int64_t)*p.nbig;\n    unsigned long long acc[10] = {};\n")
    rep("                                   in < nl ? p.big + 3 * in + 1 : nullptr, nb0, ne0);\n    }\n}",
        "                                   in < nl ? p.big + 3 * in + 1 : nullptr, nb0, ne0, acc);\n    }\n"
        "    if (DIRECT && threadIdx.x == 0) for (int i = 0; i < 10; ++i) atomicAdd(&g_k4s_prof[1][i], acc[i]);\n}")
    # crowded slots: per size class of m (9-16, 17-64, 65-256, 257-1024, > 1024 keys) the
    # slots, their distinct keys and the cycles the wave spent on them
    rep("    for (uint32_t hs = (uint32_t)wv; hs < nhot; hs += kBlk / 64) {\n"
        "        const uint32_t sw = S.sc[S.hot[hs]];\n"
        "        const uint32_t a = sw & 0xFFFFu, e = a + slot_count(sw);\n",
        "    for (uint32_t hs = (uint32_t)wv; hs < nhot; hs += kBlk / 64) {\n"
        "        const uint32_t sw = S.sc[S.hot[hs]];\n"
        "        const uint32_t a = sw & 0xFFFFu, e = a + slot_count(sw);\n"
        "        const unsigned long long t_s0 = __builtin_amdgcn_s_memtime();\n"
        "        const uint32_t m_s = e - a;\n"
        "        const int cls = m_s <= 16 ? 0 : m_s <= 64 ? 1 : m_s <= 256 ? 2 : m_s <= 1024 ? 3 : 4;\n")
    rep("            if (last) break;\n            c = nx;\n            piv = S.sk[nx];  // (not marked: a value other than piv's)\n        }\n",
        "            if (last) break;\n            c = nx;\n            piv = S.sk[nx];  // (not marked: a value other than piv's)\n        }\n"
        "        if (lane == 0) {\n"
        "            atomicAdd(&g_k4s_slots[C::kCap == kSortCapBigCfg ? 1 : 0][cls][0], 1ull);\n"
        "            atomicAdd(&g_k4s_slots[C::kCap == kSortCapBigCfg ? 1 : 0][cls][1], (unsigned long long)nd);\n"
        "            atomicAdd(&g_k4s_slots[C::kCap == kSortCapBigCfg ? 1 : 0][cls][2], __builtin_amdgcn_s_memtime() - t_s0);\n"
        "            atomicAdd(&g_k4s_slots[C::kCap == kSortCapBigCfg ? 1 : 0][cls][3], (unsigned long long)m_s);\n"
        "        }\n")
    rep("__device__ unsigned long long g_k4s_prof[2][10];\n",
        "__device__ unsigned long long g_k4s_prof[2][10];\n__device__ unsigned long long g_k4s_slots[2][5][4];\n")
    src += ('\nextern "C" __attribute__((visibility("default"))) int kmc_k4sprof_slots(unsigned long long *out) {\n'
            '    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kmc::g_k4s_slots), sizeof(kmc::g_k4s_slots)) != hipSuccess) return 1;\n'
            '    static const unsigned long long z[40] = {};\n'
            '    return hipMemcpyToSymbol(HIP_SYMBOL(kmc::g_k4s_slots), z, sizeof(z)) != hipSuccess;\n}\n')
    src += ('\nextern "C" __attribute__((visibility("default"))) int kmc_k4sprof_read(unsigned long long *out) {\n'
            '    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kmc::g_k4s_prof), sizeof(kmc::g_k4s_prof)) != hipSuccess) return 1;\n'
            '    static const unsigned long long z[20] = {};\n'
            '    return hipMemcpyToSymbol(HIP_SYMBOL(kmc::g_k4s_prof), z, sizeof(z)) != hipSuccess;\n}\n')
    os.makedirs(os.path.join(PKG, "build", "v"), exist_ok=True)
    os.makedirs(os.path.dirname(VLIB), exist_ok=True)
    tmp = os.path.join(PKG, "build", "v", "kmc_hash_k4sprof.hip")
    open(tmp, "w").write(src)
    H = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-fvisibility=hidden", "-std=c++17",
         "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc")]
    obj = tmp[:-4] + ".o"
    subprocess.check_call(H + ["-c", tmp, "-o", obj])
    others = sorted(os.path.join(PKG, "build", f) for f in os.listdir(os.path.join(PKG, "build"))
                    if f.startswith("kmc_") and f.endswith(".o") and f != "kmc_hash.o")
    subprocess.check_call(H + ["-shared", "-o", VLIB, obj] + others +
                          ["-Wl,--version-script=" + os.path.join(PKG, "libkmc.map"), "-L/opt/rocm/lib", "-lrccl",
                           "-Wl,-rpath,/opt/rocm/lib"])
    print("built", VLIB)


def run():
    os.environ["KMC_LIB"] = VLIB
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import torch
    import kmc
    import genome_synth
    dev = torch.device("cuda:0")
    if "--c4r" in sys.argv:  # the repeat-rich genome of C4R
        data, idx, _, _ = genome_synth.repeat_genome(torch, dev, 3.1)
    else:
        data, idx, _ = genome_synth.grch38_like(torch, dev, 3.1)
    lib = ctypes.CDLL(VLIB)
    out = (ctypes.c_ulonglong * 20)()
    for it in range(3):
        r = kmc.count_canonical(data, idx, 31, flags=kmc.CANON_SOFTMASK)
        torch.cuda.synchronize()
        del r
        assert lib.kmc_k4sprof_read(out) == 0
    sl = (ctypes.c_ulonglong * 40)()
    assert lib.kmc_k4sprof_slots(sl) == 0
    for inst, name in ((0, "common"), (1, "big")):
        for c, cn in enumerate(("9-16", "17-64", "65-256", "257-1024", ">1024")):
            q = sl[inst * 20 + c * 4:inst * 20 + c * 4 + 4]
            if q[0]:
                print("%s crowded slots m %-9s %9d slots, %6.2f distinct keys, %7.0f keys, %8.0f cycles per slot; "
                      "%.0f cycles per list" % (name, cn, q[0], q[1] / q[0], q[3] / q[0], q[2] / q[0], q[2] / 8.0))
    for inst, name in ((0, "common"), (1, "big")):
        v = list(out[10 * inst:10 * inst + 10])
        nl = v[9]
        tot = sum(v[:9])
        print("%s: %d lists, %.0f cycles per list (wave 0)" % (name, nl, tot / max(nl, 1)))
        for i, ph in enumerate(PH):
            print("   %-10s %8.0f cycles  %5.1f %%" % (ph, v[i] / max(nl, 1), 100.0 * v[i] / max(tot, 1)))


if __name__ == "__main__":
    build() if "--build" in sys.argv else run()
