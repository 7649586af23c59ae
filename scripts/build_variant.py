#!/usr/bin/env python3
"""Build lib/variants/libkmc_NAME.so: the current sources with text replacements in
one or more of them (measurement variants; the product sources carry no switch).
  python scripts/build_variant.py NAME FILE OLD NEW [FILE OLD NEW ...]
FILE is a csrc/ file name; OLD must occur exactly once (OLD = "@file": FILE's source
is taken whole from the path NEW, e.g. an earlier revision from `git show`).  The other translation
units are the in-tree objects of `make` (build them first).  Time a variant with
KMC_LIB=dna-kmeres-parallel_amd/lib/variants/libkmc_NAME.so python scripts/kbench.py ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dna-kmeres-parallel_amd")


def main():
    name, rest = sys.argv[1], sys.argv[2:]
    assert len(rest) % 3 == 0 and rest, __doc__
    patched = {}
    for i in range(0, len(rest), 3):
        f, old, new = rest[i:i + 3]
        old, new = old.encode().decode("unicode_escape"), new.encode().decode("unicode_escape")
        if old == "@file":
            patched[f] = open(new).read()
            continue
        src = patched.get(f) or open(os.path.join(PKG, "csrc", f)).read()
        assert src.count(old) == 1, (f, old)
        patched[f] = src.replace(old, new)
    vdir = os.path.join(PKG, "build", "v_" + name)
    os.makedirs(vdir, exist_ok=True)
    os.makedirs(os.path.join(PKG, "lib", "variants"), exist_ok=True)
    H = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-fvisibility=hidden", "-std=c++17",
         "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc")]
    objs = []
    H = H[:-1] + ["-I" + vdir] + H[-1:]  # patched headers (.h) ahead of csrc/
    for f, src in patched.items():  # every patched file first: a patched header is seen by all of them
        open(os.path.join(vdir, f), "w").write(src)
    for f in patched:
        tmp = os.path.join(vdir, f)
        if f.endswith(".h"):  # (the patched .hip / .cpp files see it; the other objects keep csrc/'s)
            continue
        obj = tmp.rsplit(".", 1)[0] + ".o"
        cc = H if f.endswith(".hip") else ["g++", "-O3", "-fPIC", "-fvisibility=hidden", "-std=c++17",
                                           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"] + H[-2:]
        subprocess.check_call(cc + ["-c", tmp, "-o", obj])
        objs.append(obj)
    done = {f.rsplit(".", 1)[0] + ".o" for f in patched if not f.endswith(".h")}
    others = sorted(os.path.join(PKG, "build", f) for f in os.listdir(os.path.join(PKG, "build"))
                    if f.startswith("kmc_") and f.endswith(".o") and f not in done)
    out = os.path.join(PKG, "lib", "variants", "libkmc_%s.so" % name)
    subprocess.check_call(H + ["-shared", "-o", out] + objs + others +
                          ["-Wl,--version-script=" + os.path.join(PKG, "libkmc.map"), "-L/opt/rocm/lib", "-lrccl",
                           "-Wl,-rpath,/opt/rocm/lib"])
    print("built", out)


if __name__ == "__main__":
    main()
