"""Diagnostic (round 5): where the k = 8 histogram launch spends the time that does
not shrink with the shard (an 8-way shard's kernel is ~20 us longer than 1/8 of
the whole job's).

Builds lib/variants/libkmc_denseprof.so from the current kmc_dense.hip with
s_memrealtime reads (100 MHz, one clock for every CU) patched in -- the product
source carries none of it: per workgroup its entry, the end of its setup (LDS
clear, first record), per wave the end of its tiles in each piece, the end of the
piece's barrier and of its flush, and its exit.  `--build` on the build host; on
the GPU box (no flag) it runs rank 0 of the bench's N-way strong-scaling shards
(scripts/shardbench.py's setup) and prints, for the last of 20 launches, the
spread of those times across the grid in microseconds."""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dna-kmeres-parallel_amd")
VLIB = os.path.join(PKG, "lib", "variants", "libkmc_denseprof.so")
NSLOT = 256  # per workgroup: 0 entry, 1 setup, 2 + 16 * piece + wave (pieces 0, 1), 34 + 3 * piece: sync/flush/-,
             # 40 exit, 48 + 16 * segment + wave: arrival at the hot-half scan, 240 + segment: scan done


def build():
    src = open(os.path.join(PKG, "csrc", "kmc_dense.hip")).read()

    def rep(a, b):
        nonlocal src
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    rep("template <int K, int R, int HM, int BLOCK>\nstruct DenseOp {",
        "__device__ unsigned long long g_dprof[1024][%d];\n"
        "#define TSW(i) (g_dprof[blockIdx.x][(i)] = __builtin_amdgcn_s_memrealtime())\n"
        "template <int K, int R, int HM, int BLOCK>\nstruct DenseOp {" % NSLOT)
    rep("    uint32_t nwin = 0u;  // HM 3: windows this lane added\n",
        "    uint32_t nwin = 0u;  // HM 3: windows this lane added\n    int pseg = 0;\n")
    rep("        if constexpr (HM == 3) {\n            lds_barrier();\n            p16_scan<BLOCK, 32768u>(pc);\n"
        "            lds_barrier();\n        }\n",
        "        if constexpr (HM == 3) {\n"
        "            if ((threadIdx.x & 63) == 0 && pseg < 12) TSW(48 + 16 * pseg + (threadIdx.x >> 6));\n"
        "            lds_barrier();\n            p16_scan<BLOCK, 32768u>(pc);\n            lds_barrier();\n"
        "            if (threadIdx.x == 0 && pseg < 12) TSW(240 + pseg);\n            ++pseg;\n        }\n")
    rep("    if (tb < te) {\n        const int64_t R0",
        "    if (tid == 0) TSW(0);\n    if (tb < te) {\n        const int64_t R0")
    rep("        P16Ctx pc;\n", "        if (tid == 0) TSW(1);\n        P16Ctx pc;\n")
    rep("                stream_chunks<K, kChunk, Op::kSegChunks>(p.data, tp0, tp1, ps, pe, g.rl, g.rh, lane, &misc[7], op);\n",
        "                stream_chunks<K, kChunk, Op::kSegChunks>(p.data, tp0, tp1, ps, pe, g.rl, g.rh, lane, &misc[7], op);\n"
        "                if (lane == 0 && npieces < 2) TSW(2 + 16 * npieces + (tid >> 6));\n")
    rep("            const bool entire = (ps == ca) && (pe == ce);\n",
        "            if (tid == 0 && npieces < 2) TSW(34 + 3 * npieces);\n"
        "            const bool entire = (ps == ca) && (pe == ce);\n")
    rep("            ++npieces;\n", "            if (tid == 0 && npieces < 2) TSW(35 + 3 * npieces);\n            ++npieces;\n")
    rep("    if (tid == 0) {\n        p.slot_rec[2 * w] = slot0;",
        "    if (tid == 0) {\n        TSW(40);\n        g_dprof[blockIdx.x][41] = (unsigned long long)(tb < te ? 1 : 0);\n"
        "        p.slot_rec[2 * w] = slot0;")
    src += ('\nextern "C" __attribute__((visibility("default"))) int kmc_denseprof_read(unsigned long long *out) {\n'
            '    return hipMemcpyFromSymbol(out, HIP_SYMBOL(kmc::g_dprof), sizeof(kmc::g_dprof)) != hipSuccess;\n}\n'
            'extern "C" __attribute__((visibility("default"))) int kmc_denseprof_clear() {\n'
            '    std::vector<unsigned long long> z(sizeof(kmc::g_dprof) / 8, 0ull);\n'
            '    return hipMemcpyToSymbol(HIP_SYMBOL(kmc::g_dprof), z.data(), sizeof(kmc::g_dprof)) != hipSuccess;\n}\n')
    os.makedirs(os.path.join(PKG, "build", "v"), exist_ok=True)
    os.makedirs(os.path.dirname(VLIB), exist_ok=True)
    tmp = os.path.join(PKG, "build", "v", "kmc_dense_prof.hip")
    open(tmp, "w").write(src)
    H = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-fvisibility=hidden", "-std=c++17",
         "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc")]
    obj = tmp[:-4] + ".o"
    subprocess.check_call(H + ["-c", tmp, "-o", obj])
    others = sorted(os.path.join(PKG, "build", f) for f in os.listdir(os.path.join(PKG, "build"))
                    if f.startswith("kmc_") and f.endswith(".o") and f != "kmc_dense.o")
    subprocess.check_call(H + ["-shared", "-o", VLIB, obj] + others +
                          ["-Wl,--version-script=" + os.path.join(PKG, "libkmc.map"), "-L/opt/rocm/lib", "-lrccl",
                           "-Wl,-rpath,/opt/rocm/lib"])
    print("built", VLIB)


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))]


def run(worlds, steps):
    import ctypes
    import json
    os.environ["KMC_LIB"] = VLIB
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    import bench
    import kmc
    lib = ctypes.CDLL(VLIB)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    k, L, nrec = 8, 1_000_000_000, 10
    for world in worlds:
        plan = bench.rank_plan("strong", world, 0, nrec, L, k)
        base, hold_hi = plan["hold"]
        (win_lo, win_hi), (read_lo, read_hi) = plan["win"], plan["read"]
        data = torch.empty(max(hold_hi - base, 16), dtype=torch.uint8, device=dev)
        kmc.synth_fill_range(data, base, hold_hi, L, bench.SEED_BASE + k)
        idx = torch.from_numpy(plan["indices"]).to(dev)
        out = torch.empty((1 << 16, plan["n_tot"]), dtype=torch.int32, device=dev)
        args = kmc.dense_args(data, idx, k, out.view(-1), read=(read_lo, read_hi), win=(win_lo, win_hi),
                              data_offset=base)
        ws = torch.empty(max(kmc.dense_ex_workspace_size(args), 1), dtype=torch.uint8, device=dev)
        args = kmc.dense_args(data, idx, k, out.view(-1), read=(read_lo, read_hi), win=(win_lo, win_hi),
                              workspace=ws, data_offset=base)
        for _ in range(steps):
            kmc.count_dense_ex(args, stream)
        torch.cuda.synchronize()
        buf = np.zeros((1024, NSLOT), np.uint64)
        assert lib.kmc_denseprof_clear() == 0
        for _ in range(2):
            kmc.count_dense_ex(args, stream)
        torch.cuda.synchronize()
        assert lib.kmc_denseprof_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
        used = buf[:, 41] == 1
        b = buf[used].astype(np.int64)
        t0 = b[:, 0].min()
        us = lambda x: (x - t0) / 100.0  # 100 MHz ticks -> us
        entry, setup, exit_ = us(b[:, 0]), us(b[:, 1]), us(b[:, 40])
        p0w = us(b[:, 2:18])            # piece 0: per wave end of its tiles
        p0s, p0f = us(b[:, 34]), us(b[:, 35])
        two = b[:, 37] > 0
        rep = {"world": world, "workgroups": int(used.sum()), "pieces2": int(two.sum()),
               "kernel_span_us": float(exit_.max()),
               "entry_us": [float(entry.min()), float(np.median(entry)), float(entry.max())],
               "setup_us(per wg)": float(np.median(setup - entry)),
               "piece0_wave_end_us": [float(p0w.min()), float(np.median(p0w)), float(p0w.max())],
               "piece0_wave_spread_in_wg_us(median)": float(np.median(p0w.max(1) - p0w.min(1))),
               "piece0_sync_us(median after last wave)": float(np.median(p0s - p0w.max(1))),
               "piece0_flush_us(median)": float(np.median(p0f - p0s)),
               "exit_us": [float(exit_.min()), float(np.median(exit_)), float(exit_.max())],
               "exit_p90_us": float(pct(list(exit_), 0.9)),
               # (round 6) per XCD (workgroup id mod 8, the dispatcher's round robin):
               # median / max exit and median duration (exit - entry)
               "per_xcd_exit_med_max_dur_us": [
                   [round(float(np.median(exit_[np.nonzero(used)[0] % 8 == x])), 1),
                    round(float(exit_[np.nonzero(used)[0] % 8 == x].max()), 1),
                    round(float(np.median((exit_ - entry)[np.nonzero(used)[0] % 8 == x])), 1)] for x in range(8)],
               "duration_us_min_med_max": [float((exit_ - entry).min()), float(np.median(exit_ - entry)),
                                           float((exit_ - entry).max())]}
        # the hot-half scans (barriers every kHm3Scan tiles per wave): per segment the
        # spread of the waves' arrivals, and the scan itself (single-piece workgroups)
        one = b[~two]
        segs = []
        for sg in range(12):
            arr = one[:, 48 + 16 * sg:64 + 16 * sg]
            if not (arr > 0).all():
                break
            prev = one[:, 240 + sg - 1] if sg else one[:, 1]
            dur = arr - prev[:, None]
            segs.append({"seg": sg, "wave_us_min_mean_max": [
                float(np.median(dur.min(1)) / 100), float(np.median(dur.mean(1)) / 100), float(np.median(dur.max(1)) / 100)],
                "scan_us": float(np.median(one[:, 240 + sg] - arr.max(1)) / 100)})
        if segs:  # after the last scan: the waves' remaining tiles
            tail = one[:, 2:18] - one[:, 240 + len(segs) - 1][:, None]
            segs.append({"seg": "tail", "wave_us_min_mean_max": [
                float(np.median(tail.min(1)) / 100), float(np.median(tail.mean(1)) / 100),
                float(np.median(tail.max(1)) / 100)]})
        rep["segments"] = segs
        if two.any():
            p1w = us(b[two][:, 18:34])
            rep["piece1_flush_us(median)"] = float(np.median(us(b[two][:, 38]) - us(b[two][:, 37])))
            rep["piece1_wave_end_max_us"] = float(p1w.max())
        print(json.dumps(rep), flush=True)
        del data, out, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--worlds", default="1,8")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    if a.build:
        build()
    else:
        run([int(x) for x in a.worlds.split(",")], a.steps)
