// kmc_main.cpp — the C++ host driver: successor of the reference program's main()
// (main.cu:120-174) and its GPU driver doParallelKmereDistance (main.cu:215-399),
// calling the HIP kernels only through the C ABI of include/kmc.h.
//
// Flow (the reference's, with its hard-coded constants turned into options):
//   importSeqs / importSeqsNoNL           -> kmc_fasta_load_device (file -> HBM, parsed on the GPU;
//                                            --host-loader: kmc_fasta_load) (main.cu:163, 474-545 / 401-473)
//   step 1: sumKmereCoincidencesGlobalMemory -> kmc_count_dense / kmc_count_multi
//                                               (--dropin: sumKmereCoincidencesGlobalMemory_hip)
//                                                                    (main.cu:287-300)
//   step 2: n x minKmeres2 launches       -> kmc_pair_distances, one launch
//                                               (--dropin: n x minKmeres2_hip) (main.cu:326-344)
//   parallel_results.csv, "%f\n" per entry of the packed upper triangle (main.cu:351-358),
//   and sequential_results.csv, the CPU path's distances (main.cu:194-202)
// and the step-1 / step-2 / total event timers the reference prints.  Extras:
// a histogram dump (--counts, F3 of SURVEY.md §8(f)), k up to 13 (the reference
// kernel is k = 3 only), multi-GPU counting over RCCL (--gpus), canonical k <= 31
// counting (--canonical).  GPU only: there is no CPU counting path here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "kmc.h"
#include "kmc_internal.h"

namespace {

struct Options {
    std::string input;
    std::string out_dir = ".";
    std::string counts_path;
    int k = KMC_DROPIN_K;
    int dialect = 0;
    int64_t max_seqs = KMC_MAX_SEQS_REFERENCE;
    int gpus = 1;
    bool dropin = false;
    bool canonical = false;
    bool softmask = false;
    bool distances = true;
    bool quiet = false;
    bool host_loader = false;
};

void usage(FILE *f) {
    fprintf(f,
            "usage: kmc [options] <input.fasta>\n"
            "       kmc synth OUT.fa RECORDS LENGTH [SEED]   (benchmark input, SURVEY.md 8(d))\n"
            "  -k K              k-mer length (default %d, the reference's K); dense path 1..%d,\n"
            "                    --canonical 1..%d\n"
            "  --dialect D       blank (importSeqs: records end at blank lines, default) or\n"
            "                    nonl (importSeqsNoNL: records also end at '>' headers)\n"
            "  --max-seqs N      the reference's MAX_SEQS cap (default %d, which keeps %d records\n"
            "                    like the reference); 0 = unlimited\n"
            "  --out DIR         directory of parallel_results.csv and sequential_results.csv\n"
            "                    (default .).  Both come from the GPU: without --dropin the two files\n"
            "                    hold the same vector (kmc_pair_distances, exact integer sums, which is\n"
            "                    what the reference's CPU sequentialKmerCount2 computes), so diffing them\n"
            "                    checks nothing; with --dropin parallel_results.csv holds minKmeres2_hip's\n"
            "                    float sums and sequential_results.csv the exact ones (no CPU path here)\n"
            "  --counts FILE     write the histogram: one line per k-mer code, 'kmer<TAB>c_0 .. c_n-1'\n"
            "                    (bin order of permutation(): first base least significant)\n"
            "  --no-distances    step 1 only (no step 2, no CSV)\n"
            "  --gpus N          count on N GPUs (records sharded, RCCL all-reduce)\n"
            "  --dropin          the exact reference launches: sumKmereCoincidencesGlobalMemory_hip\n"
            "                    and one minKmeres2_hip per record (k = %d, int32 offsets)\n"
            "  --canonical       canonical k-mers (k <= %d) instead of the dense histogram; with\n"
            "                    --counts writes 'record<TAB>kmer<TAB>count' lines\n"
            "  --softmask        with --canonical: lowercase acgt count as bases\n"
            "  --host-loader     parse the FASTA on the host (kmc_fasta_load) instead of on the GPU\n"
            "                    (kmc_fasta_load_device); --gpus > 1 always uses the host buffer\n"
            "  -q                quiet (no progress lines)\n",
            KMC_DROPIN_K, KMC_DENSE_MAX_K, KMC_CANON_MAX_K, KMC_MAX_SEQS_REFERENCE, KMC_MAX_SEQS_REFERENCE + 1,
            KMC_DROPIN_K, KMC_CANON_MAX_K);
}

int parse(int argc, char **argv, Options &o) {
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&](const char *what) -> const char * {
            if (i + 1 >= argc) {
                fprintf(stderr, "kmc: %s needs a value\n", what);
                exit(2);
            }
            return argv[++i];
        };
        if (a == "-h" || a == "--help") {
            usage(stdout);
            exit(0);
        } else if (a == "-k") {
            o.k = atoi(next("-k"));
        } else if (a == "--dialect") {
            const std::string d = next("--dialect");
            if (d == "blank") o.dialect = 0;
            else if (d == "nonl") o.dialect = 1;
            else return fprintf(stderr, "kmc: unknown dialect '%s'\n", d.c_str()), 2;
        } else if (a == "--max-seqs") {
            o.max_seqs = atoll(next("--max-seqs"));
        } else if (a == "--out") {
            o.out_dir = next("--out");
        } else if (a == "--counts") {
            o.counts_path = next("--counts");
        } else if (a == "--no-distances") {
            o.distances = false;
        } else if (a == "--gpus") {
            o.gpus = atoi(next("--gpus"));
        } else if (a == "--dropin") {
            o.dropin = true;
        } else if (a == "--canonical") {
            o.canonical = true;
        } else if (a == "--softmask") {
            o.softmask = true;
        } else if (a == "--host-loader") {
            o.host_loader = true;
        } else if (a == "-q") {
            o.quiet = true;
        } else if (!a.empty() && a[0] == '-') {
            return fprintf(stderr, "kmc: unknown option '%s'\n", a.c_str()), 2;
        } else if (o.input.empty()) {
            o.input = a;
        } else {
            return fprintf(stderr, "kmc: more than one input file\n"), 2;
        }
    }
    if (o.input.empty()) return usage(stderr), 2;
    if (o.dropin && o.k != KMC_DROPIN_K)
        return fprintf(stderr, "kmc: --dropin is the k = %d reference launch\n", KMC_DROPIN_K), 2;
    if (o.canonical ? (o.k < 1 || o.k > KMC_CANON_MAX_K) : (o.k < 1 || o.k > KMC_DENSE_MAX_K))
        return fprintf(stderr, "kmc: k = %d out of range\n", o.k), 2;
    if (o.gpus < 1) return fprintf(stderr, "kmc: --gpus must be >= 1\n"), 2;
    if (o.gpus > 1 && (o.dropin || o.canonical))
        return fprintf(stderr, "kmc: --gpus > 1 is for the dense path\n"), 2;
    return 0;
}

#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "kmc: %s failed: %s\n", #x, hipGetErrorString(e_));                    \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

#define KMCCHK(x)                                                                                  \
    do {                                                                                           \
        int rc_ = (x);                                                                             \
        if (rc_ != 0) {                                                                            \
            fprintf(stderr, "kmc: %s failed: %d (%s)\n", #x, rc_, kmc_error_string(rc_));          \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

// k-mer text of a dense code (first base = least significant 2 bits)
std::string dense_kmer(uint64_t code, int k) {
    std::string s(k, 'A');
    for (int p = 0; p < k; ++p) s[p] = "ACGT"[(code >> (2 * p)) & 3];
    return s;
}

// k-mer text of a canonical key (first base = most significant 2 bits)
std::string canon_kmer(uint64_t key, int k) {
    std::string s(k, 'A');
    for (int p = 0; p < k; ++p) s[p] = "ACGT"[(key >> (2 * (k - 1 - p))) & 3];
    return s;
}

int write_counts(const std::string &path, const std::vector<int32_t> &sum, uint64_t n, int k) {
    FILE *f = fopen(path.c_str(), "w");
    if (!f) return fprintf(stderr, "kmc: cannot write %s\n", path.c_str()), 1;
    const uint64_t nb = 1ull << (2 * k);
    std::string line;
    for (uint64_t c = 0; c < nb; ++c) {
        line = dense_kmer(c, k);
        char buf[16];
        for (uint64_t s = 0; s < n; ++s) {
            snprintf(buf, sizeof buf, "\t%d", sum[s + n * c]);
            line += buf;
        }
        line += '\n';
        fwrite(line.data(), 1, line.size(), f);
    }
    return fclose(f) == 0 ? 0 : 1;
}

int write_csv(const std::string &path, const std::vector<float> &d) {
    FILE *f = fopen(path.c_str(), "w");
    if (!f) return fprintf(stderr, "kmc: cannot write %s\n", path.c_str()), 1;
    for (float v : d) fprintf(f, "%f\n", v);  // main.cu:357
    return fclose(f) == 0 ? 0 : 1;
}

float ms_between(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return -1.f;
    return ms;
}

int run(const Options &o) {
    const int k = o.k;
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (ndev < 1) return fprintf(stderr, "kmc: no HIP device\n"), 1;
    if (o.gpus > ndev) return fprintf(stderr, "kmc: --gpus %d but %d device(s)\n", o.gpus, ndev), 1;
    HIPCHK(hipSetDevice(0));
    hipStream_t st = nullptr;
    HIPCHK(hipStreamCreate(&st));
    hipEvent_t ev[6];
    for (auto &e : ev) HIPCHK(hipEventCreate(&e));

    // the record buffer, resident on device 0 for steps 1 and 2: parsed on the GPU
    // from the raw file bytes, or parsed on the host and copied
    kmc_fasta *fa = nullptr;
    char *d_data = nullptr;
    int64_t *d_idx = nullptr;
    uint64_t n = 0, bytes = 0;
    std::vector<int64_t> hidx;
    const bool host = o.host_loader || o.gpus > 1;
    const auto tl0 = std::chrono::steady_clock::now();
    if (host) {
        KMCCHK(kmc_fasta_load(o.input.c_str(), o.dialect, o.max_seqs, &fa));
        n = kmc_fasta_num_seqs(fa);
        bytes = kmc_fasta_data_bytes(fa);
        hidx.assign(kmc_fasta_indices(fa), kmc_fasta_indices(fa) + n + 1);
        HIPCHK(hipMalloc(&d_data, bytes + 16));
        HIPCHK(hipMalloc(&d_idx, (n + 1) * sizeof(int64_t)));
        if (bytes) HIPCHK(hipMemcpyAsync(d_data, kmc_fasta_data(fa), bytes, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(d_idx, hidx.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
    } else {
        KMCCHK(kmc_fasta_load_device(o.input.c_str(), o.dialect, o.max_seqs, &d_data, &bytes, &d_idx, &n, st));
        hidx.resize(n + 1);
        HIPCHK(hipMemcpy(hidx.data(), d_idx, (n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
    }
    const auto tl1 = std::chrono::steady_clock::now();
    if (!o.quiet) {
        printf("K = %d\n", k);
        printf("Size all seqs:%" PRIu64 "\n", bytes);  // main.cu:166-167
        printf("%" PRIu64 " sequences read .\n", n);
        printf("Load (%s parse, file to device): %.1f ms\n", host ? "host" : "GPU",
               std::chrono::duration<double, std::milli>(tl1 - tl0).count());
    }
    if (o.canonical) {
        const unsigned flags = o.softmask ? KMC_CANON_SOFTMASK : 0u;
        const uint64_t cap = bytes > 0 ? bytes : 1;
        uint64_t *d_keys = nullptr, *d_off = nullptr;
        uint32_t *d_cnt = nullptr;
        HIPCHK(hipMalloc(&d_keys, cap * 8));
        HIPCHK(hipMalloc(&d_cnt, cap * 4));
        HIPCHK(hipMalloc(&d_off, (n + 1) * 8));
        uint64_t distinct = 0;
        HIPCHK(hipEventRecord(ev[2], st));
        KMCCHK(kmc_count_canonical_hash(d_data, d_idx, n, k, flags, d_keys, d_cnt, cap, d_off, &distinct, st));
        HIPCHK(hipEventRecord(ev[3], st));
        HIPCHK(hipStreamSynchronize(st));
        if (!o.quiet) {
            printf("Canonical k=%d: %" PRIu64 " distinct (record, k-mer) pairs, %.3f ms\n", k, distinct,
                   ms_between(ev[2], ev[3]));
        }
        if (!o.counts_path.empty()) {
            std::vector<uint64_t> keys(distinct), off(n + 1);
            std::vector<uint32_t> cnt(distinct);
            if (distinct) {
                HIPCHK(hipMemcpy(keys.data(), d_keys, distinct * 8, hipMemcpyDeviceToHost));
                HIPCHK(hipMemcpy(cnt.data(), d_cnt, distinct * 4, hipMemcpyDeviceToHost));
            }
            HIPCHK(hipMemcpy(off.data(), d_off, (n + 1) * 8, hipMemcpyDeviceToHost));
            FILE *f = fopen(o.counts_path.c_str(), "w");
            if (!f) return fprintf(stderr, "kmc: cannot write %s\n", o.counts_path.c_str()), 1;
            for (uint64_t s = 0; s < n; ++s)
                for (uint64_t i = off[s]; i < off[s + 1]; ++i)
                    fprintf(f, "%" PRIu64 "\t%s\t%u\n", s, canon_kmer(keys[i], k).c_str(), cnt[i]);
            if (fclose(f) != 0) return 1;
        }
        HIPCHK(hipFree(d_keys));
        HIPCHK(hipFree(d_cnt));
        HIPCHK(hipFree(d_off));
        HIPCHK(hipFree(d_data));
        HIPCHK(hipFree(d_idx));
        if (fa) kmc_fasta_free(fa);
        return 0;
    }

    const uint64_t nb = 1ull << (2 * k);
    int32_t *d_sum = nullptr;
    HIPCHK(hipMalloc(&d_sum, (nb * n > 0 ? nb * n : 1) * sizeof(int32_t)));
    int *d_idx32 = nullptr;
    if (o.dropin) {
        if (bytes > (uint64_t)INT32_MAX) return fprintf(stderr, "kmc: --dropin needs < 2 GiB of sequence\n"), 1;
        std::vector<int> i32(hidx.begin(), hidx.end());
        HIPCHK(hipMalloc(&d_idx32, (n + 1) * sizeof(int)));
        HIPCHK(hipMemcpy(d_idx32, i32.data(), (n + 1) * sizeof(int), hipMemcpyHostToDevice));
    }

    // step 1 (main.cu:287-300)
    HIPCHK(hipEventRecord(ev[2], st));
    std::vector<int32_t> hsum;
    if (o.dropin) {
        KMCCHK(sumKmereCoincidencesGlobalMemory_hip(d_data, d_idx32, (unsigned)n, d_sum, st));
    } else if (o.gpus > 1) {
        // host-buffer multi-GPU count (shards + RCCL all-reduce), result on the host
        hsum.assign(nb * n, 0);
        KMCCHK(kmc_count_multi(kmc_fasta_data(fa), hidx.data(), n, bytes, k, o.gpus, nullptr, hsum.data(), nullptr));
        if (!hsum.empty())
            HIPCHK(hipMemcpyAsync(d_sum, hsum.data(), hsum.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
    } else {
        KMCCHK(kmc_count_dense(d_data, d_idx, n, bytes, k, d_sum, nullptr, nullptr, 0, st));
    }
    HIPCHK(hipEventRecord(ev[3], st));
    HIPCHK(hipEventSynchronize(ev[3]));
    if (o.gpus <= 1) {  // the deferred status of the (asynchronous) count on this device
        int dev = 0;
        HIPCHK(hipGetDevice(&dev));
        KMCCHK(kmc_dense_status(dev));
    }
    const float t1 = ms_between(ev[2], ev[3]);
    if (!o.quiet) {
        printf("Elapsed parallel timer step 1: %g ms, %g secs\n", t1, t1 / 1000);  // main.cu:300
    }

    // step 2 (main.cu:326-344)
    std::vector<float> mins, seq;
    const uint64_t npairs = n * (n > 0 ? n - 1 : 0) / 2;
    if (o.distances && npairs > 0) {
        float *d_mins = nullptr;
        HIPCHK(hipMalloc(&d_mins, npairs * sizeof(float)));
        HIPCHK(hipMemsetAsync(d_mins, 0, npairs * sizeof(float), st));
        HIPCHK(hipEventRecord(ev[4], st));
        if (o.dropin) {
            for (uint64_t i = 0; i < n; ++i) {
                KMCCHK(minKmeres2_hip(d_sum, d_mins, (int)n, (int)i, d_idx32, st));
                HIPCHK(hipStreamSynchronize(st));  // main.cu:328
            }
        } else {
            KMCCHK(kmc_pair_distances(d_sum, n, d_idx, n, k, d_mins, nullptr, 0, st));
        }
        HIPCHK(hipEventRecord(ev[5], st));
        HIPCHK(hipEventSynchronize(ev[5]));
        const float t2 = ms_between(ev[4], ev[5]);
        if (!o.quiet) {
            printf("Elapsed parallel step 2 timer: %g ms, %g secs\n", t2, t2 / 1000);  // main.cu:344
            const float tt = ms_between(ev[2], ev[5]);
            printf("Total time elapsed parallel: %g ms, %g secs\n", tt, tt / 1000);  // main.cu:350
        }
        mins.resize(npairs);
        HIPCHK(hipMemcpy(mins.data(), d_mins, npairs * sizeof(float), hipMemcpyDeviceToHost));
        if (o.dropin) {
            // the CPU path's distances (exact integer sums) for sequential_results.csv
            KMCCHK(kmc_pair_distances(d_sum, n, d_idx, n, k, d_mins, nullptr, 0, st));
            seq.resize(npairs);
            HIPCHK(hipMemcpy(seq.data(), d_mins, npairs * sizeof(float), hipMemcpyDeviceToHost));
        }
        HIPCHK(hipFree(d_mins));
    }
    if (o.distances) {
        // the reference writes both files for diffing (main.cu:178, 194-202, 216, 351-358):
        // sequential_results.csv holds sequentialKmerCount2's distances (exact integer
        // sums, here kmc_pair_distances), parallel_results.csv the GPU path's (the
        // same numbers, or minKmeres2's float sums with --dropin)
        if (write_csv(o.out_dir + "/parallel_results.csv", mins)) return 1;
        if (write_csv(o.out_dir + "/sequential_results.csv", o.dropin ? seq : mins)) return 1;
    }
    if (!o.counts_path.empty()) {
        if (hsum.empty() && nb * n > 0) {
            hsum.resize(nb * n);
            HIPCHK(hipMemcpy(hsum.data(), d_sum, hsum.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
        }
        if (write_counts(o.counts_path, hsum, n, k)) return 1;
    }
    HIPCHK(hipFree(d_sum));
    if (d_idx32) HIPCHK(hipFree(d_idx32));
    HIPCHK(hipFree(d_data));
    HIPCHK(hipFree(d_idx));
    for (auto &e : ev) HIPCHK(hipEventDestroy(e));
    HIPCHK(hipStreamDestroy(st));
    if (fa) kmc_fasta_free(fa);
    return 0;
}


// `kmc synth OUT.fa RECORDS LENGTH [SEED]`: the SURVEY.md §8(d) benchmark input as a
// FASTA file: records of LENGTH bases in 80 columns, '>r%04d' headers, records
// separated by one blank line (the importSeqs dialect, also read by NoNL), no
// final blank line.  Base g of the concatenated records is "ACGT"[(x_{g/32} >>
// 2(g%32)) & 3], x_n = splitmix64 output n (kmc_synth_fill's stream, so the parsed
// buffer equals kmc_synth_fill's).  Lines are generated by host threads.
int synth_main(int argc, char **argv) {
    if (argc < 5) return fprintf(stderr, "usage: kmc synth OUT.fa RECORDS LENGTH [SEED]\n"), 2;
    const char *path = argv[2];
    const uint64_t nrec = strtoull(argv[3], nullptr, 10), len = strtoull(argv[4], nullptr, 10);
    const uint64_t seed = argc > 5 ? strtoull(argv[5], nullptr, 0) : 0x5EED0008ull;
    FILE *f = fopen(path, "wb");
    if (!f) return fprintf(stderr, "kmc: cannot write %s\n", path), 1;
    const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    constexpr uint64_t kBlockBases = 80ull << 20;  // whole lines per block
    std::vector<std::string> buf(nth);
    for (uint64_t r = 0; r < nrec; ++r) {
        char hdr[32];
        snprintf(hdr, sizeof hdr, "%s>r%04llu\n", r ? "\n" : "", (unsigned long long)r);
        fputs(hdr, f);
        for (uint64_t b0 = 0; b0 < len; b0 += kBlockBases * nth) {
            std::vector<std::thread> th;
            for (unsigned t = 0; t < nth; ++t) {
                th.emplace_back([&, t]() {
                    std::string &o = buf[t];
                    o.clear();
                    const uint64_t lo = b0 + t * kBlockBases;
                    if (lo >= len) return;
                    const uint64_t hi = std::min(len, lo + kBlockBases);
                    o.reserve((hi - lo) + (hi - lo) / 80 + 2);
                    for (uint64_t i = lo; i < hi; i += 80) {
                        const uint64_t e = std::min(hi, i + 80);
                        uint64_t xn = ~0ull, x = 0;
                        for (uint64_t j = i; j < e; ++j) {
                            const uint64_t g = r * len + j;
                            if ((g >> 5) != xn) x = kmc::splitmix64_at(seed, xn = g >> 5);
                            o.push_back("ACGT"[(x >> (2 * (g & 31))) & 3]);
                        }
                        o.push_back('\n');
                    }
                });
            }
            for (auto &x : th) x.join();
            for (unsigned t = 0; t < nth; ++t)
                if (!buf[t].empty() && fwrite(buf[t].data(), 1, buf[t].size(), f) != buf[t].size())
                    return fclose(f), fprintf(stderr, "kmc: write failed\n"), 1;
        }
    }
    return fclose(f) == 0 ? 0 : 1;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc > 1 && std::string(argv[1]) == "synth") return synth_main(argc, argv);
    Options o;
    const int rc = parse(argc, argv, o);
    if (rc) return rc;
    return run(o);
}
