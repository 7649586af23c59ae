/*
 * kmc_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C restatement of the reference's k-mer counting path
 * (axlwild/dna-kmeres-parallel).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product path
 * (dna-kmeres-parallel_amd/) never links or calls it.
 *
 * Parity pinning: this restatement is checked in tests/test_oracle.py against
 *   (1) golden vectors in tests/golden/ produced by oracle/_ref, which compiles the
 *       reference's OWN permutationsCountAll (main.cu:636-646) and permutation()
 *       (utils.h:21-50) from /root/reference (recipe: oracle/Makefile), and
 *   (2) the live oracle/_ref library when it is present.
 *
 * Semantics restated:
 *   - record s occupies data[indices[s] .. indices[s+1]) including one terminator
 *     byte; entryLength E = indices[s+1]-indices[s]            (kernels.h:124)
 *   - windows start at offsets i = 0 .. E-k-1                  (kernels.h:133, main.cu:641)
 *   - bin order is little-endian in the window position: the code of a window is
 *     sum_p code(x[i+p]) * 4^p with A=0,C=1,G=2,T=3            (utils.h:35-47)
 *   - a window holding any byte outside {A,C,G,T} is counted in the CPU path's
 *     bin 0 (main.cu:643-644) and dropped by the GPU path (kernels.h:136-139)
 *   - GPU output layout: sum[s + num_seqs*code], int32, overwritten (kernels.h:142)
 *   - CPU output layout: countResults[1 + code], countResults[0] = invalid (main.cu:598-603)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* A=0 C=1 G=2 T=3, everything else -1 (uppercase only, as permutationsMap keys are). */
static int base_code(unsigned char c) {
    switch (c) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        default: return -1;
    }
}

/* Number of windows of a record of entry length E (terminator included). */
static int64_t n_windows(int64_t E, int k) {
    int64_t n = E - (int64_t)k;
    return n > 0 ? n : 0;
}

/*
 * Histogram of one record in the CPU layout of permutationsCountAll
 * (main.cu:636-646): hist[0] = invalid windows, hist[1 + code] = count.
 * `rec` points at the record's first byte, E = entry length incl. terminator.
 * hist must hold 4^k + 1 ints (k <= 15).
 */
void oracle_count_record_cpu(const char *rec, int64_t E, int k, int32_t *hist) {
    const uint64_t nbins = (uint64_t)1 << (2 * k);
    memset(hist, 0, (nbins + 1) * sizeof(int32_t));
    const int64_t nw = n_windows(E, k);
    if (nw == 0) return;
    /* rolling LE code: code = (code >> 2) | (b << 2(k-1)); run = valid bases ending here */
    uint64_t code = 0;
    int run = 0;
    const int shift = 2 * (k - 1);
    /* prime with the first k-1 bases */
    for (int64_t i = 0; i < nw + k - 1; ++i) {
        int b = base_code((unsigned char)rec[i]);
        if (b < 0) {
            run = 0;
            code = 0;
        } else {
            code = (code >> 2) | ((uint64_t)b << shift);
            ++run;
        }
        int64_t start = i - (k - 1);
        if (start < 0) continue;
        if (run >= k)
            hist[1 + code]++;
        else
            hist[0]++;
    }
}

/*
 * GPU-layout dense histogram over all records (the contract of
 * sumKmereCoincidencesGlobalMemory, generalised to any k as the CPU path is):
 * sum[s + ld*code] for code < 4^k; invalid[s] (optional) = CPU bin 0.
 */
void oracle_count_dense(const char *data, const int64_t *indices, int64_t num_seqs, int k,
                        int32_t *sum, int64_t ld, int32_t *invalid) {
    const uint64_t nbins = (uint64_t)1 << (2 * k);
    if (ld == 0) ld = num_seqs;
    int32_t *hist = (int32_t *)malloc((nbins + 1) * sizeof(int32_t));
    for (int64_t s = 0; s < num_seqs; ++s) {
        const int64_t E = indices[s + 1] - indices[s];
        oracle_count_record_cpu(data + indices[s], E, k, hist);
        for (uint64_t c = 0; c < nbins; ++c) sum[s + ld * (int64_t)c] = hist[1 + c];
        if (invalid) invalid[s] = hist[0];
    }
    free(hist);
}

/*
 * Windowed variant used to check byte-range sharding: only windows whose start
 * position p (absolute offset into data) lies in [win_lo, win_hi) are counted.
 */
void oracle_count_dense_range(const char *data, const int64_t *indices, int64_t num_seqs, int k,
                              int64_t win_lo, int64_t win_hi, int32_t *sum, int64_t ld,
                              int32_t *invalid) {
    const uint64_t nbins = (uint64_t)1 << (2 * k);
    const uint64_t mask = nbins - 1;
    if (ld == 0) ld = num_seqs;
    for (int64_t s = 0; s < num_seqs; ++s) {
        for (uint64_t c = 0; c < nbins; ++c) sum[s + ld * (int64_t)c] = 0;
        if (invalid) invalid[s] = 0;
        const int64_t a = indices[s];
        const int64_t nw = n_windows(indices[s + 1] - a, k);
        for (int64_t i = 0; i < nw; ++i) {
            const int64_t p = a + i;
            if (p < win_lo || p >= win_hi) continue;
            uint64_t code = 0;
            int ok = 1;
            for (int q = 0; q < k; ++q) {
                int b = base_code((unsigned char)data[p + q]);
                if (b < 0) { ok = 0; break; }
                code |= (uint64_t)b << (2 * q);
            }
            if (ok)
                sum[s + ld * (int64_t)(code & mask)]++;
            else if (invalid)
                invalid[s]++;
        }
    }
}

/* LE code of one window (helper for tests); returns -1 when invalid. */
int64_t oracle_window_code(const char *w, int k) {
    uint64_t code = 0;
    for (int q = 0; q < k; ++q) {
        int b = base_code((unsigned char)w[q]);
        if (b < 0) return -1;
        code |= (uint64_t)b << (2 * q);
    }
    return (int64_t)code;
}

/*
 * Pairwise k-mer distance of the reference's step 2 (main.cu:604-619, kernels.h:85-109):
 * d(i,j) = 1 - sum_p min(c_i[p], c_j[p]) / (min(L_i, L_j) - k + 1), packed strict upper
 * triangle, row-major, index getIdxTriangularMatrixRowMajorSeq(i+1, j-i, n) (main.cu:671-673).
 * counts: GPU layout sum[s + n*code]; lens[s] = L_s = entry length - 1.
 * The division is done in float as in the reference ((float)sum / long -> float).
 */
static long tri_idx(long i, long j, long n) {
    return (n * (i - 1) - (((i - 2) * (i - 1)) / 2)) + (j - i);
}

void oracle_pair_distances(const int32_t *sum, const int64_t *lens, int64_t n, int k, float *out) {
    const uint64_t nbins = (uint64_t)1 << (2 * k);
    for (long i = 0; i < n - 1; ++i) {
        for (long j = i + 1; j < n; ++j) {
            long minLength = lens[i] < lens[j] ? (long)lens[i] : (long)lens[j];
            long acc = 0;
            for (uint64_t p = 0; p < nbins; ++p) {
                int32_t a = sum[i + n * (int64_t)p], b = sum[j + n * (int64_t)p];
                acc += a < b ? a : b;
            }
            float d = 1 - (float)acc / (minLength - k + 1);
            out[tri_idx(i + 1, j - i, n)] = d;
        }
    }
}

/*
 * One launch of the reference's GPU step 2, minKmeres2 (kernels.h:85-109): row
 * `cur` against every later record, the sum of minima accumulated in FLOAT in code
 * order (kernels.h:102-104), the lengths from int offsets (kernels.h:99-101).
 * counts in GPU layout sum[s + n*code], nbins = 4^k codes.  Writes only the
 * entries of row `cur` of the packed triangle.
 */
void oracle_min_kmeres2_row(const int32_t *sum, const int32_t *indexes, int n, int cur, int k, float *out) {
    const int nbins = 1 << (2 * k);
    for (int j = cur + 1; j < n; ++j) {
        float s = 0;
        for (int p = 0; p < nbins; ++p) {
            int32_t a = sum[cur + (int64_t)n * p], b = sum[j + (int64_t)n * p];
            s += (float)(a < b ? a : b);
        }
        int le = indexes[cur + 1] - indexes[cur] - 1, lc = indexes[j + 1] - indexes[j] - 1;
        if (le < lc) lc = le;
        s = 1 - s / (float)(lc - k + 1);
        out[tri_idx(cur + 1, j - cur, n)] = s;
    }
}

/*
 * Canonical k-mer counting (kmc_count_canonical_hash, include/kmc.h), k <= 31.
 * NO REFERENCE COUNTERPART (SURVEY.md §8(c) "k=31 canonical: parity unpinned"):
 * this is a self-oracle written from the definition, scalar and independent of
 * the GPU algorithm (sort + run-length instead of hashing).  Windows and validity
 * as oracle_count_record_cpu; key = MSB-first 2-bit code (first base most
 * significant), min'ed with the reverse complement's key unless `forward`.
 * Per record the distinct keys come out sorted ascending with their counts;
 * rec_off[s] .. rec_off[s+1] indexes them.  Returns the distinct total.
 */
static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

static int canon_base_code(uint8_t c, int soft) {
    if (soft && c >= 'a' && c <= 'z') c = (uint8_t)(c - 32);
    switch (c) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        default: return -1;
    }
}

int64_t oracle_count_canonical(const uint8_t *data, const int64_t *indices, int64_t n, int k, int soft, int forward,
                               uint64_t *keys, uint32_t *counts, uint64_t *rec_off) {
    int64_t total = 0;
    rec_off[0] = 0;
    for (int64_t s = 0; s < n; ++s) {
        const int64_t a = indices[s], E = indices[s + 1] - indices[s];
        const int64_t W = E - k > 0 ? E - k : 0;
        uint64_t *tmp = (uint64_t *)malloc((size_t)(W > 0 ? W : 1) * sizeof(uint64_t));
        int64_t m = 0;
        for (int64_t i = 0; i < W; ++i) {
            uint64_t fw = 0, rc = 0;
            int ok = 1;
            for (int q = 0; q < k; ++q) {
                int c = canon_base_code(data[a + i + q], soft);
                if (c < 0) { ok = 0; break; }
                fw = (fw << 2) | (uint64_t)c;                       /* first base most significant */
                rc |= (uint64_t)(3 - c) << (2 * q);                 /* complement, reversed */
            }
            if (!ok) continue;
            tmp[m++] = (forward || fw < rc) ? fw : rc;
        }
        qsort(tmp, (size_t)m, sizeof(uint64_t), cmp_u64);
        for (int64_t i = 0; i < m;) {
            int64_t j = i;
            while (j < m && tmp[j] == tmp[i]) ++j;
            keys[total] = tmp[i];
            counts[total] = (uint32_t)(j - i);
            ++total;
            i = j;
        }
        free(tmp);
        rec_off[s + 1] = (uint64_t)total;
    }
    return total;
}

/*
 * Full-size digest of canonical counting (the config-scale check of
 * kmc_count_canonical_hash, BASELINE configs[3]: 3.1 Gbase at k = 31, where the
 * sort of oracle_count_canonical would need the whole key set in memory).  Same
 * definition as oracle_count_canonical, restated as one rolling pass over ONE
 * record (rec[0 .. E-1), E = entry length incl. terminator; windows i < E - k):
 * the forward key shifts a base in at the bottom, the reverse complement's key
 * shifts the complemented base in at the top, a run counter tracks validity.
 *   *valid  = valid windows of the record
 *   *digest = sum over valid windows of dg_hash(canonical key), mod 2^64
 *             (= sum over the distinct keys of dg_hash(key) * count: any missing,
 *             substituted or miscounted key changes it)
 *   keys/counts = the distinct canonical keys with (dg_hash(key) >> sel_shift) ==
 *             sel_val and their counts, sorted ascending (a subset compared key by
 *             key with the GPU output restricted to the same predicate)
 * dg_hash is splitmix64's finaliser, unrelated to the GPU's partition multiply and
 * feistel list values (kmc_hash.hip), so the selected subset spans every list.
 * Returns the number of selected distinct keys, or -1 when more than `cap`
 * selected windows occur.
 */
uint64_t oracle_dg_hash(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int64_t oracle_canonical_digest(const uint8_t *rec, int64_t E, int k, int soft, int forward, int sel_shift,
                                uint64_t sel_val, uint64_t *valid, uint64_t *digest, uint64_t *keys,
                                uint32_t *counts, int64_t cap) {
    const uint64_t mask = k == 32 ? ~0ull : (1ull << (2 * k)) - 1;
    const int top = 2 * (k - 1);
    uint64_t fw = 0, rc = 0, nv = 0, dg = 0;
    int64_t m = 0;
    int run = 0;
    for (int64_t i = 0; i + 1 < E; ++i) { /* window ending at i starts at i - k + 1 <= E - k - 1 */
        int c = canon_base_code(rec[i], soft);
        if (c < 0) {
            run = 0;
            continue;
        }
        fw = ((fw << 2) | (uint64_t)c) & mask;
        rc = (rc >> 2) | ((uint64_t)(3 - c) << top);
        if (++run < k) continue;
        const uint64_t key = (forward || fw < rc) ? fw : rc;
        const uint64_t h = oracle_dg_hash(key);
        ++nv;
        dg += h;
        if (sel_shift >= 64 || (h >> sel_shift) == sel_val) { /* 64: every key */
            if (m >= cap) return -1;
            keys[m++] = key;
        }
    }
    *valid = nv;
    *digest = dg;
    qsort(keys, (size_t)m, sizeof(uint64_t), cmp_u64);
    int64_t d = 0;
    for (int64_t i = 0; i < m;) {
        int64_t j = i;
        while (j < m && keys[j] == keys[i]) ++j;
        keys[d] = keys[i];
        counts[d] = (uint32_t)(j - i);
        ++d;
        i = j;
    }
    return d;
}
