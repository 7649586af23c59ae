/*
 * kmc.h — C ABI of the MI355X-native k-mer counter (libkmc.so).
 *
 * Drop-in boundary for the hot path of axlwild/dna-kmeres-parallel: the step-1
 * launch of sumKmereCoincidencesGlobalMemory (kernels.h:113, launched at
 * main.cu:290) and its host-side feeders.  Plain C: pointers, sizes and int
 * error codes only (0 = success, hipError_t values pass through, library codes
 * are >= 1000).  Every device entry point is asynchronous on the given stream
 * and never calls exit().
 *
 * Count layout (identical to the reference, kernels.h:142): int32
 * sum[s + ld*code] ("k-mer-major, record-minor"), ld = num_seqs unless stated,
 * code = sum_p code(x[i+p]) * 4^p with A=0,C=1,G=2,T=3 (first base least
 * significant: the bin order of permutation(), utils.h:21-50).  Windows holding
 * any byte other than uppercase A/C/G/T are not counted (kernels.h:136-139);
 * their number per record is the reference CPU path's bin 0 (main.cu:643-644)
 * and is available through the optional `invalid` output.
 *
 * Records follow the reference's buffer convention (main.cu:474-545): record s
 * occupies data[indices[s] .. indices[s+1]), whose last byte is a terminator;
 * windows start at offsets 0 .. (indices[s+1]-indices[s]) - k - 1.
 */
#ifndef KMC_H
#define KMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* libkmc.so is built with hidden visibility: exactly the entry points declared
 * here are exported (tests/test_abi.py compares `nm -D` with this header). */
#if defined(__GNUC__) || defined(__clang__)
#define KMC_API __attribute__((visibility("default")))
#else
#define KMC_API
#endif

#ifndef KMC_HIP_STREAM_T_DEFINED
#define KMC_HIP_STREAM_T_DEFINED
typedef struct ihipStream_t *hipStream_t; /* identical to HIP's own typedef */
#endif

/* Compile-time k of the exact drop-in entry point (the reference's K, kernels.h:11-15). */
#ifndef KMC_DROPIN_K
#define KMC_DROPIN_K 3
#endif

/* Largest k of the dense (4^k-bin) histogram path. */
#define KMC_DENSE_MAX_K 13

/* Reference loader cap (main.cu:30). */
#define KMC_MAX_SEQS_REFERENCE 100

enum kmc_status {
    KMC_OK = 0,
    KMC_ERR_INVALID_ARG = 1001,   /* null pointer, bad size, bad range */
    KMC_ERR_UNSUPPORTED_K = 1002, /* k outside the supported range of the entry point */
    KMC_ERR_ALIGNMENT = 1003,     /* pointer not aligned as the entry point requires */
    KMC_ERR_WORKSPACE = 1004,     /* caller workspace smaller than *_workspace_size() */
    KMC_ERR_IO = 1005,            /* file cannot be opened/read */
    KMC_ERR_NOMEM = 1006,         /* host or device allocation failed */
    KMC_ERR_RCCL = 1007,          /* RCCL call failed */
    KMC_ERR_NO_DEVICE = 1008,     /* no HIP device visible */
    KMC_ERR_CAPACITY = 1009,      /* caller output smaller than the result (size reported) */
    KMC_ERR_RECORD_TOO_LONG = 1010, /* a record has >= 2^31 windows in one dense call: int32 counts could wrap */
    KMC_ERR_INTERNAL = 1011         /* a device-side bound check fired (a library defect): the access was
                                       skipped and the call's outputs are not valid (kmc_count_canonical_hash) */
};

/* Human-readable text for a kmc_status or hipError_t code (static storage). */
KMC_API const char *kmc_error_string(int code);

/* Library version: major*10000 + minor*100 + patch.  200 (0.2.0): kmc_dense_args
 * ends with `status` (below) and KMC_ERR_INTERNAL exists; a caller built against
 * an older header (0.1.0, a shorter kmc_dense_args) must not call
 * kmc_count_dense_ex on this library -- check kmc_version() >= 200 first. */
#define KMC_VERSION 200
KMC_API int kmc_version(void);

/* ------------------------------------------------------------------------ */
/* Exact drop-in for the reference launch
 *     sumKmereCoincidencesGlobalMemory<<<54018, PERMS_KMERES>>>(data, indices, num_seqs, sum)
 * (kernels.h:113, main.cu:290).  Same arguments, same meaning, same layout:
 *   data     device (or managed) bytes, '\0'-terminated records
 *   indices  device (or managed) int[num_seqs + 1] record offsets
 *   sum      device (or managed) int[4^KMC_DROPIN_K * num_seqs]; every entry
 *            (s < num_seqs, code < 4^K) is overwritten
 * k = KMC_DROPIN_K (3, like the reference).  No pattern table (c_perms) is
 * needed: codes are computed arithmetically in the reference's bin order.
 * Like the reference's char *data, `data` may point anywhere in a buffer (for
 * example data + off): the library rounds it down to 16 bytes internally and
 * biases the offsets (the rounded-down bytes share data's page and are never
 * counted).  Uses a library-owned device workspace (allocated on first use per device).
 * Asynchronous on `stream` (0 = the null stream); the reference synchronises
 * after the launch (main.cu:291), so should the caller. */
KMC_API int sumKmereCoincidencesGlobalMemory_hip(char *data, int *indices, unsigned num_seqs, int *sum,
                                         hipStream_t stream);

/* ------------------------------------------------------------------------ */
/* k-generic, 64-bit-offset dense counter: the generalisation the reference's CPU
 * path (permutationsCountAll, main.cu:636-646) computes for any k, on the GPU.
 *   data        device pointer (any alignment), readable for [0, data_bytes)
 *   indices     device int64[num_seqs + 1]
 *   k           1 .. KMC_DENSE_MAX_K
 *   sum         device int32[4^k * num_seqs], overwritten (layout above)
 *   invalid     optional device int32[num_seqs]: invalid windows (CPU bin 0)
 *   workspace   device scratch of kmc_count_dense_workspace_size() bytes, or
 *               NULL to use a library-owned buffer, one per device, shared by
 *               every NULL-workspace call on that device: such calls must not
 *               overlap (one stream, or the caller serialises them), and they are
 *               not graph-capture safe.  Concurrent calls pass their own workspace.
 * The same holds for the NULL workspace of kmc_pair_distances.
 * Counts are int32 like the reference's (main.cu:598,637: int counters, and the
 * kernel's int sum, kernels.h:142), which never meets a record of 2^31 windows
 * (its loader's int offsets stop at 2 GiB).  The 64-bit offsets here do, so a call
 * in which some record has 2^31 or more windows in range (valid or not) reports
 * KMC_ERR_RECORD_TOO_LONG through the call's deferred status (below) rather than
 * passing bins or invalid counts that may have wrapped as valid: count such a record in
 * window ranges of fewer than 2^31 windows (kmc_count_dense_ex) and add the parts
 * in 64-bit integers.  The offsets live on the device, so the check runs there. */
KMC_API size_t kmc_count_dense_workspace_size(int k, uint64_t num_seqs, uint64_t data_bytes, int device);

KMC_API int kmc_count_dense(const char *data, const int64_t *indices, uint64_t num_seqs, uint64_t data_bytes,
                    int k, int32_t *sum, int32_t *invalid, void *workspace, size_t workspace_bytes,
                    hipStream_t stream);

/* Extended form used for sharding: counts only the windows whose start offset
 * lies in [win_lo, win_hi), reading only data[read_lo, read_hi) (a shard plus its
 * (k-1)-byte halo), and writes sum[s + sum_ld*code] for every record s (zeros for
 * records with no window in range).  Sums of shards covering disjoint window
 * ranges equal the unsharded counts. */
typedef struct kmc_dense_args {
    const char *data;        /* device; global byte p is data[p] (only [read_lo, read_hi) is read) */
    const int64_t *indices;  /* device int64[num_seqs + 1], global offsets */
    uint64_t num_seqs;
    int k;
    int32_t *sum;            /* device */
    uint64_t sum_ld;         /* row stride of sum (>= num_seqs); 0 -> num_seqs */
    int32_t *invalid;        /* optional device int32[num_seqs] */
    uint64_t read_lo, read_hi;
    uint64_t win_lo, win_hi;
    void *workspace;
    size_t workspace_bytes;
    int32_t *status;         /* optional device-visible int32 (device memory or host-mapped), zeroed by
                                the caller before the call: this call's kernels store a kmc_status code
                                in it (KMC_ERR_CAPACITY, KMC_ERR_RECORD_TOO_LONG) when its counts are
                                not valid; read it after the stream has synchronised.  NULL: the
                                device's library flag, reported by kmc_dense_status(). */
} kmc_dense_args;

KMC_API size_t kmc_count_dense_ex_workspace_size(const kmc_dense_args *args, int device);
KMC_API int kmc_count_dense_ex(const kmc_dense_args *args, hipStream_t stream);

/* Deferred device-side status of the asynchronous dense calls on `device` that
 * passed no status word of their own (kmc_count_dense, the drop-in, and
 * kmc_count_dense_ex with status == NULL).  Two conditions are detected on the
 * device, where the offsets live: (1) the k = 8 kernel keeps its 16-bit counters
 * exact with spill entries whose number per workgroup is bounded analytically (one
 * per >= 4096 windows); should a workgroup ever emit more than its workspace holds,
 * the counts would be short: KMC_ERR_CAPACITY; (2) a record with 2^31 or more
 * windows in range: KMC_ERR_RECORD_TOO_LONG (above).  The kernels store the code in
 * a host-mapped word of the device.  This call (after the stream has synchronised)
 * returns the code stored since the last query, KMC_OK if none, and clears it.
 * No other entry point reads or clears it, so a failure is never reported to an
 * unrelated later call; callers that run dense calls concurrently on one device
 * pass each call its own status word instead. */
KMC_API int kmc_dense_status(int device);

/* ------------------------------------------------------------------------ */
/* Sharding.  A shard counts the windows starting in
 * [win_lo, win_hi) and reads data[read_lo, read_hi) = its bytes plus a k-1 byte
 * halo.  kmc_plan_shards cuts the buffer [indices[0], indices[num_seqs]) into
 * nshards contiguous, byte-balanced ranges whose inner cut points are multiples
 * of `align` (0 -> 4096); a shard may be empty.  Host memory, no device needed. */
typedef struct kmc_shard {
    uint64_t win_lo, win_hi;
    uint64_t read_lo, read_hi;
} kmc_shard;

KMC_API int kmc_plan_shards(const int64_t *indices, uint64_t num_seqs, int k, int nshards, uint64_t align,
                    kmc_shard *out);

/* Single-process multi-GPU count of a host buffer (the C++ host driver's path):
 * shards the buffer over `ndev` devices (kmc_plan_shards), copies each shard +
 * halo to its device, counts it there (kmc_count_dense_ex) and sums the per-device
 * matrices with one RCCL all-reduce (int32, sum) over xGMI; the result
 * sum[s + num_seqs*code] (and optional invalid[s]) is copied back to host
 * memory.  devices == NULL -> 0 .. ndev-1 (distinct devices).  Synchronous.
 * One host thread per device streams its shard through pinned staging buffers,
 * so all devices load concurrently.  The RCCL communicators of a device set (keyed
 * by the sorted device list) are created on its first call, and each device's
 * stream, pinned staging and device buffers (grow-only) on its first use; all are
 * reused until kmc_multi_release().  Thread-safe: a call holds its devices (locked
 * in ascending order) from load to copy-back, so calls whose sets share a device
 * take turns (RCCL communicators are not reentrant), calls on disjoint sets run
 * concurrently, and a set whose collective failed is rebuilt by the next call.
 * Each shard's count carries its own status word: KMC_ERR_CAPACITY /
 * KMC_ERR_RECORD_TOO_LONG (kmc_count_dense_ex) are returned by this call.  A record
 * of 2^31 or more windows is refused up front (KMC_ERR_RECORD_TOO_LONG, checked on
 * the host offsets before any device work): its shards would each hold fewer, but
 * the all-reduce would add their int32 parts.  HIP failures after the all-reduce
 * return their hipError_t; KMC_ERR_RCCL only when an RCCL call failed.
 * Retention: the cached per-device buffers are sized to the largest shard + halo
 * seen (GBs per device for Gbase inputs) plus 64 MB of pinned staging, and are
 * held until kmc_multi_release().  kmc_set_reserved_cus does not apply here (the
 * worker threads count with every CU). */
KMC_API int kmc_count_multi(const char *data, const int64_t *indices, uint64_t num_seqs, uint64_t data_bytes, int k,
                    int ndev, const int *devices, int32_t *sum, int32_t *invalid);
/* Destroys the communicators and frees the per-device state cached by
 * kmc_count_multi (waits for calls in flight). */
KMC_API int kmc_multi_release(void);

/* ------------------------------------------------------------------------ */
/* Pairwise k-mer distance (the reference's step 2).
 * For every pair of records i < j:
 *     d(i,j) = 1 - (float)S_ij / (float)(min(len_i, len_j) - k + 1)
 *     S_ij   = sum over the 4^k codes of min(sum[i + ld*code], sum[j + ld*code])
 *     len_s  = indices[s+1] - indices[s] - 1
 * written to out[n*i - i*(i-1)/2 + (j-i) - (i+1)], the packed upper triangle of
 * getIdxTriangularMatrixRowMajor(i+1, j-i, n) (kernels.h:46-48), n(n-1)/2 floats.
 * S_ij is summed exactly in 64-bit integers, so the result is that of the CPU
 * path (sequentialKmerCount2, main.cu:604-619) bit for bit; it replaces the host
 * loop of num_seqs minKmeres2 launches (main.cu:326-335) with one launch.
 *   sum       device int32 count matrix of kmc_count_dense (row stride sum_ld,
 *             0 -> num_seqs); counts are taken as unsigned
 *   indices   device int64[num_seqs + 1]
 *   out       device float[num_seqs*(num_seqs-1)/2]
 *   workspace device scratch of kmc_pair_distances_workspace_size() bytes (0 when
 *             the pair matrix alone fills the GPU), or NULL for a library buffer
 * Exact while every record has fewer than 2^32 windows. */
KMC_API size_t kmc_pair_distances_workspace_size(uint64_t num_seqs, int k, int device);
KMC_API int kmc_pair_distances(const int32_t *sum, uint64_t sum_ld, const int64_t *indices, uint64_t num_seqs, int k,
                       float *out, void *workspace, size_t workspace_bytes, hipStream_t stream);

/* Exact drop-in for one reference launch
 *     minKmeres2<<<blocks, threads>>>(sums, mins, num_seqs, current_seq, indexes)
 * (kernels.h:85-109, launched per row at main.cu:327): the distances of record
 * current_seq to every later record, 4^KMC_DROPIN_K codes, summed in float in
 * code order as kernels.h:103 does (so bit-identical to the reference kernel
 * also when that float sum rounds).  Device int sums/indexes, float mins. */
KMC_API int minKmeres2_hip(int *sums, float *mins, int num_seqs, int current_seq, int *indexes, hipStream_t stream);

/* ------------------------------------------------------------------------ */
/* Canonical k-mer counting, k <= 31 (BASELINE config C4).  No
 * reference counterpart (the reference's dense tables stop being feasible past
 * k ~ 13); window and record rules are the dense path's (windows i < len_s - k + 1
 * of each record, bytes other than A/C/G/T invalid).  Key of a valid window: its
 * 2-bit encoding A0 C1 G2 T3 with the FIRST base MOST significant (so key order is
 * lexicographic order), replaced by the key of its reverse complement when that is
 * smaller.  Flags:
 *   KMC_CANON_SOFTMASK  lowercase a/c/g/t count as their bases (soft-masked genomes)
 *   KMC_CANON_FORWARD   no reverse-complement folding (key = the window itself;
 *                       for k <= 13 these counts equal the dense histogram)
 * Output, per record s: the distinct keys of s and their counts in
 * keys/counts[rec_offsets[s] .. rec_offsets[s+1]) (order within a record
 * unspecified), rec_offsets device uint64[num_seqs + 1]; *num_distinct (host) =
 * rec_offsets[num_seqs].  If capacity < *num_distinct nothing is written except
 * rec_offsets and KMC_ERR_CAPACITY is returned (valid windows, <= data bytes,
 * always suffice).  data (any alignment, like the dense entry points) with
 * data[p] = byte p of the global offsets in `indices` (device int64[num_seqs + 1]).
 * Synchronous on `stream` (the distinct total is returned to the host).  The
 * workspace, about 20 bytes per window (no hash table lives in HBM), is
 * library-owned here (one per device, grown on demand, shared by the calls on that
 * device, which must not overlap); kmc_count_canonical_hash_ex takes the caller's
 * instead, of kmc_count_canonical_workspace_size() bytes (NULL: library-owned),
 * 256-byte aligned (KMC_ERR_ALIGNMENT otherwise; hipMalloc's pointers are).  The
 * size is that of a call on `device` (it depends on the device's CU count). */
#define KMC_CANON_MAX_K 31
#define KMC_CANON_SOFTMASK 1u
#define KMC_CANON_FORWARD 2u
KMC_API int kmc_count_canonical_hash(const char *data, const int64_t *indices, uint64_t num_seqs, int k, unsigned flags,
                             uint64_t *keys, uint32_t *counts, uint64_t capacity, uint64_t *rec_offsets,
                             uint64_t *num_distinct, hipStream_t stream);
/* Workspace bytes of a canonical call over records with these offsets (HOST
 * int64[num_seqs + 1], the same values as the call's device `indices`), on
 * `device`, valid for any alignment of `data`; 0 on bad arguments. */
KMC_API size_t kmc_count_canonical_workspace_size(const int64_t *host_indices, uint64_t num_seqs, int k, int device);
/* kmc_count_canonical_hash with a caller workspace (KMC_ERR_WORKSPACE when smaller
 * than the size above; NULL = the library-owned one).  Calls with their own
 * workspaces may run concurrently on different streams. */
KMC_API int kmc_count_canonical_hash_ex(const char *data, const int64_t *indices, uint64_t num_seqs, int k,
                                        unsigned flags, uint64_t *keys, uint32_t *counts, uint64_t capacity,
                                        uint64_t *rec_offsets, uint64_t *num_distinct, void *workspace,
                                        size_t workspace_bytes, hipStream_t stream);

/* ------------------------------------------------------------------------ */
/* Tracing (the reference times step 1 with cudaEvents, main.cu:262-300): when set,
 * every following dense count call on this host thread records `before` right
 * before its histogram kernel and `after` right after it, on the call's stream,
 * so the caller can time the hot kernel alone.  NULL, NULL switches it off. */
#ifndef KMC_HIP_EVENT_T_DEFINED
#define KMC_HIP_EVENT_T_DEFINED
typedef struct ihipEvent_t *hipEvent_t; /* identical to HIP's own typedef */
#endif
KMC_API int kmc_trace_set_events(hipEvent_t before, hipEvent_t after);

/* ------------------------------------------------------------------------ */
/* Launch shaping for overlapped collectives (no reference counterpart): the k <= 8
 * dense kernel runs one 1024-thread workgroup per CU over static byte ranges, so a
 * CU that another kernel holds when a count starts (an RCCL all-reduce overlapping
 * the next step, bench.py at N > 1) delays the whole launch.  With n > 0 the
 * following dense calls issued from this host thread (like kmc_trace_set_events,
 * the setting is per thread: other threads' calls are unaffected) launch n
 * workgroups fewer, leaving n CUs to the concurrent kernel (0 <= n <= 64; 0 =
 * every CU, the default).  The workspace size depends on it: query
 * kmc_count_dense_ex_workspace_size after setting it, on the same thread. */
KMC_API int kmc_set_reserved_cus(int n);

/* ------------------------------------------------------------------------ */
/* Synthetic input generator (benchmark layout): num_records
 * records of record_len bases, each followed by one '\0'; base g (global index
 * first_base + r*record_len + i) is "ACGT"[(x_{g/32} >> 2*(g%32)) & 3] where x_n
 * is output n of splitmix64 seeded with `seed`.  Writes num_records*(record_len+1)
 * bytes.  kmc_synth_indices fills the matching int64 offsets on the host. */
KMC_API int kmc_synth_fill(char *data, uint64_t num_records, uint64_t record_len, uint64_t seed,
                   uint64_t first_base, hipStream_t stream);
KMC_API void kmc_synth_indices(int64_t *indices, uint64_t num_records, uint64_t record_len);
/* Bytes [lo, hi) of the same record stream with first_base = 0 (record r occupies
 * global bytes [r*(record_len+1), (r+1)*(record_len+1)), its last one '\0'),
 * written to data[0 .. hi-lo): what a rank of a strong-scaled job holds of the
 * one global buffer (its shard and halo) without generating whole records.
 * data 16-byte aligned; lo need not be. */
KMC_API int kmc_synth_fill_range(char *data, uint64_t lo, uint64_t hi, uint64_t record_len, uint64_t seed,
                         hipStream_t stream);

/* ------------------------------------------------------------------------ */
/* FASTA loader (host), the successor of importSeqs / importSeqsNoNL
 * (main.cu:474-545 / 401-473) with identical record semantics, int64 offsets
 * and a streaming parser.
 *   dialect 0 = importSeqs: records end at a blank or '\r'-initial line (a '>'
 *               inside a record is sequence text);
 *   dialect 1 = importSeqsNoNL: records also end at a '>' header line.
 *   max_seqs  = the reference's MAX_SEQS cap (KMC_MAX_SEQS_REFERENCE keeps its
 *               behaviour, including the 101st record); <= 0 means unlimited.
 * The loaded buffer follows the reference convention ('|' bytes become '\0';
 * each record ends with '\0') and always carries num_seqs + 1 offsets. */
typedef struct kmc_fasta kmc_fasta;

KMC_API int kmc_fasta_load(const char *path, int dialect, int64_t max_seqs, kmc_fasta **out);
KMC_API uint64_t kmc_fasta_num_seqs(const kmc_fasta *f);
KMC_API const int64_t *kmc_fasta_indices(const kmc_fasta *f); /* num_seqs + 1 entries */
KMC_API const char *kmc_fasta_data(const kmc_fasta *f);
KMC_API uint64_t kmc_fasta_data_bytes(const kmc_fasta *f);
/* Number of entries the reference's indexes_aux would hold: num_seqs + 1, or
 * num_seqs when the input ends in a blank line (the reference then drops the end
 * sentinel and its kernel reads out of bounds). */
KMC_API uint64_t kmc_fasta_reference_num_indexes(const kmc_fasta *f);
KMC_API void kmc_fasta_free(kmc_fasta *f);

/* FASTA parsing on the GPU: the record rules of
 * kmc_fasta_load (importSeqs / importSeqsNoNL, main.cu:474-545 / 401-473) without
 * the MAX_SEQS cap, applied to raw FASTA bytes already in device memory, at HBM
 * speed instead of the reference's host getline loop.
 *   raw       device, 16-byte aligned, raw_bytes bytes of FASTA text
 *   data      device, 4-byte aligned, capacity data_cap >= raw_bytes + 1
 *   indices   device int64[indices_cap]; num_seqs + 1 entries are written
 * On return *num_seqs and *data_bytes describe the buffer exactly as
 * kmc_fasta_load would; KMC_ERR_CAPACITY (with *num_seqs set) when indices_cap <
 * *num_seqs + 1.  Synchronous on `stream`; library-owned scratch (~2 B per line). */
KMC_API int kmc_fasta_parse_device(const char *raw, uint64_t raw_bytes, int dialect, char *data, uint64_t data_cap,
                           int64_t *indices, uint64_t indices_cap, uint64_t *num_seqs, uint64_t *data_bytes,
                           hipStream_t stream);

/* File -> device record buffer: reads `path` through pinned staging buffers
 * into device memory (the read of one chunk overlapping the copy of the last) and
 * parses it there (kmc_fasta_parse_device).  With max_seqs > 0 and more records
 * than that, the reference's cap applies, which cuts mid-record; the file is then
 * loaded by kmc_fasta_load and copied instead.  *data (*data_bytes + 16 bytes) and
 * *indices (*num_seqs + 1 entries) are hipMalloc'ed; the caller hipFree's them.
 * Synchronous on `stream`. */
KMC_API int kmc_fasta_load_device(const char *path, int dialect, int64_t max_seqs, char **data, uint64_t *data_bytes,
                          int64_t **indices, uint64_t *num_seqs, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* KMC_H */
