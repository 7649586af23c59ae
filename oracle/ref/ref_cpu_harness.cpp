// ref_cpu_harness.cpp — TEST INFRASTRUCTURE ONLY.
//
// Builds oracle/_ref/libref_cpu.so from the reference's OWN host-path source,
// where it lies under /root/reference (recipe: oracle/Makefile).  Nothing of the
// reference is committed: the Makefile extracts the needed line ranges of
// main.cu verbatim into oracle/_ref/*.inc (git-ignored) and this file #includes
// them; utils.h is included as-is.
//
//   frag_globals.inc      main.cu:30 (MAX_SEQS), 33-35, 65-67, 113   globals the functions use
//   frag_count.inc        main.cu:636-646   permutationsCountAll       (the CPU hot loop)
//   frag_import.inc       main.cu:474-530   importSeqs, up to the point where it
//                                           allocates CUDA managed memory
//   frag_import_nonl.inc  main.cu:401-458   importSeqsNoNL, same cut
//   frag_dist.inc         main.cu:63, 118, 587-621, 671-673
//                                           sequentialKmerCount2 (CPU pairwise
//                                           distance) + its index helper/global
//
// The two import fragments stop right before `cudaError_t error;` (main.cu:531 /
// main.cu:459): the rest of each function only copies globalAcc into a
// cudaMallocManaged buffer with '|' -> '\0', which ref_get_data() below performs
// on plain host memory.  No CUDA header or API is emulated.
#include <cstring>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "utils.h"              // /root/reference/utils.h: permutation() (bin order)
#include "frag_globals.inc"     // reference globals (seqs, indexes_aux, permutationsMap, ...)
#include "frag_count.inc"       // permutationsCountAll
#include "frag_import.inc"      // importSeqs (body through main.cu:530)
}                               // closes importSeqs (see header comment)
#include "frag_import_nonl.inc" // importSeqsNoNL (body through main.cu:458)
}                               // closes importSeqsNoNL
#include "frag_dist.inc"        // sequentialKmerCount2, distancesSequential

static int g_map_k = -1;

extern "C" {

// Parse a FASTA file with the reference loader.  nonl=0 -> importSeqs (the one
// main() uses, main.cu:163), nonl=1 -> importSeqsNoNL.  Returns the number of
// records, or -1 when the file cannot be opened (the reference would exit()).
int ref_import(const char *path, int nonl) {
    {
        std::ifstream probe(path);
        if (!probe.good()) return -1;
    }
    ids.clear();
    seqs.clear();
    indexes_aux.clear();
    numberOfSequenses = 0;
    size_all_seqs = 0;
    if (nonl)
        importSeqsNoNL(path);
    else
        importSeqs(path);
    return numberOfSequenses;
}

long ref_num_indexes() { return (long)indexes_aux.size(); }

void ref_get_indexes(long long *out) {
    for (size_t i = 0; i < indexes_aux.size(); ++i) out[i] = indexes_aux[i];
}

long ref_data_size() { return (long)size_all_seqs; }

// The device buffer the reference builds from globalAcc (main.cu:537-543):
// concatenation of the records, every '|' replaced by '\0'.
void ref_get_data(char *out) {
    size_t p = 0;
    for (const std::string &s : seqs)
        for (char c : s) out[p++] = (c == '|') ? '\0' : c;
}

long ref_record_size(int s) { return (long)seqs[s].size(); }

// Build permutationsMap for k exactly as main() does (main.cu:124-135), with
// zero-filled pattern buffers (main() uses malloc and relies on fresh pages being
// zero: SURVEY.md §0.1 "Hazard").
int ref_build_map(int k) {
    if (k == g_map_k) return 0;
    permutationsMap.clear();
    const long n = 1L << (2 * k);
    char **perms = (char **)malloc(n * sizeof(char *));
    for (long i = 0; i < n; ++i) perms[i] = (char *)calloc(k + 1, 1);
    permutation("ACGT", k, perms);
    for (long i = 0; i < n; ++i) permutationsMap[perms[i]] = (int)(i + 1);
    for (long i = 0; i < n; ++i) free(perms[i]);
    free(perms);
    g_map_k = k;
    return 0;
}

// The bin-order table itself: pattern i as produced by permutation().
void ref_patterns(int k, char *out /* 4^k * k bytes */) {
    const long n = 1L << (2 * k);
    char **perms = (char **)malloc(n * sizeof(char *));
    for (long i = 0; i < n; ++i) perms[i] = (char *)calloc(k + 1, 1);
    permutation("ACGT", k, perms);
    for (long i = 0; i < n; ++i) memcpy(out + i * k, perms[i], k);
    for (long i = 0; i < n; ++i) free(perms[i]);
    free(perms);
}

// permutationsCountAll on imported record s (seqs[s] keeps its trailing '|').
void ref_count_record(int s, int k, int *out) {
    ref_build_map(k);
    permutationsCountAll(seqs[s], out, 1 << (2 * k), k);
}

// permutationsCountAll on an arbitrary byte range of entry length E (record bytes
// plus one terminator byte), as the CPU baseline timer uses it.  The map must have
// been built for k beforehand (ref_build_map) so the call is thread-safe on
// ACGT-only input (std::map::operator[] only reads when the key exists).
void ref_count_bytes(const char *bytes, long E, int k, int *out) {
    std::string seq(bytes, (size_t)E);
    if (E > 0) seq[E - 1] = '|';
    permutationsCountAll(seq, out, 1 << (2 * k), k);
}

// sequentialKmerCount2 (main.cu:587-621) over the imported records: the packed
// upper triangle of distances, n(n-1)/2 floats, into `out`.
void ref_seq_distances(int k, float *out) {
    ref_build_map(k);
    distancesSequential = out;
    std::vector<std::string> unused;
    sequentialKmerCount2(seqs, unused, k);
    distancesSequential = nullptr;
}

}  // extern "C"
