// kmc_fasta.cpp — FASTA loader, successor of importSeqs / importSeqsNoNL
// (reference main.cu:474-545 / 401-473).
//
// Same record semantics as the reference, line for line:
//   * lines are the getline() split on '\n' ('\r' stays in the line; a final
//     line without '\n' counts when non-empty);
//   * outside a record, empty lines are skipped and a '>' line starts a record
//     (the header itself is not stored: main.cu:494-499);
//   * the first non-empty, non-header line after a header opens the record; the
//     following lines are appended until a line that is empty or starts with '\r'
//     (dialect 0, main.cu:504), or also starts with '>' (dialect 1, main.cu:431-432);
//   * the cap check `seqs.size() >= MAX_SEQS` runs after each appended line
//     (main.cu:514) and after a record that ended at end of input (main.cu:524):
//     with 100 this keeps 101 multi-line records, all single-line ones;
//   * '|' bytes become '\0' and every record ends with one '\0' (main.cu:537-543).
// What differs on purpose: offsets are int64 (the reference's int overflows past
// 2^31 bytes, main.cu:475), the offset array always ends with the buffer size
// (the reference drops that sentinel after a trailing blank line and then reads
// out of bounds: kmc_fasta_reference_num_indexes reports the reference's count),
// and the file is parsed from one mmap without per-line std::string copies.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "kmc.h"

struct kmc_fasta {
    std::vector<char> data;
    std::vector<int64_t> indices;
    uint64_t ref_num_indexes = 0;
};

namespace {

struct LineReader {
    const char *p;
    const char *end;
    // getline() semantics: returns false at end of input; a trailing segment
    // without '\n' is a line only if it is non-empty.
    bool next(const char *&b, size_t &len) {
        if (p >= end) return false;
        const char *nl = static_cast<const char *>(memchr(p, '\n', (size_t)(end - p)));
        b = p;
        if (nl) {
            len = (size_t)(nl - p);
            p = nl + 1;
        } else {
            len = (size_t)(end - p);
            p = end;
        }
        return true;
    }
};

inline void append_line(std::vector<char> &out, const char *b, size_t len) {
    const size_t o = out.size();
    out.resize(o + len);
    char *dst = out.data() + o;
    memcpy(dst, b, len);
    // '|' -> '\0' (the reference converts its whole buffer, main.cu:538-540)
    char *q = dst;
    size_t rem = len;
    while (rem) {
        char *bar = static_cast<char *>(memchr(q, '|', rem));
        if (!bar) break;
        *bar = '\0';
        rem -= (size_t)(bar + 1 - q);
        q = bar + 1;
    }
}

void parse(const char *buf, size_t size, int dialect, int64_t max_seqs, kmc_fasta &f) {
    LineReader rd{buf, buf + size};
    const uint64_t cap = max_seqs > 0 ? (uint64_t)max_seqs : UINT64_MAX;
    uint64_t nrec = 0;
    uint64_t ref_idx = 0;
    bool new_seq = false;
    const char *b;
    size_t len;
    auto close_record = [&]() {
        f.data.push_back('\0');
        ++nrec;
    };
    while (rd.next(b, len)) {
        if (len == 0) continue;
        if (b[0] == '>') {
            new_seq = true;
            continue;
        }
        if (!new_seq) continue;
        new_seq = false;
        f.indices.push_back((int64_t)f.data.size());
        append_line(f.data, b, len);
        bool ended = false;
        while (rd.next(b, len)) {
            const bool hdr = dialect == 1 && len > 0 && b[0] == '>';
            if (hdr) new_seq = true;
            if (len == 0 || b[0] == '\r' || hdr) {
                close_record();
                ++ref_idx;
                ended = true;
                break;
            }
            append_line(f.data, b, len);
            if (nrec >= cap) break;
        }
        if (!ended) {
            close_record();
            ref_idx += 2;  // start offset and end sentinel (main.cu:519, 523)
            if (nrec >= cap) break;
        }
    }
    f.indices.push_back((int64_t)f.data.size());
    f.ref_num_indexes = ref_idx;
}

}  // namespace

extern "C" int kmc_fasta_load(const char *path, int dialect, int64_t max_seqs, kmc_fasta **out) {
    if (!path || !out || (dialect != 0 && dialect != 1)) return KMC_ERR_INVALID_ARG;
    *out = nullptr;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return KMC_ERR_IO;
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        return KMC_ERR_IO;
    }
    const size_t size = (size_t)st.st_size;
    const char *buf = nullptr;
    void *map = nullptr;
    if (size > 0) {
        map = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (map == MAP_FAILED) {
            close(fd);
            return KMC_ERR_IO;
        }
        madvise(map, size, MADV_SEQUENTIAL);
        buf = static_cast<const char *>(map);
    }
    kmc_fasta *f = new (std::nothrow) kmc_fasta;
    int rc = KMC_OK;
    if (!f) {
        rc = KMC_ERR_NOMEM;
    } else {
        try {
            f->data.reserve(size + 16);
            parse(buf, size, dialect, max_seqs, *f);
        } catch (const std::bad_alloc &) {
            delete f;
            f = nullptr;
            rc = KMC_ERR_NOMEM;
        }
    }
    if (map) munmap(map, size);
    close(fd);
    *out = f;
    return rc;
}

extern "C" uint64_t kmc_fasta_num_seqs(const kmc_fasta *f) { return f ? f->indices.size() - 1 : 0; }
extern "C" const int64_t *kmc_fasta_indices(const kmc_fasta *f) { return f ? f->indices.data() : nullptr; }
extern "C" const char *kmc_fasta_data(const kmc_fasta *f) { return f ? f->data.data() : nullptr; }
extern "C" uint64_t kmc_fasta_data_bytes(const kmc_fasta *f) { return f ? f->data.size() : 0; }
extern "C" uint64_t kmc_fasta_reference_num_indexes(const kmc_fasta *f) { return f ? f->ref_num_indexes : 0; }
extern "C" void kmc_fasta_free(kmc_fasta *f) { delete f; }
