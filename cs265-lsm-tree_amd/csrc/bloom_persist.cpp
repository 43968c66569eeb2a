// bloom_persist.cpp — SURVEY §8f row 2: a filter persisted beside its run,
// and a filter rebuilt from the run file itself.
//
// The reference keeps a run's entries in a temporary file that Run maps with
// mmap (src/run.cpp:34-72: map_read / map_write; Run::file_size() =
// max_size * sizeof(entry_t), src/run.h:19) and keeps the filter only in
// memory (src/run.h:11): a restarted tree would have to re-set() every key.
// Here a filter can be saved to and loaded from a small file, and rebuilt from
// the run file's AoS entries (entry_t {key, val}, 8 B stride, src/types.h:14-22)
// through the same build path as bloomhip_set_batch_run.  Host code only: it
// drives the C ABI of bloomhip.h.
//
// File layout (little-endian), version 1:
//   0  char[8]   "BLOOMHP1"
//   8  uint32    version (1)
//  12  uint32    flags: bit 0 = run metadata present
//  16  uint64    m
//  24  uint64    nwords (= ceil(m / 64))
//  32  uint32    nfences
//  36  int32     max_key
//  40  uint64[nwords]   bitmap blocks, boost::dynamic_bitset layout
//      int32[nfences]   fence pointers (ascending)
//      uint64    FNV-1a 64 of every preceding byte
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bloomhip.h"

namespace {

constexpr char kMagic[8] = {'B', 'L', 'O', 'O', 'M', 'H', 'P', '1'};
constexpr uint32_t kVersion = 1;
constexpr uint32_t kFlagMeta = 1;

struct Header {
    char magic[8];
    uint32_t version;
    uint32_t flags;
    uint64_t m;
    uint64_t nwords;
    uint32_t nfences;
    int32_t max_key;
};
static_assert(sizeof(Header) == 40, "packed header");

struct Fnv {
    uint64_t h = 1469598103934665603ull;
    void add(const void *p, size_t n) {
        const unsigned char *b = static_cast<const unsigned char *>(p);
        for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    }
};

bool write_all(FILE *fp, const void *p, size_t n, Fnv *fnv) {
    if (fnv) fnv->add(p, n);
    return n == 0 || fwrite(p, 1, n, fp) == n;
}

bool read_all(FILE *fp, void *p, size_t n, Fnv *fnv) {
    if (n && fread(p, 1, n, fp) != n) return false;
    if (fnv) fnv->add(p, n);
    return true;
}

}  // namespace

extern "C" int bloomhip_save(const bloomhip_filter *f, const char *path) {
    if (!f || !path) return BLOOMHIP_EINVAL;
    Header h{};
    memcpy(h.magic, kMagic, 8);
    h.version = kVersion;
    int rc = bloomhip_size(f, &h.m);
    if (rc) return rc;
    rc = bloomhip_nwords(f, &h.nwords);
    if (rc) return rc;
    size_t nf = 0;
    int32_t mk = INT32_MIN;
    rc = bloomhip_get_run_meta(f, nullptr, 0, &nf, &mk);
    if (rc) return rc;
    std::vector<int32_t> fences(nf);
    if (nf) {
        rc = bloomhip_get_run_meta(f, fences.data(), nf, &nf, &mk);
        if (rc) return rc;
    }
    // metadata is present once set_batch_run / set_run_meta ran (even for an
    // empty run); get_run_meta reports INT32_MIN and 0 fences otherwise
    h.flags = (nf || mk != INT32_MIN) ? kFlagMeta : 0;
    h.nfences = (uint32_t)nf;
    h.max_key = mk;
    std::vector<uint64_t> words(h.nwords);
    rc = bloomhip_download(f, words.data(), words.size(), nullptr);
    if (rc) return rc;
    const std::string tmp = std::string(path) + ".tmp";
    FILE *fp = fopen(tmp.c_str(), "wb");
    if (!fp) return BLOOMHIP_EIO;
    Fnv fnv;
    bool ok = write_all(fp, &h, sizeof h, &fnv) &&
              write_all(fp, words.data(), words.size() * 8, &fnv) &&
              write_all(fp, fences.data(), fences.size() * 4, &fnv) &&
              write_all(fp, &fnv.h, 8, nullptr);
    ok = (fclose(fp) == 0) && ok;
    if (!ok || rename(tmp.c_str(), path) != 0) {  // readers never see a partial file
        remove(tmp.c_str());
        return BLOOMHIP_EIO;
    }
    return BLOOMHIP_OK;
}

extern "C" int bloomhip_load(const char *path, int device, bloomhip_filter **out) {
    if (!path || !out) return BLOOMHIP_EINVAL;
    *out = nullptr;
    FILE *fp = fopen(path, "rb");
    if (!fp) return BLOOMHIP_EIO;
    Header h{};
    Fnv fnv;
    std::vector<uint64_t> words;
    std::vector<int32_t> fences;
    uint64_t sum = 0;
    struct stat st {};
    // The header is checked against the file's actual size before anything
    // is sized from it: a damaged or foreign header cannot ask for a huge
    // allocation.  m is bounded as bloomhip_create bounds it.
    bool ok = fstat(fileno(fp), &st) == 0 && read_all(fp, &h, sizeof h, &fnv) &&
              memcmp(h.magic, kMagic, 8) == 0 && h.version == kVersion && h.m > 0 &&
              h.m <= (1ull << 46) && h.nwords == (h.m + 63) / 64 &&
              (uint64_t)st.st_size == sizeof(Header) + 8 * h.nwords + 4 * (uint64_t)h.nfences + 8;
    if (ok) {
        try {
            words.resize(h.nwords);
            fences.resize(h.nfences);
        } catch (...) {  // nothing throws across the C ABI
            fclose(fp);
            return BLOOMHIP_ENOMEM;
        }
        ok = read_all(fp, words.data(), words.size() * 8, &fnv) &&
             read_all(fp, fences.data(), fences.size() * 4, &fnv) &&
             read_all(fp, &sum, 8, nullptr) && sum == fnv.h && fgetc(fp) == EOF;
    }
    fclose(fp);
    if (!ok) return BLOOMHIP_EINVAL;  // not a filter file, or damaged
    bloomhip_filter *f = nullptr;
    int rc = bloomhip_create(device, h.m, &f);
    if (rc) return rc;
    rc = bloomhip_upload(f, words.data(), words.size(), nullptr);
    if (!rc && (h.flags & kFlagMeta))
        rc = bloomhip_set_run_meta(f, fences.data(), fences.size(), h.max_key);
    if (rc) {
        bloomhip_destroy(f);
        return rc;
    }
    *out = f;
    return BLOOMHIP_OK;
}

extern "C" int bloomhip_build_from_run_file(const char *path, uint64_t n_entries,
                                            int64_t max_size, float bits_per_entry, int device,
                                            bloomhip_filter **out) {
    if (!path || !out) return BLOOMHIP_EINVAL;
    *out = nullptr;
    uint64_t m = 0;
    int rc = bloomhip_m_bits(max_size, bits_per_entry, &m);
    if (rc) return rc;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return BLOOMHIP_EIO;
    struct stat st {};
    const size_t bytes = (size_t)n_entries * 8;  // entry_t {KEY_t key; VAL_t val;}
    if (fstat(fd, &st) != 0 || (uint64_t)st.st_size < bytes) {
        close(fd);
        return BLOOMHIP_EINVAL;
    }
    void *map = nullptr;
    if (bytes) {
        map = mmap(nullptr, bytes, PROT_READ, MAP_PRIVATE, fd, 0);
        if (map == MAP_FAILED) {
            close(fd);
            return BLOOMHIP_EIO;
        }
    }
    bloomhip_filter *f = nullptr;
    rc = bloomhip_create(device, m, &f);
    if (!rc) rc = bloomhip_set_batch_run(f, map, (size_t)n_entries, 8, 0, nullptr);
    if (map) munmap(map, bytes);
    close(fd);
    if (rc) {
        if (f) bloomhip_destroy(f);
        return rc;
    }
    *out = f;
    return BLOOMHIP_OK;
}
