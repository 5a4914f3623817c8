// gsort_text.cpp -- the rank-0 text reader of the drop-in CLIs (host code, no GPU).
//
// The reference reads with a `!feof` loop over fscanf(fp, "%d", ...) and a realloc per element
// (mpi_radix_sort.c:85-97, mpi_sample_sort.c:50-60).  gsort_parse_text accepts exactly the
// same token syntax with the same value semantics (glibc converts %d through strtol: the long
// saturates at LONG_MIN/LONG_MAX, then truncates to int), parsing the whole buffer in chunks
// on several threads.  Divergences, both documented in DESIGN.md: a trailing delimiter adds no
// phantom element, and a non-numeric token is an error (the reference spins
// on it until realloc fails, then reports the file as invalid).
#include <limits.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "gsort.h"

namespace {

inline bool is_space(char c) {
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

// Parse [b, e) which starts and ends on token boundaries.  Returns #keys or -1.
long long parse_range(const char *buf, size_t b, size_t e, int32_t *out, size_t cap) {
    size_t n = 0, i = b;
    for (;;) {
        while (i < e && is_space(buf[i])) ++i;
        if (i >= e) break;
        bool neg = false;
        if (buf[i] == '+' || buf[i] == '-') neg = buf[i++] == '-';
        if (i >= e || buf[i] < '0' || buf[i] > '9') return -1;
        unsigned long long mag = 0;
        bool sat = false;
        for (; i < e && buf[i] >= '0' && buf[i] <= '9'; ++i) {
            const unsigned d = (unsigned)(buf[i] - '0');
            if (mag > (ULLONG_MAX - d) / 10) sat = true; else mag = mag * 10 + d;
        }
        long long v;
        if (!neg) v = (sat || mag > (unsigned long long)LLONG_MAX) ? LLONG_MAX : (long long)mag;
        else v = (sat || mag > (unsigned long long)LLONG_MAX + 1ULL) ? LLONG_MIN
                                                                     : (long long)(0ULL - mag);
        if (i < e && !is_space(buf[i])) return -1;  // "12,13": the reference spins forever
        if (out && n < cap) out[n] = (int32_t)(uint32_t)(unsigned long long)v;
        ++n;
    }
    return (long long)n;
}

}  // namespace

extern "C" long long gsort_parse_text(const char *buf, size_t len, int32_t *out, size_t cap,
                                      int threads) {
    if (!buf && len) return -1;
    if (threads < 1) threads = 1;
    if (len < (1u << 20) || threads == 1) return parse_range(buf, 0, len, out, cap);
    // split on whitespace boundaries; count per chunk, prefix, then parse into place
    std::vector<size_t> cut(threads + 1, len);
    cut[0] = 0;
    for (int t = 1; t < threads; ++t) {
        size_t p = std::max(cut[t - 1], len / threads * t);
        while (p < len && !is_space(buf[p])) ++p;
        cut[t] = p;
    }
    std::vector<long long> cnt(threads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] { cnt[t] = parse_range(buf, cut[t], cut[t + 1], nullptr, 0); });
    for (auto &x : th) x.join();
    th.clear();
    std::vector<size_t> off(threads + 1, 0);
    for (int t = 0; t < threads; ++t) {
        if (cnt[t] < 0) return -1;
        off[t + 1] = off[t] + (size_t)cnt[t];
    }
    if (out)
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                if (off[t] < cap)
                    parse_range(buf, cut[t], cut[t + 1], out + off[t], cap - off[t]);
            });
    for (auto &x : th) x.join();
    return (long long)off[threads];
}

// ---- debug dump printer -------------------------------------------------
// The reference's full sorted dump is a serial printf("%u|%u\n", i, int_buf[i]) loop on rank 0
// (mpi_radix_sort.c:198-200, mpi_sample_sort.c:202-204).  gsort_format_dump renders the same
// bytes ("%llu|%u\n": the index, then the key as unsigned) for keys[0 .. n) with indices from
// first_index, on several threads: each chunk's length is known from the digit counts, so the
// chunks are sized, prefix-summed and written in place.
namespace {

inline unsigned ndigits(unsigned long long v) {
    unsigned d = 1;
    while (v >= 10) { v /= 10; ++d; }
    return d;
}

inline char *put_u(char *p, unsigned long long v, unsigned nd) {
    char *e = p + nd;
    do { *--e = (char)('0' + v % 10); v /= 10; } while (v);
    return p + nd;
}

size_t dump_len(const int32_t *keys, size_t a, size_t b, uint64_t first) {
    size_t len = 0;
    for (size_t i = a; i < b; ++i)
        len += ndigits(first + i) + ndigits((uint32_t)keys[i]) + 2;
    return len;
}

void dump_write(const int32_t *keys, size_t a, size_t b, uint64_t first, char *p) {
    for (size_t i = a; i < b; ++i) {
        const unsigned long long idx = first + i;
        const uint32_t v = (uint32_t)keys[i];
        p = put_u(p, idx, ndigits(idx));
        *p++ = '|';
        p = put_u(p, v, ndigits(v));
        *p++ = '\n';
    }
}

}  // namespace

extern "C" long long gsort_format_dump(const int32_t *keys, size_t n, uint64_t first_index,
                                       char *out, size_t cap, int threads) {
    if (n && !keys) return -1;
    if (threads < 1) threads = 1;
    if (n < 65536) threads = 1;
    std::vector<size_t> cut(threads + 1), len(threads), off(threads + 1, 0);
    for (int t = 0; t <= threads; ++t) cut[t] = n / threads * t + std::min<size_t>(t, n % threads);
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t)
        th.emplace_back([&, t] { len[t] = dump_len(keys, cut[t], cut[t + 1], first_index); });
    len[0] = dump_len(keys, cut[0], cut[1], first_index);
    for (auto &x : th) x.join();
    th.clear();
    for (int t = 0; t < threads; ++t) off[t + 1] = off[t] + len[t];
    if (!out) return (long long)off[threads];
    if (cap < off[threads]) return -1;
    for (int t = 1; t < threads; ++t)
        th.emplace_back([&, t] { dump_write(keys, cut[t], cut[t + 1], first_index, out + off[t]); });
    dump_write(keys, cut[0], cut[1], first_index, out);
    for (auto &x : th) x.join();
    return (long long)off[threads];
}

// ---- the drop-in programs' stdout contract ----------------------------------
// Everything the reference programs print to stdout that is part of their contract, for one
// rank, in the reference's order: sample's "Each bucket" line (mpi_sample_sort.c:74), at debug
// its splitters (rank 0, :124) and bucket lengths (every rank, :157), the sorted dump (rank 0;
// radix at debug > 2, radix:198-200; sample at debug >= 1, sample:202-204) and the median
// (rank 0, radix:201, sample:205).  The reference's other debug lines are free-form progress
// output and are not reproduced.  Written with write(2) so a C host and a test harness get the
// same bytes; the dump goes in blocks rendered by gsort_format_dump.
#include <errno.h>
#include <stdio.h>
#include <unistd.h>

namespace {

bool write_all(int fd, const char *p, size_t n) {
    while (n) {
        const ssize_t w = ::write(fd, p, n);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) return false;
        p += w;
        n -= (size_t)w;
    }
    return true;
}

}  // namespace

extern "C" gsort_status gsort_write_report(const gsort_report *r, int fd) {
    if (!r || r->nranks < 1 || r->rank < 0 || r->rank >= r->nranks ||
        (r->algo != GSORT_REPORT_RADIX && r->algo != GSORT_REPORT_SAMPLE))
        return GSORT_EINVAL;
    const bool sample = r->algo == GSORT_REPORT_SAMPLE, root = r->rank == 0;
    const bool lines = sample && r->debug >= 1;
    const bool dump = root && (sample ? r->debug >= 1 : r->debug > 2);
    const bool before = r->stage != 2, after = r->stage != 1;
    if (r->stage < 0 || r->stage > 2 ||
        (after && lines && !r->bucket_counts) ||
        (after && lines && root && r->nranks > 1 && !r->splitters) ||
        (after && root && r->n_total && !r->sorted))
        return GSORT_EINVAL;
    std::string head;
    char ln[96];
    if (sample && root && before) {
        // size_bucket = ceil(N / P) (mpi_sample_sort.c:72), printed as %u there
        const unsigned long long B = (r->n_total + (uint64_t)r->nranks - 1) / (uint64_t)r->nranks;
        snprintf(ln, sizeof ln, "Each bucket will be put %llu items.\n", B);
        head += ln;
    }
    if (lines && after) {
        if (root)
            for (int i = 0; i < r->nranks - 1; ++i) {
                snprintf(ln, sizeof ln, "[MASTER] Splitter: %u.\n", (unsigned)r->splitters[i]);
                head += ln;
            }
        for (int j = 0; j < r->nranks; ++j) {
            snprintf(ln, sizeof ln, "[COMMON] %d: Bucket %d=%llu\n", r->rank, j,
                     (unsigned long long)r->bucket_counts[j]);
            head += ln;
        }
    }
    if (!write_all(fd, head.data(), head.size())) return GSORT_EINVAL;
    if (!root || !after) return GSORT_OK;
    if (dump && r->n_total) {
        constexpr size_t kBlock = 1u << 21, kMaxLine = 32;  // "%llu|%u\n" <= 32 bytes
        std::vector<char> buf(kBlock * kMaxLine);
        for (uint64_t a = 0; a < r->n_total; a += kBlock) {
            const size_t m = (size_t)std::min<uint64_t>(kBlock, r->n_total - a);
            const long long len = gsort_format_dump(r->sorted + a, m, a, buf.data(), buf.size(), 16);
            if (len < 0 || !write_all(fd, buf.data(), (size_t)len)) return GSORT_EINVAL;
        }
    }
    if (r->n_total) {
        // index N/2 - 1 (radix:201); N = 1 would read int_buf[-1] in the reference (quirk Q14)
        const uint64_t med = r->n_total >= 2 ? r->n_total / 2 - 1 : 0;
        snprintf(ln, sizeof ln, "The n/2-th sorted element: %d\n", r->sorted[med]);
        if (!write_all(fd, ln, strlen(ln))) return GSORT_EINVAL;
    }
    return GSORT_OK;
}
