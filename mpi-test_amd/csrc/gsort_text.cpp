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
