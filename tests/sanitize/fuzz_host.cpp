// fuzz_host.cpp -- randomized driver for libgsort's host-only code (gsort_text.cpp,
// gsort_plan.cpp) built with AddressSanitizer + UndefinedBehaviorSanitizer by
// tests/test_host_sanitized.py (sanitizers on the host code; GPU sanitizers are
// not available on the MI355X pool).  Every input-dependent host routine runs on random and
// adversarial inputs; invariants are checked, and any sanitizer report aborts the run.
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all \
//       -I include tests/sanitize/fuzz_host.cpp mpi-test_amd/csrc/gsort_plan.cpp \
//       mpi-test_amd/csrc/gsort_text.cpp -o fuzz_host -lpthread && ./fuzz_host [iters]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "gsort.h"

#define REQUIRE(c)                                                                \
    do {                                                                          \
        if (!(c)) {                                                               \
            fprintf(stderr, "fuzz_host: check failed at line %d: %s\n", __LINE__, #c); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

static std::mt19937_64 rng(12345);
static uint64_t urand(uint64_t n) { return n ? rng() % n : 0; }

static void fuzz_parse(int iters) {
    const char alphabet[] = "0123456789  \n\t-+-x9";
    for (int it = 0; it < iters; ++it) {
        std::string s;
        const size_t len = urand(4000);
        const bool garbage = urand(4) == 0;
        for (size_t i = 0; i < len; ++i) {
            char ch = alphabet[urand(sizeof(alphabet) - 1)];
            if (!garbage && ch == 'x') ch = ' ';
            s.push_back(ch);
        }
        if (urand(3) == 0) s += " 99999999999999999999 -2147483649 4294967296 ";
        const long long n1 = gsort_parse_text(s.data(), s.size(), nullptr, 0, 1);
        const long long n7 = gsort_parse_text(s.data(), s.size(), nullptr, 0, 7);
        REQUIRE(n1 == n7);
        if (n1 < 0) continue;
        std::vector<int32_t> a((size_t)n1 + 1), b((size_t)n1 + 1);
        REQUIRE(gsort_parse_text(s.data(), s.size(), a.data(), (size_t)n1, 1) == n1);
        REQUIRE(gsort_parse_text(s.data(), s.size(), b.data(), (size_t)n1, 5) == n1);
        REQUIRE(memcmp(a.data(), b.data(), (size_t)n1 * 4) == 0);
        if (n1 > 1) {  // a short output buffer is never overrun
            std::vector<int32_t> c((size_t)n1 / 2);
            gsort_parse_text(s.data(), s.size(), c.data(), c.size(), 3);
        }
    }
}

static void fuzz_dump(int iters) {
    for (int it = 0; it < iters; ++it) {
        const size_t n = urand(3000);
        std::vector<int32_t> k(n);
        for (auto &x : k) x = (int32_t)(uint32_t)rng();
        const uint64_t first = urand(1ull << 40);
        const int th = 1 + (int)urand(8);
        const long long need = gsort_format_dump(k.data(), n, first, nullptr, 0, th);
        REQUIRE(need >= 0);
        std::vector<char> buf((size_t)need + 1);
        REQUIRE(gsort_format_dump(k.data(), n, first, buf.data(), (size_t)need, th) == need);
        if (need > 0)
            REQUIRE(gsort_format_dump(k.data(), n, first, buf.data(), (size_t)need - 1, th) < 0);
        // round trip: "index|value\n" lines
        size_t pos = 0;
        for (size_t i = 0; i < n; ++i) {
            char *end = nullptr;
            const unsigned long long idx = strtoull(buf.data() + pos, &end, 10);
            REQUIRE(idx == first + i && *end == '|');
            const unsigned long v = strtoul(end + 1, &end, 10);
            REQUIRE((uint32_t)v == (uint32_t)k[i] && *end == '\n');
            pos = (size_t)(end + 1 - buf.data());
        }
        REQUIRE(pos == (size_t)need);
    }
}

static void fuzz_route(int iters) {
    for (int it = 0; it < iters; ++it) {
        const int P = 1 + (int)urand(9);
        std::vector<uint64_t> hist((size_t)P * 256);
        uint64_t N = 0;
        const int dens = (int)urand(3);
        for (auto &h : hist) {
            h = dens == 0 ? urand(3) : dens == 1 ? (urand(8) == 0 ? urand(5000) : 0) : urand(200);
            N += h;
        }
        const uint64_t B = (N + P - 1) / P;
        std::vector<uint64_t> recv_tot(P, 0);
        for (int me = 0; me < P; ++me) {
            std::vector<uint64_t> send(P), recv(P), seg((size_t)4 * P * 256);
            size_t nseg = 0;
            REQUIRE(gsort_plan_radix_route(P, hist.data(), B ? B : 1, me, send.data(), recv.data(),
                                           seg.data(), &nseg) == GSORT_OK);
            uint64_t s = 0, r = 0, mine = 0;
            for (int d = 0; d < 256; ++d) mine += hist[(size_t)me * 256 + d];
            for (int q = 0; q < P; ++q) { s += send[q]; r += recv[q]; }
            REQUIRE(s == mine);
            const uint64_t lo = (uint64_t)me * B, blk = lo >= N ? 0 : std::min(B, N - lo);
            REQUIRE(r == blk);
            for (size_t i = 0; i < nseg; ++i) REQUIRE(seg[4 * i + 2] + seg[4 * i + 3] <= blk);
        }
    }
}

static void fuzz_split(int iters) {
    for (int it = 0; it < iters; ++it) {
        const int P = 1 + (int)urand(9);
        std::vector<std::vector<int32_t>> blk(P);
        std::vector<uint64_t> n_all(P);
        std::vector<int32_t> all;
        const int range = 1 + (int)urand(50);
        for (int p = 0; p < P; ++p) {
            blk[p].resize(urand(60));
            for (auto &x : blk[p]) x = (int32_t)urand(range) - range / 2;
            std::sort(blk[p].begin(), blk[p].end());
            n_all[p] = blk[p].size();
            all.insert(all.end(), blk[p].begin(), blk[p].end());
        }
        std::sort(all.begin(), all.end());
        const uint64_t N = all.size(), B = (N + P - 1) / P;
        std::vector<uint64_t> lt((size_t)P * std::max(P - 1, 1)), le(lt.size());
        const bool balanced = urand(2) == 1;
        for (int q = 1; q < P; ++q) {
            const uint64_t g = std::min<uint64_t>((uint64_t)q * B, N);
            // the radix cut's v_q = the g-th smallest key; the balanced cut takes any splitter
            const int32_t v = N == 0 ? 0 : balanced ? (int32_t)urand(range) - range / 2
                                                    : all[std::min<uint64_t>(g, N - 1)];
            for (int p = 0; p < P; ++p) {
                lt[(size_t)p * (P - 1) + q - 1] =
                    std::lower_bound(blk[p].begin(), blk[p].end(), v) - blk[p].begin();
                le[(size_t)p * (P - 1) + q - 1] =
                    std::upper_bound(blk[p].begin(), blk[p].end(), v) - blk[p].begin();
            }
        }
        uint64_t got = 0;
        for (int me = 0; me < P; ++me) {
            std::vector<uint64_t> send(P), recv(P);
            const gsort_status st =
                balanced ? gsort_plan_split_balanced(P, n_all.data(), lt.data(), le.data(), me,
                                                     send.data(), recv.data())
                         : gsort_plan_split(P, n_all.data(), lt.data(), le.data(), me,
                                            send.data(), recv.data());
            REQUIRE(st == GSORT_OK || balanced);
            if (st != GSORT_OK) continue;
            uint64_t s = 0;
            for (int q = 0; q < P; ++q) { s += send[q]; got += recv[q]; }
            REQUIRE(s == n_all[me]);
        }
        if (!balanced) REQUIRE(got == N);
    }
}

static void fuzz_plans(int iters) {
    for (int it = 0; it < iters; ++it) {
        const int P = 1 + (int)urand(12);
        std::vector<int32_t> samp((size_t)P * (2 * P - 1)), spl(std::max(P - 1, 1));
        for (auto &x : samp) x = (int32_t)(uint32_t)rng();
        REQUIRE(gsort_plan_splitters(P, samp.data(), spl.data()) == GSORT_OK);
        for (int i = 1; i < P - 1; ++i) REQUIRE(spl[i - 1] <= spl[i]);
        const int32_t mx = urand(4) == 0 ? -1 : (int32_t)(rng() >> 33);
        int loop = 0;
        int32_t mod[64];
        double scale[64];
        const gsort_status st = gsort_plan_ref_digits(P, mx, &loop, mod, scale, 64);
        REQUIRE(st == GSORT_OK);
        REQUIRE(P == 1 ? loop < 1 : (loop >= 1 && loop <= 32));
        int dummy = 0;
        REQUIRE(gsort_plan_ref_digits(P, mx, &dummy, nullptr, nullptr, 0) == GSORT_OK);
    }
    int loop = 0;
    REQUIRE(gsort_plan_ref_digits(2, INT32_MIN, &loop, nullptr, nullptr, 0) == GSORT_EINVAL);
    REQUIRE(gsort_plan_ref_digits(0, 5, &loop, nullptr, nullptr, 0) == GSORT_EINVAL);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 300;
    fuzz_parse(iters);
    fuzz_dump(iters / 3 + 1);
    fuzz_route(iters);
    fuzz_split(iters * 3);
    fuzz_plans(iters);
    printf("fuzz_host ok\n");
    return 0;
}
