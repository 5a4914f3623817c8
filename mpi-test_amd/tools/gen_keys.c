/* gen_keys -- write the canonical input stream as text.
 *   gen_keys <uniform|zipf> <n> <seed> <out.txt> [start]
 * splitmix64, key i uses state = seed + (start+i+1) * 0x9E3779B97F4A7C15; one key per line,
 * '\n'-separated, no trailing newline (the reference's !feof reader would otherwise append a
 * phantom element).  Same stream as the device generator (K10). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

int main(int argc, char **argv)
{
    if (argc != 5 && argc != 6) {
        fprintf(stderr, "usage: %s <uniform|zipf> <n> <seed> <out.txt> [start]\n", argv[0]);
        return 2;
    }
    const int zipf = strcmp(argv[1], "zipf") == 0;
    if (!zipf && strcmp(argv[1], "uniform") != 0) { fprintf(stderr, "bad dist\n"); return 2; }
    const uint64_t n = strtoull(argv[2], NULL, 0), seed = strtoull(argv[3], NULL, 0);
    const uint64_t start = argc == 6 ? strtoull(argv[5], NULL, 0) : 0;
    FILE *fp = fopen(argv[4], "wb");
    if (!fp) { perror(argv[4]); return 1; }
    static char buf[1 << 22];
    size_t used = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t z = mix64(seed + (start + i + 1) * 0x9E3779B97F4A7C15ULL);
        int32_t key;
        if (!zipf) {
            key = (int32_t)(z >> 33);
        } else {
            double u = (double)((z >> 11) + 1) * 0x1p-53;
            double k = floor(1.0 / (u * u));
            key = (int32_t)(k > 2147483647.0 ? 2147483647.0 : k);
        }
        char tmp[16];
        int len = 0;
        uint32_t v = (uint32_t)key; /* keys are >= 0 for both distributions */
        do { tmp[len++] = (char)('0' + v % 10); v /= 10; } while (v);
        if (used + 16 > sizeof buf) { fwrite(buf, 1, used, fp); used = 0; }
        while (len) buf[used++] = tmp[--len];
        if (i + 1 < n) buf[used++] = '\n';
    }
    fwrite(buf, 1, used, fp);
    return fclose(fp) ? 1 : 0;
}
