/* sanitize_main.c -- TEST INFRASTRUCTURE: runs the oracle's checked build under
 * AddressSanitizer + UndefinedBehaviorSanitizer (built by tests/test_oracle_sanitized.py
 * with -fsanitize=address,undefined -fno-sanitize-recover=all). Decodes every file named
 * on the command line and prints "<error name> <n_samples> <fnv1a64 of the sample bytes>"
 * per file, so the run can be compared with the unsanitized oracle. */
#include <stdio.h>
#include <stdlib.h>

#include "zflac_oracle.h"

static unsigned long long fnv1a(const unsigned char *p, size_t n) {
    unsigned long long h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

int main(int argc, char **argv) {
    for (int i = 1; i < argc; i++) {
        FILE *f = fopen(argv[i], "rb");
        if (!f) { perror(argv[i]); return 2; }
        fseek(f, 0, SEEK_END);
        long n = ftell(f);
        fseek(f, 0, SEEK_SET);
        unsigned char *buf = (unsigned char *)malloc(n > 0 ? (size_t)n : 1);
        if (n > 0 && fread(buf, 1, (size_t)n, f) != (size_t)n) { fclose(f); return 2; }
        fclose(f);
        zfo_result r;
        zfo_decode(buf, (size_t)n, &r);
        const size_t esz = r.sample_kind == ZFO_S8 ? 1 : (r.sample_kind == ZFO_S16 ? 2 : 4);
        printf("%s %llu %016llx\n", zfo_error_name(r.err), (unsigned long long)r.n_samples,
               r.samples ? fnv1a((const unsigned char *)r.samples, r.n_samples * esz) : 0ull);
        zfo_free(&r);
        free(buf);
    }
    return 0;
}
