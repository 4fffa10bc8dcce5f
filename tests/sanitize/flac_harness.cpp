// Host sanitizer harness for libamx's FLAC decoder (csrc/amx_flac.cpp), built by
// tests/test_sanitize.py with g++ -fsanitize=address,undefined (no GPU, no HIP).
//
// Reads a manifest of cases written by the test: "<file.flac> <expected.i32|-> <threads>"
// per line.  A case with an expected file must decode to exactly those interleaved
// int32 samples; a case with "-" (a corrupted or truncated stream) must either be
// refused with an error code or decode to something -- what it must never do is read or
// write out of bounds, which the sanitizers turn into a non-zero exit.
#include "../../include/amx.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static std::vector<unsigned char> slurp(const char *path) {
    std::vector<unsigned char> v;
    FILE *f = std::fopen(path, "rb");
    if (!f) return v;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    v.resize(n > 0 ? (size_t)n : 0);
    if (n > 0 && std::fread(v.data(), 1, (size_t)n, f) != (size_t)n) v.clear();
    std::fclose(f);
    return v;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s manifest\n", argv[0]);
        return 2;
    }
    FILE *m = std::fopen(argv[1], "r");
    if (!m) return 2;
    char fl[4096], ex[4096];
    int threads, cases = 0, ok = 0, refused = 0, bad = 0;
    while (std::fscanf(m, "%4095s %4095s %d", fl, ex, &threads) == 3) {
        cases++;
        std::vector<unsigned char> data = slurp(fl);
        // the decoder reads the caller's bytes in place: an exact-size heap copy, so a
        // read past the end is a heap overflow ASan reports
        unsigned char *buf = (unsigned char *)std::malloc(data.size() ? data.size() : 1);
        if (!data.empty()) std::memcpy(buf, data.data(), data.size());
        amx_flac_info_t info;
        int rc = amx_flac_info(buf, (int64_t)data.size(), &info);
        if (rc != AMX_OK) {
            refused++;
            if (std::strcmp(ex, "-") != 0) {
                std::printf("FAIL %s: amx_flac_info %d\n", fl, rc);
                bad++;
            }
            std::free(buf);
            continue;
        }
        int64_t n = 0;
        rc = amx_flac_decode(buf, (int64_t)data.size(), nullptr, 0, &n, threads, nullptr, 0, nullptr);
        if (rc != AMX_OK || n < 0 || n > (int64_t)1 << 28) {
            refused++;
            if (std::strcmp(ex, "-") != 0) {
                std::printf("FAIL %s: size query %d\n", fl, rc);
                bad++;
            }
            std::free(buf);
            continue;
        }
        std::vector<int32_t> out((size_t)(n > 0 ? n : 1) * (size_t)info.channels);
        const int64_t max_blocks = n / 16 + 2;
        std::vector<int32_t> blocks((size_t)max_blocks);
        int64_t got = 0, nb = 0;
        rc = amx_flac_decode(buf, (int64_t)data.size(), out.data(), n, &got, threads, blocks.data(), max_blocks,
                             &nb);
        std::free(buf);
        if (std::strcmp(ex, "-") == 0) {
            if (rc == AMX_OK) ok++;
            else refused++;
            continue;
        }
        std::vector<unsigned char> want = slurp(ex);
        if (rc != AMX_OK || got != n || want.size() != (size_t)n * info.channels * 4 ||
            std::memcmp(want.data(), out.data(), want.size()) != 0) {
            std::printf("FAIL %s: rc %d frames %lld\n", fl, rc, (long long)got);
            bad++;
            continue;
        }
        int64_t tot = 0;
        for (int64_t i = 0; i < nb; i++) tot += blocks[(size_t)i];
        if (tot != n) {
            std::printf("FAIL %s: block sizes sum to %lld of %lld\n", fl, (long long)tot, (long long)n);
            bad++;
            continue;
        }
        ok++;
    }
    std::fclose(m);
    std::printf("flac_harness: %d cases, %d decoded, %d refused, %d failed\n", cases, ok, refused, bad);
    return bad ? 1 : 0;
}
