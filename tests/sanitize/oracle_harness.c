/* Host sanitizer harness for the C parity oracle (oracle/amx_oracle.c, test
 * infrastructure), built by tests/test_sanitize.py with gcc -fsanitize=address,undefined
 * and the oracle's own flags.  The oracle is compiled into this program as one
 * translation unit, so its types come with it.
 *
 *   oracle_harness <dir>
 *
 * <dir> holds what the test wrote: x16.bin (int16 [n, 2]), params.txt ("n fs n_chunks"
 * then "start len" per chunk), chunk.bin (the orc_chunk_t bytes Python's ctypes
 * struct holds; its tanh_lut pointer is replaced here) and lut.bin (65536 float32).
 * It runs the oracle's whole pipeline -- every chunk (orc_chunk), the 192 kHz loudness
 * measurement (orc_ebur128_192k), both loudnorm filter runs of the dynamic mode
 * (orc_loudnorm), the alimiter (orc_alimiter) -- and writes the outputs for the test
 * to compare with the normal oracle build's, bit for bit. */
#include "../../oracle/amx_oracle.c"

#include <stdio.h>

static void *slurp(const char *dir, const char *name, size_t *size) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void *p = malloc(n > 0 ? (size_t)n : 1);
    if (n > 0 && fread(p, 1, (size_t)n, f) != (size_t)n) {
        fclose(f);
        free(p);
        return NULL;
    }
    fclose(f);
    *size = (size_t)n;
    return p;
}

static int spill(const char *dir, const char *name, const void *p, size_t size) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    size_t w = fwrite(p, 1, size, f);
    fclose(f);
    return w == size ? 0 : -1;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const char *dir = argv[1];
    size_t sz = 0, csz = 0, lsz = 0;
    int16_t *x = (int16_t *)slurp(dir, "x16.bin", &sz);
    orc_chunk_t *p = (orc_chunk_t *)slurp(dir, "chunk.bin", &csz);
    float *lut = (float *)slurp(dir, "lut.bin", &lsz);
    char path[4096];
    snprintf(path, sizeof path, "%s/params.txt", dir);
    FILE *pf = fopen(path, "r");
    if (!x || !p || !pf || csz != sizeof(orc_chunk_t)) {
        fprintf(stderr, "bad inputs (chunk struct %zu vs %zu bytes)\n", csz, sizeof(orc_chunk_t));
        return 2;
    }
    long long n, nch;
    int fs;
    if (fscanf(pf, "%lld %d %lld", &n, &fs, &nch) != 3) return 2;
    p->tanh_lut = lut;
    /* the chunk chain (:185-204) and the concat (:205-214) */
    int16_t *cat = (int16_t *)malloc(sizeof(int16_t) * 2 * (size_t)(n + 64 * nch + 64));
    int64_t w = 0;
    for (long long c = 0; c < nch; c++) {
        long long s, len;
        if (fscanf(pf, "%lld %lld", &s, &len) != 2) return 2;
        int16_t *o = (int16_t *)malloc(sizeof(int16_t) * 2 * (size_t)(len + 64));
        int64_t m = orc_chunk(p, x + 2 * s, len, o);
        memcpy(cat + 2 * w, o, sizeof(int16_t) * 2 * (size_t)m);
        w += m;
        free(o);
    }
    fclose(pf);
    spill(dir, "cat.out", cat, sizeof(int16_t) * 2 * (size_t)w);
    /* loudnorm pass 1's measurement at 192 kHz (:229) */
    uint64_t hist[1000], st_hist[1000];
    double peak[2], stats[10];
    int64_t nb = 0;
    memset(hist, 0, sizeof hist);
    memset(st_hist, 0, sizeof st_hist);
    if (orc_ebur128_192k(cat, w, fs, 2, hist, st_hist, peak, &nb)) return 3;
    spill(dir, "hist.out", hist, sizeof hist);
    spill(dir, "peak.out", peak, sizeof peak);
    /* the loudnorm filter, pass 1's options and pass 2's (dynamic mode, :240) */
    const int64_t n192 = orc_swr_out_frames(w, fs, 192000);
    int16_t *y192 = (int16_t *)malloc(sizeof(int16_t) * 2 * (size_t)(n192 + 1));
    orc_loudnorm_opts o1 = {-14.0, 11.0, -1.5, 0.0, 0.0, 99.0, -70.0, 0.0};
    int64_t m1 = orc_loudnorm(cat, w, fs, 2, &o1, y192, stats);
    spill(dir, "ln1.out", y192, sizeof(int16_t) * 2 * (size_t)m1);
    spill(dir, "ln1stats.out", stats, sizeof stats);
    double I, lra, thr;
    {
        double s3[3];
        orc_loudness_stats(hist, st_hist, s3);
        I = s3[0];
        lra = s3[1];
        thr = s3[2];
    }
    orc_loudnorm_opts o2 = {-14.0, 11.0, -1.5, I, lra, 20.0 * log10(peak[0] > peak[1] ? peak[0] : peak[1]), thr,
                            stats[9]};
    int64_t m2 = orc_loudnorm(cat, w, fs, 2, &o2, y192, stats);
    spill(dir, "ln2.out", y192, sizeof(int16_t) * 2 * (size_t)m2);
    /* the alimiter (:223) on the 192 kHz stream and on the concatenated track */
    int16_t *lim = (int16_t *)malloc(sizeof(int16_t) * 2 * (size_t)(m2 > w ? m2 : w));
    orc_alimiter(y192, m2, 192000, 2, 1.0, 1.0, 0.98, 5.0, 50.0, 1, lim);
    spill(dir, "lim192.out", lim, sizeof(int16_t) * 2 * (size_t)m2);
    orc_alimiter(cat, w, fs, 2, 1.0, 1.0, 0.98, 5.0, 50.0, 1, lim);
    spill(dir, "lim.out", lim, sizeof(int16_t) * 2 * (size_t)w);
    printf("oracle_harness: %lld frames, %lld chunks -> %lld, 192 kHz %lld / %lld\n", n, nch, (long long)w,
           (long long)m1, (long long)m2);
    free(lim);
    free(y192);
    free(cat);
    free(x);
    free(p);
    free(lut);
    return 0;
}
