/* AddressSanitizer / UBSan driver of the CPU restatement (oracle/dmt_oracle.c, fp64 and fp32):
 * every exported numeric entry point on seeded random inputs of several sizes, including the
 * ragged edge cases the parity tests use (1-step segments, chunk boundaries 63/64/65, 511/512/513
 * scan steps, skip past the segment end).  Built by `make -C oracle asan` with
 * -fsanitize=address,undefined; run by tests/test_asan.py.  Exit 0 = no sanitizer report. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int orc_solve_segment_f64(int, int, int, const double*, int, const double*, const double*,
                      const double*, const double*, const double*, double*, double*);
int orc_solve_segment_f32(int, int, int, const double*, int, const float*, const float*,
                          const float*, const float*, const float*, float*, float*);
void orc_invsolve_segment_f64(int, int, int, const double*, int, const double*, const double*,
                          const double*, const double*, double*);
int orc_backward_filter_segment(int, const double*, const double*, const double*, int,
                                const double*, const double*, const double*, double, double*,
                                double*, double*);
void orc_normal_block_f64(uint64_t, uint32_t, uint32_t, uint32_t, uint32_t, double*);
void orc_normal_block_f32(uint64_t, uint32_t, uint32_t, uint32_t, uint32_t, float*);
double orc_exp1(uint64_t, uint32_t, uint32_t, uint32_t);
void orc_set_ll_skip(int);
void orc_set_sequential_ou(int);

static uint64_t st = 0x9E3779B97F4A7C15ull;
static double urand(void) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return (double)(st >> 11) * 0x1p-53;
}

int main(void) {
    const int sizes[] = {2, 3, 64, 65, 66, 512, 513, 514, 1301};
    const int models[][3] = {{0, 1, 1}, {0, 2, 2}, {0, 3, 3}, {1, 2, 1}, {2, 3, 3}};  /* OU, FHN, Lorenz */
    for (size_t si = 0; si < sizeof sizes / sizeof *sizes; ++si) {
        const int n = sizes[si];
        for (size_t mi = 0; mi < sizeof models / sizeof *models; ++mi) {
            const int model = models[mi][0], d = models[mi][1], m = models[mi][2];
            const int h = d * (d + 1) / 2;
            double law[64] = {0};
            for (int i = 0; i < 16; ++i) law[i] = 0.2 + 0.1 * urand();
            for (int p = 0; p < d; ++p) law[16 + p * m + (p < m ? p : 0)] = 0.5;
            for (int i = 0; i < h; ++i) law[25 + i] = (i == 0 || i == d || i == h - 1) ? 0.25 : 0.0;
            double *t = malloc(n * 8), *H = malloc((size_t)n * h * 8), *F = malloc((size_t)n * d * 8),
                   *W = malloc((size_t)n * m * 8), *X = malloc((size_t)n * d * 8),
                   *W2 = malloc((size_t)n * m * 8);
            float *tf = malloc(n * 4), *Hf = malloc((size_t)n * h * 4), *Ff = malloc((size_t)n * d * 4),
                  *Wf = malloc((size_t)n * m * 4), *Xf = malloc((size_t)n * d * 4);
            for (int i = 0; i < n; ++i) { t[i] = i / (double)(n - 1); tf[i] = (float)t[i]; }
            for (int i = 0; i < n * h; ++i) { H[i] = urand(); Hf[i] = (float)H[i]; }
            for (int i = 0; i < n * d; ++i) { F[i] = urand() - 0.5; Ff[i] = (float)F[i]; }
            for (int i = 0; i < n * m; ++i) { W[i] = 0.1 * (urand() - 0.5); Wf[i] = (float)W[i]; }
            double y1[3] = {0.1, -0.2, 0.3}, ll;
            float y1f[3] = {0.1f, -0.2f, 0.3f}, llf;
            for (int seq = 0; seq < 2; ++seq) {
                orc_set_sequential_ou(seq);
                for (int skip = 0; skip < 3; ++skip) {
                    orc_set_ll_skip(skip == 2 ? n + 5 : skip);
                    (void)orc_solve_segment_f64(model, d, m, law, n, t, H, F, W, y1, X, &ll);
                    (void)orc_solve_segment_f32(model, d, m, law, n, tf, Hf, Ff, Wf, y1f, Xf, &llf);
                }
            }
            orc_set_ll_skip(0);
            orc_set_sequential_ou(0);
            if (d == m || model == 1) orc_invsolve_segment_f64(model, d, m, law, n, t, H, F, X, W2);
            double Bt[9] = {0}, beta[3] = {0}, at[6] = {0}, HT[6] = {0}, FT[3] = {0};
            for (int i = 0; i < d * d; ++i) Bt[i] = (i % (d + 1) == 0) ? -0.5 : 0.1;
            for (int i = 0; i < h; ++i) { at[i] = (i == 0 || i == d || i == h - 1) ? 0.3 : 0.0; HT[i] = at[i] * 100; }
            double *c = malloc(n * 8);
            (void)orc_backward_filter_segment(d, Bt, beta, at, n, t, HT, FT, 1.0, H, F, c);
            free(c);
            free(t); free(H); free(F); free(W); free(X); free(W2);
            free(tf); free(Hf); free(Ff); free(Wf); free(Xf);
        }
    }
    double z[2]; float zf[4];
    for (uint32_t i = 0; i < 100000; ++i) {
        orc_normal_block_f64(0x1234 + i, i, 7, i * 3u, 2, z);
        orc_normal_block_f32(0x1234 + i, i, 7, i * 3u, 2, zf);
        if (!isfinite(z[0]) || !isfinite(z[1])) { fprintf(stderr, "non-finite normal\n"); return 2; }
        (void)orc_exp1(77, i, 3, 1);
    }
    puts("asan oracle driver: OK");
    return 0;
}
