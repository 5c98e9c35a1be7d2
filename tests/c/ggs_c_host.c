/* A plain-C host of the libggs C ABI (include/ggs.h): the boundary as a C or
 * cgo/JNI caller would bind it.  Renders a small synthetic population with
 * ggs_render, computes the weighted fitness of those images on the host in
 * double, and checks ggs_fitness (the fused device path) against it.
 * Exit status: 0 ok, 2 no HIP device (ggs_init -> GGS_ENODEV), 1 mismatch/error. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "ggs.h"

static unsigned long long rng = 88172645463325252ull;
static double urand(void) {                 /* xorshift64, [0, 1) */
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (double)(rng >> 11) / 9007199254740992.0;
}

int main(void) {
    const int B = 4, N = 24, H = 48, W = 40;
    printf("%s\n", ggs_version());
    int nd = ggs_init(0);
    if (nd == GGS_ENODEV) {
        printf("no device: %s\n", ggs_last_error());
        return 2;
    }
    if (nd < 0) { fprintf(stderr, "ggs_init: %s\n", ggs_last_error()); return 1; }
    float *g = malloc(sizeof(float) * B * N * 9), *g9 = malloc(sizeof(float) * B * N * 9);
    float *tgt = malloc(sizeof(float) * H * W * 3), *mask = malloc(sizeof(float) * H * W);
    float *img = malloc(sizeof(float) * B * H * W * 3), fit[4];
    for (int i = 0; i < B * N; ++i) {      /* axes-angle genomes (population.py:27-45 ranges) */
        float* r = g + 9 * i;
        r[0] = (float)urand(); r[1] = (float)urand();
        r[2] = (float)log(3.0 + 2.0 * urand()); r[3] = (float)log(3.0 + 2.0 * urand());
        r[4] = (float)(6.283185307179586 * urand() - 3.141592653589793);
        for (int c = 5; c < 8; ++c) r[c] = (float)(255.0 * urand());
        r[8] = (float)(180.0 + 75.0 * urand());
    }
    for (int i = 0; i < H * W * 3; ++i) tgt[i] = (float)urand();
    for (int i = 0; i < H * W; ++i) mask[i] = (float)(0.405 + 0.595 * urand());
    if (ggs_encode(g, (int64_t)B * N, 9, g9) ||
        ggs_render(g9, B, N, 9, H, W, 3.0f, NULL, img, 0) ||
        ggs_fitness(g, B, N, 9, tgt, mask, GGS_FIT_WEIGHTED, 1.0f, H, W, 3.0f, fit, 0)) {
        fprintf(stderr, "ggs: %s\n", ggs_last_error());
        return 1;
    }
    int bad = 0;
    for (int b = 0; b < B; ++b) {          /* fitness.py:28-31 on the rendered image */
        double num = 0.0, den = 0.0;
        for (int p = 0; p < H * W; ++p) {
            double d2 = 0.0;
            for (int c = 0; c < 3; ++c) {
                const double d = (double)img[((size_t)b * H * W + p) * 3 + c] - tgt[p * 3 + c];
                d2 += d * d;
            }
            num += mask[p] * d2;
            den += mask[p];
        }
        const double ref = num / (den + 1e-12);
        const double rel = fabs(fit[b] - ref) / ref;
        printf("candidate %d: fused %.8f  host-from-image %.8f  rel %.2e\n", b, fit[b], ref, rel);
        bad |= !(rel <= 1e-5);
    }
    /* the reference's assert conditions come back as GGS_EINVAL */
    if (ggs_render(g9, 1, N, 8, H, W, 3.0f, NULL, img, 0) != GGS_EINVAL) bad = 1;
    ggs_shutdown();
    free(g); free(g9); free(tgt); free(mask); free(img);
    return bad;
}
