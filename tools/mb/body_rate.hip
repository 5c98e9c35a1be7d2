// Microbenchmark: cycles per raster "body" (one splat x one row group, 64 px)
// on gfx950, body = qy add, 2 fma, exp2, mul, 3 fma, sub, with splat params
// uniform (SGPR) or in VGPRs; 16 accumulator groups per lane as in the kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int VARIANT>  // 0: params via kernel args (SGPR), 1: params in VGPRs, 2: no exp
__global__ void __launch_bounds__(256) kern(float* out, int iters, float cx, float A, float Bc,
                                            float Cc, float la, float cr, float cg, float cb) {
    float R[16], G[16], Bl[16], T[16];
#pragma unroll
    for (int g = 0; g < 16; ++g) { R[g] = G[g] = Bl[g] = 0.f; T[g] = 1.f; }
    const float X = (float)(threadIdx.x & 15), Y = (float)(threadIdx.x >> 4);
    float vcx = cx, vcc = Cc, vcr = cr, vcg = cg, vcb = cb;
    if (VARIANT == 1) {  // make them non-uniform-looking (VGPR)
        vcx += threadIdx.x * 0.0f; vcc += threadIdx.x * 0.0f; vcr += threadIdx.x * 0.0f;
        vcg += threadIdx.x * 0.0f; vcb += threadIdx.x * 0.0f;
    }
    for (int it = 0; it < iters; ++it) {
        const float qx = X - vcx - it * 1e-4f;
        const float px = __builtin_fmaf(A * qx, qx, la);
        const float bx = Bc * qx;
        const float qy0 = Y - vcx;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const float qy = qy0 + 4.f * g;
            const float e = __builtin_fmaf(qy, __builtin_fmaf(vcc, qy, bx), px);
            const float f = VARIANT == 2 ? e * 1e-3f : __builtin_amdgcn_exp2f(e);
            const float w = T[g] * f;
            R[g] = __builtin_fmaf(w, vcr, R[g]);
            G[g] = __builtin_fmaf(w, vcg, G[g]);
            Bl[g] = __builtin_fmaf(w, vcb, Bl[g]);
            T[g] = T[g] - w;
        }
    }
    float s = 0;
#pragma unroll
    for (int g = 0; g < 16; ++g) s += R[g] + G[g] + Bl[g] + T[g];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int V>
void run(const char* name, int blocks_per_cu) {
    const int blocks = 256 * blocks_per_cu, iters = 2000;
    float* out;
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    kern<V><<<blocks, 256>>>(out, iters, 7.f, -0.01f, 0.002f, -0.01f, -0.3f, 0.2f, 0.3f, 0.4f);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r)
        kern<V><<<blocks, 256>>>(out, iters, 7.f, -0.01f, 0.002f, -0.01f, -0.3f, 0.2f, 0.3f, 0.4f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 3;
    const double bodies = (double)blocks * 4 * iters * 16;   // wave-level bodies
    printf("%-12s blocks/CU=%d: %.3f ms, %.2f SIMD-cycles per body\n", name, blocks_per_cu, ms,
           ms * 1e-3 * 2.4e9 * 1024 / bodies);
    (void)hipFree(out);
}

int main() {
    for (int b : {1, 2, 4, 5, 8}) {
        run<0>("sgpr-params", b);
        run<1>("vgpr-params", b);
        run<2>("no-exp", b);
    }
    return 0;
}
