// Microbenchmark: the raster's row-pair step (7 packed ops: F*=R, R*=rho, w=T*F,
// RGB += c*w, T -= w) over 16 packed accumulator pairs per lane, straight-line as
// in the full-height visit, vs waves per SIMD.  Prints cycles per packed op per
// SIMD, i.e. how close one, two or three waves come to the VALU's issue rate.
//   hipcc -O3 --offload-arch=gfx950 tools/mb/pair_rate.hip -o tools/mb/pair_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// BR > 0: + BR scalar control-flow snippets per visit, KIND:
//   0 s_cmp + s_cbranch_scc1 over one s_nop (TAKEN) or falling through it
//   1 s_cmp only (SALU, no branch)
//   2 s_branch (unconditional) over one s_nop
//   3 s_cbranch_scc1 (taken) on an SCC set once per visit, no compare in between
//   4 indirect jump: s_getpc_b64 + s_add_u32/s_addc_u32 + s_setpc_b64 over one s_nop
template <int HEAD, int BR = 0, bool TAKEN = true, int KIND = 0>
__global__ void __launch_bounds__(64) kern(float* out, int visits, float rho, float cr, float cg, float cb) {
    f2 Rr[16], Gg[16], Bb[16], T[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { Rr[k] = Gg[k] = Bb[k] = (f2){0.f, 0.f}; T[k] = (f2){1.f, 1.f}; }
    const float X = (float)(threadIdx.x & 15), Y = (float)(threadIdx.x >> 4);
    for (int v = 0; v < visits; ++v) {
        f2 F, R;
        if (HEAD) {
            const float qx = X - 7.5f - v * 1e-6f;
            const float px = __builtin_fmaf(-0.01f * qx, qx, -0.3f);
            const float bx = 0.002f * qx;
            const f2 qy = (f2){Y - 60.f, Y - 56.f};
            const f2 e = fma2(qy, fma2((f2){-0.001f, -0.001f}, qy, (f2){bx, bx}), (f2){px, px});
            F = (f2){__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
            R.x = __builtin_amdgcn_exp2f(fminf(__builtin_fmaf(qy.y, -0.016f, 8.f * bx), 100.f));
            R.y = R.x * 0.97f;
        } else {
            F = (f2){0.5f + v * 1e-9f, 0.4f};
            R = (f2){0.99f, 0.98f};
        }
        if (KIND == 3 && BR) asm volatile("s_cmp_eq_u32 %0, %0" ::"s"(v) : "scc");
#pragma unroll
        for (int b = 0; b < BR; ++b) {
            if (KIND == 0 && TAKEN)
                asm volatile("s_cmp_eq_u32 %0, %0\n\ts_cbranch_scc1 1f\n\ts_nop 0\n1:" ::"s"(v) : "scc");
            if (KIND == 0 && !TAKEN)
                asm volatile("s_cmp_lg_u32 %0, %0\n\ts_cbranch_scc1 1f\n\ts_nop 0\n1:" ::"s"(v) : "scc");
            if (KIND == 1) asm volatile("s_cmp_eq_u32 %0, %0" ::"s"(v) : "scc");
            if (KIND == 2) asm volatile("s_branch 1f\n\ts_nop 0\n1:");
            if (KIND == 3) asm volatile("s_cbranch_scc1 1f\n\ts_nop 0\n1:");
            if (KIND == 4) {
                asm volatile("s_getpc_b64 s[92:93]\n.Lpc%=:\n\ts_add_u32 s92, s92, 1f-.Lpc%=\n\t"
                             "s_addc_u32 s93, s93, 0\n\ts_setpc_b64 s[92:93]\n\ts_nop 0\n1:" ::: "s92", "s93", "scc");
            }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (k) { F = F * R; R = R * (f2){rho, rho}; }
            const f2 w = T[k] * F;
            Rr[k] = fma2((f2){cr, cr}, w, Rr[k]);
            Gg[k] = fma2((f2){cg, cg}, w, Gg[k]);
            Bb[k] = fma2((f2){cb, cb}, w, Bb[k]);
            T[k] = T[k] - w;
        }
    }
    float s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += Rr[k].x + Gg[k].y + Bb[k].x + T[k].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int HEAD, int BR = 0, bool TAKEN = true, int KIND = 0>
void run(int waves_per_simd) {
    const int blocks = 1024 * waves_per_simd;         // one wave per block, 1024 SIMDs
    const int visits = 2000;
    float* out;
    (void)hipMalloc(&out, sizeof(float) * blocks * 64);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<HEAD, BR, TAKEN, KIND><<<blocks, 64>>>(out, visits, 0.999f, 0.2f, 0.3f, 0.4f);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) kern<HEAD, BR, TAKEN, KIND><<<blocks, 64>>>(out, visits, 0.999f, 0.2f, 0.3f, 0.4f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double pk_ops = (double)blocks * visits * (16 * 7 - 2);   // packed ops of the 16 pair steps
    const double cycles = ms * 1e-3 * 2.4e9;                        // nominal clock
    static const char* kinds[] = {"cmp+cbranch", "cmp only", "s_branch", "cbranch (scc ready)", "getpc+add+setpc"};
    printf("head=%d %2d x %-19s%s waves/SIMD=%d: %.3f ms, %.2f SIMD cycles per pair-step packed op, %.0f ns per visit per wave\n",
           HEAD, BR, BR ? kinds[KIND] : "", BR && KIND == 0 ? (TAKEN ? " taken" : " not-taken") : "", waves_per_simd, ms, cycles * 1024 / pk_ops, ms * 1e6 / visits);
    (void)hipFree(out);
}

int main() {
    for (int w : {1, 2, 3, 4}) run<0>(w);
    for (int w : {1, 2, 3, 4}) run<1>(w);
    for (int w : {1, 3}) {
        run<1, 8, true>(w); run<1, 16, true>(w); run<1, 8, false>(w); run<1, 16, false>(w);
        run<1, 8, true, 1>(w); run<1, 8, true, 2>(w); run<1, 8, true, 3>(w); run<1, 8, true, 4>(w);
    }
    return 0;
}
