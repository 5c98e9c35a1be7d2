// Microbenchmark: VALU throughput on gfx950 for v_fma_f32, v_pk_fma_f32 and
// v_exp_f32 vs. waves per SIMD and ILP.  Prints ops/cycle/SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int ILP, int MODE>  // MODE 0 fma, 1 pk_fma, 2 exp, 3 fma+exp mix (7:1)
__global__ void kern(float* out, int iters, float a, float b) {
    float x[ILP];
    f2 y[ILP];
    for (int i = 0; i < ILP; ++i) { x[i] = threadIdx.x * 1e-3f + i; y[i] = (f2){x[i], x[i] + 1}; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < ILP; ++i) {
            if (MODE == 0) x[i] = __builtin_fmaf(x[i], a, b);
            if (MODE == 1) y[i] = __builtin_elementwise_fma(y[i], (f2){a, a}, (f2){b, b});
            if (MODE == 2) x[i] = __builtin_amdgcn_exp2f(x[i]) * -1.0f;
            if (MODE == 3) {
                x[i] = __builtin_fmaf(x[i], a, b); x[i] = __builtin_fmaf(x[i], a, b);
                x[i] = __builtin_fmaf(x[i], a, b); x[i] = __builtin_fmaf(x[i], a, b);
                x[i] = __builtin_fmaf(x[i], a, b); x[i] = __builtin_fmaf(x[i], a, b);
                x[i] = __builtin_fmaf(x[i], a, b); x[i] = __builtin_amdgcn_exp2f(x[i]) * -1e-3f;
            }
        }
    }
    float s = 0;
    for (int i = 0; i < ILP; ++i) s += x[i] + y[i].x + y[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ILP, int MODE>
void run(const char* name, int waves_per_simd, int ops_per_iter_per_ilp) {
    const int cus = 256, threads = 256;               // 4 waves/WG = 1 wave per SIMD
    const int blocks = cus * waves_per_simd;
    const int iters = 4000;
    float* out;
    hipMalloc(&out, sizeof(float) * blocks * threads);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    kern<ILP, MODE><<<blocks, threads>>>(out, iters, 0.999f, 1e-3f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) kern<ILP, MODE><<<blocks, threads>>>(out, iters, 0.999f, 1e-3f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double wave_instr = (double)blocks * 4 * iters * ILP * ops_per_iter_per_ilp;
    const double cycles = ms * 1e-3 * 2.4e9;
    printf("%-10s ILP=%d waves/SIMD=%d: %.3f ms, %.2f cycles per wave-instr per SIMD\n", name, ILP,
           waves_per_simd, ms, cycles * 1024 / wave_instr);
    hipFree(out);
}

int main() {
    for (int w : {1, 2, 4, 8}) {
        run<1, 0>("fma", w, 1); run<4, 0>("fma", w, 1); run<8, 0>("fma", w, 1);
        run<4, 1>("pk_fma", w, 1); run<8, 1>("pk_fma", w, 1);
        run<4, 2>("exp", w, 2); run<8, 2>("exp", w, 2);
        run<4, 3>("7fma+exp", w, 9);
    }
    return 0;
}
