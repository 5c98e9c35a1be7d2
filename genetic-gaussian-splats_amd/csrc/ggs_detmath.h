// Deterministic binary32 elementary functions for the bounds-critical prep stage.
//
// Device mirror of oracle/detmath.py: the same Cephes-style algorithms with the
// same constants (given as bit patterns) and the same operation order.  This
// translation unit is compiled with -ffp-contract=off and without fast-math, so
// every step is one IEEE-754 binary32 add/sub/mul/div/sqrt (correctly rounded:
// ggs_div_rn / ggs_sqrt_rn below), rint/floor/ceil, or an exact bit operation —
// exactly what numpy float32 array arithmetic does.  Result: integer splat bounds
// are bit-identical between this HIP path and the numpy oracle (SURVEY.md §7
// "Hard parts" 1).  Domain conventions (shared with the oracle): exp(x)=0 for
// x<-87 (no denormal results), +inf above 88.72284; NaN in -> NaN out.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ggs {
namespace detmath {

__host__ __device__ constexpr float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }

constexpr float LOG2E = bitsf(0x3FB8AA3Bu);
constexpr float EXP_C1 = bitsf(0x3F318000u);
constexpr float EXP_C2 = bitsf(0xB95E8083u);
constexpr float EXP_P0 = bitsf(0x39506967u), EXP_P1 = bitsf(0x3AB743CEu), EXP_P2 = bitsf(0x3C088908u),
                EXP_P3 = bitsf(0x3D2AA9C1u), EXP_P4 = bitsf(0x3E2AAAAAu), EXP_P5 = bitsf(0x3F000000u);
constexpr float EXP_HI = bitsf(0x42B17218u);
constexpr float EXP_LO = bitsf(0xC2AE0000u);
constexpr float SQRTHF = bitsf(0x3F3504F3u);
constexpr float LOG_P0 = bitsf(0x3D9021BBu), LOG_P1 = bitsf(0xBDEBD1B8u), LOG_P2 = bitsf(0x3DEF251Au),
                LOG_P3 = bitsf(0xBDFE5D4Fu), LOG_P4 = bitsf(0x3E11E9BFu), LOG_P5 = bitsf(0xBE2AAE50u),
                LOG_P6 = bitsf(0x3E4CCEACu), LOG_P7 = bitsf(0xBE7FFFFCu), LOG_P8 = bitsf(0x3EAAAAAAu);
constexpr float LOG_Q1 = bitsf(0xB95E8083u);
constexpr float LOG_Q2 = bitsf(0x3F318000u);
constexpr float TWO_OVER_PI = bitsf(0x3F22F983u);
constexpr float PIO2_1 = bitsf(0x3FC90000u), PIO2_2 = bitsf(0x39FDA000u), PIO2_3 = bitsf(0x33A22169u);
constexpr float SIN_S0 = bitsf(0xB94CA1F9u), SIN_S1 = bitsf(0x3C08839Eu), SIN_S2 = bitsf(0xBE2AAAA3u);
constexpr float COS_C0 = bitsf(0x37CCF5CEu), COS_C1 = bitsf(0xBAB6061Au), COS_C2 = bitsf(0x3D2AAAA5u);
constexpr float EPS12 = bitsf(0x2B8CBCCCu);  // float32(1e-12), encode.py:15
constexpr float EPS6 = bitsf(0x358637BDu);   // float32(1e-6),  render.py:19-20
constexpr float FLT_TINY = bitsf(0x00800000u);

__device__ __forceinline__ bool isnan_(float x) { return x != x; }

// Correctly rounded sqrt and division.  hipcc's default
// (-fhip-fp32-correctly-rounded-divide-sqrt) lowers llvm.sqrt.f32 and fdiv to
// IEEE-exact sequences; HIP's __fsqrt_rn is NOT (it maps to the native ~1-ulp
// v_sqrt_f32 unless OCML_BASIC_ROUNDED_OPERATIONS is set), so it is never used.
// tests/test_gpu_parity.py::test_detmath_bit_exact checks both against numpy.
__device__ __forceinline__ float ggs_sqrt_rn(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ float ggs_div_rn(float x, float y) { return x / y; }
// NaN-propagating max/min/clamp (torch.clamp / np.maximum / np.clip semantics)
__device__ __forceinline__ float nmax(float x, float lo) { return isnan_(x) ? x : (x < lo ? lo : x); }
__device__ __forceinline__ float nclamp(float x, float lo, float hi) {
    return isnan_(x) ? x : (x < lo ? lo : (x > hi ? hi : x));
}

__device__ __forceinline__ float det_expf(float x) {
    const float fk = rintf(x * LOG2E);
    float r = x - fk * EXP_C1;
    r = r - fk * EXP_C2;
    const float zz = r * r;
    float y = EXP_P0;
    y = y * r + EXP_P1;
    y = y * r + EXP_P2;
    y = y * r + EXP_P3;
    y = y * r + EXP_P4;
    y = y * r + EXP_P5;
    y = y * zz;
    y = y + r;
    y = y + 1.0f;
    int k = isnan_(fk) ? 0 : (int)fminf(fmaxf(fk, -126.0f), 128.0f);
    if (k > 127) { y = y * 2.0f; k -= 1; }
    const float p2 = __builtin_bit_cast(float, (uint32_t)(k + 127) << 23);
    float out = y * p2;
    if (x < EXP_LO) out = 0.0f;
    if (x > EXP_HI) out = __builtin_inff();
    if (isnan_(x)) out = x;
    return out;
}

__device__ __forceinline__ float det_logf(float x) {
    const bool sub = (x > 0.0f) && (x < FLT_TINY);
    const float xs = sub ? x * 8388608.0f : x;
    const uint32_t bits = __builtin_bit_cast(uint32_t, xs);
    int e = (int)((bits >> 23) & 0xFFu) - 126;
    if (sub) e -= 23;
    float m = __builtin_bit_cast(float, (bits & 0x807FFFFFu) | 0x3F000000u);
    if (m < SQRTHF) { e -= 1; m = (m + m) - 1.0f; } else { m = m - 1.0f; }
    const float z = m * m;
    float y = LOG_P0;
    y = y * m + LOG_P1;
    y = y * m + LOG_P2;
    y = y * m + LOG_P3;
    y = y * m + LOG_P4;
    y = y * m + LOG_P5;
    y = y * m + LOG_P6;
    y = y * m + LOG_P7;
    y = y * m + LOG_P8;
    y = y * m;
    y = y * z;
    const float fe = (float)e;
    y = y + fe * LOG_Q1;
    y = y - 0.5f * z;
    float r = m + y;
    r = r + fe * LOG_Q2;
    if (x == 0.0f) r = -__builtin_inff();
    if (x == __builtin_inff()) r = __builtin_inff();
    if (x < 0.0f || isnan_(x)) r = __builtin_nanf("");
    return r;
}

__device__ __forceinline__ void det_sincosf(float x, float* sin_out, float* cos_out) {
    const float j = rintf(x * TWO_OVER_PI);
    float r = x - j * PIO2_1;
    r = r - j * PIO2_2;
    r = r - j * PIO2_3;
    const float q = j - 4.0f * floorf(j * 0.25f);
    const int qi = (isnan_(q) ? 0 : (int)q) & 3;
    const float zz = r * r;
    float t = SIN_S0 * zz;
    t = t + SIN_S1;
    t = t * zz;
    t = t + SIN_S2;
    t = t * zz;
    t = t * r;
    const float s = t + r;
    t = COS_C0 * zz;
    t = t + COS_C1;
    t = t * zz;
    t = t + COS_C2;
    t = t * zz;
    t = t * zz;
    t = t - 0.5f * zz;
    const float c = t + 1.0f;
    float so, co;
    switch (qi) {
        case 0: so = s; co = c; break;
        case 1: so = c; co = -s; break;
        case 2: so = -s; co = -c; break;
        default: so = -c; co = s; break;
    }
    if (!(fabsf(x) <= __builtin_huge_valf())) { so = __builtin_nanf(""); co = so; }
    *sin_out = so;
    *cos_out = co;
}

}  // namespace detmath
}  // namespace ggs
