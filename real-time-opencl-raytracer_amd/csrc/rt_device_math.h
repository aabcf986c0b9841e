// rt_device_math.h -- the arithmetic of the render path on gfx950, in three modes.
//
// Every mode is an exact restatement of the reference kernel's source order
// (x64/Release/volumeRender.cl); they differ only in how the reference's
// compiler lowers `/`, `sqrt`, contraction and the device-library builtins
// (DESIGN.md 3).  This translation unit is compiled with -ffp-contract=off and
// correctly rounded `/` and sqrt: every fused or approximate operation below is
// spelled out explicitly.
//
// Included once per mode (rt_render.hip); RTK_NS names the namespace and
// RTK_MATH selects the mode:
//   RTK_MATH = 0  S_strict: IEEE binary32, no contraction, correctly rounded `/`
//                 and sqrt; rsqrt(x) = (float)(1/sqrt((double)x)), pow(x,5) in
//                 binary64.  Reproducible on any IEEE host -> the CPU oracle.
//   RTK_MATH = 1  S_hw: S_strict with the device library's rsqrt (v_rsq_f32),
//                 pow (__ocml_pow_f32) and clamp (v_med3_f32) -- the reference
//                 built with -cl-fp32-correctly-rounded-divide-sqrt
//                 -ffp-contract=off (oracle/Makefile.ref "strict").
//   RTK_MATH = 2  S_ref: the reference as its host builds it,
//                 clBuildProgram(program, 0, NULL, NULL, NULL, NULL)
//                 (RayTracer.cpp:2173): S_hw's builtins, plus
//                   * OpenCL-default contraction: a*b+c inside one source
//                     expression is one fma (clang's fmuladd rule: the product
//                     on the left of +/- first, else the one on the right);
//                   * `/` to 2.5 ulp: ldexp(mant(a) * rcp(mant(b)), exp(a) - exp(b))
//                     with v_frexp_* / v_rcp_f32 / v_ldexp_f32 (the gfx950
//                     backend's expansion of an fdiv carrying !fpmath 2.5);
//                     1.0f/b: ldexp(rcp(mant(b)), -exp(b));
//                   * sqrt to 3 ulp: v_sqrt_f32 with the denormal pre/post scale.
#include <hip/hip_runtime.h>

#ifndef RTK_NS
#define RTK_NS rtk
#endif
#ifndef RTK_MATH
#define RTK_MATH 0
#endif

namespace RTK_NS {

constexpr int kMath = RTK_MATH;

struct F3 {
    float x, y, z;
};

__device__ __forceinline__ F3 mk(float x, float y, float z) { return F3{x, y, z}; }
__device__ __forceinline__ F3 xyz(const float4& a) { return F3{a.x, a.y, a.z}; }
__device__ __forceinline__ F3 operator+(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ F3 operator-(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ F3 operator*(F3 a, F3 b) { return F3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ F3 operator*(F3 a, float s) { return F3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ F3 operator*(float s, F3 a) { return F3{s * a.x, s * a.y, s * a.z}; }

// ---- the mode-dependent primitives ----
#if RTK_MATH == 2
// fdiv !fpmath 2.5 (AMDGPUCodeGenPrepare's frexp expansion; denormal-safe)
__device__ __forceinline__ float div_(float a, float b) {
    const float ma = __builtin_amdgcn_frexp_mantf(a), mb = __builtin_amdgcn_frexp_mantf(b);
    const int ea = __builtin_amdgcn_frexp_expf(a), eb = __builtin_amdgcn_frexp_expf(b);
    return __builtin_amdgcn_ldexpf(ma * __builtin_amdgcn_rcpf(mb), ea - eb);
}
// 1.0f / b under the same metadata (the backend's 1-ulp rcp expansion)
__device__ __forceinline__ float rcp_(float b) {
    return __builtin_amdgcn_ldexpf(__builtin_amdgcn_rcpf(__builtin_amdgcn_frexp_mantf(b)),
                                   -__builtin_amdgcn_frexp_expf(b));
}
// llvm.sqrt.f32 !fpmath 3.0: inputs below 2^-126 are scaled by 2^32 and the root by 2^-16
__device__ __forceinline__ float sqrt_(float x) {
    const bool small = x < 0x1p-126f;
    return __builtin_amdgcn_ldexpf(__builtin_amdgcn_sqrtf(__builtin_amdgcn_ldexpf(x, small ? 32 : 0)), small ? -16 : 0);
}
// a*b + c contracted (llvm.fmuladd -> v_fma_f32 on gfx950)
__device__ __forceinline__ float mad_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
#else
__device__ __forceinline__ float div_(float a, float b) { return a / b; }
__device__ __forceinline__ float rcp_(float b) { return 1.0f / b; }
__device__ __forceinline__ float sqrt_(float x) { return ::sqrtf(x); }
__device__ __forceinline__ float mad_(float a, float b, float c) { return a * b + c; }
#endif
// a*b - c*d as the reference compiler sees it: (a*b) on the left of `-` -> fma(a, b, -(c*d))
__device__ __forceinline__ float msub_(float a, float b, float c, float d) { return mad_(a, b, -(c * d)); }
__device__ __forceinline__ F3 mad3(F3 a, float s, F3 c) { return F3{mad_(a.x, s, c.x), mad_(a.y, s, c.y), mad_(a.z, s, c.z)}; }

// opencl.bc _Z3dotDv3_fS_ : fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
__device__ __forceinline__ float dot(F3 a, F3 b) {
    return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
// opencl.bc _Z5crossDv3_fS_
__device__ __forceinline__ F3 cross(F3 a, F3 b) {
    return F3{__builtin_fmaf(a.y, b.z, b.y * -a.z), __builtin_fmaf(a.z, b.x, b.z * -a.x),
              __builtin_fmaf(a.x, b.y, b.x * -a.y)};
}
#if RTK_MATH >= 1
__device__ __forceinline__ float rsqrt_s(float x) { return ::rsqrtf(x); }
#else
__device__ __forceinline__ float rsqrt_s(float x) { return (float)(1.0 / ::sqrt((double)x)); }
#endif

// opencl.bc _Z9normalizeDv3_f (rsqrt substituted in S_strict)
__device__ __forceinline__ F3 normalize(F3 p) {
    if (p.x == 0.0f && p.y == 0.0f && p.z == 0.0f) return p;
    float l2 = dot(p, p);
    if (l2 < 1.17549435e-38f) {
        p = p * 0x1p86f;
        l2 = dot(p, p);
    } else if (l2 == __builtin_inff()) {
        p = p * 0x1p-66f;
        l2 = dot(p, p);
        if (l2 == __builtin_inff()) {
            p = F3{__builtin_copysignf(__builtin_isinf(p.x) ? 1.0f : 0.0f, p.x),
                   __builtin_copysignf(__builtin_isinf(p.y) ? 1.0f : 0.0f, p.y),
                   __builtin_copysignf(__builtin_isinf(p.z) ? 1.0f : 0.0f, p.z)};
            l2 = dot(p, p);
        }
    }
    return p * rsqrt_s(l2);
}

#if RTK_MATH >= 1
// OpenCL clamp -> __ockl_median3_f32 -> v_med3_f32 (identical to the line below for non-NaN x)
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
__device__ __forceinline__ float pow5(float x) { return ::powf(x, 5.0f); }
#else
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ __forceinline__ float pow5(float x) {
    const double d = (double)x;
    return (float)((((d * d) * d) * d) * d);
}
#endif

// volumeRender.cl:25  i - 2.0f * n * dot(n, i)  ->  S_ref: fma(-(2n), dot, i)
__device__ __forceinline__ F3 reflect(F3 i, F3 n) {
    const float d = dot(n, i);
    if (kMath == 2) return F3{mad_(n.x * -2.0f, d, i.x), mad_(n.y * -2.0f, d, i.y), mad_(n.z * -2.0f, d, i.z)};
    return i - (2.0f * n) * d;
}

struct Ray {
    F3 ori, dir, inv_dir;
};

// volumeRender.cl:205-211 (inv_dir: double 1.0 / dir, then rounded)
__device__ __forceinline__ Ray ray_init(F3 o, F3 d) {
    Ray r;
    r.ori = o;
    r.dir = normalize(d);
    r.inv_dir = F3{(float)(1.0 / (double)r.dir.x), (float)(1.0 / (double)r.dir.y), (float)(1.0 / (double)r.dir.z)};
    return r;
}

// volumeRender.cl:236-254 (scene box, inv_dir multiply; no a*b+c in it)
__device__ __forceinline__ bool ray_box_scene(F3 bmin, F3 bmax, F3 org, F3 inv) {
    float l1 = (bmin.x - org.x) * inv.x;
    float l2 = (bmax.x - org.x) * inv.x;
    float tmin = fminf(l1, l2);
    float tmax = fmaxf(l1, l2);
    l1 = (bmin.y - org.y) * inv.y;
    l2 = (bmax.y - org.y) * inv.y;
    tmin = fmaxf(fminf(l1, l2), tmin);
    tmax = fminf(fmaxf(l1, l2), tmax);
    l1 = (bmin.z - org.z) * inv.z;
    l2 = (bmax.z - org.z) * inv.z;
    tmin = fmaxf(fminf(l1, l2), tmin);
    tmax = fminf(fmaxf(l1, l2), tmax);
    return (tmax >= tmin) && (tmax >= 0.0f);
}

// volumeRender.cl:257-282 (det = 1.0f / det: rcp_)
__device__ __forceinline__ float ray_tri(const Ray& r, F3 v0, F3 e1, F3 e2) {
    F3 tvec = r.ori - v0;
    F3 pvec = cross(r.dir, e2);
    float det = dot(e1, pvec);
    det = rcp_(det);
    float u = dot(tvec, pvec) * det;
    if (u < 0.0f || u > 1.0f) return -1.0f;
    F3 qvec = cross(tvec, e1);
    float v = dot(r.dir, qvec) * det;
    if (v < 0.0f || (u + v) > 1.0f) return -1.0f;
    return dot(e2, qvec) * det;
}

// volumeRender.cl:27-53: Cramer barycentrics on absolute positions.
//   D = p0.x*(A) - p1.x*(B) + p2.x*(C), each (..) = u*v - w*z
// S_ref contraction: (u*v - w*z) -> fma(u, v, -(w*z)); the outer
// ((p0.x*A) - (p1.x*B)) + (p2.x*C) -> fma(p2.x, C, fma(p0.x, A, -(p1.x*B)));
// normNew = l.x*vn0 + l.y*vn1 + l.z*vn2 -> fma(l.z, vn2, fma(l.x, vn0, l.y*vn1)).
__device__ __forceinline__ float det3(float a0, float A, float b0, float B, float c0, float C) {
    if (kMath == 2) return mad_(c0, C, mad_(a0, A, -(b0 * B)));
    return a0 * A - b0 * B + c0 * C;
}
__device__ __forceinline__ F3 normal_at(F3 pn, F3 p0, F3 p1, F3 p2, F3 n0, F3 n1, F3 n2) {
    const float P1 = msub_(p1.y, p2.z, p2.y, p1.z);   // p1.y*p2.z - p2.y*p1.z
    const float P2 = msub_(p0.y, p2.z, p2.y, p0.z);   // p0.y*p2.z - p2.y*p0.z
    const float P3 = msub_(p0.y, p1.z, p1.y, p0.z);   // p0.y*p1.z - p1.y*p0.z
    const float Q2 = msub_(pn.y, p2.z, p2.y, pn.z);   // pNew.y*p2.z - p2.y*pNew.z
    const float Q3 = msub_(pn.y, p1.z, p1.y, pn.z);   // pNew.y*p1.z - p1.y*pNew.z
    const float R3 = msub_(p0.y, pn.z, pn.y, p0.z);   // p0.y*pNew.z - pNew.y*p0.z
    const float S1 = msub_(p1.y, pn.z, pn.y, p1.z);   // p1.y*pNew.z - pNew.y*p1.z
    const float Det = det3(p0.x, P1, p1.x, P2, p2.x, P3);
    const float D0 = det3(pn.x, P1, p1.x, Q2, p2.x, Q3);
    const float D1 = det3(p0.x, Q2, pn.x, P2, p2.x, R3);
    const float D2 = det3(p0.x, S1, p1.x, R3, pn.x, P3);
    const float l0 = div_(D0, Det), l1 = div_(D1, Det), l2 = div_(D2, Det);
    if (kMath == 2) {
        const F3 m = n1 * l1;
        return F3{mad_(l2, n2.x, mad_(l0, n0.x, m.x)), mad_(l2, n2.y, mad_(l0, n0.y, m.y)),
                  mad_(l2, n2.z, mad_(l0, n0.z, m.z))};
    }
    return (l0 * n0 + l1 * n1) + l2 * n2;
}

// volumeRender.cl:1732-1779
__device__ __forceinline__ float ggx_partial_geometry(float c, float alpha) {
    float cs = clampf(c * c, 0.0f, 1.0f);
    float tan2 = div_(1.0f - cs, cs);
    return div_(2.0f, 1.0f + sqrt_(mad_(alpha * alpha, tan2, 1.0f)));   // 1 + alpha*alpha*tan2
}
__device__ __forceinline__ float ggx_distribution(float c, float alpha) {
    float alpha2 = alpha * alpha;
    float nh = clampf(c * c, 0.0f, 1.0f);
    float den = mad_(nh, alpha2, 1.0f - nh);                               // nh*alpha2 + (1 - nh)
    return div_(alpha2, 3.14159274101257324219f * den * den);
}
__device__ __forceinline__ F3 cook_torrance_ggx(F3 n, F3 l, F3 v, F3 albedo, float f0, float roughness) {
    n = normalize(n);
    v = normalize(v);
    l = normalize(l);
    F3 h = normalize(v + l);
    float NL = dot(n, l);
    if (NL <= 0.0f) return F3{0, 0, 0};
    float NV = dot(n, v);
    if (NV <= 0.0f) return F3{0, 0, 0};
    float NH = dot(n, h);
    float HV = dot(h, v);
    float rs = roughness * roughness;
    float G = ggx_partial_geometry(NV, rs) * ggx_partial_geometry(NL, rs);
    float D = ggx_distribution(NH, rs);
    float p = pow5(1.0f - clampf(HV, 0.0f, 1.0f));
    float Fc = mad_(1.0f - f0, p, f0);                                     // F0 + (1 - F0) * pow(..)
    F3 F = F3{Fc, Fc, Fc};
    const float den = NV + 0.001f;
    const F3 sk = ((G * D) * F) * 0.25f;
    // An IEEE division in every mode, S_ref included: F is a splat of the constant f0, so
    // the reference compiler scalarises G*D*F*0.25f/(NV+0.001f) into ONE fdiv and drops its
    // !fpmath 2.5 on the way (the kernel's IR after AMDGPUCodeGenPrepare keeps exactly this
    // fdiv, correctly rounded, while every other float `/` is expanded to the 2.5-ulp form).
    F3 specK = F3{sk.x / den, sk.y / den, sk.z / den};
    F3 diffK = F3{clampf(1.0f - F.x, 0.0f, 1.0f), clampf(1.0f - F.y, 0.0f, 1.0f), clampf(1.0f - F.z, 0.0f, 1.0f)};
    const F3 md = (albedo * diffK) * NL;
    const float kPi = 3.14159274101257324219f;
    F3 m = F3{div_(md.x, kPi), div_(md.y, kPi), div_(md.z, kPi)} + specK;
    return F3{fmaxf(0.0f, m.x), fmaxf(0.0f, m.y), fmaxf(0.0f, m.z)};
}

// volumeRender.cl:186-195
__device__ __forceinline__ uint32_t rgb_to_int(float r, float g, float b) {
    r = clampf(r, 0.0f, 255.0f);
    g = clampf(g, 0.0f, 255.0f);
    b = clampf(b, 0.0f, 255.0f);
    return ((uint32_t)b << 16) | ((uint32_t)g << 8) | (uint32_t)r;
}

}  // namespace RTK_NS
