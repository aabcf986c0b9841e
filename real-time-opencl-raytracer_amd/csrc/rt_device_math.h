// rt_device_math.h -- the S_strict arithmetic of the render path on gfx950.
//
// Exactly the operations of DESIGN.md section 3 (same as the reference kernel's
// source order, OpenCL builtins as ROCm device-libs define them, correctly
// rounded '/' and sqrt, rsqrt and pow(x,5) in binary64).  This translation
// unit is compiled with -ffp-contract=off: every fma below is explicit.
//
// Included once per math mode (rt_render.hip): RTK_NS names the namespace and
// RTK_HWMATH selects the two substituted functions:
//   RTK_HWMATH = 0  rsqrt(x) = (float)(1/sqrt((double)x)), pow(x,5) in binary64
//                   (S_strict: reproducible on any IEEE host -> the CPU oracle)
//   RTK_HWMATH = 1  rsqrt = __ocml_rsqrt_f32 (v_rsq_f32), pow = __ocml_pow_f32,
//                   i.e. what the reference kernel links on gfx950 (S_hw).
#include <hip/hip_runtime.h>

#ifndef RTK_NS
#define RTK_NS rtk
#endif
#ifndef RTK_HWMATH
#define RTK_HWMATH 0
#endif

namespace RTK_NS {

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
__device__ __forceinline__ F3 operator/(F3 a, float s) { return F3{a.x / s, a.y / s, a.z / s}; }

// opencl.bc _Z3dotDv3_fS_ : fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
__device__ __forceinline__ float dot(F3 a, F3 b) {
    return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
// opencl.bc _Z5crossDv3_fS_
__device__ __forceinline__ F3 cross(F3 a, F3 b) {
    return F3{__builtin_fmaf(a.y, b.z, b.y * -a.z), __builtin_fmaf(a.z, b.x, b.z * -a.x),
              __builtin_fmaf(a.x, b.y, b.x * -a.y)};
}
#if RTK_HWMATH
__device__ __forceinline__ float rsqrt_s(float x) { return ::rsqrtf(x); }
#else
__device__ __forceinline__ float rsqrt_s(float x) { return (float)(1.0 / ::sqrt((double)x)); }
#endif

// opencl.bc _Z9normalizeDv3_f (rsqrt substituted)
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

#if RTK_HWMATH
// OpenCL clamp -> __ockl_median3_f32 -> v_med3_f32 (identical to the line below for non-NaN x)
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
#else
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
#endif
#if RTK_HWMATH
__device__ __forceinline__ float pow5(float x) { return ::powf(x, 5.0f); }
#else
__device__ __forceinline__ float pow5(float x) {
    double d = (double)x;
    return (float)((((d * d) * d) * d) * d);
}
#endif

// volumeRender.cl:25
__device__ __forceinline__ F3 reflect(F3 i, F3 n) { return i - (2.0f * n) * dot(n, i); }

struct Ray {
    F3 ori, dir, inv_dir;
};

// volumeRender.cl:205-211
__device__ __forceinline__ Ray ray_init(F3 o, F3 d) {
    Ray r;
    r.ori = o;
    r.dir = normalize(d);
    r.inv_dir = F3{(float)(1.0 / (double)r.dir.x), (float)(1.0 / (double)r.dir.y), (float)(1.0 / (double)r.dir.z)};
    return r;
}

// volumeRender.cl:236-254 (scene box, inv_dir multiply)
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

// volumeRender.cl:257-282
__device__ __forceinline__ float ray_tri(const Ray& r, F3 v0, F3 e1, F3 e2) {
    F3 tvec = r.ori - v0;
    F3 pvec = cross(r.dir, e2);
    float det = dot(e1, pvec);
    det = 1.0f / det;
    float u = dot(tvec, pvec) * det;
    if (u < 0.0f || u > 1.0f) return -1.0f;
    F3 qvec = cross(tvec, e1);
    float v = dot(r.dir, qvec) * det;
    if (v < 0.0f || (u + v) > 1.0f) return -1.0f;
    return dot(e2, qvec) * det;
}

// volumeRender.cl:27-53
__device__ __forceinline__ F3 normal_at(F3 pn, F3 p0, F3 p1, F3 p2, F3 n0, F3 n1, F3 n2) {
    const float Det = p0.x * (p1.y * p2.z - p2.y * p1.z) - p1.x * (p0.y * p2.z - p2.y * p0.z) +
                      p2.x * (p0.y * p1.z - p1.y * p0.z);
    const float D0 = pn.x * (p1.y * p2.z - p2.y * p1.z) - p1.x * (pn.y * p2.z - p2.y * pn.z) +
                     p2.x * (pn.y * p1.z - p1.y * pn.z);
    const float D1 = p0.x * (pn.y * p2.z - p2.y * pn.z) - pn.x * (p0.y * p2.z - p2.y * p0.z) +
                     p2.x * (p0.y * pn.z - pn.y * p0.z);
    const float D2 = p0.x * (p1.y * pn.z - pn.y * p1.z) - p1.x * (p0.y * pn.z - pn.y * p0.z) +
                     pn.x * (p0.y * p1.z - p1.y * p0.z);
    const float l0 = D0 / Det, l1 = D1 / Det, l2 = D2 / Det;
    return (l0 * n0 + l1 * n1) + l2 * n2;
}

// volumeRender.cl:1732-1779
__device__ __forceinline__ float ggx_partial_geometry(float c, float alpha) {
    float cs = clampf(c * c, 0.0f, 1.0f);
    float tan2 = (1.0f - cs) / cs;
    return 2.0f / (1.0f + ::sqrtf(1.0f + alpha * alpha * tan2));
}
__device__ __forceinline__ float ggx_distribution(float c, float alpha) {
    float alpha2 = alpha * alpha;
    float nh = clampf(c * c, 0.0f, 1.0f);
    float den = nh * alpha2 + (1.0f - nh);
    return alpha2 / (3.14159274101257324219f * den * den);
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
    float Fc = f0 + (1.0f - f0) * p;
    F3 F = F3{Fc, Fc, Fc};
    F3 specK = ((G * D) * F * 0.25f) / (NV + 0.001f);
    F3 diffK = F3{clampf(1.0f - F.x, 0.0f, 1.0f), clampf(1.0f - F.y, 0.0f, 1.0f), clampf(1.0f - F.z, 0.0f, 1.0f)};
    F3 m = ((albedo * diffK) * NL) / 3.14159274101257324219f + specK;
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
