/*
 * rt_oracle.c -- CPU restatement of the reference render path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the CPU baseline.  The product (librtamd.so) never
 * links or calls it.
 *
 * What it restates (all citations into the reference tree,
 * x64/Release/volumeRender.cl unless stated):
 *   raytracer_bvh        :1043-1547  per-pixel pipeline
 *   traverse_bvh         :658-1010   stack traversal, 65-entry stack
 *   ray_box              :612-624    slab test by IEEE division
 *   RayBoxIntersection   :236-254    scene-box early-out (inv_dir)
 *   RayTriangleIntersection :257-282 Moller-Trumbore
 *   RayInit              :205-211    normalize + (double)1.0/dir
 *   get_normal_at_tri_point :27-53   Cramer barycentrics
 *   rgbToInt             :186-195    BGR pack, clamp, truncate
 *   GGX_PartialGeometry / GGX_Distribution / FresnelSchlick /
 *   CookTorrance_GGX     :1732-1779
 *   reflect              :25
 *
 * Floating-point semantics ("S_strict"):
 *   - kernel-code arithmetic is IEEE binary32, evaluated in source order,
 *     no contraction (built with -ffp-contract=off); '/' and sqrt are
 *     correctly rounded; double literals are evaluated in binary64 exactly
 *     as the OpenCL C source types them (e.g. (x-0.5)/(float)w, 1.0/dir);
 *   - OpenCL builtins follow ROCm 7.2 device-libs (opencl.bc), the library
 *     the reference kernel links when built for gfx950:
 *       dot(a,b)   = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
 *       cross(a,b) = (fma(a.y,b.z, b.y*-a.z), fma(a.z,b.x, b.z*-a.x),
 *                     fma(a.x,b.y, b.x*-a.y))
 *       normalize  = zero test, FLT_MIN / INF rescaling, p * rsqrt(dot(p,p))
 *       fmin/fmax/max = IEEE minNum/maxNum; clamp = med3
 *     with two substitutions that make the semantics exactly reproducible on
 *     any IEEE host (the device library uses hardware approximations):
 *       rsqrt(x)  := (float)(1.0 / sqrt((double)x))        [v_rsq_f32 is ~1 ulp]
 *       pow(x,5)  := (float)((((x*x)*x)*x)*x in binary64)  [ocml powf is ~1 ulp]
 *   The residual difference against the real reference kernel is measured,
 *   not assumed: tests/golden holds the reference kernel's own output
 *   (oracle/_ref, run on MI355X) and tests/test_oracle_golden.py reports it.
 *
 * Deliberate divergences from the reference kernel (documented):
 *   - threads outside the w x h frame do nothing (the reference's padded
 *     8x8 NDRange lets x >= w threads alias into the next row, :1164).
 */
#include <math.h>
#include <float.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>

typedef struct { float x, y, z, w; } of4;
typedef struct { of4 min, max; int32_t l, r, off, cnt; } onode;      /* BVH_Cuda.h:12-29, 48 B */
typedef struct { int32_t technique[4]; of4 emission, ambient, diffuse, specular, shininess,
                 reflective, reflectivity, transparent, transparency, glossiness; } omat;  /* Mesh.h:20-67, 176 B */
typedef struct { of4 a, b, c, campos, light_pos, light_color, smin, smax; } oparams;    /* RayTracer.cpp:115-161, 128 B */

typedef char o_static_node[(sizeof(onode) == 48) ? 1 : -1];
typedef char o_static_mat[(sizeof(omat) == 176) ? 1 : -1];
typedef char o_static_par[(sizeof(oparams) == 128) ? 1 : -1];

typedef struct {
    /* traversal work counters, summed over traced rays */
    uint64_t rays[3];        /* 0 = primary (closest), 1 = shadow (any), 2 = secondary (closest) */
    uint64_t inner[3];
    uint64_t leaf[3];
    uint64_t tris[3];
    uint64_t max_stack;
    uint64_t stack_overflow;
} ostats;

typedef struct { float x, y, z; } f3;

#define O_STACK_SIZE 65            /* volumeRender.cl:636 */
#define O_TMIN 0.001f              /* volumeRender.cl:640 */
#define O_M_PI_F 3.14159274101257324219f

static inline f3 v3(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 x3(of4 a) { return v3(a.x, a.y, a.z); }
static inline f3 add3(f3 a, f3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 sub3(f3 a, f3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 mul3(f3 a, f3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline f3 muls(f3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline f3 smul(float s, f3 a) { return v3(s * a.x, s * a.y, s * a.z); }
static inline f3 divs(f3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }

/* device-libs opencl.bc _Z3dotDv3_fS_ */
static inline float o_dot(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
/* device-libs opencl.bc _Z5crossDv3_fS_ */
static inline f3 o_cross(f3 a, f3 b) {
    return v3(fmaf(a.y, b.z, b.y * -a.z), fmaf(a.z, b.x, b.z * -a.x), fmaf(a.x, b.y, b.x * -a.y));
}
static inline float o_rsqrt(float x) { return (float)(1.0 / sqrt((double)x)); }
/* device-libs opencl.bc _Z9normalizeDv3_f */
static f3 o_normalize(f3 p) {
    if (p.x == 0.0f && p.y == 0.0f && p.z == 0.0f) return p;
    float l2 = o_dot(p, p);
    if (l2 < FLT_MIN) {
        p = muls(p, 0x1p86f);
        l2 = o_dot(p, p);
    } else if (l2 == INFINITY) {
        p = muls(p, 0x1p-66f);
        l2 = o_dot(p, p);
        if (l2 == INFINITY) {
            p = v3(copysignf(isinf(p.x) ? 1.0f : 0.0f, p.x), copysignf(isinf(p.y) ? 1.0f : 0.0f, p.y),
                   copysignf(isinf(p.z) ? 1.0f : 0.0f, p.z));
            l2 = o_dot(p, p);
        }
    }
    return muls(p, o_rsqrt(l2));
}
static inline float o_clamp(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
static inline float o_pow5(float x) {
    double d = (double)x;
    return (float)((((d * d) * d) * d) * d);
}

/* volumeRender.cl:25 */
static inline f3 o_reflect(f3 i, f3 n) { return sub3(i, muls(smul(2.0f, n), o_dot(n, i))); }

typedef struct { f3 ori, dir, inv_dir; } oray;

/* volumeRender.cl:205-211 */
static void o_ray_init(oray* r, f3 o, f3 d) {
    r->ori = o;
    r->dir = o_normalize(d);
    r->inv_dir = v3((float)(1.0 / (double)r->dir.x), (float)(1.0 / (double)r->dir.y),
                    (float)(1.0 / (double)r->dir.z));
}

/* volumeRender.cl:236-254 */
static int o_ray_box_scene(f3 bmin, f3 bmax, f3 org, f3 inv, float* tmin, float* tmax) {
    float l1 = (bmin.x - org.x) * inv.x;
    float l2 = (bmax.x - org.x) * inv.x;
    *tmin = fminf(l1, l2);
    *tmax = fmaxf(l1, l2);
    l1 = (bmin.y - org.y) * inv.y;
    l2 = (bmax.y - org.y) * inv.y;
    *tmin = fmaxf(fminf(l1, l2), *tmin);
    *tmax = fminf(fmaxf(l1, l2), *tmax);
    l1 = (bmin.z - org.z) * inv.z;
    l2 = (bmax.z - org.z) * inv.z;
    *tmin = fmaxf(fminf(l1, l2), *tmin);
    *tmax = fminf(fmaxf(l1, l2), *tmax);
    return (*tmax >= *tmin) && (*tmax >= 0.0f);
}

/* volumeRender.cl:257-282 */
static float o_ray_tri(const oray* r, f3 v0, f3 e1, f3 e2) {
    f3 tvec = sub3(r->ori, v0);
    f3 pvec = o_cross(r->dir, e2);
    float det = o_dot(e1, pvec);
    det = 1.0f / det;
    float u = o_dot(tvec, pvec) * det;
    if (u < 0.0f || u > 1.0f) return -1.0f;
    f3 qvec = o_cross(tvec, e1);
    float v = o_dot(r->dir, qvec) * det;
    if (v < 0.0f || (u + v) > 1.0f) return -1.0f;
    return o_dot(e2, qvec) * det;
}

/* volumeRender.cl:612-624 */
static inline void o_ray_box(const oray* r, of4 mn, of4 mx, float* tn, float* tf) {
    f3 t0 = v3((mn.x - r->ori.x) / r->dir.x, (mn.y - r->ori.y) / r->dir.y, (mn.z - r->ori.z) / r->dir.z);
    f3 t1 = v3((mx.x - r->ori.x) / r->dir.x, (mx.y - r->ori.y) / r->dir.y, (mx.z - r->ori.z) / r->dir.z);
    f3 lo = v3(fminf(t0.x, t1.x), fminf(t0.y, t1.y), fminf(t0.z, t1.z));
    f3 hi = v3(fmaxf(t0.x, t1.x), fmaxf(t0.y, t1.y), fmaxf(t0.z, t1.z));
    *tn = fmaxf(fmaxf(lo.x, lo.y), lo.z);
    *tf = fminf(fminf(hi.x, hi.y), hi.z);
}

typedef struct {
    const of4* verts;
    const int32_t* idx;
    const onode* nodes;
    int32_t num_nodes;
    const int32_t* refs;
    int32_t num_refs;
    const of4* normals;
    const int32_t* nidx;
    const omat* mats;
    const int32_t* tri2mat;
} oscene;

typedef struct { uint64_t inner, leaf, tris, max_stack, overflow; } tcount;

/* volumeRender.cl:658-1010 (live code only: :776-1009) */
static int o_traverse(const oscene* s, const oray* ray, float* tHit, int closest, tcount* c) {
    int stack[O_STACK_SIZE];
    int stack_count = 1;
    stack[0] = 0;
    int tri_index = -1;
    while (stack_count > 0) {
        if ((uint64_t)stack_count > c->max_stack) c->max_stack = (uint64_t)stack_count;
        int nodeIndex = stack[stack_count - 1];
        const onode* nd = &s->nodes[nodeIndex];
        int offset_left = nd->l;
        if (offset_left >= 0) {
            int offset_right = nd->r;
            c->inner++;
            if (offset_right < 0) return -1;
            if (offset_left >= s->num_nodes) return -1;
            if (offset_right >= s->num_nodes) return -1;
            float n0, f0, n1, f1;
            o_ray_box(ray, s->nodes[offset_left].min, s->nodes[offset_left].max, &n0, &f0);
            o_ray_box(ray, s->nodes[offset_right].min, s->nodes[offset_right].max, &n1, &f1);
            int i0 = (n0 <= f0) && (f0 >= O_TMIN) && (n0 <= *tHit);
            int i1 = (n1 <= f1) && (f1 >= O_TMIN) && (n1 <= *tHit);
            if (i0 && i1) {
                if (n0 > n1) { int t = offset_left; offset_left = offset_right; offset_right = t; }
                stack[stack_count - 1] = offset_right;
                if (stack_count >= O_STACK_SIZE) { c->overflow++; return -1; }
                stack[stack_count] = offset_left;
                ++stack_count;
            } else if (i0) {
                stack[stack_count - 1] = offset_left;
            } else if (i1) {
                stack[stack_count - 1] = offset_right;
            } else {
                --stack_count;
            }
        } else {
            c->leaf++;
            int off = nd->off, cnt = nd->cnt;
            for (int i = 0; i < cnt; ++i) {
                int tri1 = s->refs[off + i];
                of4 a = s->verts[s->idx[tri1 + 0]];
                of4 b = s->verts[s->idx[tri1 + 1]];
                of4 d = s->verts[s->idx[tri1 + 2]];
                f3 v0 = x3(a);
                f3 e1 = v3(b.x - a.x, b.y - a.y, b.z - a.z);
                f3 e2 = v3(d.x - a.x, d.y - a.y, d.z - a.z);
                c->tris++;
                float t = o_ray_tri(ray, v0, e1, e2);
                if (t < *tHit && t > O_TMIN) {
                    *tHit = t;
                    if (!closest) return tri1;
                    tri_index = tri1;
                }
            }
            --stack_count;
        }
    }
    return tri_index;
}

/* volumeRender.cl:27-53 */
static f3 o_normal_at(f3 pn, of4 p0, of4 p1, of4 p2, of4 n0, of4 n1, of4 n2) {
    const float Det = p0.x * (p1.y * p2.z - p2.y * p1.z) - p1.x * (p0.y * p2.z - p2.y * p0.z) +
                      p2.x * (p0.y * p1.z - p1.y * p0.z);
    const float D0 = pn.x * (p1.y * p2.z - p2.y * p1.z) - p1.x * (pn.y * p2.z - p2.y * pn.z) +
                     p2.x * (pn.y * p1.z - p1.y * pn.z);
    const float D1 = p0.x * (pn.y * p2.z - p2.y * pn.z) - pn.x * (p0.y * p2.z - p2.y * p0.z) +
                     p2.x * (p0.y * pn.z - pn.y * p0.z);
    const float D2 = p0.x * (p1.y * pn.z - pn.y * p1.z) - p1.x * (p0.y * pn.z - pn.y * p0.z) +
                     pn.x * (p0.y * p1.z - p1.y * p0.z);
    f3 l = v3(D0 / Det, D1 / Det, D2 / Det);
    return add3(add3(smul(l.x, x3(n0)), smul(l.y, x3(n1))), smul(l.z, x3(n2)));
}

/* volumeRender.cl:1732-1738 */
static float o_ggx_partial_geometry(float cosThetaN, float alpha) {
    float cs = o_clamp(cosThetaN * cosThetaN, 0.0f, 1.0f);
    float tan2 = (1.0f - cs) / cs;
    return 2.0f / (1.0f + sqrtf(1.0f + alpha * alpha * tan2));
}
/* volumeRender.cl:1740-1746 */
static float o_ggx_distribution(float cosThetaNH, float alpha) {
    float alpha2 = alpha * alpha;
    float nh = o_clamp(cosThetaNH * cosThetaNH, 0.0f, 1.0f);
    float den = nh * alpha2 + (1.0f - nh);
    return alpha2 / (O_M_PI_F * den * den);
}
/* volumeRender.cl:1748-1751 */
static f3 o_fresnel(f3 F0, float cosTheta) {
    float p = o_pow5(1.0f - o_clamp(cosTheta, 0.0f, 1.0f));
    return add3(F0, muls(v3(1.0f - F0.x, 1.0f - F0.y, 1.0f - F0.z), p));
}
/* volumeRender.cl:1754-1779 */
static f3 o_cook_torrance_ggx(f3 n, f3 l, f3 v, f3 albedo, f3 f0, float roughness) {
    n = o_normalize(n);
    v = o_normalize(v);
    l = o_normalize(l);
    f3 h = o_normalize(add3(v, l));
    float NL = o_dot(n, l);
    if (NL <= 0.0f) return v3(0, 0, 0);
    float NV = o_dot(n, v);
    if (NV <= 0.0f) return v3(0, 0, 0);
    float NH = o_dot(n, h);
    float HV = o_dot(h, v);
    float rs = roughness * roughness;
    float G = o_ggx_partial_geometry(NV, rs) * o_ggx_partial_geometry(NL, rs);
    float D = o_ggx_distribution(NH, rs);
    f3 F = o_fresnel(f0, HV);
    f3 specK = divs(muls(smul(G * D, F), 0.25f), NV + 0.001f);
    f3 diffK = v3(o_clamp(1.0f - F.x, 0.0f, 1.0f), o_clamp(1.0f - F.y, 0.0f, 1.0f),
                  o_clamp(1.0f - F.z, 0.0f, 1.0f));
    f3 m = add3(divs(muls(mul3(albedo, diffK), NL), O_M_PI_F), specK);
    return v3(fmaxf(0.0f, m.x), fmaxf(0.0f, m.y), fmaxf(0.0f, m.z));
}

/* volumeRender.cl:186-195 */
static uint32_t o_rgb_to_int(float r, float g, float b) {
    r = o_clamp(r, 0.0f, 255.0f);
    g = o_clamp(g, 0.0f, 255.0f);
    b = o_clamp(b, 0.0f, 255.0f);
    return ((uint32_t)b << 16) | ((uint32_t)g << 8) | (uint32_t)r;
}

#define OFLAG_NO_SHADOW 1u

typedef struct {
    const oscene* s;
    const oparams* p;
    uint32_t w, h;
    int depth;
    uint32_t flags;
    int64_t pix0, npix, stride;
    uint32_t* out;
    int32_t* hits;  /* [npix][depth][2] : closest hit, shadow hit (-2 = not traced) */
    float* tvals;   /* [npix][depth]    : closest-hit t (-1 = not traced) */
    float* rgb;     /* [npix][3]        : color before the x255 pack */
    ostats st;
    int64_t j0, j1;
} ojob;

static void o_pixel(ojob* jb, int64_t j) {
    const oscene* s = jb->s;
    const oparams* P = jb->p;
    int64_t pix = jb->pix0 + j * jb->stride;
    uint32_t x = (uint32_t)(pix % jb->w), y = (uint32_t)(pix / jb->w);
    const int depth = jb->depth;
    int32_t* hits = jb->hits ? jb->hits + j * depth * 2 : 0;
    float* tv = jb->tvals ? jb->tvals + j * depth : 0;
    for (int k = 0; k < depth; ++k) {
        if (hits) { hits[2 * k] = -2; hits[2 * k + 1] = -2; }
        if (tv) tv[k] = -1.0f;
    }
    f3 a = x3(P->a), b = x3(P->b), c = x3(P->c), campos = x3(P->campos);
    f3 light_pos = x3(P->light_pos);
    f3 smin = x3(P->smin), smax = x3(P->smax);

    /* volumeRender.cl:1169-1190 */
    float xf = (float)(((double)x - 0.5) / (double)(float)jb->w);
    float yf = (float)(((double)y - 0.5) / (double)(float)jb->h);
    int ray_depth = 0;
    f3 t1 = add3(c, muls(a, xf));
    f3 t2 = muls(b, yf);
    f3 image_pos = add3(t1, t2);
    oray r;
    o_ray_init(&r, image_pos, sub3(image_pos, campos));
    float tHit = (float)4294967295u; /* HitRecordInit: t = UINT_MAX */
    f3 color = v3(0, 0, 0);
    float tmin, tmax;
    int cont = o_ray_box_scene(smin, smax, r.ori, r.inv_dir, &tmin, &tmax);
    float shadow_sum = 0.0f;
    tcount cnt;
    while (cont && ray_depth < depth) {
        int kind = ray_depth == 0 ? 0 : 2;
        memset(&cnt, 0, sizeof cnt);
        int hit = o_traverse(s, &r, &tHit, 1, &cnt);
        jb->st.rays[kind]++;
        jb->st.inner[kind] += cnt.inner;
        jb->st.leaf[kind] += cnt.leaf;
        jb->st.tris[kind] += cnt.tris;
        if (cnt.max_stack > jb->st.max_stack) jb->st.max_stack = cnt.max_stack;
        jb->st.stack_overflow += cnt.overflow;
        if (hits) hits[2 * ray_depth] = hit;
        if (tv) tv[ray_depth] = tHit;
        float shadow_coef = 1.0f;
        if (hit >= 0) {
            int kk = ray_depth;
            ray_depth++;
            of4 p0 = s->verts[s->idx[hit + 0]], p1 = s->verts[s->idx[hit + 1]], p2 = s->verts[s->idx[hit + 2]];
            of4 n0 = s->normals[s->nidx[hit + 0]], n1 = s->normals[s->nidx[hit + 1]],
                n2 = s->normals[s->nidx[hit + 2]];
            f3 vNew = add3(r.ori, muls(r.dir, tHit - 0.001f));
            f3 normal = o_normalize(o_normal_at(vNew, p0, p1, p2, n0, n1, n2));
            f3 l1 = o_normalize(sub3(light_pos, vNew));
            f3 v = o_normalize(sub3(r.ori, vNew));
            f3 n = o_normalize(normal);
            const omat* mat = &s->mats[s->tri2mat[hit / 3]];
            f3 albedo = x3(mat->diffuse);
            float f0s = 40.0f * (1.0f / 255.0f);
            f3 rez = muls(o_cook_torrance_ggx(n, l1, v, albedo, v3(f0s, f0s, f0s), 0.5f), 3.0f);
            rez = add3(rez, mul3(v3(0.3f, 0.3f, 0.3f), albedo));
            f3 hitpoint = vNew;
            f3 L = o_normalize(sub3(light_pos, hitpoint));
            if (!(jb->flags & OFLAG_NO_SHADOW)) {
                oray sr;
                o_ray_init(&sr, add3(hitpoint, muls(L, 0.001f)), L);
                float ts = (float)4294967295u;
                memset(&cnt, 0, sizeof cnt);
                int sh = o_traverse(s, &sr, &ts, 0, &cnt);
                jb->st.rays[1]++;
                jb->st.inner[1] += cnt.inner;
                jb->st.leaf[1] += cnt.leaf;
                jb->st.tris[1] += cnt.tris;
                if (cnt.max_stack > jb->st.max_stack) jb->st.max_stack = cnt.max_stack;
                jb->st.stack_overflow += cnt.overflow;
                if (hits) hits[2 * kk + 1] = sh;
                if (sh >= 0 && ts > 0.025f) shadow_coef = 0.25f;
            }
            color = add3(color, rez);
            shadow_sum += shadow_coef;
            f3 refl = o_reflect(r.dir, normal);
            o_ray_init(&r, add3(hitpoint, muls(refl, 0.001f)), refl);
            tHit = (float)4294967295u;
        } else {
            cont = 0;
        }
    }
    if (ray_depth >= 1) {
        color = divs(color, (float)ray_depth);
        shadow_sum /= (float)ray_depth;
        color = muls(color, shadow_sum);
    } else {
        color = v3(0, 0, 0);
    }
    if (jb->rgb) { jb->rgb[3 * j] = color.x; jb->rgb[3 * j + 1] = color.y; jb->rgb[3 * j + 2] = color.z; }
    if (jb->out) jb->out[j] = o_rgb_to_int(color.x * 255.0f, color.y * 255.0f, color.z * 255.0f);
}

static void* o_worker(void* arg) {
    ojob* jb = (ojob*)arg;
    for (int64_t j = jb->j0; j < jb->j1; ++j) o_pixel(jb, j);
    return 0;
}

/*
 * Render npix pixels with linear indices pix0, pix0+stride, ... (y = idx / w).
 * Outputs are indexed by j in [0, npix).  Returns 0 on success.
 */
int oracle_render(const oparams* params, const of4* verts, const int32_t* idx, const onode* nodes,
                  int32_t num_nodes, const int32_t* refs, int32_t num_refs, const of4* normals,
                  const int32_t* nidx, const omat* mats, const int32_t* tri2mat, uint32_t w, uint32_t h,
                  int depth, uint32_t flags, int64_t pix0, int64_t npix, int64_t stride, uint32_t* out,
                  int32_t* hits, float* tvals, float* rgb, ostats* stats, int nthreads) {
    if (!params || !verts || !idx || !nodes || num_nodes < 1 || !refs || w == 0 || h == 0 || depth < 0 ||
        npix < 0 || stride < 1)
        return -1;
    oscene s = {verts, idx, nodes, num_nodes, refs, num_refs, normals, nidx, mats, tri2mat};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    ojob jobs[256];
    pthread_t th[256];
    int64_t per = (npix + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; ++t) {
        ojob* jb = &jobs[t];
        memset(jb, 0, sizeof *jb);
        jb->s = &s; jb->p = params; jb->w = w; jb->h = h; jb->depth = depth; jb->flags = flags;
        jb->pix0 = pix0; jb->npix = npix; jb->stride = stride;
        jb->out = out; jb->hits = hits; jb->tvals = tvals; jb->rgb = rgb;
        jb->j0 = t * per;
        jb->j1 = (t + 1) * per < npix ? (t + 1) * per : npix;
        if (jb->j0 > jb->j1) jb->j0 = jb->j1;
    }
    if (nthreads == 1) {
        o_worker(&jobs[0]);
    } else {
        for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], 0, o_worker, &jobs[t]);
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], 0);
    }
    if (stats) {
        memset(stats, 0, sizeof *stats);
        for (int t = 0; t < nthreads; ++t) {
            for (int k = 0; k < 3; ++k) {
                stats->rays[k] += jobs[t].st.rays[k];
                stats->inner[k] += jobs[t].st.inner[k];
                stats->leaf[k] += jobs[t].st.leaf[k];
                stats->tris[k] += jobs[t].st.tris[k];
            }
            if (jobs[t].st.max_stack > stats->max_stack) stats->max_stack = jobs[t].st.max_stack;
            stats->stack_overflow += jobs[t].st.stack_overflow;
        }
    }
    return 0;
}

/* ---- primitive probes (for unit tests of the restated helpers) ---- */
void oracle_normalize(const float* in, float* out) {
    f3 r = o_normalize(v3(in[0], in[1], in[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
float oracle_ray_tri(const float* ori, const float* dir, const float* v0, const float* e1, const float* e2) {
    oray r;
    r.ori = v3(ori[0], ori[1], ori[2]);
    r.dir = v3(dir[0], dir[1], dir[2]);
    return o_ray_tri(&r, v3(v0[0], v0[1], v0[2]), v3(e1[0], e1[1], e1[2]), v3(e2[0], e2[1], e2[2]));
}
uint32_t oracle_rgb_to_int(float r, float g, float b) { return o_rgb_to_int(r, g, b); }
