/*
 * sbvh_oracle.c -- CPU restatement of the reference's spatial-split BVH builder.
 *
 * TEST INFRASTRUCTURE ONLY (same rule as rt_oracle.c): only tests/ may load
 * it, as the checker of the product builder (csrc/host/sbvh_builder.cpp).
 *
 * Parity status: the reference builder cannot be compiled here (Mesh.h pulls
 * in ColladaLoader.h -> pugixml.hpp, absent from the image, and
 * SplitBVHBuilder.cpp:5 includes "sort.h" which only resolves on a
 * case-insensitive file system), so this restatement is pinned by the survey's
 * probe of the real builder on data/models/cubes2.obj (14,933
 * nodes, 23,836 tri refs) plus hand-checked invariants, not by byte dumps.
 *
 * What it restates, step for step (reference file:line):
 *   SplitBVHBuilder::run              SplitBVHBuilder.cpp:41-81
 *   buildNode (degenerate removal, leaf tests, split choice, right child first)
 *                                     :107-176
 *   createLeaf (pops refs off the stack end)             :181-189
 *   findObjectSplit (3 sorted sweeps, tie-break)          :193-234
 *   performObjectSplit                                    :238-248
 *   findSpatialSplit (128 bins, reference chopping)       :252-331
 *   performSpatialSplit (unsplit / duplicate choice)      :335-427
 *   splitReference                                        :431-476
 *   sortCompare (centroid sum, then triIdx)               :85-94
 *   FW::sort = quicksort, median of 3, insertion < 16, 32-entry stack
 *                                                         Sort.cpp:25-148
 *   FW::AABB (grow / intersect / area / valid)            Util.h:10-33
 *   Platform (node cost 1, tri cost 1, batch 1), leaf 1..8  Platform.h:17, BVH2.cpp:13
 *   BVH_Cuda::build_from_bvh2 / build2 (pre-order, left first, refs x3,
 *   leaf offset = m_lo)                                   BVH_Cuda.h:87-137
 * Scalar helpers: fminf1/fmaxf1 are `a<b?a:b` / `a>b?a:b`, fsumf = (x+y)+z,
 * clamp(f,a,b) = fmaxf1(a, fminf1(f,b)), lerp = a*(1-t) + b*t
 * (vectors_math.cpp:121-262).  The reference is MSVC x64 (SSE2, /fp:precise):
 * plain IEEE binary32 in source order, no contraction; float->int is cvttss2si
 * (NaN / out of range -> INT_MIN).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define F32_MAX 3.402823466e+38f
#define MAX_DEPTH 64
#define MAX_SPATIAL_DEPTH 48
#define NBINS 128
#define MIN_LEAF 1
#define MAX_LEAF 8

typedef struct { float mn[3], mx[3]; } Box;
typedef struct { int32_t tri; Box b; } Ref;
typedef struct { int32_t num; Box b; } Spec;

static float fmin1(float a, float b) { return a < b ? a : b; }
static float fmax1(float a, float b) { return a > b ? a : b; }

static Box box_empty(void) {
    Box r;
    for (int k = 0; k < 3; ++k) { r.mn[k] = F32_MAX; r.mx[k] = -F32_MAX; }
    return r;
}
static void grow_pt(Box* b, const float p[3]) {
    for (int k = 0; k < 3; ++k) { b->mn[k] = fmin1(b->mn[k], p[k]); b->mx[k] = fmax1(b->mx[k], p[k]); }
}
/* Util.h: grow(AABB) grows by both corners, valid or not */
static void grow_box(Box* b, const Box* o) { grow_pt(b, o->mn); grow_pt(b, o->mx); }
static void intersect_box(Box* b, const Box* o) {
    for (int k = 0; k < 3; ++k) { b->mn[k] = fmax1(b->mn[k], o->mn[k]); b->mx[k] = fmin1(b->mx[k], o->mx[k]); }
}
static int box_valid(const Box* b) { return b->mn[0] <= b->mx[0] && b->mn[1] <= b->mx[1] && b->mn[2] <= b->mx[2]; }
static float box_area(const Box* b) {
    if (!box_valid(b)) return 0.0f;
    const float dx = b->mx[0] - b->mn[0], dy = b->mx[1] - b->mn[1], dz = b->mx[2] - b->mn[2];
    return (dx * dy + dy * dz + dz * dx) * 2.0f;
}
/* cvttss2si */
static int32_t f2i(float f) {
    if (!(f > -2147483904.0f && f < 2147483648.0f)) return INT32_MIN;
    return (int32_t)f;
}
static int32_t imin(int32_t a, int32_t b) { return a < b ? a : b; }
static int32_t imax(int32_t a, int32_t b) { return a > b ? a : b; }

/* ---- growable arrays ---- */
typedef struct { Ref* a; int64_t n, cap; } RefVec;
static void rv_push(RefVec* v, Ref r) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 1024;
        v->a = (Ref*)realloc(v->a, (size_t)v->cap * sizeof(Ref));
    }
    v->a[v->n++] = r;
}
typedef struct { int32_t* a; int64_t n, cap; } IntVec;
static void iv_push(IntVec* v, int32_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 1024;
        v->a = (int32_t*)realloc(v->a, (size_t)v->cap * sizeof(int32_t));
    }
    v->a[v->n++] = x;
}

/* tree nodes (BVHNode.h: InnerNode children[0]=left, [1]=right; LeafNode lo/hi) */
typedef struct { Box b; int32_t left, right, lo, hi; } TNode;
typedef struct { TNode* a; int64_t n, cap; } NodeVec;
static int32_t nv_push(NodeVec* v, TNode t) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 1024;
        v->a = (TNode*)realloc(v->a, (size_t)v->cap * sizeof(TNode));
    }
    v->a[v->n] = t;
    return (int32_t)v->n++;
}

typedef struct {
    const float* verts;   /* float4 per vertex */
    const int32_t* idx;   /* 3 per triangle */
    RefVec refs;          /* m_refStack */
    Box* right_bounds;    /* m_rightBounds */
    int sort_dim;
    float min_overlap;
    struct { Box b; int32_t enter, exit; } bins[3][NBINS];
    IntVec tris;          /* m_triIndices */
    NodeVec nodes;
} Builder;

/* ---- FW::sort over refs[start, end) with sortCompare / sortSwap ---- */
static int cmp_ref(const Builder* B, int64_t ia, int64_t ib) {
    const Ref* ra = &B->refs.a[ia];
    const Ref* rb = &B->refs.a[ib];
    const int d = B->sort_dim;
    const float ca = ra->b.mn[d] + ra->b.mx[d];
    const float cb = rb->b.mn[d] + rb->b.mx[d];
    return ca < cb || (ca == cb && ra->tri < rb->tri);
}
static void swap_ref(Builder* B, int64_t i, int64_t j) {
    Ref t = B->refs.a[i];
    B->refs.a[i] = B->refs.a[j];
    B->refs.a[j] = t;
}
static void insertion(Builder* B, int64_t start, int64_t size) {
    for (int64_t i = 1; i < size; ++i) {
        int64_t j = start + i - 1;
        while (j >= start && cmp_ref(B, j + 1, j)) {
            swap_ref(B, j, j + 1);
            --j;
        }
    }
}
static int64_t median3(Builder* B, int64_t low, int64_t high) {
    int64_t l = low, c = (low + high) >> 1, h = high - 2;
    if (cmp_ref(B, h, l)) { int64_t t = l; l = h; h = t; }
    if (cmp_ref(B, c, l)) c = l;
    return cmp_ref(B, h, c) ? h : c;
}
static int64_t partition(Builder* B, int64_t low, int64_t high) {
    swap_ref(B, median3(B, low, high), high - 1);
    int64_t i = low - 1, j = high - 1;
    for (;;) {
        do ++i; while (cmp_ref(B, i, high - 1));
        do --j; while (cmp_ref(B, high - 1, j));
        if (i >= j) break;
        swap_ref(B, i, j);
    }
    swap_ref(B, i, high - 1);
    return i;
}
static void fw_sort(Builder* B, int64_t low, int64_t high) {
    if (high - low < 2) return;
    int64_t stack[32];
    int sp = 0;
    stack[sp++] = high;
    while (sp) {
        high = stack[--sp];
        if (high - low < 16 || sp + 2 > 32) {
            insertion(B, low, high - low);
            low = high + 1;
            continue;
        }
        const int64_t i = partition(B, low, high);
        if (high - i > 2) stack[sp++] = high;
        if (i - low > 1) stack[sp++] = i;
        else low = i + 1;
    }
}

/* ---- splitReference (:431-476) ---- */
static void split_ref(const Builder* B, Ref* left, Ref* right, const Ref* ref, int dim, float pos) {
    left->tri = right->tri = ref->tri;
    left->b = box_empty();
    right->b = box_empty();
    const int32_t* ind = B->idx + 3 * (int64_t)ref->tri;
    const float* v1 = B->verts + 4 * (int64_t)ind[2];
    for (int i = 0; i < 3; ++i) {
        const float* v0 = v1;
        v1 = B->verts + 4 * (int64_t)ind[i];
        const float v0p = v0[dim], v1p = v1[dim];
        if (v0p <= pos) grow_pt(&left->b, v0);
        if (v0p >= pos) grow_pt(&right->b, v0);
        if ((v0p < pos && v1p > pos) || (v0p > pos && v1p < pos)) {
            const float q = (pos - v0p) / (v1p - v0p);
            const float t = fmax1(0.0f, fmin1(q, 1.0f));
            const float s = 1.0f - t;
            float p[3];
            for (int k = 0; k < 3; ++k) p[k] = v0[k] * s + v1[k] * t;
            grow_pt(&left->b, p);
            grow_pt(&right->b, p);
        }
    }
    left->b.mx[dim] = pos;
    right->b.mn[dim] = pos;
    intersect_box(&left->b, &ref->b);
    intersect_box(&right->b, &ref->b);
}

typedef struct { float sah; int dim; int32_t num_left; Box lb, rb; } ObjSplit;
typedef struct { float sah; int dim; float pos; } SpaSplit;

static ObjSplit find_object_split(Builder* B, const Spec* spec, float node_sah) {
    ObjSplit s;
    s.sah = F32_MAX; s.dim = 0; s.num_left = 0; s.lb = box_empty(); s.rb = box_empty();
    const int64_t base = B->refs.n - spec->num;
    float best_tie = F32_MAX;
    for (B->sort_dim = 0; B->sort_dim < 3; B->sort_dim++) {
        fw_sort(B, base, B->refs.n);
        const Ref* r = B->refs.a + base;
        Box rb = box_empty();
        for (int32_t i = spec->num - 1; i > 0; --i) {
            grow_box(&rb, &r[i].b);
            B->right_bounds[i - 1] = rb;
        }
        Box lb = box_empty();
        for (int32_t i = 1; i < spec->num; ++i) {
            grow_box(&lb, &r[i - 1].b);
            const float sah = node_sah + box_area(&lb) * (float)i + box_area(&B->right_bounds[i - 1]) * (float)(spec->num - i);
            const float fi = (float)i, fr = (float)(spec->num - i);
            const float tie = fi * fi + fr * fr;
            if (sah < s.sah || (sah == s.sah && tie < best_tie)) {
                s.sah = sah;
                s.dim = B->sort_dim;
                s.num_left = i;
                s.lb = lb;
                s.rb = B->right_bounds[i - 1];
                best_tie = tie;
            }
        }
    }
    return s;
}

static void perform_object_split(Builder* B, Spec* left, Spec* right, const Spec* spec, const ObjSplit* s) {
    B->sort_dim = s->dim;
    fw_sort(B, B->refs.n - spec->num, B->refs.n);
    left->num = s->num_left;
    left->b = s->lb;
    right->num = spec->num - s->num_left;
    right->b = s->rb;
}

static SpaSplit find_spatial_split(Builder* B, const Spec* spec, float node_sah) {
    float origin[3], bin_size[3], inv[3];
    for (int k = 0; k < 3; ++k) {
        origin[k] = spec->b.mn[k];
        bin_size[k] = (spec->b.mx[k] - origin[k]) * (1.0f / (float)NBINS);
        inv[k] = 1.0f / bin_size[k];
    }
    for (int d = 0; d < 3; ++d)
        for (int i = 0; i < NBINS; ++i) {
            B->bins[d][i].b = box_empty();
            B->bins[d][i].enter = 0;
            B->bins[d][i].exit = 0;
        }
    for (int64_t ri = B->refs.n - spec->num; ri < B->refs.n; ++ri) {
        const Ref ref = B->refs.a[ri];
        int32_t first[3], last[3];
        for (int k = 0; k < 3; ++k) {
            first[k] = imax(imin(f2i((ref.b.mn[k] - origin[k]) * inv[k]), NBINS - 1), 0);
            last[k] = imax(imin(f2i((ref.b.mx[k] - origin[k]) * inv[k]), NBINS - 1), first[k]);
        }
        for (int d = 0; d < 3; ++d) {
            Ref cur = ref;
            for (int32_t i = first[d]; i < last[d]; ++i) {
                Ref l, r;
                split_ref(B, &l, &r, &cur, d, origin[d] + bin_size[d] * (float)(i + 1));
                grow_box(&B->bins[d][i].b, &l.b);
                cur = r;
            }
            grow_box(&B->bins[d][last[d]].b, &cur.b);
            B->bins[d][first[d]].enter++;
            B->bins[d][last[d]].exit++;
        }
    }
    SpaSplit s;
    s.sah = F32_MAX; s.dim = 0; s.pos = 0.0f;
    for (int d = 0; d < 3; ++d) {
        Box rb = box_empty();
        for (int i = NBINS - 1; i > 0; --i) {
            grow_box(&rb, &B->bins[d][i].b);
            B->right_bounds[i - 1] = rb;
        }
        Box lb = box_empty();
        int32_t ln = 0, rn = spec->num;
        for (int i = 1; i < NBINS; ++i) {
            grow_box(&lb, &B->bins[d][i - 1].b);
            ln += B->bins[d][i - 1].enter;
            rn -= B->bins[d][i - 1].exit;
            const float sah = node_sah + box_area(&lb) * (float)ln + box_area(&B->right_bounds[i - 1]) * (float)rn;
            if (sah < s.sah) {
                s.sah = sah;
                s.dim = d;
                s.pos = origin[d] + bin_size[d] * (float)i;
            }
        }
    }
    return s;
}

static void perform_spatial_split(Builder* B, Spec* left, Spec* right, const Spec* spec, const SpaSplit* s) {
    const int64_t left_start = B->refs.n - spec->num;
    int64_t left_end = left_start, right_start = B->refs.n;
    left->b = box_empty();
    right->b = box_empty();
    const int d = s->dim;
    const float pos = s->pos;
    for (int64_t i = left_end; i < right_start; ++i) {
        if (B->refs.a[i].b.mx[d] <= pos) {
            grow_box(&left->b, &B->refs.a[i].b);
            swap_ref(B, i, left_end++);
        } else if (B->refs.a[i].b.mn[d] >= pos) {
            grow_box(&right->b, &B->refs.a[i].b);
            swap_ref(B, i, --right_start);
            --i;
        }
    }
    while (left_end < right_start) {
        Ref lref, rref;
        split_ref(B, &lref, &rref, &B->refs.a[left_end], d, pos);
        Box lub = left->b, rub = right->b, ldb = left->b, rdb = right->b;
        grow_box(&lub, &B->refs.a[left_end].b);
        grow_box(&rub, &B->refs.a[left_end].b);
        grow_box(&ldb, &lref.b);
        grow_box(&rdb, &rref.b);
        const float lac = (float)(left_end - left_start);
        const float rac = (float)(B->refs.n - right_start);
        const float lbc = (float)(left_end - left_start + 1);
        const float rbc = (float)(B->refs.n - right_start + 1);
        const float unsplit_left = box_area(&lub) * lbc + box_area(&right->b) * rac;
        const float unsplit_right = box_area(&left->b) * lac + box_area(&rub) * rbc;
        const float duplicate = box_area(&ldb) * lbc + box_area(&rdb) * rbc;
        const float m = fmin1(fmin1(unsplit_left, unsplit_right), duplicate);
        if (m == unsplit_left) {
            left->b = lub;
            left_end++;
        } else if (m == unsplit_right) {
            right->b = rub;
            swap_ref(B, left_end, --right_start);
        } else {
            left->b = ldb;
            right->b = rdb;
            B->refs.a[left_end++] = lref;
            rv_push(&B->refs, rref);
        }
    }
    left->num = (int32_t)(left_end - left_start);
    right->num = (int32_t)(B->refs.n - right_start);
}

static int32_t create_leaf(Builder* B, const Spec* spec) {
    for (int32_t i = 0; i < spec->num; ++i) {
        iv_push(&B->tris, B->refs.a[B->refs.n - 1].tri);
        B->refs.n--;
    }
    TNode t;
    t.b = spec->b;
    t.left = t.right = -1;
    t.lo = (int32_t)B->tris.n - spec->num;
    t.hi = (int32_t)B->tris.n;
    return nv_push(&B->nodes, t);
}

static int32_t build_node(Builder* B, Spec spec, int level) {
    {   /* remove degenerates (:120-132) */
        const int64_t first = B->refs.n - spec.num;
        for (int64_t i = B->refs.n - 1; i >= first; --i) {
            const Box* b = &B->refs.a[i].b;
            const float sx = b->mx[0] - b->mn[0], sy = b->mx[1] - b->mn[1], sz = b->mx[2] - b->mn[2];
            const float mn = fmin1(fmin1(sx, sy), sz), mx = fmax1(fmax1(sx, sy), sz);
            if (mn < 0.0f || (sx + sy) + sz == mx) {
                B->refs.a[i] = B->refs.a[B->refs.n - 1];
                B->refs.n--;
            }
        }
        spec.num = (int32_t)(B->refs.n - first);
    }
    if (spec.num <= MIN_LEAF || level >= MAX_DEPTH) return create_leaf(B, &spec);

    const float area = box_area(&spec.b);
    const float leaf_sah = area * (float)spec.num;
    const float node_sah = area * 2.0f;
    const ObjSplit obj = find_object_split(B, &spec, node_sah);
    SpaSplit spa;
    spa.sah = F32_MAX; spa.dim = 0; spa.pos = 0.0f;
    if (level < MAX_SPATIAL_DEPTH) {
        Box ov = obj.lb;
        intersect_box(&ov, &obj.rb);
        if (box_area(&ov) >= B->min_overlap) spa = find_spatial_split(B, &spec, node_sah);
    }
    const float min_sah = fmin1(fmin1(leaf_sah, obj.sah), spa.sah);
    if (min_sah == leaf_sah && spec.num <= MAX_LEAF) return create_leaf(B, &spec);

    Spec left, right;
    left.num = right.num = 0;
    left.b = right.b = box_empty();
    if (min_sah == spa.sah) perform_spatial_split(B, &left, &right, &spec, &spa);
    if (!left.num || !right.num) perform_object_split(B, &left, &right, &spec, &obj);

    const int32_t rn = build_node(B, right, level + 1);
    const int32_t ln = build_node(B, left, level + 1);
    TNode t;
    t.b = spec.b;
    t.left = ln;
    t.right = rn;
    t.lo = t.hi = 0;
    return nv_push(&B->nodes, t);
}

/* BVH_Cuda::build2 (:98-137): pre-order, left child first */
typedef struct { float mn[4], mx[4]; int32_t ol, orr, ot, nt; } OutNode; /* == rt_bvh_node */
static int32_t flatten(const Builder* B, int32_t n, OutNode* out, int32_t* counter) {
    const int32_t me = (*counter);
    const TNode* t = &B->nodes.a[n];
    OutNode o;
    for (int k = 0; k < 3; ++k) { o.mn[k] = t->b.mn[k]; o.mx[k] = t->b.mx[k]; }
    o.mn[3] = o.mx[3] = 1.0f;
    o.ol = o.orr = o.ot = -1;
    o.nt = 0;
    if (t->left >= 0) {
        ++(*counter);
        o.ol = flatten(B, t->left, out, counter);
        ++(*counter);
        o.orr = flatten(B, t->right, out, counter);
    } else {
        o.ot = t->lo;
        o.nt = t->hi - t->lo;
    }
    out[me] = o;
    return me;
}

/* Builds the SBVH of (verts: nv float4, idx: 3*ntri).  Outputs malloc'ed
 * BVH_Node_ array (48 B each) and tri_indices (x3); free with sbvh_oracle_free. */
int sbvh_oracle_build(const float* verts, int32_t nv, const int32_t* idx, int32_t ntri, void** nodes_out,
                      int32_t* num_nodes, int32_t** refs_out, int32_t* num_refs) {
    (void)nv;
    Builder* B = (Builder*)calloc(1, sizeof(Builder));
    if (!B) return -1;
    B->verts = verts;
    B->idx = idx;
    Spec root;
    root.num = ntri;
    root.b = box_empty();
    for (int32_t i = 0; i < ntri; ++i) {
        Ref r;
        r.tri = i;
        r.b = box_empty();
        for (int j = 0; j < 3; ++j) grow_pt(&r.b, verts + 4 * (int64_t)idx[3 * i + j]);
        grow_box(&root.b, &r.b);
        rv_push(&B->refs, r);
    }
    B->min_overlap = box_area(&root.b) * 1.0e-5f;
    const int32_t nrb = (ntri > NBINS ? ntri : NBINS) - 1;
    B->right_bounds = (Box*)malloc((size_t)nrb * sizeof(Box));
    const int32_t rootn = build_node(B, root, 0);

    OutNode* out = (OutNode*)malloc((size_t)(B->nodes.n > 0 ? B->nodes.n : 1) * sizeof(OutNode));
    int32_t counter = 0;
    flatten(B, rootn, out, &counter);
    int32_t* refs = (int32_t*)malloc((size_t)(B->tris.n > 0 ? B->tris.n : 1) * sizeof(int32_t));
    for (int64_t i = 0; i < B->tris.n; ++i) refs[i] = B->tris.a[i] * 3;
    *nodes_out = out;
    *num_nodes = (int32_t)B->nodes.n;
    *refs_out = refs;
    *num_refs = (int32_t)B->tris.n;
    free(B->refs.a);
    free(B->right_bounds);
    free(B->tris.a);
    free(B->nodes.a);
    free(B);
    return 0;
}

void sbvh_oracle_free(void* p) { free(p); }
