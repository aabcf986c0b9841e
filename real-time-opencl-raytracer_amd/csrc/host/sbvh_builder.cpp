// sbvh_builder.cpp -- the reference's spatial-split BVH (SplitBVHBuilder,
// SplitBVHBuilder.cpp:41-476, run through BVH_Cuda::build_from_bvh2,
// BVH_Cuda.h:87-137), rebuilt to produce the same BVH_Node_ / tri_indices
// bytes in a fraction of the time:
//
//  * Same decisions, same float arithmetic (IEEE binary32 in source order,
//    `a<b?a:b` min/max, cvttss2si float->int), same physical order of the
//    reference stack at every step that depends on order (degenerate removal,
//    leaf emission, performSpatialSplit's sequential unsplit/duplicate choice,
//    bounds growth order, which matters for +-0).
//  * Sorting: within one node's range a triangle appears at most once (a
//    duplicate's two halves always go to different children), so the
//    comparator (centroid sum, triIdx) is a strict total order and every
//    correct sort yields the same permutation as the reference's quicksort
//    (Sort.cpp:93-127).  Ranges are sorted with std::sort on 64-bit keys; a
//    range with a NaN key (non-finite input) falls back to the reference's
//    exact quicksort sequence.
//  * The reference builds right child, then left, on one shared stack; the
//    two ranges never touch, so subtrees are built in parallel and the leaf
//    emission order (right-first DFS, refs popped from the range end) is
//    reassembled afterwards.
// The oracle for this file is oracle/sbvh_oracle.c (a direct restatement).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <thread>

#include "scene.hpp"

namespace rtamd {
namespace {

constexpr float kF32Max = 3.402823466e+38f;   // FW_F32_MAX (Defs.h:26)
constexpr int kMaxDepth = 64;                 // SplitBVHBuilder.h:18-20
constexpr int kMaxSpatialDepth = 48;
constexpr int kBins = 128;
constexpr int kMinLeaf = 1, kMaxLeaf = 8;     // BVH2.cpp:13
constexpr float kSplitAlpha = 1.0e-5f;        // SplitBVHBuilder.cpp:19

inline float fmin1(float a, float b) { return a < b ? a : b; }
inline float fmax1(float a, float b) { return a > b ? a : b; }
inline int32_t cvtt(float f) { return (f > -2147483904.0f && f < 2147483648.0f) ? (int32_t)f : INT32_MIN; }

struct Box {  // FW::AABB (Util.h:10-33)
    float mn[3], mx[3];
    static Box empty() {
        Box b;
        for (int k = 0; k < 3; ++k) { b.mn[k] = kF32Max; b.mx[k] = -kF32Max; }
        return b;
    }
    void grow(const float* p) {
        for (int k = 0; k < 3; ++k) { mn[k] = fmin1(mn[k], p[k]); mx[k] = fmax1(mx[k], p[k]); }
    }
    void grow(const Box& o) { grow(o.mn); grow(o.mx); }
    void intersect(const Box& o) {
        for (int k = 0; k < 3; ++k) { mn[k] = fmax1(mn[k], o.mn[k]); mx[k] = fmin1(mx[k], o.mx[k]); }
    }
    bool valid() const { return mn[0] <= mx[0] && mn[1] <= mx[1] && mn[2] <= mx[2]; }
    float area() const {
        if (!valid()) return 0.0f;
        const float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        return (dx * dy + dy * dz + dz * dx) * 2.0f;
    }
};

struct Ref {
    int32_t tri;
    Box b;
};

struct Node {  // InnerNode / LeafNode (BVHNode.h)
    Box b;
    std::unique_ptr<Node> kid[2];   // [0] left, [1] right
    std::vector<int32_t> tris;      // leaf: triIdx in emission order (popped off the range end)
    int32_t lo = 0, cnt = 0;        // leaf: LeafNode m_lo, m_hi - m_lo
    bool leaf = false;
};

struct Shared {
    const float* verts;             // float4 per vertex
    const int32_t* idx;
    float min_overlap;
    int max_threads;
    std::atomic<int> threads{0};
    std::atomic<int> max_level{0};
};

// splitReference (SplitBVHBuilder.cpp:431-476)
void split_ref(const Shared& S, Ref& l, Ref& r, const Ref& ref, int dim, float pos) {
    l.tri = r.tri = ref.tri;
    l.b = r.b = Box::empty();
    const int32_t* ind = S.idx + 3 * (int64_t)ref.tri;
    const float* v1 = S.verts + 4 * (int64_t)ind[2];
    for (int i = 0; i < 3; ++i) {
        const float* v0 = v1;
        v1 = S.verts + 4 * (int64_t)ind[i];
        const float v0p = v0[dim], v1p = v1[dim];
        if (v0p <= pos) l.b.grow(v0);
        if (v0p >= pos) r.b.grow(v0);
        if ((v0p < pos && v1p > pos) || (v0p > pos && v1p < pos)) {
            const float t = fmax1(0.0f, fmin1((pos - v0p) / (v1p - v0p), 1.0f));
            const float s = 1.0f - t;
            const float p[3] = {v0[0] * s + v1[0] * t, v0[1] * s + v1[1] * t, v0[2] * s + v1[2] * t};
            l.b.grow(p);
            r.b.grow(p);
        }
    }
    l.b.mx[dim] = pos;
    r.b.mn[dim] = pos;
    l.b.intersect(ref.b);
    r.b.intersect(ref.b);
}

inline bool ref_less(const Ref& a, const Ref& b, int d) {  // sortCompare (:85-94)
    const float ca = a.b.mn[d] + a.b.mx[d], cb = b.b.mn[d] + b.b.mx[d];
    return ca < cb || (ca == cb && a.tri < b.tri);
}

// FW::sort (Sort.cpp:25-148) on a whole vector: exact reference behaviour for
// comparators that are not a strict weak order (NaN centroids).
void fw_sort(std::vector<Ref>& v, int d) {
    const int64_t n = (int64_t)v.size();
    if (n < 2) return;
    auto cmp = [&](int64_t i, int64_t j) { return ref_less(v[i], v[j], d); };
    auto insertion = [&](int64_t start, int64_t size) {
        for (int64_t i = 1; i < size; ++i)
            for (int64_t j = start + i - 1; j >= start && cmp(j + 1, j); --j) std::swap(v[j], v[j + 1]);
    };
    int64_t stack[32];
    int sp = 0;
    int64_t low = 0, high;
    stack[sp++] = n;
    while (sp) {
        high = stack[--sp];
        if (high - low < 16 || sp + 2 > 32) {
            insertion(low, high - low);
            low = high + 1;
            continue;
        }
        int64_t l = low, c = (low + high) >> 1, h = high - 2;  // median3
        if (cmp(h, l)) std::swap(l, h);
        if (cmp(c, l)) c = l;
        std::swap(v[cmp(h, c) ? h : c], v[high - 1]);
        int64_t i = low - 1, j = high - 1;  // partition
        for (;;) {
            do ++i; while (cmp(i, high - 1));
            do --j; while (cmp(high - 1, j));
            if (i >= j) break;
            std::swap(v[i], v[j]);
        }
        std::swap(v[i], v[high - 1]);
        if (high - i > 2) stack[sp++] = high;
        if (i - low > 1) stack[sp++] = i;
        else low = i + 1;
    }
}

// Orders of the range sorted along each axis (the reference's 3 sorts).
struct Sorted {
    std::vector<Ref> by[3];
    bool exact = false;   // non-finite keys: the reference's quicksort sequence was replayed
};

// Sortable 64-bit key: centroid sum (with -0 == +0, as `<` / `==` see it), then triIdx.
inline uint64_t sort_key(const Ref& r, int d) {
    float c = r.b.mn[d] + r.b.mx[d];
    if (c == 0.0f) c = 0.0f;
    uint32_t u;
    std::memcpy(&u, &c, 4);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((uint64_t)u << 32) | (uint32_t)r.tri;
}

void sort_axis(const std::vector<Ref>& in, int d, std::vector<Ref>& out) {
    std::vector<std::pair<uint64_t, uint32_t>> k(in.size());
    for (size_t i = 0; i < in.size(); ++i) k[i] = {sort_key(in[i], d), (uint32_t)i};
    std::sort(k.begin(), k.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    out.resize(in.size());
    for (size_t i = 0; i < in.size(); ++i) out[i] = in[k[i].second];
}

// The three sorts of findObjectSplit (:201-203), each from the previous one's
// output.  Fast path when every centroid key is a number.
void sort_three(const std::vector<Ref>& range, Sorted& s, bool parallel) {
    bool finite = true;
    for (const Ref& r : range)
        for (int d = 0; d < 3 && finite; ++d)
            if (std::isnan(r.b.mn[d] + r.b.mx[d])) finite = false;
    if (!finite) {
        s.exact = true;
        s.by[0] = range;
        fw_sort(s.by[0], 0);
        s.by[1] = s.by[0];
        fw_sort(s.by[1], 1);
        s.by[2] = s.by[1];
        fw_sort(s.by[2], 2);
        return;
    }
    if (parallel) {
        std::thread t1([&] { sort_axis(range, 1, s.by[1]); });
        std::thread t2([&] { sort_axis(range, 2, s.by[2]); });
        sort_axis(range, 0, s.by[0]);
        t1.join();
        t2.join();
    } else {
        for (int d = 0; d < 3; ++d) sort_axis(range, d, s.by[d]);
    }
}

struct ObjectSplit {
    float sah = kF32Max;
    int dim = 0;
    int32_t num_left = 0;
    Box lb = Box::empty(), rb = Box::empty();
};
struct SpatialSplit {
    float sah = kF32Max;
    int dim = 0;
    float pos = 0.0f;
};

// findObjectSplit (:193-234) over the three sorted orders
ObjectSplit find_object_split(const Sorted& s, float node_sah, std::vector<Box>& rbs) {
    ObjectSplit sp;
    float best_tie = kF32Max;
    const int32_t n = (int32_t)s.by[0].size();
    rbs.resize(std::max(n, 1));
    for (int d = 0; d < 3; ++d) {
        const std::vector<Ref>& r = s.by[d];
        Box rb = Box::empty();
        for (int32_t i = n - 1; i > 0; --i) {
            rb.grow(r[i].b);
            rbs[i - 1] = rb;
        }
        Box lb = Box::empty();
        for (int32_t i = 1; i < n; ++i) {
            lb.grow(r[i - 1].b);
            const float sah = node_sah + lb.area() * (float)i + rbs[i - 1].area() * (float)(n - i);
            const float fi = (float)i, fr = (float)(n - i);
            const float tie = fi * fi + fr * fr;
            if (sah < sp.sah || (sah == sp.sah && tie < best_tie)) {
                sp.sah = sah;
                sp.dim = d;
                sp.num_left = i;
                sp.lb = lb;
                sp.rb = rbs[i - 1];
                best_tie = tie;
            }
        }
    }
    return sp;
}

// findSpatialSplit (:252-331)
SpatialSplit find_spatial_split(const Shared& S, const std::vector<Ref>& range, const Box& nb, float node_sah) {
    float origin[3], bin[3], inv[3];
    for (int k = 0; k < 3; ++k) {
        origin[k] = nb.mn[k];
        bin[k] = (nb.mx[k] - origin[k]) * (1.0f / (float)kBins);
        inv[k] = 1.0f / bin[k];
    }
    struct Bin { Box b; int32_t enter, exit; };
    std::vector<Bin> bins(3 * kBins);
    for (Bin& b : bins) { b.b = Box::empty(); b.enter = b.exit = 0; }
    for (const Ref& ref : range) {
        int32_t first[3], last[3];
        for (int k = 0; k < 3; ++k) {
            first[k] = std::max(std::min(cvtt((ref.b.mn[k] - origin[k]) * inv[k]), kBins - 1), 0);
            last[k] = std::max(std::min(cvtt((ref.b.mx[k] - origin[k]) * inv[k]), kBins - 1), first[k]);
        }
        for (int d = 0; d < 3; ++d) {
            Bin* B = &bins[d * kBins];
            Ref cur = ref;
            for (int32_t i = first[d]; i < last[d]; ++i) {
                Ref l, r;
                split_ref(S, l, r, cur, d, origin[d] + bin[d] * (float)(i + 1));
                B[i].b.grow(l.b);
                cur = r;
            }
            B[last[d]].b.grow(cur.b);
            B[first[d]].enter++;
            B[last[d]].exit++;
        }
    }
    SpatialSplit sp;
    Box rbs[kBins];
    for (int d = 0; d < 3; ++d) {
        const Bin* B = &bins[d * kBins];
        Box rb = Box::empty();
        for (int i = kBins - 1; i > 0; --i) {
            rb.grow(B[i].b);
            rbs[i - 1] = rb;
        }
        Box lb = Box::empty();
        int32_t ln = 0, rn = (int32_t)range.size();
        for (int i = 1; i < kBins; ++i) {
            lb.grow(B[i - 1].b);
            ln += B[i - 1].enter;
            rn -= B[i - 1].exit;
            const float sah = node_sah + lb.area() * (float)ln + rbs[i - 1].area() * (float)rn;
            if (sah < sp.sah) {
                sp.sah = sah;
                sp.dim = d;
                sp.pos = origin[d] + bin[d] * (float)i;
            }
        }
    }
    return sp;
}

// performSpatialSplit (:335-427) on the range in its current physical order.
// Children get [leftStart, leftEnd) and [rightStart, end) (+ appended halves).
void perform_spatial_split(const Shared& S, std::vector<Ref>& refs, const SpatialSplit& sp, std::vector<Ref>& left,
                           Box& lbox, std::vector<Ref>& right, Box& rbox) {
    const int64_t left_start = 0;
    int64_t left_end = 0, right_start = (int64_t)refs.size();
    lbox = rbox = Box::empty();
    const int d = sp.dim;
    const float pos = sp.pos;
    for (int64_t i = left_end; i < right_start; ++i) {
        if (refs[i].b.mx[d] <= pos) {
            lbox.grow(refs[i].b);
            std::swap(refs[i], refs[left_end++]);
        } else if (refs[i].b.mn[d] >= pos) {
            rbox.grow(refs[i].b);
            std::swap(refs[i], refs[--right_start]);
            --i;
        }
    }
    while (left_end < right_start) {
        Ref lref, rref;
        split_ref(S, lref, rref, refs[left_end], d, pos);
        Box lub = lbox, rub = rbox, ldb = lbox, rdb = rbox;
        lub.grow(refs[left_end].b);
        rub.grow(refs[left_end].b);
        ldb.grow(lref.b);
        rdb.grow(rref.b);
        const float lac = (float)(left_end - left_start);
        const float rac = (float)((int64_t)refs.size() - right_start);
        const float lbc = (float)(left_end - left_start + 1);
        const float rbc = (float)((int64_t)refs.size() - right_start + 1);
        const float unsplit_left = lub.area() * lbc + rbox.area() * rac;
        const float unsplit_right = lbox.area() * lac + rub.area() * rbc;
        const float duplicate = ldb.area() * lbc + rdb.area() * rbc;
        const float m = fmin1(fmin1(unsplit_left, unsplit_right), duplicate);
        if (m == unsplit_left) {
            lbox = lub;
            left_end++;
        } else if (m == unsplit_right) {
            rbox = rub;
            std::swap(refs[left_end], refs[--right_start]);
        } else {
            lbox = ldb;
            rbox = rdb;
            refs[left_end++] = lref;
            refs.push_back(rref);
        }
    }
    left.assign(refs.begin(), refs.begin() + left_end);
    right.assign(refs.begin() + right_start, refs.end());
}

std::unique_ptr<Node> make_leaf(const std::vector<Ref>& range, const Box& b) {
    auto n = std::make_unique<Node>();
    n->leaf = true;
    n->b = b;
    n->tris.resize(range.size());
    for (size_t i = 0; i < range.size(); ++i) n->tris[i] = range[range.size() - 1 - i].tri;  // createLeaf pops
    return n;
}

// buildNode (:107-176).  `range` is this node's slice of the reference stack,
// in physical order (consumed).
std::unique_ptr<Node> build(Shared& S, std::vector<Ref> range, Box bounds, int level) {
    {
        int cur = S.max_level.load(std::memory_order_relaxed);
        while (level > cur && !S.max_level.compare_exchange_weak(cur, level)) {}
    }
    // remove degenerates (:120-132): swap with the stack top, walking down
    for (int64_t i = (int64_t)range.size() - 1; i >= 0; --i) {
        const Box& b = range[i].b;
        const float sx = b.mx[0] - b.mn[0], sy = b.mx[1] - b.mn[1], sz = b.mx[2] - b.mn[2];
        if (fmin1(fmin1(sx, sy), sz) < 0.0f || (sx + sy) + sz == fmax1(fmax1(sx, sy), sz)) {
            range[i] = range.back();
            range.pop_back();
        }
    }
    const int32_t n = (int32_t)range.size();
    if (n <= kMinLeaf || level >= kMaxDepth) return make_leaf(range, bounds);

    const float area = bounds.area();
    const float leaf_sah = area * (float)n;
    const float node_sah = area * 2.0f;
    Sorted s;
    sort_three(range, s, n >= (1 << 16));
    std::vector<Ref>().swap(range);  // physical order is now s.by[2]
    std::vector<Box> rbs;
    const ObjectSplit obj = find_object_split(s, node_sah, rbs);
    std::vector<Box>().swap(rbs);
    SpatialSplit spa;
    if (level < kMaxSpatialDepth) {
        Box ov = obj.lb;
        ov.intersect(obj.rb);
        if (ov.area() >= S.min_overlap) spa = find_spatial_split(S, s.by[2], bounds, node_sah);
    }
    const float min_sah = fmin1(fmin1(leaf_sah, obj.sah), spa.sah);
    if (min_sah == leaf_sah && n <= kMaxLeaf) return make_leaf(s.by[2], bounds);

    std::vector<Ref> left, right, work;
    Box lbox = Box::empty(), rbox = Box::empty();
    if (min_sah == spa.sah) {
        work = s.by[2];
        perform_spatial_split(S, work, spa, left, lbox, right, rbox);
    }
    if (left.empty() || right.empty()) {  // performObjectSplit (:238-248): order of the chosen axis
        if (s.exact) {  // replay the sort from the current physical order
            if (work.empty()) work = s.by[2];
            fw_sort(work, obj.dim);
            s.by[obj.dim].swap(work);
        }
        const std::vector<Ref>& o = s.by[obj.dim];
        left.assign(o.begin(), o.begin() + obj.num_left);
        right.assign(o.begin() + obj.num_left, o.end());
        lbox = obj.lb;
        rbox = obj.rb;
    }
    std::vector<Ref>().swap(work);
    for (int d = 0; d < 3; ++d) std::vector<Ref>().swap(s.by[d]);

    auto node = std::make_unique<Node>();
    node->b = bounds;
    const size_t nkids = left.size() + right.size();
    if (nkids >= 4096 && S.threads.fetch_add(1) < S.max_threads - 1) {
        std::unique_ptr<Node> r;
        std::thread th([&] { r = build(S, std::move(right), rbox, level + 1); });
        node->kid[0] = build(S, std::move(left), lbox, level + 1);
        th.join();
        S.threads.fetch_sub(1);
        node->kid[1] = std::move(r);
    } else {
        if (nkids >= 4096) S.threads.fetch_sub(1);
        node->kid[1] = build(S, std::move(right), rbox, level + 1);
        node->kid[0] = build(S, std::move(left), lbox, level + 1);
    }
    return node;
}

// m_triIndices: leaves in creation order = right-first DFS (:173-174, :181-189)
void emit_tris(Node* n, std::vector<int32_t>& tris, int32_t& leaves) {
    if (n->leaf) {
        n->lo = (int32_t)tris.size();
        n->cnt = (int32_t)n->tris.size();
        tris.insert(tris.end(), n->tris.begin(), n->tris.end());
        std::vector<int32_t>().swap(n->tris);
        ++leaves;
        return;
    }
    emit_tris(n->kid[1].get(), tris, leaves);
    emit_tris(n->kid[0].get(), tris, leaves);
}

// BVH_Cuda::build2 (:98-137): pre-order, left child first
int32_t flatten(const Node* n, std::vector<rt_bvh_node>& out) {
    const int32_t me = (int32_t)out.size();
    out.emplace_back();
    rt_bvh_node nd;
    nd.min = rt_float4{n->b.mn[0], n->b.mn[1], n->b.mn[2], 1.0f};
    nd.max = rt_float4{n->b.mx[0], n->b.mx[1], n->b.mx[2], 1.0f};
    nd.offset_left = nd.offset_right = nd.offset_tris = -1;
    nd.num_tris = 0;
    if (n->leaf) {
        nd.offset_tris = n->lo;
        nd.num_tris = n->cnt;
    } else {
        nd.offset_left = flatten(n->kid[0].get(), out);
        nd.offset_right = flatten(n->kid[1].get(), out);
    }
    out[me] = nd;
    return me;
}

}  // namespace

void build_sbvh(const Mesh& m, int num_threads, Bvh& out) {
    const auto t0 = std::chrono::steady_clock::now();
    out = Bvh();
    if (num_threads < 1) num_threads = (int)std::max(1u, std::thread::hardware_concurrency());
    // vertices as packed float4 (rt_float4 is {x,y,z,w})
    static_assert(sizeof(rt_float4) == 16, "float4");
    Shared S;
    S.verts = reinterpret_cast<const float*>(m.vertices.data());
    S.idx = m.indices.data();
    S.max_threads = num_threads;
    const int32_t nt = m.num_triangles();
    std::vector<Ref> refs(nt);
    Box root = Box::empty();
    for (int32_t i = 0; i < nt; ++i) {  // run() (:47-60)
        refs[i].tri = i;
        refs[i].b = Box::empty();
        for (int j = 0; j < 3; ++j) refs[i].b.grow(S.verts + 4 * (int64_t)S.idx[3 * i + j]);
        root.grow(refs[i].b);
    }
    S.min_overlap = root.area() * kSplitAlpha;
    std::unique_ptr<Node> tree = build(S, std::move(refs), root, 0);

    int32_t leaves = 0;
    std::vector<int32_t> tris;
    tris.reserve((size_t)nt + nt / 4);
    emit_tris(tree.get(), tris, leaves);
    out.nodes.reserve(2 * (size_t)leaves);
    flatten(tree.get(), out.nodes);
    out.tri_indices.resize(tris.size());
    for (size_t i = 0; i < tris.size(); ++i) out.tri_indices[i] = 3 * tris[i];
    out.num_leaves = leaves;
    out.max_depth = S.max_level.load();
    out.build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace rtamd
