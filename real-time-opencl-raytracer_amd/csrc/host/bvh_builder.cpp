// bvh_builder.cpp -- binned-SAH BVH builder emitting the reference's node layout.
//
// Cost model as the reference builder (BVH2.cpp:13, SplitBVHBuilder.cpp:120-180,
// Platform.h:17-30): leaf SAH = area * N, split SAH = area * 2 + A_L*N_L + A_R*N_R,
// leaves hold 1..max_leaf triangles, depth limit 64, degenerate references
// (bounding box with fewer than two non-zero extents) are dropped
// (SplitBVHBuilder.cpp:120-132).  Splits are object splits over 32 centroid bins
// on all three axes (no spatial splits: SURVEY.md 8f next #1).
//
// Output: BVH_Node_ array in pre-order with the left subtree first, root = 0
// (BVH_Cuda.h:98-137), and tri_indices = 3 * triangle index (BVH_Cuda.h:90-93).
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

constexpr int kBins = 32;
constexpr int kMaxDepth = 64;

struct Box {
    float lo[3], hi[3];
    void clear() {
        for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
    }
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
    }
    void grow(const float* p) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
    }
    float area() const {
        float d[3];
        for (int k = 0; k < 3; ++k) d[k] = hi[k] - lo[k];
        if (d[0] < 0 || d[1] < 0 || d[2] < 0) return 0.0f;
        return 2.0f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
};

struct Ref {
    Box b;
    float c[3];   // bmin + bmax (twice the centroid, as sortCompare)
    int32_t tri;
};

struct TNode {
    Box b;
    std::unique_ptr<TNode> kid[2];
    int begin = 0, count = 0;  // leaf range in the ref array
    bool leaf() const { return !kid[0]; }
};

struct Builder {
    std::vector<Ref>& refs;
    int max_leaf;
    std::atomic<int> threads_left;
    std::atomic<int> max_depth{0};
    std::atomic<int> leaves{0};

    Builder(std::vector<Ref>& r, int ml, int nt) : refs(r), max_leaf(ml), threads_left(nt - 1) {}

    std::unique_ptr<TNode> make_leaf(const Box& b, int begin, int end, int depth) {
        auto n = std::make_unique<TNode>();
        n->b = b;
        n->begin = begin;
        n->count = end - begin;
        leaves++;
        int md = max_depth.load();
        while (depth > md && !max_depth.compare_exchange_weak(md, depth)) {}
        return n;
    }

    std::unique_ptr<TNode> build(int begin, int end, const Box& b, int depth) {
        const int n = end - begin;
        if (n <= 1 || depth >= kMaxDepth) return make_leaf(b, begin, end, depth);
        Box cb;
        cb.clear();
        for (int i = begin; i < end; ++i) cb.grow(refs[i].c);
        const float area = b.area();
        const float leaf_sah = area * (float)n;
        const float node_sah = area * 2.0f;
        float best = INFINITY;
        int best_axis = -1, best_split = -1;
        for (int ax = 0; ax < 3; ++ax) {
            float ext = cb.hi[ax] - cb.lo[ax];
            if (!(ext > 0.0f)) continue;
            float scale = kBins / ext;
            int cnt[kBins] = {0};
            Box bb[kBins];
            for (auto& x : bb) x.clear();
            for (int i = begin; i < end; ++i) {
                int k = (int)((refs[i].c[ax] - cb.lo[ax]) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                cnt[k]++;
                bb[k].grow(refs[i].b);
            }
            float right_area[kBins];
            int right_cnt[kBins];
            Box acc;
            acc.clear();
            int c = 0;
            for (int k = kBins - 1; k > 0; --k) {
                acc.grow(bb[k]);
                c += cnt[k];
                right_area[k] = acc.area();
                right_cnt[k] = c;
            }
            acc.clear();
            c = 0;
            for (int k = 0; k < kBins - 1; ++k) {
                acc.grow(bb[k]);
                c += cnt[k];
                int rc = right_cnt[k + 1];
                if (c == 0 || rc == 0) continue;
                float sah = node_sah + acc.area() * (float)c + right_area[k + 1] * (float)rc;
                if (sah < best) { best = sah; best_axis = ax; best_split = k; }
            }
        }
        if (n <= max_leaf && leaf_sah <= best) return make_leaf(b, begin, end, depth);
        int mid;
        if (best_axis < 0) {
            if (n <= max_leaf) return make_leaf(b, begin, end, depth);
            // all centroids coincide: split in the middle of the (tri-ordered) range
            std::sort(refs.begin() + begin, refs.begin() + end, [](const Ref& x, const Ref& y) { return x.tri < y.tri; });
            mid = begin + n / 2;
        } else {
            const int ax = best_axis;
            const float scale = kBins / (cb.hi[ax] - cb.lo[ax]);
            const float lo = cb.lo[ax];
            auto it = std::partition(refs.begin() + begin, refs.begin() + end, [&](const Ref& r) {
                int k = (int)((r.c[ax] - lo) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                return k <= best_split;
            });
            mid = (int)(it - refs.begin());
            // deterministic order inside each side regardless of partition internals
            auto by_tri = [](const Ref& x, const Ref& y) { return x.tri < y.tri; };
            if (n <= 4096) {
                std::sort(refs.begin() + begin, refs.begin() + mid, by_tri);
                std::sort(refs.begin() + mid, refs.begin() + end, by_tri);
            }
        }
        Box lb, rb;
        lb.clear();
        rb.clear();
        for (int i = begin; i < mid; ++i) lb.grow(refs[i].b);
        for (int i = mid; i < end; ++i) rb.grow(refs[i].b);
        auto node = std::make_unique<TNode>();
        node->b = b;
        if (n > 65536 && threads_left.fetch_sub(1) > 0) {
            std::unique_ptr<TNode> left;
            std::thread th([&]() { left = build(begin, mid, lb, depth + 1); });
            node->kid[1] = build(mid, end, rb, depth + 1);
            th.join();
            threads_left.fetch_add(1);
            node->kid[0] = std::move(left);
        } else {
            node->kid[0] = build(begin, mid, lb, depth + 1);
            node->kid[1] = build(mid, end, rb, depth + 1);
        }
        return node;
    }
};

int flatten(const TNode* n, const std::vector<Ref>& refs, Bvh& out) {
    int idx = (int)out.nodes.size();
    out.nodes.emplace_back();
    rt_bvh_node nd;
    nd.min = rt_float4{n->b.lo[0], n->b.lo[1], n->b.lo[2], 1.0f};
    nd.max = rt_float4{n->b.hi[0], n->b.hi[1], n->b.hi[2], 1.0f};
    if (n->leaf()) {
        nd.offset_left = -1;
        nd.offset_right = -1;
        nd.offset_tris = (int32_t)out.tri_indices.size();
        nd.num_tris = n->count;
        for (int i = 0; i < n->count; ++i) out.tri_indices.push_back(3 * refs[n->begin + i].tri);
    } else {
        nd.offset_tris = -1;
        nd.num_tris = 0;
        nd.offset_left = flatten(n->kid[0].get(), refs, out);
        nd.offset_right = flatten(n->kid[1].get(), refs, out);
    }
    out.nodes[idx] = nd;
    return idx;
}

}  // namespace

void build_bvh(const Mesh& m, int max_leaf, int num_threads, Bvh& out) {
    auto t0 = std::chrono::steady_clock::now();
    out = Bvh();
    if (max_leaf < 1) max_leaf = 8;
    if (num_threads < 1) num_threads = (int)std::max(1u, std::thread::hardware_concurrency());
    const int nt = m.num_triangles();
    std::vector<Ref> refs;
    refs.reserve(nt);
    Box root;
    root.clear();
    for (int t = 0; t < nt; ++t) {
        Ref r;
        r.b.clear();
        for (int k = 0; k < 3; ++k) {
            const rt_float4& v = m.vertices[m.indices[3 * t + k]];
            const float p[3] = {v.x, v.y, v.z};
            r.b.grow(p);
        }
        float s[3] = {r.b.hi[0] - r.b.lo[0], r.b.hi[1] - r.b.lo[1], r.b.hi[2] - r.b.lo[2]};
        float mn = std::min(s[0], std::min(s[1], s[2])), mx = std::max(s[0], std::max(s[1], s[2]));
        if (mn < 0.0f || s[0] + s[1] + s[2] == mx) continue;  // degenerate (SplitBVHBuilder.cpp:124-131)
        for (int k = 0; k < 3; ++k) r.c[k] = r.b.lo[k] + r.b.hi[k];
        r.tri = t;
        refs.push_back(r);
        root.grow(r.b);
    }
    if (refs.empty()) {
        // A single empty leaf: traversal finds nothing (the reference builds the same).
        rt_bvh_node nd;
        nd.min = rt_float4{0, 0, 0, 1};
        nd.max = rt_float4{0, 0, 0, 1};
        nd.offset_left = nd.offset_right = -1;
        nd.offset_tris = 0;
        nd.num_tris = 0;
        out.nodes.push_back(nd);
        out.num_leaves = 1;
    } else {
        Builder b(refs, max_leaf, num_threads);
        auto tree = b.build(0, (int)refs.size(), root, 0);
        out.nodes.reserve(2 * refs.size());
        out.tri_indices.reserve(refs.size());
        flatten(tree.get(), refs, out);
        out.max_depth = b.max_depth.load();
        out.num_leaves = b.leaves.load();
    }
    out.build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace rtamd
