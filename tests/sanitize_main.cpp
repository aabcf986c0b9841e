// sanitize_main.cpp -- TEST INFRASTRUCTURE: the host-side code of the render path (scene
// generators, OBJ / Collada loaders, SBVH + binned builders, BVH cache, camera) and the CPU
// oracle (oracle/rt_oracle.c, oracle/sbvh_oracle.c) driven under AddressSanitizer +
// UndefinedBehaviorSanitizer.  Built and run by tests/test_sanitizers.py with
// -fsanitize=address,undefined -fno-sanitize-recover=all, so any report ends the run with a
// non-zero status.  Also cross-checks what it runs: the product SBVH against the SBVH
// oracle byte for byte, the Collada and cache round trips, and the oracle's frame across
// thread counts.
//
//   sanitize_main <tmpdir> [obj file]
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "rt_host.h"

extern "C" {
// oracle/rt_oracle.c, oracle/sbvh_oracle.c (test infrastructure, linked only here)
typedef struct { uint64_t rays[3], inner[3], leaf[3], tris[3], max_stack, stack_overflow; } ostats_t;
int oracle_render(const void* params, const void* verts, const int32_t* idx, const void* nodes, int32_t num_nodes,
                  const int32_t* refs, int32_t num_refs, const void* normals, const int32_t* nidx, const void* mats,
                  const int32_t* tri2mat, uint32_t w, uint32_t h, int depth, uint32_t flags, int64_t pix0,
                  int64_t npix, int64_t stride, uint32_t* out, int32_t* hits, float* tvals, float* rgb, void* stats,
                  int nthreads);
int sbvh_oracle_build(const float* verts, int32_t nv, const int32_t* idx, int32_t ntri, void** nodes_out,
                      int32_t* num_nodes, int32_t** refs_out, int32_t* num_refs);
void sbvh_oracle_free(void* p);
}

static int g_fail = 0;
#define CHECK(cond, ...)                                          \
    do {                                                          \
        if (!(cond)) {                                            \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                    \
            std::fprintf(stderr, "\n");                           \
            ++g_fail;                                             \
        }                                                         \
    } while (0)

// the round trip keeps the triangles (grouped by material, -0 read back as +0:
// tests/test_collada.py pins that exactly); here: the same triangle count
static bool same_triangles(const rt_mesh* a, const rt_mesh* b) {
    rt_mesh_view x, y;
    if (rt_mesh_view_get(a, &x) || rt_mesh_view_get(b, &y)) return false;
    return x.num_indices == y.num_indices && x.num_materials == y.num_materials;
}

static void exercise(const char* name, rt_mesh* m, const std::string& dir) {
    rt_mesh_view v;
    CHECK(rt_mesh_view_get(m, &v) == RT_OK, "%s: view", name);
    const int32_t ntri = v.num_indices / 3;

    // Collada round trip (the C2-C4 scene path)
    const std::string dae = dir + "/" + name + ".dae";
    CHECK(rt_mesh_save_dae(m, dae.c_str()) == RT_OK, "%s: save_dae", name);
    rt_mesh* back = rt_mesh_create();
    CHECK(rt_mesh_load_dae(back, dae.c_str()) == RT_OK, "%s: load_dae", name);
    CHECK(same_triangles(m, back), "%s: Collada round trip changed the mesh", name);
    rt_mesh_destroy(back);

    // SBVH: product (4 threads) == oracle, byte for byte
    rt_bvh* b = nullptr;
    CHECK(rt_bvh_build_sbvh(m, 4, &b) == RT_OK && b, "%s: sbvh build", name);
    rt_bvh_view bv;
    CHECK(rt_bvh_view_get(b, &bv) == RT_OK, "%s: bvh view", name);
    void* on = nullptr;
    int32_t* orf = nullptr;
    int32_t onn = 0, onr = 0;
    CHECK(sbvh_oracle_build(&v.vertices[0].x, v.num_vertices, v.indices, ntri, &on, &onn, &orf, &onr) == 0,
          "%s: sbvh oracle", name);
    CHECK(onn == bv.num_nodes && onr == bv.num_tri_indices, "%s: sbvh sizes %d/%d vs %d/%d", name, bv.num_nodes,
          bv.num_tri_indices, onn, onr);
    if (onn == bv.num_nodes && onr == bv.num_tri_indices) {
        CHECK(!std::memcmp(on, bv.nodes, 48 * (size_t)onn), "%s: sbvh node bytes differ from the oracle", name);
        CHECK(!std::memcmp(orf, bv.tri_indices, 4 * (size_t)onr), "%s: sbvh refs differ from the oracle", name);
    }
    sbvh_oracle_free(on);
    sbvh_oracle_free(orf);

    // BVH cache round trip
    const std::string cache = dir + "/" + name + ".bvh";
    CHECK(rt_bvh_save(b, m, cache.c_str()) == RT_OK, "%s: bvh save", name);
    rt_bvh* b2 = nullptr;
    CHECK(rt_bvh_load(m, cache.c_str(), &b2) == RT_OK && b2, "%s: bvh load", name);
    if (b2) {
        rt_bvh_view bv2;
        rt_bvh_view_get(b2, &bv2);
        CHECK(bv2.num_nodes == bv.num_nodes && !std::memcmp(bv2.nodes, bv.nodes, 48 * (size_t)bv.num_nodes),
              "%s: cache round trip", name);
        rt_bvh_destroy(b2);
    }

    // binned SAH builder
    rt_bvh* bb = nullptr;
    CHECK(rt_bvh_build(m, 8, 4, &bb) == RT_OK && bb, "%s: binned build", name);
    if (bb) rt_bvh_destroy(bb);

    // camera: default and an orbit step; then the oracle frame at depth 3 on 1 and 4 threads
    rt_params p;
    CHECK(rt_camera_params(m, 64, 48, 200.f, 0.f, 0.f, nullptr, nullptr, &p) == RT_OK, "%s: camera", name);
    rt_camera* cam = rt_camera_create(200.f);
    rt_camera_add_rotate(cam, 0.3f, -0.1f);
    rt_camera_add_radius(cam, -20.f);
    rt_params p2;
    CHECK(rt_camera_frame_params(cam, m, 64, 48, nullptr, nullptr, &p2) == RT_OK, "%s: orbit camera", name);
    rt_camera_destroy(cam);
    const int W = 64, H = 48, D = 3;
    for (const rt_params* pp : {&p, &p2}) {
        std::vector<uint32_t> o1(W * H), o4(W * H);
        std::vector<int32_t> h1(W * H * D * 2), h4(W * H * D * 2);
        std::vector<float> t1(W * H * D), t4(W * H * D), c1(W * H * 3), c4(W * H * 3);
        ostats_t st;
        int rc1 = oracle_render(pp, v.vertices, v.indices, bv.nodes, bv.num_nodes, bv.tri_indices, bv.num_tri_indices,
                                v.normals, v.normals_indices, v.materials, v.tri_to_material, W, H, D, 0, 0, W * H, 1,
                                o1.data(), h1.data(), t1.data(), c1.data(), &st, 1);
        int rc4 = oracle_render(pp, v.vertices, v.indices, bv.nodes, bv.num_nodes, bv.tri_indices, bv.num_tri_indices,
                                v.normals, v.normals_indices, v.materials, v.tri_to_material, W, H, D, 0, 0, W * H, 1,
                                o4.data(), h4.data(), t4.data(), c4.data(), nullptr, 4);
        CHECK(rc1 == 0 && rc4 == 0, "%s: oracle_render", name);
        CHECK(o1 == o4 && h1 == h4 && !std::memcmp(t1.data(), t4.data(), 4 * t1.size()), "%s: threads differ", name);
        CHECK(st.rays[0] > 0, "%s: no primary rays", name);
    }
    rt_bvh_destroy(b);
    std::printf("%s: %d tris, %d nodes ok\n", name, ntri, bv.num_nodes);
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string dir = argv[1];
    {
        rt_mesh* m = rt_mesh_create();
        CHECK(rt_mesh_gen_cornell(m) == RT_OK, "cornell");
        exercise("cornell", m, dir);
        rt_mesh_destroy(m);
    }
    {
        rt_mesh* m = rt_mesh_create();
        CHECK(rt_mesh_gen_torus_knot(m, 40, 12) == RT_OK, "knot");
        exercise("knot", m, dir);
        rt_mesh_destroy(m);
    }
    {
        rt_mesh* m = rt_mesh_create();
        CHECK(rt_mesh_gen_heightfield(m, 30, 40, 10.f, 0x5EED, -150.f, 650.f, -150.f, 650.f) == RT_OK, "hf");
        exercise("heightfield", m, dir);
        rt_mesh* g = rt_mesh_create();   // the C5 merge of tiles on a grid
        CHECK(rt_mesh_append_grid(g, m, 3, 2, 160.f, 400.f, 1.f) == RT_OK, "grid");
        exercise("grid", g, dir);
        rt_mesh_destroy(g);
        rt_mesh_destroy(m);
    }
    {
        rt_mesh* m = rt_mesh_create();   // overlapping soup: big leaves, spatial splits
        CHECK(rt_mesh_gen_random(m, 3000, 60.f, 8.f, 7) == RT_OK, "random");
        exercise("random", m, dir);
        rt_mesh_destroy(m);
    }
    if (argc > 2) {
        rt_mesh* m = rt_mesh_create();
        CHECK(rt_mesh_load_obj(m, argv[2]) == RT_OK, "obj");
        exercise("obj", m, dir);
        rt_mesh_destroy(m);
    }
    // error paths: missing files, bad arguments
    {
        rt_mesh* m = rt_mesh_create();
        CHECK(rt_mesh_load_dae(m, (dir + "/missing.dae").c_str()) != RT_OK, "missing dae accepted");
        CHECK(rt_mesh_load_obj(m, (dir + "/missing.obj").c_str()) != RT_OK, "missing obj accepted");
        rt_bvh* b = nullptr;
        CHECK(rt_bvh_load(m, (dir + "/missing.bvh").c_str(), &b) != RT_OK, "missing cache accepted");
        rt_mesh_destroy(m);
    }
    std::printf(g_fail ? "FAILED %d\n" : "ALL OK\n", g_fail);
    return g_fail ? 1 : 0;
}
