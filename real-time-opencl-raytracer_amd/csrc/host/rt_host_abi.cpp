// rt_host_abi.cpp -- extern "C" wrappers over the host scene tools (include/rt_host.h).
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "rt_host.h"
#include "scene.hpp"

struct rt_mesh { rtamd::Mesh m; };
struct rt_bvh { rtamd::Bvh b; };
struct rt_camera { rtamd::Camera c; explicit rt_camera(float r) : c(r) {} };

extern "C" {

rt_mesh* rt_mesh_create(void) { return new (std::nothrow) rt_mesh(); }
void rt_mesh_destroy(rt_mesh* m) { delete m; }

int rt_mesh_view_get(const rt_mesh* mh, rt_mesh_view* o) {
    if (!mh || !o) return RT_ERR_INVALID_ARG;
    const rtamd::Mesh& m = mh->m;
    o->vertices = m.vertices.data(); o->num_vertices = (int32_t)m.vertices.size();
    o->indices = m.indices.data(); o->num_indices = (int32_t)m.indices.size();
    o->normals = m.normals.data(); o->num_normals = (int32_t)m.normals.size();
    o->normals_indices = m.normals_indices.data();
    o->materials = m.materials.data(); o->num_materials = (int32_t)m.materials.size();
    o->tri_to_material = m.tri_to_material.data();
    for (int k = 0; k < 3; ++k) { o->scene_min[k] = m.scene_min[k]; o->scene_max[k] = m.scene_max[k]; }
    return RT_OK;
}

int rt_mesh_set(rt_mesh* mh, const rt_float4* verts, int32_t nv, const int32_t* idx, int32_t nidx,
                const rt_float4* normals, int32_t nnorm, const int32_t* nidx_arr, const rt_material* mats,
                int32_t nmat, const int32_t* tri_to_mat) {
    if (!mh || !verts || nv < 0 || !idx || nidx < 0 || nidx % 3) return RT_ERR_INVALID_ARG;
    rtamd::Mesh m;
    m.vertices.assign(verts, verts + nv);
    m.indices.assign(idx, idx + nidx);
    for (int32_t i : m.indices)
        if (i < 0 || i >= nv) return RT_ERR_BAD_SCENE;
    if (normals && nidx_arr && nnorm > 0) {
        m.normals.assign(normals, normals + nnorm);
        m.normals_indices.assign(nidx_arr, nidx_arr + nidx);
        for (int32_t i : m.normals_indices)
            if (i < 0 || i >= nnorm) return RT_ERR_BAD_SCENE;
    }
    if (mats && nmat > 0) {
        m.materials.assign(mats, mats + nmat);
        if (tri_to_mat) {
            m.tri_to_material.assign(tri_to_mat, tri_to_mat + nidx / 3);
            for (int32_t i : m.tri_to_material)
                if (i < 0 || i >= nmat) return RT_ERR_BAD_SCENE;
        }
    }
    m.ensure_normals();
    m.ensure_materials();
    m.update_bounds();
    mh->m = std::move(m);
    return RT_OK;
}

int rt_mesh_load_obj(rt_mesh* mh, const char* path) {
    if (!mh || !path) return RT_ERR_INVALID_ARG;
    std::string err;
    if (rtamd::load_obj(path, mh->m, err) != 0) {
        std::fprintf(stderr, "rt_mesh_load_obj: %s\n", err.c_str());
        return RT_ERR_BAD_SCENE;
    }
    return RT_OK;
}

int rt_mesh_load_dae(rt_mesh* mh, const char* path) {
    if (!mh || !path) return RT_ERR_INVALID_ARG;
    std::string err;
    if (rtamd::load_dae(path, mh->m, err) != 0) {
        std::fprintf(stderr, "rt_mesh_load_dae: %s\n", err.c_str());
        return RT_ERR_BAD_SCENE;
    }
    return RT_OK;
}

int rt_mesh_save_dae(const rt_mesh* mh, const char* path) {
    if (!mh || !path) return RT_ERR_INVALID_ARG;
    std::string err;
    if (rtamd::save_dae(path, mh->m, err) != 0) {
        std::fprintf(stderr, "rt_mesh_save_dae: %s\n", err.c_str());
        return RT_ERR_INVALID_ARG;
    }
    return RT_OK;
}

int rt_mesh_gen_cornell(rt_mesh* mh) {
    if (!mh) return RT_ERR_INVALID_ARG;
    rtamd::gen_cornell(mh->m);
    return RT_OK;
}
int rt_mesh_gen_torus_knot(rt_mesh* mh, int32_t nu, int32_t nv) {
    if (!mh || nu < 3 || nv < 3) return RT_ERR_INVALID_ARG;
    rtamd::gen_torus_knot(mh->m, nu, nv);
    return RT_OK;
}
int rt_mesh_gen_heightfield(rt_mesh* mh, int32_t nx, int32_t nz, float amplitude, uint32_t seed, float x0, float x1,
                            float z0, float z1) {
    if (!mh || nx < 1 || nz < 1 || !(x1 > x0) || !(z1 > z0)) return RT_ERR_INVALID_ARG;
    rtamd::gen_heightfield(mh->m, nx, nz, amplitude, seed, x0, x1, z0, z1);
    return RT_OK;
}
int rt_mesh_gen_random(rt_mesh* mh, int32_t ntris, float extent, float size, uint32_t seed) {
    if (!mh || ntris < 0) return RT_ERR_INVALID_ARG;
    rtamd::gen_random(mh->m, ntris, extent, size, seed);
    return RT_OK;
}
int rt_mesh_append_grid(rt_mesh* dst, const rt_mesh* src, int32_t gx, int32_t gz, float dx, float dz,
                        float scale) {
    if (!dst || !src || dst == src || gx < 1 || gz < 1) return RT_ERR_INVALID_ARG;
    rtamd::append_grid(dst->m, src->m, gx, gz, dx, dz, scale);
    return RT_OK;
}

int rt_bvh_build(const rt_mesh* mh, int32_t max_leaf, int32_t num_threads, rt_bvh** out) {
    if (!mh || !out) return RT_ERR_INVALID_ARG;
    rt_bvh* b = new (std::nothrow) rt_bvh();
    if (!b) return RT_ERR_OUT_OF_MEMORY;
    rtamd::build_bvh(mh->m, max_leaf, num_threads, b->b);
    *out = b;
    return RT_OK;
}

int rt_bvh_build_sbvh(const rt_mesh* mh, int32_t num_threads, rt_bvh** out) {
    if (!mh || !out) return RT_ERR_INVALID_ARG;
    rt_bvh* b = new (std::nothrow) rt_bvh();
    if (!b) return RT_ERR_OUT_OF_MEMORY;
    rtamd::build_sbvh(mh->m, num_threads, b->b);
    *out = b;
    return RT_OK;
}

int rt_bvh_view_get(const rt_bvh* bh, rt_bvh_view* o) {
    if (!bh || !o) return RT_ERR_INVALID_ARG;
    o->nodes = bh->b.nodes.data(); o->num_nodes = (int32_t)bh->b.nodes.size();
    o->tri_indices = bh->b.tri_indices.data(); o->num_tri_indices = (int32_t)bh->b.tri_indices.size();
    o->max_depth = bh->b.max_depth; o->num_leaves = bh->b.num_leaves;
    o->build_seconds = bh->b.build_seconds;
    return RT_OK;
}

void rt_bvh_destroy(rt_bvh* b) { delete b; }

static const char kMagic[8] = {'R', 'T', 'B', 'V', 'H', '0', '0', '1'};

int rt_bvh_save(const rt_bvh* bh, const rt_mesh* mh, const char* path) {
    if (!bh || !mh || !path) return RT_ERR_INVALID_ARG;
    FILE* f = std::fopen(path, "wb");
    if (!f) return RT_ERR_INVALID_ARG;
    uint64_t h = mh->m.hash();
    uint64_t nn = bh->b.nodes.size(), nr = bh->b.tri_indices.size();
    int32_t meta[2] = {bh->b.max_depth, bh->b.num_leaves};
    bool ok = std::fwrite(kMagic, 8, 1, f) == 1 && std::fwrite(&h, 8, 1, f) == 1 && std::fwrite(&nn, 8, 1, f) == 1 &&
              std::fwrite(&nr, 8, 1, f) == 1 && std::fwrite(meta, sizeof meta, 1, f) == 1 &&
              std::fwrite(bh->b.nodes.data(), sizeof(rt_bvh_node), nn, f) == nn &&
              std::fwrite(bh->b.tri_indices.data(), 4, nr, f) == nr;
    std::fclose(f);
    return ok ? RT_OK : RT_ERR_DEVICE;
}

int rt_bvh_load(const rt_mesh* mh, const char* path, rt_bvh** out) {
    if (!mh || !path || !out) return RT_ERR_INVALID_ARG;
    FILE* f = std::fopen(path, "rb");
    if (!f) return RT_ERR_INVALID_ARG;
    char mg[8];
    uint64_t h = 0, nn = 0, nr = 0;
    int32_t meta[2];
    bool ok = std::fread(mg, 8, 1, f) == 1 && std::memcmp(mg, kMagic, 8) == 0 && std::fread(&h, 8, 1, f) == 1 &&
              std::fread(&nn, 8, 1, f) == 1 && std::fread(&nr, 8, 1, f) == 1 &&
              std::fread(meta, sizeof meta, 1, f) == 1 && h == mh->m.hash();
    rt_bvh* b = nullptr;
    if (ok) {
        b = new (std::nothrow) rt_bvh();
        ok = b != nullptr;
    }
    if (ok) {
        b->b.nodes.resize(nn);
        b->b.tri_indices.resize(nr);
        ok = std::fread(b->b.nodes.data(), sizeof(rt_bvh_node), nn, f) == nn &&
             std::fread(b->b.tri_indices.data(), 4, nr, f) == nr;
        b->b.max_depth = meta[0];
        b->b.num_leaves = meta[1];
    }
    std::fclose(f);
    if (!ok) {
        delete b;
        return RT_ERR_BAD_SCENE;
    }
    *out = b;
    return RT_OK;
}

int rt_camera_params(const rt_mesh* mh, uint32_t w, uint32_t h, float radius, float extra_alpha, float extra_beta,
                     const float* light_pos, const float* light_color, rt_params* out) {
    if (!mh || !out || w == 0 || h == 0) return RT_ERR_INVALID_ARG;
    *out = rtamd::camera_params(mh->m, w, h, radius, extra_alpha, extra_beta, light_pos, light_color);
    return RT_OK;
}

rt_camera* rt_camera_create(float radius) { return new (std::nothrow) rt_camera(radius); }
void rt_camera_destroy(rt_camera* c) { delete c; }
int rt_camera_add_rotate(rt_camera* c, float da, float db) {
    if (!c) return RT_ERR_INVALID_ARG;
    c->c.add_rotate(da, db);
    return RT_OK;
}
int rt_camera_add_radius(rt_camera* c, float dr) {
    if (!c) return RT_ERR_INVALID_ARG;
    c->c.add_radius(dr);
    return RT_OK;
}
int rt_camera_frame_params(const rt_camera* c, const rt_mesh* mh, uint32_t w, uint32_t h, const float* light_pos,
                           const float* light_color, rt_params* out) {
    if (!c || !mh || !out || w == 0 || h == 0) return RT_ERR_INVALID_ARG;
    *out = rtamd::frame_params(c->c, mh->m, w, h, light_pos, light_color);
    return RT_OK;
}

}  // extern "C"
