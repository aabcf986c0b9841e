// scene.hpp -- host-side scene data in the reference's shapes.
//
// rtamd::Mesh mirrors Mesh (Mesh.h:69-101): the arrays raytracer_bvh reads.
// rtamd::Bvh mirrors BVH_Cuda (BVH_Cuda.h:34-137): BVH_Node_[] + tri_indices[].
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "rt_abi.h"

namespace rtamd {

struct Mesh {
    std::vector<int32_t> indices;            // Mesh::indices (3 per triangle)
    std::vector<rt_float4> vertices;         // Mesh::vertices (w = 1)
    std::vector<int32_t> normals_indices;    // Mesh::normals_indices
    std::vector<rt_float4> normals;          // Mesh::normals
    std::vector<rt_material> materials;      // Mesh::materials
    std::vector<int32_t> tri_to_material;    // Mesh::triangle_index_to_material_index
    float scene_min[3] = {0, 0, 0};          // Mesh::scene_aabbox_min
    float scene_max[3] = {0, 0, 0};

    int32_t num_triangles() const { return (int32_t)(indices.size() / 3); }
    void update_bounds();                    // Mesh.cpp:55-61 / :103-110 (fminf1/fmaxf1 over vertices)
    void ensure_normals();                   // per-vertex normals when a source has none
    void ensure_materials();                 // default Material when a source has none
    uint64_t hash() const;                   // content hash for the BVH cache
};

struct Bvh {
    std::vector<rt_bvh_node> nodes;
    std::vector<int32_t> tri_indices;        // values = 3 * triangle index
    int32_t max_depth = 0;
    int32_t num_leaves = 0;
    double build_seconds = 0.0;
};

rt_material default_material();              // Material() (Mesh.h:37-41)
rt_material diffuse_material(float r, float g, float b);

int load_obj(const std::string& path, Mesh& m, std::string& err);
// ColladaLoader::load + Mesh::init(ColladaLoader&) (collada.cpp); save_dae writes that subset.
int load_dae(const std::string& path, Mesh& m, std::string& err);
int save_dae(const std::string& path, const Mesh& m, std::string& err);
void gen_cornell(Mesh& m);
void gen_torus_knot(Mesh& m, int nu, int nv);
void gen_heightfield(Mesh& m, int nx, int nz, float amplitude, uint32_t seed, float x0, float x1, float z0,
                     float z1);
void gen_random(Mesh& m, int ntris, float extent, float size, uint32_t seed);
void append_grid(Mesh& dst, const Mesh& src, int gx, int gz, float dx, float dz, float scale);

void build_bvh(const Mesh& m, int max_leaf, int num_threads, Bvh& out);
// The reference SplitBVHBuilder (SplitBVHBuilder.cpp:41-476) + BVH_Cuda::build_from_bvh2, same bytes.
void build_sbvh(const Mesh& m, int num_threads, Bvh& out);

// Camera (Camera.cpp:6-68): orbit around the origin; angles accumulate in float as the reference's do.
struct Camera {
    float eye[3] = {0, 0, 0}, center[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    float cam_radius = 200.0f, cam_alpha = 0.0f, cam_beta = 0.0f;
    float right[3] = {0, 0, 0}, cup[3] = {0, 0, 0}, dir[3] = {0, 0, 0};
    explicit Camera(float radius);
    void add_rotate(float da, float db);
    void add_radius(float dr);
    void update_eye();
};
rt_params frame_params(const Camera& cam, const Mesh& m, uint32_t w, uint32_t h, const float* light_pos,
                       const float* light_color);

rt_params camera_params(const Mesh& m, uint32_t w, uint32_t h, float radius, float extra_alpha,
                        float extra_beta, const float* light_pos, const float* light_color);

}  // namespace rtamd
