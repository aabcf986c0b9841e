/*
 * rt_host.h -- C ABI of the host-side scene tools that feed the render path.
 *
 * These produce exactly the arrays the reference hands to its kernel:
 *   Mesh       (Mesh.h:69-101, Mesh.cpp:10-141)   indices/vertices/normals/materials
 *   BVH arrays (BVH_Cuda.h:87-137)                 BVH_Node_[] + tri_indices[] (= 3*tri)
 *   Params     (Camera.cpp:6-68, RayTracer.cpp:609-672)
 * Two BVH builders: rt_bvh_build_sbvh is the reference's spatial-split
 * builder (same bytes, parallel); rt_bvh_build is this framework's own
 * binned-SAH builder (object splits only, leaf size 1..8, SAH node/tri cost
 * 1/1 as BVH2.cpp:11-20) in the reference's node layout and ordering.
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include "rt_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_mesh rt_mesh;
typedef struct rt_bvh rt_bvh;

/* Read-only view of a mesh's arrays (valid until the mesh is modified/destroyed). */
typedef struct rt_mesh_view {
    const rt_float4* vertices; int32_t num_vertices;
    const int32_t* indices; int32_t num_indices;          /* 3 per triangle */
    const rt_float4* normals; int32_t num_normals;
    const int32_t* normals_indices;                       /* num_indices entries */
    const rt_material* materials; int32_t num_materials;
    const int32_t* tri_to_material;                       /* num_indices/3 entries */
    float scene_min[3], scene_max[3];                     /* Mesh::scene_aabbox_min/max */
} rt_mesh_view;

typedef struct rt_bvh_view {
    const rt_bvh_node* nodes; int32_t num_nodes;
    const int32_t* tri_indices; int32_t num_tri_indices;
    int32_t max_depth, num_leaves;
    double build_seconds;
} rt_bvh_view;

rt_mesh* rt_mesh_create(void);
void rt_mesh_destroy(rt_mesh* m);
int rt_mesh_view_get(const rt_mesh* m, rt_mesh_view* out);

/* Build a mesh from caller arrays (copied).  normals may be NULL: then one
 * normal per vertex is computed (area-weighted face normals, normalized).
 * mats may be NULL: one default Material (Mesh.h:37-41) is used. */
int rt_mesh_set(rt_mesh* m, const rt_float4* verts, int32_t nv, const int32_t* idx, int32_t nidx,
                const rt_float4* normals, int32_t nnorm, const int32_t* nidx_arr,
                const rt_material* mats, int32_t nmat, const int32_t* tri_to_mat);

/* Wavefront OBJ subset, as the reference's loadObj (RayTracer.cpp:1008-1100):
 * `v`, `vn`, `f a b c`, `f a//n b//n c//n`, `f a/t/n ...`; then Mesh::init(TriangleMesh&)
 * (Mesh.cpp:80-130): indices -1, normals normalized; default material. */
int rt_mesh_load_obj(rt_mesh* m, const char* path);
/* Collada subset, as the reference's ColladaLoader::load (ColladaLoader.cpp:13-593)
 * followed by Mesh::init(ColladaLoader&) (Mesh.cpp:10-78): effects -> materials,
 * first <polygons> of each geometry (9-int <p> per triangle), per-node matrix or
 * rotate/translate transform; linear time (the reference's lookups are O(n^2)).
 * Quirks and deviations are listed in csrc/host/collada.cpp. */
int rt_mesh_load_dae(rt_mesh* m, const char* path);
/* Writes the mesh as that Collada subset (the synthetic-scene generator of
 * SURVEY.md 8d); rt_mesh_load_dae reads it back to the same arrays. */
int rt_mesh_save_dae(const rt_mesh* m, const char* path);

/* Synthetic scenes. All fit the reference's default
 * orbit camera (radius 200 around the origin). */
int rt_mesh_gen_cornell(rt_mesh* m);                                    /* C1: 12 triangles */
int rt_mesh_gen_torus_knot(rt_mesh* m, int32_t nu, int32_t nv);          /* C2: 2*nu*nv tris */
/* C3: value-noise heightfield over [x0,x1] x [z0,z1], 2*nx*nz triangles */
int rt_mesh_gen_heightfield(rt_mesh* m, int32_t nx, int32_t nz, float amplitude, uint32_t seed, float x0, float x1,
                            float z0, float z1);
int rt_mesh_gen_random(rt_mesh* m, int32_t ntris, float extent, float size, uint32_t seed);
/* Append `src` translated on a gx x gz grid with spacing (dx, dz) (C5 merge). */
int rt_mesh_append_grid(rt_mesh* dst, const rt_mesh* src, int32_t gx, int32_t gz, float dx, float dz,
                        float scale);

/* Binned-SAH BVH over the mesh; emits BVH_Node_ pre-order + tri_indices (x3). */
int rt_bvh_build(const rt_mesh* m, int32_t max_leaf, int32_t num_threads, rt_bvh** out);
/* The reference's spatial-split BVH: FW::BVH2(mesh) -> SplitBVHBuilder::run
 * (SplitBVHBuilder.cpp:41-476, BVH2.cpp:11-31) -> BVH_Cuda::build_from_bvh2
 * (BVH_Cuda.h:87-137).  Same BVH_Node_ and tri_indices bytes, built in
 * parallel (num_threads <= 0: all cores); replaces the reference's
 * single-threaded 317 s build of a 1M-triangle mesh. */
int rt_bvh_build_sbvh(const rt_mesh* m, int32_t num_threads, rt_bvh** out);
int rt_bvh_view_get(const rt_bvh* b, rt_bvh_view* out);
void rt_bvh_destroy(rt_bvh* b);
/* BVH cache file (nodes + refs + mesh hash), SURVEY.md 5 "checkpoint". */
int rt_bvh_save(const rt_bvh* b, const rt_mesh* m, const char* path);
int rt_bvh_load(const rt_mesh* m, const char* path, rt_bvh** out);

/* Camera (Camera.cpp) + updateCamera (RayTracer.cpp:609-672) -> Params.
 * The default camera is Camera() = radius 200, add_rotate(225 deg, 45 deg);
 * extra_alpha/extra_beta (radians) are further add_rotate() calls (orbit).
 * light_pos/light_color NULL -> reference defaults (-23,200,3) / (1,1,1)
 * (RayTracer.cpp:57-63); scene box from the mesh. */
int rt_camera_params(const rt_mesh* m, uint32_t w, uint32_t h, float radius, float extra_alpha,
                     float extra_beta, const float* light_pos, const float* light_color, rt_params* out);

/* Orbit camera of the interactive loop (Camera.cpp:6-68): rt_camera_create = Camera()
 * with the given radius (reference: 200), add_rotate / add_radius as the mouse handlers
 * call them (RayTracer.cpp:553-565, dx * 0.25 / 100 radians per pixel), and
 * rt_camera_frame_params = updateCamera (RayTracer.cpp:609-672) for one frame. */
typedef struct rt_camera rt_camera;
rt_camera* rt_camera_create(float radius);
void rt_camera_destroy(rt_camera* c);
int rt_camera_add_rotate(rt_camera* c, float da, float db);
int rt_camera_add_radius(rt_camera* c, float dr);
int rt_camera_frame_params(const rt_camera* c, const rt_mesh* m, uint32_t w, uint32_t h, const float* light_pos,
                           const float* light_color, rt_params* out);

#ifdef __cplusplus
}
#endif

#endif /* RT_HOST_H */
