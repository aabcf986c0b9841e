// scene.cpp -- Mesh utilities, OBJ loader, synthetic scene generators, camera.
#include "scene.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>

namespace rtamd {

static inline rt_float4 f4(float x, float y, float z, float w = 1.0f) { return rt_float4{x, y, z, w}; }

rt_material default_material() {
    // Material() (Mesh.h:37-41): PHONG, emission 0, ambient 0, diffuse 1, specular 1,
    // shininess 2, reflective 1, reflectivity 1, transparent 1, transparency 0, glossiness 1.
    rt_material m;
    std::memset(&m, 0, sizeof m);
    m.technique.x = 1;
    m.emission = f4(0, 0, 0, 1);
    m.ambient = f4(0, 0, 0, 1);
    m.diffuse = f4(1, 1, 1, 1);
    m.specular = f4(1, 1, 1, 1);
    m.shininess.x = 2;
    m.reflective = f4(1, 1, 1, 1);
    m.reflectivity.x = 1;
    m.transparent = f4(1, 1, 1, 1);
    m.transparency.x = 0;
    m.glossiness.x = 1.0f;
    return m;
}

rt_material diffuse_material(float r, float g, float b) {
    rt_material m = default_material();
    m.technique.x = 2;  // COOK_TORRANCE (ColladaLoader.h Effect)
    m.diffuse = f4(r, g, b, 1);
    return m;
}

void Mesh::update_bounds() {
    // Mesh.cpp:55-61: first vertex initialises, then fminf1/fmaxf1 (a<b?a:b).
    for (size_t i = 0; i < vertices.size(); ++i) {
        const float v[3] = {vertices[i].x, vertices[i].y, vertices[i].z};
        for (int k = 0; k < 3; ++k) {
            if (i == 0) {
                scene_min[k] = v[k];
                scene_max[k] = v[k];
            } else {
                scene_min[k] = v[k] < scene_min[k] ? v[k] : scene_min[k];
                scene_max[k] = v[k] > scene_max[k] ? v[k] : scene_max[k];
            }
        }
    }
}

void Mesh::ensure_normals() {
    if (!normals.empty() && normals_indices.size() == indices.size()) return;
    std::vector<double> acc(vertices.size() * 3, 0.0);
    for (size_t t = 0; t + 2 < indices.size(); t += 3) {
        const rt_float4 &a = vertices[indices[t]], &b = vertices[indices[t + 1]], &c = vertices[indices[t + 2]];
        double e1[3] = {b.x - (double)a.x, b.y - (double)a.y, b.z - (double)a.z};
        double e2[3] = {c.x - (double)a.x, c.y - (double)a.y, c.z - (double)a.z};
        double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        for (int k = 0; k < 3; ++k)
            for (int j = 0; j < 3; ++j) acc[(size_t)indices[t + k] * 3 + j] += n[j];
    }
    normals.resize(vertices.size());
    for (size_t i = 0; i < vertices.size(); ++i) {
        double x = acc[3 * i], y = acc[3 * i + 1], z = acc[3 * i + 2];
        double l = std::sqrt(x * x + y * y + z * z);
        if (l > 0) { x /= l; y /= l; z /= l; } else { x = 0; y = 1; z = 0; }
        normals[i] = f4((float)x, (float)y, (float)z, 1.0f);
    }
    normals_indices = indices;
}

void Mesh::ensure_materials() {
    if (materials.empty()) materials.push_back(default_material());
    if (tri_to_material.size() != indices.size() / 3) tri_to_material.assign(indices.size() / 3, 0);
}

uint64_t Mesh::hash() const {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](const void* p, size_t n) {
        const unsigned char* c = (const unsigned char*)p;
        for (size_t i = 0; i < n; ++i) { h ^= c[i]; h *= 1099511628211ull; }
    };
    uint64_t nv = vertices.size(), ni = indices.size();
    mix(&nv, 8); mix(&ni, 8);
    mix(vertices.data(), vertices.size() * sizeof(rt_float4));
    mix(indices.data(), indices.size() * sizeof(int32_t));
    return h;
}

// ---- OBJ: loadObj (RayTracer.cpp:1008-1100) + Mesh::init(TriangleMesh&) (Mesh.cpp:80-130) ----
int load_obj(const std::string& path, Mesh& m, std::string& err) {
    std::ifstream in(path.c_str());
    if (!in.good()) { err = "cannot open " + path; return -1; }
    std::vector<float> vs, ns;
    std::vector<int> fv, fn;
    bool have_vn_faces = true;
    std::string line;
    while (std::getline(in, line)) {
        const char* b = line.c_str();
        float a1, a2, a3;
        if (b[0] == 'v' && b[1] == 'n' && b[2] == ' ') {
            if (std::sscanf(b, "vn %f %f %f", &a1, &a2, &a3) != 3) { err = "bad vn"; return -1; }
            ns.push_back(a1); ns.push_back(a2); ns.push_back(a3);
        } else if (b[0] == 'v' && b[1] == ' ') {
            if (std::sscanf(b, "v %f %f %f", &a1, &a2, &a3) != 3) { err = "bad v"; return -1; }
            vs.push_back(a1); vs.push_back(a2); vs.push_back(a3);
        } else if (b[0] == 'f' && b[1] == ' ') {
            int v[3], n[3], t[3];
            if (std::sscanf(b, "f %d//%d %d//%d %d//%d", &v[0], &n[0], &v[1], &n[1], &v[2], &n[2]) == 6) {
            } else if (std::sscanf(b, "f %d/%d/%d %d/%d/%d %d/%d/%d", &v[0], &t[0], &n[0], &v[1], &t[1], &n[1],
                                   &v[2], &t[2], &n[2]) == 9) {
            } else if (std::sscanf(b, "f %d %d %d", &v[0], &v[1], &v[2]) == 3) {
                n[0] = n[1] = n[2] = 0;
                have_vn_faces = false;
            } else {
                err = "unsupported face format: " + line;
                return -1;
            }
            for (int k = 0; k < 3; ++k) { fv.push_back(v[k] - 1); fn.push_back(n[k] - 1); }
        }
    }
    m = Mesh();
    int nv = (int)(vs.size() / 3);
    m.vertices.resize(nv);
    for (int i = 0; i < nv; ++i) m.vertices[i] = f4(vs[3 * i], vs[3 * i + 1], vs[3 * i + 2], 1.0f);
    m.indices = fv;
    for (int i : fv)
        if (i < 0 || i >= nv) { err = "face index out of range"; return -1; }
    if (have_vn_faces && !ns.empty()) {
        int nn = (int)(ns.size() / 3);
        m.normals.resize(nn);
        for (int i = 0; i < nn; ++i) {
            // Mesh.cpp:125-128: normals[i] = normalize(normals[i]) with w = 0 (float4 zero-init)
            // using vectors_math normalize (invLen = 1/sqrtf(dot4)).
            float x = ns[3 * i], y = ns[3 * i + 1], z = ns[3 * i + 2], w = 0.0f;
            float d = x * x + y * y + z * z + w * w;
            float inv = 1.0f / std::sqrt(d);
            m.normals[i] = f4(inv * x, inv * y, inv * z, inv * w);
        }
        m.normals_indices = fn;
        for (int i : fn)
            if (i < 0 || i >= nn) { err = "normal index out of range"; return -1; }
    } else {
        m.ensure_normals();
    }
    m.ensure_materials();
    m.update_bounds();
    return 0;
}

// ---- C1: Cornell-style room: floor + 4 walls (10 tris) + floating quad (2 tris) ----
void gen_cornell(Mesh& m) {
    m = Mesh();
    m.materials.push_back(diffuse_material(0.73f, 0.73f, 0.73f));  // white
    m.materials.push_back(diffuse_material(0.65f, 0.05f, 0.05f));  // red
    m.materials.push_back(diffuse_material(0.12f, 0.45f, 0.15f));  // green
    m.materials.push_back(diffuse_material(0.20f, 0.30f, 0.80f));  // blue quad
    const float R = 80.0f;
    auto quad = [&m](rt_float4 a, rt_float4 b, rt_float4 c, rt_float4 d, rt_float4 n, int mat) {
        int base = (int)m.vertices.size();
        m.vertices.push_back(a); m.vertices.push_back(b); m.vertices.push_back(c); m.vertices.push_back(d);
        int nb = (int)m.normals.size();
        m.normals.push_back(n);
        const int tri[6] = {0, 1, 2, 0, 2, 3};
        for (int k = 0; k < 6; ++k) { m.indices.push_back(base + tri[k]); m.normals_indices.push_back(nb); }
        m.tri_to_material.push_back(mat); m.tri_to_material.push_back(mat);
    };
    quad(f4(-R, -R, -R), f4(-R, -R, R), f4(R, -R, R), f4(R, -R, -R), f4(0, 1, 0), 0);     // floor
    quad(f4(R, -R, -R), f4(R, -R, R), f4(R, R, R), f4(R, R, -R), f4(-1, 0, 0), 1);        // +x wall
    quad(f4(-R, -R, R), f4(-R, R, R), f4(R, R, R), f4(R, -R, R), f4(0, 0, -1), 2);        // +z wall
    quad(f4(-R, -R, -R), f4(-R, R, -R), f4(-R, R, R), f4(-R, -R, R), f4(1, 0, 0), 0);     // -x wall
    quad(f4(-R, -R, -R), f4(R, -R, -R), f4(R, R, -R), f4(-R, R, -R), f4(0, 0, 1), 0);     // -z wall
    const float s = 0.7071067811865476f;
    quad(f4(-30, 10, -30), f4(-30, 40, 30), f4(30, 40, 30), f4(30, 10, -30), f4(0, s, -s), 3);  // tilted quad
    m.update_bounds();
}

// ---- C2: (2,3) torus knot tube, 2*nu*nv triangles, smooth analytic normals ----
void gen_torus_knot(Mesh& m, int nu, int nv) {
    m = Mesh();
    m.materials.push_back(diffuse_material(0.8f, 0.55f, 0.2f));
    const double P = 2, Q = 3, Rk = 45.0, rk = 20.0, tube = 11.0;
    auto curve = [&](double t, double* c) {
        double r = Rk + rk * std::cos(Q * t);
        c[0] = r * std::cos(P * t);
        c[1] = rk * std::sin(Q * t) * 1.6;
        c[2] = r * std::sin(P * t);
    };
    m.vertices.resize((size_t)nu * nv);
    m.normals.resize((size_t)nu * nv);
    for (int i = 0; i < nu; ++i) {
        double t = 2.0 * M_PI * i / nu, c0[3], c1[3];
        curve(t, c0);
        curve(t + 1e-4, c1);
        double T[3] = {c1[0] - c0[0], c1[1] - c0[1], c1[2] - c0[2]};
        double lt = std::sqrt(T[0] * T[0] + T[1] * T[1] + T[2] * T[2]);
        for (double& x : T) x /= lt;
        double up[3] = {0, 1, 0};
        double N[3] = {T[1] * up[2] - T[2] * up[1], T[2] * up[0] - T[0] * up[2], T[0] * up[1] - T[1] * up[0]};
        double ln = std::sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
        for (double& x : N) x /= ln;
        double B[3] = {T[1] * N[2] - T[2] * N[1], T[2] * N[0] - T[0] * N[2], T[0] * N[1] - T[1] * N[0]};
        for (int j = 0; j < nv; ++j) {
            double a = 2.0 * M_PI * j / nv;
            double d[3];
            for (int k = 0; k < 3; ++k) d[k] = std::cos(a) * N[k] + std::sin(a) * B[k];
            size_t id = (size_t)i * nv + j;
            m.vertices[id] = f4((float)(c0[0] + tube * d[0]), (float)(c0[1] + tube * d[1]),
                                (float)(c0[2] + tube * d[2]), 1.0f);
            m.normals[id] = f4((float)d[0], (float)d[1], (float)d[2], 1.0f);
        }
    }
    for (int i = 0; i < nu; ++i)
        for (int j = 0; j < nv; ++j) {
            int a = i * nv + j, b = ((i + 1) % nu) * nv + j, c = ((i + 1) % nu) * nv + (j + 1) % nv,
                d = i * nv + (j + 1) % nv;
            const int q[6] = {a, b, c, a, c, d};
            for (int k = 0; k < 6; ++k) m.indices.push_back(q[k]);
        }
    m.normals_indices = m.indices;
    m.tri_to_material.assign(m.indices.size() / 3, 0);
    m.update_bounds();
}

// ---- C3: value-noise heightfield, nx*nz cells, 2 tris per cell, over [x0,x1] x [z0,z1] ----
static inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
static double lattice(int i, int j, uint32_t seed) {
    uint32_t h = hash32((uint32_t)i * 0x9E3779B1u ^ hash32((uint32_t)j + seed * 0x85EBCA77u));
    return (h & 0xFFFFFF) / (double)0xFFFFFF * 2.0 - 1.0;
}
static double value_noise(double x, double y, uint32_t seed) {
    int i = (int)std::floor(x), j = (int)std::floor(y);
    double fx = x - i, fy = y - j;
    double sx = fx * fx * (3 - 2 * fx), sy = fy * fy * (3 - 2 * fy);
    double a = lattice(i, j, seed), b = lattice(i + 1, j, seed), c = lattice(i, j + 1, seed),
           d = lattice(i + 1, j + 1, seed);
    return (a + (b - a) * sx) + ((c + (d - c) * sx) - (a + (b - a) * sx)) * sy;
}
static double fbm(double x, double y, uint32_t seed) {
    double s = 0, amp = 1, f = 1, norm = 0;
    for (int o = 0; o < 5; ++o) {
        s += amp * value_noise(x * f, y * f, seed + o * 101);
        norm += amp;
        amp *= 0.5;
        f *= 2.03;
    }
    return s / norm;
}

void gen_heightfield(Mesh& m, int nx, int nz, float amplitude, uint32_t seed, float x0, float x1, float z0, float z1) {
    m = Mesh();
    m.materials.push_back(diffuse_material(0.35f, 0.6f, 0.3f));
    m.materials.push_back(diffuse_material(0.6f, 0.5f, 0.4f));
    const double X0 = x0, X1 = x1, Z0 = z0, Z1 = z1;
    const int vx = nx + 1, vz = nz + 1;
    auto height = [&](double x, double z) { return amplitude * fbm(x * 0.04, z * 0.04, seed) - 20.0; };
    m.vertices.resize((size_t)vx * vz);
    m.normals.resize((size_t)vx * vz);
    const double dx = (X1 - X0) / nx, dz = (Z1 - Z0) / nz;
    for (int j = 0; j < vz; ++j)
        for (int i = 0; i < vx; ++i) {
            double x = X0 + dx * i, z = Z0 + dz * j;
            double y = height(x, z);
            double hx = height(x + 0.05, z) - height(x - 0.05, z), hz = height(x, z + 0.05) - height(x, z - 0.05);
            double n[3] = {-hx / 0.1, 1.0, -hz / 0.1};
            double l = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            size_t id = (size_t)j * vx + i;
            m.vertices[id] = f4((float)x, (float)y, (float)z, 1.0f);
            m.normals[id] = f4((float)(n[0] / l), (float)(n[1] / l), (float)(n[2] / l), 1.0f);
        }
    m.indices.reserve((size_t)nx * nz * 6);
    m.tri_to_material.reserve((size_t)nx * nz * 2);
    for (int j = 0; j < nz; ++j)
        for (int i = 0; i < nx; ++i) {
            int a = j * vx + i, b = a + 1, c = a + vx + 1, d = a + vx;
            const int q[6] = {a, d, c, a, c, b};
            for (int k = 0; k < 6; ++k) m.indices.push_back(q[k]);
            int mat = ((i / 25) + (j / 50)) & 1;
            m.tri_to_material.push_back(mat);
            m.tri_to_material.push_back(mat);
        }
    m.normals_indices = m.indices;
    m.update_bounds();
}

// ---- random triangle soup (BVH / traversal stress) ----
void gen_random(Mesh& m, int ntris, float extent, float size, uint32_t seed) {
    m = Mesh();
    m.materials.push_back(diffuse_material(0.9f, 0.3f, 0.3f));
    m.materials.push_back(diffuse_material(0.3f, 0.9f, 0.3f));
    m.materials.push_back(diffuse_material(0.3f, 0.3f, 0.9f));
    uint32_t s = seed ? seed : 1;
    auto rnd = [&s]() {
        s = hash32(s + 0x9E3779B9u);
        return (s & 0xFFFFFF) / (float)0xFFFFFF;
    };
    for (int t = 0; t < ntris; ++t) {
        float c[3] = {(rnd() * 2 - 1) * extent, (rnd() * 2 - 1) * extent, (rnd() * 2 - 1) * extent};
        for (int k = 0; k < 3; ++k) {
            m.vertices.push_back(f4(c[0] + (rnd() * 2 - 1) * size, c[1] + (rnd() * 2 - 1) * size,
                                    c[2] + (rnd() * 2 - 1) * size, 1.0f));
            m.indices.push_back(3 * t + k);
        }
        m.tri_to_material.push_back(t % 3);
    }
    m.ensure_normals();
    m.update_bounds();
}

void append_grid(Mesh& dst, const Mesh& src, int gx, int gz, float dx, float dz, float scale) {
    for (int iz = 0; iz < gz; ++iz)
        for (int ix = 0; ix < gx; ++ix) {
            float ox = (ix - (gx - 1) * 0.5f) * dx, oz = (iz - (gz - 1) * 0.5f) * dz;
            int vbase = (int)dst.vertices.size(), nbase = (int)dst.normals.size(),
                mbase = (int)dst.materials.size();
            for (const rt_float4& v : src.vertices)
                dst.vertices.push_back(f4(v.x * scale + ox, v.y * scale, v.z * scale + oz, 1.0f));
            dst.normals.insert(dst.normals.end(), src.normals.begin(), src.normals.end());
            dst.materials.insert(dst.materials.end(), src.materials.begin(), src.materials.end());
            for (int i : src.indices) dst.indices.push_back(vbase + i);
            for (int i : src.normals_indices) dst.normals_indices.push_back(nbase + i);
            for (int i : src.tri_to_material) dst.tri_to_material.push_back(mbase + i);
        }
    dst.update_bounds();
}

// ---- Camera (Camera.cpp:6-68) + updateCamera (RayTracer.cpp:609-672) ----
namespace {
struct V3 { float x, y, z; };
// vectors_math.cpp:73-84 (no contraction: host code is built with -ffp-contract=off)
inline float dotv(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 crossv(V3 a, V3 b) { return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline V3 normv(V3 v) {
    float inv = 1.0f / std::sqrt(dotv(v, v));
    return V3{inv * v.x, inv * v.y, inv * v.z};
}
inline V3 scalev(float s, V3 a) { return V3{s * a.x, s * a.y, s * a.z}; }
inline V3 addv(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }

}  // namespace

Camera::Camera(float radius) : cam_radius(radius) {  // Camera() (Camera.cpp:6-19)
    add_rotate((float)(45 * (3 + 2) * M_PI / 180.0f), (float)(45 * M_PI / 180.0f));
}

void Camera::add_rotate(float da, float db) {  // Camera.cpp:26-46
    cam_alpha += da;
    cam_beta += db;
    if (cam_beta < 0.0f) cam_beta = (float)(cam_beta + 2.0f * M_PI);
    else if (cam_beta > 2.0f * M_PI) cam_beta = (float)(cam_beta - 2.0f * M_PI);
    if ((cam_beta > M_PI / 2.0f) && (cam_beta < 3.0f * M_PI / 2.0f)) up[0] = 0.0f, up[1] = -1.0f, up[2] = 0.0f;
    else up[0] = 0.0f, up[1] = 1.0f, up[2] = 0.0f;
    update_eye();
}

void Camera::add_radius(float dr) {  // Camera.cpp:21-24
    cam_radius += dr;
    update_eye();
}

void Camera::update_eye() {  // Camera.cpp:48-68 (update_eye + update_full)
    eye[0] = center[0] + cam_radius * std::cos(cam_beta) * std::cos(cam_alpha);
    eye[1] = center[1] + cam_radius * std::sin(cam_beta);
    eye[2] = center[2] + cam_radius * std::cos(cam_beta) * std::sin(cam_alpha);
    const V3 e{eye[0], eye[1], eye[2]}, u{up[0], up[1], up[2]};
    const V3 d = normv(V3{center[0] - e.x, center[1] - e.y, center[2] - e.z});
    const V3 r = normv(crossv(d, u));
    const V3 cu = crossv(d, r);
    const V3 c = normv(V3{-cu.x, -cu.y, -cu.z});
    dir[0] = d.x; dir[1] = d.y; dir[2] = d.z;
    right[0] = r.x; right[1] = r.y; right[2] = r.z;
    cup[0] = c.x; cup[1] = c.y; cup[2] = c.z;
}

// updateCamera (RayTracer.cpp:609-672): Params from the camera, the frame size and the scene box
rt_params frame_params(const Camera& cam, const Mesh& m, uint32_t w, uint32_t h, const float* light_pos,
                       const float* light_color) {
    const float FOV = 60.0f;
    float theta = (float)((FOV * 3.1415 * 0.5) / 180.0f);
    float half_width = std::tan(theta);
    float aspect = (float)w / (float)h;
    float u0 = -half_width * aspect, v0 = -half_width, u1 = half_width * aspect, v1 = half_width;
    float dist_to_image = 1;
    const V3 right{cam.right[0], cam.right[1], cam.right[2]}, cup{cam.cup[0], cam.cup[1], cam.cup[2]};
    const V3 dir{cam.dir[0], cam.dir[1], cam.dir[2]}, eye{cam.eye[0], cam.eye[1], cam.eye[2]};
    V3 a = scalev(u1 - u0, right);
    V3 b = scalev(v1 - v0, cup);
    V3 c = addv(addv(addv(eye, scalev(u0, right)), scalev(v0, cup)), scalev(dist_to_image, dir));
    const float lp_def[3] = {-23.0f, 200.0f, 3.0f}, lc_def[3] = {1.0f, 1.0f, 1.0f};
    const float* lp = light_pos ? light_pos : lp_def;
    const float* lc = light_color ? light_color : lc_def;
    rt_params p;
    p.a = f4(a.x, a.y, a.z, 1.0f);
    p.b = f4(b.x, b.y, b.z, 1.0f);
    p.c = f4(c.x, c.y, c.z, 1.0f);
    p.campos = f4(eye.x, eye.y, eye.z, 1.0f);
    p.light_pos = f4(lp[0], lp[1], lp[2], 1.0f);
    p.light_color = f4(lc[0], lc[1], lc[2], 1.0f);
    p.scene_aabb_min = f4(m.scene_min[0], m.scene_min[1], m.scene_min[2], 1.0f);
    p.scene_aabb_max = f4(m.scene_max[0], m.scene_max[1], m.scene_max[2], 1.0f);
    return p;
}

rt_params camera_params(const Mesh& m, uint32_t w, uint32_t h, float radius, float extra_alpha,
                        float extra_beta, const float* light_pos, const float* light_color) {
    Camera cam(radius);
    if (extra_alpha != 0.0f || extra_beta != 0.0f) cam.add_rotate(extra_alpha, extra_beta);
    return frame_params(cam, m, w, h, light_pos, light_color);
}

}  // namespace rtamd
