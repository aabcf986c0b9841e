// rt_frameloop -- headless stand-in for the reference's interactive GLUT loop
// (SURVEY.md 8f #4): displayGL = updateCamera + render (RayTracer.cpp:284-293),
// the FPS title once a second (:497-516), and the right-button orbit drag
// (motion, :553-565: add_rotate(dx * 0.25 / 100, dy * 0.25 / 100)), driven by a
// fixed per-frame drag instead of a mouse.  Frames go through the C ABI exactly
// as the reference's host path does: rt_set_params (clEnqueueWriteBuffer of
// Params, :671) then rt_render (launch + finish + blocking read-back, :330-344).
// Optional PPM dumps replace the window.  With --gpus N (devices 0..N-1) or --devices a,b,...
// (a list; a device may repeat) every frame goes to rt_render_tiled over one context per
// entry instead: the scene is uploaded once and copied to the others (rt_scene_copy).  With
// --batch K the orbit's next K cameras go to ONE rt_render_batch call (the throughput mode: K frames
// in one launch, read back together).
//
//   rt_frameloop [--dae F | --obj F | --scene cornell|knot|heightfield] [--bvh-cache F]
//                [--width W] [--height H] [--depth D] [--frames N] [--drag DX DY]
//                [--ppm-dir DIR] [--ppm-every K] [--device I] [--flags F] [--gpus N | --devices a,b,...]
//                [--batch K]
//
// Prints "N.N fps" lines and a final JSON summary.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "rt_host.h"

namespace {

struct Args {
    std::string dae, obj, scene = "heightfield", bvh_cache, ppm_dir;
    uint32_t w = 1024, h = 768;  // RayTracer.cpp:39-40 (WIDTH, HEIGHT)
    int depth = 3, frames = 120, ppm_every = 0, device = 0, batch = 1;
    uint32_t flags = 0;
    float dx = 4.0f, dy = 0.0f;
    std::vector<int> devices;   // rt_render_tiled over these (empty: rt_render on --device)
};

int usage() {
    std::fprintf(stderr,
                 "usage: rt_frameloop [--dae F | --obj F | --scene cornell|knot|heightfield] [--bvh-cache F]\n"
                 "                    [--width W] [--height H] [--depth D] [--frames N] [--drag DX DY]\n"
                 "                    [--ppm-dir DIR] [--ppm-every K] [--device I] [--flags F]\n"
                 "                    [--gpus N | --devices a,b,...] [--batch K]\n");
    return 2;
}

bool parse(int argc, char** argv, Args& a) {
    for (int i = 1; i < argc; ++i) {
        const std::string k = argv[i];
        auto need = [&](int n) { return i + n < argc; };
        if (k == "--dae" && need(1)) a.dae = argv[++i];
        else if (k == "--obj" && need(1)) a.obj = argv[++i];
        else if (k == "--scene" && need(1)) a.scene = argv[++i];
        else if (k == "--bvh-cache" && need(1)) a.bvh_cache = argv[++i];
        else if (k == "--width" && need(1)) a.w = (uint32_t)std::atoi(argv[++i]);
        else if (k == "--height" && need(1)) a.h = (uint32_t)std::atoi(argv[++i]);
        else if (k == "--depth" && need(1)) a.depth = std::atoi(argv[++i]);
        else if (k == "--frames" && need(1)) a.frames = std::atoi(argv[++i]);
        else if (k == "--drag" && need(2)) { a.dx = (float)std::atof(argv[++i]); a.dy = (float)std::atof(argv[++i]); }
        else if (k == "--ppm-dir" && need(1)) a.ppm_dir = argv[++i];
        else if (k == "--ppm-every" && need(1)) a.ppm_every = std::atoi(argv[++i]);
        else if (k == "--device" && need(1)) a.device = std::atoi(argv[++i]);
        else if (k == "--flags" && need(1)) a.flags = (uint32_t)std::strtoul(argv[++i], nullptr, 0);
        else if (k == "--batch" && need(1)) a.batch = std::atoi(argv[++i]);
        else if (k == "--gpus" && need(1)) {
            const int n = std::atoi(argv[++i]);
            if (n < 1 || n > 64) return false;
            a.devices.clear();
            for (int d = 0; d < n; ++d) a.devices.push_back(d);
        } else if (k == "--devices" && need(1)) {
            a.devices.clear();
            for (const char* p = argv[++i]; *p;) {
                char* end = nullptr;
                const long d = std::strtol(p, &end, 10);
                if (end == p || d < 0) return false;
                a.devices.push_back((int)d);
                p = *end == ',' ? end + 1 : end;
                if (*end && *end != ',') return false;
            }
            if (a.devices.empty() || a.devices.size() > 64) return false;
        } else return false;
    }
    return a.w > 0 && a.h > 0 && a.frames > 0 && a.depth >= 0 && a.depth <= RT_MAX_DEPTH && a.batch >= 1 &&
           a.batch <= RT_MAX_BATCH && (a.batch == 1 || a.devices.size() <= 1);
}

// Packed pixels are b<<16 | g<<8 | r (volumeRender.cl:186-195); row 0 is the first image row.
bool write_ppm(const std::string& path, const std::vector<uint32_t>& px, uint32_t w, uint32_t h) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%u %u\n255\n", w, h);
    std::vector<unsigned char> row((size_t)w * 3);
    for (uint32_t y = 0; y < h; ++y) {
        for (uint32_t x = 0; x < w; ++x) {
            const uint32_t p = px[(size_t)y * w + x];
            row[3 * x + 0] = (unsigned char)(p & 0xFF);
            row[3 * x + 1] = (unsigned char)((p >> 8) & 0xFF);
            row[3 * x + 2] = (unsigned char)((p >> 16) & 0xFF);
        }
        std::fwrite(row.data(), 1, row.size(), f);
    }
    return std::fclose(f) == 0;
}

}  // namespace

int main(int argc, char** argv) {
    Args a;
    if (!parse(argc, argv, a)) return usage();
    using clk = std::chrono::steady_clock;

    rt_mesh* mesh = rt_mesh_create();
    int rc;
    if (!a.dae.empty()) rc = rt_mesh_load_dae(mesh, a.dae.c_str());
    else if (!a.obj.empty()) rc = rt_mesh_load_obj(mesh, a.obj.c_str());
    else if (a.scene == "cornell") rc = rt_mesh_gen_cornell(mesh);
    else if (a.scene == "knot") rc = rt_mesh_gen_torus_knot(mesh, 256, 137);
    else if (a.scene == "heightfield") rc = rt_mesh_gen_heightfield(mesh, 500, 1000, 10.0f, 0x5EED, -150, 650, -150, 650);
    else return usage();
    if (rc != RT_OK) { std::fprintf(stderr, "scene load failed (%d)\n", rc); return 1; }

    // BVH: the cache when it matches the mesh, else the reference's spatial-split build
    const auto tb = clk::now();
    rt_bvh* bvh = nullptr;
    bool cached = false;
    if (!a.bvh_cache.empty() && rt_bvh_load(mesh, a.bvh_cache.c_str(), &bvh) == RT_OK) cached = true;
    if (!bvh) {
        if ((rc = rt_bvh_build_sbvh(mesh, 0, &bvh)) != RT_OK) { std::fprintf(stderr, "bvh build failed\n"); return 1; }
        if (!a.bvh_cache.empty()) rt_bvh_save(bvh, mesh, a.bvh_cache.c_str());
    }
    const double bvh_s = std::chrono::duration<double>(clk::now() - tb).count();

    rt_mesh_view mv;
    rt_bvh_view bv;
    rt_mesh_view_get(mesh, &mv);
    rt_bvh_view_get(bvh, &bv);
    // one context per GPU entry (a single one on --device without --gpus / --devices)
    if (a.devices.empty()) a.devices.push_back(a.device);
    std::vector<rt_ctx*> ctxs(a.devices.size(), nullptr);
    for (size_t k = 0; k < ctxs.size(); ++k)
        if ((rc = rt_create(a.devices[k], &ctxs[k])) != RT_OK) {
            std::fprintf(stderr, "rt_create(%d): %s\n", a.devices[k], rt_last_error(nullptr));
            return 1;
        }
    rt_ctx* ctx = ctxs[0];
    rc = rt_upload_scene(ctx, mv.vertices, mv.num_vertices, mv.indices, mv.num_indices, bv.nodes, bv.num_nodes,
                         bv.tri_indices, bv.num_tri_indices, mv.normals, mv.num_normals, mv.normals_indices,
                         mv.materials, mv.num_materials, mv.tri_to_material);
    if (rc != RT_OK) { std::fprintf(stderr, "rt_upload_scene: %s\n", rt_last_error(ctx)); return 1; }
    for (size_t k = 1; k < ctxs.size(); ++k)   // the scene once per node: copied, not re-uploaded
        if ((rc = rt_scene_copy(ctxs[k], ctx)) != RT_OK) {
            std::fprintf(stderr, "rt_scene_copy: %s\n", rt_last_error(ctxs[k]));
            return 1;
        }
    const int32_t nctx = (int32_t)ctxs.size();
    // batches deeper than one bounce run in the wavefront mode (the same pixels as the fused kernel)
    if (a.batch > 1 && a.depth > 1) a.flags |= RT_FLAG_WAVEFRONT;

    rt_camera* cam = rt_camera_create(200.0f);
    const size_t npx = (size_t)a.w * a.h;
    std::vector<uint32_t> px(npx * (size_t)a.batch), one;
    std::vector<rt_params> cams((size_t)a.batch);
    int frames_in_second = 0, total = 0;
    double kernel_ms_sum = 0.0;
    auto t0 = clk::now(), tsec = t0;
    for (int f0 = 0; f0 < a.frames; f0 += a.batch) {
        const int k = std::min(a.batch, a.frames - f0);   // this call's frames f0 .. f0 + k - 1
        for (int i = 0; i < k; ++i) {
            if (f0 + i > 0) rt_camera_add_rotate(cam, a.dx * 0.25f / 100.0f, a.dy * 0.25f / 100.0f);  // motion()
            rt_camera_frame_params(cam, mesh, a.w, a.h, nullptr, nullptr, &cams[(size_t)i]);     // updateCamera()
        }
        if (a.batch > 1) {
            rc = rt_render_batch(ctx, a.w, a.h, a.depth, a.flags, cams.data(), k, px.data());
        } else if ((rc = rt_set_params(ctx, &cams[0])) == RT_OK) {
            rc = nctx > 1 ? rt_render_tiled(ctxs.data(), nctx, a.w, a.h, a.depth, a.flags, px.data())
                          : rt_render(ctx, a.w, a.h, a.depth, a.flags, px.data(), nullptr);
        }
        if (rc != RT_OK) {
            std::fprintf(stderr, "frame %d: %s\n", f0, rt_last_error(ctx));
            return 1;
        }
        float kt = 0.0f, kk = 0.0f;
        if (rt_last_timing(ctx, &kt, &kk) == RT_OK) kernel_ms_sum += kt;   // the call's kernels (k frames)
        frames_in_second += k;
        total += k;
        for (int i = 0; i < k; ++i) {
            const int f = f0 + i;
            if (a.ppm_every > 0 && !a.ppm_dir.empty() && f % a.ppm_every == 0) {
                char name[64];
                std::snprintf(name, sizeof name, "/frame_%05d.ppm", f);
                one.assign(px.begin() + (ptrdiff_t)(npx * (size_t)i), px.begin() + (ptrdiff_t)(npx * (size_t)(i + 1)));
                if (!write_ppm(a.ppm_dir + name, one, a.w, a.h)) std::fprintf(stderr, "cannot write %s\n", name);
            }
        }
        const auto now = clk::now();
        const double since = std::chrono::duration<double>(now - tsec).count();
        if (since >= 1.0) {  // update(): the window title's fps, once a second
            std::printf("%.1f fps\n", frames_in_second / since);
            std::fflush(stdout);
            frames_in_second = 0;
            tsec = now;
        }
    }
    const double wall = std::chrono::duration<double>(clk::now() - t0).count();
    std::printf("{\"frames\": %d, \"width\": %u, \"height\": %u, \"depth\": %d, \"fps\": %.2f, \"ms_per_frame\": %.4f, "
                "\"kernel_ms_per_frame\": %.4f, \"triangles\": %d, \"bvh_nodes\": %d, \"bvh_cached\": %s, "
                "\"bvh_seconds\": %.3f, \"contexts\": %d, \"frames_per_call\": %d}\n",
                total, a.w, a.h, a.depth, total / wall, 1e3 * wall / total, kernel_ms_sum / total,
                mv.num_indices / 3, bv.num_nodes, cached ? "true" : "false", bvh_s, nctx, a.batch);
    rt_camera_destroy(cam);
    for (rt_ctx* c : ctxs) rt_destroy(c);
    rt_bvh_destroy(bvh);
    rt_mesh_destroy(mesh);
    return 0;
}
