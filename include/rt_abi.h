/*
 * rt_abi.h -- C ABI of the MI355X render path (the drop-in boundary).
 *
 * Replaces the reference's OpenCL host glue for kernel `raytracer_bvh`
 * (x64/Release/volumeRender.cl:1043-1075).  Every entry point cites the
 * reference code it stands in for.  Plain pointers and sizes only; no C++,
 * torch or HIP types cross this boundary.
 *
 * Binary layouts are the reference's, byte for byte:
 *   rt_bvh_node  == BVH_Node_            (BVH_Cuda.h:12-29)      48 B
 *   rt_material  == Material             (Mesh.h:20-67)          176 B
 *   rt_params    == Params / Params2     (RayTracer.cpp:115-161,
 *                                         volumeRender.cl:320-330) 128 B
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_float4 { float x, y, z, w; } rt_float4;
typedef struct rt_int4 { int32_t x, y, z, w; } rt_int4;

/* BVH_Cuda.h:12-29 -- AABB{float4 min,max} + child/leaf words.
 * Inner node: offset_left/right >= 0, offset_tris = -1, num_tris = 0.
 * Leaf: offset_left = offset_right = -1, tris [offset_tris, +num_tris) of the
 * reference-index array (values = 3 * triangle index, BVH_Cuda.h:90-93).
 * Root = node 0; pre-order, left subtree first (BVH_Cuda.h:98-137). */
typedef struct rt_bvh_node {
    rt_float4 min, max;
    int32_t offset_left, offset_right, offset_tris, num_tris;
} rt_bvh_node;

/* Mesh.h:20-67; the live kernel reads only .diffuse (volumeRender.cl:1381). */
typedef struct rt_material {
    rt_int4 technique;
    rt_float4 emission, ambient, diffuse, specular, shininess;
    rt_float4 reflective, reflectivity, transparent, transparency, glossiness;
} rt_material;

/* RayTracer.cpp:115-161 (w components = 1). */
typedef struct rt_params {
    rt_float4 a, b, c, campos, light_pos, light_color, scene_aabb_min, scene_aabb_max;
} rt_params;

#ifdef __cplusplus
static_assert(sizeof(rt_bvh_node) == 48, "BVH_Node_ is 48 bytes");
static_assert(sizeof(rt_material) == 176, "Material is 176 bytes");
static_assert(sizeof(rt_params) == 128, "Params is 128 bytes");
#endif

/* Status codes (the reference used cl_int + CHECK_OPENCL_ERROR,
 * RayTracer.cpp:338-344; the kernel itself has no error channel). */
enum {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = -1,
    RT_ERR_DEVICE = -2,      /* HIP runtime error; see rt_last_error() */
    RT_ERR_NO_SCENE = -3,
    RT_ERR_OUT_OF_MEMORY = -4,
    RT_ERR_BAD_SCENE = -5    /* index out of range in the uploaded arrays */
};

/* rt_render flags.
 * Arithmetic.  Without a math flag the kernel computes S_ref: the
 * reference kernel exactly as the reference host builds it (RayTracer.cpp:2173,
 * clBuildProgram with no options: OpenCL-default contraction, 2.5-ulp `/`, 3-ulp
 * sqrt, the device library's rsqrt/pow) -- the same pixels as the reference on
 * gfx950.  The two flags below select the alternatives. */
enum {
    RT_FLAG_NO_SHADOW = 1u,  /* config C2 "primary rays only": skip the any-hit shadow ray
                                (volumeRender.cl:1437-1460); coefficient stays 1 */
    RT_FLAG_HW_MATH = 2u,    /* S_hw arithmetic: the reference built with
                                -cl-fp32-correctly-rounded-divide-sqrt -ffp-contract=off
                                (IEEE `/` and sqrt, no contraction, the device library's
                                rsqrt/pow: v_rsq_f32, __ocml_pow_f32) */
    RT_FLAG_STRICT_MATH = 64u, /* S_strict arithmetic: S_hw with rsqrt and pow(x,5) computed in
                                binary64 and rounded, reproducible on any IEEE host: the CPU
                                oracle's arithmetic (oracle/rt_oracle.c).  Excludes RT_FLAG_HW_MATH. */
    RT_FLAG_WAVEFRONT = 8u,  /* wavefront mode: bounce 0 over screen tiles, then one
                                launch per further bounce over a compacted queue of the rays still in
                                flight, instead of the fused one-lane-per-pixel kernel; bit-identical.
                                Depth-1 frames always run as that first launch alone. */
    RT_FLAG_WF_SORT = 32u,   /* with RT_FLAG_WAVEFRONT: sort each bounce's queue before tracing it, within
                                screen-local chunks of 1024 rays, by the direction component along the scene
                                box's thinnest axis (8 buckets; stable), so that rays of similar length share
                                waves; pixels are identical either way */
    RT_FLAG_EXACT_DIV = 4u,  /* force the division form of the slab test (volumeRender.cl:614-615) instead
                                of the bit-identical fast quotient; for A/B only */
    RT_FLAG_STATIC_ORDER = 16u /* keep the static XCD-dealt block order instead of the adaptive
                                longest-first order built from the per-block times of the context's
                                latest rebuild launch on the stream slot (every 8th launch;
                                RTAMD_LPT_EVERY); pixels are identical either way */
};

#define RT_MAX_DEPTH 8       /* reference: RAY_TRACE_DEPTH 3 (volumeRender.cl:12) */

typedef struct rt_ctx rt_ctx;

/* Optional per-pixel side outputs (parity instrumentation).
 * hits : int32 [P][depth][2] -- closest-hit id and shadow-hit id per bounce,
 *        id = 3 * triangle index (volumeRender.cl:983), -1 = miss, -2 = not traced
 * t    : float [P][depth]    -- closest-hit t per bounce (-1 = not traced)
 * rgb  : float [P][3]        -- colour before the x255 pack (volumeRender.cl:1545) */
typedef struct rt_aux {
    int32_t* hits;
    float* t;
    float* rgb;
} rt_aux;

/* Screen sharding for multi-GPU.  Rows are cut into bands of
 * band_rows rows; band b belongs to rank b % nranks.  A rank's output buffer
 * holds only its bands, in increasing band order, each band_rows*w pixels
 * (the last band may be short).  nranks = 1 renders the whole frame. */
typedef struct rt_tiling {
    int32_t rank, nranks, band_rows, reserved;
} rt_tiling;

/* Replaces setupCL's device/queue selection (RayTracer.cpp:2370-2433,
 * CreateContext :2050, CreateCommandQueue :2097). */
int rt_create(int device, rt_ctx** out);

/* Replaces initRayTrace's clCreateBuffer(COPY_HOST_PTR) block
 * (RayTracer.cpp:942-984) and initCLVolume2's argument setup (:1234-1261).
 * Deep-copies the caller's arrays (caller keeps ownership) and builds the
 * device-side layouts.  Arg numbers refer to raytracer_bvh (volumeRender.cl:1043):
 *   verts/nv        arg 6  mesh_vertices        float4[nv]
 *   idx/nidx        arg 7  mesh_indices         int[nidx]  (3 per triangle)
 *   nodes/nn        arg 8  bvh_nodes            BVH_Node_[nn]   (arg 11 = nn)
 *   refs/nref       arg 9  bvh_tris_indices     int[nref]        (arg 10 = nref)
 *   normals/nnorm   arg 13 mesh_normals         float4[nnorm]
 *   normal_idx      arg 14 mesh_normals_indices int[nidx]
 *   mats/nmat       arg 15 mesh_materials       Material[nmat]
 *   tri_to_mat      arg 16 tri -> material      int[nidx/3]
 * Args 3/4 (brute-force triangle list, NULL/0 in the live path) and 12
 * (debug `temp`) are dead in the reference and are not part of the ABI. */
int rt_upload_scene(rt_ctx* ctx, const rt_float4* verts, int32_t nv, const int32_t* idx, int32_t nidx,
                    const rt_bvh_node* nodes, int32_t nn, const int32_t* refs, int32_t nref,
                    const rt_float4* normals, int32_t nnorm, const int32_t* normal_idx,
                    const rt_material* mats, int32_t nmat, const int32_t* tri_to_mat);

/* Multi-GPU scene distribution ("ncclBroadcast of scene buffers at load").
 * The reference uploads one scene to its one device (RayTracer.cpp:942-984); here one
 * rank builds and uploads it, packs its device layouts into ONE contiguous device
 * buffer (the "scene image"), that buffer is broadcast over RCCL, and every other rank
 * loads it -- the Collada parse and the SBVH build run once per node, not per GPU.
 *   rt_scene_image_size : bytes of ctx's scene image
 *   rt_scene_image_pack : device-to-device copy of ctx's scene into d_image (synchronizes stream)
 *   rt_scene_image_load : replace ctx's scene by the image's (synchronizes stream)
 * The image is position-independent device data: pack on one ctx, load on any other. */
int rt_scene_image_size(rt_ctx* ctx, uint64_t* bytes);
int rt_scene_image_pack(rt_ctx* ctx, void* d_image, uint64_t bytes, void* stream);
int rt_scene_image_load(rt_ctx* ctx, const void* d_image, uint64_t bytes, void* stream);

/* Replaces updateCamera's clEnqueueWriteBuffer of Params (RayTracer.cpp:671). */
int rt_set_params(rt_ctx* ctx, const rt_params* params);

/* Replaces raytrace_gpgpu (RayTracer.cpp:330-344): launch, finish, blocking
 * readback of w*h packed pixels (b<<16 | g<<8 | r).  depth = number of bounces
 * (reference: 3).  aux may be NULL.  Synchronous. */
int rt_render(rt_ctx* ctx, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, uint32_t* out_bgr,
              const rt_aux* aux);

/* raytrace_gpgpu (RayTracer.cpp:330-344) on n GPUs from ONE process (SURVEY.md 7.5, 8b:
 * the reference has one device and one queue, RayTracer.cpp:2097-2131).  ctxs[0..n-1] are
 * distinct contexts (one per GPU; the same device may repeat), each holding the scene
 * (rt_upload_scene, or rt_scene_copy from one that does).  The camera is ctxs[0]'s
 * (rt_set_params; copied to the others).  The frame is cut into 8-row bands dealt round-robin
 * (band b -> ctxs[b % n]); every context renders its bands on its own stream and
 * writes each pixel straight into its row of the host frame: the caller's out_bgr when every
 * context's device maps it (hipHostGetDevicePointer on each device: hipHostMalloc'd portable
 * memory, or memory registered and mapped for all of them), else a portable pinned staging frame
 * of ctxs[0] copied to out_bgr after the join.  ctxs[1..n-1] enqueue and wait on host threads of
 * their own (started on first use, spinning between frames, stopped by rt_destroy), ctxs[0] on
 * the caller's thread (RTAMD_TILED_WORKERS=0: all on the caller's thread, in turn).  Synchronous:
 * returns when every context is done and out_bgr holds the w*h packed pixels -- the same pixels
 * as rt_render with the same flags.  n == 1 is rt_render.  Errors are reported on ctxs[0]
 * (rt_last_error). */
int rt_render_tiled(rt_ctx** ctxs, int32_t n, uint32_t w, uint32_t h, int32_t depth, uint32_t flags,
                    uint32_t* out_bgr);
/* rt_render_tiled's choice of frame, on its own so that it is testable without a GPU: given for
 * each of n contexts the device address its device resolved for the caller's host buffer (0 = that
 * device cannot address it), 1 when every context can write the buffer directly (all resolved,
 * 16-B aligned), 0 when the frame must go through the pinned staging frame. */
int32_t rt_tiled_direct_ok(int32_t n, const uint64_t* dev_addrs);
/* Host steady-clock nanoseconds at the start and end of the context's last rt_render_device
 * enqueue (rt_render_tiled's parts included): the spread of the starts over a tiled frame's
 * contexts is how far apart their GPUs start. */
int rt_last_enqueue_time(rt_ctx* ctx, uint64_t* begin_ns, uint64_t* end_ns);
/* Copies src's uploaded scene (its device layouts) into dst: device to device on one GPU,
 * peer to peer over xGMI between two (hipMemcpyPeer), with no host round trip and no second
 * BVH build (initRayTrace's upload, RayTracer.cpp:942-984, done once per node).  Synchronous. */
int rt_scene_copy(rt_ctx* dst, rt_ctx* src);

/* Device-resident variant for benchmarks and multi-GPU: renders this rank's
 * bands (tiling may be NULL = whole frame) into device buffers d_out (and the
 * optional device aux planes), enqueued on `stream` (a hipStream_t, NULL =
 * the ctx stream).  Returns after enqueue; nothing is copied to the host. */
int rt_render_device(rt_ctx* ctx, uint32_t w, uint32_t h, int32_t depth, uint32_t flags,
                     const rt_tiling* tiling, uint32_t* d_out, const rt_aux* d_aux, void* stream);

#ifndef RT_MAX_BATCH
#define RT_MAX_BATCH 8
#endif
/* Throughput mode of rt_render_device: nframes (1..RT_MAX_BATCH) frames of one size, frame i
 * with camera params[i] (updateCamera's Params, RayTracer.cpp:609-672; every params[i] must
 * carry the same scene box), rendered by ONE launch into d_out + i * frame_stride (pixels,
 * frame_stride >= the rank's pixels).  The reference renders one frame per raytrace_gpgpu
 * (RayTracer.cpp:330-344); a caller that keeps several frames in flight -- a frame loop, a
 * server -- gets the longest tiles of all of them scheduled first in one grid instead of on
 * separate streams.  depth 1 (primary + shadow ray, RT_FLAG_NO_SHADOW for primary
 * only), or depth > 1 with RT_FLAG_WAVEFRONT: bounce 0 of every frame in one launch, then each
 * bounce launch over all frames' ray queues; such a batch needs one light position for all frames
 * (the reference's light is a global, RayTracer.cpp:60).  No aux planes; every frame's pixels equal rt_render_device's for its camera.
 * Asynchronous like rt_render_device; rt_last_timing is the launch (all nframes frames).
 * The ctx's own params (rt_set_params) are neither read nor changed. */
int rt_render_device_batch(rt_ctx* ctx, uint32_t w, uint32_t h, int32_t depth, uint32_t flags,
                           const rt_tiling* tiling, const rt_params* params, int32_t nframes, uint32_t* d_out,
                           uint64_t frame_stride, void* stream);
/* The synchronous form (raytrace_gpgpu's launch + finish + blocking read-back, RayTracer.cpp:330-344,
 * for nframes frames of one launch): out_bgr receives nframes * w*h packed pixels, frame i at
 * out_bgr + i * w*h, the same as rt_render with params[i] for each.  Same depth / light rules as
 * rt_render_device_batch.  Pinned, device-mapped out_bgr is written by the kernels directly. */
int rt_render_batch(rt_ctx* ctx, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, const rt_params* params,
                    int32_t nframes, uint32_t* out_bgr);

/* Number of pixels a rank owns under `tiling` (size of its output buffer). */
int64_t rt_tiling_pixels(uint32_t w, uint32_t h, const rt_tiling* tiling);

/* Rank 0 after the per-frame gather: re-interleaves the ranks'
 * band buffers into the frame in ONE kernel launch on `stream`.  d_slots holds
 * nranks buffers of slot_pixels pixels each (rank r's at d_slots + r*slot_pixels,
 * its bands in the rt_tiling order); d_frame receives w*h pixels.  Replaces the
 * single-device readback target of RayTracer.cpp:343 (the frame the reference
 * hands to glDrawPixels).  Asynchronous: returns after enqueue. */
int rt_assemble_bands(uint32_t* d_frame, const uint32_t* d_slots, uint64_t slot_pixels, uint32_t w, uint32_t h,
                      int32_t nranks, int32_t band_rows, void* stream);
/* The same for nframes frames in one launch: rank r's slot (at d_slots + r*slot_pixels)
 * holds the frames' band buffers frame_pixels apart; d_frame receives nframes frames of
 * w*h pixels, one after the other. */
int rt_assemble_bands_batch(uint32_t* d_frame, const uint32_t* d_slots, uint64_t slot_pixels, uint64_t frame_pixels,
                            int32_t nframes, uint32_t w, uint32_t h, int32_t nranks, int32_t band_rows, void* stream);

/* Native band exchange for multi-GPU frames over RCCL: the reference
 * reads the frame back to the host (RayTracer.cpp:343); here every rank's bands go to
 * rank 0, which re-interleaves them into the frame.  The 128-byte id travels from rank 0
 * to the others over any channel (bench.py: the torch.distributed store). */
typedef struct rt_comm rt_comm;
int rt_comm_unique_id(uint8_t* id, int32_t id_bytes);
/* One communicator per rank, with its own gather stream and (rank 0) assembly stream,
 * both at the device's highest stream priority. */
int rt_comm_create(int32_t device, int32_t nranks, int32_t rank, const uint8_t* id, int32_t id_bytes, rt_comm** out);
int rt_comm_destroy(rt_comm* comm);
const char* rt_comm_last_error(void);
/* The frame path (bench.py --gather native).  The caller cycles buffer sets, "slots"
 * 0..63, each carrying a batch of nframes consecutive frames: slot j = one band buffer
 * d_bands of nframes * frame_pixels (every rank; frame f's bands at f * frame_pixels) and,
 * on rank 0, one (nranks * nframes * frame_pixels) d_slots + nframes * w*h d_frames.
 * On the batch's render stream:
 *   rt_frame_slot_wait(comm, j, stream)   -- the stream waits for slot j's last gather
 *                                            (it read d_bands), not for later ones;
 *   rt_render_device(..., d_bands + f * frame_pixels, ..., stream) for each frame f;
 *   rt_frame_exchange(comm, j, nframes, ...) -- after the renders: ncclGather to rank 0 on
 *                                            the communicator's stream (issue order = batch
 *                                            order, the same on every rank), then rank 0's
 *                                            rt_assemble_bands_batch on its assembly stream.
 * rt_frame_ready_wait(comm, j, stream): a consumer stream waits for slot j's frames
 * (rank 0: assembled; other ranks: sent).  All calls return after enqueue. */
int rt_frame_exchange(rt_comm* comm, int32_t slot, int32_t nframes, const uint32_t* d_bands, uint64_t frame_pixels,
                      uint32_t* d_slots, uint32_t* d_frames, uint32_t w, uint32_t h, int32_t band_rows, void* stream);
int rt_frame_slot_wait(rt_comm* comm, int32_t slot, void* stream);
int rt_frame_ready_wait(rt_comm* comm, int32_t slot, void* stream);
/* The same exchange entirely on `stream` (gather, then rank 0's assembly), for a caller with
 * one stream per communicator.  Every rank calls it once per frame, in the same order. */
int rt_frame_gather(rt_comm* comm, const uint32_t* d_bands, uint64_t slot_pixels, uint32_t* d_slots,
                    uint32_t* d_frame, uint32_t w, uint32_t h, int32_t band_rows, void* stream);

/* Collective-free frame exchange (bench.py --gather ipc).  Rank 0 exports its framebuffers
 * with rt_ipc_export (the 64-byte handle of the allocation they lie in + their offset in it)
 * and passes both to the other ranks (any channel), which map the allocation with rt_ipc_open
 * (d_base; the frames are at d_base + offset); then every rank, after rendering a frame's
 * bands, places them into rank 0's frame with rt_bands_put on its own stream: one copy
 * kernel, a block per row, writing whole rows (over xGMI for the other ranks).  Rank 0
 * puts its own bands the same way into its local frame.  rt_bands_put itself carries no
 * completion signal; the frame path uses rt_bands_put_sync + rt_frame_present below, which
 * tell rank 0 when each frame is complete.  Replaces
 * the host readback of RayTracer.cpp:343 for a frame rendered on N GPUs. */
int rt_ipc_export(int32_t device, void* d_ptr, uint8_t* handle, int32_t handle_bytes, uint64_t* offset);
int rt_ipc_open(int32_t device, const uint8_t* handle, int32_t handle_bytes, void** d_base);
int rt_ipc_close(int32_t device, void* d_base);
int rt_bands_put(const uint32_t* d_bands, uint32_t* d_frame, uint32_t w, uint32_t h, const rt_tiling* tiling,
                 void* stream);
/* Rank 0's shared frames + sync block for the IPC exchange: other GPUs write them over xGMI
 * while rank 0's kernels poll and read them, so they must be coherent across devices during
 * kernels -- uncached device memory (hipExtMallocWithFlags(hipDeviceMallocUncached)), zeroed,
 * exportable with rt_ipc_export.  (Coarse-grained hipMalloc memory is coherent only at kernel
 * boundaries.)  rt_copy_device: a device-to-device copy on `stream` (frame checks). */
int rt_shared_alloc(int32_t device, uint64_t bytes, void** d_ptr);
int rt_shared_free(int32_t device, void* d_ptr);
int rt_copy_device(void* d_dst, const void* d_src, uint64_t bytes, void* stream);
/* Whether `device` can map `peer`'s memory (hipDeviceCanAccessPeer; 1 for device == peer).
 * bench.py maps rank 0's frames only when every rank can; otherwise it uses the RCCL gather. */
int rt_peer_access(int32_t device, int32_t peer, int32_t* can);

/* Per-frame completion of the band puts.  The reference hands back a complete frame every
 * frame: clFinish + blocking read (RayTracer.cpp:340-343).  Here rank 0 keeps a sync block of
 * rt_frame_sync_words(nsets, nranks) uint32 words next to its frames (zeroed once, mapped into
 * every rank with them); frame buffer sets 0..nsets-1 are reused in turn, `use` counting the
 * times a set has been filled (0, 1, 2, ...).  Per frame:
 *   every rank: rt_bands_put_sync(..., d_sync, d_local, nsets, set, use, timeout, stream) --
 *     first waits until rank 0 has presented the set's previous use (no rank ever overwrites
 *     a frame rank 0 has not observed complete) -- one wave of its own waits, bounded, before the
 *     put's blocks start (RTAMD_PUT_WAIT=stream: hipStreamWaitValue32 instead, which ROCm runs as
 *     its own polling blit kernel without a bound; =kernel: every put block waits) --, then copies its rows (as rt_bands_put), then
 *     publishes "use done" for this rank with a system-scope release; d_local = nsets uint32
 *     counters in the rank's own memory, zeroed once;
 *   rank 0, after its own put: rt_frame_present(d_sync, nsets, set, use, nranks, timeout,
 *     release, stream) -- one wave that waits for every rank's publication of (set, use),
 *     acquires and counts the frame as presented.  Work enqueued on `stream` after it sees
 *     the complete frame.  With release != 0 it also hands the set back to the ranks for its
 *     next use; otherwise rank 0 calls rt_frame_release(d_sync, nsets, set, use, stream)
 *     after the frame's consumers (a display copy, a checksum) on that stream.
 * Waits are bounded (timeout_ms, 0 = 10 s); a timeout sets a status instead of hanging, and a
 * present that times out also releases every set (waits in flight end; their puts write nothing):
 * rt_frame_sync_status reads it (0 ok, 1 a put timed out, 2 a present timed out) and the
 * number of frames presented (synchronous).  rt_frame_checksum adds a position-dependent
 * 64-bit sum of a frame's pixels into *d_sum (frame checks). */
int64_t rt_frame_sync_words(int32_t nsets, int32_t nranks);
int rt_bands_put_sync(const uint32_t* d_bands, uint32_t* d_frame, uint32_t w, uint32_t h, const rt_tiling* tiling,
                      uint32_t* d_sync, uint32_t* d_local, int32_t nsets, int32_t set, uint32_t use, uint32_t timeout_ms,
                      void* stream);
int rt_frame_present(uint32_t* d_sync, int32_t nsets, int32_t set, uint32_t use, int32_t nranks, uint32_t timeout_ms,
                     int32_t release, void* stream);
int rt_frame_release(uint32_t* d_sync, int32_t nsets, int32_t set, uint32_t use, void* stream);
int rt_frame_sync_status(const uint32_t* d_sync, uint32_t* status, uint32_t* presented);
int rt_frame_checksum(const uint32_t* d_frame, uint64_t pixels, uint64_t* d_sum, void* stream);

/* Kernel-side timing of the last render, from HIP events on the launch stream
 * (ms): total_ms = every kernel of the frame (counter reset / block-order
 * build, the first-bounce or fused render kernel, further bounces);
 * traverse_ms = the frame's main kernel alone (first_bounce_kernel for depth 1
 * and the wavefront path, else the fused render kernel: what the roofline is
 * computed on). */
int rt_last_timing(rt_ctx* ctx, float* total_ms, float* traverse_ms);
/* The same two times averaged over the last n frames (n <= 64 and <= frames
 * rendered): bench.py reads the timed steps' kernel time this way, without a
 * host sync inside its timed loop. */
int rt_timing_average(rt_ctx* ctx, int32_t n, float* total_ms, float* traverse_ms);

/* Measurement: the traversal's record fetches and their ceiling.
 * rt_fetch_counts renders one frame (flags as rt_render; whole frame, static block order;
 * depth 1, or any depth on the wavefront path: every launch of the frame) with the counting
 * instantiation of the fast kernels and returns, summed over the frame: out[0..7] = inner /
 * triangle lane-fetches, inner / triangle QUAD requests (distinct records per quad of lanes
 * per wave iteration: the vector-memory path merges a quad's lanes that read one record),
 * inner / triangle records distinct per wave iteration, wave iterations, and those whose
 * active lanes mix inner and triangle steps.  Traversals restarted with the general code
 * (stacks deeper than the LDS part; rt_last_deferred) are not counted.  The pixel path itself
 * never counts (a separate kernel instantiation).
 * rt_gather_peak measures the ceiling those requests run into: every lane of 8 waves per
 * SIMD on every CU reads pseudo-random inner-record-shaped records from a table of
 * table_records 64-B records, iters (multiple of 4) per lane: ms per launch and records read. */
int rt_fetch_counts(rt_ctx* ctx, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, uint64_t* out8);
int rt_gather_peak(rt_ctx* ctx, uint32_t table_records, uint32_t iters, float* ms, uint64_t* records);
/* rt_chase_peak measures the other roof, latency: every wave of 8 per SIMD on every CU walks
 * a chain of `iters` dependent traversal-shaped iterations (three 16-B + one 8-B load of a
 * 64-B record, a dependent slab-like computation, the next record picked from the record's
 * two references) through a table of table_records records, `group` lanes (1, 2, 4, ..., 64)
 * following one chain: ms per launch and the number of waves (ms / iters = one dependent
 * iteration of a wave with the chip full). */
int rt_chase_peak(rt_ctx* ctx, uint32_t table_records, uint32_t iters, uint32_t group, float* ms, uint64_t* waves);
/* The same chain on `blocks` blocks of 4 waves instead of 8 per CU: blocks = the CU count
 * gives one wave per SIMD (a lone chain's iteration time on an otherwise idle chip). */
int rt_chase_latency(rt_ctx* ctx, uint32_t table_records, uint32_t iters, uint32_t group, uint32_t blocks, float* ms,
                     uint64_t* waves);
/* Where a frame's time goes (diagnostics): renders `frames` (1..8) frames in flight, frame f on
 * its own stream (flags as rt_render, default arithmetic; depth 1, or the wavefront path), with
 * a stamping instantiation of the same kernels, after a few untimed rounds on the same streams
 * (so with the adaptive block order the product uses).  words[0] = launches L (<= 32),
 * words[1] = frames, words[2] / [3] = the first frame's kernels / its first launch (HIP events,
 * ns); per launch i: words[8 + i] = its waves, words[40 + i] = its frame, words[72 + i] = its
 * bounce (0 = the first launch); from word 128, 16 words per wave, launch after launch, waves in
 * blockIdx * 4 + wave order: s_memrealtime (100 MHz, low 32 bits) at the wave's start, when its
 * closest-hit traversal returned, when its shading was done, at the end of its rays and at its
 * end (after the block epilogue of a launch that rebuilds the longest-first order, every 8th on
 * a stream slot: the order build in its last block; other launches have no epilogue); its
 * closest-hit main-loop and wave-uniform-prologue trips and the same two for its shadow rays;
 * HW_REG_XCC_ID; HW_REG_HW_ID; the tile it rendered (first launch) or the 64-ray groups it took
 * (bounce launches; trips summed over them, times of the last); s_memrealtime when the closest-hit
 * traversal started and when its wave-uniform prologue ended; 2 zero words.
 * *used_words = words written. */
int rt_wave_timeline(rt_ctx* ctx, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, int32_t frames, uint32_t* words,
                     uint64_t cap_words, uint64_t* used_words);

/* Traversals of the last frame that outgrew the fast kernel's LDS stack and
 * restarted in-kernel with the general traversal (same result, slower ray);
 * diagnostics, synchronizes the stream. */
int rt_last_deferred(rt_ctx* ctx, uint32_t* count);

/* Device stack-overflow counter (reference: silent miss, volumeRender.cl:914). */
int rt_overflow_count(rt_ctx* ctx, uint64_t* count);

/* Releases all device memory (RayTraceData::~RayTraceData, RayTracer.cpp:208-228). */
int rt_destroy(rt_ctx* ctx);

/* Last error message for ctx (or the global one when ctx is NULL). */
const char* rt_last_error(rt_ctx* ctx);

/* ABI version for loaders. */
int rt_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* RT_ABI_H */
