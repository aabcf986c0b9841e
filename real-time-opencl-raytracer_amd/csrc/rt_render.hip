// rt_render.hip -- MI355X (gfx950) render path: device layouts, kernels, C ABI.
//
// Replaces the reference's per-pixel OpenCL kernel raytracer_bvh
// (x64/Release/volumeRender.cl:1043-1547) and its host glue (RayTracer.cpp).
// Results follow the reference kernel's arithmetic exactly (S_ref,
// the reference as its host builds it, by default; S_strict and S_hw by flag);
// what changes is how the data sits in HBM and how the traversal is scheduled:
//
//  * inner BVH nodes are re-laid out as 64-B records that carry BOTH child
//    boxes plus the two child references (one 64-B fetch per inner visit
//    instead of the reference's 16 B node word + 2 x 32 B child boxes in two
//    dependent rounds, volumeRender.cl:836-867);
//  * a child reference encodes leaf-ness and the leaf's triangle range, so a
//    leaf never costs a node fetch;
//  * triangle references are expanded into 48-B {v0, e1, e2, id} records in
//    leaf order (the reference's 4-level ref -> index -> vertex gather,
//    volumeRender.cl:965-974, becomes one contiguous 48-B read);
//  * per-triangle shading data (3 vertices, 3 normals, albedo) is one 112-B
//    record (volumeRender.cl:1306-1374 gathers from five arrays);
//  * the 65-entry traversal stack (volumeRender.cl:636) lives in LDS for its
//    first RTK_LDS_STACK entries, laid out [entry][lane] (bank-conflict free),
//    the rest spills to a per-pixel global region; the top of stack stays in a
//    register.  Stack semantics (including the overflow -> miss rule at 65)
//    are the reference's, entry for entry;
//  * one wave = one 8x8 pixel tile (the reference's work-group, lanes in Morton
//    order), 4 waves per block; each lane takes one step of its own reference
//    sequence per iteration (traverse_ifif), so a wave's length is its slowest
//    ray, not the sum of its lanes' leaf rounds;
//  * blocks run longest-first, ordered by the previous frame's per-block times;
//    the frame's last-finishing block builds that order in-kernel (no extra launch);
//  * frame scratch is per stream, so frames enqueued on different streams run
//    concurrently (frames in flight; multi-GPU band gather overlaps rendering).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rt_abi.h"

#ifndef RTK_WF_WAVES
#define RTK_WF_WAVES 7      // waves per SIMD the wavefront kernels are bounded to
#endif
#ifndef RTK_FBN_REF_WAVES
#define RTK_FBN_REF_WAVES 8 // waves per SIMD the S_ref depth > 1 first-bounce kernel is bounded to
#endif
#ifndef RTK_SEL_NEXT
#define RTK_SEL_NEXT 0      // offset select (SEL) in the depth > 1 first-bounce kernel too
#endif
#ifndef RTK_WFB_REF_WAVES
#define RTK_WFB_REF_WAVES 8 // waves per SIMD the S_ref bounce kernel is bounded to
#endif
#ifndef RTK_WF_GRID_PCT
#define RTK_WF_GRID_PCT 50  // persistent bounce grid, percent of the blocks the chip holds at once (C5 with
                            // 8 frames per launch: 38 / 44 / 50 / 56 / 62 / 68 / 75 % -> 0.758 / 0.752 / 0.750 / 0.753 /
                            // 0.755 / 0.760 / 0.757 ms, one frame per launch 0.827 vs 0.836 at 75 %, one frame alone
                            // 1.28 vs 1.25: profiles/r06/ab/c5_grid_pct_ab*.txt; round 4 at one frame per launch: 75 %)
#endif
#ifndef RTK_FB_WAVES
#define RTK_FB_WAVES 8      // waves per SIMD the S_ref depth-1 kernel is bounded to
#endif
#ifndef RTK_EXT_EVENTS
#define RTK_EXT_EVENTS 1    // one-launch frames: timing events from hipExtLaunchKernel, no marker packets
                            // around the launch (C2 0.0747 vs 0.0764 ms, rt_render into pageable memory 0.527
                            // vs 0.548 ms; C3, C5 equal: profiles/r05/ab/ext_events_ab.log)
#endif
#ifndef RTK_SHADE_EXP
#define RTK_SHADE_EXP 0     // A/B experiments on the shading fetch only (2: none; pixels wrong)
#endif
#ifndef RTK_FAST_ENTRY
#define RTK_FAST_ENTRY 0    // 1: frame kernels' entry without vector loads (the block's tile through the
                            // scalar cache, the block size a constant): wave set-up 6.4 vs 7.3 us, but C3 /
                            // C5 equal and C2 0.0757 vs 0.0747 ms (profiles/r05/ab/fast_entry_ab.log)
#endif
#ifndef RTK_LDS_STACK
#define RTK_LDS_STACK 16    // LDS part of the traversal stack (C3 peaks at 9; deeper rays restart)
#endif
#ifndef RTK_XFRAME
#define RTK_XFRAME 1        // a batch launch's bounce queues tile-major, frame-minor (first_bounce_batch_kernel; 0: frame-major)
#endif

namespace rtk {

constexpr int kStackSize = 65;                       // volumeRender.cl:636
constexpr float kTmin = 0.001f;                      // volumeRender.cl:640
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kRefError = 0x7FFFFFFFu;          // popped -> traversal returns -1
constexpr uint32_t kCntEscape = 31u;
constexpr int kLdsStack = RTK_LDS_STACK;
constexpr int kGlobalStack = 64 - kLdsStack;         // slots kLdsStack..63
constexpr uint32_t kBlockPx = 16;                    // a block = 2 x 2 tiles of 8 x 8 pixels
constexpr uint32_t kBlockThreads = 256;              // every frame kernel's block: 4 waves, one tile each

struct DevScene {
    const float4* __restrict__ wnodes;   // [n_inner][4]
    const float4* __restrict__ tris;     // [n_refs][3] triangle reference records (tri_rec)
    const float4* __restrict__ shade;    // [n_tris][7]
    const int2* __restrict__ leaf_table; // escape leaves {offset, count}
    uint32_t tri_off;                    // byte offset of tris from wnodes (one allocation)
    uint32_t rec_bytes;                  // bytes of that allocation
    uint32_t root;
    uint32_t n_inner;                    // inner records; the first ones are the BVH's top levels (BFS order)
    int fast_div;                        // every box coordinate is 0 or in [2^-66, 2^60]
    int clean;                           // no reachable malformed inner node (kRefError)
};

// Triangle reference record k (leaf order): {v0.xyz, id}, {e1}, {e2}, 48 B.  (A 40-B
// record -- two 16-B loads + one 8-B load -- measured 5.6 % slower on C3: DESIGN.md 6.2.)
__device__ __forceinline__ const float4* tri_rec(const DevScene& S, int k) { return S.tris + (size_t)k * 3; }

struct Frame {
    float3 a, b, c, campos, light_pos, smin, smax;
    uint32_t w, h;
    int32_t depth;
    uint32_t flags;
    int32_t rank, nranks, band_rows;
    uint32_t local_rows;
    uint32_t tiles_x, tiles_y, num_blocks;   // blocks of kBlockPx x kBlockPx pixels
    const uint32_t* tile_order;   // [num_blocks] block -> tile (static column strips, or longest-first)
    uint32_t* tile_cost;          // [num_blocks] per-tile time of this frame (adaptive order), or null
    uint32_t* lpt_next;           // [num_blocks] longest-first order for the next frame on this slot
    uint32_t* done;               // blocks finished so far (the last one builds lpt_next)
    uint32_t* zero_next;          // the other parity's frame counters, zeroed by this frame
    uint32_t nzero;
    uint32_t* t0;                 // the launch's start (block 0's s_memrealtime), for RTK_LPT_BIAS
};

// A ray in flight between bounces: {pix, o.xyz}, {d.xyz, shadow_sum}, {colour.xyz, 3 * triangle it leaves from}.
struct QRay {
    float4 a, b, c;
};
// Ray queues are SEGMENTED: segment s holds slots [64 s, 64 s + 64) and the rays one wave
// appended, packed from its first slot; seg_cnt[s] says how many.  The producer's wave of
// segment s is a screen tile's 8x8 pixels (bounce 0) or the 64-ray group s of the previous
// bounce's order, so the segments are in screen order and no append contends for a counter.
// The producer also adds each count to its chunk's (kChunkSegs segments) and super-chunk's (1024
// segments) sum, from which wf_compact_sort_kernel's blocks find where their chunk starts
// in the bounce's dense order `perm` (compacted, optionally sorted), with no scan launch.
#ifndef RTK_SORT_SCALE
#define RTK_SORT_SCALE 4    // bounce sort: 2 x this many direction buckets over [-1, 1], one frame per launch
#endif
#ifndef RTK_SORT_SCALE_BATCH
#define RTK_SORT_SCALE_BATCH 8   // the same for launches of >= 4 frames (a chunk holds one tile of every frame, RTK_XFRAME:
                                 // C5 0.744 vs 0.753 ms with 8 buckets; one frame per launch loses with 16: profiles/r06/ab/)
#endif
#ifndef RTK_CHUNK_SEGS
#define RTK_CHUNK_SEGS 32   // segments per sort chunk (C5: 16 -> 0.900 ms, 32 -> 0.881, 64 -> 0.900; profiles/r04/ab/sort_chunk_ab.log)
#endif
constexpr uint32_t kChunkSegs = RTK_CHUNK_SEGS, kSuperSegs = 1024;
struct WQ {
    const QRay* in;           // this bounce's rays (segmented)
    const uint32_t* in_count; // rays in it
    const uint32_t* perm;     // dense order of `in`: i -> slot
    QRay* out;                // next bounce's rays (null: none)
    uint32_t* seg_cnt;        // rays per segment of `out`
    uint32_t* chunk_sum;      // rays per kChunkSegs segments of `out` (zeroed per frame)
    uint32_t* super_sum;      // rays per kSuperSegs segments of `out` (zeroed per frame)
    uint32_t seg;             // the segment this wave appends to (set per wave)
    uint32_t* seg_fill;       // the wave's LDS word: rays appended to `seg` so far
    uint32_t* fetch;          // the launch's work cursors (grab_group)
    int bounce;
};
constexpr uint32_t kSegRays = 64;

// Work distribution of the persistent wavefront kernels: a wave takes the next 64-ray group of
// a queue from one of eight cursors, 128 B apart (its block's group of XCD-sharing blocks,
// blockIdx % 8; MI355X_MICROARCH.md: blocks b and b + 8 share an XCD); cursor c hands out the
// groups c, c + 8, c + 16, ..., so all XCDs work through the queue's screen order together, and a
// wave whose cursor is used up takes from the next one.  One cursor for the whole chip
// serialises every grab on one address: ~8 ns each, 30 k grabs per C5 bounce launch
// (C5: 0.904 vs 0.924 ms per frame, profiles/r04/ab/split_cursor_ab.log; a persistent pass that
// only shaded C5's bounce-1 queue took 0.25 ms on one cursor, 0.16 ms on eight).
constexpr uint32_t kCursors = 8, kCursorStride = 32;
constexpr size_t kCursorSet = (size_t)kCursors * kCursorStride;
constexpr uint32_t kNoGroup = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t grab_group(uint32_t* cursors, uint32_t ngroups, uint32_t& home) {
    uint32_t g = kNoGroup, h = home;
    if ((threadIdx.x & 63u) == 0) {
        for (uint32_t k = 0; k < kCursors; ++k) {
            const uint32_t c = (h + k) & (kCursors - 1u);
            const uint32_t gg = c + kCursors * atomicAdd(cursors + c * kCursorStride, 1u);
            if (gg < ngroups) {
                g = gg;
                h = c;
                break;
            }
        }
    }
    home = __builtin_amdgcn_readfirstlane(h);
    return __builtin_amdgcn_readfirstlane(g);
}

struct Outputs {
    uint32_t* out;
    int32_t* hits;
    float* t;
    float* rgb;
    uint32_t* gstack;            // [kGlobalStack][local_pixels]
    unsigned long long* overflow;
    uint32_t* restarts;          // traversals that outgrew the LDS stack and restarted (general code)
    uint64_t local_pixels;
    // measurement instantiation only (rt_fetch_counts): the frame's 8 record-fetch counters
    unsigned long long* fcount;
    // depth-1 kernel only: out is the whole w x h frame (rt_render_tiled: every context writes
    // its bands' pixels straight into their rows of one frame); 0: out holds this rank's bands
    // (rt_tiling order), as for every other kernel
    uint32_t frame_rows;
    // diagnostic instantiation only (rt_wave_timeline): per wave {start, end, iterations, hw id}
    uint32_t* wtime;
};

// rt_render_device_batch: the cameras of a launch's frames, a kernel argument (read with uniform
// loads by first_bounce_batch_kernel), and the pixels between two frames' outputs.
constexpr int kMaxBatch = RT_MAX_BATCH;
struct BatchCam {
    float4 a, b, c, campos, light_pos;   // .w unused
};
struct BatchCams {
    BatchCam cam[kMaxBatch];
    uint64_t stride;      // pixels from one frame's output to the next
    uint32_t frame_px;    // pixels of one frame (this rank's): frame f's first pixel in the launch's pixel space
};

__device__ __forceinline__ void leaf_range(const DevScene& S, uint32_t ref, int& off, int& cnt) {
    uint32_t c = (ref >> 26) & 31u;
    if (c == kCntEscape) {
        int2 e = S.leaf_table[ref & 0x03FFFFFFu];
        off = e.x;
        cnt = e.y;
    } else {
        off = (int)(ref & 0x03FFFFFFu);
        cnt = (int)c;
    }
}

// The same range as byte offsets of the records in the fast traversal's allocation
// (triangle records after the inner records, 48 B each): [tk, tend).
__device__ __forceinline__ void leaf_bytes(const DevScene& S, uint32_t ref, uint32_t& tk, uint32_t& tend) {
    int off, cnt;
    leaf_range(S, ref, off, cnt);
    tk = S.tri_off + (uint32_t)off * 48u;
    tend = tk + (uint32_t)cnt * 48u;
}

struct Stack {
    uint32_t* lds;      // this lane's column: lds[i * 64]
    uint32_t* glb;      // this pixel's column: glb[(i - kLdsStack) * gstride]
    uint64_t gstride;
    uint32_t* fc = nullptr;       // measurement instantiation: this lane's 8 fetch counters (LDS, stride 256)
    __device__ __forceinline__ uint32_t get(int i) const {
        return i < kLdsStack ? lds[i * 64] : glb[(uint64_t)(i - kLdsStack) * gstride];
    }
    __device__ __forceinline__ void put(int i, uint32_t v) const {
        if (i < kLdsStack) lds[i * 64] = v;
        else glb[(uint64_t)(i - kLdsStack) * gstride] = v;
    }
};

// Measurement instantiation only (rt_fetch_counts): one traversal iteration's
// record fetch of every active lane, counted per lane, per quad of lanes and per wave, by
// record kind; plus the wave's iterations and those that mix inner and triangle fetches.
// The vector-memory path merges the requests of the lanes of a QUAD (lanes 4k..4k+3) that
// read the same record (scripts/gather_peak_sweep.py: ~1.2 ns per CU per distinct record per
// quad, a wave-uniform record ~0.16 ns per lane), so its unit of work is a quad request.
// fc: this lane's counters [0/1] lane fetches inner/tri, [2/3] quad-distinct, [4/5]
// wave-distinct, [6] wave iterations, [7] mixed iterations; stride 256 (one block's lanes).
// vmem = false: a record the wave read once through the scalar cache (the traversal's
// wave-uniform prologue): a lane fetch and a wave-distinct record, but no quad request.
__device__ __forceinline__ void fetch_count(uint32_t* fc, bool leaf, uint32_t id, bool vmem = true) {
    const uint64_t act = __builtin_amdgcn_read_exec();
    const int lane = (int)(threadIdx.x & 63u);
    bool quad_first = true, wave_first = true;
    for (int j = 0; j < 64; ++j) {   // a lower active lane reading the same record makes this a repeat
        const uint32_t b = (uint32_t)__shfl((int)id, j);
        if (j < lane && ((act >> j) & 1ull) && b == id) {
            wave_first = false;
            if ((j >> 2) == (lane >> 2)) quad_first = false;
        }
    }
    const uint64_t lm = __builtin_amdgcn_ballot_w64(leaf);
    const int t = leaf ? 1 : 0;
    fc[t * 256] += 1u;
    fc[(2 + t) * 256] += (vmem && quad_first) ? 1u : 0u;
    fc[(4 + t) * 256] += wave_first ? 1u : 0u;
    if (lane == (int)__builtin_ctzll(act)) {
        fc[6 * 256] += 1u;
        fc[7 * 256] += (lm != 0 && (act & ~lm) != 0) ? 1u : 0u;
    }
}

// a block's counters (every thread's 8, stride 256) to the frame's 8 (one thread each)
__device__ __forceinline__ void fetch_count_flush(const uint32_t* fc_block, unsigned long long* out) {
    __syncthreads();
    if (threadIdx.x < 8) {
        unsigned long long sum = 0;
        for (int i = 0; i < 256; ++i) sum += fc_block[threadIdx.x * 256 + i];
        atomicAdd(out + threadIdx.x, sum);
    }
}

// local row -> frame row under rt_tiling (bands of band_rows rows, band b -> rank b % nranks)
__device__ __forceinline__ uint32_t frame_row(const Frame& F, uint32_t lr) {
    if (F.nranks <= 1) return lr;
    const uint32_t band = lr / (uint32_t)F.band_rows, rib = lr % (uint32_t)F.band_rows;
    return (band * (uint32_t)F.nranks + (uint32_t)F.rank) * (uint32_t)F.band_rows + rib;
}

// Diagnostic instantiation only (rt_wave_timeline, TR = 2).  Each wave keeps kTlWords LDS words:
// [0] / [1] closest-hit main-loop / wave-uniform-prologue trips, [2] / [3] the same for the shadow
// (any-hit) traversal, [4] s_memrealtime when the closest-hit traversal returned, [5] when the
// shading was done (the shadow traversal starts), [6] when the closest-hit traversal started,
// [7] when its wave-uniform prologue ended; with RTK_TL_SPLIT (a diagnostic build) [8] / [9] the
// closest-hit / shadow main loop's ticks between issuing a trip's record loads and their arrival
// (the trip's memory wait), [10] / [11] those trips' count whose wait was >= kTlLongWait ticks;
// trips counted and times taken by the wave's first active lane.  (In a persistent bounce wave:
// trips over all its groups, times of its last.)
// inner_step's box test as n <= min(f, tHit) && f >= kTmin (1, default) instead of three compares
// and two mask ANDs (0): same result for every input (rt_kernel_body.inc); the main loop issues two
// SALU instructions fewer per trip.  C2 0.0587 vs 0.0603 ms per frame, C3 0.2914 vs 0.2978, C4
// 1.046 vs 1.073 (three runs each, profiles/r06/ab_imin/table.txt); the bound as a NaN-sentinel
// select instead (folding f >= kTmin in as well) made the loop 10 instructions longer
#ifndef RTK_IMIN
#define RTK_IMIN 1
#endif
#ifndef RTK_TL_SPLIT
#define RTK_TL_SPLIT 0
#endif
constexpr uint32_t kTlWords = 12, kTlRecord = 20, kTlLongWait = 25;
__device__ __forceinline__ void timeline_step(uint32_t* c, int which) {
    if ((uint32_t)(threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec())) c[which] += 1u;
}
__device__ __forceinline__ void timeline_wait(uint32_t* c, int which, uint32_t ticks) {
    if ((uint32_t)(threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec())) {
        c[8 + which] += ticks;
        c[10 + which] += ticks >= kTlLongWait ? 1u : 0u;
    }
}
__device__ __forceinline__ void timeline_mark(uint32_t* c, int which) {
    if ((uint32_t)(threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec()))
        c[which] = (uint32_t)__builtin_amdgcn_s_memrealtime();
}
// ... and its record (kTlRecord words, wave w of the launch): [0] s_memrealtime (100 MHz, low 32
// bits) at its start, [1] closest hit done, [2] shading done, [3] end of its rays, [4] its end (after
// the block epilogue); [5..8] the four trip counts; [9] HW_REG_XCC_ID; [10] HW_REG_HW_ID (CU, SIMD,
// wave slot); [11] a tag (the tile, or the bounce kernel's 64-ray groups); [12] closest-hit traversal
// start, [13] end of its prologue; [16..19] the RTK_TL_SPLIT words [8..11].  Stamps go to their own
// buffer only; nothing the frame computes reads them.
__device__ __forceinline__ void timeline_store(const Outputs& O, uint32_t w, uint32_t t0, uint32_t t1,
                                               const uint32_t* c, uint32_t tag) {
    const uint32_t t2 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63u) == 0) {
        uint4* r = reinterpret_cast<uint4*>(O.wtime + (size_t)w * kTlRecord);
        r[0] = make_uint4(t0, c[4], c[5], t1);
        r[1] = make_uint4(t2, c[0], c[1], c[2]);
        r[2] = make_uint4(c[3], (uint32_t)__builtin_amdgcn_s_getreg(20 | (15 << 11)),
                          (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)), tag);
        r[3] = make_uint4(c[6], c[7], 0u, 0u);
        r[4] = make_uint4(c[8], c[9], c[10], c[11]);
    }
}

// The block's tile.  A uniform address: read through the scalar cache (RTK_FAST_ENTRY), not as a
// vector load that would queue behind the traversal requests of the waves already running on the
// CU.  The table is never written while a launch that reads it runs, except by that launch's
// last block (the next frame's longest-first order), after every block has read its entry; the
// next launch starts with the scalar cache invalidated.
__device__ __forceinline__ uint32_t block_tile(const Frame& F) {
#if RTK_FAST_ENTRY
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    return *((cu32*)F.tile_order + blockIdx.x);
#else
    return F.tile_order[blockIdx.x];
#endif
}

// Lane -> pixel inside a block's 16x16 pixels: wave w holds 8x8 tile (w % 2, w / 2), lanes
// in Morton order.  The vector-memory path merges the requests of the four lanes of a quad
// that read the same record (measured 3.7x cheaper per lane than four distinct records,
// scripts/micro/share_fetch.hip), so every quad is a 2x2 pixel square, the pixels most
// likely to walk the same nodes.  Which lane holds which pixel never changes results.
__device__ __forceinline__ void tile_pixel(const Frame& F, uint32_t tb, int wave, int l, uint32_t& x, uint32_t& lr) {
    const uint32_t tx = tb % F.tiles_x, ty = tb / F.tiles_x;
    const uint32_t lx = (uint32_t)((l & 1) | ((l >> 1) & 2) | ((l >> 2) & 4));
    const uint32_t ly = (uint32_t)(((l >> 1) & 1) | ((l >> 2) & 2) | ((l >> 3) & 4));
    x = tx * kBlockPx + (uint32_t)(wave & 1) * 8u + lx;
    lr = ty * kBlockPx + (uint32_t)(wave >> 1) * 8u + ly;
}

// The frame's counters come in two parity sets; frame f uses set f & 1 and clears the
// other one for frame f + 1 on the same stream (the kernels of f never touch it), so no
// launch is spent on zeroing.
__device__ __forceinline__ void zero_next_counters(const Frame& F) {
#if RTK_FAST_ENTRY
    const uint32_t bd = kBlockThreads;   // blockDim.x is a load from the dispatch packet
#else
    const uint32_t bd = blockDim.x;
#endif
    const uint32_t n = gridDim.x * bd;
    for (uint32_t i = blockIdx.x * bd + threadIdx.x; i < F.nzero; i += n) F.zero_next[i] = 0u;
}

// Append to the wave's own segment: the active lanes get the next slots of segment `seg`,
// in lane order.  The fill count is an LDS word of the wave, taken by the group's first
// lane, so lanes that arrive in separate groups (if the wave has not reconverged) still
// get distinct slots.
__device__ __forceinline__ QRay* seg_slot(QRay* q, uint32_t seg, uint32_t* fill) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(true);
    const int lane = threadIdx.x & 63;
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(fill, (uint32_t)__builtin_popcountll(m));
    base = (uint32_t)__shfl((int)base, leader);
    return q + (size_t)seg * kSegRays + base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
}
// (all 64 lanes, after the wave's appends) the segment's count, also added to its chunk's
// and super-chunk's sums; the fill word is reset for the wave's next segment
__device__ __forceinline__ void seg_close(const WQ& W, uint32_t seg) {
    if ((threadIdx.x & 63u) == 0) {
        const uint32_t c = *W.seg_fill;
        W.seg_cnt[seg] = c;
        if (c) {
            atomicAdd(W.chunk_sum + seg / kChunkSegs, c);
            atomicAdd(W.super_sum + seg / kSuperSegs, c);
        }
        *W.seg_fill = 0u;
    }
}

// Longest-first block order (LPT list scheduling): the hardware hands blocks to free CU
// slots in blockIdx order, so dispatching the blocks that took longest last frame first
// leaves only short blocks for the tail.  Key: log2 of the cost with 3 mantissa bits
// (256 buckets, largest first).
__device__ __forceinline__ uint32_t lpt_key(uint32_t c) {
    if (c == 0) return 0;
    const uint32_t e = 31u - __builtin_clz(c);
    const uint32_t m = e >= 3 ? (c >> (e - 3)) & 7u : (c << (3 - e)) & 7u;
    return min(255u, e * 8u + m);
}

// End of every block of a frame's tile kernel (all 256 threads).  The block's wall time
// (max over its waves) goes to tile_cost[tb]; the block that finishes last sorts all of
// them into the next frame's order (a 256-bucket counting sort), so the order costs no
// launch of its own.  Inter-workgroup hand-off (MI355X_MICROARCH.md, visibility table
// row 1): one lane per block stores its cost write-through (sc1), waits for the store,
// then adds to one agent-scope counter; the block whose add returns num_blocks - 1 is
// last, acquires, and reads every cost with sc1 loads.  `scratch` is >= kEpilogueWords
// words of LDS that no wave uses any more (the traversal stacks); the rest of it holds the
// costs' bucket keys, one byte per block, between the two passes (grids of up to kKeyBytes
// blocks: every BASELINE config at 1080p; larger grids read the costs twice).
// The last block's sort sits at the very end of the frame, on its critical path: its costs
// are read 16 per thread per round trip (four 16-B sc1 loads issued together), not one load
// and one LDS atomic per round trip (RTK_LPT_VEC 0: 2 x 32 dependent L2 round trips for a
// 1080p frame's 8,160 blocks).
#ifndef RTK_LPT_VEC
#define RTK_LPT_VEC 1
#endif
#ifndef RTK_LPT_BIAS
#define RTK_LPT_BIAS 0      // > 0: a block's cost for the next frame's order adds its start offset in the
                            // launch >> RTK_LPT_BIAS (blocks that ran late measured shorter, same work)
#endif
#ifndef RTK_EPI_NOWAIT
#define RTK_EPI_NOWAIT 0   // 1: the cost store and the counter add in flight together (profiles/r05/ab/epi_nowait_ab.log: equal)
#endif
constexpr int kEpilogueWords = 8 + 256 + 2 * 256;   // wave times + flag, histogram, two scan rows
static_assert(4 * kLdsStack * 64 >= kEpilogueWords, "tile_epilogue's scratch must fit the blocks' traversal stacks");
constexpr uint32_t kKeyBytes = (4u * kLdsStack * 64u - (uint32_t)kEpilogueWords) * 4u;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// costs [4 q, 4 q + 4) .. for q = q0 + u * 256 + tid, u < 4, with four sc1 loads in flight
// (inline asm: the compiler neither merges nor splits the 16-B agent-scope loads)
__device__ __forceinline__ void load_costs16(const uint32_t* cost, uint32_t q0, uint32_t nq, u32x4 (&v)[4]) {
    const u32x4* c4 = reinterpret_cast<const u32x4*>(cost);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const u32x4* p = c4 + min(q0 + (uint32_t)u * 256u + threadIdx.x, nq - 1u);   // in range (a repeat if past)
        asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v[u]) : "v"(p) : "memory");
    }
    // the wait "writes" the four results, so no use of them is scheduled above it
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) : : "memory");
}
// RTK_LPT_BIAS: block 0 notes when the launch started (its first stamp; the frame's counter set
// is zeroed before the frame, so 0 = not yet seen)
__device__ __forceinline__ void note_launch_start(const Frame& F, uint32_t t_start) {
    if (RTK_LPT_BIAS && F.tile_cost && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(F.t0, t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ void tile_epilogue(const Frame& F, uint32_t tb, uint32_t t_start, uint32_t* scratch) {
    if (!F.tile_cost) return;   // launch-uniform
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t t_end = (uint32_t)__builtin_amdgcn_s_memrealtime();
    __syncthreads();   // every wave is done with the stacks
    if (lane == 0) scratch[wave] = t_end - t_start + 1u;
    __syncthreads();
    if (tid == 0) {
        uint32_t c = max(max(scratch[0], scratch[1]), max(scratch[2], scratch[3]));
        if (RTK_LPT_BIAS) {
            const uint32_t T0 = __hip_atomic_load(F.t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t off = t_start - T0;
            if (T0 != 0u && off < (1u << 26)) c += off >> RTK_LPT_BIAS;
        }
        __hip_atomic_store(F.tile_cost + tb, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // RTK_EPI_NOWAIT: where the last block reads every cost exactly once (the keys kept in
        // LDS), the add does not wait for the store: the store and the add are in flight together
        // (one round trip per block instead of two), and a cost that lands after the last block
        // read it leaves the previous frame's cost of that block in this sort -- a key of the
        // schedule, never of a pixel: the order is a permutation of the blocks either way.
        // Grids read twice (past kKeyBytes blocks) need every cost stable between the passes.
        if (!RTK_EPI_NOWAIT || !RTK_LPT_VEC || gridDim.x > kKeyBytes) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t prev = __hip_atomic_fetch_add(F.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        scratch[4] = prev + 1u == gridDim.x ? 1u : 0u;
    }
    __syncthreads();
    if (!scratch[4]) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    uint32_t* hist = scratch + 8;      // [256]
    uint32_t* scan = hist + 256;       // [2][256]
    const uint32_t nb = gridDim.x;   // the order's entries: every block of the launch (all frames of a batch)
    hist[tid] = 0;
    __syncthreads();
#if RTK_LPT_VEC
    uint8_t* kb = reinterpret_cast<uint8_t*>(scratch + kEpilogueWords);
    const bool keep = nb <= kKeyBytes;
    const uint32_t nq = nb >> 2;   // whole 16-B groups of costs
    for (uint32_t q0 = 0; q0 < nq; q0 += 4u * 256u) {
        u32x4 v[4];
        load_costs16(F.tile_cost, q0, nq, v);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t q = q0 + (uint32_t)u * 256u + tid;
            if (q < nq) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t k = lpt_key(v[u][j]);
                    atomicAdd(&hist[k], 1u);
                    if (keep) kb[4u * q + (uint32_t)j] = (uint8_t)k;
                }
            }
        }
    }
    for (uint32_t i = 4u * nq + tid; i < nb; i += 256u) {
        const uint32_t k = lpt_key(__hip_atomic_load(F.tile_cost + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        atomicAdd(&hist[k], 1u);
        if (keep) kb[i] = (uint8_t)k;
    }
#else
    for (uint32_t i = tid; i < nb; i += 256)
        atomicAdd(&hist[lpt_key(__hip_atomic_load(F.tile_cost + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))], 1u);
#endif
    __syncthreads();
    // exclusive prefix over the buckets, largest key first (Hillis-Steele on 256 lanes)
    scan[tid] = hist[255 - tid];
    __syncthreads();
    int src = 0;
    for (uint32_t off = 1; off < 256; off <<= 1) {
        scan[(src ^ 1) * 256 + tid] = scan[src * 256 + tid] + (tid >= off ? scan[src * 256 + tid - off] : 0u);
        __syncthreads();
        src ^= 1;
    }
    hist[255 - tid] = scan[src * 256 + tid] - hist[255 - tid];   // inclusive -> exclusive
    __syncthreads();
#if RTK_LPT_VEC
    if (keep) {
        for (uint32_t i = tid; i < nb; i += 256u) F.lpt_next[atomicAdd(&hist[kb[i]], 1u)] = i;
    } else {
        for (uint32_t q0 = 0; q0 < nq; q0 += 4u * 256u) {
            u32x4 v[4];
            load_costs16(F.tile_cost, q0, nq, v);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t q = q0 + (uint32_t)u * 256u + tid;
                if (q < nq) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) F.lpt_next[atomicAdd(&hist[lpt_key(v[u][j])], 1u)] = 4u * q + (uint32_t)j;
                }
            }
        }
        for (uint32_t i = 4u * nq + tid; i < nb; i += 256u) {
            const uint32_t c = __hip_atomic_load(F.tile_cost + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            F.lpt_next[atomicAdd(&hist[lpt_key(c)], 1u)] = i;
        }
    }
#else
    for (uint32_t i = tid; i < nb; i += 256) {
        const uint32_t c = __hip_atomic_load(F.tile_cost + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        F.lpt_next[atomicAdd(&hist[lpt_key(c)], 1u)] = i;
    }
#endif
    if (tid == 0) __hip_atomic_store(F.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- math-independent kernels ----

// Dense order of a segmented queue (wf_compact_sort_kernel): block b takes the kChunkSegs (32)
// segments [32 b, 32 b + 32), i.e. 2048 slots of one screen-local region (8 tiles of 16x16 pixels at
// bounce 1), finds where its rays start in the dense order from the super-chunk and chunk
// sums before it (d0), and writes perm[d0 ..] with their slots, in slot order -- or with
// `sort` (RT_FLAG_WF_SORT), stably by the
// component of the ray's direction along the scene box's thinnest axis (8 buckets of width
// 1/4).  Rays that leave the scene's slab steeply take few steps, rays running along it
// many: grouping them by that component puts rays of similar length (and similar direction)
// into the same waves of 64, where a wave runs as long as its longest ray.  Simulated on
// C5's bounce queues (the oracle's per-ray step counts): wave iterations -26 % at bounce 1,
// -24 % at bounce 2 against the queue order with 32 buckets; measured, finer buckets cost
// more in lost fetch sharing between neighbouring rays than they save (C5 ms per frame,
// round 3 before the segmented queues: unsorted 1.000-1.002; 2 buckets 1.023, 4 0.970-0.972,
// 6 0.965, 8 0.968-0.970, 12 0.978, 16 0.983, 32 1.004-1.005; profiles/r03/c5_sort/).
// Stable: inside a bucket the rays keep their slot order, so neighbouring pixels (a quad's
// four rays, appended side by side) stay side by side and keep sharing their record fetches.
// Slot j = c0 + 256 p + t is ranked among the entries of its bucket by (pass p, wave, lane):
// peers in a wave by a ballot match on the key's bits, earlier waves and passes by LDS counts.
// The block of the queue's last segment stores the queue's size in *total.  nseg is
// `nseg_fixed` (bounce 1: the first bounce's waves), or when 0 the previous bounce's 64-ray
// groups, ceil(*prev_total / 64).
constexpr uint32_t kLocalSortChunk = kChunkSegs * kSegRays;
__global__ void __launch_bounds__(256) wf_compact_sort_kernel(const QRay* __restrict__ q,
                                                              const uint32_t* __restrict__ seg_cnt,
                                                              const uint32_t* __restrict__ chunk_sum,
                                                              const uint32_t* __restrict__ super_sum, uint32_t nseg_fixed,
                                                              const uint32_t* __restrict__ prev_total,
                                                              uint32_t* __restrict__ total_out, uint32_t* __restrict__ perm,
                                                              uint32_t axis, uint32_t sort) {   // sort: 0, or the key's scale
    constexpr uint32_t kPasses = kLocalSortChunk / 256;
    constexpr uint32_t kBuckets = 2 * (RTK_SORT_SCALE > RTK_SORT_SCALE_BATCH ? RTK_SORT_SCALE : RTK_SORT_SCALE_BATCH);
    constexpr int kKeyBits = kBuckets <= 2 ? 1 : kBuckets <= 4 ? 2 : kBuckets <= 8 ? 3 : kBuckets <= 16 ? 4 : 5;
    static_assert((kBuckets & (kBuckets - 1)) == 0 && kBuckets <= 32, "the key's buckets: a power of two, <= 32");
    __shared__ uint32_t cnt[kBuckets][kPasses * 4];   // [bucket][pass * 4 + wave]: entries, then their offsets
    __shared__ uint32_t total[kBuckets];
    __shared__ uint32_t segc[kChunkSegs];
    __shared__ uint32_t part[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const uint32_t nseg = nseg_fixed ? nseg_fixed : (*prev_total + kSegRays - 1) / kSegRays;
    const uint32_t b = blockIdx.x, s0 = b * kChunkSegs;
    if (s0 >= nseg) return;   // the grid covers the queue's capacity
    const uint32_t c0 = s0 * kSegRays;
    // d0 = rays in the super-chunks, then the chunks of this super-chunk, before this chunk
    constexpr uint32_t kChunksPerSuper = kSuperSegs / kChunkSegs;
    const uint32_t nsup = b / kChunksPerSuper, nch = b % kChunksPerSuper;
    uint32_t x = 0;
    for (uint32_t i = t; i < nsup; i += 256) x += super_sum[i];
    if (t < nch) x += chunk_sum[nsup * kChunksPerSuper + t];
    for (int o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_down((int)x, o);
    if (lane == 0) part[wave] = x;
    if (t < kChunkSegs) segc[t] = s0 + t < nseg ? seg_cnt[s0 + t] : 0u;
    for (uint32_t i = t; i < kBuckets * kPasses * 4; i += 256) (&cnt[0][0])[i] = 0u;
    __syncthreads();
    const uint32_t d0 = part[0] + part[1] + part[2] + part[3];
    uint32_t key[kPasses], rank[kPasses];
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (uint32_t p = 0; p < kPasses; ++p) {
        const uint32_t j = c0 + 256u * p + t;   // one segment per wave and pass
        const bool valid = (j % kSegRays) < segc[(j - c0) / kSegRays];
        uint32_t k = 0;
        if (valid && sort) {
            const float4 b = q[j].b;   // {d.xyz, shadow sum}
            const float d = axis == 0 ? b.x : axis == 1 ? b.y : b.z;
            k = d == d ? (uint32_t)min(max((int)((d + 1.0f) * (float)sort), 0), 2 * (int)sort - 1) : 0u;
        }
        uint64_t peers = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
        for (int bit = 0; bit < kKeyBits; ++bit) {
            const uint64_t m = __builtin_amdgcn_ballot_w64((k >> bit) & 1u);
            peers &= ((k >> bit) & 1u) ? m : ~m;
        }
        key[p] = valid ? k : kBuckets;
        rank[p] = (uint32_t)__builtin_popcountll(peers & lt);
        if (valid && (peers & lt) == 0) cnt[k][p * 4 + wave] = (uint32_t)__builtin_popcountll(peers);
    }
    __syncthreads();
    if (t < kBuckets) {   // per bucket: exclusive prefix over (pass, wave)
        uint32_t acc = 0;
        for (uint32_t s = 0; s < kPasses * 4; ++s) {
            const uint32_t c = cnt[t][s];
            cnt[t][s] = acc;
            acc += c;
        }
        total[t] = acc;
    }
    __syncthreads();
    if (t == 0) {   // bucket starts (exclusive prefix over buckets), kept in total[]
        uint32_t acc = 0;
        for (uint32_t k = 0; k < kBuckets; ++k) {
            const uint32_t c = total[k];
            total[k] = acc;
            acc += c;
        }
        if (s0 + kChunkSegs >= nseg) *total_out = d0 + acc;   // the queue's last chunk
    }
    __syncthreads();
#pragma unroll
    for (uint32_t p = 0; p < kPasses; ++p)
        if (key[p] < kBuckets) perm[d0 + total[key[p]] + cnt[key[p]][p * 4 + wave] + rank[p]] = c0 + 256u * p + t;
}

// Random-record gather ceiling (rt_gather_peak): every lane of every wave
// reads a different pseudo-random record of the traversal's inner-record shape (three 16-B
// loads + one 8-B load, 56 of 64 B) from a table of `nrec` 64-B records, `iters` times, four
// records in flight per lane; every CU busy.  A table that fits the XCD's L2 gives the
// ceiling of distinct-record fetches the vector-memory path can serve.
__global__ void __launch_bounds__(256) gather_peak_kernel(const float4* __restrict__ table, uint32_t nrec,
                                                          uint32_t iters, uint32_t* __restrict__ sink) {
    uint32_t x = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 0x9E3779B9u;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < iters; i += 4) {
        float4 q[4][3];
        float2 r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            const float4* p = table + (size_t)(x % nrec) * 4;
            q[k][0] = p[0]; q[k][1] = p[1]; q[k][2] = p[2];
            r[k] = *reinterpret_cast<const float2*>(p + 3);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            acc ^= __float_as_uint(q[k][0].x) ^ __float_as_uint(q[k][1].y) ^ __float_as_uint(q[k][2].z) ^
                   __float_as_uint(r[k].y);
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;   // keeps the loads; practically never taken
}

// Dependent-fetch latency (rt_chase_peak, the latency roof of DESIGN.md 6.3): every wave of
// 8 per SIMD on every CU walks `iters` steps of a chain through a table of inner-record-
// shaped 64-B records, like one traversal iteration each: three 16-B loads + one 8-B load
// of the current record, a slab-like dependent chain of packed ops on the boxes, and the
// next record chosen by the result between the record's two child references.  The lanes
// of a quad (group = 4) -- or `group` lanes -- follow one chain, as the lanes of a quad of
// coherent rays do.  Time per launch / iters = the time of one dependent iteration of a
// wave when every wave slot of the chip runs such a chain.
__global__ void __launch_bounds__(256) chase_peak_kernel(const float4* __restrict__ table, uint32_t nrec, uint32_t iters,
                                                         uint32_t group, uint32_t* __restrict__ sink) {
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    uint32_t idx = ((gid / group) * 2654435761u) % nrec;
    float acc = 0.0f;
    for (uint32_t i = 0; i < iters; ++i) {
        const float4* p = table + (size_t)idx * 4;
        const float4 q0 = p[0], q1 = p[1], q2 = p[2];
        const float2 r = *reinterpret_cast<const float2*>(p + 3);
        // both children's slab intervals from the loaded planes (dependent on the data)
        const float n0 = fmaxf(fmaxf(q0.x * 0.5f - acc, q1.x * 0.5f), q2.x * 0.5f);
        const float f0 = fminf(fminf(q0.z * 0.5f, q1.z * 0.5f - acc), q2.z * 0.5f);
        const float n1 = fmaxf(fmaxf(q0.y * 0.5f, q1.y * 0.5f - acc), q2.y * 0.5f);
        const float f1 = fminf(fminf(q0.w * 0.5f - acc, q1.w * 0.5f), q2.w * 0.5f);
        const bool left = (f0 - n0) >= (f1 - n1);
        idx = __float_as_uint(left ? r.x : r.y);
        acc = (n0 + f1) * 1e-30f;
    }
    if (idx == 0xFFFFFFFFu) sink[blockIdx.x] = __float_as_uint(acc);   // keeps the chain; never taken
}

// Band re-interleave on rank 0 (rt_assemble_bands[_batch]): one block per frame row and
// frame (grid h x nframes), 16-B copies when rows and slots are 16-B aligned.  Pure HBM
// copy: 8 B/pixel.  Rank r's slot starts at r * slot_pixels and holds the frames' band
// buffers frame_pixels apart.
__global__ void __launch_bounds__(256) assemble_bands_kernel(uint32_t* __restrict__ frame,
                                                             const uint32_t* __restrict__ slots, uint64_t slot_pixels,
                                                             uint64_t frame_pixels, uint32_t w, uint32_t h,
                                                             uint32_t nranks, uint32_t band_rows) {
    const uint32_t y = blockIdx.x;
    if (y >= h) return;
    const uint32_t band = y / band_rows;
    const uint32_t rank = band % nranks;
    const uint64_t local_row = (uint64_t)(band / nranks) * band_rows + (y % band_rows);
    const uint32_t* src = slots + (uint64_t)rank * slot_pixels + blockIdx.y * frame_pixels + local_row * w;
    uint32_t* dst = frame + (uint64_t)blockIdx.y * w * h + (uint64_t)y * w;
    if ((w & 3u) == 0 && (slot_pixels & 3u) == 0 && (frame_pixels & 3u) == 0) {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (uint32_t i = threadIdx.x; i < w / 4; i += blockDim.x) d4[i] = s4[i];
    } else {
        for (uint32_t i = threadIdx.x; i < w; i += blockDim.x) dst[i] = src[i];
    }
}

// Band put (rt_bands_put): one block per local row of this rank's band buffer, written to
// its row of the frame -- a local frame, or rank 0's frame mapped over xGMI (HIP IPC), where
// whole 16-B-aligned rows make long write bursts.  Pure copy: 8 B/pixel.
__global__ void __launch_bounds__(256) bands_put_kernel(uint32_t* __restrict__ frame,
                                                        const uint32_t* __restrict__ bands, uint32_t w,
                                                        uint32_t local_rows, uint32_t rank, uint32_t nranks,
                                                        uint32_t band_rows) {
    const uint32_t lr = blockIdx.x;
    if (lr >= local_rows) return;
    const uint64_t y = (uint64_t)(lr / band_rows * nranks + rank) * band_rows + lr % band_rows;
    const uint32_t* src = bands + (uint64_t)lr * w;
    uint32_t* dst = frame + y * w;
    if ((w & 3u) == 0) {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (uint32_t i = threadIdx.x; i < w / 4; i += blockDim.x) d4[i] = s4[i];
    } else {
        for (uint32_t i = threadIdx.x; i < w; i += blockDim.x) dst[i] = src[i];
    }
}

// ---- per-frame completion of the band puts (rt_bands_put_sync / rt_frame_present) ----
// The sync block lives in rank 0's memory, mapped into every rank with the frames:
//   [0] status (0 ok, 1 a put timed out waiting for its set, 2 a present timed out waiting
//   for the puts), [1] frames presented, [2 .. 2+nsets) release[set] (uses of the set rank 0
//   has presented), then arrive[set][rank] (uses of the set whose rows the rank has put).
// Every wait is bounded (s_memrealtime, 100 MHz): a lost peer ends in a status, never a hang;
// after the first failed wait every later one returns at once (the status is sticky).
constexpr uint32_t kSyncHead = 2;
__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The first failure's code is kept: a later wait that returns early because the status is
// already set does not overwrite it (compare-and-swap from 0).
__device__ __forceinline__ void set_status(uint32_t* sync, uint32_t code) {
    uint32_t expect = 0u;
    __hip_atomic_compare_exchange_strong(sync, &expect, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
}

// rt_bands_put_sync: at most kPutBlocks blocks, each copying every gridDim.x-th local row.
// Before writing set `set` for its use `use` the put waits until rank 0 has presented the set's
// previous use (back-pressure: a peer never overwrites a frame rank 0 has not yet observed
// complete).  Round 5 found that wait starving a GPU shared by three ranks: every block of every
// waiting put spun, holding its CU slot, while the renders the wait depended on queued behind
// them.  Now (prewaited, the default, RTAMD_PUT_WAIT=wave) the wait is ONE wave of its own
// (put_wait_kernel, bounded by timeout_ticks, status 1 on expiry) enqueued before the put, and the
// put's blocks only check the status word.  RTAMD_PUT_WAIT=stream enqueues hipStreamWaitValue32
// instead -- on device memory that is not HSA signal memory ROCm runs that as its own polling blit
// kernel (__amd_rocclr_streamOpsWait, one per wait in a kernel trace, profiles/r06/qwait_trace/),
// i.e. the same single polling wave but without a bound; RTAMD_PUT_WAIT=kernel: every put block
// waits (round 5).  A present that times out poisons every release word (kReleasePoison) after
// setting the status, so waits in flight end and their puts, seeing the status, write nothing.
// After its rows, every block releases its stores at system scope (each XCD's L2 written back) and counts itself on this
// rank's own counter for the set; the block that completes the count publishes
// arrive[set][rank] = use + 1 with a system-scope release store.
constexpr uint32_t kPutBlocks = 64;
constexpr uint32_t kReleasePoison = 0x7FFFFFFFu;   // >= every use, signed or unsigned compare
__global__ void __launch_bounds__(256) bands_put_sync_kernel(uint32_t* __restrict__ frame,
                                                             const uint32_t* __restrict__ bands, uint32_t w,
                                                             uint32_t local_rows, uint32_t rank, uint32_t nranks,
                                                             uint32_t band_rows, uint32_t* sync, uint32_t* local,
                                                             uint32_t nsets, uint32_t set, uint32_t use,
                                                             uint64_t timeout_ticks, uint32_t prewaited) {
    __shared__ uint32_t s_abort;
    if (threadIdx.x == 0) {
        uint32_t ab = 0;
        if (prewaited) {
            ab = sys_load(sync) != 0u ? 1u : 0u;   // waited for before this launch; a failed exchange writes nothing
        } else if (use > 0) {
            const uint64_t t0 = now_ticks();
            while (sys_load(sync + kSyncHead + set) < use) {
                // once any wait has failed (status != 0) the exchange is over: no further wait
                if (sys_load(sync) != 0u || now_ticks() - t0 > timeout_ticks) {
                    set_status(sync, 1u);
                    ab = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(8);
            }
        }
        s_abort = ab;
    }
    __syncthreads();
    if (s_abort) return;   // the set's arrival is never published: rank 0's present times out too
    for (uint32_t lr = blockIdx.x; lr < local_rows; lr += gridDim.x) {
        const uint64_t y = (uint64_t)(lr / band_rows * nranks + rank) * band_rows + lr % band_rows;
        const uint32_t* src = bands + (uint64_t)lr * w;
        uint32_t* dst = frame + y * w;
        if ((w & 3u) == 0) {
            const uint4* s4 = reinterpret_cast<const uint4*>(src);
            uint4* d4 = reinterpret_cast<uint4*>(dst);
            for (uint32_t i = threadIdx.x; i < w / 4; i += blockDim.x) d4[i] = s4[i];
        } else {
            for (uint32_t i = threadIdx.x; i < w; i += blockDim.x) dst[i] = src[i];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: this block's rows are out of every cache
        const uint32_t prev = __hip_atomic_fetch_add(local + set, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1u == (use + 1u) * gridDim.x) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(sync + kSyncHead + nsets + set * nranks + rank, use + 1u, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// rt_bands_put_sync's wait for set `set`'s release (the default mode): one wave, its first lane
// polling, bounded; on expiry status 1 (the put that follows then writes nothing)
__global__ void __launch_bounds__(64) put_wait_kernel(uint32_t* sync, uint32_t set, uint32_t use, uint64_t timeout_ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = now_ticks();
    while (sys_load(sync + kSyncHead + set) < use) {
        if (sys_load(sync) != 0u) return;   // the exchange has already failed
        if (now_ticks() - t0 > timeout_ticks) {
            set_status(sync, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

// rt_frame_present (rank 0, one wave): waits until every rank has published its rows of
// use `use` of set `set`, acquires them (system scope) and counts the frame as presented;
// with `release`, also releases the set for its next use (else rt_frame_release does, after
// the caller's consumers of the frame).
__global__ void __launch_bounds__(64) frame_present_kernel(uint32_t* sync, uint32_t nsets, uint32_t set, uint32_t use,
                                                           uint32_t nranks, uint64_t timeout_ticks, uint32_t release) {
    const uint32_t lane = threadIdx.x;
    const uint64_t t0 = now_ticks();
    bool ok = true;
    for (uint32_t r = lane; r < nranks; r += 64) {
        while (sys_load(sync + kSyncHead + nsets + set * nranks + r) < use + 1u) {
            if (sys_load(sync) != 0u || now_ticks() - t0 > timeout_ticks) { ok = false; break; }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    const bool all_ok = __builtin_amdgcn_ballot_w64(!ok) == 0;
    if (!all_ok) {
        if (lane == 0) set_status(sync, 2u);
        // every put waiting in a queue for a set's release goes on (and, seeing the status, writes nothing)
        for (uint32_t s2 = lane; s2 < nsets; s2 += 64)
            __hip_atomic_store(sync + kSyncHead + s2, kReleasePoison, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (lane == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        __hip_atomic_fetch_add(sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (release) __hip_atomic_store(sync + kSyncHead + set, use + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// rt_frame_release: rank 0 is done with use `use` of set `set`; the ranks may refill it.
__global__ void __launch_bounds__(64) frame_release_kernel(uint32_t* sync, uint32_t set, uint32_t use) {
    if (threadIdx.x == 0 && sys_load(sync) == 0u) {   // after a failure the sets stay poisoned (released for good)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // the frame's readers are done (stream order)
        __hip_atomic_store(sync + kSyncHead + set, use + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// rt_frame_checksum: a position-dependent 64-bit sum of a frame (a pixel in the wrong row,
// or a row from another frame, changes it), added into sums[index].
__global__ void __launch_bounds__(256) frame_checksum_kernel(const uint32_t* __restrict__ frame, uint64_t pixels,
                                                             unsigned long long* __restrict__ sums) {
    unsigned long long acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < pixels; i += (uint64_t)gridDim.x * 256u)
        acc += (((unsigned long long)frame[i] << 32) | (i & 0xFFFFFFFFull)) * 0x9E3779B97F4A7C15ull;
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
    if ((threadIdx.x & 63u) == 0) atomicAdd(sums, acc);
}

}  // namespace rtk

// Three instantiations of the math + kernels:
//   rtk_ref    (default)            S_ref: the reference as its host builds it
//   rtk_strict (RT_FLAG_STRICT_MATH) S_strict: CPU-reproducible, the oracle's arithmetic
//   rtk_hw     (RT_FLAG_HW_MATH)     S_hw: the reference built with correctly rounded / and sqrt
#define RTK_NS rtk_strict
#define RTK_MATH 0
#include "rt_device_math.h"
#include "rt_kernel_body.inc"
#undef RTK_NS
#undef RTK_MATH
#define RTK_NS rtk_hw
#define RTK_MATH 1
#include "rt_device_math.h"
#include "rt_kernel_body.inc"
#undef RTK_NS
#undef RTK_MATH
#define RTK_NS rtk_ref
#define RTK_MATH 2
#include "rt_device_math.h"
#include "rt_kernel_body.inc"
#undef RTK_NS
#undef RTK_MATH

// ============================================================================
// Host side: context, upload/repack, launch.
// ============================================================================

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // per-frame timing events, a ring over the last kRing frames: e[0]/e[1] around all
    // kernels of the frame; e[2] after the main render kernel when more kernels follow it
    // (has_k; the main kernel is the frame's first, so it spans e[0]..e[2]).  Two records per
    // depth-1 frame: each costs host time on the per-frame path.
    struct FrameEv { hipEvent_t e[3] = {nullptr, nullptr, nullptr}; bool has_k = false; };
    static constexpr int kRing = 64;
    FrameEv ring[kRing];
    uint64_t frames = 0;
    float4* d_wnodes = nullptr;
    float4* d_tris = nullptr;
    float4* d_shade = nullptr;
    int2* d_leaf = nullptr;
    size_t n_wnodes4 = 0, n_tris4 = 0, n_shade4 = 0, n_leaf = 0;   // element counts of the scene arrays
    uint32_t root = 0;
    uint32_t n_inner = 0;
    int fast_div = 0;
    int clean = 0;
    bool split_records = false;   // records >= 2 GiB: two allocations, general traversal only
    bool have_scene = false;
    bool have_params = false;
    rt_params params{};
    uint32_t* d_out = nullptr; size_t out_cap = 0;
    int32_t* d_hits = nullptr; size_t hits_cap = 0;
    float* d_t = nullptr; size_t t_cap = 0;
    float* d_rgb = nullptr; size_t rgb_cap = 0;
    unsigned long long* d_overflow = nullptr;
    // Per-stream frame scratch.  Frames enqueued on different streams may run
    // concurrently (frames in flight); each stream gets its own global stack,
    // frame counters, wavefront queues and adaptive-order state.  Frames on one
    // stream are ordered by it and share one slot.
    struct FrameSlot {
        void* stream = nullptr;
        uint64_t tkey = 0;                                                  // the tiling it renders (0: whole frame)
        uint64_t last_use = 0;
        hipEvent_t idle = nullptr;                                          // recorded after each frame
        uint64_t nframe = 0;                                                // frames rendered on this slot
        uint32_t* d_gstack = nullptr; size_t gstack_cap = 0;                // in pixels
        float4* d_wq[2] = {nullptr, nullptr}; size_t wq_cap[2] = {0, 0};   // wavefront ray queues (ping-pong)
        uint32_t* d_wcnt = nullptr; size_t wcnt_cap = 0;                    // frame counters, 2 parity sets
        size_t wcnt_set = 0;                                                //   of this many words each
        uint32_t* d_perm = nullptr; size_t perm_cap = 0;                    // wavefront: dense queue order
        uint32_t* d_seg = nullptr; size_t seg_cap = 0;                      // wavefront: rays per queue segment
        uint32_t* d_cost = nullptr; size_t cost_cap = 0;   // adaptive order: per-tile times,
        uint32_t* d_lpt = nullptr; size_t lpt_cap = 0;     //   the longest-first order built from them,
        uint32_t* d_done = nullptr;                        //   and the finished-block counter
        uint64_t cost_key = 0; bool cost_ready = false;
    };
    static constexpr int kMaxSlots = 16;
    std::vector<FrameSlot> slots;
    FrameSlot* last_slot = nullptr;
    uint64_t slot_clock = 0;
    // static block orders (column strips), one per block grid: the row groups of rt_render and
    // the contexts of rt_render_tiled may differ in grid, and a grid's table is never rewritten
    // while a frame may read it (no stream sync to switch grids)
    struct OrderTab { uint32_t tx, ty, k; uint32_t* d; };   // k: frames per launch (rt_render_device_batch)
    static constexpr size_t kMaxOrders = 16;
    std::vector<OrderTab> orders;
    uint32_t scene_gen = 0;                                   // bumped by every upload
    int wf_grid[3] = {0, 0, 0};   // persistent wavefront grid per math mode
    struct { bool on = false; unsigned long long* d_counts = nullptr; } trace;   // rt_fetch_counts
    struct {                                                                    // rt_wave_timeline
        bool on = false;
        uint32_t* d_words = nullptr; size_t cap = 0;   // device buffer, words
        size_t limit = 0, used = 0;                    // words the caller takes, words written
        std::vector<uint32_t> waves;                   // waves per launch
        std::vector<uint32_t> frame, bounce;           // per launch: its frame (of those in flight), its bounce
        uint32_t cur_frame = 0;
    } tline;
    bool frame_rows = false;   // rt_render_tiled: d_out is the whole frame (rtk::Outputs::frame_rows)
    uint32_t* h_stage = nullptr; size_t stage_cap = 0;   // rt_render_tiled: pinned frame for pageable callers
    struct TiledWorker* worker = nullptr;   // rt_render_tiled: this context's host thread (ctxs[1..])
    uint64_t enq_ns[2] = {0, 0};            // host steady clock at the start / end of the last frame's enqueue
    double wait_ms = 0.0;                   // the last synchronous wait (wait_stream's spin cap)
    // rt_render's row groups: one stream (so one frame slot) per group, and the event they start after
    hipStream_t gstream[8] = {};
    hipEvent_t gstart = nullptr;
    std::vector<FrameSlot*> last_group;   // the slots of the last grouped rt_render
    bool timing_valid = false;
    std::string err;
};

static std::string g_err;

// How the synchronous entry points (rt_render, rt_render_tiled: the reference's blocking
// raytrace_gpgpu) wait for a frame.  hipStreamSynchronize may sleep until an interrupt; a frame
// is a fraction of a millisecond, so they poll instead (hipStreamQuery, RTAMD_SYNC=query, the
// default) for up to kSpinWaitMs and only then block.  RTAMD_SYNC=block: hipStreamSynchronize
// at once (A/B).
constexpr double kSpinWaitMs = 50.0;    // cap of the spin
constexpr double kSpinMinMs = 1.0;      // the spin lasts 4x the context's last wait, within [1, 50] ms
static int sync_mode() {
    static const int m = [] {
        const char* v = std::getenv("RTAMD_SYNC");
        return v && std::strcmp(v, "block") == 0 ? 1 : 0;
    }();
    return m;
}
static inline void cpu_relax() { __builtin_ia32_pause(); }
static uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}
// spin_ms: how long to poll before blocking (about the expected frame time: the caller passes a
// multiple of its last wait); a pause between queries leaves the core's sibling and the memory
// system alone
static hipError_t wait_stream(hipStream_t s, double spin_ms = kSpinWaitMs, double* waited_ms = nullptr) {
    const auto t0 = std::chrono::steady_clock::now();
    auto done = [&](hipError_t e) {
        if (waited_ms) *waited_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return e;
    };
    if (sync_mode() == 1) return done(hipStreamSynchronize(s));
    spin_ms = std::min(kSpinWaitMs, std::max(kSpinMinMs, spin_ms));
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipErrorNotReady) return done(e);
        if (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > spin_ms)
            return done(hipStreamSynchronize(s));
        for (int i = 0; i < 16; ++i) cpu_relax();
    }
}
// a context's synchronous wait: spins about 4x its previous wait, then blocks
static hipError_t wait_ctx(rt_ctx* c, hipStream_t s) {
    double ms = 0.0;
    const hipError_t e = wait_stream(s, 4.0 * c->wait_ms, &ms);
    c->wait_ms = ms;
    return e;
}

// frame counters (one parity set): 8 per bounce ([0] queue size, [2] the bounce launch's
// work cursor), then the restart count (then, sized per frame, the queues' chunk sums)
// per bounce k: [0] its queue size, then (128-B aligned) the work cursors of its persistent
// bounce kernel (rtk::grab_group)
constexpr size_t kBounceWords = 32 + rtk::kCursorSet;
constexpr size_t kRestartSlot = kBounceWords * (RT_MAX_DEPTH + 1);
constexpr size_t kT0Slot = kRestartSlot + 1;   // the launch's start (RTK_LPT_BIAS)
constexpr size_t kCounters = kRestartSlot + 2;

static int set_err(rt_ctx* c, const std::string& m, int code) {
    if (c) c->err = m; else g_err = m;
    return code;
}

#define HIPC(ctx, expr)                                                                          \
    do {                                                                                         \
        hipError_t e__ = (expr);                                                                 \
        if (e__ != hipSuccess)                                                                   \
            return set_err(ctx, std::string(#expr) + ": " + hipGetErrorString(e__), RT_ERR_DEVICE); \
    } while (0)

template <class T>
static int ensure(rt_ctx* c, T*& p, size_t& cap, size_t n) {
    if (n <= cap && p) return RT_OK;
    if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
    hipError_t e = hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) { p = nullptr; return set_err(c, std::string("hipMalloc: ") + hipGetErrorString(e), RT_ERR_OUT_OF_MEMORY); }
    cap = n;
    return RT_OK;
}

static void free_slot(rt_ctx::FrameSlot& f) {
    for (void* p : {(void*)f.d_gstack, (void*)f.d_wq[0], (void*)f.d_wq[1], (void*)f.d_wcnt,
                    (void*)f.d_perm, (void*)f.d_seg, (void*)f.d_cost, (void*)f.d_lpt, (void*)f.d_done})
        if (p) (void)hipFree(p);
    if (f.idle) (void)hipEventDestroy(f.idle);
    f = rt_ctx::FrameSlot{};
}

// The frame scratch of `stream` (created on first use; beyond kMaxSlots streams the
// least recently used slot is recycled once its last frame has finished -- waited on
// through the slot's own event, the stream itself may be gone by then).
static int slot_for(rt_ctx* c, void* stream, uint64_t tkey, rt_ctx::FrameSlot** out) {
    ++c->slot_clock;
    for (auto& f : c->slots)
        if (f.stream == stream && f.tkey == tkey) { f.last_use = c->slot_clock; *out = &f; return RT_OK; }
    if ((int)c->slots.size() < rt_ctx::kMaxSlots) {
        c->slots.reserve(rt_ctx::kMaxSlots);   // slot pointers stay valid
        c->slots.emplace_back();
        rt_ctx::FrameSlot& f = c->slots.back();
        f.stream = stream;
        f.tkey = tkey;
        f.last_use = c->slot_clock;
        HIPC(c, hipEventCreateWithFlags(&f.idle, hipEventDisableTiming));
        *out = &f;
        return RT_OK;
    }
    rt_ctx::FrameSlot* lru = &c->slots[0];
    for (auto& f : c->slots)
        if (f.last_use < lru->last_use) lru = &f;
    HIPC(c, hipEventSynchronize(lru->idle));
    lru->stream = stream;
    lru->tkey = tkey;
    lru->cost_key = 0;
    lru->cost_ready = false;
    lru->last_use = c->slot_clock;
    *out = lru;
    return RT_OK;
}

// Inner and triangle records in ONE allocation (triangles right after the inner records),
// so the fast traversal addresses both with 32-bit offsets from one buffer descriptor.
// Buffer-load offsets are 31-bit: records of 2 GiB or more (roughly 25 M triangle
// references) get two allocations instead, and such a scene renders with the general
// traversal (pointer loads, any size).  RTAMD_RECORD_LIMIT (bytes) lowers that limit for
// tests.
static uint64_t record_limit() {
    const char* v = std::getenv("RTAMD_RECORD_LIMIT");
    const uint64_t lim = v ? std::strtoull(v, nullptr, 10) : 0;
    return lim && lim < 0x80000000ull ? lim : 0x80000000ull;
}

static hipError_t alloc_records(rt_ctx* c, size_t n_wnodes4, size_t n_tris4) {
    c->split_records = (n_wnodes4 + n_tris4) * 16 >= record_limit();
    if (c->split_records) {
        hipError_t e = hipMalloc((void**)&c->d_wnodes, n_wnodes4 * sizeof(float4));
        if (e != hipSuccess) { c->d_wnodes = nullptr; return e; }
        e = hipMalloc((void**)&c->d_tris, n_tris4 * sizeof(float4));
        if (e != hipSuccess) c->d_tris = nullptr;
        return e;
    }
    float4* p = nullptr;
    const hipError_t e = hipMalloc((void**)&p, (n_wnodes4 + n_tris4) * sizeof(float4));
    if (e != hipSuccess) return e;
    c->d_wnodes = p;
    c->d_tris = p + n_wnodes4;
    return hipSuccess;
}

static void free_scene(rt_ctx* c) {
    if (c->split_records && c->d_tris) (void)hipFree(c->d_tris);
    if (c->d_wnodes) (void)hipFree(c->d_wnodes);   // (one block: inner records, then triangle records)
    if (c->d_shade) (void)hipFree(c->d_shade);
    if (c->d_leaf) (void)hipFree(c->d_leaf);
    c->d_wnodes = nullptr; c->d_tris = nullptr; c->d_shade = nullptr; c->d_leaf = nullptr;
    c->have_scene = false;
}

// Static block -> tile order (the first frame of a geometry, and RT_FLAG_STATIC_ORDER).
// Blocks b, b+8, b+16, ... run on one XCD (round-robin dispatch; a speed assumption
// only, never correctness): XCD k gets the k-th eighth of the tile columns and walks it
// row by row, so all XCDs sweep the frame bottom-up together (balanced) while each L2
// sees one compact screen region.
static std::vector<uint32_t> tile_order_table(uint32_t tx, uint32_t ty) {
    const uint32_t nb = tx * ty;
    std::vector<uint32_t> order(nb);
    std::vector<std::vector<uint32_t>> want(8);
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t c0 = k * tx / 8, c1 = (k + 1) * tx / 8;
        for (uint32_t y = 0; y < ty; ++y)
            for (uint32_t x = c0; x < c1; ++x) want[k].push_back(y * tx + x);
    }
    // blocks of XCD k: b = k, k+8, ...; quota_k = number of such b below nb
    std::vector<uint32_t> quota(8), cursor(8, 0);
    for (uint32_t k = 0; k < 8; ++k) quota[k] = nb > k ? (nb - k + 7) / 8 : 0;
    // surplus tiles of over-full strips go to XCDs with room, keeping row order (by tile index)
    std::vector<uint32_t> spill;
    for (uint32_t k = 0; k < 8; ++k)
        while (want[k].size() > quota[k]) { spill.push_back(want[k].back()); want[k].pop_back(); }
    std::sort(spill.begin(), spill.end());
    size_t si = 0;
    for (uint32_t k = 0; k < 8; ++k)
        while (want[k].size() < quota[k] && si < spill.size()) want[k].push_back(spill[si++]);
    for (uint32_t k = 0; k < 8; ++k) std::sort(want[k].begin(), want[k].end(), [tx](uint32_t a, uint32_t b) {
        return a / tx != b / tx ? a / tx < b / tx : a < b;
    });
    for (uint32_t b = 0; b < nb; ++b) order[b] = want[b & 7][cursor[b & 7]++];
    return order;
}

// Kernels of one math mode (namespace NS), picked at launch by the frame's flags.
template <int M> struct Kernels;
#define RTK_KERNELS(M, NS)                                                                                 \
    template <> struct Kernels<M> {                                                                        \
        static void* first(bool fast, bool next) {                                                        \
            return fast ? (next ? (void*)NS::first_bounce_kernel<true, true> : (void*)NS::first_bounce_kernel<true, false>) \
                        : (next ? (void*)NS::first_bounce_kernel<false, true> : (void*)NS::first_bounce_kernel<false, false>); \
        }                                                                                                  \
        static void* fused(bool fast) { return fast ? (void*)NS::render_kernel<true> : (void*)NS::render_kernel<false>; } \
        static void* bounce(bool fast) {                                                                   \
            return fast ? (void*)NS::wf_bounce_kernel<true> : (void*)NS::wf_bounce_kernel<false>;          \
        }                                                                                                  \
        static void* traced(bool next) {                                                                   \
            return next ? (void*)NS::first_bounce_kernel<true, true, 1> : (void*)NS::first_bounce_kernel<true, false, 1>; \
        }                                                                                                  \
        static void* traced_bounce() { return (void*)NS::wf_bounce_kernel<true, 1>; }                     \
        static void* batch(bool fast, bool next) {                                                         \
            return fast ? (next ? (void*)NS::first_bounce_batch_kernel<true, true> : (void*)NS::first_bounce_batch_kernel<true, false>) \
                        : (next ? (void*)NS::first_bounce_batch_kernel<false, true> : (void*)NS::first_bounce_batch_kernel<false, false>); \
        }                                                                                                  \
    };
RTK_KERNELS(0, rtk_strict)
RTK_KERNELS(1, rtk_hw)
RTK_KERNELS(2, rtk_ref)
#undef RTK_KERNELS

static void* kernel_first(int m, bool fast, bool next) {
    return m == 0 ? Kernels<0>::first(fast, next) : m == 1 ? Kernels<1>::first(fast, next) : Kernels<2>::first(fast, next);
}
static void* kernel_batch(int m, bool fast, bool next) {
    return m == 0 ? Kernels<0>::batch(fast, next) : m == 1 ? Kernels<1>::batch(fast, next) : Kernels<2>::batch(fast, next);
}
static void* kernel_fused(int m, bool fast) {
    return m == 0 ? Kernels<0>::fused(fast) : m == 1 ? Kernels<1>::fused(fast) : Kernels<2>::fused(fast);
}
static void* kernel_traced(int m, bool next) {
    return m == 0 ? Kernels<0>::traced(next) : m == 1 ? Kernels<1>::traced(next) : Kernels<2>::traced(next);
}
static void* kernel_traced_bounce(int m) {
    return m == 0 ? Kernels<0>::traced_bounce() : m == 1 ? Kernels<1>::traced_bounce() : Kernels<2>::traced_bounce();
}
static void* kernel_bounce(int m, bool fast) {
    return m == 0 ? Kernels<0>::bounce(fast) : m == 1 ? Kernels<1>::bounce(fast) : Kernels<2>::bounce(fast);
}
// the timeline instantiation (rt_wave_timeline): S_ref, the fast kernels
static void* kernel_timeline_first(bool next) {
    return next ? (void*)rtk_ref::first_bounce_kernel<true, true, 2> : (void*)rtk_ref::first_bounce_kernel<true, false, 2>;
}
static void* kernel_timeline_bounce() { return (void*)rtk_ref::wf_bounce_kernel<true, 2>; }

extern "C" {

int rt_abi_version(void) { return 3; }

int rt_assemble_bands_batch(uint32_t* d_frame, const uint32_t* d_slots, uint64_t slot_pixels, uint64_t frame_pixels,
                            int32_t nframes, uint32_t w, uint32_t h, int32_t nranks, int32_t band_rows, void* stream) {
    if (!d_frame || !d_slots || w == 0 || h == 0 || nranks < 1 || band_rows < 1 || nframes < 1 || nframes > 65535)
        return set_err(nullptr, "rt_assemble_bands: invalid argument", RT_ERR_INVALID_ARG);
    // every rank's bands must fit a frame's buffer (rt_tiling_pixels of the fullest rank),
    // and a rank's frames its slot
    rt_tiling t0{0, nranks, band_rows, 0};
    const uint64_t need = (uint64_t)rt_tiling_pixels(w, h, &t0);
    if (need > frame_pixels || (uint64_t)nframes * frame_pixels > slot_pixels)
        return set_err(nullptr, "rt_assemble_bands: slot_pixels smaller than rank 0's bands", RT_ERR_INVALID_ARG);
    if (((uintptr_t)d_frame | (uintptr_t)d_slots) & 15u)
        return set_err(nullptr, "rt_assemble_bands: buffers must be 16-byte aligned", RT_ERR_INVALID_ARG);
    (void)hipGetLastError();   // an earlier call's error is not this launch's
    hipLaunchKernelGGL(rtk::assemble_bands_kernel, dim3(h, nframes), dim3(256), 0, (hipStream_t)stream, d_frame, d_slots,
                       slot_pixels, frame_pixels, w, h, (uint32_t)nranks, (uint32_t)band_rows);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(nullptr, std::string("rt_assemble_bands: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    return RT_OK;
}

int rt_assemble_bands(uint32_t* d_frame, const uint32_t* d_slots, uint64_t slot_pixels, uint32_t w, uint32_t h,
                      int32_t nranks, int32_t band_rows, void* stream) {
    return rt_assemble_bands_batch(d_frame, d_slots, slot_pixels, slot_pixels, 1, w, h, nranks, band_rows, stream);
}

int rt_bands_put(const uint32_t* d_bands, uint32_t* d_frame, uint32_t w, uint32_t h, const rt_tiling* tiling,
                 void* stream) {
    if (!d_bands || !d_frame || w == 0 || h == 0) return set_err(nullptr, "rt_bands_put: invalid argument", RT_ERR_INVALID_ARG);
    rt_tiling whole{0, 1, 16, 0};
    const rt_tiling* T = tiling && tiling->nranks > 1 ? tiling : &whole;
    if (T->rank < 0 || T->rank >= T->nranks || T->band_rows < 1)
        return set_err(nullptr, "rt_bands_put: bad tiling", RT_ERR_INVALID_ARG);
    const int64_t npix = rt_tiling_pixels(w, h, T);
    if (npix <= 0) return npix < 0 ? set_err(nullptr, "rt_bands_put: bad tiling", RT_ERR_INVALID_ARG) : RT_OK;
    if ((w & 3u) == 0 && (((uintptr_t)d_frame | (uintptr_t)d_bands) & 15u))
        return set_err(nullptr, "rt_bands_put: buffers must be 16-byte aligned", RT_ERR_INVALID_ARG);
    const uint32_t local_rows = (uint32_t)(npix / w);
    (void)hipGetLastError();   // an earlier call's error is not this launch's
    hipLaunchKernelGGL(rtk::bands_put_kernel, dim3(local_rows), dim3(256), 0, (hipStream_t)stream, d_frame, d_bands, w,
                       local_rows, (uint32_t)T->rank, (uint32_t)T->nranks, (uint32_t)T->band_rows);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(nullptr, std::string("rt_bands_put: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    return RT_OK;
}

int64_t rt_frame_sync_words(int32_t nsets, int32_t nranks) {
    if (nsets < 1 || nranks < 1) return -1;
    return (int64_t)rtk::kSyncHead + nsets + (int64_t)nsets * nranks;
}

// rt_bands_put_sync's wait for a set's release (RTAMD_PUT_WAIT): 0 = one bounded wait wave before the
// put (default, "wave"), 1 = hipStreamWaitValue32 ("stream", where the device supports stream wait
// values), 2 = every put block waits ("kernel", round 5)
// Launches per rebuild of the adaptive longest-first block order (RTAMD_LPT_EVERY=K, K >= 1;
// default 8).  A rebuild launch times its blocks (each block's epilogue: a barrier, its cost
// store and a counter round trip) and its last block sorts them; every other launch runs the
// order as it is and has no epilogue at all, so a wave that is done leaves at once.  Against a
// rebuild every launch (K = 1): C2 0.0605 vs 0.0693 ms per frame, one frame alone 0.172 vs 0.239
// ms; C3 0.2988 vs 0.3028, one frame 0.364 vs 0.372; C4 1.0765 vs 1.089; the orbiting camera
// 0.280 vs 0.283 (K = 16 lets its order go stale: one frame's mean 0.376 vs 0.373 at K = 8);
// profiles/r06/ab_lpt_every/table.txt.  The order is a schedule, never a pixel: same frames.
static uint64_t lpt_every() {
    static const uint64_t k = [] {
        const char* v = std::getenv("RTAMD_LPT_EVERY");
        const long n = v ? std::atol(v) : 8L;
        return (uint64_t)(n >= 1 ? n : 1);
    }();
    return k;
}

static int put_wait_mode() {
    const char* v = std::getenv("RTAMD_PUT_WAIT");
    if (v && std::strcmp(v, "kernel") == 0) return 2;
    if (v && std::strcmp(v, "stream") == 0) {
        int dev = 0, ok = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, dev) == hipSuccess && ok)
            return 1;
        (void)hipGetLastError();
        return 2;
    }
    return 0;
}
static uint64_t timeout_ticks(uint32_t ms) { return (uint64_t)(ms ? ms : 10000u) * 100000ull; }   // s_memrealtime: 100 MHz

int rt_bands_put_sync(const uint32_t* d_bands, uint32_t* d_frame, uint32_t w, uint32_t h, const rt_tiling* tiling,
                      uint32_t* d_sync, uint32_t* d_local, int32_t nsets, int32_t set, uint32_t use, uint32_t timeout_ms,
                      void* stream) {
    if (!d_bands || !d_frame || !d_sync || !d_local || w == 0 || h == 0 || nsets < 1 || set < 0 || set >= nsets)
        return set_err(nullptr, "rt_bands_put_sync: invalid argument", RT_ERR_INVALID_ARG);
    rt_tiling whole{0, 1, 16, 0};
    const rt_tiling* T = tiling && tiling->nranks > 1 ? tiling : &whole;
    if (T->rank < 0 || T->rank >= T->nranks || T->band_rows < 1)
        return set_err(nullptr, "rt_bands_put_sync: bad tiling", RT_ERR_INVALID_ARG);
    const int64_t npix = rt_tiling_pixels(w, h, T);
    if (npix <= 0) return set_err(nullptr, "rt_bands_put_sync: this rank owns no rows", RT_ERR_INVALID_ARG);
    if ((w & 3u) == 0 && (((uintptr_t)d_frame | (uintptr_t)d_bands) & 15u))
        return set_err(nullptr, "rt_bands_put_sync: buffers must be 16-byte aligned", RT_ERR_INVALID_ARG);
    const uint32_t local_rows = (uint32_t)(npix / w);
    (void)hipGetLastError();   // an earlier call's error is not this launch's
    const int mode = put_wait_mode();
    if (mode == 0 && use > 0) {   // one wave waits for the set's release; the put's blocks do not
        hipLaunchKernelGGL(rtk::put_wait_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_sync, (uint32_t)set, use,
                           timeout_ticks(timeout_ms));
    } else if (mode == 1 && use > 0) {
        const hipError_t we = hipStreamWaitValue32((hipStream_t)stream, d_sync + rtk::kSyncHead + set, use,
                                                   hipStreamWaitValueGte, 0xFFFFFFFFu);
        if (we != hipSuccess) return set_err(nullptr, std::string("rt_bands_put_sync: hipStreamWaitValue32: ") +
                                                          hipGetErrorString(we), RT_ERR_DEVICE);
    }
    const bool qwait = mode != 2;
    hipLaunchKernelGGL(rtk::bands_put_sync_kernel, dim3(std::min<uint32_t>(local_rows, rtk::kPutBlocks)), dim3(256), 0,
                       (hipStream_t)stream, d_frame, d_bands,
                       w, local_rows, (uint32_t)T->rank, (uint32_t)T->nranks, (uint32_t)T->band_rows, d_sync, d_local,
                       (uint32_t)nsets, (uint32_t)set, use, timeout_ticks(timeout_ms), qwait ? 1u : 0u);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(nullptr, std::string("rt_bands_put_sync: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    return RT_OK;
}

int rt_frame_present(uint32_t* d_sync, int32_t nsets, int32_t set, uint32_t use, int32_t nranks, uint32_t timeout_ms,
                     int32_t release, void* stream) {
    if (!d_sync || nsets < 1 || set < 0 || set >= nsets || nranks < 1)
        return set_err(nullptr, "rt_frame_present: invalid argument", RT_ERR_INVALID_ARG);
    (void)hipGetLastError();   // an earlier call's error is not this launch's
    hipLaunchKernelGGL(rtk::frame_present_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_sync, (uint32_t)nsets,
                       (uint32_t)set, use, (uint32_t)nranks, timeout_ticks(timeout_ms), release ? 1u : 0u);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(nullptr, std::string("rt_frame_present: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    return RT_OK;
}

int rt_frame_release(uint32_t* d_sync, int32_t nsets, int32_t set, uint32_t use, void* stream) {
    if (!d_sync || nsets < 1 || set < 0 || set >= nsets)
        return set_err(nullptr, "rt_frame_release: invalid argument", RT_ERR_INVALID_ARG);
    (void)hipGetLastError();   // an earlier call's error is not this launch's
    hipLaunchKernelGGL(rtk::frame_release_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_sync, (uint32_t)set, use);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(nullptr, std::string("rt_frame_release: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    return RT_OK;
}

int rt_frame_sync_status(const uint32_t* d_sync, uint32_t* status, uint32_t* presented) {
    if (!d_sync || !status || !presented) return set_err(nullptr, "rt_frame_sync_status: invalid argument", RT_ERR_INVALID_ARG);
    uint32_t v[2] = {0, 0};
    hipError_t e = hipMemcpy(v, d_sync, sizeof v, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return set_err(nullptr, std::string("rt_frame_sync_status: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    *status = v[0];
    *presented = v[1];
    return RT_OK;
}

int rt_frame_checksum(const uint32_t* d_frame, uint64_t pixels, uint64_t* d_sum, void* stream) {
    if (!d_frame || !d_sum || pixels == 0) return set_err(nullptr, "rt_frame_checksum: invalid argument", RT_ERR_INVALID_ARG);
    const uint64_t blocks = std::min<uint64_t>(1024, (pixels + 255) / 256);
    (void)hipGetLastError();   // an earlier call's error is not this launch's
    hipLaunchKernelGGL(rtk::frame_checksum_kernel, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, d_frame,
                       pixels, (unsigned long long*)d_sum);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(nullptr, std::string("rt_frame_checksum: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    return RT_OK;
}

const char* rt_last_error(rt_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int rt_create(int device, rt_ctx** out) {
    if (!out) return set_err(nullptr, "rt_create: out is NULL", RT_ERR_INVALID_ARG);
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return set_err(nullptr, "rt_create: no HIP device", RT_ERR_DEVICE);
    if (device < 0 || device >= n) return set_err(nullptr, "rt_create: bad device index", RT_ERR_INVALID_ARG);
    rt_ctx* c = new rt_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void**)&c->d_overflow, sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_overflow, 0, sizeof(unsigned long long)) != hipSuccess) {
        delete c;
        return set_err(nullptr, "rt_create: HIP init failed", RT_ERR_DEVICE);
    }
    *out = c;
    return RT_OK;
}

static void tiled_worker_stop(rt_ctx* c);
int rt_destroy(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID_ARG;
    tiled_worker_stop(c);   // rt_render_tiled's host thread for this context, if it has one
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& f : c->slots)
        if (f.idle) (void)hipEventSynchronize(f.idle);   // frames may still run on caller streams
    free_scene(c);
    if (c->d_out) (void)hipFree(c->d_out);
    if (c->d_hits) (void)hipFree(c->d_hits);
    if (c->d_t) (void)hipFree(c->d_t);
    if (c->d_rgb) (void)hipFree(c->d_rgb);
    if (c->d_overflow) (void)hipFree(c->d_overflow);
    for (auto& f : c->slots) free_slot(f);
    for (auto& o : c->orders) (void)hipFree(o.d);
    if (c->tline.d_words) (void)hipFree(c->tline.d_words);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    for (auto& f : c->ring)
        for (hipEvent_t& e : f.e)
            if (e) (void)hipEventDestroy(e);
    for (int g = 0; g < 8; ++g) {
        if (c->gstream[g]) (void)hipStreamSynchronize(c->gstream[g]);
        if (c->gstream[g]) (void)hipStreamDestroy(c->gstream[g]);
    }
    if (c->gstart) (void)hipEventDestroy(c->gstart);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return RT_OK;
}

int rt_upload_scene(rt_ctx* c, const rt_float4* verts, int32_t nv, const int32_t* idx, int32_t nidx,
                    const rt_bvh_node* nodes, int32_t nn, const int32_t* refs, int32_t nref,
                    const rt_float4* normals, int32_t nnorm, const int32_t* normal_idx, const rt_material* mats,
                    int32_t nmat, const int32_t* tri_to_mat) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (!verts || nv <= 0 || !idx || nidx <= 0 || nidx % 3 || !nodes || nn <= 0 || !refs || nref < 0 || !normals ||
        nnorm <= 0 || !normal_idx || !mats || nmat <= 0 || !tri_to_mat)
        return set_err(c, "rt_upload_scene: missing or empty array", RT_ERR_INVALID_ARG);
    const int32_t ntri = nidx / 3;
    for (int32_t i = 0; i < nidx; ++i) {
        if (idx[i] < 0 || idx[i] >= nv) return set_err(c, "mesh_indices out of range", RT_ERR_BAD_SCENE);
        if (normal_idx[i] < 0 || normal_idx[i] >= nnorm) return set_err(c, "mesh_normals_indices out of range", RT_ERR_BAD_SCENE);
    }
    for (int32_t t = 0; t < ntri; ++t)
        if (tri_to_mat[t] < 0 || tri_to_mat[t] >= nmat) return set_err(c, "tri_to_material out of range", RT_ERR_BAD_SCENE);
    for (int32_t i = 0; i < nref; ++i)
        if (refs[i] < 0 || refs[i] % 3 != 0 || refs[i] + 2 >= nidx)
            return set_err(c, "bvh_tris_indices entry out of range", RT_ERR_BAD_SCENE);

    // --- reference encoding of every node (traverse_bvh semantics, volumeRender.cl:829-856) ---
    std::vector<int32_t> inner_id(nn, -1);
    std::vector<int2> leaf_table;
    std::vector<uint32_t> ref_of(nn, 0);
    // inner ids in pre-order of reachability from the root; detect cycles (the
    // reference would spin forever on some of them).
    std::vector<uint8_t> state(nn, 0);  // 0 new, 1 on path, 2 done
    {
        std::vector<std::pair<int32_t, int>> stk;
        int32_t next = 0;
        stk.push_back({0, 0});
        while (!stk.empty()) {
            auto& top = stk.back();
            const int32_t n = top.first;
            const rt_bvh_node& nd = nodes[n];
            if (top.second == 0) {
                if (state[n] == 2) { stk.pop_back(); continue; }
                if (state[n] == 1) return set_err(c, "BVH has a cycle", RT_ERR_BAD_SCENE);
                state[n] = 1;
                bool valid_inner = nd.offset_left >= 0 && nd.offset_right >= 0 && nd.offset_left < nn && nd.offset_right < nn;
                if (nd.offset_left >= 0 && valid_inner) inner_id[n] = next++;
            }
            const bool is_inner = nd.offset_left >= 0 && inner_id[n] >= 0;
            if (is_inner && top.second < 2) {
                int32_t child = top.second == 0 ? nd.offset_left : nd.offset_right;
                top.second++;
                if (state[child] == 1) return set_err(c, "BVH has a cycle", RT_ERR_BAD_SCENE);
                if (state[child] == 0) stk.push_back({child, 0});
                continue;
            }
            state[n] = 2;
            stk.pop_back();
        }
        // the first kBfsTop inner nodes in breadth-first order from the root get ids
        // 0..kBfsTop-1 (the top of the tree, which every ray walks, in 64 KB); the rest
        // keep their pre-order
        constexpr int32_t kBfsTop = 1024;
        std::vector<int32_t> bfs;
        std::vector<uint8_t> seen(nn, 0);
        if (inner_id[0] >= 0) { bfs.push_back(0); seen[0] = 1; }
        for (size_t i = 0; i < bfs.size() && (int32_t)bfs.size() < kBfsTop; ++i) {
            const rt_bvh_node& nd = nodes[bfs[i]];
            for (int32_t ch : {nd.offset_left, nd.offset_right})
                if (inner_id[ch] >= 0 && !seen[ch] && (int32_t)bfs.size() < kBfsTop) {
                    seen[ch] = 1;
                    bfs.push_back(ch);
                }
        }
        std::vector<int32_t> by_old(next, -1);
        for (int32_t n = 0; n < nn; ++n)
            if (inner_id[n] >= 0) by_old[inner_id[n]] = n;
        int32_t id = 0;
        for (int32_t n : bfs) inner_id[n] = id++;
        for (int32_t o = 0; o < next; ++o)
            if (!seen[by_old[o]]) inner_id[by_old[o]] = id++;
    }
    bool clean = true;
    for (int32_t n = 0; n < nn; ++n)
        if (state[n] != 0 && nodes[n].offset_left >= 0 && inner_id[n] < 0) clean = false;
    int32_t n_inner = 0;
    for (int32_t n = 0; n < nn; ++n) {
        const rt_bvh_node& nd = nodes[n];
        if (inner_id[n] >= 0) ++n_inner;
        if (nd.offset_left >= 0) {
            ref_of[n] = inner_id[n] >= 0 ? (uint32_t)inner_id[n] : rtk::kRefError;
        } else {
            int32_t off = nd.offset_tris, cnt = nd.num_tris < 0 ? 0 : nd.num_tris;
            if (cnt > 0 && (off < 0 || (int64_t)off + cnt > nref))
                return set_err(c, "leaf triangle range out of bounds", RT_ERR_BAD_SCENE);
            if (cnt == 0) off = 0;
            if (cnt < (int32_t)rtk::kCntEscape && off < (1 << 26)) {
                ref_of[n] = rtk::kLeafBit | ((uint32_t)cnt << 26) | (uint32_t)off;
            } else {
                if (leaf_table.size() >= (1u << 26)) return set_err(c, "too many escape leaves", RT_ERR_BAD_SCENE);
                ref_of[n] = rtk::kLeafBit | (rtk::kCntEscape << 26) | (uint32_t)leaf_table.size();
                leaf_table.push_back(make_int2(off, cnt));
            }
        }
    }
    std::vector<float4> wn((size_t)std::max(n_inner, 1) * 4, make_float4(0, 0, 0, 0));
    bool fast_ok = true;  // slab-test fast quotient domain (rt_kernel_body.inc axis_ok)
    for (int32_t n = 0; n < nn; ++n) {
        if (inner_id[n] < 0) continue;
        const rt_bvh_node& L = nodes[nodes[n].offset_left];
        const rt_bvh_node& R = nodes[nodes[n].offset_right];
        float4* q = &wn[(size_t)inner_id[n] * 4];
        // axis-major: {L.min, R.min, L.max, R.max} per axis (rt_kernel_body.inc slab2_pk)
        q[0] = make_float4(L.min.x, R.min.x, L.max.x, R.max.x);
        q[1] = make_float4(L.min.y, R.min.y, L.max.y, R.max.y);
        q[2] = make_float4(L.min.z, R.min.z, L.max.z, R.max.z);
        uint32_t r0 = ref_of[nodes[n].offset_left], r1 = ref_of[nodes[n].offset_right];
        float f0, f1;
        std::memcpy(&f0, &r0, 4);
        std::memcpy(&f1, &r1, 4);
        q[3] = make_float4(f0, f1, 0.0f, 0.0f);
        for (int k = 0; k < 3; ++k) {
            const float* qf = &q[k].x;
            for (int j = 0; j < 4; ++j) {
                const float a = std::fabs(qf[j]);
                if (!(a == 0.0f || (a >= 0x1p-66f && a <= 0x1p60f))) fast_ok = false;
            }
        }
    }
    // triangle reference records {v0|id, e1, e2} (volumeRender.cl:965-974), layout of tri_rec
    std::vector<float4> tr((size_t)std::max(nref, 1) * 3 + 1, make_float4(0, 0, 0, 0));
    for (int32_t i = 0; i < nref; ++i) {
        const int32_t tri1 = refs[i];
        const rt_float4 v0 = verts[idx[tri1]], v1 = verts[idx[tri1 + 1]], v2 = verts[idx[tri1 + 2]];
        float idf;
        std::memcpy(&idf, &tri1, 4);
        tr[(size_t)i * 3 + 0] = make_float4(v0.x, v0.y, v0.z, idf);
        tr[(size_t)i * 3 + 1] = make_float4(v1.x - v0.x, v1.y - v0.y, v1.z - v0.z, 0.0f);
        tr[(size_t)i * 3 + 2] = make_float4(v2.x - v0.x, v2.y - v0.y, v2.z - v0.z, 0.0f);
    }
    // per-triangle shading records (volumeRender.cl:1306-1374)
    std::vector<float4> sh((size_t)ntri * 7);
    for (int32_t t = 0; t < ntri; ++t) {
        float4* s = &sh[(size_t)t * 7];
        for (int k = 0; k < 3; ++k) {
            const rt_float4 v = verts[idx[3 * t + k]];
            const rt_float4 n = normals[normal_idx[3 * t + k]];
            s[k] = make_float4(v.x, v.y, v.z, 0.0f);
            s[3 + k] = make_float4(n.x, n.y, n.z, 0.0f);
        }
        const rt_float4 d = mats[tri_to_mat[t]].diffuse;
        s[6] = make_float4(d.x, d.y, d.z, 0.0f);
    }
    if (leaf_table.empty()) leaf_table.push_back(make_int2(0, 0));

    HIPC(c, hipSetDevice(c->device));
    for (auto& f : c->slots)
        if (f.idle) HIPC(c, hipEventSynchronize(f.idle));   // frames in flight still read the old scene
    free_scene(c);
    HIPC(c, alloc_records(c, wn.size(), tr.size()));
    HIPC(c, hipMalloc((void**)&c->d_shade, sh.size() * sizeof(float4)));
    HIPC(c, hipMalloc((void**)&c->d_leaf, leaf_table.size() * sizeof(int2)));
    HIPC(c, hipMemcpy(c->d_wnodes, wn.data(), wn.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(c->d_tris, tr.data(), tr.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(c->d_shade, sh.data(), sh.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(c->d_leaf, leaf_table.data(), leaf_table.size() * sizeof(int2), hipMemcpyHostToDevice));
    c->n_wnodes4 = wn.size();
    c->n_tris4 = tr.size();
    c->n_shade4 = sh.size();
    c->n_leaf = leaf_table.size();
    c->root = ref_of[0];
    c->n_inner = (uint32_t)n_inner;
    c->fast_div = fast_ok ? 1 : 0;
    c->clean = clean ? 1 : 0;
    c->have_scene = true;
    ++c->scene_gen;
    return RT_OK;
}

// ---- scene image: the uploaded device layouts as one contiguous device buffer ----
// [header, 256 B][inner records][triangle records][shading records][escape leaves],
// each section 256-B aligned.  Multi-GPU runs build the scene once and broadcast the image
// over RCCL ("ncclBroadcast of scene buffers at load"); every rank loads it.
namespace {
constexpr uint32_t kImageMagic = 0x52544D49u;   // "IMTR"
constexpr uint32_t kImageVersion = 2;            // 2: no triangle-rank section (round 2's hit-node sort keys)
struct ImageHeader {
    uint32_t magic, version;
    uint64_t n_wnodes4, n_tris4, n_shade4, n_leaf;
    uint32_t root, n_inner;
    int32_t fast_div, clean;
};
static_assert(sizeof(ImageHeader) <= 256, "image header fits its section");
inline uint64_t sect(uint64_t bytes) { return (bytes + 255u) & ~uint64_t(255u); }
uint64_t image_bytes(const ImageHeader& h) {
    return 256 + sect(h.n_wnodes4 * 16) + sect(h.n_tris4 * 16) + sect(h.n_shade4 * 16) + sect(h.n_leaf * 8);
}
}  // namespace

int rt_scene_image_size(rt_ctx* c, uint64_t* bytes) {
    if (!c || !bytes) return RT_ERR_INVALID_ARG;
    if (!c->have_scene) return set_err(c, "rt_scene_image_size: no scene uploaded", RT_ERR_NO_SCENE);
    ImageHeader h{kImageMagic, kImageVersion, c->n_wnodes4, c->n_tris4, c->n_shade4, c->n_leaf, 0, 0, 0, 0};
    *bytes = image_bytes(h);
    return RT_OK;
}

int rt_scene_image_pack(rt_ctx* c, void* d_image, uint64_t bytes, void* stream) {
    if (!c || !d_image) return RT_ERR_INVALID_ARG;
    if (!c->have_scene) return set_err(c, "rt_scene_image_pack: no scene uploaded", RT_ERR_NO_SCENE);
    const ImageHeader h{kImageMagic, kImageVersion, c->n_wnodes4, c->n_tris4, c->n_shade4, c->n_leaf,
                        c->root, c->n_inner, c->fast_div, c->clean};
    if (bytes < image_bytes(h)) return set_err(c, "rt_scene_image_pack: buffer too small", RT_ERR_INVALID_ARG);
    HIPC(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    uint8_t* p = (uint8_t*)d_image;
    HIPC(c, hipMemcpyAsync(p, &h, sizeof h, hipMemcpyHostToDevice, s));
    p += 256;
    const std::pair<const void*, uint64_t> parts[] = {{c->d_wnodes, h.n_wnodes4 * 16}, {c->d_tris, h.n_tris4 * 16},
                                                      {c->d_shade, h.n_shade4 * 16}, {c->d_leaf, h.n_leaf * 8}};
    for (const auto& q : parts) {
        HIPC(c, hipMemcpyAsync(p, q.first, q.second, hipMemcpyDeviceToDevice, s));
        p += sect(q.second);
    }
    HIPC(c, hipStreamSynchronize(s));   // the header's host copy is a stack object
    return RT_OK;
}

int rt_scene_image_load(rt_ctx* c, const void* d_image, uint64_t bytes, void* stream) {
    if (!c || !d_image || bytes < 256) return set_err(c, "rt_scene_image_load: invalid argument", RT_ERR_INVALID_ARG);
    HIPC(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    ImageHeader h;
    HIPC(c, hipMemcpyAsync(&h, d_image, sizeof h, hipMemcpyDeviceToHost, s));
    HIPC(c, hipStreamSynchronize(s));
    if (h.magic != kImageMagic || h.version != kImageVersion || image_bytes(h) > bytes || h.n_wnodes4 == 0 || h.n_tris4 == 0 ||
        h.n_leaf == 0)
        return set_err(c, "rt_scene_image_load: not a scene image", RT_ERR_BAD_SCENE);
    for (auto& f : c->slots)
        if (f.idle) HIPC(c, hipEventSynchronize(f.idle));   // frames in flight still read the old scene
    free_scene(c);
    HIPC(c, alloc_records(c, h.n_wnodes4, h.n_tris4));
    HIPC(c, hipMalloc((void**)&c->d_shade, std::max<uint64_t>(h.n_shade4, 1) * 16));
    HIPC(c, hipMalloc((void**)&c->d_leaf, h.n_leaf * 8));
    const uint8_t* p = (const uint8_t*)d_image + 256;
    const std::pair<void*, uint64_t> parts[] = {{c->d_wnodes, h.n_wnodes4 * 16}, {c->d_tris, h.n_tris4 * 16},
                                                {c->d_shade, h.n_shade4 * 16}, {c->d_leaf, h.n_leaf * 8}};
    for (const auto& q : parts) {
        HIPC(c, hipMemcpyAsync(q.first, p, q.second, hipMemcpyDeviceToDevice, s));
        p += sect(q.second);
    }
    HIPC(c, hipStreamSynchronize(s));
    c->n_wnodes4 = h.n_wnodes4; c->n_tris4 = h.n_tris4; c->n_shade4 = h.n_shade4; c->n_leaf = h.n_leaf;
    c->root = h.root;
    c->n_inner = h.n_inner;
    c->fast_div = h.fast_div;
    c->clean = h.clean;
    c->have_scene = true;
    ++c->scene_gen;
    return RT_OK;
}

int rt_set_params(rt_ctx* c, const rt_params* p) {
    if (!c || !p) return RT_ERR_INVALID_ARG;
    c->params = *p;
    c->have_params = true;
    return RT_OK;
}

int64_t rt_tiling_pixels(uint32_t w, uint32_t h, const rt_tiling* t) {
    if (!t || t->nranks <= 1) return (int64_t)w * h;
    if (t->band_rows <= 0 || t->rank < 0 || t->rank >= t->nranks) return -1;
    const int64_t nbands = ((int64_t)h + t->band_rows - 1) / t->band_rows;
    int64_t rows = 0;
    for (int64_t b = t->rank; b < nbands; b += t->nranks) rows += std::min<int64_t>(t->band_rows, (int64_t)h - b * t->band_rows);
    return rows * w;
}

// rt_render_device, and (batch != null) rt_render_device_batch: nbatch depth-1 frames with the
// cameras batch[0..nbatch-1] in one launch, frame i at d_out + i * bstride
static int render_frames(rt_ctx* c, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, const rt_tiling* tiling,
                         uint32_t* d_out, const rt_aux* d_aux, void* stream, const rt_params* batch, int32_t nbatch,
                         uint64_t bstride) {
    if (!c || !d_out || w == 0 || h == 0 || depth < 0 || depth > RT_MAX_DEPTH)
        return set_err(c, "rt_render_device: invalid argument", RT_ERR_INVALID_ARG);
    if (batch) {
        if (nbatch < 1 || nbatch > rtk::kMaxBatch)
            return set_err(c, "rt_render_device_batch: nframes must be 1.." + std::to_string(rtk::kMaxBatch), RT_ERR_INVALID_ARG);
        if (depth < 1 || (depth > 1 && !(flags & RT_FLAG_WAVEFRONT)))
            return set_err(c, "rt_render_device_batch: depth 1, or depth > 1 with RT_FLAG_WAVEFRONT", RT_ERR_INVALID_ARG);
        for (int32_t i = 1; i < nbatch; ++i) {
            if (std::memcmp(&batch[i].scene_aabb_min, &batch[0].scene_aabb_min, 2 * sizeof(rt_float4)) != 0)
                return set_err(c, "rt_render_device_batch: the frames' scene boxes differ", RT_ERR_INVALID_ARG);
            // the bounce launches shade every frame's rays with one light (the reference's is a
            // global, RayTracer.cpp:60)
            if (depth > 1 && std::memcmp(&batch[i].light_pos, &batch[0].light_pos, sizeof(rt_float4)) != 0)
                return set_err(c, "rt_render_device_batch: depth > 1 needs one light position for all frames",
                               RT_ERR_INVALID_ARG);
        }
        if (c->trace.on || c->tline.on)
            return set_err(c, "rt_render_device_batch: not with rt_fetch_counts / rt_wave_timeline", RT_ERR_INVALID_ARG);
    }
    const uint32_t K = batch ? (uint32_t)nbatch : 1u;
    if ((flags & RT_FLAG_STRICT_MATH) && (flags & RT_FLAG_HW_MATH))
        return set_err(c, "rt_render_device: RT_FLAG_STRICT_MATH and RT_FLAG_HW_MATH exclude each other", RT_ERR_INVALID_ARG);
    if (!c->have_scene) return set_err(c, "rt_render_device: no scene uploaded", RT_ERR_NO_SCENE);
    if (!batch && !c->have_params) return set_err(c, "rt_render_device: no params set", RT_ERR_NO_SCENE);
    rt_tiling whole{0, 1, 16, 0};
    const rt_tiling* T = tiling ? tiling : &whole;
    const int64_t npix = rt_tiling_pixels(w, h, T);
    if (npix < 0) return set_err(c, "rt_render_device: bad tiling", RT_ERR_INVALID_ARG);
    if (batch && bstride < (uint64_t)npix)
        return set_err(c, "rt_render_device_batch: frame_stride below the frame's pixels", RT_ERR_INVALID_ARG);
    // a batch launch's pixel space: frame f's pixel p is f * fpx + p -- the global traversal stack
    // is indexed in it, and at depth > 1 so are the rays the bounce launches carry, which finish
    // at out[f * fpx + p]: there fpx is the frame stride (frames need not be contiguous: a rank's
    // band buffers padded to the largest rank's, bench.py at N > 1), at depth 1 the frame's pixels
    const uint64_t fpx = batch && depth > 1 ? bstride : (uint64_t)npix;
    if (batch && fpx * K >= (1ull << 32))
        return set_err(c, "rt_render_device_batch: more than 2^32 pixels in one launch", RT_ERR_INVALID_ARG);
    if (batch && d_aux) return set_err(c, "rt_render_device_batch: no aux planes", RT_ERR_INVALID_ARG);
    const bool aux = d_aux && d_aux->hits && d_aux->t && d_aux->rgb;
    if (d_aux && !aux && (d_aux->hits || d_aux->t || d_aux->rgb))
        return set_err(c, "rt_render_device: aux needs hits, t and rgb together", RT_ERR_INVALID_ARG);
    HIPC(c, hipSetDevice(c->device));
    if (npix == 0) return RT_OK;
    int rc = RT_OK;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    rt_ctx::FrameSlot* Lp = nullptr;
    // a slot per (stream, tiling): one stream may render several tilings in turn (rt_render's row
    // groups), each with its own longest-first order
    const uint64_t tkey = T->nranks > 1 ? ((uint64_t)(uint32_t)T->rank << 40) ^ ((uint64_t)(uint32_t)T->nranks << 20) ^
                                              (uint64_t)(uint32_t)T->band_rows ^ (1ull << 63)
                                        : 0;
    if ((rc = slot_for(c, (void*)s, tkey, &Lp))) return rc;
    rt_ctx::FrameSlot& L = *Lp;
    c->last_slot = &L;
    c->last_group.clear();
    const int math = (flags & RT_FLAG_STRICT_MATH) ? 0 : (flags & RT_FLAG_HW_MATH) ? 1 : 2;

    rtk::Frame F;
    const rt_params& P = batch ? batch[0] : c->params;
    F.a = make_float3(P.a.x, P.a.y, P.a.z);
    F.b = make_float3(P.b.x, P.b.y, P.b.z);
    F.c = make_float3(P.c.x, P.c.y, P.c.z);
    F.campos = make_float3(P.campos.x, P.campos.y, P.campos.z);
    F.light_pos = make_float3(P.light_pos.x, P.light_pos.y, P.light_pos.z);
    F.smin = make_float3(P.scene_aabb_min.x, P.scene_aabb_min.y, P.scene_aabb_min.z);
    F.smax = make_float3(P.scene_aabb_max.x, P.scene_aabb_max.y, P.scene_aabb_max.z);
    F.w = w;
    F.h = h;
    F.depth = depth;
    F.flags = flags;
    F.rank = T->nranks > 1 ? T->rank : 0;
    F.nranks = T->nranks > 1 ? T->nranks : 1;
    F.band_rows = T->nranks > 1 ? T->band_rows : 16;
    F.local_rows = (uint32_t)(npix / w);
    F.tiles_x = (w + rtk::kBlockPx - 1) / rtk::kBlockPx;
    F.tiles_y = (F.local_rows + rtk::kBlockPx - 1) / rtk::kBlockPx;
    F.num_blocks = F.tiles_x * F.tiles_y;

    rtk::DevScene S{c->d_wnodes,
                    c->d_tris,
                    c->d_shade,
                    c->d_leaf,
                    (uint32_t)(c->n_wnodes4 * 16),
                    (uint32_t)((c->n_wnodes4 + c->n_tris4) * 16),
                    c->root,
                    c->n_inner,
                    (c->fast_div && !(flags & RT_FLAG_EXACT_DIV)) ? 1 : 0,
                    c->clean};
    rtk::Outputs O;
    O.out = d_out;
    O.hits = aux ? d_aux->hits : nullptr;
    O.t = aux ? d_aux->t : nullptr;
    O.rgb = aux ? d_aux->rgb : nullptr;
    O.overflow = c->d_overflow;
    O.local_pixels = fpx * K;   // a batch launch's pixel space: its frames one after the other
    O.fcount = nullptr;
    O.frame_rows = c->frame_rows && !batch ? 1u : 0u;
    O.wtime = nullptr;
    const bool traced = c->trace.on;
    const bool tline = c->tline.on;
    // rt_wave_timeline: launch k's wave records at the next free words of the device buffer
    auto tline_region = [&](uint32_t waves) -> uint32_t* {
        if (c->tline.used + (size_t)waves * rtk::kTlRecord > c->tline.limit) return nullptr;
        uint32_t* p = c->tline.d_words + c->tline.used;
        c->tline.used += (size_t)waves * rtk::kTlRecord;
        c->tline.waves.push_back(waves);
        c->tline.frame.push_back(c->tline.cur_frame);
        c->tline.bounce.push_back((uint32_t)c->tline.waves.size() - 1u);   // fixed up by the caller below
        return p;
    };

    rt_ctx::FrameEv& E = c->ring[c->frames % rt_ctx::kRing];
    for (hipEvent_t& e : E.e)
        if (!e) HIPC(c, hipEventCreate(&e));
    E.has_k = false;
    // depth 1 always takes the wavefront route: it is then one first_bounce_kernel launch,
    // the fused kernel specialised to a single bounce
    const bool wavefront = ((flags & RT_FLAG_WAVEFRONT) && depth > 0) || depth == 1;

    if ((rc = ensure(c, L.d_gstack, L.gstack_cap, (size_t)fpx * rtk::kGlobalStack * K))) return rc;
    O.gstack = L.d_gstack;
    // frame counters, two parity sets: per bounce k (kBounceWords from kBounceWords k) its
    // queue size and its work cursor; [kRestartSlot] restarted traversals; then per queue
    // k = 1 .. its chunk sums and super-chunk sums (segmented queues, rtk::WQ)
    const size_t nseg = (size_t)F.num_blocks * 4 * K;   // bounce 0's waves (every frame's); later queues have fewer groups
    const size_t nchunk = (nseg + rtk::kChunkSegs - 1) / rtk::kChunkSegs;
    const size_t nsuper = (nseg + rtk::kSuperSegs - 1) / rtk::kSuperSegs;
    const size_t set_words = (kCounters + (depth > 1 ? (size_t)(depth - 1) * (nchunk + nsuper) : 0) + 31) & ~(size_t)31;
    if (!L.d_wcnt || L.wcnt_set < set_words) {
        if ((rc = ensure(c, L.d_wcnt, L.wcnt_cap, 2 * set_words))) return rc;
        HIPC(c, hipMemsetAsync(L.d_wcnt, 0, 2 * set_words * sizeof(uint32_t), s));
        L.wcnt_set = set_words;
    }
    const uint64_t par = L.nframe & 1u;
    uint32_t* cnt = L.d_wcnt + par * L.wcnt_set;
    F.zero_next = L.d_wcnt + (par ^ 1u) * L.wcnt_set;
    F.nzero = (uint32_t)L.wcnt_set;   // all of it: the next frame may be deeper than this one
    auto sums = [&](int k) { return cnt + kCounters + (size_t)(k - 1) * (nchunk + nsuper); };   // queue k >= 1
    O.restarts = cnt + kRestartSlot;
    F.t0 = cnt + kT0Slot;

    // static block order: a host-built table per block grid, made once (a new table goes into
    // a new allocation, so frames in flight that read another grid's table never wait)
    F.tile_order = nullptr;
    for (const auto& o : c->orders)
        if (o.tx == F.tiles_x && o.ty == F.tiles_y && o.k == K) F.tile_order = o.d;
    if (!F.tile_order) {
        if (c->orders.size() >= rt_ctx::kMaxOrders) {   // many grids: drop them all, once every frame is done
            HIPC(c, hipStreamSynchronize(s));
            for (auto& f : c->slots)
                if (f.idle) HIPC(c, hipEventSynchronize(f.idle));
            for (auto& o : c->orders) (void)hipFree(o.d);
            c->orders.clear();
        }
        std::vector<uint32_t> tab = tile_order_table(F.tiles_x, F.tiles_y);
        if (K > 1) {   // a batch: each tile of the static order for every frame, side by side
            std::vector<uint32_t> tk((size_t)tab.size() * K);
            for (size_t i = 0; i < tk.size(); ++i) tk[i] = tab[i / K] + (uint32_t)(i % K) * F.num_blocks;
            tab.swap(tk);
        }
        uint32_t* d = nullptr;
        size_t cap = 0;
        if ((rc = ensure(c, d, cap, tab.size()))) return rc;
        const hipError_t e = hipMemcpy(d, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(d);
            return set_err(c, std::string("rt_render_device: order table: ") + hipGetErrorString(e), RT_ERR_DEVICE);
        }
        c->orders.push_back(rt_ctx::OrderTab{F.tiles_x, F.tiles_y, K, d});
        F.tile_order = d;
    }
    // Adaptive longest-first order from the previous frame of the same geometry on this
    // slot, built by that frame's last block; the first frame runs the static order.
    F.tile_cost = nullptr;
    F.lpt_next = nullptr;
    F.done = nullptr;
    if (!(flags & RT_FLAG_STATIC_ORDER)) {
        const uint32_t units = F.num_blocks * K;   // every frame's blocks (the order's entries)
        const bool fresh = L.cost_cap < units || !L.d_done;
        if ((rc = ensure(c, L.d_cost, L.cost_cap, units))) return rc;
        if ((rc = ensure(c, L.d_lpt, L.lpt_cap, units))) return rc;
        if (!L.d_done) {
            size_t one = 0;
            if ((rc = ensure(c, L.d_done, one, 1))) return rc;
        }
        const uint64_t key = ((uint64_t)F.tiles_x << 48) ^ ((uint64_t)F.tiles_y << 32) ^ F.local_rows ^
                             ((uint64_t)c->scene_gen << 20) ^ ((uint64_t)K << 60);
        if (fresh || key != L.cost_key) {
            HIPC(c, hipMemsetAsync(L.d_done, 0, sizeof(uint32_t), s));
            L.cost_key = key;
            L.cost_ready = false;
        }
        if (L.cost_ready) F.tile_order = L.d_lpt;
        // The order is rebuilt every lpt_every()-th launch on the slot (and whenever it is not
        // ready): only those launches time their blocks, and their last block sorts; the others
        // run the order as it is, with no epilogue at all (a wave that is done leaves at once).
        if (!L.cost_ready || L.nframe % lpt_every() == 0) {
            F.tile_cost = L.d_cost;
            F.lpt_next = L.d_lpt;
            F.done = L.d_done;
        }
    }
    // the fast kernels (any quotient domain: traverse_fast picks the variant) need a clean scene
    // whose records one buffer descriptor covers
    const bool fast = S.clean != 0 && !c->split_records;
    const dim3 grid(F.num_blocks * K), block(rtk::kBlockThreads);
    int ax = aux ? 1 : 0;
    // A frame of one launch (depth 1, or the fused kernel) with RTK_EXT_EVENTS takes its timing
    // events from the launch itself (hipExtLaunchKernel: start and stop stamped by the dispatch),
    // instead of two marker packets around it on the stream.
    const bool one_launch = (!wavefront || depth == 1) && !traced && !tline;
    const bool ext_ev = RTK_EXT_EVENTS && one_launch;
    if (!ext_ev) HIPC(c, hipEventRecord(E.e[0], s));
    (void)hipGetLastError();   // the launches below are checked with hipGetLastError: not an earlier call's error

    // The frame's first kernel zeroes the other parity set for the next frame: from then on
    // the next frame on this slot must use that set, even if a later launch of this frame
    // fails (its set's queue counts and cursors are then stale).
    if (!wavefront) {
        void* args[] = {&S, &F, &O, &ax};
        if (ext_ev) HIPC(c, hipExtLaunchKernel(kernel_fused(math, fast), grid, block, args, 0, s, E.e[0], E.e[1], 0));
        else HIPC(c, hipLaunchKernel(kernel_fused(math, fast), grid, block, args, 0, s));
        ++L.nframe;
    } else {
        // Wavefront: bounce 0 over tiles, then one persistent launch per further bounce
        // over the queue of rays still in flight.
        if (!c->wf_grid[math] && depth > 1) {
            int cus = 0, b1 = 0;
            HIPC(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
            HIPC(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&b1, (const void*)kernel_bounce(math, true), 256, 0));
            c->wf_grid[math] = std::max(8, std::max(b1, 1) * cus * RTK_WF_GRID_PCT / 100);
        }
        // segmented queues: bounce 0's waves (4 per block) each own a segment of 64 slots;
        // later bounces have at most as many 64-ray groups
        const size_t slots = nseg * rtk::kSegRays;
        if (depth > 1) {
            if ((rc = ensure(c, L.d_wq[0], L.wq_cap[0], slots * 3))) return rc;   // 3 float4 per QRay
            if ((rc = ensure(c, L.d_wq[1], L.wq_cap[1], slots * 3))) return rc;
            if ((rc = ensure(c, L.d_perm, L.perm_cap, slots))) return rc;
            if ((rc = ensure(c, L.d_seg, L.seg_cap, nseg))) return rc;
        }
        const bool sort = (flags & RT_FLAG_WF_SORT) && depth > 1;
        // the local sort's key axis: the scene box's thinnest
        const float ext[3] = {F.smax.x - F.smin.x, F.smax.y - F.smin.y, F.smax.z - F.smin.z};
        const uint32_t thin = ext[1] <= ext[0] && ext[1] <= ext[2] ? 1u : ext[2] < ext[0] ? 2u : 0u;
        auto qbuf = [&](int k) { return depth > 1 ? (rtk::QRay*)L.d_wq[k & 1] : (rtk::QRay*)nullptr; };
        {
            rtk::WQ W{};
            W.out = depth > 1 ? qbuf(1) : nullptr;
            W.seg_cnt = L.d_seg;
            W.chunk_sum = sums(1);
            W.super_sum = sums(1) + nchunk;
            W.bounce = 0;
            void* args[] = {&S, &F, &O, &W, &ax};
            if (traced) {   // rt_fetch_counts: the counting instantiation of the same kernel
                O.fcount = c->trace.d_counts;
                HIPC(c, hipLaunchKernel(kernel_traced(math, depth > 1), grid, block, args, 0, s));
            } else if (tline) {   // rt_wave_timeline: the stamping instantiation
                if (!(O.wtime = tline_region(F.num_blocks * 4u)))
                    return set_err(c, "rt_wave_timeline: buffer too small", RT_ERR_INVALID_ARG);
                HIPC(c, hipLaunchKernel(kernel_timeline_first(depth > 1), grid, block, args, 0, s));
            } else if (batch) {
                rtk::BatchCams C{};
                for (uint32_t i = 0; i < K; ++i) {
                    const rt_params& Q = batch[i];
                    C.cam[i] = rtk::BatchCam{make_float4(Q.a.x, Q.a.y, Q.a.z, 0.0f), make_float4(Q.b.x, Q.b.y, Q.b.z, 0.0f),
                                             make_float4(Q.c.x, Q.c.y, Q.c.z, 0.0f),
                                             make_float4(Q.campos.x, Q.campos.y, Q.campos.z, 0.0f),
                                             make_float4(Q.light_pos.x, Q.light_pos.y, Q.light_pos.z, 0.0f)};
                }
                C.stride = bstride;
                C.frame_px = (uint32_t)fpx;
                void* bargs[] = {&S, &F, &O, &W, &C};
                void* kb = kernel_batch(math, fast, depth > 1);
                if (ext_ev) HIPC(c, hipExtLaunchKernel(kb, grid, block, bargs, 0, s, E.e[0], E.e[1], 0));
                else HIPC(c, hipLaunchKernel(kb, grid, block, bargs, 0, s));
            } else if (ext_ev) {
                HIPC(c, hipExtLaunchKernel(kernel_first(math, fast, depth > 1), grid, block, args, 0, s, E.e[0], E.e[1], 0));
            } else {
                HIPC(c, hipLaunchKernel(kernel_first(math, fast, depth > 1), grid, block, args, 0, s));
            }
            ++L.nframe;
        }
        if (depth > 1) {
            HIPC(c, hipEventRecord(E.e[2], s));
            E.has_k = true;
        }
        // the bounce launches take no part in the adaptive order or the counter clearing
        rtk::Frame Fb = F;
        Fb.tile_cost = nullptr;
        Fb.nzero = 0;
        for (int k = 1; k < depth; ++k) {  // bounce k over its queue
            rtk::WQ W{};
            W.in = qbuf(k);
            uint32_t* bc = cnt + kBounceWords * k;
            W.in_count = bc;
            // the queue's dense (compacted, optionally sorted) order and its size
            hipLaunchKernelGGL(rtk::wf_compact_sort_kernel, dim3((uint32_t)nchunk), dim3(256), 0, s,
                               (const rtk::QRay*)qbuf(k), (const uint32_t*)L.d_seg, (const uint32_t*)sums(k),
                               (const uint32_t*)(sums(k) + nchunk), k == 1 ? (uint32_t)nseg : 0u,
                               (const uint32_t*)(bc - kBounceWords), bc, L.d_perm, thin,
                               sort ? (K >= 4 ? (uint32_t)RTK_SORT_SCALE_BATCH : (uint32_t)RTK_SORT_SCALE) : 0u);
            W.perm = L.d_perm;
            W.out = k + 1 < depth ? qbuf(k + 1) : nullptr;
            W.seg_cnt = L.d_seg;
            W.chunk_sum = sums(k + 1);
            W.super_sum = sums(k + 1) + nchunk;
            W.fetch = bc + 32;
            W.bounce = k;
            void* args[] = {&S, &Fb, &O, &W, &ax};
            void* kb = traced ? kernel_traced_bounce(math) : kernel_bounce(math, fast);
            if (tline) {
                if (!(O.wtime = tline_region((uint32_t)c->wf_grid[math] * 4u)))
                    return set_err(c, "rt_wave_timeline: buffer too small", RT_ERR_INVALID_ARG);
                kb = kernel_timeline_bounce();
            }
            HIPC(c, hipLaunchKernel(kb, dim3(c->wf_grid[math]), dim3(256), args, 0, s));
        }
    }
    HIPC(c, hipGetLastError());
    if (!ext_ev) HIPC(c, hipEventRecord(E.e[1], s));
    HIPC(c, hipEventRecord(L.idle, s));
    if (F.tile_cost) L.cost_ready = true;
    c->timing_valid = true;
    ++c->frames;
    return RT_OK;
}

int rt_render_device(rt_ctx* c, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, const rt_tiling* tiling,
                     uint32_t* d_out, const rt_aux* d_aux, void* stream) {
    const uint64_t t0 = now_ns();
    const int rc = render_frames(c, w, h, depth, flags, tiling, d_out, d_aux, stream, nullptr, 1, 0);
    if (c) {
        c->enq_ns[0] = t0;
        c->enq_ns[1] = now_ns();
    }
    return rc;
}

int rt_last_enqueue_time(rt_ctx* c, uint64_t* begin_ns, uint64_t* end_ns) {
    if (!c || !begin_ns || !end_ns) return RT_ERR_INVALID_ARG;
    *begin_ns = c->enq_ns[0];
    *end_ns = c->enq_ns[1];
    return RT_OK;
}

int rt_render_device_batch(rt_ctx* c, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, const rt_tiling* tiling,
                           const rt_params* params, int32_t nframes, uint32_t* d_out, uint64_t frame_stride,
                           void* stream) {
    if (!params) return set_err(c, "rt_render_device_batch: no params", RT_ERR_INVALID_ARG);
    return render_frames(c, w, h, depth, flags, tiling, d_out, nullptr, stream, params, nframes, frame_stride);
}

// rt_render_batch: rt_render's synchronous boundary for nframes frames of one launch (the frames
// of a camera path the host already knows): into pinned, device-mapped memory directly, else
// through the ctx's device frame buffer and one read-back of all frames.
int rt_render_batch(rt_ctx* c, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, const rt_params* params,
                    int32_t nframes, uint32_t* out_bgr) {
    if (!c || !out_bgr || !params || w == 0 || h == 0 || nframes < 1 || nframes > rtk::kMaxBatch)
        return set_err(c, "rt_render_batch: invalid argument", RT_ERR_INVALID_ARG);
    const size_t npix = (size_t)w * h;
    HIPC(c, hipSetDevice(c->device));
    hipPointerAttribute_t pa;
    if (hipPointerGetAttributes(&pa, out_bgr) == hipSuccess && pa.type == hipMemoryTypeHost && pa.devicePointer) {
        const int rc = render_frames(c, w, h, depth, flags, nullptr, (uint32_t*)pa.devicePointer, nullptr, c->stream,
                                     params, nframes, npix);
        if (rc) return rc;
        HIPC(c, wait_ctx(c, c->stream));
        return RT_OK;
    }
    (void)hipGetLastError();   // pageable memory: not an error, the read-back path below
    int rc = ensure(c, c->d_out, c->out_cap, npix * (size_t)nframes);
    if (rc) return rc;
    if ((rc = render_frames(c, w, h, depth, flags, nullptr, c->d_out, nullptr, c->stream, params, nframes, npix)))
        return rc;
    HIPC(c, hipMemcpyAsync(out_bgr, c->d_out, npix * (size_t)nframes * 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, wait_ctx(c, c->stream));
    return RT_OK;
}

// rt_render: the reference's synchronous boundary (raytrace_gpgpu renders the whole frame, then
// reads it back: RayTracer.cpp:330-344), with the readback overlapped with the rendering.
//  * Pinned host memory the device can write (hipHostMalloc, or registered as mapped): the
//    frame is rendered straight into it; the kernel's pixel stores cross the host link while
//    the frame renders, with no readback after it (C3: 0.40 ms per frame against 0.55 for
//    render-then-copy, profiles/r04/ab/host_boundary_ab.log).
//  * Otherwise (pageable memory, or aux planes wanted), a frame of at least kGroupMinPixels is
//    cut into kRenderGroups groups of contiguous rows (rt_tiling with one band per "rank", so a
//    group's rows are one contiguous run of the frame and of its aux planes), each rendered
//    straight into its part of the device frame on its own stream (its own frame slot and
//    longest-first order), concurrently; a group's rows are copied to the host as soon as it is
//    done (C3 pageable: 0.49 vs 0.55 ms; 3, 6 or 8 groups, stream priorities, or the groups
//    rendered one after another on one or several streams measured slower, same log).
// The pixels are those of one whole-frame launch (a pixel's arithmetic does not depend on how
// the frame is cut: DESIGN.md 5; tests/test_render_gpu.py test_render_readback_paths_agree).
constexpr uint32_t kRenderGroups = 4;
constexpr uint64_t kGroupMinPixels = 512 * 512;

int rt_render(rt_ctx* c, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, uint32_t* out_bgr,
              const rt_aux* aux) {
    if (!c || !out_bgr) return set_err(c, "rt_render: invalid argument", RT_ERR_INVALID_ARG);
    if (w == 0 || h == 0 || depth < 0 || depth > RT_MAX_DEPTH) return set_err(c, "rt_render: invalid argument", RT_ERR_INVALID_ARG);
    const size_t npix = (size_t)w * h;
    HIPC(c, hipSetDevice(c->device));
    int rc = ensure(c, c->d_out, c->out_cap, npix);
    if (rc) return rc;
    rt_aux dev{nullptr, nullptr, nullptr};
    const bool want = aux && (aux->hits || aux->t || aux->rgb);
    const size_t dd = (size_t)std::max(depth, 1);
    if (want) {
        if ((rc = ensure(c, c->d_hits, c->hits_cap, npix * dd * 2))) return rc;
        if ((rc = ensure(c, c->d_t, c->t_cap, npix * dd))) return rc;
        if ((rc = ensure(c, c->d_rgb, c->rgb_cap, npix * 3))) return rc;
        dev = rt_aux{c->d_hits, c->d_t, c->d_rgb};
    }
    if (!want) {
        // the caller's buffer is pinned host memory the device can write (hipHostMalloc, or
        // registered as mapped): the kernel's pixel stores go straight to it over the host link
        // while the frame renders, with no readback after it
        hipPointerAttribute_t pa;
        if (hipPointerGetAttributes(&pa, out_bgr) == hipSuccess && pa.type == hipMemoryTypeHost && pa.devicePointer) {
            rc = rt_render_device(c, w, h, depth, flags, nullptr, (uint32_t*)pa.devicePointer, nullptr, c->stream);
            if (rc) return rc;
            HIPC(c, wait_ctx(c, c->stream));
            return RT_OK;
        }
        (void)hipGetLastError();   // pageable memory: not an error, the readback path below
    }
    // the group's rows: band_rows a multiple of the 16-row block, at most one band per group
    uint32_t groups = npix >= kGroupMinPixels ? kRenderGroups : 1;
    const uint32_t band_rows = ((h + groups - 1) / groups + 15u) & ~15u;
    groups = (h + band_rows - 1) / band_rows;
    if (groups <= 1) {
        rc = rt_render_device(c, w, h, depth, flags, nullptr, c->d_out, want ? &dev : nullptr, c->stream);
        if (rc) return rc;
        HIPC(c, hipMemcpyAsync(out_bgr, c->d_out, npix * 4, hipMemcpyDeviceToHost, c->stream));
        if (want) {
            if (aux->hits) HIPC(c, hipMemcpyAsync(aux->hits, c->d_hits, npix * depth * 2 * 4, hipMemcpyDeviceToHost, c->stream));
            if (aux->t) HIPC(c, hipMemcpyAsync(aux->t, c->d_t, npix * depth * 4, hipMemcpyDeviceToHost, c->stream));
            if (aux->rgb) HIPC(c, hipMemcpyAsync(aux->rgb, c->d_rgb, npix * 3 * 4, hipMemcpyDeviceToHost, c->stream));
        }
        HIPC(c, wait_ctx(c, c->stream));
        return RT_OK;
    }
    for (uint32_t g = 0; g < groups; ++g)   // group g's kernels and readback on gstream[g]
        if (!c->gstream[g]) HIPC(c, hipStreamCreateWithFlags(&c->gstream[g], hipStreamNonBlocking));
    // after whatever the ctx's own stream still holds (the synchronous entry points leave it idle)
    if (!c->gstart) HIPC(c, hipEventCreateWithFlags(&c->gstart, hipEventDisableTiming));
    // The frame's timing entry (rt_last_timing / rt_timing_average): the span from here, on the
    // ctx stream, to the end of the last group's kernels, joined back to the ctx stream.  The
    // groups' own entries go into the ring after it and are dropped again below, so one
    // grouped frame is one timing entry, like any other frame.
    const uint64_t f0 = c->frames;
    rt_ctx::FrameEv& FE = c->ring[f0 % rt_ctx::kRing];
    for (hipEvent_t& e : FE.e)
        if (!e) HIPC(c, hipEventCreate(&e));
    FE.has_k = false;
    HIPC(c, hipEventRecord(FE.e[0], c->stream));
    HIPC(c, hipEventRecord(c->gstart, c->stream));
    c->frames = f0 + 1;
    std::vector<rt_ctx::FrameSlot*> slots;
    // every group's kernels first, then the readbacks in group order: a copy into pageable
    // memory may block the host until it is done, and the later groups must already be queued
    for (uint32_t g = 0; g < groups; ++g) {
        hipStream_t s = c->gstream[g];
        HIPC(c, hipStreamWaitEvent(s, c->gstart, 0));
        const rt_tiling t{(int32_t)g, (int32_t)groups, (int32_t)band_rows, 0};
        const size_t p0 = (size_t)g * band_rows * w;
        rt_aux ga{nullptr, nullptr, nullptr};
        if (want) ga = rt_aux{c->d_hits + p0 * depth * 2, c->d_t + p0 * depth, c->d_rgb + p0 * 3};
        rc = rt_render_device(c, w, h, depth, flags, &t, c->d_out + p0, want ? &ga : nullptr, s);
        if (rc) return rc;
        slots.push_back(c->last_slot);
    }
    for (uint32_t g = 0; g < groups; ++g)   // the frame ends with the last group's kernels
        HIPC(c, hipStreamWaitEvent(c->stream, c->ring[(f0 + 1 + g) % rt_ctx::kRing].e[1], 0));
    HIPC(c, hipEventRecord(FE.e[1], c->stream));
    c->frames = f0 + 1;
    for (uint32_t g = 0; g < groups; ++g) {
        hipStream_t s = c->gstream[g];
        const size_t p0 = (size_t)g * band_rows * w, np = (size_t)std::min<uint64_t>(band_rows, h - (uint64_t)g * band_rows) * w;
        HIPC(c, hipMemcpyAsync(out_bgr + p0, c->d_out + p0, np * 4, hipMemcpyDeviceToHost, s));
        if (want) {
            if (aux->hits) HIPC(c, hipMemcpyAsync(aux->hits + p0 * depth * 2, c->d_hits + p0 * depth * 2, np * depth * 2 * 4, hipMemcpyDeviceToHost, s));
            if (aux->t) HIPC(c, hipMemcpyAsync(aux->t + p0 * depth, c->d_t + p0 * depth, np * depth * 4, hipMemcpyDeviceToHost, s));
            if (aux->rgb) HIPC(c, hipMemcpyAsync(aux->rgb + p0 * 3, c->d_rgb + p0 * 3, np * 3 * 4, hipMemcpyDeviceToHost, s));
        }
    }
    for (uint32_t g = 0; g < groups; ++g) HIPC(c, wait_ctx(c, c->gstream[g]));
    c->last_group = slots;
    return RT_OK;
}

static int frame_times(rt_ctx* c, uint64_t f, float& total, float& kernel) {
    rt_ctx::FrameEv& E = c->ring[f % rt_ctx::kRing];
    HIPC(c, hipEventSynchronize(E.e[1]));
    HIPC(c, hipEventElapsedTime(&total, E.e[0], E.e[1]));
    kernel = total;
    if (E.has_k) HIPC(c, hipEventElapsedTime(&kernel, E.e[0], E.e[2]));
    return RT_OK;
}

int rt_last_timing(rt_ctx* c, float* total_ms, float* traverse_ms) {
    if (!c || !total_ms) return RT_ERR_INVALID_ARG;
    if (!c->timing_valid || c->frames == 0) return set_err(c, "rt_last_timing: nothing rendered", RT_ERR_NO_SCENE);
    float t = 0, k = 0;
    int rc;
    if ((rc = frame_times(c, c->frames - 1, t, k))) return rc;
    *total_ms = t;
    if (traverse_ms) *traverse_ms = k;
    return RT_OK;
}

int rt_timing_average(rt_ctx* c, int32_t n, float* total_ms, float* traverse_ms) {
    if (!c || !total_ms || n < 1) return RT_ERR_INVALID_ARG;
    if (c->frames == 0) return set_err(c, "rt_timing_average: nothing rendered", RT_ERR_NO_SCENE);
    const uint64_t m = std::min<uint64_t>({(uint64_t)n, c->frames, (uint64_t)rt_ctx::kRing});
    double st = 0, sk = 0;
    for (uint64_t i = 0; i < m; ++i) {
        float t = 0, k = 0;
        int rc;
        if ((rc = frame_times(c, c->frames - 1 - i, t, k))) return rc;
        st += t;
        sk += k;
    }
    *total_ms = (float)(st / (double)m);
    if (traverse_ms) *traverse_ms = (float)(sk / (double)m);
    return RT_OK;
}

int rt_last_deferred(rt_ctx* c, uint32_t* count) {
    if (!c || !count) return RT_ERR_INVALID_ARG;
    *count = 0;
    // the last frame: one slot, or every row group of the last grouped rt_render
    std::vector<rt_ctx::FrameSlot*> ls = c->last_group;
    if (ls.empty()) ls.push_back(c->last_slot);
    for (rt_ctx::FrameSlot* L : ls) {
        if (!L || !L->d_wcnt || L->nframe == 0) continue;
        HIPC(c, hipEventSynchronize(L->idle));
        const uint64_t par = (L->nframe - 1) & 1u;   // the last frame's parity set
        uint32_t v = 0;
        HIPC(c, hipMemcpy(&v, L->d_wcnt + par * L->wcnt_set + kRestartSlot, sizeof(uint32_t), hipMemcpyDeviceToHost));
        *count += v;
    }
    return RT_OK;
}

int rt_fetch_counts(rt_ctx* c, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, uint64_t* out8) {
    if (!c || !out8 || w == 0 || h == 0 || depth < 1 || depth > RT_MAX_DEPTH)
        return set_err(c, "rt_fetch_counts: invalid argument", RT_ERR_INVALID_ARG);
    if ((depth > 1 && !(flags & RT_FLAG_WAVEFRONT)) || (flags & RT_FLAG_EXACT_DIV) || !c->have_scene || !c->clean ||
        c->split_records)
        return set_err(c, "rt_fetch_counts: the fast kernels of a clean scene, depth 1 or the wavefront path",
                       RT_ERR_INVALID_ARG);
    HIPC(c, hipSetDevice(c->device));
    int rc = ensure(c, c->d_out, c->out_cap, (size_t)w * h);
    if (rc) return rc;
    unsigned long long* d = nullptr;
    HIPC(c, hipMalloc((void**)&d, 8 * sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(d, 0, 8 * sizeof(unsigned long long), c->stream);
    if (e == hipSuccess) {
        c->trace.on = true;
        c->trace.d_counts = d;
        rc = rt_render_device(c, w, h, depth, flags | RT_FLAG_STATIC_ORDER, nullptr, c->d_out, nullptr, c->stream);
        c->trace.on = false;
        c->trace.d_counts = nullptr;
    }
    unsigned long long hc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (e == hipSuccess && rc == RT_OK) e = hipMemcpyAsync(hc, d, sizeof hc, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    if (rc) return rc;
    if (e != hipSuccess) return set_err(c, std::string("rt_fetch_counts: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    for (int k = 0; k < 8; ++k) out8[k] = hc[k];
    return RT_OK;
}

int rt_gather_peak(rt_ctx* c, uint32_t table_records, uint32_t iters, float* ms, uint64_t* records) {
    if (!c || !ms || !records || table_records == 0 || iters == 0 || iters % 4)
        return set_err(c, "rt_gather_peak: invalid argument", RT_ERR_INVALID_ARG);
    HIPC(c, hipSetDevice(c->device));
    int cus = 0;
    HIPC(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    const uint32_t blocks = (uint32_t)cus * 8u;   // 8 blocks of 4 waves per CU: 8 waves per SIMD
    float4* table = nullptr;
    uint32_t* sink = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPC(c, hipMalloc((void**)&table, (size_t)table_records * 64));
    hipError_t e = hipMalloc((void**)&sink, blocks * 4);
    if (e == hipSuccess) e = hipMemsetAsync(table, 0x3C, (size_t)table_records * 64, c->stream);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(rtk::gather_peak_kernel, dim3(blocks), dim3(256), 0, c->stream, table, table_records, iters, sink);
        e = hipEventRecord(e0, c->stream);
    }
    if (e == hipSuccess) {
        for (int k = 0; k < 4; ++k)
            hipLaunchKernelGGL(rtk::gather_peak_kernel, dim3(blocks), dim3(256), 0, c->stream, table, table_records, iters,
                               sink);
        e = hipEventRecord(e1, c->stream);
    }
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float t = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
    if (e == hipSuccess) e = hipGetLastError();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(table);
    if (sink) (void)hipFree(sink);
    if (e != hipSuccess) return set_err(c, std::string("rt_gather_peak: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    *ms = t / 4.0f;
    *records = (uint64_t)blocks * 256u * iters;
    return RT_OK;
}

int rt_chase_peak(rt_ctx* c, uint32_t table_records, uint32_t iters, uint32_t group, float* ms, uint64_t* waves) {
    if (!c) return RT_ERR_INVALID_ARG;
    int cus = 0;
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    return rt_chase_latency(c, table_records, iters, group, (uint32_t)cus * 8u, ms, waves);   // 8 waves per SIMD
}

int rt_chase_latency(rt_ctx* c, uint32_t table_records, uint32_t iters, uint32_t group, uint32_t blocks, float* ms,
                     uint64_t* waves) {
    if (!c || !ms || !waves || table_records < 2 || iters == 0 || group == 0 || group > 64 || (64 % group) ||
        blocks == 0 || blocks > (1u << 20))
        return set_err(c, "rt_chase_peak: invalid argument", RT_ERR_INVALID_ARG);
    HIPC(c, hipSetDevice(c->device));
    // the table: random child references (two per record, both valid), boxes from a fixed pattern
    std::vector<float4> tab((size_t)table_records * 4);
    uint32_t x = 0x9E3779B9u;
    for (uint32_t i = 0; i < table_records; ++i) {
        uint32_t rr[2];
        for (uint32_t& v : rr) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            v = x % table_records;
        }
        const float a = (float)(i % 97), b = (float)(i % 89);
        tab[(size_t)i * 4 + 0] = make_float4(a, b, a + 3.0f, b + 5.0f);
        tab[(size_t)i * 4 + 1] = make_float4(b, a, b + 7.0f, a + 2.0f);
        tab[(size_t)i * 4 + 2] = make_float4(a + 1.0f, b + 1.0f, a + 9.0f, b + 4.0f);
        float r0, r1;
        std::memcpy(&r0, &rr[0], 4);
        std::memcpy(&r1, &rr[1], 4);
        tab[(size_t)i * 4 + 3] = make_float4(r0, r1, 0.0f, 0.0f);
    }
    float4* table = nullptr;
    uint32_t* sink = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPC(c, hipMalloc((void**)&table, tab.size() * sizeof(float4)));
    hipError_t e = hipMalloc((void**)&sink, blocks * 4);
    if (e == hipSuccess) e = hipMemcpy(table, tab.data(), tab.size() * sizeof(float4), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(rtk::chase_peak_kernel, dim3(blocks), dim3(256), 0, c->stream, table, table_records, iters, group, sink);
        e = hipEventRecord(e0, c->stream);
    }
    if (e == hipSuccess) {
        for (int k = 0; k < 4; ++k)
            hipLaunchKernelGGL(rtk::chase_peak_kernel, dim3(blocks), dim3(256), 0, c->stream, table, table_records, iters,
                               group, sink);
        e = hipEventRecord(e1, c->stream);
    }
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float t = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
    if (e == hipSuccess) e = hipGetLastError();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(table);
    if (sink) (void)hipFree(sink);
    if (e != hipSuccess) return set_err(c, std::string("rt_chase_peak: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    *ms = t / 4.0f;
    *waves = (uint64_t)blocks * 4u;
    return RT_OK;
}

// ---- one frame on several GPUs, one process (rt_render_tiled) ----

int rt_scene_copy(rt_ctx* dst, rt_ctx* src) {
    if (!dst || !src) return set_err(dst, "rt_scene_copy: invalid argument", RT_ERR_INVALID_ARG);
    if (dst == src) return RT_OK;
    if (!src->have_scene) return set_err(dst, "rt_scene_copy: the source context has no scene", RT_ERR_NO_SCENE);
    HIPC(dst, hipSetDevice(dst->device));
    for (auto& f : dst->slots)
        if (f.idle) HIPC(dst, hipEventSynchronize(f.idle));   // frames in flight still read the old scene
    free_scene(dst);
    HIPC(dst, alloc_records(dst, src->n_wnodes4, src->n_tris4));
    HIPC(dst, hipMalloc((void**)&dst->d_shade, std::max<size_t>(src->n_shade4, 1) * 16));
    HIPC(dst, hipMalloc((void**)&dst->d_leaf, src->n_leaf * 8));
    // device to device on one GPU, else peer to peer (xGMI), both on dst's stream
    const std::pair<std::pair<void*, const void*>, size_t> parts[] = {
        {{dst->d_wnodes, src->d_wnodes}, src->n_wnodes4 * 16}, {{dst->d_tris, src->d_tris}, src->n_tris4 * 16},
        {{dst->d_shade, src->d_shade}, src->n_shade4 * 16}, {{dst->d_leaf, src->d_leaf}, src->n_leaf * 8}};
    for (const auto& q : parts) {
        if (!q.second) continue;
        if (dst->device == src->device)
            HIPC(dst, hipMemcpyAsync(q.first.first, q.first.second, q.second, hipMemcpyDeviceToDevice, dst->stream));
        else
            HIPC(dst, hipMemcpyPeerAsync(q.first.first, dst->device, q.first.second, src->device, q.second, dst->stream));
    }
    HIPC(dst, hipStreamSynchronize(dst->stream));
    dst->n_wnodes4 = src->n_wnodes4; dst->n_tris4 = src->n_tris4; dst->n_shade4 = src->n_shade4; dst->n_leaf = src->n_leaf;
    dst->root = src->root;
    dst->n_inner = src->n_inner;
    dst->fast_div = src->fast_div;
    dst->clean = src->clean;
    dst->have_scene = true;
    ++dst->scene_gen;
    return RT_OK;
}

// rt_render_tiled: the frame is cut into 8-row bands dealt round-robin over the contexts
// (rt_tiling).  Every context renders its bands on its own stream with the
// frame-row output of the kernels (rtk::Outputs::frame_rows): each pixel store goes straight to
// its place in ONE host frame, so every GPU sends its own rows over its own host link while it
// renders, and there is no gather, copy or re-interleave step.  That frame is the caller's
// buffer when it is pinned memory the devices can write, else ctx 0's pinned staging frame,
// copied to the caller's memory after the join.  Then every stream is synchronised: returns
// with the frame complete in out_bgr, like raytrace_gpgpu (RayTracer.cpp:330-344).
constexpr int32_t kTiledBandRows = 8;
constexpr int32_t kMaxTiled = 64;

// One context's part of a tiled frame: its bands straight into the frame's rows (depth 1), or
// into its band buffer and then one row-copy kernel; then the wait for its stream (also after a
// failed enqueue: nothing may still write into the frame when rt_render_tiled returns).
struct TiledJob {
    uint32_t w, h;
    int32_t depth;
    uint32_t flags;
    rt_tiling t;
    uint32_t* frame;   // the frame as THIS context's device addresses it
};
static int tiled_enqueue(rt_ctx* c, const TiledJob& j) {
    int rc = RT_OK;
    if (hipSetDevice(c->device) != hipSuccess) return set_err(c, "hipSetDevice failed", RT_ERR_DEVICE);
    if (j.depth == 1) {   // the depth-1 kernel writes its pixels into the frame's rows itself
        c->frame_rows = true;
        rc = rt_render_device(c, j.w, j.h, j.depth, j.flags, &j.t, j.frame, nullptr, c->stream);
        c->frame_rows = false;
    } else {              // other kernels: the context's bands, then one row-copy kernel into the frame
        const int64_t lp = rt_tiling_pixels(j.w, j.h, &j.t);
        if (lp > 0 && (rc = ensure(c, c->d_out, c->out_cap, (size_t)lp)) == RT_OK &&
            (rc = rt_render_device(c, j.w, j.h, j.depth, j.flags, &j.t, c->d_out, nullptr, c->stream)) == RT_OK &&
            rt_bands_put(c->d_out, j.frame, j.w, j.h, &j.t, c->stream) != RT_OK)
            rc = set_err(c, g_err, RT_ERR_DEVICE);
    }
    return rc;
}
static int tiled_wait(rt_ctx* c, int rc) {
    const hipError_t e = hipSetDevice(c->device) == hipSuccess ? wait_ctx(c, c->stream) : hipErrorInvalidDevice;
    if (e != hipSuccess && rc == RT_OK) rc = set_err(c, hipGetErrorString(e), RT_ERR_DEVICE);
    return rc;
}
static int tiled_part(rt_ctx* c, const TiledJob& j) { return tiled_wait(c, tiled_enqueue(c, j)); }

// rt_render_tiled's host thread per context (ctxs[1..n-1]; ctxs[0]'s part runs on the caller's
// thread).  The hand-off is a sequence number the worker spins on, so all contexts enqueue at
// once instead of one after another (~3-4 us of host time each): a condition
// variable costs about as much as the enqueue it would save, so a worker spins for
// kWorkerSpinMs after its last frame (a frame loop keeps it spinning) and only then sleeps.
// RTAMD_TILED_WORKERS=0: every part on the caller's thread, one after another (A/B).
constexpr double kWorkerSpinMs = 20.0;
struct TiledWorker {
    std::thread th;
    std::atomic<uint64_t> posted{0}, finished{0};
    std::atomic<bool> stop{false}, asleep{false};
    std::mutex m;
    std::condition_variable cv;
    TiledJob job{};
    int rc = RT_OK;
};
static void tiled_worker_loop(rt_ctx* c, TiledWorker* W) {
    (void)hipSetDevice(c->device);
    uint64_t seen = 0;
    for (;;) {
        auto t0 = std::chrono::steady_clock::now();
        uint32_t spins = 0;
        while (W->posted.load(std::memory_order_acquire) == seen && !W->stop.load(std::memory_order_relaxed)) {
            cpu_relax();
            if ((++spins & 4095u) == 0 &&
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > kWorkerSpinMs) {
                std::unique_lock<std::mutex> lk(W->m);
                W->asleep.store(true);   // seq_cst with the poster's store of `posted` then load of `asleep`
                W->cv.wait(lk, [&] { return W->posted.load() != seen || W->stop.load(); });
                W->asleep.store(false);
                t0 = std::chrono::steady_clock::now();
            }
        }
        if (W->stop.load()) return;
        seen = W->posted.load(std::memory_order_acquire);
        W->rc = tiled_part(c, W->job);
        W->finished.store(seen, std::memory_order_release);
    }
}
static void tiled_post(rt_ctx* c, const TiledJob& j) {
    if (!c->worker) {
        c->worker = new TiledWorker();
        c->worker->th = std::thread(tiled_worker_loop, c, c->worker);
    }
    TiledWorker* W = c->worker;
    W->job = j;
    W->posted.fetch_add(1);   // seq_cst (the worker's asleep store / posted load pair)
    if (W->asleep.load()) {
        std::lock_guard<std::mutex> lk(W->m);
        W->cv.notify_one();
    }
}
static int tiled_join(rt_ctx* c) {
    TiledWorker* W = c->worker;
    const uint64_t want = W->posted.load();
    while (W->finished.load(std::memory_order_acquire) != want) cpu_relax();
    return W->rc;
}
static void tiled_worker_stop(rt_ctx* c) {
    if (!c->worker) return;
    {
        std::lock_guard<std::mutex> lk(c->worker->m);
        c->worker->stop.store(true);
        c->worker->cv.notify_one();
    }
    if (c->worker->th.joinable()) c->worker->th.join();
    delete c->worker;
    c->worker = nullptr;
}
static bool tiled_workers_on() {
    const char* v = std::getenv("RTAMD_TILED_WORKERS");
    return !(v && std::strcmp(v, "0") == 0);
}

int32_t rt_tiled_direct_ok(int32_t n, const uint64_t* dev_addrs) {
    if (n < 1 || !dev_addrs) return 0;
    for (int32_t k = 0; k < n; ++k)
        if (!dev_addrs[k] || (dev_addrs[k] & 15u)) return 0;   // unmapped on that device, or not 16-B aligned
    return 1;
}

// rt_render_tiled: the frame is cut into 8-row bands dealt round-robin over the contexts
// (rt_tiling).  Every context renders its bands on its own stream with the
// frame-row output of the kernels (rtk::Outputs::frame_rows): each pixel store goes straight to
// its place in ONE host frame, so every GPU sends its own rows over its own host link while it
// renders, and there is no gather, copy or re-interleave step.  That frame is the caller's
// buffer when every context's device can address it (hipHostGetDevicePointer on each device:
// portable pinned memory, or memory registered and mapped for all of them), else ctxs[0]'s
// portable pinned staging frame, copied to the caller's memory after the join.  Each context
// addresses the frame through its own device's mapping.  ctxs[1..] enqueue and wait on their own
// host threads (TiledWorker), ctxs[0] on the caller's; returns with the frame complete in out_bgr,
// like raytrace_gpgpu (RayTracer.cpp:330-344).
int rt_render_tiled(rt_ctx** ctxs, int32_t n, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, uint32_t* out_bgr) {
    if (!ctxs || n < 1 || n > kMaxTiled || !out_bgr || w == 0 || h == 0 || depth < 0 || depth > RT_MAX_DEPTH)
        return set_err(nullptr, "rt_render_tiled: invalid argument", RT_ERR_INVALID_ARG);
    for (int32_t k = 0; k < n; ++k) {
        if (!ctxs[k]) return set_err(nullptr, "rt_render_tiled: ctxs[k] is NULL", RT_ERR_INVALID_ARG);
        for (int32_t j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k]) return set_err(nullptr, "rt_render_tiled: a context appears twice", RT_ERR_INVALID_ARG);
    }
    rt_ctx* c0 = ctxs[0];
    if ((flags & RT_FLAG_STRICT_MATH) && (flags & RT_FLAG_HW_MATH))
        return set_err(c0, "rt_render_tiled: RT_FLAG_STRICT_MATH and RT_FLAG_HW_MATH exclude each other", RT_ERR_INVALID_ARG);
    if (!c0->have_params) return set_err(c0, "rt_render_tiled: no params set on ctxs[0]", RT_ERR_NO_SCENE);
    for (int32_t k = 0; k < n; ++k)
        if (!ctxs[k]->have_scene)
            return set_err(c0, "rt_render_tiled: ctxs[" + std::to_string(k) + "] has no scene (rt_scene_copy)", RT_ERR_NO_SCENE);
    if (n == 1) return rt_render(c0, w, h, depth, flags, out_bgr, nullptr);
    const size_t npix = (size_t)w * h;
    // the frame as every context's device addresses it: the caller's buffer if all of them map it
    uint64_t addr[kMaxTiled] = {};
    for (int32_t k = 0; k < n; ++k) {
        void* dp = nullptr;
        if (hipSetDevice(ctxs[k]->device) == hipSuccess && hipHostGetDevicePointer(&dp, out_bgr, 0) == hipSuccess)
            addr[k] = (uint64_t)(uintptr_t)dp;
    }
    (void)hipGetLastError();   // pageable memory: not an error
    const bool staged = !rt_tiled_direct_ok(n, addr);
    if (staged) {
        HIPC(c0, hipSetDevice(c0->device));
        if (c0->stage_cap < npix) {
            if (c0->h_stage) (void)hipHostFree(c0->h_stage);
            c0->h_stage = nullptr;
            c0->stage_cap = 0;
            HIPC(c0, hipHostMalloc((void**)&c0->h_stage, npix * 4, hipHostMallocPortable | hipHostMallocMapped));
            c0->stage_cap = npix;
        }
        for (int32_t k = 0; k < n; ++k) {
            void* dp = nullptr;
            HIPC(c0, hipSetDevice(ctxs[k]->device));
            HIPC(c0, hipHostGetDevicePointer(&dp, c0->h_stage, 0));
            addr[k] = (uint64_t)(uintptr_t)dp;
        }
    }
    const bool workers = tiled_workers_on();
    int32_t posted = 0;
    for (int32_t k = 1; k < n; ++k) {
        rt_ctx* c = ctxs[k];
        c->params = c0->params;   // ctxs[0]'s camera drives the frame (updateCamera, RayTracer.cpp:671)
        c->have_params = true;
    }
    if (workers)
        for (; posted < n - 1; ++posted)
            tiled_post(ctxs[posted + 1], TiledJob{w, h, depth, flags, rt_tiling{posted + 1, n, kTiledBandRows, 0},
                                                  (uint32_t*)(uintptr_t)addr[posted + 1]});
    int rc = RT_OK;
    if (workers) {
        rc = tiled_part(c0, TiledJob{w, h, depth, flags, rt_tiling{0, n, kTiledBandRows, 0}, (uint32_t*)(uintptr_t)addr[0]});
    } else {   // every part enqueued on this thread, one after another, then every stream waited for
        int rk[kMaxTiled];
        for (int32_t k = 0; k < n; ++k)
            rk[k] = tiled_enqueue(ctxs[k], TiledJob{w, h, depth, flags, rt_tiling{k, n, kTiledBandRows, 0},
                                                    (uint32_t*)(uintptr_t)addr[k]});
        for (int32_t k = 0; k < n; ++k) {
            const int r = tiled_wait(ctxs[k], rk[k]);
            if (r && rc == RT_OK) {
                rc = r;
                if (k) c0->err = "rt_render_tiled: ctxs[" + std::to_string(k) + "]: " + ctxs[k]->err;
            }
        }
    }
    // join every posted part, also after a failure (nothing may still write into the frame)
    for (int32_t k = 1; k <= posted; ++k) {
        const int r = tiled_join(ctxs[k]);
        if (r && rc == RT_OK) {
            rc = r;
            c0->err = "rt_render_tiled: ctxs[" + std::to_string(k) + "]: " + ctxs[k]->err;
        }
    }
    (void)hipSetDevice(c0->device);
    if (rc) return rc;
    if (staged) std::memcpy(out_bgr, c0->h_stage, npix * 4);
    return RT_OK;
}

// ---- diagnostics: where a frame's time goes ----

int rt_wave_timeline(rt_ctx* c, uint32_t w, uint32_t h, int32_t depth, uint32_t flags, int32_t frames, uint32_t* words,
                     uint64_t cap_words, uint64_t* used_words) {
    constexpr uint32_t kHead = 128, kMaxLaunches = 32;
    if (!c || !words || !used_words || cap_words < kHead || w == 0 || h == 0 || depth < 1 || depth > RT_MAX_DEPTH ||
        frames < 1 || frames > 8 || (uint64_t)frames * (uint64_t)depth > kMaxLaunches)
        return set_err(c, "rt_wave_timeline: invalid argument", RT_ERR_INVALID_ARG);
    if ((flags & (RT_FLAG_STRICT_MATH | RT_FLAG_HW_MATH | RT_FLAG_EXACT_DIV)) || (depth > 1 && !(flags & RT_FLAG_WAVEFRONT)) ||
        !c->have_scene || !c->clean || c->split_records)
        return set_err(c, "rt_wave_timeline: the default arithmetic's fast kernels of a clean scene, depth 1 or the wavefront path",
                       RT_ERR_INVALID_ARG);
    HIPC(c, hipSetDevice(c->device));
    const size_t npix = (size_t)w * h;
    int rc = ensure(c, c->d_out, c->out_cap, npix * (size_t)frames);
    if (rc) return rc;
    if ((rc = ensure(c, c->tline.d_words, c->tline.cap, (size_t)cap_words))) return rc;
    // frame f in flight renders on stream f: the ctx stream, then the row-group streams (their own
    // frame slots and longest-first orders); a few untimed rounds first, so every stream's order is
    // built from its own previous frame, as for the frames the product keeps in flight
    hipStream_t st[8];
    st[0] = c->stream;
    for (int32_t f = 1; f < frames; ++f) {
        if (!c->gstream[f - 1]) HIPC(c, hipStreamCreateWithFlags(&c->gstream[f - 1], hipStreamNonBlocking));
        st[f] = c->gstream[f - 1];
    }
    if (frames > 1) {
        for (int r = 0; r < 3; ++r)
            for (int32_t f = 0; f < frames; ++f)
                if ((rc = rt_render_device(c, w, h, depth, flags, nullptr, c->d_out + (size_t)f * npix, nullptr, st[f])))
                    return rc;
        for (int32_t f = 0; f < frames; ++f) HIPC(c, hipStreamSynchronize(st[f]));
    }
    HIPC(c, hipMemsetAsync(c->tline.d_words, 0, (size_t)cap_words * 4, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    c->tline.on = true;
    c->tline.limit = (size_t)cap_words - kHead;
    c->tline.used = 0;
    c->tline.waves.clear();
    c->tline.frame.clear();
    c->tline.bounce.clear();
    const uint64_t f0 = c->frames;
    for (int32_t f = 0; f < frames && rc == RT_OK; ++f) {
        c->tline.cur_frame = (uint32_t)f;
        const size_t first = c->tline.waves.size();
        rc = rt_render_device(c, w, h, depth, flags, nullptr, c->d_out + (size_t)f * npix, nullptr, st[f]);
        for (size_t i = first; i < c->tline.bounce.size(); ++i) c->tline.bounce[i] = (uint32_t)(i - first);
    }
    c->tline.on = false;
    for (int32_t f = 0; f < frames; ++f) HIPC(c, hipStreamSynchronize(st[f]));
    if (rc) return rc;
    float t = 0.0f, k = 0.0f;
    if ((rc = frame_times(c, f0, t, k))) return rc;   // the first frame's kernels
    const size_t L = c->tline.waves.size();
    if (L > kMaxLaunches) return set_err(c, "rt_wave_timeline: too many launches", RT_ERR_INVALID_ARG);
    std::memset(words, 0, kHead * 4);
    words[0] = (uint32_t)L;
    words[1] = (uint32_t)frames;
    words[2] = (uint32_t)std::lround((double)t * 1e6);   // the first frame's kernels, HIP events, ns
    words[3] = (uint32_t)std::lround((double)k * 1e6);   // its first launch
    words[4] = rtk::kTlRecord;                            // words per wave record
    words[5] = RTK_TL_SPLIT;                              // memory-wait words stamped
    for (size_t i = 0; i < L; ++i) {
        words[8 + i] = c->tline.waves[i];
        words[40 + i] = c->tline.frame[i];
        words[72 + i] = c->tline.bounce[i];
    }
    HIPC(c, hipMemcpy(words + kHead, c->tline.d_words, c->tline.used * 4, hipMemcpyDeviceToHost));
    *used_words = kHead + c->tline.used;
    return RT_OK;
}

int rt_overflow_count(rt_ctx* c, uint64_t* count) {
    if (!c || !count) return RT_ERR_INVALID_ARG;
    unsigned long long v = 0;
    HIPC(c, hipMemcpy(&v, c->d_overflow, sizeof v, hipMemcpyDeviceToHost));
    *count = v;
    return RT_OK;
}

}  // extern "C"
