// Wave-level simulation of the tile kernel's traversal (8x8 tile per wave, Morton lanes,
// ifif steps, wave-uniform prologue) for C3: counts vector quad requests by record kind and
// by BFS rank of inner records.  Analysis only.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float mn[4], mx[4]; int32_t l, r, off, cnt; } node;
static node* N; static int NN;
static float* V; static int32_t* IDX; static int32_t* REF;
static float P[32]; static float SMIN[3], SMAX[3];
static int* bfs;   // inner node -> bfs rank (-1 for leaves)

static void* rd(const char* f, size_t* n) {
    FILE* fp = fopen(f, "rb"); fseek(fp, 0, SEEK_END); size_t s = ftell(fp); fseek(fp, 0, SEEK_SET);
    void* p = malloc(s); fread(p, 1, s, fp); fclose(fp); if (n) *n = s; return p;
}
typedef struct { float x, y, z; } f3;
static f3 v3(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static f3 sub(f3 a, f3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static f3 add(f3 a, f3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static f3 mul(f3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static f3 cross(f3 a, f3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static f3 nrm(f3 a) { float l = sqrtf(dot(a, a)); return l > 0 ? mul(a, 1.0f / l) : a; }

typedef struct {
    f3 o, d;
    int stack[70]; int sc;   // stack[sc-1] = cur
    float dist[70];          // CULL: entry distance of a pushed far child (-inf: unknown)
    int tk, tend;            // leaf state
    float th; int res; int any; int done;
} lane;

static void lane_init(lane* L, f3 o, f3 d, int any) {
    L->o = o; L->d = nrm(d); L->sc = 1; L->stack[0] = 0; L->dist[0] = -INFINITY; L->th = 4294967296.0f; L->res = -1; L->any = any; L->done = 0;
    L->tk = L->tend = 0;
    if (N[0].l < 0) { L->tk = N[0].off; L->tend = N[0].off + N[0].cnt; }
}
static void slab(const lane* L, const node* b, float* tn, float* tf) {
    float t0[3], t1[3];
    const float* o = &L->o.x; const float* d = &L->d.x;
    for (int k = 0; k < 3; ++k) { t0[k] = (b->mn[k] - o[k]) / d[k]; t1[k] = (b->mx[k] - o[k]) / d[k]; }
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) { lo[k] = fminf(t0[k], t1[k]); hi[k] = fmaxf(t0[k], t1[k]); }
    *tn = fmaxf(fmaxf(lo[0], lo[1]), lo[2]); *tf = fminf(fminf(hi[0], hi[1]), hi[2]);
}
// the record this lane fetches this iteration: >= 0 inner node id, < 0: -(tri ref + 1)
static int lane_record(const lane* L) {
    int cur = L->stack[L->sc - 1];
    if (N[cur].l >= 0) return cur;
    return -(L->tk + 1);
}
static void enter_top(lane* L) {
    if (L->sc > 0) { int c = L->stack[L->sc - 1]; if (N[c].l < 0) { L->tk = N[c].off; L->tend = N[c].off + N[c].cnt; } }
}
static int CULL = 0;             // env CULL=1: a popped inner entry whose entry distance (from its push)
                                 // is beyond tHit is skipped (every entry); CULL=2: only the last pushed one
static long long culled = 0;
// pops: skip inner entries whose box entry (computed when pushed) is beyond the current tHit:
// their visit would cull both children (child boxes lie inside)
static void cull_top(lane* L) {
    if (!CULL || L->any) return;
    while (L->sc > 0) {
        const int top = L->sc - 1, c = L->stack[top];
        if (N[c].l < 0 || !(L->dist[top] > L->th)) return;
        L->sc--; culled++;
        if (CULL == 2) { for (int k = 0; k < L->sc; ++k) L->dist[k] = -INFINITY; }   // LDS entries carry none
    }
}
static long long deep_lanes = 0;   // lanes whose stack outgrew the LDS part (the product restarts them)
static int HELP = 0, HELP_G = 4;   // env HELP=L: with <= L live lanes, a lane in a leaf tests up to HELP_G of
                                  // its triangles per iteration (idle lanes of the wave testing them for it)
static long long helped_extra = 0;
static int T2 = 0, TT2 = 0;   // TT2=1: two triangles of one leaf per iteration   // env T2=1: an inner step that descends into an inner child runs that child's step too
static int descended;  // set by lane_step: this inner step moved cur to a child (push or advance)
static void lane_step(lane* L) {
    int cur = L->stack[L->sc - 1];
    const node* n = &N[cur];
    descended = 0;
    if (n->l >= 0) {
        float n0, f0, n1, f1;
        slab(L, &N[n->l], &n0, &f0); slab(L, &N[n->r], &n1, &f1);
        int i0 = n0 <= f0 && f0 >= 0.001f && n0 <= L->th, i1 = n1 <= f1 && f1 >= 0.001f && n1 <= L->th;
        int a = n->l, b = n->r;
        if (i0 && i1) { float fb = n0 > n1 ? n0 : n1; if (n0 > n1) { int t = a; a = b; b = t; }
                        if (CULL == 2) for (int k = 0; k < L->sc - 1; ++k) L->dist[k] = -INFINITY;
                        L->dist[L->sc - 1] = fb; L->stack[L->sc - 1] = b; L->dist[L->sc] = -INFINITY; L->stack[L->sc++] = a;
                        if (L->sc - 2 == 16) deep_lanes++;   // kLdsStack = 16: the product restarts this ray
                        if (L->sc >= 65) { L->done = 1; L->sc = 0; return; } }
        else if (i0) { L->stack[L->sc - 1] = a; L->dist[L->sc - 1] = -INFINITY; }
        else if (i1) { L->stack[L->sc - 1] = b; L->dist[L->sc - 1] = -INFINITY; }
        else { L->sc--; cull_top(L); }
        descended = (i0 || i1) && L->sc > 0;
        enter_top(L);
    } else {
        int stop = 0;
        if (L->tk < L->tend) {
            int t1 = REF[L->tk];
            f3 a = v3(V[IDX[t1] * 4], V[IDX[t1] * 4 + 1], V[IDX[t1] * 4 + 2]);
            f3 b = v3(V[IDX[t1 + 1] * 4], V[IDX[t1 + 1] * 4 + 1], V[IDX[t1 + 1] * 4 + 2]);
            f3 c = v3(V[IDX[t1 + 2] * 4], V[IDX[t1 + 2] * 4 + 1], V[IDX[t1 + 2] * 4 + 2]);
            f3 e1 = sub(b, a), e2 = sub(c, a), tv = sub(L->o, a), pv = cross(L->d, e2);
            float det = 1.0f / dot(e1, pv); float u = dot(tv, pv) * det;
            if (!(u < 0 || u > 1)) {
                f3 qv = cross(tv, e1); float v = dot(L->d, qv) * det;
                if (!(v < 0 || u + v > 1)) {
                    float t = dot(e2, qv) * det;
                    if (t < L->th && t > 0.001f) { L->th = t; L->res = t1; if (L->any) stop = 1; }
                }
            }
        }
        L->tk++;
        if (stop) L->sc = 0;
        else if (L->tk >= L->tend) { L->sc--; cull_top(L); enter_top(L); }
    }
    if (L->sc == 0) L->done = 1;
}

// per-lane vector loads if a lane took its record from lane 0 of its quad / of its row of 16
// when that lane is still traversing and fetches the same record (RTK_QSHARE 1 / 2)
static long long ld_all = 0, ld_quad = 0, ld_row = 0, ld_both = 0;
static long long q_vec = 0, q_vec_inner = 0, q_vec_tri = 0, lanes_vec = 0, iters = 0, iters_pro = 0;
static long long q_rank[4];   // inner vector quad requests with bfs rank < 256, 512, 1024, 4096
static const int KR[4] = {256, 512, 1024, 4096};
static long long t2_second = 0, lane_steps = 0;   // every lane step of the main loop and the prologue

static void run_wave(lane* L, int* act) {
    // prologue: while all active lanes sit on the same inner node
    for (;;) {
        int first = -1, uni = 1, any = 0;
        for (int i = 0; i < 64; ++i) if (act[i] && L[i].sc > 0) { any = 1; int c = L[i].stack[L[i].sc - 1]; if (first < 0) first = c; else if (c != first) uni = 0; }
        if (!any || !uni || N[first].l < 0) break;
        iters_pro++;
        for (int i = 0; i < 64; ++i) if (act[i] && L[i].sc > 0) { lane_step(&L[i]); lane_steps++; }
    }
    for (;;) {
        int any = 0;
        int rec[64];
        for (int i = 0; i < 64; ++i) { rec[i] = 0x7fffffff; if (act[i] && L[i].sc > 0) { any = 1; rec[i] = lane_record(&L[i]); } }
        if (!any) break;
        iters++;
        for (int q = 0; q < 16; ++q) {
            int seen[4], ns = 0;
            for (int j = 0; j < 4; ++j) {
                int r = rec[q * 4 + j]; if (r == 0x7fffffff) continue;
                lanes_vec++;
                int dup = 0; for (int s = 0; s < ns; ++s) if (seen[s] == r) dup = 1;
                if (!dup) {
                    seen[ns++] = r; q_vec++;
                    if (r >= 0) { q_vec_inner++; for (int k = 0; k < 4; ++k) if (bfs[r] >= 0 && bfs[r] < KR[k]) q_rank[k]++; }
                    else q_vec_tri++;
                }
            }
        }
        for (int i = 0; i < 64; ++i) {
            if (rec[i] == 0x7fffffff) continue;
            const int q0 = i & ~3, r0 = i & ~15;
            const int sq = i != q0 && rec[q0] != 0x7fffffff && rec[q0] == rec[i];
            const int sr = i != r0 && rec[r0] != 0x7fffffff && rec[r0] == rec[i];
            ld_all++;
            ld_quad += !sq;
            ld_row += !sr;
            ld_both += !sq && !sr;
        }
        int live = 0;
        for (int i = 0; i < 64; ++i) live += act[i] && L[i].sc > 0;
        const int help = HELP && live <= HELP;
        for (int i = 0; i < 64; ++i) if (act[i] && L[i].sc > 0) {
            const int leaf0 = L[i].stack[L[i].sc - 1];
            const int in_leaf = N[leaf0].l < 0;
            lane_step(&L[i]); lane_steps++;
            if (help && in_leaf)
                for (int k = 1; k < HELP_G && L[i].sc > 0 && L[i].stack[L[i].sc - 1] == leaf0 && L[i].tk < L[i].tend; ++k) {
                    lane_step(&L[i]); helped_extra++;
                }
            if (T2 && descended && L[i].sc > 0 && N[L[i].stack[L[i].sc - 1]].l >= 0) { lane_step(&L[i]); t2_second++; }
            else if (TT2 && rec[i] < 0 && L[i].sc > 0 && N[L[i].stack[L[i].sc - 1]].l < 0 && L[i].tk < L[i].tend &&
                     lane_record(&L[i]) == rec[i] - 1) { lane_step(&L[i]); t2_second++; }   // the leaf's next triangle
        }
    }
}

int main(int argc, char** argv) {
    const int shadow = argc > 1 ? atoi(argv[1]) : 1;   // 0: primary rays only (C2)
    T2 = getenv("T2") ? atoi(getenv("T2")) : 0;
    TT2 = getenv("TT2") ? atoi(getenv("TT2")) : 0;
    CULL = getenv("CULL") ? atoi(getenv("CULL")) : 0;
    HELP = getenv("HELP") ? atoi(getenv("HELP")) : 0;
    HELP_G = getenv("HELP_G") ? atoi(getenv("HELP_G")) : 4;
    size_t s;
    N = (node*)rd("c3_nodes.bin", &s); NN = (int)(s / sizeof(node));
    V = (float*)rd("c3_vertices.bin", 0); IDX = (int32_t*)rd("c3_indices.bin", 0); REF = (int32_t*)rd("c3_tri_indices.bin", 0);
    memcpy(P, rd("c3_params.bin", 0), 128); memcpy(SMIN, rd("c3_scene_min.bin", 0), 12); memcpy(SMAX, rd("c3_scene_max.bin", 0), 12);
    bfs = malloc(sizeof(int) * NN); for (int i = 0; i < NN; ++i) bfs[i] = -1;
    int* qq = malloc(sizeof(int) * NN); int h = 0, t = 0, rank = 0; qq[t++] = 0;
    while (h < t) { int n = qq[h++]; if (N[n].l < 0) continue; bfs[n] = rank++; qq[t++] = N[n].l; qq[t++] = N[n].r; }
    const int W = 1920, H = 1080;
    f3 a = v3(P[0], P[1], P[2]), b = v3(P[4], P[5], P[6]), c = v3(P[8], P[9], P[10]), cam = v3(P[12], P[13], P[14]);
    f3 light = v3(P[16], P[17], P[18]);
    static lane L[64]; int act[64];
    long long waves_by_live[65] = {0}, it_primary = 0, pro_primary = 0;
    static int wave_len[(1920 / 8) * (1080 / 8)]; int nwl = 0;   // per active wave: primary + shadow iterations
    for (int ty = 0; ty < H / 8; ++ty)
        for (int tx = 0; tx < W / 8; ++tx) {
            for (int l = 0; l < 64; ++l) {
                int lx = (l & 1) | ((l >> 1) & 2) | ((l >> 2) & 4), ly = ((l >> 1) & 1) | ((l >> 2) & 2) | ((l >> 3) & 4);
                int x = tx * 8 + lx, y = ty * 8 + ly;
                float xf = (float)((x - 0.5) / W), yf = (float)((y - 0.5) / H);
                f3 ip = add(add(c, mul(a, xf)), mul(b, yf));
                lane_init(&L[l], ip, sub(ip, cam), 0);
                // scene box
                float tmin = -1e30f, tmax = 1e30f; int hit = 1;
                const float* o = &L[l].o.x; const float* d = &L[l].d.x;
                for (int k = 0; k < 3; ++k) { float i1 = (SMIN[k] - o[k]) / d[k], i2 = (SMAX[k] - o[k]) / d[k]; tmin = fmaxf(tmin, fminf(i1, i2)); tmax = fminf(tmax, fmaxf(i1, i2)); }
                if (!(tmax >= tmin && tmax >= 0)) hit = 0;
                act[l] = hit;
            }
            { int na = 0; for (int l = 0; l < 64; ++l) na += act[l]; waves_by_live[na]++; }
            const long long w0 = iters + iters_pro;
            { const long long i0 = iters, p0 = iters_pro;
              run_wave(L, act);
              it_primary += iters - i0; pro_primary += iters_pro - p0; }
            if (!shadow) { if (iters + iters_pro > w0) wave_len[nwl++] = (int)(iters + iters_pro - w0); continue; }
            for (int l = 0; l < 64; ++l) {
                int hit = act[l] && L[l].res >= 0;
                act[l] = hit;
                if (hit) {
                    f3 hp = add(L[l].o, mul(L[l].d, L[l].th - 0.001f));
                    f3 Ld = nrm(sub(light, hp));
                    lane_init(&L[l], add(hp, mul(Ld, 0.001f)), Ld, 1);
                }
            }
            run_wave(L, act);
            if (iters + iters_pro > w0) wave_len[nwl++] = (int)(iters + iters_pro - w0);
        }
    {   // distribution of a wave's dependent iterations (prologue + main loop): the chain each wave runs
        int cmp(const void* x, const void* y) { return *(const int*)x - *(const int*)y; }
        qsort(wave_len, nwl, sizeof(int), cmp);
        long long sum = 0; for (int i = 0; i < nwl; ++i) sum += wave_len[i];
        printf("waves with work %d: iterations per wave mean %.1f p50 %d p90 %d p99 %d p99.9 %d max %d\n", nwl,
               (double)sum / nwl, wave_len[nwl / 2], wave_len[nwl * 9 / 10], wave_len[nwl * 99 / 100],
               wave_len[nwl * 999 / 1000], wave_len[nwl - 1]);
    }
    printf("lane steps %lld: lane utilisation of the wave iterations %.3f\n", lane_steps,
           (double)lane_steps / (64.0 * (double)(iters + iters_pro)));
    if (T2 || TT2) printf("T2: second inner steps taken without a fetch: %lld\n", t2_second);
    if (CULL) printf("CULL=%d: popped inner entries skipped %lld\n", CULL, culled);
    if (HELP) printf("HELP=%d (groups of %d): triangle tests taken by helper lanes %lld\n", HELP, HELP_G, helped_extra);
    printf("rays whose stack outgrew 16 LDS entries: %lld\n", deep_lanes);
    printf("iters %lld prologue %lld  lane fetches(vec) %lld  quad req %lld (inner %lld tri %lld) lanes/qreq %.3f\n",
           iters, iters_pro, lanes_vec, q_vec, q_vec_inner, q_vec_tri, (double)lanes_vec / q_vec);
    printf("  primary: %lld iterations + %lld prologue; shadow: %lld + %lld\n",
           it_primary, pro_primary, iters - it_primary, iters_pro - pro_primary);
    { long long part = 0; for (int k = 1; k < 64; ++k) part += waves_by_live[k];
      printf("  tiles by lanes inside the scene box: none %lld, all 64 %lld, some %lld\n", waves_by_live[0], waves_by_live[64], part); }
    printf("  vector lane loads: %lld; sharing with quad lane 0: %lld; with row lane 0: %lld; both: %lld\n", ld_all, ld_quad, ld_row, ld_both);
    for (int k = 0; k < 4; ++k) printf("  inner vector quad requests on bfs rank < %d: %lld (%.1f%% of all vector quad requests)\n", KR[k], q_rank[k], 100.0 * q_rank[k] / q_vec);
    return 0;
}
