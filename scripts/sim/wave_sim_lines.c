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
    int tk, tend;            // leaf state
    float th; int res; int any; int done;
} lane;

static void lane_init(lane* L, f3 o, f3 d, int any) {
    L->o = o; L->d = nrm(d); L->sc = 1; L->stack[0] = 0; L->th = 4294967296.0f; L->res = -1; L->any = any; L->done = 0;
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
static void lane_step(lane* L) {
    int cur = L->stack[L->sc - 1];
    const node* n = &N[cur];
    if (n->l >= 0) {
        float n0, f0, n1, f1;
        slab(L, &N[n->l], &n0, &f0); slab(L, &N[n->r], &n1, &f1);
        int i0 = n0 <= f0 && f0 >= 0.001f && n0 <= L->th, i1 = n1 <= f1 && f1 >= 0.001f && n1 <= L->th;
        int a = n->l, b = n->r;
        if (i0 && i1) { if (n0 > n1) { int t = a; a = b; b = t; } L->stack[L->sc - 1] = b; L->stack[L->sc++] = a; if (L->sc >= 65) { L->done = 1; L->sc = 0; return; } }
        else if (i0) L->stack[L->sc - 1] = a;
        else if (i1) L->stack[L->sc - 1] = b;
        else L->sc--;
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
        else if (L->tk >= L->tend) { L->sc--; enter_top(L); }
    }
    if (L->sc == 0) L->done = 1;
}


static int* pre_id; static int* pair_id;   // inner node -> record id in the two layouts
static long long lines_pre = 0, lines_pair = 0, waves = 0, inner_visits = 0;
static int lane_steps_rec(lane* L, int* recs, int* nrec) {
    int n = 0;
    while (!L->done && L->sc > 0) {
        int cur = L->stack[L->sc - 1];
        if (N[cur].l >= 0) recs[(*nrec)++] = cur;
        lane_step(L); ++n;
    }
    return n;
}
static int cmpi(const void* x, const void* y) { int a = *(const int*)x, b = *(const int*)y; return a < b ? -1 : a > b; }
static long long distinct_lines(int* recs, int n, const int* idmap, int* tmp) {
    for (int i = 0; i < n; ++i) tmp[i] = idmap[recs[i]] >> 1;
    qsort(tmp, n, sizeof(int), cmpi);
    long long d = 0;
    for (int i = 0; i < n; ++i) if (i == 0 || tmp[i] != tmp[i - 1]) ++d;
    return d;
}
int main() {
    size_t s;
    N = (node*)rd("c3_nodes.bin", &s); NN = (int)(s / sizeof(node));
    V = (float*)rd("c3_vertices.bin", 0); IDX = (int32_t*)rd("c3_indices.bin", 0); REF = (int32_t*)rd("c3_tri_indices.bin", 0);
    memcpy(P, rd("c3_params.bin", 0), 128); memcpy(SMIN, rd("c3_scene_min.bin", 0), 12); memcpy(SMAX, rd("c3_scene_max.bin", 0), 12);
    bfs = malloc(sizeof(int) * NN); for (int i = 0; i < NN; ++i) bfs[i] = -1;
    int* qq = malloc(sizeof(int) * NN); int h = 0, t = 0, rank = 0; qq[t++] = 0;
    while (h < t) { int n = qq[h++]; if (N[n].l < 0) continue; bfs[n] = rank++; qq[t++] = N[n].l; qq[t++] = N[n].r; }
    // layout 1 (product): BFS top 1024 then pre-order of inner nodes
    pre_id = malloc(sizeof(int) * NN); pair_id = malloc(sizeof(int) * NN);
    for (int i = 0; i < NN; ++i) pre_id[i] = pair_id[i] = -1;
    {
        int id = 0;
        for (int i = 0; i < NN; ++i) if (bfs[i] >= 0 && bfs[i] < 1024) pre_id[i] = bfs[i];
        id = 1024;
        int* st = malloc(sizeof(int) * NN); int sp = 0; st[sp++] = 0;
        while (sp) { int n = st[--sp]; if (N[n].l < 0) continue; if (pre_id[n] < 0) pre_id[n] = id++; st[sp++] = N[n].r; st[sp++] = N[n].l; }
        // layout 2: children pairs aligned (2k, 2k+1); root alone at 1; BFS for the top, then DFS allocating pairs
        int nid = 2;
        pair_id[0] = 1;
        // BFS top: allocate children pairs level by level until 1024 ids
        int* q = malloc(sizeof(int) * NN); int h = 0, t = 0; q[t++] = 0;
        while (h < t && nid < 1024) { int n = q[h++]; if (N[n].l < 0) continue;
            int L = N[n].l, R = N[n].r; int li = N[L].l >= 0, ri = N[R].l >= 0;
            if (li || ri) { if (li) pair_id[L] = nid; if (ri) pair_id[R] = nid + 1; nid += 2; }
            if (li) q[t++] = L; if (ri) q[t++] = R; }
        // the rest: DFS from the unexpanded frontier
        sp = 0; for (int i = t - 1; i >= h; --i) st[sp++] = q[i];
        while (sp) { int n = st[--sp]; if (N[n].l < 0) continue;
            int L = N[n].l, R = N[n].r; int li = N[L].l >= 0, ri = N[R].l >= 0;
            if (li || ri) { if (nid & 1) nid++; if (li) pair_id[L] = nid; if (ri) pair_id[R] = nid + 1; nid += 2; }
            if (ri) st[sp++] = R; if (li) st[sp++] = L; }
        printf("records: pre-order %d, pairs %d\n", id, nid);
    }
    const int W = 1920, H = 1080;
    f3 a = v3(P[0], P[1], P[2]), b = v3(P[4], P[5], P[6]), c = v3(P[8], P[9], P[10]), cam = v3(P[12], P[13], P[14]);
    f3 light = v3(P[16], P[17], P[18]);
    static lane L[64];
    int* recs = malloc(sizeof(int) * 200000); int* tmp = malloc(sizeof(int) * 200000);
    for (int ty = 0; ty < H / 8; ++ty)
        for (int tx = 0; tx < W / 8; ++tx) {
            int nrec = 0;
            for (int l = 0; l < 64; ++l) {
                int lx = (l & 1) | ((l >> 1) & 2) | ((l >> 2) & 4), ly = ((l >> 1) & 1) | ((l >> 2) & 2) | ((l >> 3) & 4);
                int x = tx * 8 + lx, y = ty * 8 + ly;
                float xf = (float)((x - 0.5) / W), yf = (float)((y - 0.5) / H);
                f3 ip = add(add(c, mul(a, xf)), mul(b, yf));
                lane_init(&L[l], ip, sub(ip, cam), 0);
                float tmin = -1e30f, tmax = 1e30f; int hit = 1;
                const float* o = &L[l].o.x; const float* d = &L[l].d.x;
                for (int k = 0; k < 3; ++k) { float i1 = (SMIN[k] - o[k]) / d[k], i2 = (SMAX[k] - o[k]) / d[k]; tmin = fmaxf(tmin, fminf(i1, i2)); tmax = fminf(tmax, fmaxf(i1, i2)); }
                if (!(tmax >= tmin && tmax >= 0)) hit = 0;
                if (hit) lane_steps_rec(&L[l], recs, &nrec);
                if (hit && L[l].res >= 0) {
                    f3 hp = add(L[l].o, mul(L[l].d, L[l].th - 0.001f));
                    f3 Ld = nrm(sub(light, hp));
                    lane_init(&L[l], add(hp, mul(Ld, 0.001f)), Ld, 1);
                    lane_steps_rec(&L[l], recs, &nrec);
                }
            }
            inner_visits += nrec;
            lines_pre += distinct_lines(recs, nrec, pre_id, tmp);
            lines_pair += distinct_lines(recs, nrec, pair_id, tmp);
            waves++;
        }
    printf("inner visits %lld; distinct 128-B lines per wave: pre-order %.1f, child pairs %.1f (%.3f)\n", inner_visits,
           (double)lines_pre / waves, (double)lines_pair / waves, (double)lines_pair / lines_pre);
    return 0;
}
