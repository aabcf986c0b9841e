/*
 * Analysis tool (not product, not a test): replays the reference-order traversal of every
 * lane of sampled 8x8 tiles (oracle/rt_oracle.c's arithmetic and visit order) and
 * simulates how a wave's lanes could be scheduled in the fast kernel's if-if loop.
 * Scheduling never changes a lane's own sequence of steps (so never its result); it only
 * decides which lanes take their next step in a given iteration.  The cost model is the
 * one measured by scripts/micro/share_fetch.hip and td_mask.hip: per iteration and per
 * quad of lanes, one fetch unit when every stepping lane of the quad reads the same record,
 * otherwise one unit per stepping lane; idle lanes cost nothing.
 *
 * Policies:  0 = every live lane steps (the current kernel);
 *            1 = in each quad only the lanes whose next step is first in left-first DFS
 *                order step (key = reference node index, then triangle position);
 *            2..= policy 1, except a lane that has waited W iterations steps anyway.
 * Build: gcc -O2 -shared -fPIC -o scripts/libquadsim.so scripts/quad_sched_sim.c -lm
 */
#include <stdlib.h>
#include "../oracle/rt_oracle.c"

typedef struct { uint32_t rec; uint32_t key; } qstep;
typedef struct { qstep* v; int n, cap; } qseq;

/* key mode 1: the key a kernel can form from a ref alone -- inner node: its rank in
 * pre-order over inner nodes scaled by (tri refs / inner nodes); triangle step: its
 * tri-ref offset in leaf order */
static int g_keymode = 0;
static const int32_t* g_irank = 0;
static double g_ratio = 1.0;

static void qpush(qseq* s, uint32_t rec, uint32_t key) {
    if (s->n == s->cap) { s->cap = s->cap ? 2 * s->cap : 64; s->v = (qstep*)realloc(s->v, sizeof(qstep) * s->cap); }
    s->v[s->n].rec = rec; s->v[s->n].key = key; s->n++;
}

/* o_traverse (volumeRender.cl:776-1009) with every fetch logged */
static int q_traverse(const oscene* s, const oray* ray, float* tHit, int closest, qseq* log) {
    int stack[O_STACK_SIZE];
    int stack_count = 1;
    stack[0] = 0;
    int tri_index = -1;
    while (stack_count > 0) {
        int nodeIndex = stack[stack_count - 1];
        const onode* nd = &s->nodes[nodeIndex];
        int offset_left = nd->l;
        if (offset_left >= 0) {
            int offset_right = nd->r;
            qpush(log, (uint32_t)nodeIndex, g_keymode ? (uint32_t)((double)g_irank[nodeIndex] * g_ratio)
                                                      : (uint32_t)nodeIndex << 5);
            if (offset_right < 0 || offset_left >= s->num_nodes || offset_right >= s->num_nodes) return -1;
            float n0, f0, n1, f1;
            o_ray_box(ray, s->nodes[offset_left].min, s->nodes[offset_left].max, &n0, &f0);
            o_ray_box(ray, s->nodes[offset_right].min, s->nodes[offset_right].max, &n1, &f1);
            int i0 = (n0 <= f0) && (f0 >= O_TMIN) && (n0 <= *tHit);
            int i1 = (n1 <= f1) && (f1 >= O_TMIN) && (n1 <= *tHit);
            if (i0 && i1) {
                if (n0 > n1) { int t = offset_left; offset_left = offset_right; offset_right = t; }
                stack[stack_count - 1] = offset_right;
                if (stack_count >= O_STACK_SIZE) return -1;
                stack[stack_count] = offset_left;
                ++stack_count;
            } else if (i0) {
                stack[stack_count - 1] = offset_left;
            } else if (i1) {
                stack[stack_count - 1] = offset_right;
            } else {
                --stack_count;
            }
        } else {
            int off = nd->off, cnt = nd->cnt;
            for (int i = 0; i < cnt; ++i) {
                int tri1 = s->refs[off + i];
                of4 a = s->verts[s->idx[tri1 + 0]];
                of4 b = s->verts[s->idx[tri1 + 1]];
                of4 d = s->verts[s->idx[tri1 + 2]];
                qpush(log, 0x80000000u | (uint32_t)(off + i),
                      g_keymode ? (uint32_t)(off + i) : ((uint32_t)nodeIndex << 5) | (uint32_t)(i < 30 ? i + 1 : 31));
                float t = o_ray_tri(ray, x3(a), v3(b.x - a.x, b.y - a.y, b.z - a.z), v3(d.x - a.x, d.y - a.y, d.z - a.z));
                if (t < *tHit && t > O_TMIN) {
                    *tHit = t;
                    if (!closest) return tri1;
                    tri_index = tri1;
                }
            }
            --stack_count;
        }
    }
    return tri_index;
}

/* depth-1 pixel (o_pixel, volumeRender.cl:1169-1500): primary and shadow fetch logs */
static void q_pixel(const oscene* s, const oparams* P, uint32_t w, uint32_t h, uint32_t x, uint32_t y, qseq* prim,
                    qseq* shad) {
    f3 a = x3(P->a), b = x3(P->b), c = x3(P->c), campos = x3(P->campos), light_pos = x3(P->light_pos);
    float xf = (float)(((double)x - 0.5) / (double)(float)w);
    float yf = (float)(((double)y - 0.5) / (double)(float)h);
    f3 image_pos = add3(add3(c, muls(a, xf)), muls(b, yf));
    oray r;
    o_ray_init(&r, image_pos, sub3(image_pos, campos));
    float tHit = (float)4294967295u, tmin, tmax;
    if (!o_ray_box_scene(x3(P->smin), x3(P->smax), r.ori, r.inv_dir, &tmin, &tmax)) return;
    int hit = q_traverse(s, &r, &tHit, 1, prim);
    if (hit < 0 || !shad) return;
    f3 vNew = add3(r.ori, muls(r.dir, tHit - 0.001f));
    f3 L = o_normalize(sub3(light_pos, vNew));
    oray sr;
    o_ray_init(&sr, add3(vNew, muls(L, 0.001f)), L);
    float ts = (float)4294967295u;
    q_traverse(s, &sr, &ts, 0, shad);
}

/* one wave's loop under a policy: returns iterations, adds fetch units */
static int64_t q_wave(qseq* seq, int policy, double* units) {
    int pos[64] = {0}, waited[64] = {0};
    int64_t it = 0;
    for (;;) {
        int live = 0;
        for (int l = 0; l < 64; ++l) live |= pos[l] < seq[l].n;
        if (!live) break;
        it++;
        int step[64];
        for (int q = 0; q < 16; ++q) {
            uint32_t kmin = 0xFFFFFFFFu;
            for (int l = 4 * q; l < 4 * q + 4; ++l)
                if (pos[l] < seq[l].n && seq[l].v[pos[l]].key < kmin) kmin = seq[l].v[pos[l]].key;
            int nst = 0, same = 1;
            uint32_t rec0 = 0;
            for (int l = 4 * q; l < 4 * q + 4; ++l) {
                step[l] = 0;
                if (pos[l] >= seq[l].n) continue;
                int go = policy == 0 || seq[l].v[pos[l]].key == kmin || (policy >= 2 && waited[l] >= policy);
                if (!go) { waited[l]++; continue; }
                step[l] = 1;
                waited[l] = 0;
                if (nst == 0) rec0 = seq[l].v[pos[l]].rec;
                else if (seq[l].v[pos[l]].rec != rec0) same = 0;
                nst++;
            }
            if (nst) *units += same ? 1.0 : (double)nst;
        }
        for (int l = 0; l < 64; ++l) pos[l] += step[l];
    }
    return it;
}

/* Morton lane -> (x, y) inside an 8x8 tile: quads are 2x2 squares */
static void q_lane_xy(int l, int* x, int* y) {
    *x = (l & 1) | ((l >> 1) & 2) | ((l >> 2) & 4);
    *y = ((l >> 1) & 1) | ((l >> 2) & 2) | ((l >> 3) & 4);
}

/*
 * out[p*4 + {0,1,2,3}] for policy p in [0, npol): primary units, primary iterations (sum
 * over waves), shadow units, shadow iterations.  out2[p*2 + {0,1}]: max wave iterations
 * (primary + shadow).  Tiles sampled every tile_stride-th tile.
 */
int quad_sim(const oparams* params, const of4* verts, const int32_t* idx, const onode* nodes, int32_t num_nodes,
             const int32_t* refs, int32_t num_refs, const of4* normals, const int32_t* nidx, const omat* mats,
             const int32_t* tri2mat, uint32_t w, uint32_t h, int shadow, int tile_stride, const int* policies,
             int npol, double* out, double* out2, int64_t* nlane_steps, int keymode) {
    int32_t* irank = (int32_t*)malloc(sizeof(int32_t) * (size_t)num_nodes);
    int32_t ninner = 0;
    for (int32_t n = 0; n < num_nodes; ++n) irank[n] = nodes[n].l >= 0 ? ninner++ : -1;
    g_irank = irank;
    g_ratio = (double)num_refs / (double)(ninner ? ninner : 1);
    g_keymode = keymode;
    oscene s = {verts, idx, nodes, num_nodes, refs, num_refs, normals, nidx, mats, tri2mat};
    uint32_t tx = (w + 7) / 8, ty = (h + 7) / 8;
    qseq prim[64], shad[64];
    memset(prim, 0, sizeof prim);
    memset(shad, 0, sizeof shad);
    for (int p = 0; p < npol; ++p) { out[4 * p] = out[4 * p + 1] = out[4 * p + 2] = out[4 * p + 3] = 0; out2[2 * p] = out2[2 * p + 1] = 0; }
    nlane_steps[0] = nlane_steps[1] = 0;
    for (uint64_t t = 0; t < (uint64_t)tx * ty; t += (uint64_t)tile_stride) {
        uint32_t bx = (uint32_t)(t % tx), by = (uint32_t)(t / tx);
        for (int l = 0; l < 64; ++l) {
            int x, y;
            q_lane_xy(l, &x, &y);
            prim[l].n = shad[l].n = 0;
            uint32_t px = bx * 8 + (uint32_t)x, py = by * 8 + (uint32_t)y;
            if (px < w && py < h) q_pixel(&s, params, w, h, px, py, &prim[l], shadow ? &shad[l] : 0);
            nlane_steps[0] += prim[l].n;
            nlane_steps[1] += shad[l].n;
        }
        for (int p = 0; p < npol; ++p) {
            int64_t ip = q_wave(prim, policies[p], &out[4 * p]);
            int64_t is = q_wave(shad, policies[p], &out[4 * p + 2]);
            out[4 * p + 1] += (double)ip;
            out[4 * p + 3] += (double)is;
            if ((double)(ip + is) > out2[2 * p]) out2[2 * p] = (double)(ip + is);
            out2[2 * p + 1] += 1;
        }
    }
    for (int l = 0; l < 64; ++l) { free(prim[l].v); free(shad[l].v); }
    free(irank);
    return 0;
}
