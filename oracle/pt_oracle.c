/*
 * pt_oracle.c — CPU ORACLE, TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, float64 restatement of the reference's per-pixel radiance loop
 * (thiagoald/pathtracerpython: main.py:23-280, utils.py:21-147) used as the
 * parity checker for the HIP library and as bench.py's `cpu_baseline`
 * ("port").  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it; the product path (pathtracerpython_amd) never does.
 *
 * Parity pin: tests/test_oracle_golden.py checks this file against golden
 * vectors produced by running the unmodified reference under the keyed-RNG
 * harness tests/golden/gen_golden.py (framebuffers, KATs, scene dump).
 *
 * Arithmetic follows the reference formula by formula, in the same operation
 * order, so results agree with numpy to ~1 ulp per op (compile with
 * -ffp-contract=off; x86-64 SSE2 doubles).  Intentional deviations, all
 * sign/rounding-neutral: in_triangle skips the three normalisations
 * (utils.py:81-83) because only the signs of the dot products are used and a
 * zero cross product gives dot 0 -> "not inside" exactly as the reference's
 * NaN does.
 *
 * RNG: the keyed Philox4x32-10 stream documented in tests/golden/philox_ref.py
 * replaces random.uniform (main.py:16, utils.py:9).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/pt_capi.h"

#define ZERO 1e-5      /* main.py:20, utils.py:18 */
#define TAU 6.28       /* main.py:19 */
#define N_LIGHT_SAMPLES 3 /* main.py:23 */

/* ------------------------------------------------------------------ RNG -- */
static void philox4x32_10(const uint32_t ctr_in[4], uint32_t k0, uint32_t k1,
                          uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    philox4x32_10(ctr, key[0], key[1], out);
}

typedef struct { uint64_t seed; uint32_t pixel, sample, bounce; } rng_ctx;

static double keyed_u(const rng_ctx* c, int slot) {
    uint32_t ctr[4] = {c->pixel, c->sample, c->bounce, (uint32_t)(slot >> 2)};
    uint32_t w[4];
    philox4x32_10(ctr, (uint32_t)c->seed, (uint32_t)(c->seed >> 32), w);
    return (double)(w[slot & 3] >> 8) * (1.0 / 16777216.0);
}

/* random.uniform(a, b) = a + (b-a) * random() */
static double uniform_ab(double a, double b, double u) { return a + (b - a) * u; }

/* ------------------------------------------------------------- vectors -- */
static double dot3(const double* a, const double* b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static void sub3(const double* a, const double* b, double* o) {
    o[0] = a[0] - b[0]; o[1] = a[1] - b[1]; o[2] = a[2] - b[2];
}
static void cross3(const double* a, const double* b, double* o) { /* np.cross */
    double x = a[1] * b[2] - a[2] * b[1];
    double y = a[2] * b[0] - a[0] * b[2];
    double z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
static double norm3(const double* a) { return sqrt(dot3(a, a)); } /* np.linalg.norm */
static void normalize3(double* a) {                            /* v / norm(v) */
    double n = norm3(a);
    a[0] /= n; a[1] /= n; a[2] /= n;
}
/* utils.py:48-49 squared_dist(pt1, pt2): sum((pt1_i - pt2_i)^2), from 0 */
static double squared_dist(const double* p1, const double* p2) {
    double s = 0.0;
    for (int i = 0; i < 3; ++i) { double d = p1[i] - p2[i]; s += d * d; }
    return s;
}

/* --------------------------------------------------------------- scene -- */
typedef struct {
    const pt_scene_desc* d;
    double* plane_n;     /* [n_tri][3] normalize(cross(v1-v2, v3-v2)), utils.py:109-111 */
    double light_sum;    /* sum(light areas), utils.py:30 */
    double* light_cum;   /* [n_light+1] running sums, utils.py:31-35 */
    int32_t n_light;
    int32_t light0;      /* first light triangle */
} oscene;

static int oscene_init(oscene* s, const pt_scene_desc* d) {
    memset(s, 0, sizeof(*s));
    s->d = d;
    s->plane_n = (double*)malloc(sizeof(double) * 3 * (size_t)(d->n_tri > 0 ? d->n_tri : 1));
    s->n_light = d->n_tri - d->n_obj_tri;
    s->light0 = d->n_obj_tri;
    s->light_cum = (double*)malloc(sizeof(double) * (size_t)(s->n_light + 1));
    if (!s->plane_n || !s->light_cum) return -1;
    for (int t = 0; t < d->n_tri; ++t) {
        const double* v = d->tri_v + 9 * t;
        double a[3], b[3];
        sub3(v + 0, v + 3, a);
        sub3(v + 6, v + 3, b);
        cross3(a, b, s->plane_n + 3 * t);
        normalize3(s->plane_n + 3 * t);
    }
    double acc = 0.0;
    s->light_cum[0] = 0.0;
    for (int i = 0; i < s->n_light; ++i) {
        acc += d->tri_area[s->light0 + i];
        s->light_cum[i + 1] = acc;
    }
    s->light_sum = acc; /* Python sum() adds left to right from 0, like acc */
    return 0;
}
static void oscene_free(oscene* s) { free(s->plane_n); free(s->light_cum); }

/* ------------------------------------------------------- intersection -- */
/* utils.py:72-91 in_triangle (signs only, see header) */
static int in_triangle(const double* p, const double* v) {
    const double *v1 = v, *v2 = v + 3, *v3 = v + 6;
    double e[3], w[3], c1[3], c2[3], c3[3];
    sub3(v1, v2, e); sub3(p, v2, w); cross3(e, w, c1);
    sub3(v2, v3, e); sub3(p, v3, w); cross3(e, w, c2);
    sub3(v3, v1, e); sub3(p, v1, w); cross3(e, w, c3);
    return dot3(c1, c2) > 0.0 && dot3(c1, c3) > 0.0;
}

/* utils.py:98-147 intersect(ray, triangle): returns 1 and P on a hit.
 * `dn` is the already-normalised direction (utils.py:110). */
static int intersect_tri(const oscene* s, int t, const double* o, const double* dn,
                         double* P) {
    const double* vp = s->plane_n + 3 * t;
    const double* v1 = s->d->tri_v + 9 * t;
    double dot = dot3(dn, vp);
    if (!(fabs(dot) > ZERO)) return 0;
    double tt = (dot3(vp, v1) - dot3(vp, o)) / dot3(vp, dn);
    P[0] = o[0] + dn[0] * tt;
    P[1] = o[1] + dn[1] * tt;
    P[2] = o[2] + dn[2] * tt;
    return in_triangle(P, v1);
}

int oracle_intersect(const double* tri_v9, const double* o, const double* d,
                     double* P) {
    pt_scene_desc dd;
    memset(&dd, 0, sizeof(dd));
    dd.n_tri = 1; dd.n_obj_tri = 1; dd.tri_v = tri_v9;
    double area = 0.0; dd.tri_area = &area;
    oscene s;
    if (oscene_init(&s, &dd)) return -1;
    double dn[3] = {d[0], d[1], d[2]};
    normalize3(dn);
    int h = intersect_tri(&s, 0, o, dn, P);
    oscene_free(&s);
    return h;
}

typedef struct {
    uint64_t closest_tests, shadow_tests, ray_bounces, shading_points;
    uint64_t light_hits, escapes;
} ocount;

/* main.py:83-122 intersect_objects: closest triangle with sqd > ZERO; first
 * minimum wins (min() keeps the first of equal keys). */
static int closest_hit(const oscene* s, const double* o, const double* d,
                       double* P_out, ocount* cnt) {
    double dn[3] = {d[0], d[1], d[2]};
    normalize3(dn);
    int best = -1;
    double best_sqd = 0.0;
    for (int t = 0; t < s->d->n_tri; ++t) {
        double P[3];
        if (cnt) cnt->closest_tests++;
        if (!intersect_tri(s, t, o, dn, P)) continue;
        double sqd = squared_dist(P, o);
        if (!(sqd > ZERO)) continue;
        if (best < 0 || sqd < best_sqd) {
            best = t; best_sqd = sqd;
            P_out[0] = P[0]; P_out[1] = P[1]; P_out[2] = P[2];
        }
    }
    return best;
}

int oracle_intersect_objects(const pt_scene_desc* d, const double* rays, int64_t n,
                             int32_t* out_tri, double* out_p) {
    oscene s;
    if (oscene_init(&s, d)) return -1;
    for (int64_t i = 0; i < n; ++i) {
        double P[3] = {0, 0, 0};
        out_tri[i] = closest_hit(&s, rays + 6 * i, rays + 6 * i + 3, P, NULL);
        out_p[3 * i] = P[0]; out_p[3 * i + 1] = P[1]; out_p[3 * i + 2] = P[2];
    }
    oscene_free(&s);
    return 0;
}

/* utils.py:28-39 pick_random_triangle: index i with cum[i] <= n < cum[i+1] */
static int pick_light(const oscene* s, double u) {
    double n = uniform_ab(0.0, s->light_sum, u);
    for (int i = 0; i < s->n_light; ++i)
        if (s->light_cum[i] <= n && n < s->light_cum[i + 1]) return i;
    return -1; /* the reference returns None and then fails on indexing */
}

int oracle_pick_light(const pt_scene_desc* d, double u) {
    oscene s;
    if (oscene_init(&s, d)) return -2;
    int i = pick_light(&s, u);
    oscene_free(&s);
    return i;
}

/* utils.py:42-46 + :21-25 sample_random_pt(triangle) with bary = u/sum(u) */
static void sample_light_pt(const double* v, const double* u3, double* L) {
    double sum = 0.0 + u3[0] + u3[1] + u3[2];
    double a = u3[0] / sum, b = u3[1] / sum, c = u3[2] / sum;
    for (int i = 0; i < 3; ++i) L[i] = a * v[i] + b * v[3 + i] + c * v[6 + i];
}

/* main.py:23-73 compute_shadow_rays + main.py:76-80 ambient + main.py:142-145.
 * u12: the 12 uniforms of slots 0..11 in draw order. */
static void compute_color(const oscene* s, int obj, const double* P, const double* n,
                          const double* u12, double* rgb, ocount* cnt) {
    const pt_scene_desc* d = s->d;
    const double* m = d->mat + 8 * obj;
    double dot = 0.0;            /* main.py:65 */
    int leak = d->n_obj - 1;     /* the loop variable `obj` of main.py:42 */
    for (int k = 0; k < N_LIGHT_SAMPLES; ++k) {
        int li = pick_light(s, u12[4 * k]);
        if (li < 0) li = 0;
        double L[3], l[3];
        sample_light_pt(d->tri_v + 9 * (s->light0 + li), u12 + 4 * k + 1, L);
        sub3(L, P, l);
        normalize3(l);
        double light_sqd = squared_dist(P, L);
        int done = 0;
        int obj_last = d->n_obj - 1;
        for (int t = 0; t < d->n_obj_tri && !done; ++t) {
            double Q[3];
            obj_last = d->tri_obj[t];
            if (cnt) cnt->shadow_tests++;
            if (!intersect_tri(s, t, P, l, Q)) continue;
            double sqd = squared_dist(Q, P);
            if (sqd < ZERO) continue;
            if (sqd < light_sqd) done = 1;
        }
        if (done) leak = obj_last;
        else leak = d->n_obj - 1;
        if (!done) dot += dot3(l, n);
    }
    dot /= (double)N_LIGHT_SAMPLES;
    const double* lm = d->mat + 8 * leak;
    for (int c = 0; c < 3; ++c) {
        double amb = m[c] * m[3] * d->ambient;
        double sha = d->light_rgb[c] * lm[c] * dot;
        rgb[c] = amb + sha;
    }
}

int oracle_compute_color(const pt_scene_desc* d, const int32_t* obj, const double* point,
                         const double* normal, const double* u, int64_t n, double* out) {
    oscene s;
    if (oscene_init(&s, d)) return -1;
    for (int64_t i = 0; i < n; ++i)
        compute_color(&s, obj[i], point + 3 * i, normal + 3 * i, u + 12 * i, out + 3 * i, NULL);
    oscene_free(&s);
    return 0;
}

/* main.py:148-162 rotate(axis=(0,1,0), angle, v), literal formula */
static void rotate_y(double angle, const double* v, double* out) {
    double a = cos(angle / 2.0);
    double sn = sin(angle / 2.0);
    double b = -0.0 * sn, c = -1.0 * sn, dd = -0.0 * sn;
    double aa = a * a, bb = b * b, cc = c * c, d2 = dd * dd;
    double bc = b * c, ad = a * dd, ac = a * c, ab = a * b, bd = b * dd, cd = c * dd;
    double M[3][3] = {{aa + bb - cc - d2, 2 * (bc + ad), 2 * (bd - ac)},
                      {2 * (bc - ad), aa + cc - bb - d2, 2 * (cd + ab)},
                      {2 * (bd + ac), 2 * (cd - ab), aa + d2 - bb - cc}};
    for (int i = 0; i < 3; ++i) out[i] = M[i][0] * v[0] + M[i][1] * v[1] + M[i][2] * v[2];
}

void oracle_rotate(const double* n, const double* v, double* out) {
    /* angle = arccos(dot((0,1,0), normal)) = arccos(n_y), main.py:248-249 */
    rotate_y(acos(0.0 * n[0] + 1.0 * n[1] + 0.0 * n[2]), v, out);
}

/* utils.py:64-69 make_screen_pts: np.linspace semantics */
static double linspace_at(double a, double b, int n, int i) {
    if (n == 1) return a;
    if (i == n - 1) return b;
    double step = (b - a) / (double)(n - 1);
    return (double)i * step + a;
}

/* One path sample of pixel k = ix*H + iy: main.py:186-271 for a single ray. */
static void path_sample(const oscene* s, const pt_render_params* p, int64_t pixel_k,
                        int sample, double* rgb, ocount* cnt) {
    const pt_scene_desc* d = s->d;
    int H = p->height, W = p->width;
    int ix = (int)(pixel_k / H), iy = (int)(pixel_k % H);
    double pt[3] = {linspace_at(d->ortho[0], d->ortho[2], W, ix),
                    linspace_at(d->ortho[1], d->ortho[3], H, iy), 0.0};
    double o[3] = {d->eye[0], d->eye[1], d->eye[2]};
    double dir[3];
    sub3(pt, o, dir);                        /* utils.py:57-58, unnormalised */
    double k = 1.0;                          /* accumulated_k, main.py:190 */
    rgb[0] = rgb[1] = rgb[2] = 0.0;
    rng_ctx rc = {p->seed, (uint32_t)pixel_k, (uint32_t)sample, 0};
    for (int b = 0; b < p->bounces; ++b) {
        double P[3];
        if (cnt) cnt->ray_bounces++;
        int t = closest_hit(s, o, dir, P, cnt);
        if (t < 0) { if (cnt) cnt->escapes++; break; }
        if (t >= d->n_obj_tri) {             /* light: main.py:214-215, :266 */
            for (int c = 0; c < 3; ++c) rgb[c] += d->light_rgb[c] * k;
            if (cnt) cnt->light_hits++;
            break;
        }
        int obj = d->tri_obj[t];
        const double* n = d->tri_n + 3 * t;
        const double* m = d->mat + 8 * obj;
        rc.bounce = (uint32_t)b;
        double u12[12], col[3];
        for (int j = 0; j < 12; ++j) u12[j] = keyed_u(&rc, j);
        if (cnt) cnt->shading_points++;
        compute_color(s, obj, P, n, u12, col, cnt);
        for (int c = 0; c < 3; ++c) rgb[c] += col[c] * k;   /* main.py:230-231 */
        /* next ray, main.py:236-268 */
        double nd[3];
        double xi = uniform_ab(0.0, m[4] + m[5], keyed_u(&rc, 12));
        if (xi <= m[4]) {                    /* diffuse */
            double phi = acos(sqrt(uniform_ab(0.0, 1.0, keyed_u(&rc, 13))));
            double theta = TAU * uniform_ab(0.0, 1.0, keyed_u(&rc, 14));
            double v[3] = {sin(phi) * cos(theta), sin(phi) * sin(theta), cos(phi)};
            normalize3(v);
            oracle_rotate(n, v, nd);
            k *= m[4] * dot3(nd, n);
        } else {                             /* "specular" */
            double ndd = dot3(n, dir);
            double r[3], e[3];
            for (int c = 0; c < 3; ++c) r[c] = ndd * 2 * n[c] - dir[c];
            normalize3(r);
            sub3(d->eye, P, e);
            normalize3(e);
            oracle_rotate(n, r, nd);
            k *= m[5] * pow(dot3(e, nd), m[7]);
        }
        if ((p->flags & PT_FLAG_RR) && b >= p->rr_depth) {   /* build extension */
            double q = fabs(k);
            q = q < 0.05 ? 0.05 : (q > 1.0 ? 1.0 : q);
            if (keyed_u(&rc, 15) >= q) break;
            k /= q;
        }
        o[0] = P[0]; o[1] = P[1]; o[2] = P[2];
        dir[0] = nd[0]; dir[1] = nd[1]; dir[2] = nd[2];
    }
}

/* ------------------------------------------------------------- render -- */
typedef struct {
    const oscene* s;
    const pt_render_params* p;
    const int64_t* pixels;
    int64_t n_pixels;
    double* out;
    int64_t next;
    pthread_mutex_t mu;
    ocount total;
} job_t;

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    ocount c;
    memset(&c, 0, sizeof(c));
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int64_t i0 = j->next;
        j->next += 16;
        pthread_mutex_unlock(&j->mu);
        if (i0 >= j->n_pixels) break;
        int64_t i1 = i0 + 16 < j->n_pixels ? i0 + 16 : j->n_pixels;
        for (int64_t i = i0; i < i1; ++i) {
            double acc[3] = {0, 0, 0};
            for (int sidx = 0; sidx < j->p->spp; ++sidx) {
                double rgb[3];
                path_sample(j->s, j->p, j->pixels[i], j->p->sample_begin + sidx, rgb, &c);
                for (int q = 0; q < 3; ++q) acc[q] += rgb[q];
            }
            for (int q = 0; q < 3; ++q) j->out[3 * i + q] = acc[q] / (double)j->p->spp;
        }
    }
    pthread_mutex_lock(&j->mu);
    j->total.closest_tests += c.closest_tests;
    j->total.shadow_tests += c.shadow_tests;
    j->total.ray_bounces += c.ray_bounces;
    j->total.shading_points += c.shading_points;
    j->total.light_hits += c.light_hits;
    j->total.escapes += c.escapes;
    pthread_mutex_unlock(&j->mu);
    return NULL;
}

/* Render the listed pixels (reference list index k = ix*H + iy); out[i][3] is
 * the averaged colour of pixels[i] (main.py:274-280), before make_image. */
int oracle_render(const pt_scene_desc* d, const pt_render_params* p,
                  const int64_t* pixels, int64_t n_pixels, int n_threads,
                  double* out, pt_stats* stats) {
    if (!d || !p || !out || p->width <= 0 || p->height <= 0 || p->spp <= 0) return -1;
    oscene s;
    if (oscene_init(&s, d)) return -1;
    job_t j;
    memset(&j, 0, sizeof(j));
    j.s = &s; j.p = p; j.pixels = pixels; j.n_pixels = n_pixels; j.out = out;
    pthread_mutex_init(&j.mu, NULL);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 512) n_threads = 512;
    pthread_t th[512];
    for (int i = 0; i < n_threads; ++i) pthread_create(&th[i], NULL, worker, &j);
    for (int i = 0; i < n_threads; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&j.mu);
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->closest_tests = j.total.closest_tests;
        stats->shadow_tests = j.total.shadow_tests;
        stats->ray_bounces = j.total.ray_bounces;
        stats->shading_points = j.total.shading_points;
        stats->light_hits = j.total.light_hits;
        stats->escapes = j.total.escapes;
    }
    oscene_free(&s);
    return 0;
}
