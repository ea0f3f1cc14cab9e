/*
 * rtw_oracle.c — TEST INFRASTRUCTURE ONLY: plain-C restatement of the
 * reference's per-pixel render path, used as the parity checker and as the
 * "port" CPU baseline.  Never linked into the product library.
 *
 * Every function cites the reference file:line it restates.  fp64 throughout;
 * operation order follows the reference's C++ expressions (the vec3 broadcast
 * constructor makes `double * vec3` a component-wise product; g++ evaluates
 * constructor arguments right to left, which fixes the order of the random
 * draws inside vec3(random_double(), ...) expressions — spelled out below).
 */
#include "rtw_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* libm calls of the path.  The default build calls glibc's, as the
 * reference does.  RTW_ORACLE_DEVLIBM (librtw_oracle_devlibm.so, the checker
 * of the strict-radiance GPU build) calls the device's own functions instead
 * (oracle/devlibm.cpp over raytracingweekend_amd/csrc/rtw_math.h), so that
 * every other operation can be compared with the GPU to the last bit; the
 * device functions' distance to glibc's is tested on its own
 * (tests/test_sincos.py). */
#ifdef RTW_ORACLE_DEVLIBM
double rtw_devlibm_cos(double x);
double rtw_devlibm_sin(double x);
double rtw_devlibm_sin_tex(double x);
double rtw_devlibm_log(double x);
double rtw_devlibm_pow5(double x);
#define O_COS(x) rtw_devlibm_cos(x)
#define O_SIN(x) rtw_devlibm_sin(x)
#define O_SIN_TEX(x) rtw_devlibm_sin_tex(x)
#define O_LOG(x) rtw_devlibm_log(x)
#define O_POW5(x) rtw_devlibm_pow5(x)
#else
#define O_COS(x) cos(x)
#define O_SIN(x) sin(x)
#define O_SIN_TEX(x) sin(x)
#define O_LOG(x) log(x)
#define O_POW5(x) pow((x), 5)
#endif

/* ------------------------------------------------------------------ */
/* vec3 (vec3.h:9-91)                                                  */
/* ------------------------------------------------------------------ */
typedef struct { double x, y, z; } v3;

static inline v3 mk(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 divs(v3 a, double s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline double len2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline double len(v3 a) { return sqrt(len2(a)); }
static inline v3 cross(v3 a, v3 b) {                     /* vec3.h:54-59 */
    return mk(a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x);
}
static inline v3 normalize(v3 v) { return divs(v, len(v)); } /* vec3.h:61-67 */
static inline v3 lda(const double* p) { return mk(p[0], p[1], p[2]); }

typedef struct { v3 o, d; double t; } ray;

static inline v3 at(const ray* r, double t) { return add(r->o, muls(r->d, t)); } /* ray.h:103 */

/* ------------------------------------------------------------------ */
/* RNG: per-path std::minstd_rand + libstdc++ generate_canonical        */
/* ------------------------------------------------------------------ */
typedef struct { uint64_t s; } rng;

static inline uint32_t draw(rng* g) { /* linear_congruential_engine<uint_fast32_t,48271,0,2147483647> */
    g->s = (g->s * 48271u) % 2147483647u;
    return (uint32_t)g->s;
}

/* generate_canonical<double,53>(minstd_rand): k = 2 raw draws,
 * sum = (e1-1) + (e2-1)*R, divided by R*R (R = max-min+1, products of the
 * running factor taken in long double as libstdc++ does). */
static double canon(rng* g) {
    const long double R = 2147483646.0L;
    double sum = 0.0, tmp = 1.0;
    sum += (double)(draw(g) - 1u) * tmp;
    tmp = (double)((long double)tmp * R);
    sum += (double)(draw(g) - 1u) * tmp;
    tmp = (double)((long double)tmp * R);
    double ret = sum / tmp;
    if (ret >= 1.0) ret = nextafter(1.0, 0.0);
    return ret;
}

/* utility.h:14-20 (uniform_real_distribution(0,1) -> U*(1-0)+0 = U) */
static inline double rnd01(rng* g) { return canon(g) * (1.0 - 0.0) + 0.0; }
static inline double random_double(rng* g, double a, double b) { return a + (b - a) * rnd01(g); }

static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint32_t rtw_oracle_path_seed(uint64_t seed, uint32_t pixel, uint32_t s) {
    uint64_t k = ((uint64_t)s << 32) ^ (uint64_t)pixel;
    return (uint32_t)(1u + splitmix64(splitmix64(seed) ^ k) % 2147483646ull);
}

double rtw_oracle_canonical(uint32_t* state) {
    rng g = {*state};
    double u = canon(&g);
    *state = (uint32_t)g.s;
    return u;
}

/* utility.h:22-25 */
static int random_int(rng* g, int a, int b) {
    int span = (int)((b - a + 1) * random_double(g, 0.0, 1.0));
    return a + ((b - a) < span ? (b - a) : span);
}

/* utility.h:27-35: vec3(random_double() x3) evaluates z, y, x */
static v3 random_in_unit_sphere(rng* g) {
    v3 p;
    do {
        double z = random_double(g, 0.0, 1.0);
        double y = random_double(g, 0.0, 1.0);
        double x = random_double(g, 0.0, 1.0);
        p = sub(muls(mk(x, y, z), 2.0), mk(1, 1, 1));
    } while (dot(p, p) >= 1.0);
    return p;
}

/* utility.h:54-67 */
static v3 random_cosine_direction(rng* g) {
    double r1 = random_double(g, 0.0, 1.0);
    double r2 = random_double(g, 0.0, 1.0);
    double z = sqrt(1 - r2);
    double phi = 2 * M_PI * r1;
    double x = O_COS(phi) * sqrt(r2);
    double y = O_SIN(phi) * sqrt(r2);
    return mk(x, y, z);
}

/* utility.h:69-81 */
static v3 random_to_sphere(rng* g, double radius, double distance_squared) {
    double r1 = random_double(g, 0.0, 1.0);
    double r2 = random_double(g, 0.0, 1.0);
    double z = 1 + r2 * (sqrt(1 - radius * radius / distance_squared) - 1);
    double phi = 2 * M_PI * r1;
    double x = O_COS(phi) * sqrt(1 - z * z);
    double y = O_SIN(phi) * sqrt(1 - z * z);
    return mk(x, y, z);
}

/* ------------------------------------------------------------------ */
/* onb (onb.h:5-38)                                                    */
/* ------------------------------------------------------------------ */
typedef struct { v3 u, v, w; } onb;

static onb onb_from_w(v3 n) {
    onb b;
    b.w = normalize(n);
    v3 a = (fabs(b.w.x) > 0.9) ? mk(0, 1, 0) : mk(1, 0, 0);
    b.v = normalize(cross(b.w, a));
    b.u = cross(b.w, b.v);
    return b;
}
static v3 onb_local(const onb* b, v3 a) {
    return add(add(muls(b->u, a.x), muls(b->v, a.y)), muls(b->w, a.z));
}

/* ------------------------------------------------------------------ */
/* scene access                                                        */
/* ------------------------------------------------------------------ */
typedef struct {
    double t;
    v3 p, normal;
    int mat;
} hit_rec;

/* sphere.h:22-25: center0 + ((time - time0) / (time1 - time0)) * (center1 - center0) */
static v3 sphere_center(const rtw_prim* s, double time) {
    v3 c0 = lda(s->p);
    if (s->type != RTW_PRIM_MOVING_SPHERE) return c0;
    v3 c1 = lda(s->p + 4);
    double f = (time - s->p[7]) / (s->p[8] - s->p[7]);
    return add(c0, muls(sub(c1, c0), f));
}

/* sphere.h:46-81 */
static int sphere_hit(const rtw_prim* s, const ray* r, double t_min, double t_max, hit_rec* rec) {
    v3 cc = sphere_center(s, r->t);
    double radius = s->p[3];
    v3 oc = sub(r->o, cc);
    double a = dot(r->d, r->d);
    double b = dot(oc, r->d);
    double c = dot(oc, oc) - radius * radius;
    double disc = b * b - a * c;
    if (disc > 0) {
        double temp = (-b - sqrt(disc)) / a;
        if (temp < t_max && temp > t_min) {
            rec->t = temp;
            rec->p = at(r, temp);
            rec->normal = divs(sub(rec->p, cc), radius);
            rec->mat = s->material;
            return 1;
        }
        temp = (-b + sqrt(disc)) / a;
        if (temp < t_max && temp > t_min) {
            rec->t = temp;
            rec->p = at(r, temp);
            rec->normal = divs(sub(rec->p, cc), radius);
            rec->mat = s->material;
            return 1;
        }
    }
    return 0;
}

/* hittable.h:149-165 (xy), :184-200 (xz), :241-257 (yz) */
static int rect_hit(const rtw_prim* q, const ray* r, double t0, double t1, hit_rec* rec) {
    const double* P = q->p;
    double ok, od, a_o, a_d, b_o, b_d;
    v3 n;
    switch (q->type) {
    case RTW_PRIM_RECT_XY: ok = r->o.z, od = r->d.z, a_o = r->o.x, a_d = r->d.x, b_o = r->o.y, b_d = r->d.y, n = mk(0, 0, 1); break;
    case RTW_PRIM_RECT_XZ: ok = r->o.y, od = r->d.y, a_o = r->o.x, a_d = r->d.x, b_o = r->o.z, b_d = r->d.z, n = mk(0, 1, 0); break;
    default: ok = r->o.x, od = r->d.x, a_o = r->o.y, a_d = r->d.y, b_o = r->o.z, b_d = r->d.z, n = mk(1, 0, 0); break;
    }
    double t = (P[4] - ok) / od;
    if (t < t0 || t > t1) return 0;
    double a = a_o + t * a_d;
    double b = b_o + t * b_d;
    if (a < P[0] || a > P[1] || b < P[2] || b > P[3]) return 0;
    rec->t = t;
    rec->mat = q->material;
    rec->p = at(r, t);
    rec->normal = n;
    return 1;
}

static int prim_hit(const rtw_prim* q, const ray* r, double t0, double t1, hit_rec* rec) {
    int h = (q->type == RTW_PRIM_SPHERE || q->type == RTW_PRIM_MOVING_SPHERE) ? sphere_hit(q, r, t0, t1, rec)
                                                                              : rect_hit(q, r, t0, t1, rec);
    if (h && (q->flip & 1)) rec->normal = neg(rec->normal); /* flip_normals, hittable.h:273-284 */
    return h;
}

/* translate::hit hittable.h:299-311, rotate_y::hit :373-404, flip :273-284 */
static void op_ray_in(const rtw_entry* e, int k, ray* r) {
    const double* q = e->op_param[k];
    if (e->op[k] == RTW_OP_TRANSLATE) {
        r->o = sub(r->o, lda(q));
    } else if (e->op[k] == RTW_OP_ROTATE_Y) {
        double s = q[0], c = q[1];
        v3 o = r->o, d = r->d;
        o.x = c * r->o.x - s * r->o.z;
        o.z = s * r->o.x + c * r->o.z;
        d.x = c * r->d.x - s * r->d.z;
        d.z = s * r->d.x + c * r->d.z;
        r->o = o;
        r->d = d;
    }
}
static void op_rec_out(const rtw_entry* e, int k, hit_rec* rec) {
    const double* q = e->op_param[k];
    if (e->op[k] == RTW_OP_TRANSLATE) {
        rec->p = add(rec->p, lda(q));
    } else if (e->op[k] == RTW_OP_ROTATE_Y) {
        double s = q[0], c = q[1];
        v3 p = rec->p, n = rec->normal;
        p.x = c * rec->p.x + s * rec->p.z;
        p.z = -s * rec->p.x + c * rec->p.z;
        n.x = c * rec->normal.x + s * rec->normal.z;
        n.z = -s * rec->normal.x + c * rec->normal.z;
        rec->p = p;
        rec->normal = n;
    } else if (e->op[k] == RTW_OP_FLIP) {
        rec->normal = neg(rec->normal);
    }
}

/* Closest hit over an entry's group (ops, then its primitives in list order).
 * The reference walks nested lists twice (hittable_list.h:16-34); for these
 * deterministic primitives the second walk re-accepts only what the first
 * kept, so one walk gives the same record. */
static int group_hit_ops(const rtw_scene_desc* S, const rtw_entry* e, int k0, const ray* r0, double t_min,
                         double t_max, hit_rec* rec) {
    ray r = *r0;
    for (int k = k0; k < e->n_ops; k++) op_ray_in(e, k, &r);
    hit_rec tmp;
    int any = 0;
    double closest = t_max;
    for (int i = 0; i < e->n_prims; i++) {
        if (prim_hit(&S->prims[e->first_prim + i], &r, t_min, closest, &tmp)) {
            any = 1;
            closest = tmp.t;
            *rec = tmp;
        }
    }
    if (!any) return 0;
    for (int k = e->n_ops - 1; k >= k0; k--) op_rec_out(e, k, rec);
    return 1;
}
static int group_hit(const rtw_scene_desc* S, const rtw_entry* e, const ray* r0, double t_min, double t_max,
                     hit_rec* rec) {
    return group_hit_ops(S, e, 0, r0, t_min, t_max, rec);
}

/* constant_medium::hit hittable.h:430-479 (one call = at most one draw), in
 * the frame of the transforms enclosing it (ops [0, n_outer_ops): translate /
 * rotate_y hand it their moved ray and move its record back out); its
 * boundary is the rest of the chain over the group. */
static int medium_hit(const rtw_scene_desc* S, const rtw_entry* e, const ray* rw, double t_min, double t_max,
                      hit_rec* rec, rng* g) {
    hit_rec rec1, rec2;
    ray rm = *rw;
    for (int k = 0; k < e->n_outer_ops; k++) op_ray_in(e, k, &rm);
    const ray* r = &rm;
    if (group_hit_ops(S, e, e->n_outer_ops, r, -DBL_MAX, DBL_MAX, &rec1)) {
        if (group_hit_ops(S, e, e->n_outer_ops, r, rec1.t + 0.0001f, DBL_MAX, &rec2)) {
            if (rec1.t < t_min) rec1.t = t_min;
            if (rec2.t > t_max) rec2.t = t_max;
            if (rec1.t >= rec2.t) return 0;
            if (rec1.t < 0) rec1.t = 0;
            double distance_inside_boundary = (rec2.t - rec1.t) * len(r->d);
            double hit_distance = -(1 / e->density) * O_LOG(rnd01(g));
            if (hit_distance < distance_inside_boundary) {
                rec->t = rec1.t + hit_distance / len(r->d);
                rec->p = at(r, rec->t);
                rec->normal = mk(1, 0, 0);
                rec->mat = e->phase_material;
                for (int k = e->n_outer_ops - 1; k >= 0; k--) op_rec_out(e, k, rec);
                return 1;
            }
        }
    }
    return 0;
}

static int entry_hit(const rtw_scene_desc* S, const rtw_entry* e, const ray* r, double t0, double t1, hit_rec* rec,
                     rng* g) {
    if (e->kind == RTW_ENTRY_MEDIUM) return medium_hit(S, e, r, t0, t1, rec, g);
    return group_hit(S, e, r, t0, t1, rec);
}

/* hittable_list::hit hittable_list.h:11-37 — the world list, walked twice;
 * with a visit program (nested lists holding media), the entries in the
 * order the reference's nested walks call them, replays included */
static int world_hit(const rtw_scene_desc* S, const ray* r, double t_min, double t_max, hit_rec* rec, rng* g) {
    hit_rec tmp;
    int any = 0;
    double closest = t_max;
    if (S->n_visits > 0) {
        for (int k = 0; k < S->n_visits; k++) {
            const rtw_entry* e = &S->entries[S->visits[k] & RTW_VISIT_ENTRY];
            if (entry_hit(S, e, r, t_min, closest, &tmp, g)) {
                any = 1;
                closest = tmp.t;
                *rec = tmp;
            }
        }
        return any;
    }
    for (int pass = 0; pass < 2; pass++) {
        for (int i = 0; i < S->n_entries; i++) {
            if (entry_hit(S, &S->entries[i], r, t_min, closest, &tmp, g)) {
                any = 1;
                closest = tmp.t;
                *rec = tmp;
            }
        }
    }
    return any;
}

/* ------------------------------------------------------------------ */
/* textures (texture.h:16-71, noise.h:9-151)                           */
/* ------------------------------------------------------------------ */
static double smooth(double x) { return x * x * (3 - 2 * x); } /* noise.h:9-12 */

double rtw_oracle_noise(const rtw_scene_desc* S, const double pp[3]) { /* noise.h:89-151 PERLIN */
    v3 p = lda(pp);
    double u = p.x - floor(p.x);
    double v = p.y - floor(p.y);
    double w = p.z - floor(p.z);
    int i = (int)floor(p.x);
    int j = (int)floor(p.y);
    int k = (int)floor(p.z);
    const int* px = S->perlin_perm;
    const int* py = S->perlin_perm + 256;
    const int* pz = S->perlin_perm + 512;
    v3 c[2][2][2];
    for (int di = 0; di < 2; di++)
        for (int dj = 0; dj < 2; dj++)
            for (int dk = 0; dk < 2; dk++)
                c[di][dj][dk] = lda(S->perlin_ranvec + 3 * (px[(i + di) & 255] ^ py[(j + dj) & 255] ^ pz[(k + dk) & 255]));
    /* perlin_interp noise.h:40-60 */
    double uu = smooth(u), vv = smooth(v), ww = smooth(w);
    double accum = 0;
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
            for (int d = 0; d < 2; d++) {
                v3 weight_v = mk(u - a, v - b, w - d);
                accum += (a * uu + (1 - a) * (1 - uu)) * (b * vv + (1 - b) * (1 - vv)) *
                         (d * ww + (1 - d) * (1 - ww)) * dot(c[a][b][d], weight_v);
            }
    return accum;
}

double rtw_oracle_turb(const rtw_scene_desc* S, const double pp[3]) { /* noise.h:74-86 */
    double accum = 0;
    double temp_p[3] = {pp[0], pp[1], pp[2]};
    double weight = 1.0;
    for (int i = 0; i < 7; i++) {
        accum += weight * rtw_oracle_noise(S, temp_p);
        weight *= 0.5f;
        temp_p[0] *= 2, temp_p[1] *= 2, temp_p[2] *= 2;
    }
    return fabs(accum);
}

static v3 texture_value(const rtw_scene_desc* S, int id, v3 p) {
    const rtw_texture* t = &S->textures[id];
    switch (t->type) {
    case RTW_TEX_CONSTANT: return lda(t->color);
    case RTW_TEX_CHECKER: { /* texture.h:38-49 */
        double sines = O_SIN_TEX(10.0 * p.x) * O_SIN_TEX(10.0 * p.y) * O_SIN_TEX(10.0 * p.z);
        return texture_value(S, sines < 0 ? t->odd : t->even, p);
    }
    default: { /* texture.h:57-68: vec3(1,1,1) * 0.5f * (1 + sin(scale*p.z + 10*turb(p))) */
        double pp[3] = {p.x, p.y, p.z};
        double s = 1 + O_SIN_TEX(t->scale * p.z + 10 * rtw_oracle_turb(S, pp));
        double v = (1.0 * (double)0.5f) * s;
        return mk(v, v, v);
    }
    }
}

/* ------------------------------------------------------------------ */
/* lights: hittable_pdf over scene::lights (pdf.h:35-53)               */
/* ------------------------------------------------------------------ */
static double light_pdf_value(const rtw_scene_desc* S, const rtw_light* L, v3 o, v3 v) {
    hit_rec rec;
    if (L->kind == RTW_LIGHT_XZ_RECT) { /* hittable.h:208-222 */
        const rtw_prim* q = &S->prims[L->prim];
        ray r = {o, v, (double)FLT_MAX};
        if (!rect_hit(q, &r, 0.001, INFINITY, &rec)) return 0;
        double area = (q->p[1] - q->p[0]) * (q->p[3] - q->p[2]);
        double distance_squared = rec.t * rec.t * len2(v);
        double cosine = fabs(dot(v, rec.normal) / len(v));
        return distance_squared / (cosine * area);
    }
    if (L->kind == RTW_LIGHT_SPHERE) { /* sphere.h:88-99 */
        const rtw_prim* q = &S->prims[L->prim];
        ray r = {o, v, (double)FLT_MAX};
        if (!sphere_hit(q, &r, 0.001, INFINITY, &rec)) return 0.0;
        double radius = q->p[3];
        double cos_theta_max = sqrt(1 - radius * radius / len2(sub(lda(q->p), o)));
        double solid_angle = 2.0 * M_PI * (1.0 - cos_theta_max);
        return 1.0 / solid_angle;
    }
    return 0.0; /* hittable.h:36 */
}

static v3 light_random(const rtw_scene_desc* S, const rtw_light* L, v3 o, rng* g) {
    if (L->kind == RTW_LIGHT_XZ_RECT) { /* hittable.h:224-228: vec3(rd(x0,x1), k, rd(z0,z1)), z drawn first */
        const rtw_prim* q = &S->prims[L->prim];
        double rz = random_double(g, q->p[2], q->p[3]);
        double rx = random_double(g, q->p[0], q->p[1]);
        return sub(mk(rx, q->p[4], rz), o);
    }
    if (L->kind == RTW_LIGHT_SPHERE) { /* sphere.h:101-108 */
        const rtw_prim* q = &S->prims[L->prim];
        v3 direction = sub(lda(q->p), o);
        double distance_squared = len2(direction);
        onb uvw = onb_from_w(direction);
        return onb_local(&uvw, random_to_sphere(g, q->p[3], distance_squared));
    }
    return mk(1, 0, 0); /* hittable.h:37 */
}

/* hittable_list::pdf_value / random, hittable_list.h:44-59 */
static double lights_pdf_value(const rtw_scene_desc* S, v3 o, v3 v) {
    double weight = 1.0 / (double)S->n_lights;
    double sum = 0.0;
    for (int i = 0; i < S->n_lights; i++) sum += weight * light_pdf_value(S, &S->lights[i], o, v);
    return sum;
}
static v3 lights_random(const rtw_scene_desc* S, v3 o, rng* g) {
    return light_random(S, &S->lights[random_int(g, 0, S->n_lights - 1)], o, g);
}

/* ------------------------------------------------------------------ */
/* integrator color() RayTracingWeekend.cpp:45-160                     */
/* ------------------------------------------------------------------ */
typedef struct {
    double* rows; /* optional trace rows */
    int max_rows;
    int n;
    uint64_t segments;
} trace_ctx;

/* material.h:10-13 */
static v3 reflect(v3 v, v3 n) { return sub(v, muls(n, 2.0 * dot(v, n))); }

/* material.h:17-39 */
static int refract(v3 v, v3 n, double ni_over_nt, v3* refracted) {
    v3 uv = normalize(v);
    double dt = dot(uv, n);
    double discriminant = 1.0 - ni_over_nt * ni_over_nt * (1 - dt * dt);
    if (discriminant > 0) {
        *refracted = sub(muls(sub(uv, muls(n, dt)), ni_over_nt), muls(n, sqrt(discriminant)));
        return 1;
    }
    return 0;
}

/* material.h:44-49 */
static double schlick(double cosine, double ref_idx) {
    double r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 = r0 * r0;
    return r0 + (1 - r0) * O_POW5(1 - cosine);
}

static v3 color(const rtw_scene_desc* S, const ray* r, int depth, rng* g, trace_ctx* tc) {
    if (depth <= 0) return mk(0, 0, 0);
    hit_rec rec;
    tc->segments++;
    int hit = world_hit(S, r, 0.001f, DBL_MAX, &rec, g);
    if (tc->rows && tc->n < tc->max_rows) {
        double* row = tc->rows + 8 * tc->n++;
        row[0] = r->o.x, row[1] = r->o.y, row[2] = r->o.z;
        row[3] = r->d.x, row[4] = r->d.y, row[5] = r->d.z;
        row[6] = hit ? rec.t : -1.0;
        row[7] = r->t;
    }
    if (hit) {
        if (S->render_type == RTW_RENDER_NORMAL) /* :135-136 */
            return mul(mk(0.5f, 0.5f, 0.5f), add(rec.normal, mk(1, 1, 1)));
        const rtw_material* m = &S->materials[rec.mat];
        v3 emitted = mk(0, 0, 0); /* material.h:69-72 */
        if (m->type == RTW_MAT_DIFFUSE_LIGHT) { /* material.h:238-244 */
            if (dot(rec.normal, r->d) > 0) emitted = texture_value(S, m->texture, rec.p);
            return emitted; /* scatter() is false, :62-63 */
        }
        if (m->type == RTW_MAT_METAL) { /* material.h:128-136, then :114-115 */
            v3 reflected = reflect(normalize(r->d), rec.normal);
            ray sc = {rec.p, add(reflected, muls(random_in_unit_sphere(g), m->fuzz)), r->t};
            return mul(lda(m->albedo), color(S, &sc, depth - 1, g, tc));
        }
        if (m->type == RTW_MAT_DIELECTRIC) { /* material.h:146-222 */
            v3 outward_normal;
            double ni_over_nt, cosine;
            double ref_idx = m->ref_idx;
            if (dot(r->d, rec.normal) > 0) {
                outward_normal = neg(rec.normal);
                ni_over_nt = ref_idx;
                cosine = dot(r->d, rec.normal) / len(r->d);
                cosine = sqrt(1 - ref_idx * ref_idx * (1 - cosine * cosine));
            } else {
                outward_normal = rec.normal;
                ni_over_nt = 1.0 / ref_idx;
                cosine = -dot(r->d, rec.normal) / len(r->d);
            }
            v3 reflected = reflect(r->d, rec.normal);
            v3 refracted = mk(0, 0, 0);
            double reflect_prob;
            if (refract(r->d, outward_normal, ni_over_nt, &refracted))
                reflect_prob = schlick(cosine, ref_idx);
            else
                reflect_prob = 1.0;
            double u = rnd01(g);
            ray sc = {rec.p, (u < reflect_prob) ? reflected : refracted, r->t};
            return mul(mk(1.0, 1.0, 1.0), color(S, &sc, depth - 1, g, tc));
        }
        if (m->type == RTW_MAT_ISOTROPIC) { /* material.h:257-262 */
            ray sc = {rec.p, random_in_unit_sphere(g), r->t};
            v3 att = texture_value(S, m->texture, rec.p);
            return mul(att, color(S, &sc, depth - 1, g, tc));
        }
        /* lambertian material.h:81-119 with the pdf logic of :112-132 */
        v3 att = texture_value(S, m->texture, rec.p);
        onb uvw = onb_from_w(rec.normal); /* cosine_pdf(rec.normal), pdf.h:262 */
        v3 dir;
        double pdf_val;
        if (S->n_lights > 0) { /* mixture_pdf(material_pdf, hittable_pdf(lights, p)), pdf.h:55-79 */
            if (random_double(g, 0.0, 1.0) < 0.5)
                dir = onb_local(&uvw, random_cosine_direction(g));
            else
                dir = lights_random(S, rec.p, g);
            double c = dot(normalize(dir), uvw.w);
            double p0 = (c <= 0) ? 0 : c / M_PI;
            pdf_val = 0.5 * p0 + 0.5 * lights_pdf_value(S, rec.p, dir);
        } else {
            dir = onb_local(&uvw, random_cosine_direction(g));
            double c = dot(normalize(dir), uvw.w);
            pdf_val = (c <= 0) ? 0 : c / M_PI;
        }
        ray scattered = {rec.p, dir, r->t};
        if (pdf_val <= 0.0) return emitted;
        double cosine = dot(rec.normal, normalize(scattered.d)); /* material.h:115-119 */
        double spdf = cosine < 0 ? 0 : cosine / M_PI;
        v3 Li = color(S, &scattered, depth - 1, g, tc);
        return add(emitted, divs(mul(muls(att, spdf), Li), pdf_val));
    }
    if (S->background == RTW_BG_GRADIENT) { /* :145-151 */
        v3 unit_direction = normalize(r->d);
        double t = 0.5f * (unit_direction.y + 1.0);
        /* lerp(from, to, t) = (1.0 - t) * to + t * from, vec3.h:84-87 */
        return add(muls(mk(1.0, 1.0, 1.0), 1.0 - t), muls(mk(0.5f, 0.7f, 1.0), t));
    }
    return mk(0, 0, 0);
}

/* camera::get_ray camera.h:36-50 with random_in_unit_disk :61-69
 * (vec3(U, U, 0): y drawn first). */
static ray get_ray(const rtw_camera_desc* c, double s, double t, rng* g) {
    v3 p;
    do {
        double y = rnd01(g);
        double x = rnd01(g);
        p = sub(muls(mk(x, y, 0), 2.0), mk(1, 1, 0));
    } while (dot(p, p) >= 1.0);
    v3 rd = muls(p, c->lens_radius);
    v3 offset = add(muls(lda(c->u), rd.x), muls(lda(c->v), rd.y));
    double time = c->time0 + rnd01(g) * (c->time1 - c->time0);
    v3 dir = sub(sub(add(add(lda(c->lower_left), muls(lda(c->horizontal), s)), muls(lda(c->vertical), t)),
                     lda(c->origin)),
                 offset);
    ray r = {add(lda(c->origin), offset), normalize(dir), time};
    return r;
}

/* render-loop body RayTracingWeekend.cpp:227-232 for one (i, j, s) */
static v3 sample(const rtw_scene_desc* S, const rtw_camera_desc* cam, int nx, int ny, int i, int j, int s,
                 int max_depth, uint64_t seed, trace_ctx* tc) {
    rng g = {rtw_oracle_path_seed(seed, (uint32_t)(j * nx + i), (uint32_t)s)};
    double u = (double)(i + rnd01(&g)) / (double)nx;
    double v = (double)(j + rnd01(&g)) / (double)ny;
    ray r = get_ray(cam, u, v, &g);
    return color(S, &r, max_depth, &g, tc);
}

/* Rows row_begin, row_begin + row_stride, ... (row_count of them), one
 * OpenMP task per row: the bounded CPU sample bench.py times (every
 * stride-th row of the image) in one multithreaded call. */
int rtw_oracle_render_strided(const rtw_scene_desc* S, const rtw_camera_desc* cam, int nx, int ny, int row_begin,
                              int row_stride, int row_count, int spp_begin, int spp_count, int max_depth,
                              uint64_t seed, int threads, double* sums, uint64_t* segments) {
    if (!S || !cam || !sums || nx <= 0 || ny <= 0 || row_stride <= 0 || row_count < 0) return -1;
    if (row_count > 0 && (row_begin < 0 || row_begin + (int64_t)(row_count - 1) * row_stride >= ny)) return -1;
    if (S->has_perlin && (!S->perlin_ranvec || !S->perlin_perm)) return -1;
    uint64_t seg_total = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : seg_total)
    for (int k = 0; k < row_count; k++) {
        const int j = row_begin + k * row_stride;
        trace_ctx tc = {0, 0, 0, 0};
        for (int i = 0; i < nx; i++) {
            v3 sum = mk(0, 0, 0);
            for (int s = spp_begin; s < spp_begin + spp_count; s++)
                sum = add(sum, sample(S, cam, nx, ny, i, j, s, max_depth, seed, &tc));
            double* o = sums + ((size_t)j * nx + i) * 3;
            o[0] = sum.x, o[1] = sum.y, o[2] = sum.z;
        }
        seg_total += tc.segments;
    }
    if (segments) *segments = seg_total;
    return 0;
}

int rtw_oracle_render(const rtw_scene_desc* S, const rtw_camera_desc* cam, int nx, int ny, int row_begin,
                      int row_count, int spp_begin, int spp_count, int max_depth, uint64_t seed, int threads,
                      double* sums, uint64_t* segments) {
    return rtw_oracle_render_strided(S, cam, nx, ny, row_begin, 1, row_count, spp_begin, spp_count, max_depth,
                                     seed, threads, sums, segments);
}

int rtw_oracle_trace(const rtw_scene_desc* S, const rtw_camera_desc* cam, int nx, int ny, int i, int j, int s,
                     int max_depth, uint64_t seed, double* radiance3, double* seg_rows, int max_seg) {
    trace_ctx tc = {seg_rows, max_seg, 0, 0};
    v3 L = sample(S, cam, nx, ny, i, j, s, max_depth, seed, &tc);
    radiance3[0] = L.x, radiance3[1] = L.y, radiance3[2] = L.z;
    return tc.n;
}
