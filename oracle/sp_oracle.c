/*
 * sp_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of kjeffery/SimplePath's per-pixel
 * integration path, used as the checker for the HIP implementation.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product never does.
 *
 * It follows the reference literally: recursive BVH traversal (shapes/BVHAccelerator.h:45-90)
 * over a BVH built by the reference's own midpoint/std::partition construction
 * (shapes/BVHAccelerator.h:173), the reference's x86 arithmetic (RSQRTSS + Newton normalize,
 * DPPS dot, FMA-based cross), and glibc's float libm (or, when built with ORC_LIBM_SPM, the
 * product's device libm so the GPU can be checked bit for bit while that libm is not yet an
 * exact glibc emulation -- see DESIGN.md "Parity chain").
 *
 * Pinning: built as liboracle_glibc.so it is compared bit for bit with the real reference
 * compiled from /root/reference sources (oracle/_ref, tests/test_oracle_vs_ref.py) on the
 * same scenes.  Each function names the reference file:line it restates.
 */
#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/simplepath_hip.h"

/* ------------------------------------------------------------------ libm selection */
float orc_sinf(float);
float orc_cosf(float);
float orc_expf(float);
float orc_logf(float);
float orc_powf(float, float);
float orc_erff(float);
float orc_acosf(float);
float orc_atan2f(float, float);

/* ------------------------------------------------------------------ math (math/*.h) */
typedef struct { float x, y, z; } V3;
typedef struct { float r, g, b; } C3;
typedef struct { V3 vx, vy, vz, p; } Aff;
typedef struct { V3 vx, vy, vz; } Lin;

static const float PI_F = 3.14159265358979323846f;
static const float RAY_EPS = 0.001f;                /* math/Ray.h:163 */
static const float INF_DIST = 3.40282346638528859812e+38f; /* base/Constants.h:257 */

static inline V3 v3(float x, float y, float z) { V3 r = { x, y, z }; return r; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 vmulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 vmulf(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline V3 fmulv(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
static inline V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline V3 vdivf(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
/* madd(Vector3, Vector3, Vector3) = _mm_fmadd_ps (math/Vector3.h:402) */
static inline V3 vmadd(V3 a, V3 b, V3 c) { return v3(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z)); }
static inline V3 splat(float s) { return v3(s, s, s); }
/* dot: _mm_dp_ps(a, b, 0x7F) (math/Vector3.h:743) */
static inline float vdot(V3 a, V3 b)
{
    float t0 = a.x * b.x, t1 = a.y * b.y, t2 = a.z * b.z, t3 = 0.0f;
    return (t0 + t1) + (t2 + t3);
}
/* sp::rsqrt (math/Math.h:205) */
static inline float rsqrt_ref(float x)
{
    __m128 a = _mm_set_ss(x);
    __m128 r = _mm_rsqrt_ss(a);
    __m128 c = _mm_add_ss(_mm_mul_ss(_mm_set_ss(1.5f), r),
                          _mm_mul_ss(_mm_mul_ss(_mm_mul_ss(a, _mm_set_ss(-0.5f)), r), _mm_mul_ss(r, r)));
    return _mm_cvtss_f32(c);
}
static inline V3 vnormalize(V3 a) { return vmulf(a, rsqrt_ref(vdot(a, a))); } /* math/Vector3.h:797 */
static inline float vlength(V3 a) { return sqrtf(vdot(a, a)); }
static inline float fmaxstd(float a, float b) { return (a < b) ? b : a; } /* std::max */
static inline float fminstd(float a, float b) { return (b < a) ? b : a; } /* std::min */
static inline float fclampstd(float v, float lo, float hi) { return (v < lo) ? lo : ((hi < v) ? hi : v); }

static inline C3 c3(float r, float g, float b) { C3 c = { r, g, b }; return c; }
static inline C3 cadd(C3 a, C3 b) { return c3(a.r + b.r, a.g + b.g, a.b + b.b); }
static inline C3 csub(C3 a, C3 b) { return c3(a.r - b.r, a.g - b.g, a.b - b.b); }
static inline C3 cmul(C3 a, C3 b) { return c3(a.r * b.r, a.g * b.g, a.b * b.b); }
static inline C3 cmulf(C3 a, float s) { return c3(a.r * s, a.g * s, a.b * s); }
static inline C3 fmulc(float s, C3 a) { return c3(s * a.r, s * a.g, s * a.b); }
static inline C3 cdivf(C3 a, float s) { return c3(a.r / s, a.g / s, a.b / s); }
static inline int cblack(C3 a) { return a.r == 0.0f && a.g == 0.0f && a.b == 0.0f; }
static inline float lum(C3 c) { return 0.2126f * c.r + 0.7152f * c.g + 0.0722f * c.b; } /* math/RGB.h:224 */

/* AffineSpace::operator()(Point3) (math/AffineSpace.h:79) */
static inline V3 aff_point(const Aff* m, V3 p)
{
    return vmadd(splat(p.x), m->vx, vmadd(splat(p.y), m->vy, vmadd(splat(p.z), m->vz, m->p)));
}
/* LinearSpace3x3::operator()(Vector3) (math/LinearSpace3x3.h:158) */
static inline V3 lin_vec(V3 vx, V3 vy, V3 vz, V3 a)
{
    return vmadd(splat(a.x), vx, vmadd(splat(a.y), vy, vmulv(splat(a.z), vz)));
}

static V3 from3(const float* f) { return v3(f[0], f[1], f[2]); }
static Aff from_aff(const sp_affine* a)
{
    Aff r = { from3(a->vx), from3(a->vy), from3(a->vz), from3(a->p) };
    return r;
}
static Lin from_lin(const sp_linear* a)
{
    Lin r = { from3(a->vx), from3(a->vy), from3(a->vz) };
    return r;
}

/* ------------------------------------------------------------------ samplers */
typedef struct {
    uint64_t mt[312];
    int      p;
} Mt;

static void mt_seed(Mt* s, uint32_t seed) /* std::mt19937_64(seed) */
{
    s->mt[0] = seed;
    for (int i = 1; i < 312; ++i) s->mt[i] = 6364136223846793005ull * (s->mt[i - 1] ^ (s->mt[i - 1] >> 62)) + (uint64_t)i;
    s->p = 312;
}
static uint64_t mt_next(Mt* s)
{
    if (s->p >= 312) {
        const uint64_t um = 0xFFFFFFFF80000000ull, lm = 0x7FFFFFFFull, A = 0xB5026F5AA96619E9ull;
        int k;
        for (k = 0; k < 156; ++k) {
            uint64_t y = (s->mt[k] & um) | (s->mt[k + 1] & lm);
            s->mt[k]   = s->mt[k + 156] ^ (y >> 1) ^ ((y & 1) ? A : 0);
        }
        for (; k < 311; ++k) {
            uint64_t y = (s->mt[k] & um) | (s->mt[k + 1] & lm);
            s->mt[k]   = s->mt[k - 156] ^ (y >> 1) ^ ((y & 1) ? A : 0);
        }
        uint64_t y = (s->mt[311] & um) | (s->mt[0] & lm);
        s->mt[311] = s->mt[155] ^ (y >> 1) ^ ((y & 1) ? A : 0);
        s->p       = 0;
    }
    uint64_t z = s->mt[s->p++];
    z ^= (z >> 29) & 0x5555555555555555ull;
    z ^= (z << 17) & 0x71D67FFFEDA60000ull;
    z ^= (z << 37) & 0xFFF7EEE000000000ull;
    z ^= (z >> 43);
    return z;
}
/* IncoherentSampler::canonical via uniform_real_distribution<float> (math/Sampler.h:125) */
static float canonical(Mt* s)
{
    float r = (float)mt_next(s) / 18446744073709551616.0f;
    if (r >= 1.0f) r = nextafterf(1.0f, 0.0f);
    return r;
}
typedef struct { float x, y; } P2;
static P2 next2(Mt* s)
{
    P2 p;
    p.x = canonical(s);
    p.y = canonical(s);
    return p;
}

static float g_alpha2[2];
static void init_rsequence(void) /* RSequence<2> ctor (math/Sampler.h:47) */
{
    float x = 2.0f;
    for (int i = 0; i < 10; ++i) x = powf(1.0f + x, 1.0f / (2.0f + 1.0f));
    const float g = x;
    float d;
    g_alpha2[0] = modff(powf(1.0f / g, 0u + 1.0f), &d);
    g_alpha2[1] = modff(powf(1.0f / g, 1u + 1.0f), &d);
}

/* ------------------------------------------------------------------ scene model */
typedef struct {
    float lo[3], hi[3];
    int   left, right; /* -1 for leaf */
    int   first, count;
} ONode;

typedef struct {
    int   kind; /* SP_PRIM_* or 10 + light index for light accelerator */
    int   index;
    float lo[3], hi[3];
} OPrim;

typedef struct {
    OPrim* prims; /* leaf order */
    ONode* nodes;
    int    n_nodes, n_prims;
} OBvh;

typedef struct {
    const sp_scene_desc* d;
    Aff                  cam;
    int                  n_unbounded;
    OPrim*               unbounded;
    OBvh                 bvh;
    int                  n_unbounded_lights;
    int*                 unbounded_lights;
    OBvh                 lbvh;
    int                  max_depth, rr_depth;
    struct OEnv*         envs; /* per sp_env_image */
} OScene;

typedef struct {
    const OScene* sc;
    Mt            rng;
    uint64_t      rays, shadow;
} Ctx;

/* BBox extend/merge (math/BBox.h:173,192) with _mm_min_ps/_mm_max_ps operand order */
static inline float ssemin(float a, float b) { return (a < b) ? a : b; }
static inline float ssemax(float a, float b) { return (a > b) ? a : b; }

static void prim_bounds(const sp_scene_desc* d, OPrim* p)
{
    for (int i = 0; i < 3; ++i) { p->lo[i] = INFINITY; p->hi[i] = -INFINITY; }
    if (p->kind == SP_PRIM_TRIANGLE) {
        for (int k = 0; k < 3; ++k) {
            const float* v = d->vertices + 3 * d->indices[3 * p->index + k];
            for (int i = 0; i < 3; ++i) { p->lo[i] = ssemin(v[i], p->lo[i]); p->hi[i] = ssemax(v[i], p->hi[i]); }
        }
        return;
    }
    const sp_affine* o2w = (p->kind == SP_PRIM_SPHERE) ? &d->shapes[p->index].object_to_world : &d->lights[p->index - 0].object_to_world;
    if (p->kind >= 10) o2w = &d->lights[p->kind - 10].object_to_world;
    Aff a = from_aff(o2w);
    const float cs[8][3] = { { -1, -1, -1 }, { -1, -1, 1 }, { -1, 1, -1 }, { -1, 1, 1 },
                             { 1, -1, -1 },  { 1, -1, 1 },  { 1, 1, -1 },  { 1, 1, 1 } };
    for (int c = 0; c < 8; ++c) {
        V3 q = aff_point(&a, v3(cs[c][0], cs[c][1], cs[c][2]));
        float v[3] = { q.x, q.y, q.z };
        for (int i = 0; i < 3; ++i) { p->lo[i] = ssemin(v[i], p->lo[i]); p->hi[i] = ssemax(v[i], p->hi[i]); }
    }
}

/* libstdc++ std::partition (bidirectional) */
static int partition_prims(OPrim* v, int first, int last, int dim, float split)
{
    for (;;) {
        for (;;) {
            if (first == last) return first;
            if ((v[first].lo[dim] + v[first].hi[dim]) / 2.0f < split) ++first;
            else break;
        }
        --last;
        for (;;) {
            if (first == last) return first;
            if (!((v[last].lo[dim] + v[last].hi[dim]) / 2.0f < split)) --last;
            else break;
        }
        OPrim t = v[first]; v[first] = v[last]; v[last] = t;
        ++first;
    }
}

/* BVHAccelerator::construct (shapes/BVHAccelerator.h:173) */
static int build(OBvh* b, int first, int last)
{
    float lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
    for (int i = first; i < last; ++i)
        for (int k = 0; k < 3; ++k) { lo[k] = ssemin(lo[k], b->prims[i].lo[k]); hi[k] = ssemax(hi[k], b->prims[i].hi[k]); }
    const int me = b->n_nodes++;
    ONode*    n  = &b->nodes[me];
    for (int k = 0; k < 3; ++k) { n->lo[k] = lo[k]; n->hi[k] = hi[k]; }
    n->left = n->right = -1;
    n->first = first;
    n->count = last - first;
    if (last - first <= 4) return me;
    const float sx = fabsf(hi[0] - lo[0]), sy = fabsf(hi[1] - lo[1]), sz = fabsf(hi[2] - lo[2]);
    int dim = (sx > sy) ? ((sx > sz) ? 0 : 2) : ((sy > sz) ? 1 : 2);
    const float split = (lo[dim] + hi[dim]) / 2.0f;
    const int   mid   = partition_prims(b->prims, first, last, dim, split);
    if (mid == first || mid == last) return me;
    const int l = build(b, first, mid);
    const int r = build(b, mid, last);
    b->nodes[me].left  = l;
    b->nodes[me].right = r;
    return me;
}

static void build_bvh(OBvh* b, OPrim* prims, int n)
{
    b->prims   = prims;
    b->n_prims = n;
    b->nodes   = (ONode*)calloc((size_t)(2 * n + 1), sizeof(ONode));
    b->n_nodes = 0;
    if (n) build(b, 0, n);
}

/* ------------------------------------------------------------------ shapes */
typedef struct { V3 o, d; } Ray;
static inline V3 ray_at(const Ray* r, float t) { return vadd(r->o, vmulf(r->d, t)); }
static inline float ray_offset1(float c) { return (c == 0.0f) ? RAY_EPS : RAY_EPS / c; } /* math/Ray.h:201 */
static inline float ray_offset(V3 n, V3 d) { return ray_offset1(fabsf(vdot(n, d))); }

typedef struct {
    float t;
    V3    n, p;
    int   material;
} Isect;

/* Sphere::intersect_impl (shapes/Sphere.h:295) */
static int sphere_isect(const Aff* w2o, const Aff* o2w, const Lin* nrm, const Ray* ray, float tmin, float tmax, Isect* out)
{
    V3 o = aff_point(w2o, ray->o);
    V3 d = lin_vec(w2o->vx, w2o->vy, w2o->vz, ray->d);
    (void)o2w;
    float a = vdot(d, d), b = 2.0f * vdot(d, o), c = vdot(o, o) - 1.0f * 1.0f;
    float disc = b * b - 4.0f * a * c;
    if (disc > 0.0f) {
        disc    = sqrtf(disc);
        float t = (-b - disc) / (2.0f * a);
        if (t < tmin) t = (-b + disc) / (2.0f * a);
        if (t < tmin || t > tmax) return 0;
        if (out) {
            V3 nl   = vdivf(vmadd(splat(t), d, o), 1.0f);
            out->n  = vnormalize(lin_vec(nrm->vx, nrm->vy, nrm->vz, nl));
            out->p  = ray_at(ray, t);
            out->t  = t;
        }
        return 1;
    }
    return 0;
}
/* Plane::intersect_impl (shapes/Plane.h:391) */
static int plane_isect(const Aff* w2o, const Lin* nrm, const Ray* ray, float tmin, float tmax, Isect* out)
{
    V3 d = lin_vec(w2o->vx, w2o->vy, w2o->vz, ray->d);
    if (d.y == 0.0f) return 0;
    V3    o = aff_point(w2o, ray->o);
    float t = -o.y / d.y;
    if (t < tmin || t > tmax) return 0;
    if (out) {
        out->n = lin_vec(nrm->vx, nrm->vy, nrm->vz, v3(0.0f, 1.0f, 0.0f));
        out->p = ray_at(ray, t);
        out->t = t;
    }
    return 1;
}
/* Triangle::intersect_impl (shapes/Triangle.h:97) */
static int tri_isect(const sp_scene_desc* sd, int tri, const Ray* ray, float tmin, float tmax, Isect* out)
{
    const uint32_t* id = sd->indices + 3 * tri;
    V3 p0 = from3(sd->vertices + 3 * id[0]), p1 = from3(sd->vertices + 3 * id[1]), p2 = from3(sd->vertices + 3 * id[2]);
    float A = p0.x - p1.x, B = p0.y - p1.y, C = p0.z - p1.z;
    float D = p0.x - p2.x, E = p0.y - p2.y, F = p0.z - p2.z;
    float G = ray->d.x, H = ray->d.y, I = ray->d.z;
    float J = p0.x - ray->o.x, K = p0.y - ray->o.y, L = p0.z - ray->o.z;
    float EIHF = fmaf(E, I, -(H * F)), GFDI = fmaf(G, F, -(D * I)), DHEG = fmaf(D, H, -(E * G));
    float denom = fmaf(A, EIHF, fmaf(B, GFDI, C * DHEG));
    if (denom == 0) return 0;
    float beta = fmaf(J, EIHF, fmaf(K, GFDI, L * DHEG)) / denom;
    if (beta <= 0.0f || beta >= 1.0f) return 0;
    float AKJB = fmaf(A, K, -(J * B)), JCAL = fmaf(J, C, -(A * L)), BLKC = fmaf(B, L, -(K * C));
    float gamma = fmaf(I, AKJB, fmaf(H, JCAL, G * BLKC)) / denom;
    if (gamma <= 0.0f || beta + gamma >= 1.0f) return 0;
    float t = -fmaf(F, AKJB, fmaf(E, JCAL, D * BLKC)) / denom;
    if (t < tmin || t > tmax) return 0;
    if (out) {
        V3 n0 = from3(sd->normals + 3 * id[0]), n1 = from3(sd->normals + 3 * id[1]), n2 = from3(sd->normals + 3 * id[2]);
        float alpha = 1.0f - beta - gamma;
        out->n = vnormalize(vmadd(splat(alpha), n0, vmadd(splat(beta), n1, fmulv(gamma, n2))));
        out->p = ray_at(ray, t);
        out->t = t;
        out->material = sd->tri_material[tri];
    }
    return 1;
}

static int prim_isect(const OScene* sc, const OPrim* p, const Ray* ray, float tmin, float tmax, Isect* out)
{
    const sp_scene_desc* d = sc->d;
    if (p->kind == SP_PRIM_TRIANGLE) return tri_isect(d, p->index, ray, tmin, tmax, out);
    const sp_xform_shape* s = &d->shapes[p->index];
    Aff w2o = from_aff(&s->world_to_object), o2w = from_aff(&s->object_to_world);
    Lin nrm = from_lin(&s->normal_to_world);
    int hit = (p->kind == SP_PRIM_SPHERE) ? sphere_isect(&w2o, &o2w, &nrm, ray, tmin, tmax, out)
                                          : plane_isect(&w2o, &nrm, ray, tmin, tmax, out);
    if (hit && out) out->material = s->material;
    return hit;
}

/* intersect_p(BBox, Ray, RayLimits) (math/BBox.h:254) */
static int box_p(const ONode* n, const Ray* r, float tmin, float tmax)
{
    float t0 = tmin, t1 = tmax;
    const float o[3] = { r->o.x, r->o.y, r->o.z }, dd[3] = { r->d.x, r->d.y, r->d.z };
    for (int i = 0; i < 3; ++i) {
        const float inv = 1.0f / dd[i];
        float tn = (n->lo[i] - o[i]) * inv, tf = (n->hi[i] - o[i]) * inv;
        if (tn > tf) { float s = tn; tn = tf; tf = s; }
        t0 = fmaxstd(tn, t0);
        t1 = fminstd(tf, t1);
        if (t0 > t1) return 0;
    }
    return 1;
}

/* NodeInternal::intersect / NodeLeaf::intersect (shapes/BVHAccelerator.h:62, 110) */
static int node_intersect(const OScene* sc, const OBvh* b, int ni, const Ray* ray, float tmin, float* tmax, Isect* out,
                          int lights, C3* L)
{
    const ONode* n = &b->nodes[ni];
    int          result = 0;
    if (n->left < 0) {
        for (int i = n->first; i < n->first + n->count; ++i) {
            const OPrim* p = &b->prims[i];
            if (lights) {
                const sp_light_desc* l = &sc->d->lights[p->index];
                Aff w2o = from_aff(&l->world_to_object), o2w = from_aff(&l->object_to_world);
                Lin nrm = from_lin(&l->normal_to_world);
                Isect is;
                if (sphere_isect(&w2o, &o2w, &nrm, ray, tmin, *tmax, &is)) {
                    *tmax = is.t;
                    *L    = c3(l->radiance[0], l->radiance[1], l->radiance[2]);
                    result = 1;
                }
            } else {
                Isect is;
                if (prim_isect(sc, p, ray, tmin, *tmax, &is)) {
                    *tmax  = is.t;
                    *out   = is;
                    result = 1;
                }
            }
        }
        return result;
    }
    const int ch[2] = { n->left, n->right };
    for (int c = 0; c < 2; ++c) {
        if (box_p(&b->nodes[ch[c]], ray, tmin, *tmax)) {
            if (node_intersect(sc, b, ch[c], ray, tmin, tmax, out, lights, L)) result = 1;
        }
    }
    return result;
}
static int node_any(const OScene* sc, const OBvh* b, int ni, const Ray* ray, float tmin, float tmax, int lights)
{
    const ONode* n = &b->nodes[ni];
    if (n->left < 0) {
        for (int i = n->first; i < n->first + n->count; ++i) {
            const OPrim* p = &b->prims[i];
            if (lights) {
                const sp_light_desc* l = &sc->d->lights[p->index];
                Aff w2o = from_aff(&l->world_to_object), o2w = from_aff(&l->object_to_world);
                Lin nrm = from_lin(&l->normal_to_world);
                if (sphere_isect(&w2o, &o2w, &nrm, ray, tmin, tmax, NULL)) return 1;
            } else if (prim_isect(sc, p, ray, tmin, tmax, NULL)) {
                return 1;
            }
        }
        return 0;
    }
    const int ch[2] = { n->left, n->right };
    for (int c = 0; c < 2; ++c)
        if (box_p(&b->nodes[ch[c]], ray, tmin, tmax) && node_any(sc, b, ch[c], ray, tmin, tmax, lights)) return 1;
    return 0;
}

/* Scene::intersect (base/Scene.h:74) */
static int scene_intersect(const OScene* sc, const Ray* ray, float tmin, float tmax, Isect* out)
{
    int hit = 0;
    for (int i = 0; i < sc->n_unbounded; ++i) {
        Isect is;
        if (prim_isect(sc, &sc->unbounded[i], ray, tmin, tmax, &is)) { tmax = is.t; *out = is; hit = 1; }
    }
    if (sc->bvh.n_prims && node_intersect(sc, &sc->bvh, 0, ray, tmin, &tmax, out, 0, NULL)) hit = 1;
    return hit;
}
/* ------------------------------------------------------------------ image environment light
 * ImageBasedEnvironmentLight (Lights/Light.h:196): constructor (modify_image :296,
 * create_distribution :317, math/Distribution1D.h:16, math/Distribution2D.h:10) and its
 * sample / pdf / intersect_lights (:206-290), in the reference's operation order. */
typedef struct OEnv {
    int    w, h, nu, nv;
    float *rad, *cfunc, *ccdf, *cint, *mfunc, *mcdf;
    float  mint;
    Lin    l2w, w2l;
} OEnv;
static const float MAX_LESS_THAN_ONE = 0x1.fffffep-1f; /* base/Constants.h:15 */
static float rel_lum(float r, float g, float b) { return 0.2126f * r + 0.7152f * g + 0.0722f * b; } /* math/RGB.h:224 */
/* sample_nearest_neighbor(img, s, t, RemapWrap{}, RemapClamp{}) (Image/Image.h:84-117) */
static size_t env_texel_index(int w, int h, float s, float t)
{
    s = fmodf(1.0f + fmodf(s, 1.0f), 1.0f);
    t = (t < 0.0f) ? 0.0f : ((MAX_LESS_THAN_ONE < t) ? MAX_LESS_THAN_ONE : t);
    float u = roundf(s * (float)w), v = roundf(t * (float)h);
    uint32_t x = (uint32_t)u, y = (uint32_t)v;
    if (x > (uint32_t)(w - 1)) x = (uint32_t)(w - 1);
    if (y > (uint32_t)(h - 1)) y = (uint32_t)(h - 1);
    return (size_t)y * (size_t)w + x;
}
static C3 env_texel(const OEnv* e, float s, float t)
{
    const float* c = &e->rad[env_texel_index(e->w, e->h, s, t) * 3];
    return c3(c[0], c[1], c[2]);
}
/* Distribution1D(f, 0, 1) constructor, including its one-slot-shifted normalisation */
static void dist1d_build(const float* fin, size_t n, float* func, float* cdf, float* integral)
{
    for (size_t i = 0; i < n; ++i) func[i] = fabsf(fin[i]);
    cdf[0] = 0.0f;
    for (size_t i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + func[i - 1] * (1.0f - 0.0f) / (float)n;
    float I = cdf[n];
    *integral = I;
    if (I == 0.0f) {
        for (size_t i = 1; i < n + 1; ++i) cdf[i] = (float)i / (float)n;
    } else {
        for (size_t i = 0; i < n; ++i) cdf[i] = cdf[i + 1] / I;
    }
}
static void env_build(const sp_env_image* img, OEnv* e)
{
    const float maxr = img->max_radiance;
    e->w = img->width;
    e->h = img->height;
    size_t np = (size_t)e->w * (size_t)e->h;
    e->rad = (float*)malloc(np * 3 * sizeof(float));
    memcpy(e->rad, img->pixels, np * 3 * sizeof(float));
    for (size_t p = 0; p < np; ++p) { /* modify_image */
        float* c = &e->rad[p * 3];
        for (int i = 0; i < 3; ++i)
            if (isinf(c[i])) c[i] = maxr;
        if (rel_lum(c[0], c[1], c[2]) > maxr) {
            int mi = (c[0] > c[1]) ? ((c[0] > c[2]) ? 0 : 2) : ((c[1] > c[2]) ? 1 : 2);
            for (int i = 0; i < 3; ++i) c[i] = c[i] * maxr / c[mi];
        }
    }
    int width = 2 * e->w, height = 2 * e->h; /* create_distribution */
    float* f = (float*)malloc((size_t)width * height * sizeof(float));
    for (int v = 0; v < height; ++v) {
        float vp = ((float)v + 0.5f) / (float)height;
        float st = orc_sinf(PI_F * ((float)v + 0.5f) / (float)height);
        for (int u = 0; u < width; ++u) {
            float up = ((float)u + 0.5f) / (float)width;
            const float* c = &e->rad[env_texel_index(e->w, e->h, up, vp) * 3];
            float x = rel_lum(c[0], c[1], c[2]);
            x *= st;
            if (isinf(x)) x = maxr;
            x = (maxr < x) ? maxr : x;
            f[(size_t)u + (size_t)v * width] = x;
        }
    }
    e->nu = width;
    e->nv = height;
    e->cfunc = (float*)malloc((size_t)width * height * sizeof(float));
    e->ccdf = (float*)malloc((size_t)(width + 1) * height * sizeof(float));
    e->cint = (float*)malloc((size_t)height * sizeof(float));
    for (int v = 0; v < height; ++v)
        dist1d_build(&f[(size_t)v * width], (size_t)width, &e->cfunc[(size_t)v * width], &e->ccdf[(size_t)v * (width + 1)], &e->cint[v]);
    e->mfunc = (float*)malloc((size_t)height * sizeof(float));
    e->mcdf = (float*)malloc((size_t)(height + 1) * sizeof(float));
    dist1d_build(e->cint, (size_t)height, e->mfunc, e->mcdf, &e->mint);
    e->l2w = from_lin(&img->light_to_world);
    e->w2l = from_lin(&img->world_to_light);
    free(f);
}
static void env_free(OEnv* e)
{
    free(e->rad); free(e->cfunc); free(e->ccdf); free(e->cint); free(e->mfunc); free(e->mcdf);
}
/* Distribution1D::get_offset: std::ranges::upper_bound (libstdc++) over cdf[0..n] */
static size_t dist_offset(const float* cdf, size_t n, float u)
{
    size_t first = 0, len = n + 1;
    while (len > 0) {
        size_t half = len >> 1, mid = first + half;
        if (u < cdf[mid]) len = half;
        else { first = mid + 1; len = len - half - 1; }
    }
    if (first == n + 1 || first == n) return n - 1;
    return first;
}
/* Distribution1D::sample_continuous (math/Distribution1D.h:72) */
static float dist_sample(const float* func, const float* cdf, size_t n, float integral, float u, float* pdf, size_t* off)
{
    size_t o = dist_offset(cdf, n, u);
    *off = o;
    float du = u - cdf[o];
    if ((cdf[o + 1] - cdf[o]) > 0) du /= (cdf[o + 1] - cdf[o]);
    *pdf = (integral > 0) ? func[o] / integral : 0.0f;
    float x = ((float)o + du) / (float)n;
    return (1.0f - x) * 0.0f + x * 1.0f; /* sp::lerp(x, m_min, m_max) */
}
static float sph_theta(V3 v) { return orc_acosf(v.y < -1.0f ? -1.0f : (1.0f < v.y ? 1.0f : v.y)); } /* math/Sampling.h:82 */
static float sph_phi(V3 v) /* math/Sampling.h:87 */
{
    float p = orc_atan2f(v.z, v.x);
    return (p < 0.0f) ? (p + 2.0f * PI_F) : p;
}
static const float INV_2_PI = 1.0f / (2.0f * 3.14159265358979323846f);
static const float INV_PI = 0.318309886183790671538f;
static C3 env_radiance(const OEnv* e, V3 dir) /* intersect_lights_impl (Lights/Light.h:206) */
{
    V3 w = vnormalize(lin_vec(e->w2l.vx, e->w2l.vy, e->w2l.vz, dir));
    return env_texel(e, sph_phi(w) * INV_2_PI, sph_theta(w) * INV_PI);
}
/* size_t conversion + std::clamp of Distribution2D::pdf, as x86-64 GCC converts float -> size_t */
static size_t size_clamp(float x, size_t n)
{
    if (x >= 0.0f) return (x >= (float)n) ? n - 1 : (size_t)x;
    return (x > -1.0f) ? 0 : n - 1;
}
static float env_pdf(const OEnv* e, V3 wi) /* pdf_impl (Lights/Light.h:270) */
{
    V3 w = lin_vec(e->w2l.vx, e->w2l.vy, e->w2l.vz, wi);
    float theta = sph_theta(w), phi = sph_phi(w);
    float st = orc_sinf(theta);
    if (st == 0.0f) return 0.0f;
    float p0 = phi * INV_2_PI, p1 = theta * PI_F;
    size_t iu = size_clamp(p0 * (float)e->nu, (size_t)e->nu), iv = size_clamp(p1 * (float)e->nv, (size_t)e->nv);
    float dpdf = e->cfunc[iv * (size_t)e->nu + iu] / e->mint;
    return dpdf / (2.0f * (PI_F * PI_F) * st);
}
/* Scene::intersect_lights (base/Scene.h:69) */
static int scene_intersect_lights(const OScene* sc, const Ray* ray, float tmin, float tmax, float* dist, C3* L)
{
    int hit = 0;
    for (int i = 0; i < sc->n_unbounded_lights; ++i) {
        const sp_light_desc* l = &sc->d->lights[sc->unbounded_lights[i]];
        if (!(tmax < INF_DIST)) { /* EnvironmentLight / ImageBasedEnvironmentLight::intersect_lights_impl (Lights/Light.h:152, :206) */
            tmax = INF_DIST;
            if (l->kind == SP_LIGHT_IMAGE_ENVIRONMENT) *L = env_radiance(&sc->envs[l->image], ray->d);
            else *L = c3(l->radiance[0], l->radiance[1], l->radiance[2]);
            hit  = 1;
        }
    }
    if (sc->lbvh.n_prims && node_intersect(sc, &sc->lbvh, 0, ray, tmin, &tmax, NULL, 1, L)) hit = 1;
    *dist = tmax;
    return hit;
}
/* Scene::intersect_p (base/Scene.h:79) */
static int scene_any(Ctx* c, const Ray* ray, float tmin, float tmax)
{
    const OScene* sc = c->sc;
    c->shadow++;
    c->rays++;
    for (int i = 0; i < sc->n_unbounded; ++i)
        if (prim_isect(sc, &sc->unbounded[i], ray, tmin, tmax, NULL)) return 1;
    if (sc->bvh.n_prims && node_any(sc, &sc->bvh, 0, ray, tmin, tmax, 0)) return 1;
    if (sc->lbvh.n_prims && node_any(sc, &sc->lbvh, 0, ray, tmin, tmax, 1)) return 1;
    return 0;
}

/* ------------------------------------------------------------------ sampling (math/Sampling.*) */
static V3 uniform_sphere(P2 u)
{
    float z = 1.0f - 2.0f * u.x;
    float r = sqrtf(fmaxstd(0.0f, 1.0f - z * z));
    float phi = 2.0 * PI_F * u.y; /* double product, as written in math/Sampling.h:226 */
    return v3(r * orc_cosf(phi), r * orc_sinf(phi), z);
}
static V3 uniform_hemisphere(P2 u)
{
    float y = u.x;
    float r = sqrtf(fmaxstd(0.0f, 1.0f - y * y));
    float phi = 2.0f * PI_F * u.y;
    return v3(r * orc_cosf(phi), y, r * orc_sinf(phi));
}
static P2 concentric(P2 u)
{
    const float pi4 = PI_F / 4.0f, pi2 = PI_F / 2.0f;
    P2 o = { 2.0f * u.x - 1.0f, 2.0f * u.y - 1.0f };
    if (o.x == 0.0f && o.y == 0.0f) { P2 z = { 0.0f, 0.0f }; return z; }
    float th, r;
    if (fabsf(o.x) > fabsf(o.y)) { r = o.x; th = pi4 * (o.y / o.x); }
    else { r = o.y; th = pi2 - pi4 * (o.x / o.y); }
    P2 res = { r * orc_cosf(th), r * orc_sinf(th) };
    return res;
}
static V3 cosine_hemisphere(P2 u)
{
    P2 d = concentric(u);
    float y = sqrtf(fmaxstd(0.0f, 1.0f - d.x * d.x - d.y * d.y));
    return v3(d.x, y, d.y);
}
#define UNIFORM_SPHERE_PDF (1.0f / (4.0f * PI_F))
#define UNIFORM_HEMI_PDF (1.0f / (2.0f * PI_F))

/* ONB (math/ONB.h) */
typedef struct { V3 u, v, w; } Onb;
static Onb onb_from_v(V3 n)
{
    V3 v = vnormalize(n);
    float sign = copysignf(1.0f, v.z);
    float a = -1.0f / (sign + v.z);
    float b = v.x * v.y * a;
    V3 b1 = v3(1.0f + sign * v.x * v.x * a, sign * b, -sign * v.x);
    V3 b2 = v3(b, sign + v.y * v.y * a, -v.y);
    Onb o = { b2, v, b1 };
    return o;
}
static V3 to_world(const Onb* o, V3 a) { return vadd(vadd(fmulv(a.x, o->u), fmulv(a.y, o->v)), fmulv(a.z, o->w)); }
static V3 to_onb(const Onb* o, V3 a) { return v3(vdot(a, o->u), vdot(a, o->v), vdot(a, o->w)); }

/* ------------------------------------------------------------------ materials (materials/*) */
typedef struct {
    C3    color;
    V3    dir;
    float pdf;
    int   props;
} MS;
enum { P_DIFFUSE = 1, P_GLOSSY = 2, P_SPECULAR = 4, P_REFLECTIVE = 8 };

static float cos2t(V3 w) { return w.y * w.y; }
static float sin2t(V3 w) { return fmaxstd(0.0f, 1.0f - cos2t(w)); }
static float sint(V3 w) { return sqrtf(sin2t(w)); }
static float tant(V3 w) { return sint(w) / w.y; }
static float tan2t(V3 w) { return sin2t(w) / cos2t(w); }
static float cosp(V3 w) { float s = sint(w); return (s == 0.0f) ? 1.0f : fclampstd(w.x / s, -1.0f, 1.0f); }
static float sinp(V3 w) { float s = sint(w); return (s == 0.0f) ? 1.0f : fclampstd(w.z / s, -1.0f, 1.0f); }

static float fresnel(float ci, float ei, float et) /* materials/Material.h:114 */
{
    ci = fclampstd(ci, -1.0f, 1.0f);
    if (!(ci > 0.0f)) { float t = ei; ei = et; et = t; ci = fabsf(ci); }
    float si = sqrtf(fmaxstd(0.0f, 1.0f - ci * ci));
    float st = ei / et * si;
    if (st >= 1) return 1.0f;
    float ct = sqrtf(fmaxstd(0.0f, 1.0f - st * st));
    float rpa = ((et * ci) - (ei * ct)) / ((et * ci) + (ei * ct));
    float rpe = ((ei * ci) - (et * ct)) / ((ei * ci) + (et * ct));
    return (rpa * rpa + rpe * rpe) / 2.0f;
}

static float erfinv_ref(float a) /* math/Math.h:230 */
{
    float p;
    const float t = orc_logf(fmaf(a, 0.0f - a, 1.0f));
    if (fabsf(t) > 6.125f) {
        p = 3.03697567e-10f;
        p = fmaf(p, t, 2.93243101e-8f); p = fmaf(p, t, 1.22150334e-6f); p = fmaf(p, t, 2.84108955e-5f);
        p = fmaf(p, t, 3.93552968e-4f); p = fmaf(p, t, 3.02698812e-3f); p = fmaf(p, t, 4.83185798e-3f);
        p = fmaf(p, t, -2.64646143e-1f); p = fmaf(p, t, 8.40016484e-1f);
    } else {
        p = 5.43877832e-9f;
        p = fmaf(p, t, 1.43285448e-7f); p = fmaf(p, t, 1.22774793e-6f); p = fmaf(p, t, 1.12963626e-7f);
        p = fmaf(p, t, -5.61530760e-5f); p = fmaf(p, t, -1.47697632e-4f); p = fmaf(p, t, 2.31468678e-3f);
        p = fmaf(p, t, 1.15392581e-2f); p = fmaf(p, t, -2.32015476e-1f); p = fmaf(p, t, 8.86226892e-1f);
    }
    return a * p;
}

static P2 beck11(float cti, float U1, float U2) /* materials/Material.cpp:14 */
{
    P2 s;
    if (cti > .9999f) {
        float r = sqrtf(-orc_logf(1.0f - U1));
        float sp = orc_sinf(2.0f * PI_F * U2), cp = orc_cosf(2.0f * PI_F * U2);
        s.x = r * cp; s.y = r * sp;
        return s;
    }
    float sti = sqrtf(fmaxstd(0.0f, 1.0f - cti * cti));
    float tti = sti / cti;
    float coti = 1.0f / tti;
    float a = -1.0f, c = orc_erff(coti);
    float sx = fmaxstd(U1, 1e-6f);
    float thi = orc_acosf(cti);
    float fit = 1.0f + thi * (-0.876f + thi * (0.4265f - 0.0594f * thi));
    float b = c - (1.0f + c) * orc_powf(1.0f - sx, fit);
    const float spi = 1.0f / sqrtf(PI_F);
    float norm = 1.0f / (1.0f + c + spi * tti * orc_expf(-coti * coti));
    for (int it = 0; it < 9; ++it) {
        if (!(b >= a && b <= c)) b = 0.5f * (a + c);
        float ie = erfinv_ref(b);
        float value = norm * (1.0f + b + spi * tti * orc_expf(-ie * ie)) - sx;
        float der = norm * (1.0f - ie * tti);
        if (fabsf(value) < 1e-5f) break;
        if (value > 0) c = b; else a = b;
        b -= value / der;
    }
    s.x = erfinv_ref(b);
    s.y = erfinv_ref(2.0f * fmaxstd(U2, 1e-6f) - 1.0f);
    return s;
}

static V3 beck_sample(V3 wi, float ax, float ay, float U1, float U2) /* materials/Material.cpp:89 */
{
    V3 st = vnormalize(v3(ax * wi.x, wi.y, ay * wi.z));
    P2 sl = beck11(st.y, U1, U2);
    float tmp = cosp(st) * sl.x - sinp(st) * sl.y;
    sl.y = sinp(st) * sl.x + cosp(st) * sl.y;
    sl.x = tmp;
    sl.x = ax * sl.x;
    sl.y = ay * sl.y;
    return vnormalize(v3(-sl.x, 1.0f, -sl.y));
}

static float bD(const sp_material_desc* m, V3 wh)
{
    float t2 = tan2t(wh);
    if (isinf(t2)) return 0.0f;
    float c4 = cos2t(wh) * cos2t(wh);
    float cp = cosp(wh), sp = sinp(wh);
    return orc_expf(-t2 * ((cp * cp) / (m->alpha_x * m->alpha_x) + (sp * sp) / (m->alpha_y * m->alpha_y))) /
           (PI_F * m->alpha_x * m->alpha_y * c4);
}
static float blambda(const sp_material_desc* m, V3 w)
{
    float at = fabsf(tant(w));
    if (isinf(at)) return 0.0f;
    float cp = cosp(w), sp = sinp(w);
    float alpha = sqrtf((cp * cp) * (m->alpha_x * m->alpha_x) + (sp * sp) * (m->alpha_y * m->alpha_y));
    float a = 1.0f / (alpha * at);
    if (a >= 1.6f) return 0.0f;
    return (1.0f - 1.259f * a + 0.396f * (a * a)) / (3.535f * a + 2.181f * (a * a));
}
static float bpdf(const sp_material_desc* m, V3 wo, V3 wh)
{
    if (m->sample_visible_area) return bD(m, wh) * (1.0f / (1.0f + blambda(m, wo))) * fabsf(vdot(wo, wh)) / fabsf(wo.y);
    return bD(m, wh) * fabsf(wh.y);
}
static C3 mf_eval(const sp_material_desc* m, V3 wo, V3 wi)
{
    float ao = fabsf(wo.y), ai = fabsf(wi.y);
    if (ai == 0.0f || ao == 0.0f) return c3(0, 0, 0);
    V3 wh = vadd(wi, wo);
    if (wh.x == 0.0f && wh.y == 0.0f && wh.z == 0.0f) return c3(0, 0, 0);
    wh = vnormalize(wh);
    float f = fresnel(vdot(wi, wh), 1.0f, m->microfacet_ior);
    float G = 1.0f / (1.0f + blambda(m, wo) + blambda(m, wi));
    C3 r = c3(m->microfacet_r[0], m->microfacet_r[1], m->microfacet_r[2]);
    return cdivf(cmulf(cmulf(cmulf(r, bD(m, wh)), G), f), 4.0f * ai * ao);
}
static float mf_pdf(const sp_material_desc* m, V3 wo, V3 wi)
{
    if (!(wo.y * wi.y > 0.0f)) return 0.0f;
    V3 wh = vnormalize(vadd(wo, wi));
    return bpdf(m, wo, wh) / (4.0f * vdot(wo, wh));
}
static MS ms_zero(void) { MS z; memset(&z, 0, sizeof z); return z; }
static MS mf_sample(const sp_material_desc* m, V3 wo, Mt* rng)
{
    if (wo.y == 0.0f) return ms_zero();
    int flip = wo.y < 0.0f;
    /* beckmann_sample(..., get_next_1D(), get_next_1D()): GCC evaluates right to left */
    float U2 = canonical(rng);
    float U1 = canonical(rng);
    V3 wh = beck_sample(flip ? vneg(wo) : wo, m->alpha_x, m->alpha_y, U1, U2);
    if (flip) wh = vneg(wh);
    float dp = vdot(wo, wh);
    if (dp < 0.0f) return ms_zero();
    V3 wi = vadd(vneg(wo), fmulv(2.0f * vdot(wo, wh), wh));
    if (!(wo.y * wi.y > 0.0f)) return ms_zero();
    MS r;
    r.pdf = bpdf(m, wo, wh) / (4.0f * dp);
    r.color = mf_eval(m, wo, wi);
    r.dir = wi;
    r.props = P_GLOSSY | P_REFLECTIVE;
    return r;
}
static C3 albedo(const sp_material_desc* m) { return c3(m->lambert_albedo[0], m->lambert_albedo[1], m->lambert_albedo[2]); }
static MS lam_sample(const sp_material_desc* m, Mt* rng)
{
    MS r;
    V3 s = uniform_hemisphere(next2(rng));
    r.color = albedo(m);
    r.dir = s;
    r.pdf = UNIFORM_HEMI_PDF;
    r.props = P_DIFFUSE | P_REFLECTIVE;
    return r;
}
/* OneSampleMaterial::get_selection_weights (materials/Material.h:546) */
static int weights(const sp_material_desc* m, V3 wo, Mt* rng, float* w)
{
    float sum = 0.0f;
    if (m->kind == SP_MAT_LAMBERTIAN) {
        w[0] = lum(cmulf(albedo(m), PI_F));
        sum += w[0];
        w[0] = w[0] / sum;
        return 1;
    }
    C3 r = c3(0, 0, 0);
    for (unsigned i = 0; i < 16u; ++i) {
        MS s = mf_sample(m, wo, rng);
        if (s.pdf > 0.0f) r = cadd(r, cdivf(cmulf(s.color, fabsf(s.dir.y)), s.pdf));
    }
    r = cdivf(r, (float)16u);
    w[0] = lum(r);
    sum += w[0];
    w[1] = lum(cmulf(albedo(m), PI_F));
    sum += w[1];
    w[0] = w[0] / sum;
    w[1] = w[1] / sum;
    return 2;
}
static float bx_pdf(const sp_material_desc* m, int i, V3 wo, V3 wi) { return (m->kind == SP_MAT_GLOSSY && i == 0) ? mf_pdf(m, wo, wi) : UNIFORM_HEMI_PDF; }
static C3 bx_eval(const sp_material_desc* m, int i, V3 wo, V3 wi) { return (m->kind == SP_MAT_GLOSSY && i == 0) ? mf_eval(m, wo, wi) : albedo(m); }

static MS os_sample(const sp_material_desc* m, V3 wo, Mt* rng)
{
    if (m->kind == SP_MAT_LAMBERTIAN) return lam_sample(m, rng);
    float w[2];
    weights(m, wo, rng, w);
    float u = canonical(rng), cdf = 0.0f;
    int sel = 1;
    for (int i = 0; i < 2; ++i) {
        if (w[i] + cdf > u) { sel = i; break; }
        cdf += w[i];
    }
    MS res = (sel == 0) ? mf_sample(m, wo, rng) : lam_sample(m, rng);
    if (res.pdf == 0.0f || cblack(res.color)) return ms_zero();
    C3 values[2];
    float pdfs[2];
    for (int i = 0; i < 2; ++i) {
        if (i == sel) { values[i] = res.color; pdfs[i] = res.pdf * w[i]; }
        else { values[i] = bx_eval(m, i, wo, res.dir); pdfs[i] = bx_pdf(m, i, wo, res.dir) * w[i]; }
    }
    float inner = (0.0f + pdfs[0]) + pdfs[1];
    C3 col = c3(0, 0, 0);
    float pdf = 0.0f;
    for (int i = 0; i < 2; ++i)
        if (pdfs[i] > 0.0f) {
            float mw = (inner == 0.0f) ? 0.0f : pdfs[i] / inner;
            col = cadd(col, fmulc(mw, values[i]));
            pdf += pdfs[i];
        }
    MS out = { col, res.dir, pdf, res.props };
    return out;
}
static C3 os_eval(const sp_material_desc* m, V3 wo, V3 wi, Mt* rng)
{
    float w[2];
    int n = weights(m, wo, rng, w);
    float pdfs[2];
    for (int i = 0; i < n; ++i) pdfs[i] = bx_pdf(m, i, wo, wi) * w[i];
    float inner = 0.0f;
    for (int i = 0; i < n; ++i) inner += pdfs[i];
    C3 r = c3(0, 0, 0);
    for (int i = 0; i < n; ++i)
        if (pdfs[i] > 0.0f) r = cadd(r, fmulc((inner == 0.0f) ? 0.0f : pdfs[i] / inner, bx_eval(m, i, wo, wi)));
    return r;
}
static float os_pdf(const sp_material_desc* m, V3 wo, V3 wi, Mt* rng)
{
    float w[2];
    int n = weights(m, wo, rng, w);
    float p = 0.0f;
    for (int i = 0; i < n; ++i) p += w[i] * bx_pdf(m, i, wo, wi);
    return p;
}
/* ClearcoatMaterial (materials/Material.h:723) + Material::sample/eval/pdf (Material.h:461) */
static MS mat_sample_local(const sp_scene_desc* d, int mid, V3 wo, Mt* rng)
{
    const sp_material_desc* m = &d->materials[mid];
    if (m->kind != SP_MAT_CLEARCOAT) return os_sample(m, wo, rng);
    float f = fresnel(wo.y, 1.0f, m->coat_ior);
    C3 cc = c3(m->coat_color[0], m->coat_color[1], m->coat_color[2]);
    if (canonical(rng) < f) {
        MS s;
        s.dir = v3(-wo.x, wo.y, -wo.z);
        s.color = cdivf(fmulc(f, cc), fabsf(s.dir.y));
        s.pdf = f;
        s.props = P_SPECULAR | P_REFLECTIVE;
        return s;
    }
    MS b = os_sample(&d->materials[m->base], wo, rng);
    if (b.pdf == 0.0f) return b;
    MS s = { cmul(csub(c3(1, 1, 1), fmulc(f, cc)), b.color), b.dir, (1.0f - f) * b.pdf, b.props };
    return s;
}
static MS mat_sample(const sp_scene_desc* d, int mid, V3 wo, V3 n, Mt* rng)
{
    Onb o = onb_from_v(n);
    MS r = mat_sample_local(d, mid, to_onb(&o, wo), rng);
    if (r.pdf == 0.0f || cblack(r.color)) return r;
    r.dir = to_world(&o, r.dir);
    return r;
}
static C3 mat_eval(const sp_scene_desc* d, int mid, V3 wo, V3 wi, V3 n, Mt* rng)
{
    Onb o = onb_from_v(n);
    V3 lo = to_onb(&o, wo), li = to_onb(&o, wi);
    const sp_material_desc* m = &d->materials[mid];
    if (m->kind != SP_MAT_CLEARCOAT) return os_eval(m, lo, li, rng);
    float f = fresnel(lo.y, 1.0f, m->coat_ior);
    return fmulc(1.0f - f, os_eval(&d->materials[m->base], lo, li, rng));
}
static float mat_pdf(const sp_scene_desc* d, int mid, V3 wo, V3 wi, V3 n, Mt* rng)
{
    Onb o = onb_from_v(n);
    V3 lo = to_onb(&o, wo), li = to_onb(&o, wi);
    const sp_material_desc* m = &d->materials[mid];
    if (m->kind != SP_MAT_CLEARCOAT) return os_pdf(m, lo, li, rng);
    float f = fresnel(lo.y, 1.0f, m->coat_ior);
    return (1.0f - f) * os_pdf(&d->materials[m->base], lo, li, rng);
}

/* ------------------------------------------------------------------ lights (Lights/Light.h) */
typedef struct {
    C3    L;
    float pdf, tmin, tmax;
    Ray   ray;
} LS;
static float sphere_pdf(const sp_light_desc* l, V3 obs) /* shapes/Sphere.h:271 */
{
    Aff w2o = from_aff(&l->world_to_object);
    V3 o = aff_point(&w2o, obs);
    float sq = vdot(o, o);
    if (sq <= 1.0f) return UNIFORM_SPHERE_PDF;
    float s2 = 1.0f / sq;
    float cm = sqrtf(fmaxstd(0.0f, 1.0f - s2));
    float omc = (s2 < 0.00068523f) ? s2 / 2.0f : 1.0f - cm;
    return 1.0f / (2.0f * PI_F * omc);
}
static LS light_sample(const OScene* sc, const sp_light_desc* l, V3 obs, V3 obs_n, P2 u)
{
    LS s;
    V3 wi;
    float pdf, maxd;
    s.L = c3(l->radiance[0], l->radiance[1], l->radiance[2]);
    if (l->kind == SP_LIGHT_IMAGE_ENVIRONMENT) { /* ImageBasedEnvironmentLight::light_sample (Lights/Light.h:243) */
        const OEnv* e = &sc->envs[l->image];
        float pdf1, pdf0;
        size_t v, iu;
        float d1 = dist_sample(e->mfunc, e->mcdf, (size_t)e->nv, e->mint, u.y, &pdf1, &v);
        float d0 = dist_sample(&e->cfunc[v * (size_t)e->nu], &e->ccdf[v * (size_t)(e->nu + 1)], (size_t)e->nu, e->cint[v], u.x, &pdf0, &iu);
        float map_pdf = pdf0 * pdf1;
        maxd = INF_DIST;
        if (map_pdf == 0.0f) {
            pdf = 0.0f;
            s.L = c3(0, 0, 0);
            wi = v3(0, 0, 0);
        } else {
            float theta = d1 * PI_F, phi = d0 * 2.0f * PI_F;
            float ct = orc_cosf(theta), st = orc_sinf(theta), sp = orc_sinf(phi), cp = orc_cosf(phi);
            wi = lin_vec(e->l2w.vx, e->l2w.vy, e->l2w.vz, v3(st * cp, ct, st * sp));
            pdf = (st == 0.0f) ? 0.0f : map_pdf / (2.0f * (PI_F * PI_F) * st);
            s.L = env_texel(e, d0, d1);
        }
    } else if (l->kind == SP_LIGHT_SPHERE) {
        Aff w2o = from_aff(&l->world_to_object), o2w = from_aff(&l->object_to_world);
        Lin nrm = from_lin(&l->normal_to_world);
        V3 lo = aff_point(&w2o, obs), local;
        if (vdot(lo, lo) <= 1.0f) local = uniform_sphere(u);
        else {
            V3 smp = cosine_hemisphere(u);
            Onb o = onb_from_v(lo);
            local = to_world(&o, smp);
        }
        V3 sp = aff_point(&o2w, local);
        V3 sn = lin_vec(nrm.vx, nrm.vy, nrm.vz, local);
        V3 ts = vsub(sp, obs);
        wi = vnormalize(ts);
        pdf = sphere_pdf(l, obs);
        maxd = vlength(ts) - ray_offset(sn, vneg(wi));
    } else {
        wi = uniform_sphere(u);
        pdf = UNIFORM_SPHERE_PDF;
        maxd = INF_DIST;
    }
    s.pdf = pdf;
    s.tmin = ray_offset(obs_n, wi);
    s.tmax = maxd;
    s.ray.o = obs;
    s.ray.d = wi;
    return s;
}

/* ------------------------------------------------------------------ integrators (Integrators/Integrator.cpp) */
static C3 nee_direct(Ctx* c, const Isect* is, V3 wo) /* Integrator.cpp:295-307 */
{
    const sp_scene_desc* d = c->sc->d;
    C3 L = c3(0, 0, 0);
    for (int li = 0; li < d->info.num_lights; ++li) {
        LS ls = light_sample(c->sc, &d->lights[li], is->p, is->n, next2(&c->rng));
        if (ls.pdf == 0.0f || cblack(ls.L)) continue;
        V3 wi = ls.ray.d;
        C3 f = mat_eval(d, is->material, wo, wi, is->n, &c->rng);
        if (!cblack(f) && !scene_any(c, &ls.ray, ls.tmin, ls.tmax))
            L = cadd(L, cdivf(cmulf(cmul(f, ls.L), fabsf(vdot(wi, is->n))), ls.pdf));
    }
    return L;
}
static int trace(Ctx* c, const Ray* r, float tmin, float tmax, int* lhit, float* ldist, C3* lL, Isect* is)
{
    c->rays++;
    *lhit = scene_intersect_lights(c->sc, r, tmin, tmax, ldist, lL);
    if (*lhit) tmax = *ldist;
    return scene_intersect(c->sc, r, tmin, tmax, is);
}
static C3 integrate_direct(Ctx* c, Ray ray) /* Integrator.cpp:277 */
{
    C3 L = c3(0, 0, 0);
    if (0 >= c->sc->max_depth) return L;
    int lh; float ld; C3 lL; Isect is;
    if (trace(c, &ray, RAY_EPS, INF_DIST, &lh, &ld, &lL, &is)) L = nee_direct(c, &is, vneg(ray.d));
    else if (lh) L = cadd(L, cmul(c3(1, 1, 1), lL));
    return L;
}
static C3 integrate_iterative(Ctx* c, Ray ray, int rr) /* Integrator.cpp:160, 211 */
{
    const sp_scene_desc* d = c->sc->d;
    C3 thr = c3(1, 1, 1), L = c3(0, 0, 0);
    float tmin = RAY_EPS, tmax = INF_DIST;
    for (int depth = 0; depth < c->sc->max_depth; ++depth) {
        int lh; float ld; C3 lL; Isect is;
        if (trace(c, &ray, tmin, tmax, &lh, &ld, &lL, &is)) {
            V3 wo = vneg(ray.d), n = is.n;
            MS s = mat_sample(d, is.material, wo, n, &c->rng);
            if (s.pdf == 0.0f || cblack(s.color)) break;
            float cosine = fabsf(vdot(s.dir, n));
            thr = cmul(thr, cdivf(fmulc(cosine, s.color), s.pdf));
            if (rr && depth >= c->sc->rr_depth) {
                float lu = lum(thr);
                if (lu < 0.1f) {
                    float q = fmaxstd(0.05f, lu / 0.1f);
                    if (canonical(&c->rng) < q) thr = cdivf(thr, q);
                    else break;
                }
            }
            ray.o = ray_at(&ray, is.t);
            ray.d = s.dir;
            tmin = ray_offset1(cosine);
            tmax = INF_DIST;
        } else if (lh) {
            L = cadd(L, cmul(thr, lL));
            break;
        } else break;
    }
    return L;
}
static C3 integrate_bruteforce(Ctx* c, Ray ray, int depth) /* Integrator.cpp:116 (recursive) */
{
    if (depth >= c->sc->max_depth) return c3(0, 0, 0);
    int lh; float ld; C3 lL; Isect is;
    if (trace(c, &ray, RAY_EPS, INF_DIST, &lh, &ld, &lL, &is)) {
        V3 wo = vneg(ray.d), n = is.n;
        MS s = mat_sample(c->sc->d, is.material, wo, n, &c->rng);
        if (s.pdf == 0.0f || cblack(s.color)) return c3(0, 0, 0);
        float cosine = vdot(s.dir, n);
        Ray out = { ray_at(&ray, is.t), s.dir };
        C3 inc = integrate_bruteforce(c, out, depth + 1);
        return cdivf(cmul(cmulf(inc, cosine), s.color), s.pdf);
    } else if (lh) return lL;
    return c3(0, 0, 0);
}
static C3 integrate_whitted(Ctx* c, Ray ray, int depth) /* Integrator.cpp:323 */
{
    C3 L = c3(0, 0, 0);
    if (depth >= c->sc->max_depth) return L;
    int lh; float ld; C3 lL; Isect is;
    if (trace(c, &ray, RAY_EPS, INF_DIST, &lh, &ld, &lL, &is)) {
        V3 wo = vneg(ray.d);
        L = nee_direct(c, &is, wo);
        if (depth < c->sc->max_depth) {
            MS s = mat_sample(c->sc->d, is.material, wo, is.n, &c->rng);
            if (s.props & P_SPECULAR) {
                Ray out = { is.p, s.dir };
                L = cadd(L, integrate_whitted(c, out, depth + 1));
            }
        }
    } else if (lh) L = cadd(L, cmul(c3(1, 1, 1), lL));
    return L;
}
static C3 est_direct_mis(Ctx* c, int li, V3 p, V3 n, V3 wo, int mid) /* Integrator.cpp:486 */
{
    const sp_scene_desc* d = c->sc->d;
    const sp_light_desc* l = &d->lights[li];
    C3 Lr = c3(0, 0, 0);
    LS ls = light_sample(c->sc, l, p, n, next2(&c->rng));
    if (ls.pdf == 0.0f || cblack(ls.L)) return Lr;
    if (scene_any(c, &ls.ray, ls.tmin, ls.tmax)) return Lr;
    V3 wi = ls.ray.d;
    C3 be = mat_eval(d, mid, wo, wi, n, &c->rng);
    if (!cblack(be)) {
        float bp = mat_pdf(d, mid, wo, wi, n, &c->rng);
        if (bp > 0.0f) {
            float inner = ls.pdf + bp;
            float w = (inner == 0.0f) ? 0.0f : ls.pdf / inner;
            Lr = cadd(Lr, cmulf(cmul(be, ls.L), fabsf(vdot(wi, n)) * w / ls.pdf));
        }
    }
    MS ms = mat_sample(d, mid, wo, n, &c->rng);
    if (ms.pdf == 0.0f || cblack(ms.color)) return Lr;
    float lp = (l->kind == SP_LIGHT_SPHERE) ? sphere_pdf(l, p) : (l->kind == SP_LIGHT_IMAGE_ENVIRONMENT) ? env_pdf(&c->sc->envs[l->image], ms.dir) : UNIFORM_SPHERE_PDF;
    if (lp == 0.0f) return Lr;
    float inner = ms.pdf + lp;
    float w = (inner == 0.0f) ? 0.0f : ms.pdf / inner;
    Ray mr = { p, ms.dir };
    float mmin = ray_offset(n, ms.dir), ld;
    C3 lL;
    c->rays++;
    if (scene_intersect_lights(c->sc, &mr, mmin, INF_DIST, &ld, &lL)) {
        if (!scene_any(c, &mr, mmin, INF_DIST))
            Lr = cadd(Lr, cdivf(cmulf(cmulf(cmul(ms.color, lL), fabsf(vdot(ms.dir, n))), w), ms.pdf));
    }
    return Lr;
}
static C3 integrate_rrnee(Ctx* c, Ray ray) /* Integrator.cpp:550 */
{
    const sp_scene_desc* d = c->sc->d;
    C3 thr = c3(1, 1, 1), L = c3(0, 0, 0);
    float tmin = RAY_EPS, tmax = INF_DIST;
    for (int depth = 0; depth < c->sc->max_depth; ++depth) {
        int lh; float ld; C3 lL; Isect is;
        if (trace(c, &ray, tmin, tmax, &lh, &ld, &lL, &is)) {
            V3 wo = vneg(ray.d), n = is.n;
            MS s = mat_sample(d, is.material, wo, n, &c->rng);
            if (s.pdf == 0.0f || cblack(s.color)) break;
            for (int li = 0; li < d->info.num_lights; ++li)
                L = cadd(L, cmul(thr, est_direct_mis(c, li, is.p, n, wo, is.material)));
            V3 next_o = ray_at(&ray, is.t);
            float cosine = fabsf(vdot(s.dir, n));
            thr = cmul(thr, cdivf(fmulc(cosine, s.color), s.pdf));
            if (depth >= c->sc->rr_depth) {
                float lu = lum(thr);
                if (lu < 0.1f) {
                    float q = fmaxstd(0.05f, lu / 0.1f);
                    if (canonical(&c->rng) < q) thr = cdivf(thr, q);
                    else break;
                }
            }
            ray.o = next_o;
            ray.d = s.dir;
            tmin = ray_offset1(cosine);
            tmax = INF_DIST;
        } else if (lh) {
            L = cadd(L, cmul(thr, lL));
            break;
        } else break;
    }
    return L;
}

/* ------------------------------------------------------------------ render (main.cpp:77) */
static uint32_t morton1(uint32_t a)
{
    a &= 0x55555555u;
    a = (a | (a >> 1)) & 0x33333333u;
    a = (a | (a >> 2)) & 0x0F0F0F0Fu;
    a = (a | (a >> 4)) & 0x00FF00FFu;
    a = (a | (a >> 8)) & 0x0000FFFFu;
    return a;
}

typedef struct {
    const OScene*  sc;
    int            integrator;
    uint32_t       spp;
    const int32_t* tiles;
    int64_t        n_tiles;
    float*         out;
    int64_t        next;
    pthread_mutex_t mu;
    uint64_t       rays, shadow, samples;
} Job;

/* MandelbrotIntegrator::integrate_impl + mandel (Integrators/Integrator.cpp:59-105), HSV
 * to_rgb (math/HSV.h:133, the active #else branch) */
static C3 integrate_mandelbrot(float px, float py, int W, int H)
{
    const float x0 = -2.0f, x1 = 1.0f, y0 = -1.0f, y1 = 1.0f;
    const float dx = (x1 - x0) / (float)W;
    const float dy = (y1 - y0) / (float)H;
    const float cre = x0 + px * dx, cim = y0 + py * dy;
    float zr = cre, zi = cim;
    int it = 0;
    for (; it < 4096; ++it) {
        if (zr * zr + zi * zi > 4.0f) break;
        const float nr = zr * zr - zi * zi;
        const float ni = 2.0f * zr * zi;
        zr = cre + nr;
        zi = cim + ni;
    }
    const float value = (float)it / (float)4096;
    const float hue   = fmodf(orc_powf(value * 360.0f, 1.5f), 360.0f) / 360.0f;
    const float Cc    = value * 1.0f;
    const int   hp    = (int)floorf(hue * 6.0f);
    const float X     = (float)((double)Cc * (1.0 - fabs(fmod((double)hp, 2.0) - 1.0)));
    switch (hp % 6) {
    case 0: return c3(Cc, X, 0);
    case 1: return c3(X, Cc, 0);
    case 2: return c3(0, Cc, X);
    case 3: return c3(0, X, Cc);
    case 4: return c3(X, 0, Cc);
    case 5: return c3(Cc, 0, X);
    }
    return c3(0, 0, 0);
}

static void render_tile(Job* j, int64_t slot)
{
    const OScene* sc = j->sc;
    const int W = sc->d->info.image_width, H = sc->d->info.image_height;
    const int tw = (W + 7) / 8;
    const int32_t tile = j->tiles ? j->tiles[slot] : (int32_t)slot;
    const int x0 = (tile % tw) * 8, y0 = (tile / tw) * 8;
    Ctx c;
    c.sc = sc;
    c.rays = c.shadow = 0;
    uint64_t samples = 0;
    for (uint32_t m = 0; m < 64; ++m) {
        const uint32_t px = (uint32_t)x0 + morton1(m), py = (uint32_t)y0 + morton1(m >> 1);
        float* o = j->out + ((size_t)slot * 64 + m) * 3;
        if ((int)px >= W || (int)py >= H) { o[0] = o[1] = o[2] = 0.0f; continue; }
        const uint32_t seed = (px << 16u) | py;
        mt_seed(&c.rng, seed ^ 0xb0ae9d99u);
        const uint32_t s2 = seed ^ 0x6184faf4u;
        C3 acc = c3(0, 0, 0);
        for (uint32_t i = 0; i < j->spp; ++i) {
            const float fseed = (float)s2 / 3.40282346638528859812e+38f;
            float dummy;
            const float sx = modff(fseed + g_alpha2[0] * ((float)i + 1.0f), &dummy);
            const float sy = modff(fseed + g_alpha2[1] * ((float)i + 1.0f), &dummy);
            const float fx = (float)(int)px + sx, fy = (float)(int)py + sy;
            Ray ray;
            ray.o = sc->cam.p;
            ray.d = vnormalize(vadd(vadd(fmulv(fx, sc->cam.vx), fmulv(fy, sc->cam.vy)), sc->cam.vz));
            C3 L;
            switch (j->integrator) {
            case SP_INTEGRATOR_MANDELBROT: L = integrate_mandelbrot(fx, fy, W, H); break;
            case SP_INTEGRATOR_BRUTE_FORCE: L = integrate_bruteforce(&c, ray, 0); break;
            case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE: L = integrate_iterative(&c, ray, 0); break;
            case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR: L = integrate_iterative(&c, ray, 1); break;
            case SP_INTEGRATOR_ITERATIVE_RRNEE: L = integrate_rrnee(&c, ray); break;
            case SP_INTEGRATOR_WHITTED: L = integrate_whitted(&c, ray, 0); break;
            default: L = integrate_direct(&c, ray); break;
            }
            acc = cadd(acc, L);
        }
        acc = cdivf(acc, (float)j->spp);
        o[0] = acc.r; o[1] = acc.g; o[2] = acc.b;
        samples += j->spp;
    }
    pthread_mutex_lock(&j->mu);
    j->rays += c.rays;
    j->shadow += c.shadow;
    j->samples += samples;
    pthread_mutex_unlock(&j->mu);
}

static void* worker(void* arg)
{
    Job* j = (Job*)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int64_t s = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (s >= j->n_tiles) break;
        render_tile(j, s);
    }
    return NULL;
}

/* Public entry: render tiles into out[(slot*64 + morton)*3 + c]; stats = {rays, shadow, samples}. */
int orc_render(const sp_scene_desc* d, int integrator, uint32_t spp, const int32_t* tile_ids, int64_t n_tiles,
               int threads, float* out, uint64_t* stats)
{
    if (!d || !out || spp == 0) return -3;
    init_rsequence();
    OScene sc;
    memset(&sc, 0, sizeof sc);
    sc.d = d;
    sc.cam = from_aff(&d->camera.transform);
    sc.max_depth = d->info.max_depth;
    sc.rr_depth = d->info.russian_roulette_depth;
    if (integrator == SP_INTEGRATOR_NOT_SPECIFIED) integrator = d->info.integrator_type;
    if (integrator == SP_INTEGRATOR_NOT_SPECIFIED) integrator = SP_INTEGRATOR_DIRECT_LIGHTING;
    /* geometry: partition bounded/unbounded (base/Scene.h:34) then BVH */
    int64_t np = d->num_prims;
    OPrim* prims = (OPrim*)calloc((size_t)np + 1, sizeof(OPrim));
    for (int64_t i = 0; i < np; ++i) { prims[i].kind = d->prim_kind[i]; prims[i].index = d->prim_index[i]; }
    int first = 0, last = (int)np;
    for (;;) { /* std::partition(is_bounded) */
        int done = 0;
        for (;;) {
            if (first == last) { done = 1; break; }
            if (prims[first].kind != SP_PRIM_PLANE) ++first; else break;
        }
        if (done) break;
        --last;
        for (;;) {
            if (first == last) { done = 1; break; }
            if (!(prims[last].kind != SP_PRIM_PLANE)) --last; else break;
        }
        if (done) break;
        OPrim t = prims[first]; prims[first] = prims[last]; prims[last] = t;
        ++first;
    }
    const int nb = first;
    for (int i = 0; i < nb; ++i) prim_bounds(d, &prims[i]);
    sc.unbounded = prims + nb;
    sc.n_unbounded = (int)np - nb;
    build_bvh(&sc.bvh, prims, nb);
    /* lights */
    int nl = d->info.num_lights;
    int* lid = (int*)calloc((size_t)nl + 1, sizeof(int));
    for (int i = 0; i < nl; ++i) lid[i] = i;
    first = 0; last = nl;
    for (;;) {
        int done = 0;
        for (;;) {
            if (first == last) { done = 1; break; }
            if (d->lights[lid[first]].kind == SP_LIGHT_SPHERE) ++first; else break;
        }
        if (done) break;
        --last;
        for (;;) {
            if (first == last) { done = 1; break; }
            if (!(d->lights[lid[last]].kind == SP_LIGHT_SPHERE)) --last; else break;
        }
        if (done) break;
        int t = lid[first]; lid[first] = lid[last]; lid[last] = t;
        ++first;
    }
    OPrim* lprims = (OPrim*)calloc((size_t)first + 1, sizeof(OPrim));
    for (int i = 0; i < first; ++i) { lprims[i].kind = 10 + lid[i]; lprims[i].index = lid[i]; prim_bounds(d, &lprims[i]); }
    build_bvh(&sc.lbvh, lprims, first);
    sc.unbounded_lights = lid + first;
    sc.n_unbounded_lights = nl - first;
    OEnv* envs = (OEnv*)calloc((size_t)d->num_env_images + 1, sizeof(OEnv));
    for (int i = 0; i < d->num_env_images; ++i) env_build(&d->env_images[i], &envs[i]);
    sc.envs = envs;

    Job j;
    memset(&j, 0, sizeof j);
    j.sc = &sc;
    j.integrator = integrator;
    j.spp = spp;
    j.tiles = tile_ids;
    int64_t total = (int64_t)((d->info.image_width + 7) / 8) * ((d->info.image_height + 7) / 8);
    j.n_tiles = tile_ids ? n_tiles : total;
    j.out = out;
    pthread_mutex_init(&j.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &j);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&j.mu);
    if (stats) { stats[0] = j.rays; stats[1] = j.shadow; stats[2] = j.samples; }
    free(sc.bvh.nodes);
    free(sc.lbvh.nodes);
    free(prims);
    free(lprims);
    free(lid);
    for (int i = 0; i < d->num_env_images; ++i) env_free(&envs[i]);
    free(envs);
    return 0;
}

/* Unit hooks for the tests. */
void orc_mt_stream(uint32_t seed, int n, float* out)
{
    Mt s;
    mt_seed(&s, seed);
    for (int i = 0; i < n; ++i) out[i] = canonical(&s);
}
float orc_rsqrt(float x) { return rsqrt_ref(x); }
