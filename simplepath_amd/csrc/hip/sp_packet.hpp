// sp_packet.hpp -- wave-coherent BVH traversal for coherent rays (camera rays of one 8x8 tile,
// shadow rays of one tile towards a light).
//
// The per-lane traversal of sp_path.hpp gives every lane its own node sequence: each node fetch
// is a 64-way divergent gather, and the vector L1 address path, not HBM, bounds the kernel
// (profiles/r01: 85% of wave cycles in s_waitcnt at 7 waves/SIMD).  Here the active lanes of a
// wave walk ONE depth-first order together:
//
//   visit(node, M): M' = { lane in M : box_hit(node, lane's ray, lane's current t_max) }
//                   if M' empty: return
//                   leaf  -> every lane in M' tests the leaf's primitives
//                   inner -> visit(child0, M'); visit(child1, M')
//
// For each lane, the nodes where it is active are exactly the nodes its own recursion
// (shapes/BVHAccelerator.h:62-77) visits, in the same order, each box tested against the limits
// current at that moment -- so results are bit-identical to the per-lane traversal and to the
// reference, for either BVH build.  Node and primitive addresses are wave-uniform: one coalesced
// request per node (lane i fetches dword i, v_readlane broadcasts) instead of 64 lane requests.  The stack is wave-uniform too and lives in
// three VGPRs used as 64-entry arrays across lanes (entry e in lane e: select on push, v_readlane on pop),
// so the traversal needs no LDS at all; BVHs deeper than 64 fall back to the per-lane path.
#pragma once
#include "sp_path.hpp"

namespace spd {

constexpr int PACKET_MAX_DEPTH = 64;

struct WStack {
    uint32_t node = 0, mlo = 0, mhi = 0; // lane e holds entry e
    int      sp   = 0;                   // wave-uniform
};

__device__ __forceinline__ void wpush(WStack& s, uint32_t node, uint64_t mask)
{
    const bool sel = (int)(threadIdx.x & 63) == s.sp; // one v_cmp + v_cndmask per word
    s.node         = sel ? node : s.node;
    s.mlo          = sel ? (uint32_t)mask : s.mlo;
    s.mhi          = sel ? (uint32_t)(mask >> 32) : s.mhi;
    ++s.sp;
}
__device__ __forceinline__ void wpop(WStack& s, uint32_t& node, uint64_t& mask)
{
    --s.sp;
    node = (uint32_t)__builtin_amdgcn_readlane((int)s.node, s.sp);
    mask = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)s.mlo, s.sp) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)s.mhi, s.sp) << 32);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ bool lane_in(uint64_t m) { return (m >> (threadIdx.x & 63)) & 1ull; }

// Wave-uniform fetches through the constant address space (scalar loads) -- used for the
// light records; BVH nodes and leaves use the cooperative vector fetch below.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) u32x4  c_u32x4;
typedef const __attribute__((address_space(4))) uint32_t c_u32;

__device__ __forceinline__ u32x4 cld4(const void* base, uint32_t i) { return ((c_u32x4*)base)[i]; }
__device__ __forceinline__ uint32_t cld1(const void* base, uint32_t i) { return ((c_u32*)base)[i]; }
__device__ __forceinline__ float4 as_f4(u32x4 v)
{
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

__device__ __forceinline__ uint32_t bcast(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ float bcastf(uint32_t v, int l) { return __uint_as_float(bcast(v, l)); }

// Cooperative fetch: lane i reads dword i of the record (one coalesced vector request for the
// whole wave; the vector memory path keeps far more misses in flight than the scalar cache),
// then v_readlane moves each dword into an SGPR.  Requires the full wave to be active (EXEC =
// all ones), which every call site guarantees: the walk runs in wave-uniform control flow.
__device__ __forceinline__ Node wnode(const Node* nodes, uint32_t i)
{
    const uint32_t* p = reinterpret_cast<const uint32_t*>(nodes) + (size_t)uni(i) * 8;
    const uint32_t  v = p[threadIdx.x & 7];
    Node            n;
    n.lo[0] = bcastf(v, 0); n.lo[1] = bcastf(v, 1); n.lo[2] = bcastf(v, 2); n.a = bcast(v, 3);
    n.hi[0] = bcastf(v, 4); n.hi[1] = bcastf(v, 5); n.hi[2] = bcastf(v, 6); n.b = bcast(v, 7);
    return n;
}

// Up to LEAF_CHUNK primitives of a leaf in one request: lanes 0..47 = triangle vertex dwords
// (12 per slot), lanes 48..51 = slot codes.
constexpr uint32_t LEAF_CHUNK = 4;
__device__ __forceinline__ uint32_t wleaf(const Scene& sc, uint32_t first, uint32_t n)
{
    const uint32_t l = threadIdx.x & 63;
    const uint32_t* tri  = reinterpret_cast<const uint32_t*>(sc.slot_tri) + (size_t)first * 12;
    const uint32_t  cnt  = n < LEAF_CHUNK ? n : LEAF_CHUNK;
    const uint32_t* addr = (l < 48) ? tri + (l < 12 * cnt ? l : 0) : sc.slot_code + first + (l - 48 < cnt ? l - 48 : 0);
    return *addr;
}
__device__ __forceinline__ float4 leaf_q(uint32_t v, uint32_t k, int j)
{
    const int b = (int)(12 * k + 4 * j);
    return make_float4(bcastf(v, b), bcastf(v, b + 1), bcastf(v, b + 2), bcastf(v, b + 3));
}

// Scene::intersect (base/Scene.h:74) for the active lanes; `on` = this lane has a ray.
__device__ __forceinline__ Hit scene_intersect_w(const Scene& sc, const Ray& ray, float tmin, float tmax, bool on,
                                              uint32_t* steps = nullptr)
{
    Hit h;
    h.t    = tmax;
    h.code = 0xffffffffu;
    if (on) {
        for (int i = 0; i < sc.n_unbounded; ++i) {
            const int    sid = sc.unbounded[i];
            const Shape& s   = sc.shapes[sid];
            float        t;
            const bool   hit = (s.kind == SP_PRIM_SPHERE) ? sphere_t(s.w2o, ray, tmin, h.t, t) : plane_t(s.w2o, ray, tmin, h.t, t);
            if (hit) { h.t = t; h.code = ((uint32_t)s.kind << CODE_SHIFT) | (uint32_t)sid; }
        }
    }
    uint64_t m = __ballot(on);
    if (sc.n_nodes == 0 || m == 0) return h;
    const f3 inv      = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    WStack   st;
    uint32_t cur      = 0;     // root: no box test (as the per-lane path)
    bool     test_box = false;
    while (true) {
        const Node n  = wnode(sc.nodes, cur);
        if (steps) ++*steps;
        bool       me = lane_in(m);
        if (me && test_box) me = box_hit(n, ray, inv, tmin, h.t);
        const uint64_t m2 = __ballot(me);
        if (m2) {
            const uint32_t nb = uni(n.b);
            if (nb & LEAF_BIT) {
                const uint32_t first = uni(n.a), cnt = nb & ~LEAF_BIT;
                uint32_t       blk   = 0;
                for (uint32_t k = 0; k < cnt; ++k) {
                    if (k % LEAF_CHUNK == 0) blk = wleaf(sc, first + k, cnt - k);
                    const uint32_t kk   = k % LEAF_CHUNK;
                    const uint32_t code = bcast(blk, (int)(48 + kk));
                    const uint32_t kind = code >> CODE_SHIFT;
                    if (kind == KIND_TRI) {
                        const float4 q0 = leaf_q(blk, kk, 0), q1 = leaf_q(blk, kk, 1), q2 = leaf_q(blk, kk, 2);
                        float        t, be, ga;
                        if (me && tri_hit(q0, q1, q2, ray, tmin, h.t, t, be, ga)) {
                            h.t = t; h.code = code; h.beta = be; h.gamma = ga;
                        }
                    } else {
                        const Shape& s = sc.shapes[code & CODE_MASK];
                        float        t;
                        if (me && ((kind == KIND_SPHERE) ? sphere_t(s.w2o, ray, tmin, h.t, t) : plane_t(s.w2o, ray, tmin, h.t, t))) {
                            h.t = t; h.code = code;
                        }
                    }
                }
            } else {
                wpush(st, nb, m2); // child 1 deferred, its box tested when popped
                cur      = uni(n.a) & CHILD_MASK;
                m        = m2;
                test_box = true;
                continue;
            }
        }
        if (st.sp == 0) break;
        wpop(st, cur, m);
        test_box = true;
    }
    return h;
}

// Scene::intersect_lights (base/Scene.h:69) for the active lanes.
__device__ __forceinline__ LightHit scene_intersect_lights_w(const Scene& sc, const Ray& ray, float tmin, float tmax, bool on)
{
    LightHit lh;
    lh.hit = false;
    lh.t   = tmax;
    lh.env = -1;
    if (on) {
        for (int i = 0; i < sc.n_unbounded_lights; ++i) {
            const Light& l = sc.lights[sc.unbounded_lights[i]];
            if (!(lh.t < k_infinite)) { // EnvironmentLight::intersect_lights_impl (Lights/Light.h:242)
                lh.hit = true;
                lh.t   = k_infinite;
                lh.L   = l.radiance;
                lh.env = (l.kind == SP_LIGHT_IMAGE_ENVIRONMENT) ? l.image : -1;
            }
        }
    }
    uint64_t m = __ballot(on);
    if (sc.n_light_nodes == 0 || m == 0) return lh;
    const f3 inv      = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    WStack   st;
    uint32_t cur      = 0;
    bool     test_box = false;
    while (true) {
        const Node n  = wnode(sc.light_nodes, cur);
        bool       me = lane_in(m);
        if (me && test_box) me = box_hit(n, ray, inv, tmin, lh.t);
        const uint64_t m2 = __ballot(me);
        if (m2) {
            const uint32_t nb = uni(n.b);
            if (nb & LEAF_BIT) {
                const uint32_t first = uni(n.a), cnt = nb & ~LEAF_BIT;
                for (uint32_t k = 0; k < cnt; ++k) {
                    const Light& l = sc.lights[cld1(sc.light_slot, first + k)];
                    float        t;
                    if (me && sphere_t(l.w2o, ray, tmin, lh.t, t)) {
                        lh.hit = true;
                        lh.t   = t;
                        lh.L   = l.radiance;
                        lh.env = -1;
                    }
                }
            } else {
                wpush(st, nb, m2);
                cur      = uni(n.a) & CHILD_MASK;
                m        = m2;
                test_box = true;
                continue;
            }
        }
        if (st.sp == 0) break;
        wpop(st, cur, m);
        test_box = true;
    }
    return lh;
}

// Scene::intersect_p (base/Scene.h:79) for the active lanes: geometry, then lights.  A lane
// leaves the walk at its first hit; the walk ends when no lane is still searching.
__device__ __forceinline__ bool any_hit_w(const Scene& sc, const Node* nodes, int n_nodes, bool lights, const Ray& ray,
                                          float tmin, float tmax, bool on, uint32_t* steps = nullptr)
{
    bool found = false;
    if (!lights && on) {
        for (int i = 0; i < sc.n_unbounded; ++i) {
            const Shape& s = sc.shapes[sc.unbounded[i]];
            float        t;
            if ((s.kind == SP_PRIM_SPHERE) ? sphere_t(s.w2o, ray, tmin, tmax, t) : plane_t(s.w2o, ray, tmin, tmax, t)) {
                found = true;
                break;
            }
        }
    }
    uint64_t live = __ballot(on && !found);
    uint64_t m    = live;
    if (n_nodes == 0 || m == 0) return found;
    const f3 inv      = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    WStack   st;
    uint32_t cur      = 0;
    bool     test_box = false;
    while (true) {
        const Node n  = wnode(nodes, cur);
        if (steps) ++*steps;
        bool       me = lane_in(m) && !found;
        if (me && test_box) me = box_hit(n, ray, inv, tmin, tmax);
        const uint64_t m2 = __ballot(me);
        if (m2) {
            const uint32_t nb = uni(n.b);
            if (nb & LEAF_BIT) {
                const uint32_t first = uni(n.a), cnt = nb & ~LEAF_BIT;
                uint32_t       blk   = 0;
                for (uint32_t k = 0; k < cnt; ++k) {
                    const uint32_t slot = first + k;
                    bool           hit  = false;
                    if (!lights && k % LEAF_CHUNK == 0) blk = wleaf(sc, first + k, cnt - k);
                    if (lights) {
                        const Light& l = sc.lights[cld1(sc.light_slot, slot)];
                        float        t;
                        hit = me && !found && sphere_t(l.w2o, ray, tmin, tmax, t);
                    } else {
                        const uint32_t kk   = k % LEAF_CHUNK;
                        const uint32_t code = bcast(blk, (int)(48 + kk));
                        const uint32_t kind = code >> CODE_SHIFT;
                        if (kind == KIND_TRI) {
                            const float4 q0 = leaf_q(blk, kk, 0), q1 = leaf_q(blk, kk, 1), q2 = leaf_q(blk, kk, 2);
                            float        t, be, ga;
                            hit = me && !found && tri_hit(q0, q1, q2, ray, tmin, tmax, t, be, ga);
                        } else {
                            const Shape& s = sc.shapes[code & CODE_MASK];
                            float        t;
                            hit = me && !found &&
                                  ((kind == KIND_SPHERE) ? sphere_t(s.w2o, ray, tmin, tmax, t) : plane_t(s.w2o, ray, tmin, tmax, t));
                        }
                    }
                    found = found || hit;
                }
                live = __ballot(on && !found);
                if (live == 0) break;
            } else {
                wpush(st, nb, m2);
                cur      = uni(n.a) & CHILD_MASK;
                m        = m2;
                test_box = true;
                continue;
            }
        }
        if (st.sp == 0) break;
        wpop(st, cur, m);
        m &= live; // lanes that already hit leave the walk
        test_box = true;
    }
    return found;
}

__device__ __forceinline__ bool scene_any_w(const Scene& sc, const Ray& ray, float tmin, float tmax, bool on,
                                            uint32_t* steps = nullptr)
{
    const bool g = any_hit_w(sc, sc.nodes, sc.n_nodes, false, ray, tmin, tmax, on, steps);
    const bool l = any_hit_w(sc, sc.light_nodes, sc.n_light_nodes, true, ray, tmin, tmax, on && !g);
    return g || l;
}

} // namespace spd
