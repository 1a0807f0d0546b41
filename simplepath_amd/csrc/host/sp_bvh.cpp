// sp_bvh.cpp -- bounding volume hierarchies over the bounded primitives.
//
// build_bvh_reference restates shapes/BVHAccelerator.h:173 `construct` exactly (same split
// axis, same split position, libstdc++ std::partition element order, same leaf contents and
// order) so a depth-first, child-0-first traversal visits primitives in the reference's order
// and resolves equal-distance ties identically.  build_bvh_sah is the throughput build: binned
// SAH (Wald 2007) with the same node format; it changes only the visiting order.
#include "sp_host.hpp"

#include <cstdio>

#include <stdexcept>
#include <cstring>

#include <algorithm>
#include <cmath>
#include <functional>

namespace sph {

namespace {
struct Box {
    float lo[3], hi[3];
};
Box empty_box()
{
    Box b;
    for (int i = 0; i < 3; ++i) {
        b.lo[i] = INFINITY;
        b.hi[i] = -INFINITY;
    }
    return b;
}
// merge (math/BBox.h:192) with _mm_min_ps / _mm_max_ps operand order
Box merge(const Box& a, const PrimBounds& b)
{
    Box r;
    for (int i = 0; i < 3; ++i) {
        r.lo[i] = spm::sse_min(a.lo[i], b.lo[i]);
        r.hi[i] = spm::sse_max(a.hi[i], b.hi[i]);
    }
    return r;
}
float center_of(const PrimBounds& b, int d) { return (b.lo[d] + b.hi[d]) / 2.0f; }

struct RefBuilder {
    const std::vector<PrimBounds>& bounds;
    std::vector<int32_t>           ids;
    std::vector<BvhNode>           nodes;
    int                            max_depth = 0;

    uint32_t build(size_t first, size_t last, int depth)
    {
        max_depth = std::max(max_depth, depth);
        Box bb    = empty_box();
        for (size_t i = first; i < last; ++i) bb = merge(bb, bounds[ids[i]]);
        const uint32_t me = static_cast<uint32_t>(nodes.size());
        nodes.push_back(BvhNode{});
        auto make_leaf = [&]() {
            BvhNode& n = nodes[me];
            for (int i = 0; i < 3; ++i) { n.lo[i] = bb.lo[i]; n.hi[i] = bb.hi[i]; }
            n.a = static_cast<uint32_t>(first);
            n.b = static_cast<uint32_t>(last - first) | BVH_LEAF;
            return me;
        };
        if (last - first <= 4) return make_leaf();
        // max_dim(bounds.size()) (math/Vector3.h:654)
        const float sx = std::fabs(bb.hi[0] - bb.lo[0]);
        const float sy = std::fabs(bb.hi[1] - bb.lo[1]);
        const float sz = std::fabs(bb.hi[2] - bb.lo[2]);
        int         dim;
        if (sx > sy) dim = (sx > sz) ? 0 : 2;
        else dim = (sy > sz) ? 1 : 2;
        const float split_point = (bb.lo[dim] + bb.hi[dim]) / 2.0f;
        const size_t split = stl_partition(ids, first, last, [&](int32_t id) { return center_of(bounds[id], dim) < split_point; });
        if (split == first || split == last) return make_leaf();
        const uint32_t l = build(first, split, depth + 1);
        const uint32_t r = build(split, last, depth + 1);
        BvhNode& n = nodes[me];
        for (int i = 0; i < 3; ++i) { n.lo[i] = bb.lo[i]; n.hi[i] = bb.hi[i]; }
        n.a = l;
        n.b = r;
        return me;
    }
};
} // namespace

Bvh build_bvh_reference(const std::vector<PrimBounds>& bounds)
{
    Bvh        out;
    RefBuilder b{ bounds, {}, {} };
    b.ids.resize(bounds.size());
    for (size_t i = 0; i < bounds.size(); ++i) b.ids[i] = static_cast<int32_t>(i);
    if (!bounds.empty()) b.build(0, bounds.size(), 1);
    out.nodes      = std::move(b.nodes);
    out.prim_order = std::move(b.ids);
    out.max_depth  = b.max_depth;
    return out;
}

// ------------------------------------------------------------------------------ binned SAH
namespace {
struct SahBuilder {
    const std::vector<PrimBounds>& bounds;
    std::vector<int32_t>           ids;
    std::vector<float>             cx, cy, cz;
    std::vector<BvhNode>           nodes;
    int                            max_leaf;
    float                          trav_cost = 1.0f; // node visit cost in triangle tests
    int                            max_depth = 0;

    static float area(const Box& b)
    {
        const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
        if (!(dx >= 0.0f)) return 0.0f;
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
    const float* cen(int d) const { return d == 0 ? cx.data() : (d == 1 ? cy.data() : cz.data()); }

    uint32_t build(size_t first, size_t last, int depth)
    {
        max_depth = std::max(max_depth, depth);
        Box bb = empty_box(), cb = empty_box();
        for (size_t i = first; i < last; ++i) {
            const int32_t id = ids[i];
            bb               = merge(bb, bounds[id]);
            PrimBounds c;
            c.lo[0] = c.hi[0] = cx[id];
            c.lo[1] = c.hi[1] = cy[id];
            c.lo[2] = c.hi[2] = cz[id];
            cb = merge(cb, c);
        }
        const uint32_t me = static_cast<uint32_t>(nodes.size());
        nodes.push_back(BvhNode{});
        const size_t n = last - first;
        auto make_leaf = [&]() {
            BvhNode& nd = nodes[me];
            for (int i = 0; i < 3; ++i) { nd.lo[i] = bb.lo[i]; nd.hi[i] = bb.hi[i]; }
            nd.a = static_cast<uint32_t>(first);
            nd.b = static_cast<uint32_t>(n) | BVH_LEAF;
            return me;
        };
        if (n <= 1) return make_leaf();
        constexpr int BINS = 32;
        float best_cost = INFINITY;
        int   best_dim = -1, best_bin = -1;
        for (int d = 0; d < 3; ++d) {
            const float lo = cb.lo[d], hi = cb.hi[d];
            if (!(hi > lo)) continue;
            const float  k = BINS * (1.0f - 1e-5f) / (hi - lo);
            Box          bins[BINS];
            int          cnt[BINS] = {};
            for (auto& b : bins) b = empty_box();
            const float* c = cen(d);
            for (size_t i = first; i < last; ++i) {
                const int32_t id = ids[i];
                int           bi = static_cast<int>((c[id] - lo) * k);
                bi               = std::min(std::max(bi, 0), BINS - 1);
                cnt[bi]++;
                bins[bi] = merge(bins[bi], bounds[id]);
            }
            float right_area[BINS];
            int   right_cnt[BINS];
            Box   acc = empty_box();
            int   ac  = 0;
            for (int b = BINS - 1; b > 0; --b) {
                PrimBounds pb;
                for (int i = 0; i < 3; ++i) { pb.lo[i] = bins[b].lo[i]; pb.hi[i] = bins[b].hi[i]; }
                if (cnt[b]) acc = merge(acc, pb);
                ac += cnt[b];
                right_area[b] = area(acc);
                right_cnt[b]  = ac;
            }
            acc = empty_box();
            ac  = 0;
            for (int b = 0; b < BINS - 1; ++b) {
                PrimBounds pb;
                for (int i = 0; i < 3; ++i) { pb.lo[i] = bins[b].lo[i]; pb.hi[i] = bins[b].hi[i]; }
                if (cnt[b]) acc = merge(acc, pb);
                ac += cnt[b];
                if (ac == 0 || right_cnt[b + 1] == 0) continue;
                const float cost = area(acc) * ac + right_area[b + 1] * right_cnt[b + 1];
                if (cost < best_cost) { best_cost = cost; best_dim = d; best_bin = b; }
            }
        }
        const float leaf_cost = area(bb) * static_cast<float>(n);
        // traversal cost ~ 1 triangle test per node visit; stop when the split does not pay
        if (best_dim < 0 || (n <= static_cast<size_t>(max_leaf) && best_cost + trav_cost * area(bb) >= leaf_cost)) {
            if (best_dim < 0 && n > static_cast<size_t>(max_leaf)) {
                // all centroids coincide: median split by index
                const size_t mid = first + n / 2;
                const uint32_t l = build(first, mid, depth + 1);
                const uint32_t r = build(mid, last, depth + 1);
                BvhNode& nd = nodes[me];
                for (int i = 0; i < 3; ++i) { nd.lo[i] = bb.lo[i]; nd.hi[i] = bb.hi[i]; }
                nd.a = l; nd.b = r;
                return me;
            }
            return make_leaf();
        }
        const float  lo = cb.lo[best_dim], hi = cb.hi[best_dim];
        const float  k  = BINS * (1.0f - 1e-5f) / (hi - lo);
        const float* c  = cen(best_dim);
        auto mid_it = std::stable_partition(ids.begin() + first, ids.begin() + last, [&](int32_t id) {
            int bi = static_cast<int>((c[id] - lo) * k);
            bi     = std::min(std::max(bi, 0), BINS - 1);
            return bi <= best_bin;
        });
        size_t mid = static_cast<size_t>(mid_it - ids.begin());
        if (mid == first || mid == last) mid = first + n / 2;
        const uint32_t l = build(first, mid, depth + 1);
        const uint32_t r = build(mid, last, depth + 1);
        BvhNode& nd = nodes[me];
        for (int i = 0; i < 3; ++i) { nd.lo[i] = bb.lo[i]; nd.hi[i] = bb.hi[i]; }
        nd.a = l | (static_cast<uint32_t>(best_dim) << BVH_AXIS_SHIFT); // split axis: near-first order
        nd.b = r;
        return me;
    }
};
} // namespace

Bvh build_bvh_sah(const std::vector<PrimBounds>& bounds, int max_leaf)
{
    Bvh        out;
    SahBuilder b{ bounds, {}, {}, {}, {}, {}, max_leaf };
    const size_t n = bounds.size();
    b.ids.resize(n);
    b.cx.resize(n); b.cy.resize(n); b.cz.resize(n);
    for (size_t i = 0; i < n; ++i) {
        b.ids[i] = static_cast<int32_t>(i);
        b.cx[i]  = center_of(bounds[i], 0);
        b.cy[i]  = center_of(bounds[i], 1);
        b.cz[i]  = center_of(bounds[i], 2);
    }
    if (n >= (size_t(1) << BVH_AXIS_SHIFT)) throw std::runtime_error("too many primitives for the SAH BVH");
    if (n) b.build(0, n, 1);
    out.nodes      = std::move(b.nodes);
    out.prim_order = std::move(b.ids);
    out.max_depth  = b.max_depth;
    return out;
}

// ---------------------------------------------------------------- 8-wide collapse
namespace {

float node_area(const BvhNode& n)
{
    const float dx = n.hi[0] - n.lo[0], dy = n.hi[1] - n.lo[1], dz = n.hi[2] - n.lo[2];
    if (!(dx >= 0.0f)) return 0.0f;
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

struct WideBuilder {
    const Bvh& b;
    WideBvh&   out;

    bool is_leaf(uint32_t i) const { return (b.nodes[i].b & BVH_LEAF) != 0; }
    uint32_t left(uint32_t i) const { return b.nodes[i].a & BVH_CHILD_MASK; }
    uint32_t right(uint32_t i) const { return b.nodes[i].b; }

    // Quantise one axis of the children onto origin p with the smallest power-of-two step that
    // keeps every decoded box (fma(q, step, p), as the device decodes it) outside the exact one.
    void quantise(const float* lo, const float* hi, int n, float p, float extent, uint8_t* qlo, uint8_t* qhi,
                  uint8_t& ebyte)
    {
        int k = -126;
        if (extent > 0.0f) {
            int e2;
            std::frexp(extent / 254.0f, &e2); // extent/254 < 2^e2
            k = std::max(e2, -126);
        }
        for (;; ++k) {
            const float step = std::ldexp(1.0f, k);
            bool        ok   = true;
            for (int c = 0; c < n && ok; ++c) {
                float ql = std::floor((lo[c] - p) / step);
                ql       = std::min(std::max(ql, 0.0f), 255.0f);
                while (ql > 0.0f && std::fma(ql, step, p) > lo[c]) ql -= 1.0f;
                float qh = std::ceil((hi[c] - p) / step);
                qh       = std::min(std::max(qh, 0.0f), 255.0f);
                while (qh < 255.0f && std::fma(qh, step, p) < hi[c]) qh += 1.0f;
                if (std::fma(ql, step, p) > lo[c] || std::fma(qh, step, p) < hi[c]) ok = false;
                qlo[c] = (uint8_t)ql;
                qhi[c] = (uint8_t)qh;
            }
            if (ok) {
                ebyte = (uint8_t)(k + 127);
                return;
            }
            if (k >= 127) throw std::runtime_error("wide BVH: cannot quantise child boxes");
        }
    }

    void emit(uint32_t wi, uint32_t bi, int depth)
    {
        out.depth = std::max(out.depth, depth);
        // collapse: open the internal child of largest area until 8 children
        std::vector<uint32_t> kids;
        if (is_leaf(bi)) kids.push_back(bi);
        else { kids.push_back(left(bi)); kids.push_back(right(bi)); }
        while (kids.size() < 8) {
            int   best = -1;
            float ba   = -1.0f;
            for (size_t i = 0; i < kids.size(); ++i)
                if (!is_leaf(kids[i]) && node_area(b.nodes[kids[i]]) > ba) { ba = node_area(b.nodes[kids[i]]); best = (int)i; }
            if (best < 0) break;
            const uint32_t n = kids[(size_t)best];
            kids[(size_t)best] = left(n);
            kids.insert(kids.begin() + best + 1, right(n));
        }
        // Slots by octant: slot s takes the child lying towards (+ on axis a iff bit a of s) from
        // the node's centre, so a ray whose direction has sign bits o (bit a: d_a < 0) meets the
        // children roughly near to far in the order slot ^ o = 0, 1, ... (sp_path.hpp key_mask).
        // Greedy assignment of the largest projection first; inner child in slot s is node
        // child_base + s (slots taken by leaves or empty leave holes).
        const int n = (int)kids.size();
        float     ulo[3], uhi[3], cen[8][3];
        for (int a = 0; a < 3; ++a) { ulo[a] = INFINITY; uhi[a] = -INFINITY; }
        for (int c = 0; c < n; ++c)
            for (int a = 0; a < 3; ++a) {
                ulo[a]    = std::min(ulo[a], b.nodes[kids[(size_t)c]].lo[a]);
                uhi[a]    = std::max(uhi[a], b.nodes[kids[(size_t)c]].hi[a]);
                cen[c][a] = 0.5f * (b.nodes[kids[(size_t)c]].lo[a] + b.nodes[kids[(size_t)c]].hi[a]);
            }
        int  slot_kid[8];
        bool kid_done[8] = {};
        for (int s = 0; s < 8; ++s) slot_kid[s] = -1;
        for (int round = 0; round < n; ++round) {
            int   bc = -1, bs = -1;
            float best = -INFINITY;
            for (int c = 0; c < n; ++c) {
                if (kid_done[c]) continue;
                for (int s = 0; s < 8; ++s) {
                    if (slot_kid[s] >= 0) continue;
                    float score = 0.0f;
                    for (int a = 0; a < 3; ++a) score += ((s >> a) & 1 ? 1.0f : -1.0f) * (cen[c][a] - 0.5f * (ulo[a] + uhi[a]));
                    if (bc < 0 || score > best) { best = score; bc = c; bs = s; } // NaN (empty box): any slot
                }
            }
            slot_kid[bs] = bc;
            kid_done[bc] = true;
        }
        float lo[3][8], hi[3][8];
        for (int s = 0; s < 8; ++s)
            for (int a = 0; a < 3; ++a) {
                const int c = slot_kid[s] >= 0 ? slot_kid[s] : 0; // empty slots: any box (never tested)
                lo[a][s]    = b.nodes[kids[(size_t)c]].lo[a];
                hi[a][s]    = b.nodes[kids[(size_t)c]].hi[a];
            }
        uint8_t q[6][8] = {};
        uint8_t eb[3];
        for (int a = 0; a < 3; ++a) quantise(lo[a], hi[a], 8, ulo[a], uhi[a] - ulo[a], q[a], q[3 + a], eb[a]);
        uint32_t imask = 0;
        int      span  = 0; // child slots allocated: last inner slot + 1
        for (int s = 0; s < 8; ++s)
            if (slot_kid[s] >= 0 && !is_leaf(kids[(size_t)slot_kid[s]])) { imask |= 1u << s; span = s + 1; }
        const uint32_t child_base = (uint32_t)(out.words.size() / 20);
        out.words.resize(out.words.size() + 20 * (size_t)span);
        const uint32_t leaf_base = (uint32_t)out.slot_of.size();
        uint8_t        meta[8]   = {};
        for (int s = 0; s < 8; ++s) {
            if (slot_kid[s] < 0 || ((imask >> s) & 1u)) continue;
            const BvhNode& lf  = b.nodes[kids[(size_t)slot_kid[s]]];
            const uint32_t cnt = lf.b & ~BVH_LEAF;
            const uint32_t off = (uint32_t)out.slot_of.size() - leaf_base;
            if (cnt == 0 || cnt > 7 || off > 31) throw std::runtime_error("wide BVH: leaf does not fit a meta byte");
            meta[s] = (uint8_t)(cnt << 5 | off);
            for (uint32_t j = 0; j < cnt; ++j) out.slot_of.push_back((int32_t)(lf.a + j));
        }
        uint32_t* w = &out.words[(size_t)wi * 20];
        std::memcpy(&w[0], &ulo[0], 4);
        std::memcpy(&w[1], &ulo[1], 4);
        std::memcpy(&w[2], &ulo[2], 4);
        w[3] = (uint32_t)eb[0] | (uint32_t)eb[1] << 8 | (uint32_t)eb[2] << 16 | imask << 24;
        w[4] = child_base;
        w[5] = leaf_base;
        w[6] = (uint32_t)meta[0] | (uint32_t)meta[1] << 8 | (uint32_t)meta[2] << 16 | (uint32_t)meta[3] << 24;
        w[7] = (uint32_t)meta[4] | (uint32_t)meta[5] << 8 | (uint32_t)meta[6] << 16 | (uint32_t)meta[7] << 24;
        for (int r = 0; r < 6; ++r)
            for (int h = 0; h < 2; ++h)
                w[8 + 2 * r + h] = (uint32_t)q[r][4 * h] | (uint32_t)q[r][4 * h + 1] << 8 | (uint32_t)q[r][4 * h + 2] << 16 |
                                   (uint32_t)q[r][4 * h + 3] << 24;
        for (int s = 0; s < 8; ++s)
            if ((imask >> s) & 1u) emit(child_base + (uint32_t)s, kids[(size_t)slot_kid[s]], depth + 1);
    }
};

} // namespace

WideBvh build_wide(const Bvh& bvh)
{
    WideBvh out;
    if (bvh.nodes.empty()) return out;
    out.words.resize(20);
    WideBuilder wb{ bvh, out };
    wb.emit(0, 0, 1);
    if (out.words.size() / 20 >= (1u << 24)) throw std::runtime_error("wide BVH: more than 2^24 nodes");
    if (std::getenv("SP_WIDE_STATS"))
        std::fprintf(stderr, "wide BVH: %zu node records, %zu leaf slots, depth %d\n", out.words.size() / 20, out.slot_of.size(), out.depth);
    return out;
}

} // namespace sph
