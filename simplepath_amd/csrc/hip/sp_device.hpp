// sp_device.hpp -- device-resident scene layout and per-lane samplers (gfx950).
//
// Layout in HBM (all arrays allocated once per scene upload, read-only during rendering):
//   nodes/light_nodes : 32-byte binary BVH nodes (sp_host.hpp BvhNode)
//   slot_tri          : per BVH leaf slot, 3 x float4 {p0|code, p1, p2} -- the triangle's three
//                       world-space vertices in leaf order, one 48-byte contiguous read per test
//   slot_code         : per leaf slot, primitive code (kind << 30 | index)
//   normals/indices   : vertex normals and triangle indices, read once per closest hit
//   mt_state          : per persistent wave slot, 2 x 312 x 64 uint64 MT19937-64 words,
//                       [buffer][word][lane] so twists are coalesced 512-byte row accesses
#pragma once
#include "../common/sp_libm.h"
#include "../common/sp_rng.h"
#include "../common/sp_twist4.h"
#include "../../../include/simplepath_hip.h"

namespace spd {

using spm::aff;
using spm::f3;
using spm::lin;
using spm::rgb;

constexpr uint32_t LEAF_BIT   = 0x80000000u;
constexpr uint32_t CODE_SHIFT = 30;
constexpr uint32_t CODE_MASK  = (1u << CODE_SHIFT) - 1u;
constexpr uint32_t AXIS_SHIFT = 30;                      // sp_host.hpp BVH_AXIS_SHIFT
constexpr uint32_t CHILD_MASK = (1u << AXIS_SHIFT) - 1u;

struct Node {
    float    lo[3];
    uint32_t a;
    float    hi[3];
    uint32_t b;
};

struct Shape { // sphere / plane
    aff      o2w, w2o;
    lin      nrm; // normal_to_world
    int32_t  material, kind;
};

struct Light {
    int32_t kind, image; // image: index into Scene::envs for SP_LIGHT_IMAGE_ENVIRONMENT
    rgb     radiance;
    aff     o2w, w2o;
    lin     nrm;
};

// ImageBasedEnvironmentLight (Lights/Light.h:196) after its constructor: clamped radiance image
// and the Distribution2D tables (sp_host.hpp EnvMap), read with per-lane binary searches.
struct EnvMap {
    lin             l2w, w2l;
    int32_t         w, h, nu, nv;
    const float4*   radiance;  // w * h, {r, g, b, 0}
    const float*    cond_func; // nv * nu
    const float*    cond_cdf;  // nv * (nu + 1)
    const float*    cond_int;  // nv
    const float*    marg_func; // nv
    const float*    marg_cdf;  // nv + 1
    float           marg_int;
    const uint32_t* cond_guide; // nv x (2^cond_bits + 1); nullptr: exact upper_bound replay
    const uint32_t* marg_guide; // 2^marg_bits + 1
    int32_t         cond_bits, marg_bits;
};

struct Material {
    int32_t kind, base;
    rgb     lambert_albedo;
    rgb     microfacet_r;
    float   alpha_x, alpha_y, microfacet_ior;
    int32_t sample_visible_area;
    float   coat_ior;
    rgb     coat_color;
};

struct Scene {
    aff   camera;
    int   width, height, max_depth, rr_depth;
    float alpha2_0, alpha2_1;

    // geometry: Scene::m_accelerator_geometry = ListAccelerator{unbounded..., BVH}
    int             n_unbounded;
    const int32_t*  unbounded; // shape indices (planes), reference partition order
    int             n_nodes;
    const Node*     nodes;
    const uint4*    wnodes;    // 8-wide BVH (sp_host.hpp WideBvh), 5 per node; nullptr = binary walk
    const float4*   wslot_tri; // 3 per wide-BVH primitive slot
    const float4*   slot_tri;  // 3 per slot
    const uint32_t* slot_code;
    const float*    normals;   // 3 per vertex
    const uint32_t* indices;   // 3 per triangle
    const int32_t*  tri_material;
    const Shape*    shapes;

    // lights: Scene::m_lights order + m_accelerator_lights
    int             n_lights;
    const Light*    lights;
    int             n_unbounded_lights;
    const int32_t*  unbounded_lights;
    int             n_light_nodes;
    const Node*     light_nodes;
    const uint32_t* light_slot; // slot -> light index
    const EnvMap*   envs;       // image environment lights (Light::image)

    const Material* materials;

    const uint32_t* rsqrt_entries; // 2 << rsqrt_bits entries; 16-bit when rsqrt_shift > 0 (sp_math.h)
    int32_t         rsqrt_bits;
    uint32_t        rsqrt_zero, rsqrt_denorm;
    int32_t         rsqrt_shift;
    uint32_t        rsqrt_hi;
    int             stack_depth;   // LDS traversal stack entries per lane (0 when stackless)
    int             stack_words;   // LDS words per lane
    // any-hit-only kernels (wf_shadow): their walks need max(wide or binary depth, light depth) + 1
    // stack entries, usually far fewer than stack_words (which covers the binary closest-hit walk)
    int             any_stack_words;
    int             ordered;       // 1: SAH BVH -- visit the near child (split axis, ray sign) first
    int             wide_closest;  // 1: closest-hit queries walk the 8-wide BVH too (stack: 2 words per level)
    // BVHs too deep for the LDS stack budget: binary walks climb parent links instead of popping
    // a stack (same visiting order and box tests; sp_path.hpp bvh_next)
    int             stackless;
    // IterativeRRNEE: a bounce's MIS-ray and next closest-hit BVH walks dealt over the wave
    // (sp_path.hpp mq_run; needs wide_closest and the stack).  Set per render: 1 unless
    // SP_RENDER_PER_LANE_QUERIES asks for the per-lane walks (the comparison).
    int             merge_queries;
    const uint32_t* parents;       // parent of each geometry node (root: itself)
    const uint32_t* light_parents; // parent of each light-BVH node
};
// 32-bit words of the RSQRTSS table (the LDS copy every shading kernel makes)
// RSQRTSS table words on the device: an 8-word header {bits, zero, denorm, shift, hi, 0, 0, 0}
// then the entries (16-bit packed when shift > 0).  Kernels copy all of it to LDS and read the
// parameters from the header where they are used (sp_path.hpp rsqrt_ref): held in SGPRs they were
// spilled to VGPR lanes and read back with v_readlane in every sample of the rho loop (elf
// 1024^2 @ 16 spp 571-586 -> 600-603 Mrays/s, bunny +1 %, profiles/r03).
constexpr int RSQ_HDR = 8;

// Device layout of the std::mt19937_64 states (main.cpp:73: one per pixel; 312 words per
// generation).  A wave slot holds 64 lanes' states; word k of lane l of one generation buffer is at
// (k / MT_BLK) * 64 * MT_BLK + l * MT_BLK + k % MT_BLK: each lane's MT_BLK consecutive words share
// one 128-byte line.  A lane draws its words in order, and the served estimates of IterativeRRNEE
// read 32 consecutive words of another lane's stream, while the lanes' stream positions drift
// apart after the first sample; with the words interleaved by lane (MT_BLK = 1, rounds 1-3) every
// draw touched its own line -- elf's 8-way shard fetched 39.7 TB per frame for ~7 TB of state
// reads (profiles/r04/traffic).  A twist (all lanes, word by word) now reuses each lane's line
// for MT_BLK consecutive words from L1/L2.  Buffers are padded to whole blocks.
#ifndef SP_MT_BLK
#define SP_MT_BLK 4
#endif
// Everything that depends on the block size -- this layout, and all of sp_path.hpp / the megakernel
// body built on it -- lives in an inline namespace named after it (spd::mt_blk4, spd::mt_blk1), so
// the sample-chunk TU (MT_BLK 1) and the others (4) never define one inline function two ways (the
// one-definition rule holds even with -fgpu-rdc or a host caller).  The host-visible launch
// interfaces (sp_mega.hpp, sp_chunk.hpp, sp_wave.hpp) and the shared records stay in spd.
#define SPD_CAT2_(a, b) a##b
#define SPD_CAT_(a, b) SPD_CAT2_(a, b)
#define SPD_LAYOUT_NS SPD_CAT_(mt_blk, SP_MT_BLK)
inline namespace SPD_LAYOUT_NS {
constexpr int MT_BLK       = SP_MT_BLK;
// no padding: every translation unit sizes a generation buffer the same (the sample-chunk TU keeps
// its own block size for its generator store, sp_chunk.hip)
static_assert(spm::MT_N % MT_BLK == 0, "MT_BLK must divide 312");
constexpr int MT_ROWS      = (spm::MT_N + MT_BLK - 1) / MT_BLK;
constexpr int MT_GEN_WORDS = MT_ROWS * MT_BLK * 64; // words of one generation buffer of a wave slot
__host__ __device__ inline size_t mt_off(int k) { return (size_t)(k / MT_BLK) * (64 * MT_BLK) + (size_t)(k % MT_BLK); }
} // inline namespace SPD_LAYOUT_NS
__host__ __device__ inline int rsqrt_words(const Scene& sc) { return RSQ_HDR + (sc.rsqrt_shift ? (1 << sc.rsqrt_bits) : (2 << sc.rsqrt_bits)); }


// Tail chunks of the DirectLighting megakernel (sp_mega.hpp tail_prep / tail_chunk): the K most
// expensive tiles of the tile order (order[0 .. K)) are rendered as sample chunks at the END of the
// persistent queue, so the frame's last work items are a few samples of one tile instead of whole
// tiles.  Queue: items [0, K) prepare those tiles (camera rays, draw counts, every generation of
// each pixel's stream into a store), items [K, num_tiles) are the other tiles as before, items
// [num_tiles, num_tiles + K * chunks) shade one chunk each; sp_chunk.hip chunk_sum adds each pixel's
// samples in order afterwards.  n_prep == 0: no tail chunks.
struct TailArgs {
    int64_t   n_prep;      // K
    int64_t   n_items;     // K * chunks
    uint32_t  chunks, chunk_len, gens_per_px;
    size_t    n_px;        // K * 64 pixel slots (chunk slot k = queue item k)
    float4*   hits;        // [spp][n_px] camera hit {t, code, beta, gamma}; code 0xffffffff = none
    float*    L;           // [spp][3][n_px] per-sample radiance
    uint64_t* gens;        // [K][gens_per_px] generation buffers (mt_off layout), generation g in buffer g
    uint32_t* snap_ctl;    // [chunks][n_px] stream position at each chunk start: idx | gen << 16
    uint32_t* ready;       // [K] 1 once tile k's prep item has published its store (zeroed per render)
    // The sample-chunk pipeline's fused form (sp_fused_kernel, sp_capi.hip): ck_camera has
    // stored the hit records, light-only radiance and each sample's draw count, so a prep item only
    // turns the counts into chunk starts and twists the store; every tile is cut (K = num_tiles, no
    // whole tiles), and the preps run interleaved with the chunks (tail_front).
    const uint16_t* draws; // [spp][n_px] draw counts; nullptr: the prep item traces the camera rays
    // sp_tail_kernel<4, true> (an image light): a sample's draw count depends on the drawn numbers
    // (Light::sample's usability), so the prep item replays each sample's Light::sample draws on the
    // stream itself (sp_chunk.hip ck_count's replay), twisting the store generation by generation
    int32_t         replay;
    // sp_fused_kernel with the camera pass in its queue (n_cam > 0): items [0, n_cam) trace the
    // camera rays of samples [b cam_block, (b + 1) cam_block) of one slot, tile-major, and count them
    // into cam_done[slot]; a slot's prep waits for spp.  n_cam 0: ck_camera ran before the kernel.
    int64_t         n_cam;
    uint32_t        cam_block;
    uint32_t*       cam_done;  // [K], zeroed per render
    uint16_t*       draws_out; // [spp][n_px] the camera items' draw counts (= draws)
};

struct RenderArgs {
    float*          out;        // tile-packed radiance
    const int32_t*  tile_ids;   // nullptr => identity
    int64_t         num_tiles;
    int32_t         tiles_x;
    uint32_t        spp;
    int32_t         integrator;
    int32_t*        tile_counter;
    uint64_t*       mt_state;
    unsigned long long* counters; // [rays, shadow_rays, samples, draws]
    float*          deep;       // recursive integrators, max_depth > 32: per-lane level records
    size_t          deep_stride;// lanes of the launch (= blocks * 256)
    unsigned long long* tile_diag; // SP_TILE_DIAG: per slot {t0, t1 (s_memrealtime), wave, item, 4 stage clocks}
    const int32_t*  order;      // queue position -> tile slot (nullptr: slot order); sp_mega.hip tile_order
    float*          tile_time;  // probe pass: per slot, the wave's time for the tile; no radiance written
    // sp_tail_kernel only: the queue's prep and chunk item counts, and the rest of TailArgs in
    // device memory (read per item: kernel arguments held across the persistent loop cost SGPRs)
    int64_t         tail_prep, tail_items;
    // sp_tail_kernel: queue [prep 0..K) [whole tiles K..num_tiles) [chunks]; sp_fused_kernel (all
    // tiles cut, K = num_tiles): [prep 0..P) then per tile g its chunks followed by prep g + P,
    // P = tail_front -- the memory-bound preps run beside the compute-bound chunks, each P tiles
    // ahead of its own chunks
    int64_t         tail_front;
    int64_t         tail_cam;   // sp_fused_kernel: camera items ahead of the preps (TailArgs::n_cam)
    const TailArgs* tail;
    int32_t         probe_step; // sp_probe_kernel: times every probe_step-th slot (the order kernel fills the rest)
};

} // namespace spd
