// sp_chunk.hpp -- sample-chunked DirectLighting (sp_chunk.hip): host-visible launch interface.
#pragma once
#include "sp_device.hpp"

namespace spd {

struct ChunkArgs {
    const int32_t*      tile_ids;  // caller's tile list (nullptr: slot = tile)
    int64_t             num_tiles;
    int32_t             tiles_x;
    uint32_t            spp;
    uint32_t            chunks;    // sample chunks per pixel
    uint32_t            chunk_len; // samples per chunk (ceil(spp / chunks))
    size_t              n_px;      // num_tiles * 64 pixel slots
    float4*             hits;      // [spp][n_px] {t, code, beta, gamma}; code 0xffffffff = no geometry
    float*              L;         // [spp][3][n_px] per-sample radiance
    uint16_t*           draws;     // [spp][n_px] stream words each sample draws, when the camera pass
                                   // can tell (no image light); nullptr: ck_count replays Light::sample
    uint64_t*           gens;      // [num_tiles][gens_per_px][312][64]: every generation of each pixel's
                                   // mt19937_64 stream, written once by ck_count, read by ck_shade
    uint32_t            gens_per_px;
    uint32_t*           snap_ctl;  // [chunks][n_px] stream position at each chunk start: idx | gen << 16
    int32_t             n_lights;
    int32_t*            counter;   // [2] work queues of ck_count and ck_shade (zeroed by the caller)
    unsigned long long* counters;  // stats: [1] shadow rays, [3] RNG draws
    float*              out;       // tile-packed radiance [n_px][3]
    const int32_t*      slot_map;  // chunk slot -> slot of the caller's list (nullptr: identity); the
                                   // megakernel's tail chunks (sp_mega.hpp) map slot k to order[k]
};

int        chunk_blocks_per_cu(size_t lds_bytes);
hipError_t chunk_render(const Scene& sc, const ChunkArgs& a, int persistent_blocks, int n_cu, hipStream_t stream);
// ck_camera alone (the fused form: sp_capi.hip runs the counts and the shading in the megakernel's
// tail kernel, sp_mega.hpp)
hipError_t chunk_camera(const Scene& sc, const ChunkArgs& a, int n_cu, hipStream_t stream);
// ck_sum alone: image(p) from the per-sample radiance a.L, written at the slots a.slot_map names
hipError_t chunk_sum(const Scene& sc, const ChunkArgs& a, hipStream_t stream);

} // namespace spd
