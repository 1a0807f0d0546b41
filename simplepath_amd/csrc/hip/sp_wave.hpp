// sp_wave.hpp -- arguments and host entry points of the wavefront pipeline (sp_wave.hip).
#pragma once
#include "sp_device.hpp"

#include <hip/hip_runtime.h>

namespace spd {

struct WaveArgs {
    int64_t             n;         // pixel slots in flight = tiles * 64 (array strides)
    int64_t             pb, pe;    // pixel slot range handled by this launch sequence
    int32_t             interleave;// >0: tile block size dealt round-robin to the parts (caller_slot)
    int32_t             n_parts;   // parts the caller's tiles are dealt to (1..WF_MAX_PARTS)
    const int32_t*      tile_ids;  // nullptr => identity
    int32_t             tiles_x;
    uint32_t            spp;
    float*              acc;       // [3][n]
    uint32_t*           rstate;    // [n]
    float4*             hit;       // [n]
    float4*             shp;       // [n]
    float4*             sh;        // [n_lights][n][2]
    uint8_t*            vis;       // [n_lights][n] shadow ray reached the light
    uint32_t*           queue;     // QSEG segments (sp_wave.hip) of shadow-ray pixel slots
    uint32_t*           qcount;    // QSEG segment counters, QSTRIDE words apart
    size_t              qcap;      // entries per queue segment
    uint64_t*           mt_state;  // [n/64][2][312][64]
    unsigned long long* counters;  // [rays, shadow_rays, samples, draws, primary_hits]
    unsigned long long* wstat;     // per-wave statistics slots (wave_stat_bytes)
    int64_t             sh_slot0;  // first wstat slot of this part's shadow waves
    unsigned long long* diag;      // optional per-wave timeline (SP_WAVE_DIAG): 4 u64 per wave
};

constexpr int WF_MAX_LIGHTS = 32; // light mask is one u32 per pixel
constexpr int WF_MAX_PARTS  = 4;  // overlapped parts of the wavefront pipeline (streams)

size_t     wave_bytes_per_pixel(int n_lights);
size_t     wave_stat_bytes(int64_t n);
size_t     wave_queue_bytes(int64_t n, int n_lights);
// ev: optional 3 * spp + 3 events recorded around the launches of part 0 (stage timing);
// aux[0..n_aux): streams of the overlapped parts 1.., fork / join[k] their events,
// shade_done[WF_MAX_PARTS] the shade-alternation events.
hipError_t wave_render(const Scene& sc, const WaveArgs& w, float* out, int traverse_blocks_per_cu, int n_cu,
                       hipStream_t stream, hipEvent_t* ev, const hipStream_t* aux, int n_aux, hipEvent_t fork,
                       const hipEvent_t* join, hipEvent_t* shade_done, int* parts_out);
int        wave_traverse_blocks_per_cu(const Scene& sc);

} // namespace spd
