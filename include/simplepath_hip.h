/*
 * simplepath_hip.h -- C-ABI boundary of the MI355X-native SimplePath renderer.
 *
 * This is the drop-in boundary for the reference's per-pixel integration hot path
 * (kjeffery/SimplePath, main.cpp:77-107 `render_thread` driving
 * Integrators/Integrator.h:37 `Integrator::integrate` over
 * base/TileScheduler.h:29 `TileScheduler::get_next_tile`).  Every entry point takes
 * plain pointers and sizes; no C++ or torch types cross it.
 *
 * Entry points and the reference interface each one replaces:
 *
 *   sp_scene_load / sp_scene_load_string  base/FileParser.cpp:929 `sp::parse_file`
 *                                         + base/Scene.h:59 `Scene::Scene` (accelerators)
 *   sp_scene_from_desc                    base/Scene.h:59 `Scene::Scene` from an already-built
 *                                         scene (main.cpp:368-395 holds one)
 *   sp_scene_get_info                     base/Scene.h:90-96 (image_width, image_height,
 *                                         russian_roulette_depth, max_depth, integrator_type)
 *   sp_scene_get_desc                     the primitive / light / material / camera state
 *                                         held by base/Scene.h:99-105 (flattened, host memory)
 *   sp_scene_upload / sp_scene_upload_ex  (no reference counterpart: HBM residency; the
 *                                         Scene ctor's accelerator build, base/Scene.h:59)
 *   sp_scene_bvh_build_info               base/Scene.h:59 Scene ctor's BVHAccelerator build
 *                                         (shapes/BVHAccelerator.h:173), host only: statistics
 *   sp_render_tiles                       main.cpp:77-107 `render_thread`: for each scheduled
 *                                         tile, for each pixel, num_pixel_samples x
 *                                         `integrator.integrate(camera.generate_ray(...))`,
 *                                         averaged -- executed by HIP kernels on the device
 *   sp_tiles_to_image                     main.cpp:100-102 `image(p.x, p.y) += ... /= spp`
 *                                         scatter of tile-packed radiance into the Image
 *   sp_tile_count                         base/TileScheduler.h:38-48 `get_num_tiles`
 *   sp_tile_origin                        base/TileScheduler.h:72-86 ColumnMajor tile order
 *   sp_string_to_integrator               Integrators/Integrator.cpp:25 `string_to_integrator_type`
 *
 * Error behaviour: every function returns SP_OK (0) or a negative SP_ERR_* code and
 * records a message retrievable with sp_last_error() (thread-local), mirroring the
 * reference's exceptions (ParsingException, std::runtime_error("Unknown integrator type")).
 */
#ifndef SIMPLEPATH_HIP_H
#define SIMPLEPATH_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SP_ABI_VERSION 6

/* ---- status codes ------------------------------------------------------------- */
enum {
    SP_OK               = 0,
    SP_ERR_PARSE        = -1, /* sp::ParsingException                                 */
    SP_ERR_IO           = -2, /* unable to open file                                  */
    SP_ERR_ARG          = -3, /* invalid argument                                     */
    SP_ERR_HIP          = -4, /* HIP runtime failure / no device                      */
    SP_ERR_UNSUPPORTED  = -5, /* feature present in the reference but not on this path */
    SP_ERR_STATE        = -6  /* call order violated (e.g. render before upload)      */
};

/* ---- integrators: Integrators/Integrator.h:18 IntegratorType ---------------------- */
enum {
    SP_INTEGRATOR_NOT_SPECIFIED          = 0,
    SP_INTEGRATOR_MANDELBROT             = 1,
    SP_INTEGRATOR_BRUTE_FORCE            = 2,
    SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE  = 3,
    SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR = 4,
    SP_INTEGRATOR_ITERATIVE_RRNEE        = 5,
    SP_INTEGRATOR_DIRECT_LIGHTING        = 6,
    SP_INTEGRATOR_WHITTED                = 7
};

/* ---- flattened scene (host memory, owned by the sp_scene) ------------------------- */

/* AffineSpace (math/AffineSpace.h:12): three columns + translation. */
typedef struct sp_affine {
    float vx[3], vy[3], vz[3], p[3];
} sp_affine;

/* LinearSpace3x3 (math/LinearSpace3x3.h:13): three columns. */
typedef struct sp_linear {
    float vx[3], vy[3], vz[3];
} sp_linear;

/* Material kinds produced by base/FileParser.cpp (materials/Material.h:808-829). */
enum {
    SP_MAT_LAMBERTIAN = 0, /* OneSampleMaterial{ LambertianBRDF }                             */
    SP_MAT_GLOSSY     = 1, /* OneSampleMaterial{ MicrofacetReflection(Beckmann), LambertianBRDF } */
    SP_MAT_CLEARCOAT  = 2  /* ClearcoatMaterial{ base }                                       */
};

typedef struct sp_material_desc {
    int32_t kind;
    int32_t base;               /* clearcoat: index of base material, else -1                 */
    float   lambert_albedo[3];  /* LambertianBRDF::m_albedo == albedo / pi (Material.h:317)   */
    float   microfacet_r[3];    /* MicrofacetReflection::m_r (white)                          */
    float   alpha_x, alpha_y;   /* BeckmannDistribution alphas (roughness_to_alpha, Material.h:231) */
    float   microfacet_ior;     /* MicrofacetReflection::m_ior                                */
    int32_t sample_visible_area;/* MicrofacetDistribution::m_sample_visible_area              */
    float   coat_ior;           /* ClearcoatMaterial::m_ior                                    */
    float   coat_color[3];      /* ClearcoatMaterial::m_specular_color                         */
} sp_material_desc;

/* Primitive kinds in Scene::m_accelerator_geometry order. */
enum { SP_PRIM_TRIANGLE = 0, SP_PRIM_SPHERE = 1, SP_PRIM_PLANE = 2 };

/* Sphere / Plane (shapes/Shape.h:42 TransformableShape). normal_to_world is
 * object_to_world.linear.inverse().transposed() -- what LinearSpace3x3::operator()(Normal3)
 * (math/LinearSpace3x3.h:163) recomputes on every call; here computed once with the same
 * arithmetic. */
typedef struct sp_xform_shape {
    sp_affine object_to_world;
    sp_affine world_to_object;
    sp_linear normal_to_world;
    int32_t   material;
    int32_t   kind; /* SP_PRIM_SPHERE or SP_PRIM_PLANE */
} sp_xform_shape;

/* Light kinds (Lights/Light.h). */
enum { SP_LIGHT_SPHERE = 0, SP_LIGHT_ENVIRONMENT = 1, SP_LIGHT_IMAGE_ENVIRONMENT = 2 };

typedef struct sp_light_desc {
    int32_t   kind;
    int32_t   image;           /* SP_LIGHT_IMAGE_ENVIRONMENT: index into sp_scene_desc.env_images, else -1 */
    float     radiance[3];
    sp_affine object_to_world; /* sphere light */
    sp_affine world_to_object;
    sp_linear normal_to_world;
} sp_light_desc;

/* Image-based environment light (Lights/Light.h:196 ImageBasedEnvironmentLight) as the parser
 * hands it to the light's constructor (base/FileParser.cpp:366-368): the PFM image (Image/
 * Image.cpp:78 read_pfm) already multiplied by `radiance`, before the constructor's
 * modify_image / create_distribution (those run at sp_scene_upload, and in the oracle). */
typedef struct sp_env_image {
    int32_t      width, height;
    const float* pixels;          /* img(x, y) = pixels[(y * width + x) * 3 + c]              */
    float        max_radiance;    /* std::numeric_limits<float>::max() when not given          */
    int32_t      reserved;
    sp_linear    light_to_world;  /* LinearTransformation: rotate/scale attributes             */
    sp_linear    world_to_light;  /* its inverse (Transformation::get_inverse)                  */
} sp_env_image;

/* PerspectiveCamera (Cameras/Camera.h:85): the transform built by create_transform. */
typedef struct sp_camera_desc {
    sp_affine transform;
    int32_t   film_width, film_height;
} sp_camera_desc;

typedef struct sp_scene_info {
    int32_t image_width, image_height;
    int32_t russian_roulette_depth, max_depth;
    int32_t integrator_type; /* SP_INTEGRATOR_* as parsed (0 = not specified)          */
    int32_t num_triangles, num_vertices, num_shapes, num_lights, num_materials;
    char    output_file_name[256];
} sp_scene_info;

typedef struct sp_scene_desc {
    sp_scene_info          info;
    sp_camera_desc         camera;
    /* mesh data: world-space (Mesh ctor pre-transforms, shapes/Triangle.h:25) */
    const float*           vertices;   /* num_vertices * 3                                   */
    const float*           normals;    /* num_vertices * 3 (transformed, not re-normalized)  */
    const uint32_t*        indices;    /* num_triangles * 3                                  */
    const int32_t*         tri_material;/* num_triangles                                     */
    const sp_xform_shape*  shapes;     /* num_shapes (spheres, planes)                       */
    /* Scene::m_geometry order before partitioning: (kind, index) pairs. kind = SP_PRIM_*;
     * index into triangles or shapes. */
    const int32_t*         prim_kind;
    const int32_t*         prim_index;
    int64_t                num_prims;
    const sp_light_desc*   lights;     /* Scene::m_lights order                              */
    const sp_material_desc* materials;
    const sp_env_image*    env_images; /* referenced by sp_light_desc.image (ABI 2)          */
    int32_t                num_env_images;
    int32_t                reserved;
} sp_scene_desc;

/* ---- render ------------------------------------------------------------------------ */

/* Zero-initialise (`sp_render_params p = {0};`): every field added in a later ABI means
 * "automatic" at 0.  Stream order: with stats == NULL, no SP_RENDER_STAGE_TIMING flag and the
 * tile list on the device (d_tile_ids) or absent, sp_render_tiles only enqueues work on `stream`
 * and returns -- two calls and a dependent kernel can be queued back to back with no host wait.
 * Requesting stats waits for the render (the counters are read back).  Calls on one scene share
 * its device scratch; they may come from several host threads and streams (the reference's
 * render() shares one Scene across threads, main.cpp:122-130): the scene serialises them, on the
 * host with a per-scene lock and on the device by making each call's stream wait for the previous
 * call's work (ABI 5).  A host tile list is copied before the call returns. */
typedef struct sp_render_params {
    int32_t        integrator;        /* SP_INTEGRATOR_*; 0 => scene's (DirectLighting if unset: main.cpp:387-392) */
    uint32_t       samples_per_pixel; /* main.cpp `--samples`                                    */
    const int32_t* tile_ids;          /* host array of tile indices (ColumnMajor order); NULL => d_tile_ids or all tiles */
    int64_t        num_tiles;         /* length of tile_ids / d_tile_ids (ignored when both are NULL) */
    void*          stream;            /* hipStream_t, NULL = default stream                      */
    int32_t        bvh_mode;          /* unused: the BVH is chosen at upload (kept for layout)     */
    int32_t        flags;             /* SP_PIPELINE_* (0 = automatic) | SP_RENDER_STAGE_TIMING   */
    /* ---- ABI 4 ---- */
    const int32_t* d_tile_ids;        /* DEVICE array of num_tiles tile indices, used when tile_ids is
                                         NULL: not copied or checked on the host (an id outside
                                         [0, tiles) -- negative ones included -- renders as zeros) */
    int32_t        waves_per_simd;    /* megakernel occupancy (__launch_bounds__ variant): 0 = automatic
                                         (DirectLighting 4, IterativeRRNEE 3, fewer if the LDS caps it);
                                         else DirectLighting 1-4, IterativeRRNEE 2-4               */
    int32_t        chunks_per_pixel;  /* sample-chunk pipeline: 0 = automatic (~120K (tile, chunk) items),
                                         else 1..samples_per_pixel                                 */
    float          chunk_max_gb;      /* sample-chunk buffer budget in GB: 0 = 96, never more than the
                                         device's free memory; AUTO falls back to the megakernel when
                                         the buffers do not fit                                    */
    /* ---- ABI 5 ---- */
    float          tile_order_factor; /* megakernel tile order (DirectLighting, IterativeRRNEE): 0 =
                                         automatic (a one-sample probe times every tile; tiles
                                         slower than 2x the mean go first, then 24 cost classes a
                                         quarter octave apart; from 6 tiles per wave and 128 spp --
                                         2.5 with tail chunks (ABI 6) --, IterativeRRNEE from 4 tiles
                                         per wave and 16 spp);
                                         > 0: with this factor whenever it can apply; < 0: queue
                                         order.  It cannot apply, and the frame renders in queue
                                         order whatever the factor, when the megakernel does not
                                         run (wavefront, sample chunks), when n_tiles is at most
                                         the persistent waves (each wave takes one tile), or for
                                         an integrator without a probe kernel (BruteForce*,
                                         Whitted, Mandelbrot).  A tile's estimate is its probe time
                                         blended with its queue neighbours' for a whole frame (the
                                         tiles left, right, above and below) or a host list with a
                                         constant stride k (a rank's interleaved shard: the tiles k
                                         columns left and right, and the tile below when k divides
                                         the tile columns); any other list uses each tile's own
                                         probe time.                                                  */
    /* ---- ABI 6 ---- */
    float          tail_fraction;     /* megakernel tail chunks (DirectLighting at 4 waves per SIMD, or
                                         3 without an image light, with the tile order):
                                         the most expensive tail_fraction x n_tiles tiles of the
                                         order are rendered as sample chunks at the end of the
                                         persistent queue, so the frame ends on short work items
                                         (identical image and counts).  0 = automatic: where it
                                         applies, waves / n_tiles clamped to [0.12, 0.4] (and AUTO
                                         then picks the megakernel with the order from 2.5 tiles per
                                         persistent wave and 128 spp -- the 2- and 3-GPU shards of a
                                         1080p frame -- or 4 tiles per wave and 64 spp);
                                         < 0 off, else (0, 1].                                      */
    int32_t        reserved;          /* must be 0                                                  */
} sp_render_params;

/* Device pipeline selection (sp_render_params.flags).  All produce identical images. */
enum {
    SP_PIPELINE_AUTO       = 0, /* by work size: megakernel, or sample chunks for DirectLighting
                                   below 24000 tiles when their buffers fit     */
    SP_PIPELINE_MEGAKERNEL = 1, /* one lane owns one pixel for all samples (sp_mega.hpp)        */
    SP_PIPELINE_WAVEFRONT  = 2, /* DirectLighting: per-sample primary/shade/shadow kernels with
                                   ballot/prefix-sum shadow-ray compaction (sp_wave.hip)         */
    SP_PIPELINE_SAMPLE_CHUNKS = 3, /* DirectLighting: each pixel's samples in parallel chunks
                                      (stream state snapshots; sp_chunk.hip)                      */
    SP_RENDER_STAGE_TIMING = 4, /* flag: HIP events between launches fill sp_render_stats.stage_ms
                                   (waits for the render)                                          */
    SP_RENDER_PER_LANE_QUERIES = 8 /* flag (ABI 5): IterativeRRNEE walks each ray on its own lane
                                   instead of dealing a bounce's MIS and next closest-hit walks
                                   over the wave (identical images; the comparison path)           */
};

/* Accelerator options of sp_scene_upload_ex (ABI 4).  Zero-initialise: 0 = automatic. */
enum { SP_WALK_AUTO = 0, SP_WALK_STACKLESS = 1 };
typedef struct sp_upload_params {
    int32_t bvh_mode;         /* 0 = SAH (fast), 1 = reference median-split order (tie-exact)       */
    int32_t walk;             /* SP_WALK_AUTO: per-wave LDS stack unless the BVH is deeper than
                                 stack_max_levels; SP_WALK_STACKLESS: parent links always         */
    int32_t stack_max_levels; /* 0 = 96                                                            */
    int32_t no_wide_bvh;      /* 1: all queries walk the binary BVH instead of the 8-wide one       */
    int32_t env_replay;       /* 1: image-light CDF lookups replay libstdc++ upper_bound step by step
                                 instead of the guide tables (identical results)                    */
    int32_t sah_leaf;         /* SAH leaf size 1-4: 0 = 4                                          */
    int32_t binary_closest;   /* 1: closest-hit queries keep the binary near-first walk (any-hit
                                 queries stay on the 8-wide BVH)                                    */
    int32_t reserved;         /* must be 0                                                          */
} sp_upload_params;

typedef struct sp_render_stats {
    uint64_t rays;            /* every ray cast: camera/extension + shadow + MIS rays            */
    uint64_t shadow_rays;     /* intersect_p queries                                              */
    uint64_t samples;         /* pixel samples (paths)                                            */
    uint64_t rng_draws;       /* IncoherentSampler draws                                          */
    float    kernel_ms;       /* HIP-event time of the render kernel(s)                           */
    int32_t  pipeline;        /* SP_PIPELINE_* that ran                                           */
    int32_t  launches;        /* kernel launches issued                                           */
    uint64_t primary_hits;    /* wavefront: camera rays that hit geometry (shading work items)     */
    float    stage_ms[4];     /* with SP_RENDER_STAGE_TIMING, wavefront: [init+resolve, primary,   */
                              /* shade, shadow] of part 0 summed over launches; megakernel: [0]   */
                              /* the render kernel, [1] the tile-order probe + partition           */
    int32_t  parts;           /* wavefront: concurrent parts (streams); part 0 holds ceil(tiles/2) */
    int32_t  stack_depth;     /* traversal-stack entries per lane the BVH walks needed (ABI 3)      */
    int32_t  tail_tiles;      /* megakernel: tiles rendered as tail chunks (ABI 6; 0: none)         */
    int32_t  tail_chunks;     /* ... and sample chunks per such tile                                */
} sp_render_stats;

/* BVH statistics (sp_scene_bvh_build_info).  depth = levels below the root of the binary BVH
 * (the reference's recursive BVHAccelerator walk, shapes/BVHAccelerator.h:62-77, nests this deep);
 * wide_depth = depth of the 8-wide any-hit BVH (SAH only, else 0); light_depth = the light
 * accelerator's; stack_depth = traversal-stack entries per lane a render needs. */
typedef struct sp_bvh_info {
    int32_t depth, wide_depth, light_depth, stack_depth;
    int64_t nodes, slots;
} sp_bvh_info;

/* ---- API ------------------------------------------------------------------------------ */
typedef struct sp_scene sp_scene;

const char* sp_version(void);
/* ABI 5: content hash (16 hex digits) of the sources, headers and flags the library was built from. */
const char* sp_build_id(void);
const char* sp_last_error(void);

int  sp_string_to_integrator(const char* name, int32_t* out);

int  sp_scene_load(const char* path, sp_scene** out);
int  sp_scene_load_string(const char* text, const char* base_dir, sp_scene** out);
/* Build a scene from a caller's flattened scene (a host that already parsed its scene, e.g.
 * the reference's main.cpp:368-395 sp::Scene): every array is copied and validated; nothing is
 * re-parsed.  Layout as sp_scene_get_desc returns it (world-space mesh, Scene::m_geometry order,
 * camera transform for film_width x film_height).  sp_scene_set_resolution can then not change
 * the image size (the camera transform fixes it). */
int  sp_scene_from_desc(const sp_scene_desc* desc, sp_scene** out);
void sp_scene_free(sp_scene* scene);
int  sp_scene_get_info(const sp_scene* scene, sp_scene_info* out);
/* Arrays in *out are owned by the scene: valid until sp_scene_free or sp_scene_set_resolution. */
int  sp_scene_get_desc(const sp_scene* scene, sp_scene_desc* out);
/* Override image size after load (camera rebuilt as FileParser would with these values). */
int  sp_scene_set_resolution(sp_scene* scene, int32_t width, int32_t height);

int  sp_tile_count(int32_t width, int32_t height, int64_t* out);
int  sp_tile_origin(int32_t width, int32_t height, int64_t tile, int32_t* x0, int32_t* y0);

/* Device side. */
int  sp_device_count(int32_t* out);
int  sp_scene_upload(sp_scene* scene, int32_t device, int32_t bvh_mode);
/* sp_scene_upload with explicit accelerator options (NULL = all automatic with bvh_mode 0).  A
 * scene already resident on `device` with the same effective options is not re-uploaded.  The
 * SP_STACKLESS / SP_STACK_MAX / SP_WIDE / SP_ENV_GUIDE / SP_SAH_LEAF environment variables
 * override fields left automatic (test hooks). */
int  sp_scene_upload_ex(sp_scene* scene, int32_t device, const sp_upload_params* params);
/* Render tiles into a DEVICE buffer laid out tile-packed: out[(slot*64 + morton)*3 + c],
 * slot = position of the tile in params->tile_ids (or the tile index itself when NULL).
 * Pixels of clipped border tiles that fall outside the image are written as 0. */
int  sp_render_tiles(sp_scene* scene, const sp_render_params* params, float* d_out,
                     sp_render_stats* stats);
/* Same as sp_render_tiles but allocates the device buffer itself and copies the tile-packed
 * radiance back into h_out (num_tiles * 64 * 3 floats). */
int  sp_render_tiles_host(sp_scene* scene, const sp_render_params* params, float* h_out,
                          sp_render_stats* stats);
/* BVH statistics of the uploaded scene (depth, node count, primitive slots). */
int  sp_scene_bvh_info(const sp_scene* scene, int32_t* depth, int64_t* nodes, int64_t* slots);
/* ABI 5: bytes the uploaded scene occupies in HBM (BVHs, primitive records, normals, materials,
 * lights, image-light tables, RSQRTSS table) -- what a frame streams at least once. */
int  sp_scene_device_bytes(const sp_scene* scene, int64_t* bytes);
/* Host only (no device needed): build the geometry BVH sp_scene_upload would build for bvh_mode
 * and report its statistics; nothing is uploaded. */
int  sp_scene_bvh_build_info(const sp_scene* scene, int32_t bvh_mode, sp_bvh_info* out);
/* Scatter tile-packed radiance (host memory) into a row-major width x height x 3 image. */
int  sp_tiles_to_image(int32_t width, int32_t height, const int32_t* tile_ids, int64_t num_tiles,
                       const float* tiles, float* image);
/* Write an image as PFM exactly as Image/Image.cpp:40 write_pfm does. */
int  sp_write_pfm(const char* path, int32_t width, int32_t height, const float* image);

/* RSQRTSS emulation table.  The reference normalises with RSQRTSS + one Newton step
 * (math/Math.h:205); RSQRTSS is a hardware table whose outputs differ between CPU vendors, so the
 * reference's images are those of the CPU it ran on.  By default scenes are built (host) and
 * rendered (device) with the table of this host's CPU, captured at start-up.  sp_rsqrt_table_set
 * installs another CPU's table -- e.g. the one recorded with a golden image made elsewhere -- for
 * every scene loaded and uploaded afterwards (entries == NULL: back to this host's table).
 * entries holds 2 << bits words: [exponent parity][leading mantissa bits]. */
int  sp_rsqrt_table_get(uint32_t* entries, int64_t capacity, int32_t* bits, uint32_t* zero_result,
                        uint32_t* denorm_result);
int  sp_rsqrt_table_set(const uint32_t* entries, int32_t bits, uint32_t zero_result, uint32_t denorm_result);

/* Numerics self-checks used by the tests (no GPU needed). */
int  sp_rsqrt_table_info(int32_t* mantissa_bits, int32_t* verified);
float sp_host_rsqrt_emulated(float x); /* table emulation of RSQRTSS, host-evaluated */

#ifdef __cplusplus
}
#endif
#endif /* SIMPLEPATH_HIP_H */
