// sp_host.hpp -- host-side scene model of the MI355X SimplePath renderer.
//
// Mirrors what the reference's FileParser (base/FileParser.cpp) and Scene (base/Scene.h) build,
// flattened into arrays that can be copied to HBM.  All transforms, mesh vertices/normals,
// material constants and camera vectors are computed on the host with the reference's own
// arithmetic (sp_math.h helpers + the host CPU's RSQRTSS + glibc libm) so the device sees the
// exact same bits the reference would hold in memory.
#pragma once

#include "../common/sp_math.h"
#include "../../../include/simplepath_hip.h"

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace sph {

using spm::aff;
using spm::f3;
using spm::lin;
using spm::rgb;

struct SpError : std::runtime_error {
    int code;
    SpError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// ---- host versions of the reference's vector ops that need RSQRTSS ----------------------------
// RSQRTSS of the host CPU, or -- after sp_rsqrt_table_set -- of the CPU whose table was given
// (sp_rsqrt.cpp), so a scene is built exactly as the reference built it on that CPU.
float rsqrtss_active(float a);
inline float host_rsqrt(float a) { return spm::rsqrt_newton(a, rsqrtss_active(a)); }
inline f3 host_normalize(f3 a) { return spm::scale(a, host_rsqrt(spm::dot(a, a))); }

// Transformation<T> (math/Transformation.h:37): forward and inverse kept side by side.
struct AffXf {
    aff fwd, inv;
};

aff  aff_identity();
lin  lin_identity();
aff  aff_mul(const aff& a, const aff& b);  // AffineSpace * AffineSpace
aff  aff_mul_lin(const aff& a, const lin& b);  // AffineSpace * LinearSpace3x3
aff  lin_mul_aff(const lin& a, const aff& b);  // LinearSpace3x3 * AffineSpace
lin  lin_mul(const lin& a, const lin& b);
lin  lin_inverse(const lin& a);            // adjoint() / determinant()
lin  lin_transposed(const lin& a);
lin  normal_matrix(const aff& m);          // m.linear.inverse().transposed()
f3   xfm_normal(const lin& nm, f3 n);      // madd chain with the normal matrix

struct Material {
    sp_material_desc d;
};

struct Mesh {
    std::vector<f3>       vertices; // world space
    std::vector<f3>       normals;  // transformed, not re-normalised
    std::vector<uint32_t> indices;
};

// ImageBasedEnvironmentLight constructor input (base/FileParser.cpp:366-368).
struct EnvImage {
    int                width = 0, height = 0;
    std::vector<float> pixels; // img(x, y) at (y * width + x) * 3, already * radiance
    float              max_radiance = 3.40282347e38f;
    lin                light_to_world{}, world_to_light{};
};

// What the ImageBasedEnvironmentLight constructor derives (Lights/Light.h:196-330): the clamped
// radiance image (modify_image) and the Distribution2D over a 2x-resolution luminance x
// sin(theta) image (create_distribution, math/Distribution2D.h, math/Distribution1D.h),
// restated with the same float operation order.
struct EnvMap {
    int                w = 0, h = 0;          // radiance image
    std::vector<float> radiance;              // 3 per pixel, modify_image applied
    int                nu = 0, nv = 0;        // distribution grid (2w x 2h)
    std::vector<float> cond_func;             // nv x nu   Distribution1D::m_function (abs)
    std::vector<float> cond_cdf;              // nv x (nu + 1) m_cdf as the constructor leaves it
    std::vector<float> cond_int;              // nv        m_function_integral
    std::vector<float> marg_func, marg_cdf;   // nv, nv + 1
    float              marg_int = 0.0f;
    // Guide tables for Distribution1D::get_offset: cdf[0..n-1] is non-decreasing (only cdf[n],
    // the integral, breaks the order), so the libstdc++ upper_bound result equals "first i < n
    // with u < cdf[i], else n - 1".  guide[b] = that index for u = b / 2^bits (first i with
    // cdf[i] > b / 2^bits, clamped to n - 1): u in [b, b+1) / 2^bits lies in [guide[b], guide[b+1]].
    bool                  guided = false;     // false: some row is not ordered (NaN texels)
    int                   cond_bits = 0, marg_bits = 0;
    std::vector<uint32_t> cond_guide;         // nv x (2^cond_bits + 1)
    std::vector<uint32_t> marg_guide;         // 2^marg_bits + 1
};
EnvMap build_env_map(const EnvImage& img);
// Image/Image.cpp:78 read_pfm: img(x, y), rows stored bottom-up in the file.
void read_pfm(const std::string& path, int& w, int& h, std::vector<float>& pixels);

struct Scene {
    int         image_width  = 512; // FileParser defaults (base/FileParser.cpp:256-259)
    int         image_height = 512;
    int         rr_depth     = 3;
    int         max_depth    = 10;
    int         integrator   = SP_INTEGRATOR_NOT_SPECIFIED;
    std::string output_file_name;
    bool        has_camera = false;
    bool        camera_fixed = false; // built from a caller's sp_scene_desc: the transform is given
    // camera parameters kept so the resolution can be overridden
    f3    cam_origin{}, cam_look_at{}, cam_up{};
    float cam_fov_deg = 45.0f;
    aff   camera{};

    std::vector<Material>       materials;
    std::vector<std::string>    material_names;
    std::vector<sp_xform_shape> shapes;
    std::vector<sp_light_desc>  lights;
    std::vector<EnvImage>       env_images; // sp_light_desc.image indexes this
    // triangles of all meshes, concatenated (global vertex numbering)
    std::vector<f3>       vertices;
    std::vector<f3>       normals;
    std::vector<uint32_t> indices;
    std::vector<int32_t>  tri_material;
    // Scene::m_geometry order
    std::vector<int32_t> prim_kind;
    std::vector<int32_t> prim_index;

    void rebuild_camera();
};

std::unique_ptr<Scene> parse_scene(const std::string& text, const std::string& base_dir);
std::unique_ptr<Scene> parse_scene_file(const std::string& path);

// Camera (Cameras/Camera.h:99 PerspectiveCamera::create_transform)
aff perspective_camera_transform(f3 eye, f3 look_at, f3 up, float fov_degrees, int w, int h);

// RSequence<dim> alphas (math/Sampler.h:47), computed with glibc powf like the reference.
void rsequence_alphas(float alpha1[1], float alpha2[2]);

// ---- BVH ---------------------------------------------------------------------------------------
// Binary BVH node, 32 bytes: bounds + (left child, right child) or (first prim, count | LEAF_BIT).
struct BvhNode {
    float    lo[3];
    uint32_t a;   // internal: left child index;  leaf: first primitive slot
    float    hi[3];
    uint32_t b;   // internal: right child index; leaf: count | 0x80000000
};
static_assert(sizeof(BvhNode) == 32, "BvhNode layout");
constexpr uint32_t BVH_LEAF = 0x80000000u;
// SAH builds store the split axis of an internal node in the top bits of `a` (0..2); the
// reference-order build leaves them 0.  Child index = a & BVH_CHILD_MASK.
constexpr uint32_t BVH_AXIS_SHIFT = 30;
constexpr uint32_t BVH_CHILD_MASK = (1u << BVH_AXIS_SHIFT) - 1u;

struct Bvh {
    std::vector<BvhNode> nodes;
    std::vector<int32_t> prim_order; // slot -> primitive id (into the bounded list given)
    int                  max_depth = 0;
};

struct PrimBounds {
    float lo[3], hi[3];
};

// Reference construction (shapes/BVHAccelerator.h:173): midpoint split on the longest axis with
// libstdc++'s std::partition (unstable, two-sided swap), leaves of <= 4, leaf on failed split.
Bvh build_bvh_reference(const std::vector<PrimBounds>& bounds);
// Binned SAH construction (product default).
Bvh build_bvh_sah(const std::vector<PrimBounds>& bounds, int max_leaf = 4);

// 8-wide BVH collapsed from a binary SAH BVH (sp_bvh.cpp build_wide): 80-byte nodes with
// child boxes quantised outward on a per-node power-of-two grid, internal children first.
// Layout per node (5 x 16 bytes, u32 words):
//   [0..2] grid origin xyz (float bits)  [3] exponent bytes ex | ey << 8 | ez << 16 | imask << 24
//   [4] first child node  [5] first primitive slot  [6..7] meta bytes of slots 0-7
//       (leaf: count << 5 | offset from [5]; 0 = empty slot; internal slots 0..ni-1 per imask)
//   [8..19] quantised bytes: lo_x[8] lo_y[8] lo_z[8] hi_x[8] hi_y[8] hi_z[8] (4 per word)
struct WideBvh {
    std::vector<uint32_t> words;   // 20 per node
    std::vector<int32_t>  slot_of; // wide primitive slot -> binary primitive slot
    int                   depth = 0;
};
WideBvh build_wide(const Bvh& bvh);

// libstdc++ std::partition on a bidirectional range, returning the split point.
template <typename T, typename Pred>
size_t stl_partition(std::vector<T>& v, size_t first, size_t last, Pred pred)
{
    while (true) {
        while (true) {
            if (first == last) return first;
            if (pred(v[first])) ++first;
            else break;
        }
        --last;
        while (true) {
            if (first == last) return first;
            if (!pred(v[last])) --last;
            else break;
        }
        std::swap(v[first], v[last]);
        ++first;
    }
}

// RSQRTSS table capture (sp_rsqrt.cpp)
struct RsqrtCapture {
    std::vector<uint32_t> entries;
    int32_t               bits     = 0;
    bool                  verified = false;
    uint32_t              zero_result = 0, denorm_result = 0;
};
const RsqrtCapture& rsqrt_capture();
// The table the device emulates and host_rsqrt uses: the capture, or the installed override.
const RsqrtCapture& rsqrt_active();
// Install another CPU's table (entries == nullptr: back to this host's).  Throws SpError when
// the table is malformed.
void rsqrt_set_override(const uint32_t* entries, int32_t bits, uint32_t zero_result, uint32_t denorm_result);

} // namespace sph
