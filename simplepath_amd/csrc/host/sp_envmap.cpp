// sp_envmap.cpp -- host side of the image-based environment light.
//
// read_pfm restates Image/Image.cpp:78; build_env_map restates what the
// ImageBasedEnvironmentLight constructor computes (Lights/Light.h:196 modify_image /
// create_distribution, math/Distribution2D.h, math/Distribution1D.h).  Every float operation
// keeps the reference's order (this file is built without FP contraction, and sinf is the host
// glibc's, as in the reference), because the device samples these tables and must land on the
// same texel and pdf bits as the reference.
#include "sp_host.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>

namespace sph {

void read_pfm(const std::string& path, int& w, int& h, std::vector<float>& pixels)
{
    std::ifstream ins(path, std::ios::binary);
    if (!ins) throw SpError(SP_ERR_IO, "Unable to open " + path);
    std::string format;
    std::getline(ins, format);
    if (format != "PF") throw SpError(SP_ERR_PARSE, "Unexpected format");
    int   nx = 0, ny = 0;
    float byte_order = 0.0f;
    ins >> nx >> ny >> byte_order;
    ins.get(); // last '\n'
    if (!ins || nx <= 0 || ny <= 0) throw SpError(SP_ERR_PARSE, "Bad PFM header: " + path);
    const bool big = byte_order > 0.0f;
    w              = nx;
    h              = ny;
    pixels.assign((size_t)nx * (size_t)ny * 3, 0.0f);
    std::vector<uint32_t> row((size_t)nx * 3);
    for (int j = ny - 1; j >= 0; --j) { // bottom row first
        ins.read(reinterpret_cast<char*>(row.data()), (std::streamsize)(row.size() * 4));
        if (!ins) throw SpError(SP_ERR_IO, "Truncated PFM: " + path);
        for (int i = 0; i < nx * 3; ++i) {
            uint32_t u = row[(size_t)i];
            if (big) u = __builtin_bswap32(u);
            float f;
            std::memcpy(&f, &u, 4);
            pixels[((size_t)j * (size_t)nx) * 3 + (size_t)i] = f;
        }
    }
}

namespace {

constexpr float k_max_less_than_one = 0x1.fffffep-1f; // base/Constants.h:15

float relative_luminance(float r, float g, float b) { return 0.2126f * r + 0.7152f * g + 0.0722f * b; } // math/RGB.h:224

// RemapWrap / RemapClamp + sample_nearest_neighbor (Image/Image.h:84-117)
size_t nearest_texel(int w, int h, float s, float t)
{
    s = std::fmod(1.0f + std::fmod(s, 1.0f), 1.0f);
    t = (t < 0.0f) ? 0.0f : ((k_max_less_than_one < t) ? k_max_less_than_one : t);
    const float    u = std::round(s * static_cast<float>(w));
    const float    v = std::round(t * static_cast<float>(h));
    const uint32_t x = std::min(static_cast<uint32_t>(u), static_cast<uint32_t>(w - 1));
    const uint32_t y = std::min(static_cast<uint32_t>(v), static_cast<uint32_t>(h - 1));
    return (size_t)y * (size_t)w + x;
}

// Distribution1D(std::vector<float> f) == Distribution1D(f, 0, 1) (math/Distribution1D.h:16).
// Note the constructor's normalisation writes cdf[i] = cdf[i + 1] / integral for i < n (a
// one-slot shifted std::transform) and leaves cdf[n] = integral; that is what sampling sees.
void distribution_1d(const float* f_in, size_t n, float* func, float* cdf, float* integral)
{
    const float range = 1.0f - 0.0f;
    for (size_t i = 0; i < n; ++i) func[i] = std::abs(f_in[i]);
    cdf[0] = 0.0f;
    for (size_t i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + func[i - 1] * range / static_cast<float>(n);
    const float I = cdf[n];
    *integral     = I;
    if (I == 0.0f) {
        for (size_t i = 1; i < n + 1; ++i) cdf[i] = static_cast<float>(i) / static_cast<float>(n);
    } else {
        for (size_t i = 0; i < n; ++i) cdf[i] = cdf[i + 1] / I;
    }
}

// guide table (sp_host.hpp EnvMap): returns false if cdf[0..n-1] is not non-decreasing
bool build_guide(const float* cdf, size_t n, int bits, uint32_t* guide)
{
    for (size_t i = 1; i < n; ++i)
        if (!(cdf[i - 1] <= cdf[i])) return false;
    const size_t G = (size_t)1 << bits;
    size_t       i = 0;
    for (size_t b = 0; b <= G; ++b) {
        const float v = std::ldexp((float)b, -bits); // exact: b / 2^bits
        while (i < n && !(cdf[i] > v)) ++i;
        guide[b] = (uint32_t)std::min(i, n - 1);
    }
    return true;
}
int guide_bits(size_t n)
{
    int b = 0;
    while (((size_t)1 << b) < n && b < 16) ++b;
    return b;
}

} // namespace

EnvMap build_env_map(const EnvImage& img)
{
    EnvMap m;
    m.w = img.width;
    m.h = img.height;
    const float maxr = img.max_radiance;
    // modify_image (Lights/Light.h:296)
    m.radiance = img.pixels;
    for (size_t p = 0; p < m.radiance.size(); p += 3) {
        float* c = &m.radiance[p];
        for (int i = 0; i < 3; ++i)
            if (std::isinf(c[i])) c[i] = maxr;
        if (relative_luminance(c[0], c[1], c[2]) > maxr) {
            const int mi = (c[0] > c[1]) ? ((c[0] > c[2]) ? 0 : 2) : ((c[1] > c[2]) ? 1 : 2); // index_of_max
            for (int i = 0; i < 3; ++i) c[i] = c[i] * maxr / c[mi]; // c[mi] changes at i == mi
        }
    }
    // create_distribution (Lights/Light.h:317)
    const int    width = 2 * m.w, height = 2 * m.h;
    const float  pi    = 3.14159265358979323846f;
    std::vector<float> fimg((size_t)width * (size_t)height);
    for (int v = 0; v < height; ++v) {
        const float vp        = (static_cast<float>(v) + 0.5f) / static_cast<float>(height);
        const float sin_theta = std::sin(pi * (static_cast<float>(v) + 0.5f) / static_cast<float>(height));
        for (int u = 0; u < width; ++u) {
            const float  up = (static_cast<float>(u) + 0.5f) / static_cast<float>(width);
            const float* c  = &m.radiance[nearest_texel(m.w, m.h, up, vp) * 3];
            float        x  = relative_luminance(c[0], c[1], c[2]);
            x *= sin_theta;
            if (std::isinf(x)) x = maxr;
            x = (maxr < x) ? maxr : x; // std::min
            fimg[(size_t)u + (size_t)v * width] = x;
        }
    }
    // Distribution2D(function, nu, nv) (math/Distribution2D.h:10)
    m.nu = width;
    m.nv = height;
    m.cond_func.resize((size_t)width * height);
    m.cond_cdf.resize((size_t)(width + 1) * height);
    m.cond_int.resize((size_t)height);
    for (int v = 0; v < height; ++v)
        distribution_1d(&fimg[(size_t)v * width], (size_t)width, &m.cond_func[(size_t)v * width],
                        &m.cond_cdf[(size_t)v * (width + 1)], &m.cond_int[(size_t)v]);
    m.marg_func.resize((size_t)height);
    m.marg_cdf.resize((size_t)height + 1);
    distribution_1d(m.cond_int.data(), (size_t)height, m.marg_func.data(), m.marg_cdf.data(), &m.marg_int);
    m.cond_bits = guide_bits((size_t)width);
    m.marg_bits = guide_bits((size_t)height);
    const size_t cg = ((size_t)1 << m.cond_bits) + 1;
    m.cond_guide.resize(cg * (size_t)height);
    m.marg_guide.resize(((size_t)1 << m.marg_bits) + 1);
    m.guided = build_guide(m.marg_cdf.data(), (size_t)height, m.marg_bits, m.marg_guide.data());
    for (int v = 0; v < height && m.guided; ++v)
        m.guided = build_guide(&m.cond_cdf[(size_t)v * (width + 1)], (size_t)width, m.cond_bits, &m.cond_guide[(size_t)v * cg]);
    if (!m.guided) { m.cond_guide.clear(); m.marg_guide.clear(); }
    return m;
}

} // namespace sph
