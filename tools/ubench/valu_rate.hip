// Microbenchmark: VALU issue throughput per SIMD on gfx950 for the instruction classes the
// shading kernels use.  Inline-asm chains (8 independent per lane, so latency never binds) of one
// instruction each; every SIMD holds W waves.  Reports SIMD cycles per wave-instruction at the
// measured clock.  Calibrates tools/pmc_valu.py's VALU cycle model.  Test infrastructure only.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 16384;

#define CH8(INS)                                                                                                    \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS         \
                     " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"                   \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)                       \
                 : "v"(b))

template <int KIND>
__global__ void __launch_bounds__(256) k(unsigned long long* out, unsigned long long* clk)
{
    using T = typename std::conditional<KIND == 2 || KIND == 3, double, float>::type;
    T a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    T b  = (T)0.5;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (KIND == 0) CH8("v_mul_f32");
        if constexpr (KIND == 1) CH8("v_xor_b32");
        if constexpr (KIND == 2) CH8("v_mul_f64");
        if constexpr (KIND == 3) CH8("v_add_f64");
        if constexpr (KIND == 4) { CH8("v_exp_f32"); }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    T s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned long long)s;
    if (threadIdx.x == 0) { clk[3 * blockIdx.x] = t1 - t0; clk[3 * blockIdx.x + 1] = r0; clk[3 * blockIdx.x + 2] = r1; }
}
// exp: "v_exp_f32 %0, %0, %8" is not a valid form (one source); use a dedicated kernel
__global__ void __launch_bounds__(256) kexp(unsigned long long* out, unsigned long long* clk)
{
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1e-3f, a2 = a0 + 2e-3f, a3 = a0 + 3e-3f, a4 = a0 + 4e-3f, a5 = a0 + 5e-3f,
          a6 = a0 + 6e-3f, a7 = a0 + 7e-3f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITERS; ++i)
        asm volatile("v_exp_f32 %0, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_exp_f32 %3, %3\n\t"
                     "v_exp_f32 %4, %4\n\tv_exp_f32 %5, %5\n\tv_exp_f32 %6, %6\n\tv_exp_f32 %7, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned long long)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
    if (threadIdx.x == 0) { clk[3 * blockIdx.x] = t1 - t0; clk[3 * blockIdx.x + 1] = r0; clk[3 * blockIdx.x + 2] = r1; }
}

template <typename K>
void run(const char* name, K kern, int waves_per_simd, int n_cu)
{
    const int blocks = waves_per_simd * n_cu; // 4 waves per block = one per SIMD
    unsigned long long *o, *c;
    (void)hipMalloc(&o, (size_t)blocks * 256 * 8);
    (void)hipMalloc(&c, (size_t)blocks * 3 * 8);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, c);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, c);
    (void)hipDeviceSynchronize();
    unsigned long long* h = new unsigned long long[3 * blocks];
    (void)hipMemcpy(h, c, (size_t)blocks * 3 * 8, hipMemcpyDeviceToHost);
    // wall span of all waves (s_memrealtime, 100 MHz) and the clock (shader cycles / real time)
    unsigned long long rmin = ~0ull, rmax = 0;
    double cyc = 0, real = 0;
    for (int i = 0; i < blocks; ++i) {
        rmin = h[3 * i + 1] < rmin ? h[3 * i + 1] : rmin;
        rmax = h[3 * i + 2] > rmax ? h[3 * i + 2] : rmax;
        cyc += (double)h[3 * i];
        real += (double)(h[3 * i + 2] - h[3 * i + 1]);
    }
    const double ghz   = cyc / real * 0.1;       // cycles per 10 ns tick -> GHz
    const double span  = (double)(rmax - rmin) * 10.0; // ns
    const double insts = (double)ITERS * 8 * waves_per_simd; // per SIMD
    printf("%-10s waves/SIMD=%d: %.2f cycles per wave-instruction per SIMD (clock %.2f GHz, span %.1f us)\n", name,
           waves_per_simd, span * ghz / insts, ghz, span / 1e3);
    delete[] h;
    (void)hipFree(o);
    (void)hipFree(c);
}

int main()
{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    for (int w : { 1, 2, 4, 8 }) {
        run("v_mul_f32", k<0>, w, p.multiProcessorCount);
        run("v_xor_b32", k<1>, w, p.multiProcessorCount);
        run("v_mul_f64", k<2>, w, p.multiProcessorCount);
        run("v_add_f64", k<3>, w, p.multiProcessorCount);
        run("v_exp_f32", kexp, w, p.multiProcessorCount);
    }
    return 0;
}
