// Microbenchmark: calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths
// the render kernels use -- 16, 8 and 4 bytes per lane, 64 lanes reading one contiguous row (the
// mt19937_64 state is read 8 B per lane, 512 B per wave-instruction).  Each kernel streams a known
// number of bytes through a buffer far larger than the Infinity Cache, so every byte comes from
// HBM once.  Run it under `rocprofv3 --kernel-trace --pmc FETCH_SIZE` and, separately,
// `--pmc WRITE_SIZE`; tools/fetch_calib.py divides the counters by the byte counts printed here.
// Test infrastructure only.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t BYTES = size_t(2) << 30; // 2 GiB per kernel

template <typename T>
__global__ void __launch_bounds__(256) rd(const T* __restrict__ a, size_t n, unsigned* out)
{
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const T v = a[i];
        const unsigned* w = reinterpret_cast<const unsigned*>(&v);
        for (size_t k = 0; k < sizeof(T) / 4; ++k) acc ^= w[k];
    }
    if (acc == 0x9e3779b9u) out[0] = acc; // keeps the loads; practically never stores
}

template <typename T>
__global__ void __launch_bounds__(256) wr(T* __restrict__ a, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        T v;
        unsigned* w = reinterpret_cast<unsigned*>(&v);
        for (size_t k = 0; k < sizeof(T) / 4; ++k) w[k] = (unsigned)(i + k);
        a[i] = v;
    }
}

int main()
{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const unsigned grid = (unsigned)p.multiProcessorCount * 8;
    void*     buf = nullptr;
    unsigned* out = nullptr;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, BYTES);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(rd<uint4>, dim3(grid), dim3(256), 0, 0, (const uint4*)buf, BYTES / 16, out);
    hipLaunchKernelGGL(rd<uint2>, dim3(grid), dim3(256), 0, 0, (const uint2*)buf, BYTES / 8, out);
    hipLaunchKernelGGL(rd<unsigned>, dim3(grid), dim3(256), 0, 0, (const unsigned*)buf, BYTES / 4, out);
    hipLaunchKernelGGL(wr<uint4>, dim3(grid), dim3(256), 0, 0, (uint4*)buf, BYTES / 16);
    hipLaunchKernelGGL(wr<uint2>, dim3(grid), dim3(256), 0, 0, (uint2*)buf, BYTES / 8);
    hipLaunchKernelGGL(wr<unsigned>, dim3(grid), dim3(256), 0, 0, (unsigned*)buf, BYTES / 4);
    (void)hipDeviceSynchronize();
    printf("{\"bytes_per_kernel\": %zu, \"kernels\": [\"rd<uint4>\", \"rd<uint2>\", \"rd<unsigned>\", \"wr<uint4>\", \"wr<uint2>\", \"wr<unsigned>\"]}\n",
           BYTES);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
