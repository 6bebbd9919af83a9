// Zero-copy PCIe probe: kernels that read pinned host memory into HBM (H2D) and write HBM into
// pinned host memory (D2H), alone and concurrently on two streams, against SDMA copies.
// Build: hipcc --offload-arch=gfx950 -O3 tools/src/pcie_kernel.hip -o tools/pcie_kernel
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void copy16(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n16) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n16; i += size_t(gridDim.x) * blockDim.x)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const size_t n = size_t(argc > 1 ? atoi(argv[1]) : 128) << 20;
    const int blocks = argc > 2 ? atoi(argv[2]) : 1024;
    void *hin, *hout, *da, *db;
    CK(hipHostMalloc(&hin, n, hipHostMallocMapped));
    CK(hipHostMalloc(&hout, n, hipHostMallocMapped));
    CK(hipMalloc(&da, n));
    CK(hipMalloc(&db, n));
    void *dhin, *dhout;
    CK(hipHostGetDevicePointer(&dhin, hin, 0));
    CK(hipHostGetDevicePointer(&dhout, hout, 0));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto run = [&](int mode, bool kern) {  // 1 H2D, 2 D2H, 3 both
        CK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < 5; r++) {
            if (mode & 1) {
                if (kern) hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s1, (const u32x4*)dhin, (u32x4*)da, n / 16);
                else CK(hipMemcpyAsync(da, hin, n, hipMemcpyHostToDevice, s1));
            }
            if (mode & 2) {
                if (kern) hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s2, (const u32x4*)db, (u32x4*)dhout, n / 16);
                else CK(hipMemcpyAsync(hout, db, n, hipMemcpyDeviceToHost, s2));
            }
        }
        CK(hipDeviceSynchronize());
        const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 5;
        const double gb = double(n) * ((mode & 1) + ((mode >> 1) & 1)) / t / 1e9;
        printf("%s %-5s %7.2f ms %6.1f GB/s total\n", kern ? "kernel" : "sdma  ", mode == 1 ? "H2D" : mode == 2 ? "D2H" : "both",
               t * 1e3, gb);
    };
    for (int k = 0; k < 2; k++) {
        run(3, k);
        for (int m = 1; m <= 3; m++) run(m, k);
    }
    return 0;
}
