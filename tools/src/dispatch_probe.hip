// Workgroup dispatch cost probe: an (almost) empty kernel over G workgroups of T threads.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void empty_kernel(int* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = 1;
}
__global__ void spin_kernel(int* out, int iters) {
    int v = threadIdx.x;
    for (int i = 0; i < iters; i++) v = v * 1664525 + 1013904223;
    if (v == 0x12345) out[0] = v;
}
int main() {
    int* d;
    hipMalloc(&d, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int Ts[] = {64, 256, 1024};
    const int Gs[] = {1024, 4096, 16384, 65536};
    for (int T : Ts)
        for (int G : Gs) {
            for (int w = 0; w < 3; w++) hipLaunchKernelGGL(empty_kernel, dim3(G), dim3(T), 0, 0, d);
            hipEventRecord(a);
            for (int r = 0; r < 10; r++) hipLaunchKernelGGL(empty_kernel, dim3(G), dim3(T), 0, 0, d);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("empty T=%4d G=%6d  %8.2f us/launch\n", T, G, ms * 100.f);
        }
    for (int it : {100, 1000})
        for (int G : {4096, 16384}) {
            hipEventRecord(a);
            for (int r = 0; r < 10; r++) hipLaunchKernelGGL(spin_kernel, dim3(G), dim3(64), 0, 0, d, it);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("spin%d T=64 G=%6d  %8.2f us/launch\n", it, G, ms * 100.f);
        }
    return 0;
}
