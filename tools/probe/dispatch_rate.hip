// Workgroup dispatch-rate probe with the encoder's footprint: 256 threads, 22 KB of dynamic LDS,
// 80 VGPRs (an asm clobber), so six workgroups per CU are resident.  Each workgroup waits T
// microseconds (100 MHz realtime clock) and records its start and end; the host prints the
// launch time, the mean concurrency in the steady state and the start rate.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ __launch_bounds__(256, 6) void sleeper(uint64_t* rec, int T10ns) {
    extern __shared__ uint32_t lds[];
    asm volatile("" ::: "v79");
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x < 64) lds[threadIdx.x] = uint32_t(t0);
    while (__builtin_amdgcn_s_memrealtime() - t0 < uint64_t(T10ns)) __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    if (threadIdx.x == 0) {
        rec[2 * blockIdx.x] = t0 + lds[5] * 0;
        rec[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

int main() {
    const int G = 8100;
    uint64_t* d;
    (void)hipMalloc(&d, 2 * G * sizeof(uint64_t));
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    int per = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, sleeper, 256, 22144);
    printf("occupancy API: %d workgroups per CU\n", per);
    for (int T : {200, 500, 1000, 1500}) {  // x 10 ns
        for (int w = 0; w < 2; w++) hipLaunchKernelGGL(sleeper, dim3(G), dim3(256), 22144, 0, d, T);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(sleeper, dim3(G), dim3(256), 22144, 0, d, T);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        std::vector<uint64_t> h(2 * G);
        (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
        uint64_t s0 = ~0ull, e1 = 0;
        for (int i = 0; i < G; i++) { s0 = std::min(s0, h[2 * i]); e1 = std::max(e1, h[2 * i + 1]); }
        const double span = (e1 - s0) / 100.0;
        // concurrency sampled every 0.5 us
        double conc_sum = 0; int ns = 0, cmax = 0;
        for (double x = 0.25; x < span; x += 0.5) {
            int c = 0;
            for (int i = 0; i < G; i++) { double st = (h[2*i]-s0)/100.0, en = (h[2*i+1]-s0)/100.0; c += (st <= x && en > x); }
            if (x > T / 100.0 && x < span - T / 100.0) { conc_sum += c; ns++; }
            cmax = std::max(cmax, c);
        }
        std::vector<double> st(G);
        for (int i = 0; i < G; i++) st[i] = (h[2 * i] - s0) / 100.0;
        std::sort(st.begin(), st.end());
        printf("T=%5.1f us: launch %.2f us (events), span %.2f us, ideal %.2f us; steady concurrency %.0f (max %d); "
               "starts of wg 1536..8100 over %.2f us = %.1f per us\n", T / 100.0, ms * 1000, span,
               (double(G) / (per * 256)) * T / 100.0, ns ? conc_sum / ns : 0.0, cmax, st[G - 1] - st[1536],
               (G - 1536) / (st[G - 1] - st[1536]));
    }
    return 0;
}
