// Probe: the 4x4 block transform's integer stage on the i8 matrix pipe.
// Each lane holds one 4x4 block's 16 pixel bytes (4 row words, XOR 0x80 = signed x - 128) as the
// B fragment of v_mfma_i32_32x32x32_i8; the A fragment is a lane-dependent {-1,0,1} pattern so
// that D register rho of lane l is J_rho of lane l's OWN block (rho = 4*ia + ib, ia/ib the row /
// column basis e0, e2, o0, o1).  Checks every lane and register against a host evaluation.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

static int basis(int b, int i) {  // e0, e2, o0, o1
    static const int B[4][4] = {{1, 1, 1, 1}, {1, -1, -1, 1}, {1, 0, 0, -1}, {0, 1, -1, 0}};
    return B[b][i];
}

__global__ void probe(const uint32_t* px, const uint32_t* wfrag, int* out, long long* cyc) {
    const int l = threadIdx.x;
    v4i a = {int(wfrag[4 * l]), int(wfrag[4 * l + 1]), int(wfrag[4 * l + 2]), int(wfrag[4 * l + 3])};
    v4i b;
    for (int r = 0; r < 4; r++) b[r] = int(px[4 * l + r] ^ 0x80808080u);
    v16i c = {};
    long long t0 = clock64();
    v16i d = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int k = 0; k < 16; k++) out[16 * l + k] = d[k];
    long long t1 = clock64();
    if (l == 0) *cyc = t1 - t0;
}

int main() {
    std::vector<uint32_t> px(256), w(256, 0);
    srand(7);
    for (auto& v : px) v = uint32_t(rand()) ^ (uint32_t(rand()) << 16);
    for (int l = 0; l < 64; l++) {
        const int r = l & 31, h = l >> 5;
        const int rho = (r & 3) + 4 * (r >> 3), hr = (r >> 2) & 1;
        const int ia = rho >> 2, ib = rho & 3;
        for (int j = 0; j < 16; j++) {
            const int row = j >> 2, col = j & 3;
            const int c = (h == hr) ? basis(ia, row) * basis(ib, col) : 0;
            w[4 * l + (j >> 2)] |= uint32_t(uint8_t(int8_t(c))) << (8 * (j & 3));
        }
    }
    uint32_t *dpx, *dw; int* dout; long long* dc;
    hipMalloc(&dpx, 1024); hipMalloc(&dw, 1024); hipMalloc(&dout, 64 * 16 * 4); hipMalloc(&dc, 8);
    hipMemcpy(dpx, px.data(), 1024, hipMemcpyHostToDevice);
    hipMemcpy(dw, w.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, 1, 64, 0, 0, dpx, dw, dout, dc);
    std::vector<int> out(1024); long long cyc;
    hipMemcpy(out.data(), dout, 4096, hipMemcpyDeviceToHost);
    hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++)
        for (int rho = 0; rho < 16; rho++) {
            long J = 0;
            for (int j = 0; j < 16; j++) {
                const int x = int((px[4 * l + (j >> 2)] >> (8 * (j & 3))) & 0xFF) - 128;
                J += long(basis(rho >> 2, j >> 2) * basis(rho & 3, j & 3)) * x;
            }
            if (J != out[16 * l + rho]) { if (bad < 10) printf("lane %d rho %d: got %d want %ld\n", l, rho, out[16 * l + rho], J); bad++; }
        }
    printf("mfma_i8_probe: %s (%d mismatches of 1024), %lld cycles\n", bad ? "FAIL" : "OK", bad, cyc);
    return bad ? 1 : 0;
}
