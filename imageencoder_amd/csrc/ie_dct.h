// imageencoder_amd/csrc/ie_dct.h -- the FP32 fast-path forward DCT, written ONCE over a generic
// arithmetic type T so that the very same operation sequence runs
//   - on the device with T = float (encode_kernel), and
//   - on the host with T = ie::Trk, which tracks every value as an exact linear form of the 64
//     input pixels plus a rigorous bound on the accumulated FP32 rounding error.
// The host run yields, per coefficient, the real linear map the FP32 code implements (checked
// against the reference's c[u][i]*c[v][j]*C(u)C(v)/q) and a worst-case error bound; the kernel
// re-evaluates in FP64 every coefficient whose quotient falls within that bound of a rounding
// tie, so the FAST path returns the reference's integers exactly.
//
// Reference DCT (algo.cpp:309-331): D[u][v] = C(u)C(v) sum_ij c[u][i] c[v][j] x[i][j] with
// c[u][i] = cos((2i+1) u pi / 2N).  It is separable, so rows then columns of an N-point DCT-II
// (unscaled) compute it; the N-point DCTs use the even/odd butterfly of the cos symmetries
// c[u][N-1-i] = (-1)^u c[u][i].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ie {

// FP32 constants of the butterflies: k-th entry = cos(k pi / 16) rounded to float, k = 0..8
// (4-point DCT uses cos(pi/8)=K[2], cos(pi/4)=K[4], cos(3pi/8)=K[6]).
struct DctConsts {
    float K[9];
};

template <class T, class Op>
__host__ __device__ inline void dct4(const T* x, T* y, const DctConsts& k, const Op& op) {
    // y0 = (x0+x3)+(x1+x2);  y2 = c(pi/4)*((x0+x3)-(x1+x2))
    // y1 = c(pi/8)*(x0-x3) + c(3pi/8)*(x1-x2);  y3 = c(3pi/8)*(x0-x3) - c(pi/8)*(x1-x2)
    const T s0 = op.add(x[0], x[3]), s1 = op.add(x[1], x[2]);
    const T d0 = op.sub(x[0], x[3]), d1 = op.sub(x[1], x[2]);
    y[0] = op.add(s0, s1);
    y[2] = op.mul(op.sub(s0, s1), k.K[4]);
    y[1] = op.fma(d1, k.K[6], op.mul(d0, k.K[2]));
    y[3] = op.fma(d1, -k.K[2], op.mul(d0, k.K[6]));
}

template <class T, class Op>
__host__ __device__ inline void dct8(const T* x, T* y, const DctConsts& k, const Op& op) {
    // even half: 4-point DCT (pi/8 constants) of s_i = x_i + x_{7-i}
    T s[4], d[4], e[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s[i] = op.add(x[i], x[7 - i]);
        d[i] = op.sub(x[i], x[7 - i]);
    }
    dct4(s, e, k, op);
    y[0] = e[0];
    y[2] = e[1];
    y[4] = e[2];
    y[6] = e[3];
    // odd half: y[2m+1] = sum_i d_i cos((2i+1)(2m+1) pi / 16), entries +-cos(k pi/16), k odd
    // m=0: c1 c3 c5 c7;  m=1: c3 -c7 -c1 -c5;  m=2: c5 -c1 c7 c3;  m=3: c7 -c5 c3 -c1
    y[1] = op.fma(d[3], k.K[7], op.fma(d[2], k.K[5], op.fma(d[1], k.K[3], op.mul(d[0], k.K[1]))));
    y[3] = op.fma(d[3], -k.K[5], op.fma(d[2], -k.K[1], op.fma(d[1], -k.K[7], op.mul(d[0], k.K[3]))));
    y[5] = op.fma(d[3], k.K[3], op.fma(d[2], k.K[7], op.fma(d[1], -k.K[1], op.mul(d[0], k.K[5]))));
    y[7] = op.fma(d[3], -k.K[1], op.fma(d[2], k.K[3], op.fma(d[1], -k.K[5], op.mul(d[0], k.K[7]))));
}

// 2-D transform of an N x N block in place: rows (over j) then columns (over i).
// x[i*N+j] in, D[u*N+v] out (unscaled: the C(u)C(v)/q factor is applied by the caller).
template <int N, class T, class Op>
__host__ __device__ inline void dct2d(T* b, const DctConsts& k, const Op& op) {
    T t[N], o[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int j = 0; j < N; j++) t[j] = b[i * N + j];
        if constexpr (N == 4) dct4(t, o, k, op);
        else dct8(t, o, k, op);
#pragma unroll
        for (int v = 0; v < N; v++) b[i * N + v] = o[v];
    }
#pragma unroll
    for (int v = 0; v < N; v++) {
#pragma unroll
        for (int i = 0; i < N; i++) t[i] = b[i * N + v];
        if constexpr (N == 4) dct4(t, o, k, op);
        else dct8(t, o, k, op);
#pragma unroll
        for (int u = 0; u < N; u++) b[u * N + v] = o[u];
    }
}

// ---- quotient transforms: raw pixels in, t[uv] ~ D[uv] / q[uv] out -------------------------
// The level shift (x - 128, Block.cpp:141-143) is folded into the DC term: every other
// coefficient's linear form has coefficient sum 0 (its butterfly path passes through a
// difference), so shifting all pixels by 128 leaves it unchanged, and the DC path is an exact
// integer sum, from which 128*N*N is subtracted exactly before the scaling.

// N = 4, with the per-coefficient scale C(u)C(v)/q and the butterfly constants folded into the
// column stage.  Row stage (8 ops/row): R0 = s0+s1, R2 = s0-s1, R1 = d0 + r*d1, R3 = r*d0 - d1
// (r = cos(3pi/8)/cos(pi/8); the common factors K4, K2 move into the column constants).
// Column stage for column v (12 ops): t[0v] = (s0+s1)*G0, t[2v] = (s0-s1)*G2,
// t[1v] = d0*G1a + d1*G1b, t[3v] = d0*G3a + d1*G3b.
struct Dct4Plan {
    float r;
    float col[4][6];  // per column v: G0, G2, G1a, G1b, G3a, G3b
};

template <class T, class Op>
__host__ __device__ inline void quot4(T* b, const Dct4Plan& P, const Op& op) {
    T R[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const T s0 = op.add(b[4 * i + 0], b[4 * i + 3]), s1 = op.add(b[4 * i + 1], b[4 * i + 2]);
        const T d0 = op.sub(b[4 * i + 0], b[4 * i + 3]), d1 = op.sub(b[4 * i + 1], b[4 * i + 2]);
        R[4 * i + 0] = op.add(s0, s1);
        R[4 * i + 2] = op.sub(s0, s1);
        R[4 * i + 1] = op.fma(d1, P.r, d0);
        R[4 * i + 3] = op.fms(d0, P.r, d1);
    }
#pragma unroll
    for (int v = 0; v < 4; v++) {
        const float* G = P.col[v];
        const T s0 = op.add(R[v], R[12 + v]), s1 = op.add(R[4 + v], R[8 + v]);
        const T d0 = op.sub(R[v], R[12 + v]), d1 = op.sub(R[4 + v], R[8 + v]);
        T e = op.add(s0, s1);
        if (v == 0) e = op.addc(e, -2048.0f);  // level shift: -128 * 16, exact
        b[0 * 4 + v] = op.mul(e, G[0]);
        b[2 * 4 + v] = op.mul(op.sub(s0, s1), G[1]);
        b[1 * 4 + v] = op.fma(d1, G[3], op.mul(d0, G[2]));
        b[3 * 4 + v] = op.fma(d1, G[5], op.mul(d0, G[4]));
    }
}

// N = 4 on the matrix pipe (encode4p_kernel).  The 1-D DCT rows are integer combinations of four
// basis vectors -- e0 = (1,1,1,1), e2 = (1,-1,-1,1), o0 = (1,0,0,-1), o1 = (0,1,-1,0):
//   row u=0: e0;  u=2: K4 e2;  u=1: K2 o0 + K6 o1;  u=3: K6 o0 - K2 o1      (Kk = cos(k pi/16))
// so D[u][v] = C(u)C(v) sum_ij c[u][i] c[v][j] x[i][j] (algo.cpp:309-331) is a combination of the
// sixteen INTEGER sums J[4 ia + ib] = sum_ij B_ia(i) B_ib(j) (x[i][j] - 128) with 1, 2 or 4
// terms.  The device forms every J exactly in one v_mfma_i32_32x32x32_i8 per 64 blocks (pixels as
// signed bytes x ^ 0x80 = x - 128, the {-1,0,1} pattern as the other operand); quot4j is the FP32
// stage after it: t[uv] = sum_m G[uv][m] J[m-th term], one mul and up to three fmas per
// coefficient (36 operations), G = S(uv)/q(uv) * the basis factors, each rounded once on the host.
// dct4j_ints is the integer stage in plain arithmetic (the host's tracked run; exact either way).
struct Dct4JPlan {
    float G[16][4];  // [u*4+v][term]: terms (ia, ib) in the order of dct4j_terms
};
// the row (or column) basis indices of frequency u and how many there are
__host__ __device__ constexpr int dct4j_nb(int u) { return (u & 1) ? 2 : 1; }
__host__ __device__ constexpr int dct4j_b(int u, int m) { return (u & 1) ? 2 + m : (u >> 1); }

template <class T, class Op>
__host__ __device__ inline void dct4j_ints(const T* x, T* J, const Op& op) {
    T R[4][4];  // R[i][ib]: row i against column basis ib
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const T s0 = op.add(x[4 * i + 0], x[4 * i + 3]), s1 = op.add(x[4 * i + 1], x[4 * i + 2]);
        R[i][2] = op.sub(x[4 * i + 0], x[4 * i + 3]);
        R[i][3] = op.sub(x[4 * i + 1], x[4 * i + 2]);
        R[i][0] = op.add(s0, s1);
        R[i][1] = op.sub(s0, s1);
    }
#pragma unroll
    for (int ib = 0; ib < 4; ib++) {
        const T s0 = op.add(R[0][ib], R[3][ib]), s1 = op.add(R[1][ib], R[2][ib]);
        J[4 * 2 + ib] = op.sub(R[0][ib], R[3][ib]);
        J[4 * 3 + ib] = op.sub(R[1][ib], R[2][ib]);
        J[4 * 0 + ib] = op.add(s0, s1);
        J[4 * 1 + ib] = op.sub(s0, s1);
    }
}

// HALF: every quotient is formed as t + 1/2 (the first product's addend, no extra operation): the
// rounding then takes floor and fract of it (encode4p_kernel, round_half4).
template <bool HALF = false, class T, class Op, class Plan = Dct4JPlan>
__host__ __device__ inline void quot4j(const T* J, T* t, const Plan& P, const Op& op) {
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int k = 4 * u + v;
            T acc = HALF ? op.fmac(J[4 * dct4j_b(u, 0) + dct4j_b(v, 0)], P.G[k][0], 0.5f)
                         : op.mul(J[4 * dct4j_b(u, 0) + dct4j_b(v, 0)], P.G[k][0]);
            int m = 1;
#pragma unroll
            for (int a = 0; a < dct4j_nb(u); a++)
#pragma unroll
                for (int b = 0; b < dct4j_nb(v); b++) {
                    if (a == 0 && b == 0) continue;
                    acc = op.fma(J[4 * dct4j_b(u, a) + dct4j_b(v, b)], P.G[k][m], acc);
                    m++;
                }
            t[k] = acc;
        }
}

// N = 8: the separable butterfly (dct2d<8>), the exact DC level shift, then the scale g.
template <class T, class Op>
__host__ __device__ inline void quot8(T* b, const DctConsts& k, const float* g, const Op& op) {
    dct2d<8>(b, k, op);
    b[0] = op.addc(b[0], -8192.0f);  // -128 * 64, exact (integer sum)
#pragma unroll
    for (int m = 0; m < 64; m++) b[m] = op.mul(b[m], g[m]);
}

struct FloatOp {
    __device__ __forceinline__ float add(float a, float b) const { return a + b; }
    __device__ __forceinline__ float sub(float a, float b) const { return a - b; }
    __device__ __forceinline__ float mul(float a, float c) const { return a * c; }
    __device__ __forceinline__ float fma(float a, float c, float b) const { return __builtin_fmaf(a, c, b); }
    __device__ __forceinline__ float fms(float a, float c, float b) const { return __builtin_fmaf(a, c, -b); }
    __device__ __forceinline__ float addc(float a, float c) const { return a + c; }
    __device__ __forceinline__ float fmac(float a, float c, float k) const { return __builtin_fmaf(a, c, k); }
};

}  // namespace ie
