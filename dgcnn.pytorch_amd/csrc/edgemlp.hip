// Per-edge two-layer MLP of the PositionEmbedding block (reference
// models/layers.py:45-52):
//     e  = get_graph_feature(x, k)                       (B, 2C, N, k)
//     h1 = LeakyReLU(BN1(Conv2d(2C -> C1, 1x1)(e)))       per edge, NOT maxed
//     z2 = Conv2d(C1 -> C2, 1x1)(h1)                      per edge
//     t  = max_k LeakyReLU(BN2(z2))                       (B, C2, N)
// Layout: edges are rows e = i*k + s (i = global point, s = neighbour slot),
// point-major like the EdgeConv chain. The first conv is decomposed as in
// edgeconv.hip (y_e = P_j + Q_i from PQ = X [W1;W2]^T), so only h1 (E x C1)
// and z2 (E x C2) exist per edge; both feed / come from the caller's MFMA GEMM
// (gemm.hip) as dense row-major operands. BN1 statistics come from
// dgx_edge_fwd_gather_f32 (sums over all edges of P_j + Q_i), BN2 statistics
// from the z2 GEMM's epilogue (or dgx_colstats_f32).
//
// Kernels (all HBM/L2 streaming, 16-byte accesses along channels):
//   mlp_h1_kernel        h1 = LReLU(a1 (P_j + Q_i) + b1), fp32 or bf16 rows
//   mlp_max_kernel       max_k (min_k where a2 < 0) of z2 and its slot
//   mlp_dz2_kernel       dZ2 = a2 dz [slot] + c0 + c1 z2 (BN2 backward), dense
//   mlp_h1_bwd_kernel    g = dH1 * LReLU'(z1) in place + BN1-backward partials
//   mlp_h1_scatter_kernel dP_j / dQ_i from g over the edge rows and the reverse kNN graph
//   mlp_h1_scatter4_kernel the same for bf16 g and C1 = 64, four points per wave
#include "common.h"

namespace {

constexpr int EM_THREADS = 256;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

// 8 consecutive floats as two float4 loads into v[0..7]
__device__ __forceinline__ void ld8(const float* p, float* v) {
    const float4 a = ld4(p), b = ld4(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

__device__ __forceinline__ float4 ld4_any(const void* base, int64_t off, bool b16) {
    if (b16) {
        const bf16x4_t h = *reinterpret_cast<const bf16x4_t*>(static_cast<const __bf16*>(base) + off);
        return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
    }
    return ld4(static_cast<const float*>(base) + off);
}

__device__ __forceinline__ void st4_any(void* base, int64_t off, float4 v, bool b16) {
    if (b16) {
        const bf16x4_t h = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
        *reinterpret_cast<bf16x4_t*>(static_cast<__bf16*>(base) + off) = h;
    } else {
        *reinterpret_cast<float4*>(static_cast<float*>(base) + off) = v;
    }
}

__device__ __forceinline__ float comp(const float4& v, int u) {
    return u == 0 ? v.x : (u == 1 ? v.y : (u == 2 ? v.z : v.w));
}

inline int grid_of(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

// h1[e][c] = LReLU(fmaf(a_c, P_j[c] + Q_i[c], b_c)), 8 channels per thread
// (two float4 loads of P_j and Q_i, one 16-byte bf16 or two float4 stores).
template <bool OUT16>
__global__ __launch_bounds__(EM_THREADS) void mlp_h1_kernel(const float* __restrict__ PQ, int ldpq,
                                                            const int32_t* __restrict__ idx, int N, int k, int C1,
                                                            int64_t E, const float* __restrict__ scale,
                                                            const float* __restrict__ shift, float slope,
                                                            void* __restrict__ H1) {
    const int co = C1 >> 3;
    const int64_t total = E * co;
    for (int64_t t = (int64_t)blockIdx.x * EM_THREADS + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * EM_THREADS) {
        const int c = (int)(t % co) * 8;
        const int64_t e = t / co;
        const int64_t i = e / k;
        const int64_t j = (i / N) * N + idx[e];
        float p[8], q[8], a[8], b[8], h[8];
        ld8(PQ + j * ldpq + c, p);
        ld8(PQ + i * ldpq + C1 + c, q);
        ld8(scale + c, a);
        ld8(shift + c, b);
#pragma unroll
        for (int u = 0; u < 8; ++u) h[u] = lrelu(fmaf(a[u], p[u] + q[u], b[u]), slope);
        if (OUT16) {
            bf16x8_t o;
#pragma unroll
            for (int u = 0; u < 8; ++u) o[u] = (__bf16)h[u];
            *reinterpret_cast<bf16x8_t*>(static_cast<__bf16*>(H1) + e * C1 + c) = o;
        } else {
            float* dst = static_cast<float*>(H1) + e * C1 + c;
            *reinterpret_cast<float4*>(dst) = make_float4(h[0], h[1], h[2], h[3]);
            *reinterpret_cast<float4*>(dst + 4) = make_float4(h[4], h[5], h[6], h[7]);
        }
    }
}

// 8 consecutive values of a fp32 or bf16 row as floats
template <bool B16>
__device__ __forceinline__ void ld8_any(const void* base, int64_t off, float* v) {
    if (B16) {
        const bf16x8_t h = *reinterpret_cast<const bf16x8_t*>(static_cast<const __bf16*>(base) + off);
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = (float)h[u];
    } else {
        ld8(static_cast<const float*>(base) + off, v);
    }
}

// ysel[i][c] = max_s z2[i*k+s][c] (min where scale[c] < 0: BN's affine is
// decreasing there, so LReLU(BN(.)) is maximised by the smallest z), arg = s
// of the first extremum (the order torch.max keeps on ties). 8 channels per
// thread, 16-byte row loads, EM_MU rows in flight.
constexpr int EM_MU = 8;
template <bool IN16>
__global__ __launch_bounds__(EM_THREADS) void mlp_max_kernel(const void* __restrict__ Z, int64_t M, int k, int C2,
                                                             const float* __restrict__ scale,
                                                             float* __restrict__ ysel, uint8_t* __restrict__ arg) {
    const int co = C2 >> 3;
    const int64_t total = M * co;
    for (int64_t t = (int64_t)blockIdx.x * EM_THREADS + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * EM_THREADS) {
        const int c = (int)(t % co) * 8;
        const int64_t i = t / co;
        float a[8];
        ld8(scale + c, a);
        float bv[8];
        int bs[8];
        ld8_any<IN16>(Z, i * k * C2 + c, bv);
#pragma unroll
        for (int u = 0; u < 8; ++u) bs[u] = 0;
        for (int s0 = 1; s0 < k; s0 += EM_MU) {
            float v[EM_MU][8];
#pragma unroll
            for (int m = 0; m < EM_MU; ++m) ld8_any<IN16>(Z, (i * k + min(s0 + m, k - 1)) * C2 + c, v[m]);
#pragma unroll
            for (int m = 0; m < EM_MU; ++m) {
                if (s0 + m >= k) break;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const float x = v[m][u];
                    if (a[u] < 0.f ? x < bv[u] : x > bv[u]) { bv[u] = x; bs[u] = s0 + m; }
                }
            }
        }
        *reinterpret_cast<float4*>(ysel + i * C2 + c) = make_float4(bv[0], bv[1], bv[2], bv[3]);
        *reinterpret_cast<float4*>(ysel + i * C2 + c + 4) = make_float4(bv[4], bv[5], bv[6], bv[7]);
        uint2 packed;
        packed.x = (uint32_t)bs[0] | ((uint32_t)bs[1] << 8) | ((uint32_t)bs[2] << 16) | ((uint32_t)bs[3] << 24);
        packed.y = (uint32_t)bs[4] | ((uint32_t)bs[5] << 8) | ((uint32_t)bs[6] << 16) | ((uint32_t)bs[7] << 24);
        *reinterpret_cast<uint2*>(arg + i * C2 + c) = packed;
    }
}

// BN2 backward, dense over edges: dZ2[e][c] = a_c dz_i[c] [s == slot_i[c]] + c0_c + c1_c z2[e][c].
// A thread owns 8 channels of one point: the point's dz, selected slots and
// the per-channel constants are loaded once, then its k edge rows stream through
// (16-byte bf16 rows, or two float4).
template <bool IO16>
__global__ __launch_bounds__(EM_THREADS) void mlp_dz2_kernel(const float* __restrict__ dz,
                                                             const uint8_t* __restrict__ arg, const void* __restrict__ Z,
                                                             int64_t M, int k, int C2, const float* __restrict__ scale,
                                                             const float* __restrict__ c0,
                                                             const float* __restrict__ c1, void* __restrict__ dZ) {
    const int co = C2 >> 3;
    const int64_t total = M * co;
    for (int64_t t = (int64_t)blockIdx.x * EM_THREADS + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * EM_THREADS) {
        const int c = (int)(t % co) * 8;
        const int64_t i = t / co;
        float d[8], a[8], k0[8], k1[8];
        ld8(dz + i * C2 + c, d);
        const uint2 sw = *reinterpret_cast<const uint2*>(arg + i * C2 + c);
        ld8(scale + c, a);
        ld8(c0 + c, k0);
        ld8(c1 + c, k1);
        int slot[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            slot[u] = (int)(((u < 4 ? sw.x : sw.y) >> (8 * (u & 3))) & 0xffu);
            d[u] = a[u] * d[u];
        }
#pragma unroll 2
        for (int s = 0; s < k; ++s) {
            const int64_t e = i * k + s;
            float z[8], r[8];
            if (IO16) {
                const bf16x8_t h = *reinterpret_cast<const bf16x8_t*>(static_cast<const __bf16*>(Z) + e * C2 + c);
#pragma unroll
                for (int u = 0; u < 8; ++u) z[u] = (float)h[u];
            } else {
                ld8(static_cast<const float*>(Z) + e * C2 + c, z);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float v = fmaf(k1[u], z[u], k0[u]);
                r[u] = slot[u] == s ? v + d[u] : v;
            }
            if (IO16) {
                bf16x8_t h;
#pragma unroll
                for (int u = 0; u < 8; ++u) h[u] = (__bf16)r[u];
                *reinterpret_cast<bf16x8_t*>(static_cast<__bf16*>(dZ) + e * C2 + c) = h;
            } else {
                float* dst = static_cast<float*>(dZ) + e * C2 + c;
                *reinterpret_cast<float4*>(dst) = make_float4(r[0], r[1], r[2], r[3]);
                *reinterpret_cast<float4*>(dst + 4) = make_float4(r[4], r[5], r[6], r[7]);
            }
        }
    }
}

// LReLU + BN1 backward, first half: g = dH1 * LReLU'(z1) (written over dH1)
// and per-block partials (sum g, sum g * yhat) per channel -> partials[block][2][C1].
// Block = (256 / cq) edge rows x cq channel quads; each thread keeps fixed
// channels, so the block's partial is a fixed-order sum (deterministic).
__global__ __launch_bounds__(EM_THREADS) void mlp_h1_bwd_kernel(
    float* __restrict__ dH, const float* __restrict__ PQ, int ldpq, const int32_t* __restrict__ idx, int N, int k,
    int C1, int64_t E, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd, float slope, float* __restrict__ partials) {
    __shared__ float red[2][EM_THREADS][4];
    const int cq = C1 >> 2;
    const int epb = EM_THREADS / cq;
    const int tid = threadIdx.x;
    const int er = tid / cq, c = (tid - er * cq) * 4;
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    if (er < epb) {
        const float4 a = ld4(scale + c), b = ld4(shift + c), mu = ld4(mean + c), is = ld4(invstd + c);
        for (int64_t e = (int64_t)blockIdx.x * epb + er; e < E; e += (int64_t)gridDim.x * epb) {
            const int64_t i = e / k;
            const int64_t j = (i / N) * N + idx[e];
            const float4 p = ld4(PQ + j * ldpq + c), q = ld4(PQ + i * ldpq + C1 + c);
            const float4 dh = ld4(dH + e * C1 + c);
            float g[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float y = comp(p, u) + comp(q, u);
                const float z = fmaf(comp(a, u), y, comp(b, u));
                g[u] = comp(dh, u) * (z > 0.f ? 1.f : slope);
                s1[u] += g[u];
                s2[u] = fmaf(g[u], (y - comp(mu, u)) * comp(is, u), s2[u]);
            }
            *reinterpret_cast<float4*>(dH + e * C1 + c) = make_float4(g[0], g[1], g[2], g[3]);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        red[0][tid][u] = s1[u];
        red[1][tid][u] = s2[u];
    }
    __syncthreads();
    if (tid < cq) {
        float t1[4] = {0.f, 0.f, 0.f, 0.f}, t2[4] = {0.f, 0.f, 0.f, 0.f};
        for (int r = 0; r < epb; ++r) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                t1[u] += red[0][r * cq + tid][u];
                t2[u] += red[1][r * cq + tid][u];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            partials[(int64_t)blockIdx.x * 2 * C1 + c + u] = t1[u];
            partials[(int64_t)blockIdx.x * 2 * C1 + C1 + c + u] = t2[u];
        }
    }
}

// BN1 backward, second half, one wave per point p (lanes = channels):
//   dy_e = a g_e + c0 + c1 (P_j + Q_i) for edge e = (i, s), j = idx[e]
//   dQ_p = sum over p's own k edges of dy,  dP_p = sum over p's in-edges of dy
// (in-edges from dgx_graph_reverse: id = (i << 6) | s, sorted lists; sumP_p =
// sum_s P_j from the BN1-statistics gather). The row loads are issued EM_U at
// a time into separate accumulators so several HBM/L2 requests are in flight
// per wave (the loop is latency-bound otherwise); the combination order is
// fixed, so the result is deterministic.
constexpr int EM_U = 8;
template <typename GT>
__global__ __launch_bounds__(EM_THREADS) void mlp_h1_scatter_kernel(
    const GT* __restrict__ g, const float* __restrict__ PQ, int ldpq, const float* __restrict__ sumP,
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ edges, int64_t M, int k, int C1,
    const float* __restrict__ scale, const float* __restrict__ c0, const float* __restrict__ c1,
    float* __restrict__ dPQ) {
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * (EM_THREADS / 64) + (threadIdx.x >> 6);
    if (p >= M) return;
    const int32_t beg = rowptr[p], end = rowptr[p + 1];
    const float kf = (float)k, deg = (float)(end - beg);
    for (int c = lane; c < C1; c += 64) {
        const float a = scale[c], k0 = c0[c], k1 = c1[c];
        const GT* __restrict__ gp = g + p * k * C1 + c;
        float sgv[EM_U];
#pragma unroll
        for (int u = 0; u < EM_U; ++u) sgv[u] = 0.f;
        int s = 0;
        for (; s + EM_U <= k; s += EM_U) {
#pragma unroll
            for (int u = 0; u < EM_U; ++u) sgv[u] += (float)gp[(int64_t)(s + u) * C1];
        }
        for (; s < k; ++s) sgv[0] += (float)gp[(int64_t)s * C1];
        float igv[EM_U], iqv[EM_U];
#pragma unroll
        for (int u = 0; u < EM_U; ++u) { igv[u] = 0.f; iqv[u] = 0.f; }
        // the in-edge ids come in with one load per 64 (lane u holds id u of the
        // chunk) and are broadcast with readlane: no dependent id load per batch
        // (needs every lane active: C1 a multiple of 64; else one id load per batch)
        if (C1 % 64 != 0) {
            int32_t r = beg;
            for (; r + EM_U <= end; r += EM_U) {
                int32_t id[EM_U];
#pragma unroll
                for (int u = 0; u < EM_U; ++u) id[u] = edges[r + u];
#pragma unroll
                for (int u = 0; u < EM_U; ++u) {
                    const int64_t src = (int64_t)(id[u] >> 6);
                    igv[u] += (float)g[(src * k + (id[u] & 63)) * C1 + c];
                    iqv[u] += PQ[src * ldpq + C1 + c];
                }
            }
            for (; r < end; ++r) {
                const int32_t id = edges[r];
                const int64_t src = (int64_t)(id >> 6);
                igv[0] += (float)g[(src * k + (id & 63)) * C1 + c];
                iqv[0] += PQ[src * ldpq + C1 + c];
            }
        }
        for (int32_t r0 = beg; C1 % 64 == 0 && r0 < end; r0 += 64) {
            const int cnt = min(64, (int)(end - r0));
            const int32_t mine = lane < cnt ? edges[r0 + lane] : 0;
            int u0 = 0;
            for (; u0 + EM_U <= cnt; u0 += EM_U) {
                int32_t id[EM_U];
#pragma unroll
                for (int u = 0; u < EM_U; ++u) id[u] = __builtin_amdgcn_readlane(mine, u0 + u);
#pragma unroll
                for (int u = 0; u < EM_U; ++u) {
                    const int64_t src = (int64_t)(id[u] >> 6);
                    igv[u] += (float)g[(src * k + (id[u] & 63)) * C1 + c];
                    iqv[u] += PQ[src * ldpq + C1 + c];
                }
            }
            for (; u0 < cnt; ++u0) {
                const int32_t id = __builtin_amdgcn_readlane(mine, u0);
                const int64_t src = (int64_t)(id >> 6);
                igv[0] += (float)g[(src * k + (id & 63)) * C1 + c];
                iqv[0] += PQ[src * ldpq + C1 + c];
            }
        }
        float sg = 0.f, ig = 0.f, iq = 0.f;
#pragma unroll
        for (int u = 0; u < EM_U; ++u) { sg += sgv[u]; ig += igv[u]; iq += iqv[u]; }
        const float Pp = PQ[p * ldpq + c], Qp = PQ[p * ldpq + C1 + c];
        dPQ[p * 2 * C1 + c] = fmaf(a, ig, fmaf(k0, deg, k1 * fmaf(deg, Pp, iq)));
        dPQ[p * 2 * C1 + C1 + c] = fmaf(a, sg, fmaf(k0, kf, k1 * fmaf(kf, Qp, sumP[p * C1 + c])));
    }
}

// bf16 g with C1 = 64: 64 / LPP points per wave (LPP lanes each, CPL = 64 /
// LPP channels per lane: 2·CPL-byte g loads, 4·CPL-byte Q loads), so one load
// instruction carries 64 / LPP in-edges instead of one and a wave keeps that
// many more rows in flight (the one-point-per-wave kernel above is bound by
// its dependent load latency). In-edge ids are loaded one batch ahead. Sums in
// a fixed order (batch slot u, then u = 0..EM_U4-1): deterministic.
template <int EM_U4, int LPP>
__global__ __launch_bounds__(EM_THREADS) void mlp_h1_scatter4_kernel(
    const __bf16* __restrict__ g, const float* __restrict__ PQ, int ldpq, const float* __restrict__ sumP,
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ edges, int B, int N, int tiles, int k,
    const float* __restrict__ scale, const float* __restrict__ c0, const float* __restrict__ c1,
    float* __restrict__ dPQ) {
    constexpr int C1 = 64, CPL = C1 / LPP, PPW = 64 / LPP;
    const int lane = threadIdx.x & 63, c = CPL * (lane % LPP);
    // blocks of a cloud stay on one XCD: its in-edge rows are gathered from its own g rows
    int b, tile;
    if (!dgx_xcd_cloud_map(blockIdx.x, B, tiles, b, tile)) return;
    const int n = tile * (EM_THREADS / LPP) + (threadIdx.x >> 6) * PPW + lane / LPP;
    const bool live = n < N;
    const int64_t p = (int64_t)b * N + n;
    const int64_t pc = live ? p : (int64_t)b * N + N - 1;  // lanes past the end shadow the last point, write nothing
    const int32_t beg = rowptr[pc], cnt = live ? rowptr[pc + 1] - beg : 0;
    auto addg = [](float* acc, const __bf16* q) {
#pragma unroll
        for (int h = 0; h < CPL / 4; ++h) {
            const uint2 w = *reinterpret_cast<const uint2*>(q + 4 * h);
            acc[4 * h + 0] += __uint_as_float(w.x << 16);
            acc[4 * h + 1] += __uint_as_float(w.x & 0xffff0000u);
            acc[4 * h + 2] += __uint_as_float(w.y << 16);
            acc[4 * h + 3] += __uint_as_float(w.y & 0xffff0000u);
        }
    };
    auto addf = [](float* acc, const float* q) {
#pragma unroll
        for (int h = 0; h < CPL / 4; ++h) {
            const float4 v = ld4(q + 4 * h);
            acc[4 * h + 0] += v.x; acc[4 * h + 1] += v.y; acc[4 * h + 2] += v.z; acc[4 * h + 3] += v.w;
        }
    };
    float sgv[EM_U4][CPL], igv[EM_U4][CPL], iqv[EM_U4][CPL];
#pragma unroll
    for (int u = 0; u < EM_U4; ++u)
#pragma unroll
        for (int e = 0; e < CPL; ++e) { sgv[u][e] = 0.f; igv[u][e] = 0.f; iqv[u][e] = 0.f; }
    int32_t idn[EM_U4];
    auto load_ids = [&](int r) {
#pragma unroll
        for (int u = 0; u < EM_U4; ++u) idn[u] = r + u < cnt ? edges[beg + r + u] : -1;
    };
    load_ids(0);
    const __bf16* __restrict__ gp = g + pc * k * C1 + c;
    int s = 0;
    for (; s + EM_U4 <= k; s += EM_U4) {
#pragma unroll
        for (int u = 0; u < EM_U4; ++u) addg(sgv[u], gp + (int64_t)(s + u) * C1);
    }
    for (; s < k; ++s) addg(sgv[0], gp + (int64_t)s * C1);
    int cmax = cnt;
#pragma unroll
    for (int o = LPP; o < 64; o <<= 1) cmax = max(cmax, __shfl_xor(cmax, o));
    for (int r = 0; r < cmax; r += EM_U4) {
        int32_t id[EM_U4];
#pragma unroll
        for (int u = 0; u < EM_U4; ++u) id[u] = idn[u];
        load_ids(r + EM_U4);
#pragma unroll
        for (int u = 0; u < EM_U4; ++u) {
            if (id[u] >= 0) {
                const int64_t src = (int64_t)(id[u] >> 6);
                addg(igv[u], g + (src * k + (id[u] & 63)) * C1 + c);
                addf(iqv[u], PQ + src * ldpq + C1 + c);
            }
        }
    }
    if (!live) return;
    const float kf = (float)k, deg = (float)cnt;
#pragma unroll
    for (int h = 0; h < CPL / 4; ++h) {
        const int ch = c + 4 * h;
        const float4 a4 = ld4(scale + ch), k04 = ld4(c0 + ch), k14 = ld4(c1 + ch);
        const float4 P4 = ld4(PQ + p * ldpq + ch), Q4 = ld4(PQ + p * ldpq + C1 + ch), S4 = ld4(sumP + p * C1 + ch);
        const float a[4] = {a4.x, a4.y, a4.z, a4.w}, k0[4] = {k04.x, k04.y, k04.z, k04.w};
        const float k1[4] = {k14.x, k14.y, k14.z, k14.w}, Pp[4] = {P4.x, P4.y, P4.z, P4.w};
        const float Qp[4] = {Q4.x, Q4.y, Q4.z, Q4.w}, sP[4] = {S4.x, S4.y, S4.z, S4.w};
        float dP[4], dQ[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float sg = sgv[0][4 * h + e], ig = igv[0][4 * h + e], iq = iqv[0][4 * h + e];
#pragma unroll
            for (int u = 1; u < EM_U4; ++u) { sg += sgv[u][4 * h + e]; ig += igv[u][4 * h + e]; iq += iqv[u][4 * h + e]; }
            dP[e] = fmaf(a[e], ig, fmaf(k0[e], deg, k1[e] * fmaf(deg, Pp[e], iq)));
            dQ[e] = fmaf(a[e], sg, fmaf(k0[e], kf, k1[e] * fmaf(kf, Qp[e], sP[e])));
        }
        *reinterpret_cast<float4*>(dPQ + p * 2 * C1 + ch) = make_float4(dP[0], dP[1], dP[2], dP[3]);
        *reinterpret_cast<float4*>(dPQ + p * 2 * C1 + C1 + ch) = make_float4(dQ[0], dQ[1], dQ[2], dQ[3]);
    }
}

// ---- fused forward (bf16 mode): h1 -> conv2 on the MFMA -> max over k + BN2
// statistics, without writing z2. A block is a pair of waves and takes
// EMF_PPB points one at a time; wave `half` owns C2 output channels
// [C2/2 half, C2/2 (half + 1)). The point's k edge rows, padded to KT tiles of
// 16, are the MFMA row tiles. Per row tile the pair builds h1 = LReLU(a1 (P_j +
// Q_i) + b1) once (as LReLU(a1 P_j + qb), qb = a1 Q_i + b1 per point, rounded
// to bf16 as the unfused path stores it): wave `half` gathers rows 8 half ..
// 8 half + 7, eight lanes per 256-byte P_j row (two whole 128-byte lines per
// load instruction), and writes its bf16 rows to an LDS tile (double-buffered
// by tile parity: one barrier per tile). Each wave then reads the A fragments
// (row = lane & 15, channels 32 ks + 8 g .. +7, g = lane >> 4), multiplies by
// its half of W2 (B fragments in registers for the whole kernel) and folds the
// 16 x C2/2 result into the point's running max (and first slot) and the
// per-column sums of z2 and z2^2. W2's rows come pre-multiplied by dir =
// sign(gamma2) (exact), so the max of dir * z2 is the max (or min) the BN2 +
// LReLU ordering needs; outputs are multiplied back. Optionally writes h1
// (bf16, the unfused backward's operand). Blocks of a cloud stay on one XCD
// (its P rows are L2-resident); partial-stat row = block. Held to 3 waves per
// SIMD (168 VGPRs; BN1's scale / shift read from LDS where used, not held in
// registers): 184 us at cfg4, against 228 us at the 2 waves the compiler picks
// unasked, 303-436 us at 4 waves (spills), and 298 us for the previous kernel,
// which built every h1 tile in both waves of a pair.
constexpr int EMF_PPB = 8;
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint2 pack4_bf16(const __bf16* h) {
    return make_uint2((uint32_t)__builtin_bit_cast(uint16_t, h[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, h[1]) << 16),
                      (uint32_t)__builtin_bit_cast(uint16_t, h[2]) | ((uint32_t)__builtin_bit_cast(uint16_t, h[3]) << 16));
}

template <int KT, int NTW>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(3))) void emlp_fwd_kernel(
    const float* __restrict__ PQ, int ldpq, const int32_t* __restrict__ idx, int B, int N, int k, int tiles,
    const float* __restrict__ scale1, const float* __restrict__ shift1, float slope1, const __bf16* __restrict__ W2d,
    const float* __restrict__ dir2, float* __restrict__ ysel, uint8_t* __restrict__ arg, float* __restrict__ part,
    __bf16* __restrict__ H1) {
    constexpr int C1 = 64, C2 = 32 * NTW, HP = C1 + 8;  // h1 tile pitch: +16 B staggers rows over the banks
    __shared__ __attribute__((aligned(16))) __bf16 h1s[2][16 * HP];
    __shared__ __attribute__((aligned(16))) float cs[2][C1];  // BN1 scale | shift
    int b, tile;
    if (!dgx_xcd_cloud_map(blockIdx.x, B, tiles, b, tile)) return;
    cs[threadIdx.x >> 6][threadIdx.x & 63] = (threadIdx.x >> 6 ? shift1 : scale1)[threadIdx.x & 63];
    __syncthreads();
    const int lane = threadIdx.x & 63, half = threadIdx.x >> 6;
    const int g = lane >> 4, r16 = lane & 15;
    const int cb = half * NTW;  // first channel tile of this wave
    // gather role: tile row R, channels 4m .. 4m+3 and 32 + 4m .. 32 + 4m+3
    const int R = 8 * half + (lane >> 3), m = lane & 7;
    bf16x8_t wf[NTW][2];
#pragma unroll
    for (int ct = 0; ct < NTW; ++ct)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
            wf[ct][ks] = *reinterpret_cast<const bf16x8_t*>(W2d + ((cb + ct) * 16 + r16) * C1 + ks * 32 + 8 * g);
    auto ldrow = [&](const float* row, float* v) {
        const float4 x = ld4(row + 4 * m), y = ld4(row + 32 + 4 * m);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    };
    auto lds8 = [&](const float* row, float* v) {
        const float4 x = *reinterpret_cast<const float4*>(row + 4 * m), y = *reinterpret_cast<const float4*>(row + 32 + 4 * m);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    };
    float2 s1[NTW], s2[NTW];
#pragma unroll
    for (int ct = 0; ct < NTW; ++ct) { s1[ct] = make_float2(0.f, 0.f); s2[ct] = make_float2(0.f, 0.f); }
    const int64_t cbase = (int64_t)b * N;
    const int n0 = tile * EMF_PPB;
    const int np = max(0, min(EMF_PPB, N - n0));  // block-uniform: both waves meet every barrier
    // Per point its KT row tiles are unrolled with the P_j loads one tile
    // ahead (ids of all tiles up front); the next point's Q_i and ids are issued
    // during the current point. The point loop is not unrolled (I-cache).
    int jv[KT];
    float qv[8];
    auto load_ids = [&](int pp) {
        const int64_t i = cbase + n0 + pp;
#pragma unroll
        for (int rt = 0; rt < KT; ++rt) jv[rt] = idx[i * k + min(rt * 16 + R, k - 1)];
    };
    if (np > 0) {
        load_ids(0);
        ldrow(PQ + (cbase + n0) * ldpq + C1, qv);
    }
    int buf = 0;
#pragma unroll 1
    for (int pp = 0; pp < np; ++pp) {
        const int64_t i = cbase + n0 + pp;
        float pb[2][8];
        ldrow(PQ + (cbase + jv[0]) * ldpq, pb[0]);
        float qb[8];
        {
            float a1[8], b1[8];
            lds8(cs[0], a1);
            lds8(cs[1], b1);
#pragma unroll
            for (int u = 0; u < 8; ++u) qb[u] = fmaf(a1[u], qv[u], b1[u]);
        }
        if (pp + 1 < np) ldrow(PQ + (i + 1) * ldpq + C1, qv);
        float best[NTW];
        int barg[NTW];
#pragma unroll
        for (int ct = 0; ct < NTW; ++ct) { best[ct] = -INFINITY; barg[ct] = 0; }
#pragma unroll
        for (int rt = 0; rt < KT; ++rt) {
            if (rt + 1 < KT)
                ldrow(PQ + (cbase + jv[rt + 1]) * ldpq, pb[(rt + 1) & 1]);
            else if (pp + 1 < np)
                load_ids(pp + 1);
            __bf16 hv[8];
            float a1[8];
            lds8(cs[0], a1);
#pragma unroll
            for (int u = 0; u < 8; ++u) hv[u] = (__bf16)lrelu(fmaf(a1[u], pb[rt & 1][u], qb[u]), slope1);
            const uint2 lo = pack4_bf16(hv), hi = pack4_bf16(hv + 4);
            const int sR = rt * 16 + R;
            if (H1 && sR < k) {
                *reinterpret_cast<uint2*>(H1 + (i * k + sR) * C1 + 4 * m) = lo;
                *reinterpret_cast<uint2*>(H1 + (i * k + sR) * C1 + 32 + 4 * m) = hi;
            }
            __bf16* hrow = h1s[buf] + R * HP;
            *reinterpret_cast<uint2*>(hrow + 4 * m) = lo;
            *reinterpret_cast<uint2*>(hrow + 32 + 4 * m) = hi;
            __syncthreads();
            bf16x8_t af[2];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                af[ks] = *reinterpret_cast<const bf16x8_t*>(h1s[buf] + r16 * HP + ks * 32 + 8 * g);
            buf ^= 1;
            f32x4_t acc[NTW];
#pragma unroll
            for (int ct = 0; ct < NTW; ++ct) {
                acc[ct] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
                    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], wf[ct][ks], acc[ct], 0, 0, 0);
            }
            // acc[ct][r]: edge row rt*16 + 4g + r, channel (cb + ct)*16 + r16. Tiles
            // before the last are full; the last masks rows >= k by value.
            const int sb = rt * 16 + 4 * g;
#pragma unroll
            for (int ct = 0; ct < NTW; ++ct) {
                const f32x4_t v = acc[ct];
                float w[4], x[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const bool ok = rt + 1 < KT || sb + r < k;
                    w[r] = ok ? v[r] : 0.f;
                    x[r] = ok ? v[r] : -INFINITY;
                }
                s1[ct].x += w[0] + w[2];
                s1[ct].y += w[1] + w[3];
                s2[ct].x = fmaf(w[0], w[0], fmaf(w[2], w[2], s2[ct].x));
                s2[ct].y = fmaf(w[1], w[1], fmaf(w[3], w[3], s2[ct].y));
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const bool better = x[r] > best[ct];
                    best[ct] = better ? x[r] : best[ct];
                    barg[ct] = better ? sb + r : barg[ct];
                }
            }
        }
        // the four lane groups hold rows 4g.. of the same channel: canonical
        // (larger value, then smaller slot) reduction; group g then writes tile g
#pragma unroll
        for (int ct = 0; ct < NTW; ++ct) {
#pragma unroll
            for (int o = 16; o <= 32; o <<= 1) {
                const float ov = __shfl_xor(best[ct], o);
                const int oa = __shfl_xor(barg[ct], o);
                const bool take = ov > best[ct] || (ov == best[ct] && oa < barg[ct]);
                best[ct] = take ? ov : best[ct];
                barg[ct] = take ? oa : barg[ct];
            }
        }
        if (g < NTW) {
            float bv = best[0];
            int ba = barg[0];
#pragma unroll
            for (int u = 1; u < NTW; ++u) {
                bv = g == u ? best[u] : bv;
                ba = g == u ? barg[u] : ba;
            }
            const int c2 = (cb + g) * 16 + r16;
            ysel[i * C2 + c2] = dir2[c2] * bv;
            arg[i * C2 + c2] = (uint8_t)ba;
        }
    }
    // BN2 partials of this block: lane sums -> over the lane groups; the wave
    // owns its channels, so it writes them directly
    const int prow = b * tiles + tile;
#pragma unroll
    for (int ct = 0; ct < NTW; ++ct) {
        float t1 = s1[ct].x + s1[ct].y, t2 = s2[ct].x + s2[ct].y;
        t1 += __shfl_xor(t1, 16);
        t2 += __shfl_xor(t2, 16);
        t1 += __shfl_xor(t1, 32);
        t2 += __shfl_xor(t2, 32);
        if (g == 0) {
            const int c = (cb + ct) * 16 + r16;
            part[(int64_t)prow * 2 * C2 + c] = dir2[c] * t1;
            part[(int64_t)prow * 2 * C2 + C2 + c] = t2;
        }
    }
}

// ---- fused backward (bf16 mode) of conv2 + LReLU/BN1: per edge row e = (i, s)
//   z2   = W2 h1_e                         (recomputed, h1 rebuilt from P_j, Q_i)
//   dZ2  = c1 z2 + c0 + [arg_i == s] a2 dz_i   (BN2 backward; rounded to bf16
//                                             as the unfused path stores it)
//   dH1  = W2^T dZ2,  g = dH1 LReLU'(z1)  -> gE (bf16) + BN1-backward partials
// with z2 and dZ2 living only in registers: the chain runs TRANSPOSED,
// z2^T = W2 h1^T (A = W2 rows, B = the h1 fragments the forward builds), so
// each lane's z2^T accumulators (4 consecutive c2 of one edge per 16-row tile)
// are, after the BN2 backward and a bf16 pack, exactly the B fragments of
// dH1^T = W2^T dZ2^T when W2^T's K columns are taken in the same permuted c2
// order (wt below): no LDS round trip, no HBM for z2 / dZ2 / dH1.
// A pair of waves (one block) takes EMB_PPB points; wave `half` holds c2 in
// [64 half, 64 half + 64) and forms a partial dH1^T over its c2; the pair adds
// the partials through LDS (double-buffered by tile parity: one barrier per
// tile) and wave `half` finishes c1 tiles 2 half, 2 half + 1.
// dW2 = sum_e dZ2_e h1_e^T is accumulated in the same pass: the tile's dZ2 and
// h1 rows are written to LDS as [edge][channel] and read back with the gfx950
// transposing read (ds_read_b64_tr_b16) as 16x16x16 MFMA operands whose K is
// the 16 edges; wave `half` owns dW2 rows c2 in its half. Blocks of a cloud
// stay on one XCD (its P rows are L2-resident); partial-stat / dW2-slab row =
// block.
constexpr int EMB_PPB = 64;
constexpr int EMB_DZW = (128 + 8) / 2;  // words per LDS dZ2 row (16-bit, padded)
constexpr int EMB_HW = (64 + 8) / 2;    // words per LDS h1 row
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

// Transposed 16x16x16 operand from a row-major [16][*] 16-bit LDS tile: lane
// (g, i) gets t[4 g + q][c0 + i], q = 0..3 (K = tile row, M/N = column). Lane
// 4q + p of a 16-lane group supplies the address of row 4g + q, columns 4p..
__device__ __forceinline__ s16x4_t lds_tr4(const uint32_t* t, int rsw, int c0, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(t + (4 * g + q) * rsw + (c0 + 4 * p) / 2));
}

// One wave of the pair; HALF (the wave's c2 half) is a template constant so
// every register-array index below is static (a runtime half made each such
// access a select chain: ~1100 VALU per tile instead of ~300).
template <int KT, int HALF>
__device__ __forceinline__ void emlp_bwd_wave(
    const float* __restrict__ PQ, int ldpq, const int32_t* __restrict__ idx, int N, int k, int tiles, int b,
    int tile, const float* __restrict__ scale1, float slope1, const __bf16* __restrict__ W2,
    const float* __restrict__ dz, const uint8_t* __restrict__ arg, __bf16* __restrict__ gE,
    float* __restrict__ part1, float* __restrict__ dw2slab, float (*xch)[2][2][4][64],
    uint32_t (*dzt)[16 * EMB_DZW], uint32_t (*h1t)[16 * EMB_HW], const float* cst) {
    constexpr int C1 = 64, C2 = 128, NTW = 4;
    constexpr int half = HALF;
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, r16 = lane & 15;
    // A fragments of W2 (z2^T = W2 h1^T): rows c2 = (4 half + ct) * 16 + r16, K = c1 32 ks + 8 g ..
    bf16x8_t wf[NTW][2];
#pragma unroll
    for (int ct = 0; ct < NTW; ++ct)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
            wf[ct][ks] = *reinterpret_cast<const bf16x8_t*>(W2 + ((4 * half + ct) * 16 + r16) * C1 + ks * 32 + 8 * g);
    // A fragments of W2^T over this wave's c2 half, K slots in the z2^T register
    // order: slot 8 g + t of step kk is c2 = 64 half + 32 kk + 16 (t / 4) + 4 g + t % 4
    bf16x8_t wt[4][2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int t = 0; t < 8; ++t)
                wt[mt][kk][t] = W2[(64 * half + 32 * kk + 16 * (t >> 2) + 4 * g + (t & 3)) * C1 + 16 * mt + r16];
    // h1 build (as emlp_fwd_kernel): channels 32 ks + 8 g + u
    float a1[2][8];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) ld8(scale1 + ks * 32 + 8 * g, a1[ks]);
    float t1[2][4], t2[2][4];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) { t1[jt][r] = 0.f; t2[jt][r] = 0.f; }
    // dW2 rows c2 = 64 half + 16 ct + 4 g + r, columns c1 = 16 nt + r16
    f32x4_t wacc[NTW][4];
#pragma unroll
    for (int ct = 0; ct < NTW; ++ct)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) wacc[ct][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int64_t cbase = (int64_t)b * N;
    const int n0 = tile * EMB_PPB;
    const int np = max(0, min(EMB_PPB, N - n0));
    int par = 0;  // exchange buffer parity
    // Software pipeline: the next tile's P_j rows are loaded during the current
    // tile, the next point's ids / Q_i / dz / slots during the current point
    // (a tile's own gather would otherwise cost two dependent L2 round trips).
    int jv[KT], jn[KT];
    float qr[2][8], qen[2][4];  // next point's raw Q_i (h1 channels, epilogue channels)
    float4 dzn[NTW];
    uint32_t sln[NTW];
    auto load_point = [&](int pp) {
        const int64_t i = cbase + n0 + pp;
#pragma unroll
        for (int rt = 0; rt < KT; ++rt) jn[rt] = idx[i * k + min(rt * 16 + r16, k - 1)];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) ld8(PQ + i * ldpq + C1 + ks * 32 + 8 * g, qr[ks]);
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            const float4 v = ld4(PQ + i * ldpq + C1 + 16 * (2 * half + jt) + 4 * g);
            qen[jt][0] = v.x; qen[jt][1] = v.y; qen[jt][2] = v.z; qen[jt][3] = v.w;
        }
#pragma unroll
        for (int ct = 0; ct < NTW; ++ct) {
            const int c = 64 * half + 16 * ct + 4 * g;
            dzn[ct] = ld4(dz + i * C2 + c);
            sln[ct] = *reinterpret_cast<const uint32_t*>(arg + i * C2 + c);
        }
    };
    float pbn[2][8], pen[2][4];  // next tile's P_j (h1 channels, epilogue channels)
    auto load_p = [&](int j) {
        const float* __restrict__ pj = PQ + (cbase + j) * ldpq;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) ld8(pj + ks * 32 + 8 * g, pbn[ks]);
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            const float4 v = ld4(pj + 16 * (2 * half + jt) + 4 * g);
            pen[jt][0] = v.x; pen[jt][1] = v.y; pen[jt][2] = v.z; pen[jt][3] = v.w;
        }
    };
    float qb[2][8], T[NTW][4], qe[2][4];
    uint32_t sl[NTW];
    if (np > 0) {
        load_point(0);
        load_p(jn[0]);
    }
#pragma unroll 1
    for (int pp = 0; pp < np; ++pp) {
        const int64_t i = cbase + n0 + pp;
        // this point's state from the prefetched raw values
        {
            float b1[2][8];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) ld8(cst + 3 * C2 + C1 + ks * 32 + 8 * g, b1[ks]);  // shift1 (LDS)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int u = 0; u < 8; ++u) qb[ks][u] = fmaf(a1[ks][u], qr[ks][u], b1[ks][u]);
        }
#pragma unroll
        for (int rt = 0; rt < KT; ++rt) jv[rt] = jn[rt];
#pragma unroll
        for (int ct = 0; ct < NTW; ++ct) {
            const float4 a2 = *reinterpret_cast<const float4*>(cst + 2 * C2 + 64 * half + 16 * ct + 4 * g);
            T[ct][0] = a2.x * dzn[ct].x; T[ct][1] = a2.y * dzn[ct].y;
            T[ct][2] = a2.z * dzn[ct].z; T[ct][3] = a2.w * dzn[ct].w;
            sl[ct] = sln[ct];
        }
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
#pragma unroll
            for (int r = 0; r < 4; ++r) qe[jt][r] = qen[jt][r];
        if (pp + 1 < np) load_point(pp + 1);
#pragma unroll
        for (int rt = 0; rt < KT; ++rt) {
            const int s = rt * 16 + r16;
            const bool valid = s < k;
            float pb[2][8], pe[2][4];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int u = 0; u < 8; ++u) pb[ks][u] = pbn[ks][u];
#pragma unroll
            for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                for (int r = 0; r < 4; ++r) pe[jt][r] = pen[jt][r];
            if (rt + 1 < KT) load_p(jv[rt + 1]);
            else if (pp + 1 < np) load_p(jn[0]);
            bf16x8_t af[2];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int u = 0; u < 8; ++u) af[ks][u] = (__bf16)lrelu(fmaf(a1[ks][u], pb[ks][u], qb[ks][u]), slope1);
            // z2^T tiles: acc[ct][r] = z2[edge s][c2 = 64 half + 16 ct + 4 g + r]
            f32x4_t acc[NTW];
#pragma unroll
            for (int ct = 0; ct < NTW; ++ct) {
                acc[ct] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
                    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ct][ks], af[ks], acc[ct], 0, 0, 0);
            }
            // dZ2^T (bf16), packed as the B fragments of step kk = ct / 2
            bf16x8_t dzb[2];
#pragma unroll
            for (int ct = 0; ct < NTW; ++ct) {
                const int c = 64 * half + 16 * ct + 4 * g;
                const float4 v0 = *reinterpret_cast<const float4*>(cst + c);
                const float4 v1 = *reinterpret_cast<const float4*>(cst + C2 + c);
                const float k0[4] = {v0.x, v0.y, v0.z, v0.w}, k1[4] = {v1.x, v1.y, v1.z, v1.w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t slot = (sl[ct] >> (8 * r)) & 0xffu;
                    float d = fmaf(k1[r], acc[ct][r], k0[r]) + (slot == (uint32_t)s ? T[ct][r] : 0.f);
                    d = valid ? d : 0.f;
                    dzb[ct >> 1][4 * (ct & 1) + r] = (__bf16)d;
                }
            }
            // partial dH1^T over this wave's c2: dacc[mt][r] = dH1[edge s][c1 = 16 mt + 4 g + r]
            f32x4_t dacc[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                dacc[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < 2; ++kk)
                    dacc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wt[mt][kk], dzb[kk], dacc[mt], 0, 0, 0);
            }
            // pair exchange: hand the partner its two c1 tiles, take ours; this
            // tile's dZ2 (this wave's c2) and h1 (channels 32 half ..) rows to LDS
#pragma unroll
            for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                for (int r = 0; r < 4; ++r) xch[par][half][jt][r][lane] = dacc[2 * (1 - half) + jt][r];
#pragma unroll
            for (int ct = 0; ct < NTW; ++ct) {
                // whole-vector bit cast (element-wise casts of the bf16 vector miscompile)
                const uint4 w = __builtin_bit_cast(uint4, dzb[ct >> 1]);
                *reinterpret_cast<uint2*>(dzt[par] + r16 * EMB_DZW + (64 * half + 16 * ct + 4 * g) / 2) =
                    (ct & 1) ? make_uint2(w.z, w.w) : make_uint2(w.x, w.y);
            }
            *reinterpret_cast<bf16x8_t*>(h1t[par] + r16 * EMB_HW + (32 * half + 8 * g) / 2) = af[half];
            __syncthreads();
            // dW2 += dZ2^T h1 over the tile's 16 edges (padding edges carry dZ2 = 0)
#pragma unroll
            for (int ct = 0; ct < NTW; ++ct) {
                const s16x4_t a = lds_tr4(dzt[par], EMB_DZW, 64 * half + 16 * ct, lane);
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
                    wacc[ct][nt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, lds_tr4(h1t[par], EMB_HW, 16 * nt, lane),
                                                                           wacc[ct][nt], 0, 0, 0);
            }
            float dh[2][4];
#pragma unroll
            for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                for (int r = 0; r < 4; ++r) dh[jt][r] = dacc[2 * half + jt][r] + xch[par][1 - half][jt][r][lane];
            par ^= 1;
            // g = dH1 LReLU'(z1) -> gE (bf16) and the BN1-backward partials
            if (valid) {
                __bf16* __restrict__ ge = gE + (i * k + s) * C1;
#pragma unroll
                for (int jt = 0; jt < 2; ++jt) {
                    const int c = 16 * (2 * half + jt) + 4 * g;
                    const float4 va = *reinterpret_cast<const float4*>(cst + 3 * C2 + c);
                    const float4 vb = *reinterpret_cast<const float4*>(cst + 3 * C2 + C1 + c);
                    const float4 vm = *reinterpret_cast<const float4*>(cst + 3 * C2 + 2 * C1 + c);
                    const float4 vi = *reinterpret_cast<const float4*>(cst + 3 * C2 + 3 * C1 + c);
                    const float ea[4] = {va.x, va.y, va.z, va.w}, eb[4] = {vb.x, vb.y, vb.z, vb.w};
                    const float em[4] = {vm.x, vm.y, vm.z, vm.w}, ei[4] = {vi.x, vi.y, vi.z, vi.w};
                    bf16x4_t h;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float y = pe[jt][r] + qe[jt][r];
                        const float z = fmaf(ea[r], y, eb[r]);
                        const float gv = dh[jt][r] * (z > 0.f ? 1.f : slope1);
                        t1[jt][r] += gv;
                        t2[jt][r] = fmaf(gv, (y - em[r]) * ei[r], t2[jt][r]);
                        h[r] = (__bf16)gv;
                    }
                    *reinterpret_cast<bf16x4_t*>(ge + 16 * (2 * half + jt) + 4 * g) = h;
                }
            }
        }
    }
    // BN1 partials: sum over the 16 edge lanes, lanes r16 == 0 write
    const int prow = b * tiles + tile;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v1 = t1[jt][r], v2 = t2[jt][r];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                v1 += __shfl_xor(v1, o);
                v2 += __shfl_xor(v2, o);
            }
            if (r16 == 0) {
                const int c = 16 * (2 * half + jt) + 4 * g + r;
                part1[(int64_t)prow * 2 * C1 + c] = v1;
                part1[(int64_t)prow * 2 * C1 + C1 + c] = v2;
            }
        }
    float* __restrict__ ws = dw2slab + (int64_t)prow * C2 * C1;
#pragma unroll
    for (int ct = 0; ct < NTW; ++ct)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) ws[(64 * half + 16 * ct + 4 * g + r) * C1 + 16 * nt + r16] = wacc[ct][nt][r];
}

template <int KT>
__global__ __launch_bounds__(128) void emlp_bwd_kernel(
    const float* __restrict__ PQ, int ldpq, const int32_t* __restrict__ idx, int B, int N, int k, int tiles,
    const float* __restrict__ scale1, const float* __restrict__ shift1, const float* __restrict__ mean1,
    const float* __restrict__ invstd1, float slope1, const __bf16* __restrict__ W2, const float* __restrict__ dz,
    const uint8_t* __restrict__ arg, const float* __restrict__ consts2, __bf16* __restrict__ gE,
    float* __restrict__ part1, float* __restrict__ dw2slab) {
    constexpr int C1 = 64, C2 = 128;
    __shared__ float xch[2][2][2][4][64];  // [tile parity][from wave][its tile j][r][lane]
    __shared__ __attribute__((aligned(16))) uint32_t dzt[2][16 * EMB_DZW];  // [parity][edge][c2] bf16
    __shared__ __attribute__((aligned(16))) uint32_t h1t[2][16 * EMB_HW];   // [parity][edge][c1] bf16
    // block constants in LDS (read back as 4-lane broadcasts): BN2-backward
    // [c0 | c1 | a2] (3 x C2) and BN1 [scale | shift | mean | invstd] (4 x C1)
    __shared__ __attribute__((aligned(16))) float cst[3 * C2 + 4 * C1];
    int b, tile;
    if (!dgx_xcd_cloud_map(blockIdx.x, B, tiles, b, tile)) return;
    for (int t = threadIdx.x; t < 3 * C2; t += 128) cst[t] = consts2[t];
    for (int t = threadIdx.x; t < C1; t += 128) {
        cst[3 * C2 + t] = scale1[t];
        cst[3 * C2 + C1 + t] = shift1[t];
        cst[3 * C2 + 2 * C1 + t] = mean1[t];
        cst[3 * C2 + 3 * C1 + t] = invstd1[t];
    }
    __syncthreads();
    if (threadIdx.x >> 6)
        emlp_bwd_wave<KT, 1>(PQ, ldpq, idx, N, k, tiles, b, tile, scale1, slope1, W2, dz, arg, gE, part1, dw2slab, xch,
                             dzt, h1t, cst);
    else
        emlp_bwd_wave<KT, 0>(PQ, ldpq, idx, N, k, tiles, b, tile, scale1, slope1, W2, dz, arg, gE, part1, dw2slab, xch,
                             dzt, h1t, cst);
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" {

int dgx_edge_mlp_h1_f32(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int C1,
                        const float* scale, const float* shift, float slope, void* H1, int out_bf16, void* stream) {
    if (!PQ || !idx || !scale || !shift || !H1 || B < 1 || N < 1 || k < 1 || C1 < 4 || ldpq < 2 * C1)
        return DGX_EINVAL;
    if (C1 % 8 || ldpq % 4 || !al16(PQ) || !al16(scale) || !al16(shift) || !al16(H1)) return DGX_EUNSUPPORTED;
    const int64_t E = (int64_t)B * N * k;
    const int grid = grid_of(E * (C1 / 8), EM_THREADS);
    if (out_bf16)
        hipLaunchKernelGGL(mlp_h1_kernel<true>, dim3(grid), dim3(EM_THREADS), 0, dgx_stream(stream), PQ, ldpq, idx, N,
                           k, C1, E, scale, shift, slope, H1);
    else
        hipLaunchKernelGGL(mlp_h1_kernel<false>, dim3(grid), dim3(EM_THREADS), 0, dgx_stream(stream), PQ, ldpq, idx,
                           N, k, C1, E, scale, shift, slope, H1);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_mlp_fused_rows(int B, int N) {
    if (B < 1 || N < 1) return DGX_EINVAL;
    return B * ((N + EMF_PPB - 1) / EMF_PPB);
}

int dgx_edge_mlp_fused_fwd_bf16(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int C1, int C2,
                                const float* scale1, const float* shift1, float slope1, const void* W2d,
                                const float* dir2, float* ysel, uint8_t* arg, float* partials, int nrows, void* H1,
                                void* stream) {
    if (!PQ || !idx || !scale1 || !shift1 || !W2d || !dir2 || !ysel || !arg || !partials) return DGX_EINVAL;
    if (B < 1 || N < 1 || k < 1 || ldpq < 2 * C1) return DGX_EINVAL;
    if (C1 != 64 || (C2 != 64 && C2 != 128) || k > 64 || ldpq % 4 || !al16(PQ) || !al16(scale1) || !al16(shift1) ||
        !al16(W2d) || (H1 && !al16(H1)))
        return DGX_EUNSUPPORTED;
    const int tiles = (N + EMF_PPB - 1) / EMF_PPB;
    if (nrows != B * tiles) return DGX_EINVAL;
    const dim3 grid(dgx_xcd_cloud_grid(B, tiles));
    const __bf16* w = static_cast<const __bf16*>(W2d);
    __bf16* h = static_cast<__bf16*>(H1);
    hipStream_t st = dgx_stream(stream);
    const int kt = (k + 15) / 16;
#define DGX_EMF(KTV, NTV)                                                                                        \
    hipLaunchKernelGGL((emlp_fwd_kernel<KTV, NTV / 2>), grid, dim3(128), 0, st, PQ, ldpq, idx, B, N, k, tiles, scale1, \
                       shift1, slope1, w, dir2, ysel, arg, partials, h)
    if (C2 == 128) {
        switch (kt) {
            case 1: DGX_EMF(1, 8); break;
            case 2: DGX_EMF(2, 8); break;
            case 3: DGX_EMF(3, 8); break;
            default: DGX_EMF(4, 8); break;
        }
    } else {
        switch (kt) {
            case 1: DGX_EMF(1, 4); break;
            case 2: DGX_EMF(2, 4); break;
            case 3: DGX_EMF(3, 4); break;
            default: DGX_EMF(4, 4); break;
        }
    }
#undef DGX_EMF
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_mlp_fused_bwd_rows(int B, int N) {
    if (B < 1 || N < 1) return DGX_EINVAL;
    return B * ((N + EMB_PPB - 1) / EMB_PPB);
}

int dgx_edge_mlp_fused_bwd_bf16(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int C1, int C2,
                                const float* scale1, const float* shift1, const float* mean1, const float* invstd1,
                                float slope1, const void* W2, const float* dz, const uint8_t* arg,
                                const float* consts2, void* gE, float* part1, float* dw2slab, int nrows,
                                void* stream) {
    if (!PQ || !idx || !scale1 || !shift1 || !mean1 || !invstd1 || !W2 || !dz || !arg || !consts2 || !gE || !part1 ||
        !dw2slab)
        return DGX_EINVAL;
    if (B < 1 || N < 1 || k < 1 || ldpq < 2 * C1) return DGX_EINVAL;
    if (C1 != 64 || C2 != 128 || k > 64 || ldpq % 4 || !al16(PQ) || !al16(scale1) || !al16(shift1) || !al16(mean1) ||
        !al16(invstd1) || !al16(W2) || !al16(dz) || !al16(consts2) || (reinterpret_cast<uintptr_t>(arg) & 3) ||
        (reinterpret_cast<uintptr_t>(gE) & 7))
        return DGX_EUNSUPPORTED;
    const int tiles = (N + EMB_PPB - 1) / EMB_PPB;
    if (nrows != B * tiles) return DGX_EINVAL;
    const dim3 grid(dgx_xcd_cloud_grid(B, tiles));
    const __bf16* w = static_cast<const __bf16*>(W2);
    __bf16* ge = static_cast<__bf16*>(gE);
    hipStream_t st = dgx_stream(stream);
#define DGX_EMB(KTV)                                                                                              \
    hipLaunchKernelGGL((emlp_bwd_kernel<KTV>), grid, dim3(128), 0, st, PQ, ldpq, idx, B, N, k, tiles, scale1, shift1, \
                       mean1, invstd1, slope1, w, dz, arg, consts2, ge, part1, dw2slab)
    switch ((k + 15) / 16) {
        case 1: DGX_EMB(1); break;
        case 2: DGX_EMB(2); break;
        case 3: DGX_EMB(3); break;
        default: DGX_EMB(4); break;
    }
#undef DGX_EMB
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_mlp_max_f32(const void* Z, int z_bf16, int B, int N, int k, int C2, const float* scale, float* ysel,
                         uint8_t* arg, void* stream) {
    if (!Z || !scale || !ysel || !arg || B < 1 || N < 1 || k < 1 || k > 64 || C2 < 4) return DGX_EINVAL;
    if (C2 % 8 || !al16(Z) || !al16(scale) || !al16(ysel) || (reinterpret_cast<uintptr_t>(arg) & 7))
        return DGX_EUNSUPPORTED;
    const int64_t M = (int64_t)B * N;
    const int grid = grid_of(M * (C2 / 8), EM_THREADS);
    if (z_bf16)
        hipLaunchKernelGGL(mlp_max_kernel<true>, dim3(grid), dim3(EM_THREADS), 0, dgx_stream(stream), Z, M, k, C2,
                           scale, ysel, arg);
    else
        hipLaunchKernelGGL(mlp_max_kernel<false>, dim3(grid), dim3(EM_THREADS), 0, dgx_stream(stream), Z, M, k, C2,
                           scale, ysel, arg);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_mlp_dz_f32(const float* dz, const uint8_t* arg, const void* Z, int bf16, int B, int N, int k, int C2,
                        const float* scale, const float* c0, const float* c1, void* dZ, void* stream) {
    if (!dz || !arg || !Z || !scale || !c0 || !c1 || !dZ || B < 1 || N < 1 || k < 1 || k > 255 || C2 < 4)
        return DGX_EINVAL;
    if (C2 % 8 || !al16(dz) || !al16(Z) || !al16(dZ) || !al16(scale) || !al16(c0) || !al16(c1) ||
        reinterpret_cast<uintptr_t>(arg) % 8)
        return DGX_EUNSUPPORTED;
    const int64_t M = (int64_t)B * N;
    const int grid = grid_of(M * (C2 / 8), EM_THREADS);
    if (bf16)
        hipLaunchKernelGGL(mlp_dz2_kernel<true>, dim3(grid), dim3(EM_THREADS), 0, dgx_stream(stream), dz, arg, Z, M, k,
                           C2, scale, c0, c1, dZ);
    else
        hipLaunchKernelGGL(mlp_dz2_kernel<false>, dim3(grid), dim3(EM_THREADS), 0, dgx_stream(stream), dz, arg, Z, M, k,
                           C2, scale, c0, c1, dZ);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_mlp_h1_bwd_rows(int B, int N, int k, int C1) {
    if (B < 1 || N < 1 || k < 1 || C1 < 4) return DGX_EINVAL;
    const int64_t E = (int64_t)B * N * k;
    const int epb = EM_THREADS / (C1 / 4 > 0 ? C1 / 4 : 1);
    int64_t rows = (E + epb * 8 - 1) / (epb * 8);  // ~8 edge rows per thread
    return (int)(rows < 1 ? 1 : (rows > 2048 ? 2048 : rows));
}

int dgx_edge_mlp_h1_bwd_f32(float* dH, const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int C1,
                            const float* scale, const float* shift, const float* mean, const float* invstd,
                            float slope, float* partials, int nrows, void* stream) {
    if (!dH || !PQ || !idx || !scale || !shift || !mean || !invstd || !partials || B < 1 || N < 1 || k < 1 ||
        ldpq < 2 * C1 || nrows != dgx_edge_mlp_h1_bwd_rows(B, N, k, C1))
        return DGX_EINVAL;
    // fixed channel quads per thread: C1/4 must divide the block
    if (C1 % 4 || EM_THREADS % (C1 / 4) || ldpq % 4 || !al16(dH) || !al16(PQ) || !al16(scale) || !al16(shift) ||
        !al16(mean) || !al16(invstd))
        return DGX_EUNSUPPORTED;
    const int64_t E = (int64_t)B * N * k;
    hipLaunchKernelGGL(mlp_h1_bwd_kernel, dim3(nrows), dim3(EM_THREADS), 0, dgx_stream(stream), dH, PQ, ldpq, idx, N,
                       k, C1, E, scale, shift, mean, invstd, slope, partials);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_mlp_scatter_f32(const void* g, int g_bf16, const float* PQ, int ldpq, const float* sumP,
                             const int32_t* rowptr, const int32_t* edges, int B, int N, int k, int C1,
                             const float* scale, const float* c0, const float* c1, float* dPQ, void* stream) {
    if (!g || !PQ || !sumP || !rowptr || !edges || !scale || !c0 || !c1 || !dPQ || B < 1 || N < 1 || k < 1 ||
        k > 64 || C1 < 1 || ldpq < 2 * C1)
        return DGX_EINVAL;
    const int64_t M = (int64_t)B * N;
    const int64_t blocks = (M + EM_THREADS / 64 - 1) / (EM_THREADS / 64);
    if (blocks > 0x7fffffff) return DGX_EUNSUPPORTED;
    if (g_bf16 && C1 == 64 && ldpq % 4 == 0 && al16(g) && al16(PQ) && al16(sumP) && al16(scale) && al16(c0) &&
        al16(c1) && al16(dPQ)) {
        constexpr int LPP = 16, PPB = EM_THREADS / LPP;
        const int tiles = (N + PPB - 1) / PPB;
        hipLaunchKernelGGL((mlp_h1_scatter4_kernel<4, LPP>), dim3(dgx_xcd_cloud_grid(B, tiles)), dim3(EM_THREADS), 0,
                           dgx_stream(stream), static_cast<const __bf16*>(g), PQ, ldpq, sumP, rowptr, edges, B, N, tiles, k,
                           scale, c0, c1, dPQ);
    } else if (g_bf16)
        hipLaunchKernelGGL(mlp_h1_scatter_kernel<__bf16>, dim3((unsigned)blocks), dim3(EM_THREADS), 0,
                           dgx_stream(stream), static_cast<const __bf16*>(g), PQ, ldpq, sumP, rowptr, edges, M, k, C1,
                           scale, c0, c1, dPQ);
    else
        hipLaunchKernelGGL(mlp_h1_scatter_kernel<float>, dim3((unsigned)blocks), dim3(EM_THREADS), 0,
                           dgx_stream(stream), static_cast<const float*>(g), PQ, ldpq, sumP, rowptr, edges, M, k, C1,
                           scale, c0, c1, dPQ);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

}  // extern "C"
