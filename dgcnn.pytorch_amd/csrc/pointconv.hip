// a4 — pointwise Conv(1x1) + BatchNorm + LeakyReLU on point-major features
// (reference models/dgcnn.py:74-78, 100-102: conv5 over cat(x1..x4)).
//
// The GEMM Z = X W^T (M x Co, M = B*N points) is done by the caller; these
// kernels are the memory-bound rest, each one pass over Z:
//   colstats   per-row-block partial (sum z, sum z^2) per channel -> the
//              shared bn_finalize (edgeconv.hip) turns them into a, b.
//   apply_T    out(b, o, n) = LeakyReLU(a_o z(b*N+n, o) + b_o), transposed
//              through a 64x64 LDS tile so both the point-major read and the
//              channel-major (B,Co,N) write of the reference layout coalesce.
//   bwd_T      dz = dout * LeakyReLU'(a z + b) read from (B,Co,N), written
//              point-major, + partial (sum dz, sum dz*zhat)   [tile transpose]
//   bwd_dZ     dZ = a*dz + c0 + c1*z (BN train-mode input gradient), written
//              fp32 or bf16 (the operand of the caller's two weight GEMMs).
#include "common.h"

namespace {

constexpr int PT = 64;  // tile edge (points x channels)

__device__ __forceinline__ float lrelu(float v, float slope) { return v > 0.f ? v : v * slope; }

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// grid (nrows, ceil(C/64)), block 256: lanes over 64 channels, 4 waves over rows
__global__ __launch_bounds__(256) void colstats_kernel(const float* __restrict__ Z, int ldz, int64_t M, int C,
                                                       int rows_per_blk, float* __restrict__ partials) {
    __shared__ float red[2][4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int o = blockIdx.y * 64 + lane;
    float s1 = 0.f, s2 = 0.f;
    if (o < C) {
        const int64_t i0 = (int64_t)blockIdx.x * rows_per_blk;
        for (int r = wave; r < rows_per_blk; r += 4) {
            const int64_t i = i0 + r;
            if (i >= M) break;
            const float z = Z[i * ldz + o];
            s1 += z;
            s2 = fmaf(z, z, s2);
        }
    }
    red[0][wave][lane] = s1;
    red[1][wave][lane] = s2;
    __syncthreads();
    if (wave == 0 && o < C) {
        partials[(int64_t)blockIdx.x * 2 * C + o] = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
        partials[(int64_t)blockIdx.x * 2 * C + C + o] = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
    }
}

// grid (B * ceil(N/64), ceil(C/64)), block 256
__global__ __launch_bounds__(256) void apply_T_kernel(const float* __restrict__ Z, int ldz, int N, int C,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift, float slope,
                                                      float* __restrict__ out) {
    __shared__ float tile[PT][PT + 1];
    const int ntile = (N + PT - 1) / PT;
    const int b = blockIdx.x / ntile, n0 = (blockIdx.x - b * ntile) * PT, o0 = blockIdx.y * PT;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int o = o0 + tx;
    const float a = o < C ? scale[o] : 0.f, sh = o < C ? shift[o] : 0.f;
    for (int r = ty; r < PT; r += 4) {  // read 64 points x 64 channels, channel-contiguous
        const int n = n0 + r;
        tile[r][tx] = (n < N && o < C) ? lrelu(fmaf(a, Z[((int64_t)b * N + n) * ldz + o], sh), slope) : 0.f;
    }
    __syncthreads();
    for (int r = ty; r < PT; r += 4) {  // write channel rows, point-contiguous
        const int oo = o0 + r, n = n0 + tx;
        if (oo < C && n < N) out[((int64_t)b * C + oo) * N + n] = tile[tx][r];
    }
}

// dz (point-major) from dout (B,C,N); partial row = blockIdx.x (one 64-point tile)
__global__ __launch_bounds__(256) void bwd_T_kernel(const float* __restrict__ dout, const float* __restrict__ Z,
                                                    int ldz, int N, int C, const float* __restrict__ scale,
                                                    const float* __restrict__ shift,
                                                    const float* __restrict__ mean,
                                                    const float* __restrict__ invstd, float slope,
                                                    float* __restrict__ dz, float* __restrict__ partials) {
    __shared__ float tile[PT][PT + 1];
    __shared__ float red[2][4][64];
    const int ntile = (N + PT - 1) / PT;
    const int b = blockIdx.x / ntile, n0 = (blockIdx.x - b * ntile) * PT, o0 = blockIdx.y * PT;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < PT; r += 4) {  // dout rows: channel o0+r, points n0..n0+63
        const int oo = o0 + r, n = n0 + tx;
        tile[tx][r] = (oo < C && n < N) ? dout[((int64_t)b * C + oo) * N + n] : 0.f;
    }
    __syncthreads();
    const int o = o0 + tx;
    float s1 = 0.f, s2 = 0.f;
    if (o < C) {
        const float a = scale[o], sh = shift[o], mu = mean[o], is = invstd[o];
        for (int r = ty; r < PT; r += 4) {
            const int n = n0 + r;
            if (n >= N) break;
            const int64_t i = (int64_t)b * N + n;
            const float z = Z[i * ldz + o];
            const float d = tile[r][tx] * (fmaf(a, z, sh) > 0.f ? 1.f : slope);
            dz[i * C + o] = d;
            s1 += d;
            s2 = fmaf(d, (z - mu) * is, s2);
        }
    }
    red[0][ty][tx] = s1;
    red[1][ty][tx] = s2;
    __syncthreads();
    if (ty == 0 && o < C) {
        partials[(int64_t)blockIdx.x * 2 * C + o] = red[0][0][tx] + red[0][1][tx] + red[0][2][tx] + red[0][3][tx];
        partials[(int64_t)blockIdx.x * 2 * C + C + o] = red[1][0][tx] + red[1][1][tx] + red[1][2][tx] + red[1][3][tx];
    }
}

template <bool BF16>
__global__ void bwd_dZ_kernel(const float* __restrict__ dz, const float* __restrict__ Z, int ldz, int64_t M, int C,
                              const float* __restrict__ scale, const float* __restrict__ c0,
                              const float* __restrict__ c1, void* __restrict__ dZ) {
    const int64_t total = M * C;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int o = (int)(t % C);
        const int64_t i = t / C;
        const float v = fmaf(scale[o], dz[t], fmaf(c1[o], Z[i * ldz + o], c0[o]));
        if (BF16) static_cast<uint16_t*>(dZ)[t] = f32_to_bf16_rne(v);
        else static_cast<float*>(dZ)[t] = v;
    }
}

// fp32 -> bf16 (RNE) copy of a strided row-major matrix into a dense one
__global__ void to_bf16_kernel(const float* __restrict__ src, int64_t lds_, int64_t rows, int cols,
                               uint16_t* __restrict__ dst) {
    const int64_t total = rows * cols;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / cols;
        const int c = (int)(t - r * cols);
        dst[t] = f32_to_bf16_rne(src[r * lds_ + c]);
    }
}

// ---- bf16 Z (precision "bf16": the conv5 GEMM stores Z as bf16, as autocast
// stores a conv output; statistics come from the fp32 accumulators) ----------
typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int RT_P = 128;  // points per block



// 4 consecutive points of channel row `oo` of a (B,C,N) fp32 tensor
__device__ __forceinline__ float4 load_row4(const float* __restrict__ p, int64_t rowbase, int n, int N, bool ok) {
    if (!ok || n >= N) return make_float4(0.f, 0.f, 0.f, 0.f);
    if ((N % 4) == 0) return *reinterpret_cast<const float4*>(p + rowbase + n);
    float v[4];
    for (int i = 0; i < 4; ++i) v[i] = n + i < N ? p[rowbase + n + i] : 0.f;
    return make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void store_row4(float* __restrict__ p, int64_t rowbase, int n, int N, const float (&v)[4]) {
    if (n >= N) return;
    if ((N % 4) == 0) {
        *reinterpret_cast<float4*>(p + rowbase + n) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
        for (int i = 0; i < 4 && n + i < N; ++i) p[rowbase + n + i] = v[i];
    }
}

// LDS-transposed tiles (128 points x 64 channels per block, 4 waves). Z / dZ
// (point-major bf16) move as 16-B row pieces of the tile through LDS; dout /
// out ((B,C,N) fp32) move with lanes along the points: lane = (pg = lane & 31,
// half = lane >> 5), thread owns points 4pg..4pg+3 and channels 8cg..8cg+7 with
// cg = 2*wave + half, so a wave-instruction covers 2 channel rows x 512
// contiguous bytes. The Z tile's 16-B chunk c of row r sits at c ^ ((r>>2)&7):
// the per-thread 16-B reads of rows 4pg+i are bank-conflict-free.
constexpr int ZT_LD = 72;  // bf16 per LDS row (64 + 8 pad)

struct ZTile {
    int b, n0, o0, pg, cg;
    __device__ __forceinline__ explicit ZTile(int N) {
        const int nt = (N + RT_P - 1) / RT_P;
        const int bt = blockIdx.x;
        b = bt / nt;
        n0 = (bt - b * nt) * RT_P;
        o0 = blockIdx.y * 64;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        pg = lane & 31;
        cg = 2 * w + (lane >> 5);
    }
};

__device__ __forceinline__ int zt_off(int row, int chunk) { return row * ZT_LD + ((chunk ^ ((row >> 2) & 7)) << 3); }

// rows [n0, n0+128) x channels [o0, o0+64) of Z into zt (zeros outside)
__device__ __forceinline__ void stage_ztile(const bf16* __restrict__ Z, int b, int n0, int o0, int N, int C,
                                            bf16* zt) {
    for (int e = threadIdx.x; e < RT_P * 8; e += 256) {
        const int row = e >> 3, ch = e & 7;
        const int n = n0 + row, o = o0 + 8 * ch;
        bf16x8 v;
        if (n < N && o + 8 <= C && (C % 8) == 0) {
            v = *reinterpret_cast<const bf16x8*>(Z + ((int64_t)b * N + n) * C + o);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (n < N && o + j < C) ? Z[((int64_t)b * N + n) * C + o + j] : (bf16)0.f;
        }
        *reinterpret_cast<bf16x8*>(zt + zt_off(row, ch)) = v;
    }
}

__device__ __forceinline__ void read_z48(const bf16* zt, int pg, int cg, float (&z)[4][8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(zt + zt_off(4 * pg + i, cg));
#pragma unroll
        for (int j = 0; j < 8; ++j) z[i][j] = (float)v[j];
    }
}

// out(b, o, n) = LeakyReLU(a_o z + b_o)
__global__ __launch_bounds__(256) void apply16_lt_kernel(const bf16* __restrict__ Z, int N, int C,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, float slope,
                                                         float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) bf16 zt[RT_P * ZT_LD];
    const ZTile T(N);
    stage_ztile(Z, T.b, T.n0, T.o0, N, C, zt);
    __syncthreads();
    float z[4][8];
    read_z48(zt, T.pg, T.cg, z);
    const int n = T.n0 + 4 * T.pg;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int oo = T.o0 + 8 * T.cg + j;
        if (oo >= C) break;
        const float a = scale[oo], sh = shift[oo];
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = lrelu(fmaf(a, z[i][j], sh), slope);
        store_row4(out, ((int64_t)T.b * C + oo) * N, n, N, v);
    }
}

// PASS 1 of the BN backward with the transposed tile: dZ = a d + c0 + c1 z,
// d = dout * LeakyReLU'(a z + b); dZ goes back through the LDS tile so the
// point-major bf16 rows are written as 16-B pieces.
__global__ __launch_bounds__(256) void bwd16_dz_lt_kernel(const float* __restrict__ dout, const bf16* __restrict__ Z,
                                                          int N, int C, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, float slope,
                                                          const float* __restrict__ c0, const float* __restrict__ c1,
                                                          bf16* __restrict__ dZ) {
    __shared__ __attribute__((aligned(16))) bf16 zt[RT_P * ZT_LD];
    const ZTile T(N);
    const int n = T.n0 + 4 * T.pg;
    float g[8][4];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int oo = T.o0 + 8 * T.cg + j;
        const float4 v = load_row4(dout, ((int64_t)T.b * C + oo) * N, n, N, oo < C);
        g[j][0] = v.x; g[j][1] = v.y; g[j][2] = v.z; g[j][3] = v.w;
    }
    stage_ztile(Z, T.b, T.n0, T.o0, N, C, zt);
    __syncthreads();
    float z[4][8];
    read_z48(zt, T.pg, T.cg, z);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int oo = min(T.o0 + 8 * T.cg + j, C - 1);
        const float a = scale[oo], sh = shift[oo], k0 = c0[oo], k1 = c1[oo];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float d = g[j][i] * (fmaf(a, z[i][j], sh) > 0.f ? 1.f : slope);
            z[i][j] = fmaf(a, d, fmaf(k1, z[i][j], k0));
        }
    }
    __syncthreads();  // every thread has read its Z values
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        bf16x8 w;
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = (bf16)z[i][j];
        *reinterpret_cast<bf16x8*>(zt + zt_off(4 * T.pg + i, T.cg)) = w;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < RT_P * 8; e += 256) {
        const int row = e >> 3, ch = e & 7;
        const int nn = T.n0 + row, o = T.o0 + 8 * ch;
        if (nn >= N) continue;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(zt + zt_off(row, ch));
        bf16* dst = dZ + ((int64_t)T.b * N + nn) * C + o;
        if (o + 8 <= C && (C % 8) == 0) {
            *reinterpret_cast<bf16x8*>(dst) = v;
        } else {
            for (int j = 0; j < 8 && o + j < C; ++j) dst[j] = v[j];
        }
    }
}

// PASS 0 with the transposed tile over RS_LT consecutive 128-point tiles per
// block: per-thread sums over its 4 points, then over the 32 lanes of its
// channel group (one shuffle tree), one partial row per block.
constexpr int RS_LT = 2;
__global__ __launch_bounds__(256, 4) void bwd16_stats_lt_kernel(const float* __restrict__ dout,
                                                             const bf16* __restrict__ Z, int N, int C,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd, float slope,
                                                             float* __restrict__ partials) {
    __shared__ __attribute__((aligned(16))) bf16 zt[RT_P * ZT_LD];
    __shared__ __attribute__((aligned(16))) float4 cst[64];   // per channel {scale, shift, mean, invstd}
    const int nt = (N + RT_P * RS_LT - 1) / (RT_P * RS_LT);
    const int b = blockIdx.x / nt;
    const int nb = (blockIdx.x - b * nt) * RT_P * RS_LT;
    const int o0 = blockIdx.y * 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int pg = lane & 31, cg = 2 * w + (lane >> 5);
    if (threadIdx.x < 64) {
        const int oj = min(o0 + (int)threadIdx.x, C - 1);
        cst[threadIdx.x] = make_float4(scale[oj], shift[oj], mean[oj], invstd[oj]);
    }
    // the channel constants come from LDS at each use (they would hold 32 VGPRs)
    float s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        s1[j] = 0.f;
        s2[j] = 0.f;
    }
#pragma unroll 1
    for (int it = 0; it < RS_LT; ++it) {
        const int n0 = nb + it * RT_P;
        if (n0 >= N) break;
        const int n = n0 + 4 * pg;
        float g[8][4];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int oo = o0 + 8 * cg + j;
            const float4 v = load_row4(dout, ((int64_t)b * C + oo) * N, n, N, oo < C);
            g[j][0] = v.x; g[j][1] = v.y; g[j][2] = v.z; g[j][3] = v.w;
        }
        if (it > 0) __syncthreads();  // previous tile's reads done (a barrier here would also wait for the dout loads)
        stage_ztile(Z, b, n0, o0, N, C, zt);
        __syncthreads();
        float z[4][8];
        read_z48(zt, pg, cg, z);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float4 k4 = cst[8 * cg + j];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float d = g[j][i] * (fmaf(k4.x, z[i][j], k4.y) > 0.f ? 1.f : slope);
                s1[j] += d;
                s2[j] = fmaf(d, (z[i][j] - k4.z) * k4.w, s2[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int m = 1; m < 32; m <<= 1) {
            s1[j] += __shfl_xor(s1[j], m);
            s2[j] += __shfl_xor(s2[j], m);
        }
    }
    if (pg == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int oo = o0 + 8 * cg + j;
            if (oo < C) {
                partials[(int64_t)blockIdx.x * 2 * C + oo] = s1[j];
                partials[(int64_t)blockIdx.x * 2 * C + C + oo] = s2[j];
            }
        }
    }
}

// ---- fp32 Z (precision "fp32"): the same LDS-transposed tiles, 128 points x
// 64 channels x 4 B; a row is 16 chunks of 16 B, chunk c of row r stored at
// c ^ ((r >> 2) & 7), so the per-thread 16-B reads of rows 4pg+i (and the
// staging writes of one row) fall in distinct bank groups. ------------------
__device__ __forceinline__ int zt32_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 7)) << 2); }

__device__ __forceinline__ void stage_ztile32(const float* __restrict__ Z, int b, int n0, int o0, int N, int C,
                                              float* zt) {
    for (int e = threadIdx.x; e < RT_P * 16; e += 256) {
        const int row = e >> 4, ch = e & 15;
        const int n = n0 + row, o = o0 + 4 * ch;
        float4 v;
        if (n < N && o + 4 <= C && (C % 4) == 0) {
            v = *reinterpret_cast<const float4*>(Z + ((int64_t)b * N + n) * C + o);
        } else {
            float t[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) t[j] = (n < N && o + j < C) ? Z[((int64_t)b * N + n) * C + o + j] : 0.f;
            v = make_float4(t[0], t[1], t[2], t[3]);
        }
        *reinterpret_cast<float4*>(zt + zt32_off(row, ch)) = v;
    }
}

__device__ __forceinline__ void read_z48_32(const float* zt, int pg, int cg, float (&z)[4][8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float4 v = *reinterpret_cast<const float4*>(zt + zt32_off(4 * pg + i, 2 * cg + h));
            z[i][4 * h] = v.x; z[i][4 * h + 1] = v.y; z[i][4 * h + 2] = v.z; z[i][4 * h + 3] = v.w;
        }
}

// out(b, o, n) = LeakyReLU(a_o z + b_o), fp32 Z
__global__ __launch_bounds__(256) void apply32_lt_kernel(const float* __restrict__ Z, int N, int C,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, float slope,
                                                         float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float zt[RT_P * 64];
    const ZTile T(N);
    stage_ztile32(Z, T.b, T.n0, T.o0, N, C, zt);
    __syncthreads();
    float z[4][8];
    read_z48_32(zt, T.pg, T.cg, z);
    const int n = T.n0 + 4 * T.pg;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int oo = T.o0 + 8 * T.cg + j;
        if (oo >= C) break;
        const float a = scale[oo], sh = shift[oo];
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = lrelu(fmaf(a, z[i][j], sh), slope);
        store_row4(out, ((int64_t)T.b * C + oo) * N, n, N, v);
    }
}

// PASS 0 (fp32 Z): as bwd16_stats_lt_kernel
__global__ __launch_bounds__(256, 4) void bwd32_stats_lt_kernel(const float* __restrict__ dout,
                                                             const float* __restrict__ Z, int N, int C,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd, float slope,
                                                             float* __restrict__ partials) {
    __shared__ __attribute__((aligned(16))) float zt[RT_P * 64];
    __shared__ __attribute__((aligned(16))) float4 cst[64];   // per channel {scale, shift, mean, invstd}
    const int nt = (N + RT_P * RS_LT - 1) / (RT_P * RS_LT);
    const int b = blockIdx.x / nt;
    const int nb = (blockIdx.x - b * nt) * RT_P * RS_LT;
    const int o0 = blockIdx.y * 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int pg = lane & 31, cg = 2 * w + (lane >> 5);
    if (threadIdx.x < 64) {
        const int oj = min(o0 + (int)threadIdx.x, C - 1);
        cst[threadIdx.x] = make_float4(scale[oj], shift[oj], mean[oj], invstd[oj]);
    }
    float s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        s1[j] = 0.f;
        s2[j] = 0.f;
    }
#pragma unroll 1
    for (int it = 0; it < RS_LT; ++it) {
        const int n0 = nb + it * RT_P;
        if (n0 >= N) break;
        const int n = n0 + 4 * pg;
        float g[8][4];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int oo = o0 + 8 * cg + j;
            const float4 v = load_row4(dout, ((int64_t)b * C + oo) * N, n, N, oo < C);
            g[j][0] = v.x; g[j][1] = v.y; g[j][2] = v.z; g[j][3] = v.w;
        }
        if (it > 0) __syncthreads();
        stage_ztile32(Z, b, n0, o0, N, C, zt);
        __syncthreads();
        float z[4][8];
        read_z48_32(zt, pg, cg, z);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float4 k4 = cst[8 * cg + j];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float d = g[j][i] * (fmaf(k4.x, z[i][j], k4.y) > 0.f ? 1.f : slope);
                s1[j] += d;
                s2[j] = fmaf(d, (z[i][j] - k4.z) * k4.w, s2[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int m = 1; m < 32; m <<= 1) {
            s1[j] += __shfl_xor(s1[j], m);
            s2[j] += __shfl_xor(s2[j], m);
        }
    }
    if (pg == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int oo = o0 + 8 * cg + j;
            if (oo < C) {
                partials[(int64_t)blockIdx.x * 2 * C + oo] = s1[j];
                partials[(int64_t)blockIdx.x * 2 * C + C + oo] = s2[j];
            }
        }
    }
}

// PASS 1 (fp32 Z) straight into the split-bf16 operand planes of the 3-pass
// GEMMs: v = a d + c0 + c1 z (the fp32 dZ of bwd_dZ_kernel), hi = bf16(v),
// lo = bf16(v - hi) (dgx_split_bf16), written point-major through the tile.
__global__ __launch_bounds__(256) void bwd32_split_lt_kernel(const float* __restrict__ dout,
                                                             const float* __restrict__ Z, int N, int C,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, float slope,
                                                             const float* __restrict__ c0,
                                                             const float* __restrict__ c1, bf16* __restrict__ hi,
                                                             bf16* __restrict__ lo) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) float zt[RT_P * 64];
    const ZTile T(N);
    const int n = T.n0 + 4 * T.pg;
    float g[8][4];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int oo = T.o0 + 8 * T.cg + j;
        const float4 v = load_row4(dout, ((int64_t)T.b * C + oo) * N, n, N, oo < C);
        g[j][0] = v.x; g[j][1] = v.y; g[j][2] = v.z; g[j][3] = v.w;
    }
    stage_ztile32(Z, T.b, T.n0, T.o0, N, C, zt);
    __syncthreads();
    float z[4][8];
    read_z48_32(zt, T.pg, T.cg, z);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int oo = min(T.o0 + 8 * T.cg + j, C - 1);
        const float a = scale[oo], sh = shift[oo], k0 = c0[oo], k1 = c1[oo];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float d = g[j][i] * (fmaf(a, z[i][j], sh) > 0.f ? 1.f : slope);
            z[i][j] = fmaf(a, d, fmaf(k1, z[i][j], k0));
        }
    }
    __syncthreads();  // every thread has read its Z values
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h)
            *reinterpret_cast<float4*>(zt + zt32_off(4 * T.pg + i, 2 * T.cg + h)) =
                make_float4(z[i][4 * h], z[i][4 * h + 1], z[i][4 * h + 2], z[i][4 * h + 3]);
    __syncthreads();
    for (int e = threadIdx.x; e < RT_P * 16; e += 256) {
        const int row = e >> 4, ch = e & 15;
        const int nn = T.n0 + row, o = T.o0 + 4 * ch;
        if (nn >= N) continue;
        const float4 v = *reinterpret_cast<const float4*>(zt + zt32_off(row, ch));
        const float f[4] = {v.x, v.y, v.z, v.w};
        bf16x4 h, l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            h[j] = (bf16)f[j];
            l[j] = (bf16)(f[j] - (float)h[j]);
        }
        const int64_t off = ((int64_t)T.b * N + nn) * C + o;
        if (o + 4 <= C && (C % 4) == 0) {
            *reinterpret_cast<bf16x4*>(hi + off) = h;
            *reinterpret_cast<bf16x4*>(lo + off) = l;
        } else {
            for (int j = 0; j < 4 && o + j < C; ++j) {
                hi[off + j] = h[j];
                lo[off + j] = l[j];
            }
        }
    }
}

inline int grid_for(int64_t total, int block) {
    int64_t g = (total + block - 1) / block;
    return (int)(g < 16384 ? (g < 1 ? 1 : g) : 16384);
}

}  // namespace

extern "C" {

int dgx_colstats_rows(int64_t M) {
    if (M < 1) return DGX_EINVAL;
    return (int)((M + 127) / 128);
}

int dgx_colstats_f32(const float* Z, int ldz, int64_t M, int C, float* partials, int nrows, void* stream) {
    if (!Z || !partials || M < 1 || C < 1 || ldz < C || nrows != dgx_colstats_rows(M)) return DGX_EINVAL;
    hipLaunchKernelGGL(colstats_kernel, dim3(nrows, (C + 63) / 64), dim3(256), 0, dgx_stream(stream), Z, ldz, M, C,
                       128, partials);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_pointconv_apply_f32(const float* Z, int ldz, int B, int N, int C, const float* scale, const float* shift,
                              float slope, float* out, void* stream) {
    if (!Z || !scale || !shift || !out || B < 1 || N < 1 || C < 1 || ldz < C) return DGX_EINVAL;
    if (ldz == C && C % 4 == 0 && (reinterpret_cast<uintptr_t>(Z) & 15) == 0) {   // dense rows: 128-point LDS tiles
        hipLaunchKernelGGL(apply32_lt_kernel, dim3(B * ((N + RT_P - 1) / RT_P), (C + 63) / 64), dim3(256), 0,
                           dgx_stream(stream), Z, N, C, scale, shift, slope, out);
        return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
    }
    dim3 grid(B * ((N + PT - 1) / PT), (C + PT - 1) / PT);
    hipLaunchKernelGGL(apply_T_kernel, grid, dim3(256), 0, dgx_stream(stream), Z, ldz, N, C, scale, shift, slope, out);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_pointconv_bwd_rows(int B, int N) {
    if (B < 1 || N < 1) return DGX_EINVAL;
    return B * ((N + PT - 1) / PT);
}

int dgx_pointconv_bwd_f32(const float* dout, const float* Z, int ldz, int B, int N, int C, const float* scale,
                            const float* shift, const float* mean, const float* invstd, float slope, float* dz,
                            float* partials, void* stream) {
    if (!dout || !Z || !scale || !shift || !mean || !invstd || !dz || !partials) return DGX_EINVAL;
    if (B < 1 || N < 1 || C < 1 || ldz < C) return DGX_EINVAL;
    dim3 grid(B * ((N + PT - 1) / PT), (C + PT - 1) / PT);
    hipLaunchKernelGGL(bwd_T_kernel, grid, dim3(256), 0, dgx_stream(stream), dout, Z, ldz, N, C, scale, shift, mean,
                       invstd, slope, dz, partials);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_pointconv_input_grad(const float* dz, const float* Z, int ldz, int64_t M, int C, const float* scale,
                         const float* c0, const float* c1, void* dZ, int bf16, void* stream) {
    if (!dz || !Z || !scale || !c0 || !c1 || !dZ || M < 1 || C < 1 || ldz < C) return DGX_EINVAL;
    const int g = grid_for(M * C, 256);
    if (bf16)
        hipLaunchKernelGGL(bwd_dZ_kernel<true>, dim3(g), dim3(256), 0, dgx_stream(stream), dz, Z, ldz, M, C, scale, c0,
                           c1, dZ);
    else
        hipLaunchKernelGGL(bwd_dZ_kernel<false>, dim3(g), dim3(256), 0, dgx_stream(stream), dz, Z, ldz, M, C, scale,
                           c0, c1, dZ);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_pointconv_bf16_rows(int B, int N) {
    if (B < 1 || N < 1) return DGX_EINVAL;
    return B * ((N + RT_P * RS_LT - 1) / (RT_P * RS_LT));  // pass-0 partial rows
}

int dgx_pointconv_apply_bf16(const void* Z, int B, int N, int C, const float* scale, const float* shift, float slope,
                             float* out, void* stream) {
    if (!Z || !scale || !shift || !out || B < 1 || N < 1 || C < 1) return DGX_EINVAL;
    dim3 grid(B * ((N + RT_P - 1) / RT_P), (C + 63) / 64);
    hipLaunchKernelGGL(apply16_lt_kernel, grid, dim3(256), 0, dgx_stream(stream), static_cast<const bf16*>(Z), N, C,
                       scale, shift, slope, out);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_pointconv_bwd_bf16(const float* dout, const void* Z, int B, int N, int C, const float* scale,
                           const float* shift, const float* mean, const float* invstd, float slope, const float* c0,
                           const float* c1, float* partials, void* dZ, int pass, void* stream) {
    if (!dout || !Z || !scale || !shift || B < 1 || N < 1 || C < 1) return DGX_EINVAL;
    if (pass == 0 ? (!mean || !invstd || !partials) : (!c0 || !c1 || !dZ)) return DGX_EINVAL;
    dim3 grid(B * ((N + RT_P - 1) / RT_P), (C + 63) / 64);
    const bf16* z = static_cast<const bf16*>(Z);
    if (pass == 0)
        hipLaunchKernelGGL(bwd16_stats_lt_kernel, dim3(B * ((N + RT_P * RS_LT - 1) / (RT_P * RS_LT)), (C + 63) / 64),
                           dim3(256), 0, dgx_stream(stream), dout, z, N, C, scale, shift, mean, invstd, slope,
                           partials);
    else
        hipLaunchKernelGGL(bwd16_dz_lt_kernel, grid, dim3(256), 0, dgx_stream(stream), dout, z, N, C, scale, shift,
                           slope, c0, c1, static_cast<bf16*>(dZ));
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_pointconv_bwd_split_f32(const float* dout, const float* Z, int B, int N, int C, const float* scale,
                                const float* shift, const float* mean, const float* invstd, float slope,
                                const float* c0, const float* c1, float* partials, void* dZ_hi, void* dZ_lo, int pass,
                                void* stream) {
    if (!dout || !Z || !scale || !shift || B < 1 || N < 1 || C < 1) return DGX_EINVAL;
    if (pass == 0 ? (!mean || !invstd || !partials) : (!c0 || !c1 || !dZ_hi || !dZ_lo)) return DGX_EINVAL;
    if (C % 4 || (reinterpret_cast<uintptr_t>(Z) & 15)) return DGX_EUNSUPPORTED;
    if (pass == 0)
        hipLaunchKernelGGL(bwd32_stats_lt_kernel, dim3(B * ((N + RT_P * RS_LT - 1) / (RT_P * RS_LT)), (C + 63) / 64),
                           dim3(256), 0, dgx_stream(stream), dout, Z, N, C, scale, shift, mean, invstd, slope,
                           partials);
    else
        hipLaunchKernelGGL(bwd32_split_lt_kernel, dim3(B * ((N + RT_P - 1) / RT_P), (C + 63) / 64), dim3(256), 0,
                           dgx_stream(stream), dout, Z, N, C, scale, shift, slope, c0, c1,
                           static_cast<bf16*>(dZ_hi), static_cast<bf16*>(dZ_lo));
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_to_bf16(const float* src, int64_t ld, int64_t rows, int cols, void* dst, void* stream) {
    if (!src || !dst || rows < 0 || cols < 1 || ld < cols) return DGX_EINVAL;
    if (rows == 0) return DGX_OK;
    hipLaunchKernelGGL(to_bf16_kernel, dim3(grid_for(rows * cols, 256)), dim3(256), 0, dgx_stream(stream), src, ld,
                       rows, cols, static_cast<uint16_t*>(dst));
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

}  // extern "C"
