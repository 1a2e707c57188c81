// a1 — kNN for the shapes the fused selection kernel (knn.hip) is not built
// for: C > 128 channels, k > 64 neighbours, N > 12288 points (reference
// models/dgcnn.py:6-12 takes any C, k <= N and N). Same arithmetic, same
// canonical output, in three stages per chunk of query rows:
//   |x|^2      sqnorm_generic_kernel: torch's CPU sum order for any C (the full
//              4-level cascade of aten SumKernel.cpp; knn.hip's sqnorm stops at
//              level 1, enough for C <= 128), one thread per point.
//   x_q . x_j  dgx_gemm_f32 (gemm32.hip) on the cloud's rows: one
//              v_mfma_f32_16x16x4_f32 accumulation chain per output over
//              c = 0..C-1, i.e. the k-ordered fmaf chain MKL's sgemm runs for
//              the reference (bit-exact; pinned up to C = 256, where the
//              reference's sgemm stops blocking K in one chain).
//   top-k      knn_select_generic_kernel, one workgroup per query row:
//              pd = fl(fl(2 dot - xx_j) - xx_i) recomputed from the dot row, an
//              exact radix select of the k-th largest value (4 x 8-bit
//              digits of an order-preserving key), every value above it plus
//              the lowest-index values equal to it, then a bitonic sort by
//              (value desc, index asc): the canonical order of the fast path.
// Scratch: |x|^2 (B*N) and one chunk of dot rows (rows x N floats) in the
// caller's workspace (dgx_knn_generic_workspace_bytes).
#include "common.h"

extern "C" int dgx_gemm_f32(const float* A, int a_ic, int lda, const float* B, int b_ic, int ldb, int M, int N, int K,
                            int epi, int splits, float* C, int64_t ldc, const float* addend, int64_t ldd,
                            void* stream);

namespace {

constexpr int KG_THREADS = 256;
constexpr int KG_MAXK = 8192;               // bitonic buffer: 8192 (value, index) pairs = 64 KiB of LDS
constexpr int64_t KG_CHUNK_FLOATS = 1 << 24; // dot rows per chunk: rows * N <= 16 Mi floats (64 MiB)
constexpr int SQG_THREADS = 128;

// ---- |x|^2 in torch's CPU summation order, any C ----------------------------
// e(i) = x[c0 + i * step]^2 of one point (squares recomputed from x: no staging)
struct SqAt {
    const float* p;
    int64_t sC;
    __device__ __forceinline__ float operator()(int c) const {
        const float v = p[(int64_t)c * sC];
        return v * v;
    }
};

// torch multi_row_sum: levels of 16 (oracle/knn_oracle.c cascade) over
// e(first + i * step), i < m
__device__ float cascade_g(const SqAt& e, int first, int step, int m) {
#pragma clang fp contract(off)
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int i = 0;
    while (i + 16 <= m) {
        for (int j = 0; j < 16; ++j, ++i) acc[0] = acc[0] + e(first + i * step);
        for (int l = 1; l < 4; ++l) {
            acc[l] = acc[l] + acc[l - 1];
            acc[l - 1] = 0.f;
            if ((i & (15 << (4 * l))) != 0) break;
        }
    }
    for (; i < m; ++i) acc[0] = acc[0] + e(first + i * step);
    for (int l = 1; l < 4; ++l) acc[0] = acc[0] + acc[l];
    return acc[0];
}

// torch row_sum, ILP 4, over e(first + i * step), i < n
__device__ float rowsum_g(const SqAt& e, int first, int step, int n) {
#pragma clang fp contract(off)
    const int si = n / 4;
    float l[4];
    for (int q = 0; q < 4; ++q) l[q] = si > 0 ? cascade_g(e, first + q * step, 4 * step, si) : 0.f;
    for (int i = 4 * si; i < n; ++i) l[0] = l[0] + e(first + i * step);
    return ((l[0] + l[1]) + l[2]) + l[3];
}

__global__ __launch_bounds__(SQG_THREADS) void sqnorm_generic_kernel(const float* __restrict__ x, int64_t sB,
                                                                     int64_t sC, int64_t sN, int B, int C, int N,
                                                                     int order, float* __restrict__ xx) {
#pragma clang fp contract(off)
    const int64_t t = (int64_t)blockIdx.x * SQG_THREADS + threadIdx.x;
    if (t >= (int64_t)B * N) return;
    const int b = (int)(t / N), n = (int)(t - (int64_t)b * N);
    const SqAt e{x + b * sB + n * sN, sC};
    float r;
    if (order == DGX_ORDER_VEC8X4) {
        if (C < 8) {
            r = rowsum_g(e, 0, 1, C);
        } else {
            const int vs = C / 8;
            float fin = 0.f;
            for (int c = 8 * vs; c < C; ++c) fin = fin + e(c);
            for (int l = 0; l < 8; ++l) fin = fin + rowsum_g(e, l, 8, vs);
            r = fin;
        }
    } else {
        // full 32-point blocks: the cascade over all channels; the tail points: row_sum
        r = n >= (N & ~31) ? rowsum_g(e, 0, 1, C) : cascade_g(e, 0, 1, C);
    }
    xx[t] = r;
}

// ---- exact top-k of one query row -------------------------------------------
// order-preserving 32-bit key of a float (larger float <-> larger key)
__device__ __forceinline__ uint32_t fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ bool canon_better_g(float va, int ia, float vb, int ib) {
    return va > vb || (va == vb && ia < ib);
}

// block-wide exclusive prefix of one flag per thread (returns the thread's offset; *total = block sum)
__device__ __forceinline__ int block_prefix(int flag, int* wsum, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t bal = __ballot(flag);
    const int in_wave = __popcll(bal & ((1ull << lane) - 1ull));
    __syncthreads();
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int u = 0; u < KG_THREADS / 64; ++u) {
        if (u < w) off += wsum[u];
        tot += wsum[u];
    }
    *total = tot;
    return off + in_wave;
}

__global__ __launch_bounds__(KG_THREADS) void knn_select_generic_kernel(const float* __restrict__ dot, int64_t ldd,
                                                                        const float* __restrict__ xx, int N, int k,
                                                                        int q0, int b, int P2,
                                                                        int64_t* __restrict__ idx64,
                                                                        int32_t* __restrict__ idx32,
                                                                        float* __restrict__ vals) {
#pragma clang fp contract(off)
    extern __shared__ float2 pairs[];   // [P2] (value, index bits)
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh_prefix;
    __shared__ int sh_rem, cnt_gt, wsum[KG_THREADS / 64];
    const int t = threadIdx.x;
    const int r = blockIdx.x, i = q0 + r;
    const float* __restrict__ drow = dot + (int64_t)r * ldd;
    const float* __restrict__ xb = xx + (int64_t)b * N;
    const float xi = xb[i];
    // pd_ij = fl(fl(2 dot - xx_j) - xx_i), dgcnn.py:7-9; -0 folded into +0 (equal values)
    auto pdv = [&](int j) { return ((2.f * drow[j] - xb[j]) - xi) + 0.f; };
    // radix select of the k-th largest key, most significant digit first
    uint32_t prefix = 0;
    int rem = k;   // rank of the k-th largest within the keys matching `prefix`
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        const uint32_t hmask = pass == 0 ? 0u : (0xffffffffu << (32 - 8 * pass));
        hist[t] = 0;   // KG_THREADS == 256 bins
        __syncthreads();
        for (int j = t; j < N; j += KG_THREADS) {
            const uint32_t key = fkey(pdv(j));
            if ((key & hmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (t == 0) {
            int cum = 0, d = 255;
            for (; d > 0; --d) {
                if (cum + (int)hist[d] >= rem) break;
                cum += (int)hist[d];
            }
            sh_prefix = prefix | ((uint32_t)d << shift);
            sh_rem = rem - cum;
        }
        __syncthreads();
        prefix = sh_prefix;
        rem = sh_rem;
        __syncthreads();
    }
    const uint32_t T = prefix;    // key of the k-th largest value
    const int need = rem;         // values equal to it that enter the top k (lowest indices first)
    const int gt = k - need;      // values above it
    if (t == 0) cnt_gt = 0;
    __syncthreads();
    for (int j = t; j < N; j += KG_THREADS) {
        const float v = pdv(j);
        if (fkey(v) > T) pairs[atomicAdd(&cnt_gt, 1)] = make_float2(v, __int_as_float(j));
    }
    // ties at the k-th value in index order
    int taken = 0;
    for (int base = 0; base < N && taken < need; base += KG_THREADS) {
        const int j = base + t;
        float v = 0.f;
        int flag = 0;
        if (j < N) {
            v = pdv(j);
            flag = fkey(v) == T;
        }
        int tot;
        const int pos = taken + block_prefix(flag, wsum, &tot);
        if (flag && pos < need) pairs[gt + pos] = make_float2(v, __int_as_float(j));
        taken += tot;
    }
    for (int p = k + t; p < P2; p += KG_THREADS) pairs[p] = make_float2(-INFINITY, __int_as_float(0x7fffffff));
    __syncthreads();
    // bitonic sort of P2 pairs, best first
    for (int size = 2; size <= P2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int p = t; p < P2 / 2; p += KG_THREADS) {
                const int lo = 2 * p - (p & (stride - 1));
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;   // this run sorts best-first
                const float2 a = pairs[lo], c = pairs[hi];
                const bool c_first = canon_better_g(c.x, __float_as_int(c.y), a.x, __float_as_int(a.y));
                if (c_first == up) {
                    pairs[lo] = c;
                    pairs[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    const int64_t row = ((int64_t)b * N + i) * k;
    for (int p = t; p < k; p += KG_THREADS) {
        const float2 e = pairs[p];
        const int j = __float_as_int(e.y);
        if (idx64) idx64[row + p] = j;
        if (idx32) idx32[row + p] = j;
        if (vals) vals[row + p] = e.x;
    }
}

int chunk_rows(int N) {
    int64_t rows = KG_CHUNK_FLOATS / N;
    rows = rows < 64 ? 64 : rows;
    rows -= rows % 64;
    return (int)(rows < N ? rows : N);
}

}  // namespace

extern "C" {

size_t dgx_knn_generic_workspace_bytes(int B, int C, int N) {
    if (B < 0 || C < 1 || N < 1) return 0;
    const size_t xxf = (((size_t)B * N + 3) & ~(size_t)3);
    return (xxf + (size_t)chunk_rows(N) * N) * sizeof(float);
}

int dgx_knn_generic_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int C, int N, int k, int order,
                        int64_t* idx64, int32_t* idx32, float* vals, void* workspace, size_t workspace_bytes,
                        void* stream) {
    if (!x || B < 0 || C < 1 || N < 1 || k < 1 || k > N || (!idx64 && !idx32)) return DGX_EINVAL;
    if (!workspace || workspace_bytes < dgx_knn_generic_workspace_bytes(B, C, N)) return DGX_EINVAL;
    if (k > KG_MAXK) return DGX_EUNSUPPORTED;
    // the Gram GEMM reads the cloud in place: one of the two inner strides must be 1
    const bool ic = sN == 1, kc = sC == 1 && !ic;
    if (!ic && !kc) return DGX_EUNSUPPORTED;
    if ((ic ? sC : sN) > INT32_MAX || (int64_t)N * N > ((int64_t)1 << 40)) return DGX_EUNSUPPORTED;
    if (B == 0) return DGX_OK;
    hipStream_t st = dgx_stream(stream);
    float* xx = static_cast<float*>(workspace);
    float* dot = xx + (((size_t)B * N + 3) & ~(size_t)3);
    const int64_t pts = (int64_t)B * N;
    hipLaunchKernelGGL(sqnorm_generic_kernel, dim3((unsigned)((pts + SQG_THREADS - 1) / SQG_THREADS)),
                       dim3(SQG_THREADS), 0, st, x, sB, sC, sN, B, C, N, order, xx);
    if (hipGetLastError() != hipSuccess) return DGX_ELAUNCH;
    int P2 = 1;
    while (P2 < k) P2 <<= 1;
    const size_t lds = (size_t)P2 * sizeof(float2);
    const int rows = chunk_rows(N);
    const int ld = (int)(ic ? sC : sN);
    for (int b = 0; b < B; ++b) {
        const float* xb = x + (int64_t)b * sB;
        for (int q0 = 0; q0 < N; q0 += rows) {
            const int m = rows < N - q0 ? rows : N - q0;
            // dot[r][j] = sum_c x[q0 + r][c] x[j][c] (one MFMA chain per output, c in order)
            const float* A = xb + (int64_t)q0 * (ic ? 1 : sN);
            int rc = dgx_gemm_f32(A, ic ? 1 : 0, ld, xb, ic ? 1 : 0, ld, m, N, C, 0, 1, dot, N, nullptr, 0, stream);
            if (rc != DGX_OK) return rc;
            hipLaunchKernelGGL(knn_select_generic_kernel, dim3((unsigned)m), dim3(KG_THREADS), lds, st, dot,
                               (int64_t)N, xx, N, k, q0, b, P2, idx64, idx32, vals);
            if (hipGetLastError() != hipSuccess) return DGX_ELAUNCH;
        }
    }
    return DGX_OK;
}

}  // extern "C"
