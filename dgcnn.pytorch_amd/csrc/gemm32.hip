// fp32 MFMA GEMM of the parity mode (precision "fp32"): exact fp32 products,
// fp32 accumulation on v_mfma_f32_16x16x4_f32.
//
// Serves every Conv(1x1) GEMM of the EdgeConv chain, conv5 and the
// PositionEmbedding edge MLP when the engine runs in fp32 (reference
// models/dgcnn.py:54-78 and models/layers.py:17-24 are fp32 Conv2d; the
// bf16 family in gemm.hip serves the bf16 mode). Same contract as
// dgx_gemm_bf16:   C[i][j] = sum_k opA(i,k) * opB(j,k)
// with opA(i,k) = A[i*lda + k] ("KC") or A[k*lda + i] ("IC"), the same for B,
// so transposed views of existing buffers (dPQ^T, W^T) are read in place.
// Epilogues: STORE, ACCUM (C = addend + .. or C += ..), SLAB (split-K partial
// tiles; slab_reduce_kernel sums them in a fixed order: deterministic weight
// gradients over the B*N rows).
//
// Tile 64 x 64 x 16, 256 threads = 4 waves in 2 x 2, each a 32 x 32 quadrant
// of 2 x 2 MFMA tiles. Both operands are staged k-major in LDS ([k][64 + 16]:
// the 16-float pad puts the four k rows a 16x16x4 fragment read touches on
// distinct bank groups) through a register double buffer: the next K-step's
// global loads are issued before the current step's MFMAs.
#include "common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int G32_THREADS = 256;
constexpr int G32_BM = 64, G32_BN = 64, G32_BK = 16;
constexpr int G32_LD = G32_BM + 16;
enum { E32_STORE = 0, E32_ACCUM = 1, E32_SLAB = 3 };

// 4 elements of one operand tile (64 rows x 16 k) per thread, registers
struct Frag4 {
    float v[4];
};

// Load thread t's share of the (rows r0.., k k0..) tile of op(row, k):
// KC: row = t / 4, k = 4 (t % 4) .. +3 (contiguous k); IC: k = t / 16,
// row = 4 (t % 16) .. +3 (contiguous rows). Out-of-range elements are 0.
template <bool IC>
__device__ __forceinline__ Frag4 load_tile(const float* __restrict__ P, int ld, int rows, int K, int r0, int k0,
                                           int kend, bool vec) {
    Frag4 f;
    const int t = threadIdx.x;
    if constexpr (!IC) {
        const int r = r0 + t / 4, k = k0 + 4 * (t % 4);
        if (vec && r < rows && k + 3 < kend) {
            const float4 q = *reinterpret_cast<const float4*>(P + (int64_t)r * ld + k);
            f.v[0] = q.x; f.v[1] = q.y; f.v[2] = q.z; f.v[3] = q.w;
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) f.v[u] = (r < rows && k + u < kend) ? P[(int64_t)r * ld + k + u] : 0.f;
        }
    } else {
        const int k = k0 + t / 16, r = r0 + 4 * (t % 16);
        if (vec && k < kend && r + 3 < rows) {
            const float4 q = *reinterpret_cast<const float4*>(P + (int64_t)k * ld + r);
            f.v[0] = q.x; f.v[1] = q.y; f.v[2] = q.z; f.v[3] = q.w;
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) f.v[u] = (k < kend && r + u < rows) ? P[(int64_t)k * ld + r + u] : 0.f;
        }
    }
    (void)K;
    return f;
}

template <bool IC>
__device__ __forceinline__ void store_tile(float (*S)[G32_LD], const Frag4& f) {
    const int t = threadIdx.x;
    if constexpr (!IC) {
        const int r = t / 4, k = 4 * (t % 4);
#pragma unroll
        for (int u = 0; u < 4; ++u) S[k + u][r] = f.v[u];
    } else {
        const int k = t / 16, r = 4 * (t % 16);
        *reinterpret_cast<float4*>(&S[k][r]) = make_float4(f.v[0], f.v[1], f.v[2], f.v[3]);
    }
}

template <bool AIC, bool BIC, int EPI>
__global__ __launch_bounds__(G32_THREADS) void gemm32_kernel(const float* __restrict__ A, int lda,
                                                            const float* __restrict__ Bm, int ldb, int M, int N,
                                                            int K, int kchunk, float* __restrict__ C, int64_t ldc,
                                                            const float* __restrict__ addend, int64_t ldd,
                                                            int ntn, bool avec, bool bvec) {
    __shared__ __attribute__((aligned(16))) float As[G32_BK][G32_LD];
    __shared__ __attribute__((aligned(16))) float Bs[G32_BK][G32_LD];
    const int tm = blockIdx.x / ntn, tn = blockIdx.x - tm * ntn;
    const int m0 = tm * G32_BM, n0 = tn * G32_BN;
    const int kb = blockIdx.y * kchunk, ke = min(K, kb + kchunk);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    Frag4 fa = load_tile<AIC>(A, lda, M, K, m0, kb, ke, avec);
    Frag4 fb = load_tile<BIC>(Bm, ldb, N, K, n0, kb, ke, bvec);
    for (int k0 = kb; k0 < ke; k0 += G32_BK) {
        store_tile<AIC>(As, fa);
        store_tile<BIC>(Bs, fb);
        __syncthreads();
        if (k0 + G32_BK < ke) {   // next step's loads in flight during this step's MFMAs
            fa = load_tile<AIC>(A, lda, M, K, m0, k0 + G32_BK, ke, avec);
            fb = load_tile<BIC>(Bm, ldb, N, K, n0, k0 + G32_BK, ke, bvec);
        }
#pragma unroll
        for (int kk = 0; kk < G32_BK; kk += 4) {
            const int kr = kk + (lane >> 4), c = lane & 15;
            float a[2], b[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                a[u] = As[kr][wm * 32 + u * 16 + c];
                b[u] = Bs[kr][wn * 32 + u * 16 + c];
            }
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj)
                    acc[ti][tj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ti], b[tj], acc[ti][tj], 0, 0, 0);
        }
        __syncthreads();
    }
    // lane holds C[4 (lane / 16) + r][lane % 16] of each 16 x 16 tile
    float* __restrict__ out = EPI == E32_SLAB ? C + (int64_t)blockIdx.y * M * N : C;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = m0 + wm * 32 + ti * 16 + 4 * (lane >> 4) + r;
                const int j = n0 + wn * 32 + tj * 16 + (lane & 15);
                if (i >= M || j >= N) continue;
                const float v = acc[ti][tj][r];
                if constexpr (EPI == E32_SLAB) {
                    out[(int64_t)i * N + j] = v;
                } else if constexpr (EPI == E32_ACCUM) {
                    float* d = out + (int64_t)i * ldc + j;
                    *d = (addend ? addend[(int64_t)i * ldd + j] : *d) + v;
                } else {
                    out[(int64_t)i * ldc + j] = v;
                }
            }
}

bool al16f(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" {

int dgx_gemm_f32(const float* A, int a_ic, int lda, const float* B, int b_ic, int ldb, int M, int N, int K, int epi,
                 int splits, float* C, int64_t ldc, const float* addend, int64_t ldd, void* stream) {
    if (!A || !B || !C || M < 0 || N < 0 || K < 0 || lda < 1 || ldb < 1 || splits < 1) return DGX_EINVAL;
    if (epi != E32_STORE && epi != E32_ACCUM && epi != E32_SLAB) return DGX_EINVAL;
    if (M == 0 || N == 0) return DGX_OK;
    if (epi != E32_SLAB && ldc < N) return DGX_EINVAL;
    const int ntm = (M + G32_BM - 1) / G32_BM, ntn = (N + G32_BN - 1) / G32_BN;
    int kchunk = (K + splits - 1) / splits;
    kchunk = ((kchunk + G32_BK - 1) / G32_BK) * G32_BK;
    const int used = K > 0 ? (K + kchunk - 1) / kchunk : 1;
    if (epi != E32_SLAB && used > 1) return DGX_EINVAL;   // split-K only through slabs
    const bool avec = lda % 4 == 0 && al16f(A), bvec = ldb % 4 == 0 && al16f(B);
    const dim3 grid((unsigned)(ntm * ntn), (unsigned)used);
    hipStream_t st = dgx_stream(stream);
#define DGX_G32(AIC, BIC, E)                                                                                 \
    hipLaunchKernelGGL((gemm32_kernel<AIC, BIC, E>), grid, dim3(G32_THREADS), 0, st, A, lda, B, ldb, M, N, K, \
                       kchunk, C, ldc, addend, ldd, ntn, avec, bvec)
#define DGX_G32_E(AIC, BIC)                          \
    if (epi == E32_STORE) DGX_G32(AIC, BIC, E32_STORE); \
    else if (epi == E32_ACCUM) DGX_G32(AIC, BIC, E32_ACCUM); \
    else DGX_G32(AIC, BIC, E32_SLAB)
    if (!a_ic && !b_ic) { DGX_G32_E(false, false); }
    else if (!a_ic && b_ic) { DGX_G32_E(false, true); }
    else if (a_ic && !b_ic) { DGX_G32_E(true, false); }
    else { DGX_G32_E(true, true); }
#undef DGX_G32_E
#undef DGX_G32
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

// split count for dgx_gemm_f32's SLAB epilogue: enough K slices that the grid
// holds ~512 workgroups, each slice at least 512 k deep
int dgx_gemm_f32_splits(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0) return 1;
    const int tiles = ((M + G32_BM - 1) / G32_BM) * ((N + G32_BN - 1) / G32_BN);
    int s = (512 + tiles - 1) / tiles;
    const int cap = K / 512 > 0 ? K / 512 : 1;
    s = s < cap ? s : cap;
    return s < 1 ? 1 : (s > 256 ? 256 : s);
}

}  // extern "C"
