// bf16 MFMA GEMMs of the EdgeConv chain and conv5 (v_mfma_f32_16x16x32_bf16).
//
// Replaces the Conv2d(1x1) GEMMs of reference models/dgcnn.py:54-78 (forward
// K11/K15 of SURVEY §2.3 and their autograd dgrad/wgrad). After the EdgeConv
// decomposition every GEMM of the chain is a per-point GEMM over
// M = B*N rows:
//   forward   PQ = X [W1;W2]^T            (M x 2Co),  K = C
//             Z  = Xcat W5^T  + BN stats  (M x emb),  K = 512
//   backward  dX += dPQ Wcat / dZ W5      (M x C),    K = 2Co / emb
//             dW  = dPQ^T X / dZ^T Xcat   (small),    K = M  (split-K)
//
// One kernel template computes   C[i][j] = sum_k opA(i,k) * opB(j,k)
// where opA(i,k) is A[i*lda+k] ("KC": k contiguous) or A[k*lda+i] ("IC": i
// contiguous), the same for B. Operands are fp32 or bf16 in HBM and are
// converted to bf16 (round-to-nearest-even) while being staged into LDS, so no
// separate conversion pass touches HBM. LDS holds both tiles k-contiguous
// ([row][BK + 8] bf16, 80-byte rows: the 16-row ds_read_b128 fragment reads hit
// 16 distinct 4-bank groups). Accumulation is fp32 in the MFMA.
//
// Epilogues (all fp32): STORE, ACCUM (C += ..., used to add dX straight into
// the concat-gradient buffer), STATS (STORE + per-column sum / sum of squares
// of the block's rows: the train-mode BatchNorm statistics of conv5, so Z is
// never re-read for them) and SLAB (split-K partial tile; slab_reduce_kernel
// sums the slabs in a fixed order -> deterministic weight gradients).
#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int GB_THREADS = 256;
constexpr int GB_BM = 128;
constexpr int GB_BK = 32;
constexpr int GB_LDK = GB_BK + 8;  // bf16 per LDS row (80 B)

enum { EPI_STORE = 0, EPI_ACCUM = 1, EPI_STATS = 2, EPI_SLAB = 3, EPI_STATS16 = 4, EPI_DZ2 = 5, EPI_H1BWD = 6,
       EPI_EDZ = 7 };

// Extra operands of the PositionEmbedding edge-MLP epilogues (EPI_H1BWD):
// g = dH1 * LReLU'(z1) with z1 = a1 (P_j + Q_i) + b1 for edge row e = i*k + s,
// j = idx[e] (local), plus the BN1-backward column partials (sum g, sum g*yhat).
struct EpiEdge {
    const float* PQ;
    int ldpq;
    const int32_t* idx;
    int N, k;
    const float *scale, *shift, *mean, *invstd;
    float slope;
};

template <typename T> struct VecOf;
template <> struct VecOf<float> { static constexpr int V = 4; typedef float4 type; };
template <> struct VecOf<bf16> { static constexpr int V = 8; typedef uint4 type; };

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(bf16 v) { return (float)v; }

// Blocks b and b+8 share an XCD (MI355X_MICROARCH.md); give each XCD a
// contiguous range of logical tiles (bijective for any grid size) so the blocks
// that share an A row panel share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int id, int n) {
    const int q = n >> 3, r = n & 7, x = id & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (id >> 3);
}

// Stages a TILE x BK slab of op(i,k), i in [i0, i0+TILE) clipped to `rows`,
// k in [k0, k0+BK) clipped to `kend`, into LDS [i][GB_LDK] as bf16. Global
// loads go to registers first (load) and reach LDS after the current tile's
// MFMAs (store), so their latency hides behind the compute.
template <typename T, bool IC, int TILE>
struct Stager {
    static constexpr int V = VecOf<T>::V;
    // KC: task = (row, V-wide k vector). IC: task = (V-wide i vector, 4 k rows).
    static constexpr int TASKS = IC ? (TILE / V) * (GB_BK / 4) : TILE * (GB_BK / V);
    static constexpr int NT = (TASKS + GB_THREADS - 1) / GB_THREADS;
    static constexpr int PER = IC ? 4 * V : V;
    float r[NT][PER];

    __device__ __forceinline__ void load(const T* __restrict__ p, int64_t ld, int i0, int rows, int k0, int kend,
                                         bool vec, int tid) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int task = tid + t * GB_THREADS;
            if (task >= TASKS) break;
            if (!IC) {
                const int row = task / (GB_BK / V), kv = (task % (GB_BK / V)) * V;
                const int i = i0 + row, k = k0 + kv;
                if (vec && i < rows && k + V <= kend) {
                    const typename VecOf<T>::type w =
                        *reinterpret_cast<const typename VecOf<T>::type*>(p + (int64_t)i * ld + k);
                    const T* e = reinterpret_cast<const T*>(&w);
#pragma unroll
                    for (int u = 0; u < V; ++u) r[t][u] = to_f(e[u]);
                } else {
#pragma unroll
                    for (int u = 0; u < V; ++u)
                        r[t][u] = (i < rows && k + u < kend) ? to_f(p[(int64_t)i * ld + k + u]) : 0.f;
                }
            } else {
                const int ig = task % (TILE / V), kg = task / (TILE / V);
                const int i = i0 + ig * V, k = k0 + kg * 4;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const bool krow = k + kk < kend;
                    if (vec && krow && i + V <= rows) {
                        const typename VecOf<T>::type w =
                            *reinterpret_cast<const typename VecOf<T>::type*>(p + (int64_t)(k + kk) * ld + i);
                        const T* e = reinterpret_cast<const T*>(&w);
#pragma unroll
                        for (int u = 0; u < V; ++u) r[t][kk * V + u] = to_f(e[u]);
                    } else {
#pragma unroll
                        for (int u = 0; u < V; ++u)
                            r[t][kk * V + u] = (krow && i + u < rows) ? to_f(p[(int64_t)(k + kk) * ld + i + u]) : 0.f;
                    }
                }
            }
        }
    }

    __device__ __forceinline__ void store(bf16* __restrict__ lds, int tid) const {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int task = tid + t * GB_THREADS;
            if (task >= TASKS) break;
            if (!IC) {
                const int row = task / (GB_BK / V), kv = (task % (GB_BK / V)) * V;
                if constexpr (V == 4) {
                    bf16x4 h = {(bf16)r[t][0], (bf16)r[t][1], (bf16)r[t][2], (bf16)r[t][3]};
                    *reinterpret_cast<bf16x4*>(lds + row * GB_LDK + kv) = h;
                } else {
                    bf16x8 h;
#pragma unroll
                    for (int u = 0; u < 8; ++u) h[u] = (bf16)r[t][u];
                    *reinterpret_cast<bf16x8*>(lds + row * GB_LDK + kv) = h;
                }
            } else {
                const int ig = task % (TILE / V), kg = task / (TILE / V);
#pragma unroll
                for (int u = 0; u < V; ++u) {
                    bf16x4 h = {(bf16)r[t][u], (bf16)r[t][V + u], (bf16)r[t][2 * V + u], (bf16)r[t][3 * V + u]};
                    *reinterpret_cast<bf16x4*>(lds + (ig * V + u) * GB_LDK + kg * 4) = h;
                }
            }
        }
    }
};

// C[i][j] = sum_k opA(i,k) opB(j,k); i < M, j < N, k in this split's range.
template <typename TA, bool AIC, typename TB, bool BIC, int BN, int EPI>
__global__ __launch_bounds__(GB_THREADS, 2) void gemm_bf16_kernel(
    const TA* __restrict__ A, int64_t lda, const TB* __restrict__ B, int64_t ldb, int M, int N, int K, int kchunk,
    int vec_a, int vec_b, float* __restrict__ C, int64_t ldc, float* __restrict__ part) {
    constexpr int BM = GB_BM;
    constexpr int WN = BN >= 128 ? 2 : 1;
    constexpr int WM = 4 / WN;
    constexpr int TM = BM / WM / 16;
    constexpr int TN = BN / WN / 16;
    constexpr int STAGE = (BM + BN) * GB_LDK;
    __shared__ __attribute__((aligned(16))) bf16 lds[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int nJ = (N + BN - 1) / BN;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    // tile order in groups of two row tiles: the 4 consecutive tiles an XCD
    // takes (xcd_remap) form a 2 x 2 square, so each A row panel and each B
    // column panel of a K-chunk is fetched by half as many XCDs as in row-major
    // order (which shares A panels but sends every B panel to all eight)
    const int nI = (M + BM - 1) / BM;
    int ti, tj;
    {
        const int gsz = 2 * nJ, grp = L / gsz, first = grp * 2, gm = min(nI - first, 2), r = L - grp * gsz;
        ti = first + r % gm;
        tj = r / gm;
    }
    const int i0 = ti * BM, j0 = tj * BN;
    const int kbeg = blockIdx.y * kchunk;
    const int kend = min(K, kbeg + kchunk);
    const int nk = kend > kbeg ? (kend - kbeg + GB_BK - 1) / GB_BK : 0;

    f32x4 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    Stager<TA, AIC, BM> sa;
    Stager<TB, BIC, BN> sb;
    if (nk > 0) {
        sa.load(A, lda, i0, M, kbeg, kend, vec_a, tid);
        sb.load(B, ldb, j0, N, kbeg, kend, vec_b, tid);
        sa.store(lds, tid);
        sb.store(lds + BM * GB_LDK, tid);
    }
    __syncthreads();
    const int fr = lane & 15, fk = 8 * (lane >> 4);
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const bool more = kt + 1 < nk;
        if (more) {
            const int kn = kbeg + (kt + 1) * GB_BK;
            sa.load(A, lda, i0, M, kn, kend, vec_a, tid);
            sb.load(B, ldb, j0, N, kn, kend, vec_b, tid);
        }
        const bf16* As = lds + cur * STAGE;
        const bf16* Bs = As + BM * GB_LDK;
        bf16x8 af[TM], bfv[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a)
            af[a] = *reinterpret_cast<const bf16x8*>(As + (wm * TM * 16 + a * 16 + fr) * GB_LDK + fk);
#pragma unroll
        for (int b = 0; b < TN; ++b)
            bfv[b] = *reinterpret_cast<const bf16x8*>(Bs + (wn * TN * 16 + b * 16 + fr) * GB_LDK + fk);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfv[b], acc[a][b], 0, 0, 0);
        if (more) {
            bf16* nxt = lds + (cur ^ 1) * STAGE;
            sa.store(nxt, tid);
            sb.store(nxt + BM * GB_LDK, tid);
        }
        __syncthreads();
    }

    // ---- epilogue: lane holds rows (lane>>4)*4 + r, column lane&15 of each 16x16 tile
    float* out = C;
    if (EPI == EPI_SLAB) out = C + (int64_t)blockIdx.y * M * N;
    const int rb = i0 + wm * TM * 16 + (lane >> 4) * 4;
    const int cb = j0 + wn * TN * 16 + fr;
    float s1[TN], s2[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) { s1[b] = 0.f; s2[b] = 0.f; }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = rb + a * 16 + r;
            if (i >= M) continue;
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                const int j = cb + b * 16;
                if (j >= N) continue;
                const float v = acc[a][b][r];
                float* dst = out + (int64_t)i * ldc + j;
                if (EPI == EPI_ACCUM) *dst += v;
                else *dst = v;
                if (EPI == EPI_STATS) { s1[b] += v; s2[b] = fmaf(v, v, s2[b]); }
            }
        }
    }
    if (EPI == EPI_STATS) {
        // column partials of this block's rows: lanes l, l^16, l^32, l^48 share a column,
        // then the WM waves of the column are summed through LDS (free after the loop)
        float* red = reinterpret_cast<float*>(lds);  // [WM][BN][2]
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            float a1 = s1[b], a2 = s2[b];
            a1 += __shfl_xor(a1, 16);
            a2 += __shfl_xor(a2, 16);
            a1 += __shfl_xor(a1, 32);
            a2 += __shfl_xor(a2, 32);
            if (lane < 16) {
                const int jl = wn * TN * 16 + b * 16 + lane;
                red[(wm * BN + jl) * 2 + 0] = a1;
                red[(wm * BN + jl) * 2 + 1] = a2;
            }
        }
        __syncthreads();
        for (int jl = tid; jl < BN; jl += GB_THREADS) {
            const int j = j0 + jl;
            if (j >= N) continue;
            float t1 = 0.f, t2 = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) { t1 += red[(w * BN + jl) * 2]; t2 += red[(w * BN + jl) * 2 + 1]; }
            part[(int64_t)ti * 2 * N + j] = t1;
            part[(int64_t)ti * 2 * N + N + j] = t2;
        }
    }
}

// out[orow][ocol] = sum_s slab[s][r][c]; rows r >= split go to (r - split,
// c + cols) — the [W1;W2] -> W = [W1 | W2] un-stacking of an EdgeConv weight.
// Block = 64 output elements x 4 slab groups; group g sums slabs s = g mod 4 in
// ascending s with 8 loads in flight, then the 4 group sums are added in a
// fixed order: the result does not depend on timing (deterministic).
constexpr int SR_E = 64, SR_G = 4, SR_U = 8;
__global__ __launch_bounds__(SR_E * SR_G) void slab_reduce_kernel(const float* __restrict__ slab, int S, int rows,
                                                                  int cols, int split, float* __restrict__ out,
                                                                  int64_t ldo) {
    __shared__ float red[SR_G][SR_E];
    const int64_t total = (int64_t)rows * cols;
    const int el = threadIdx.x % SR_E, g = threadIdx.x / SR_E;
    const int64_t e = (int64_t)blockIdx.x * SR_E + el;
    float acc = 0.f;
    if (e < total) {
        int s = g;
        for (; s + (SR_U - 1) * SR_G < S; s += SR_U * SR_G) {
            float v[SR_U];
#pragma unroll
            for (int u = 0; u < SR_U; ++u) v[u] = slab[(int64_t)(s + u * SR_G) * total + e];
#pragma unroll
            for (int u = 0; u < SR_U; ++u) acc += v[u];
        }
        for (; s < S; s += SR_G) acc += slab[(int64_t)s * total + e];
    }
    red[g][el] = acc;
    __syncthreads();
    if (g == 0 && e < total) {
        const float sum = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
        const int r = (int)(e / cols), c = (int)(e - (int64_t)r * cols);
        const int orow = r < split ? r : r - split;
        const int ocol = r < split ? c : c + cols;
        out[(int64_t)orow * ldo + ocol] = sum;
    }
}

// slab_reduce_kernel for up to SRM_MAXJ independent reductions in one launch
// (the weight gradients of a backward pass, reduced together at its end): job j
// owns blocks [first[j], first[j+1]); every output element is summed exactly as
// slab_reduce_kernel sums it (same groups, same order), so results are identical.
constexpr int SRM_MAXJ = 8;
struct SlabJobs {
    const float* slab[SRM_MAXJ];
    float* out[SRM_MAXJ];
    int64_t ldo[SRM_MAXJ];
    int S[SRM_MAXJ], rows[SRM_MAXJ], cols[SRM_MAXJ], split[SRM_MAXJ], first[SRM_MAXJ + 1];
    int vec4[SRM_MAXJ];   // job reduced 4 consecutive elements per lane (slab_reduce_block4)
    int n;
};
// one job's block, one element per lane (slab_reduce_kernel's groups and order)
__device__ __forceinline__ void slab_reduce_block1(const SlabJobs& jobs, int j, float (*red)[SR_E]) {
    const float* __restrict__ slab = jobs.slab[j];
    const int S = jobs.S[j], cols = jobs.cols[j], split = jobs.split[j];
    const int64_t total = (int64_t)jobs.rows[j] * cols;
    const int el = threadIdx.x % SR_E, g = threadIdx.x / SR_E;
    const int64_t e = (int64_t)(blockIdx.x - jobs.first[j]) * SR_E + el;
    float acc = 0.f;
    if (e < total) {
        int s = g;
        for (; s + (SR_U - 1) * SR_G < S; s += SR_U * SR_G) {
            float v[SR_U];
#pragma unroll
            for (int u = 0; u < SR_U; ++u) v[u] = slab[(int64_t)(s + u * SR_G) * total + e];
#pragma unroll
            for (int u = 0; u < SR_U; ++u) acc += v[u];
        }
        for (; s < S; s += SR_G) acc += slab[(int64_t)s * total + e];
    }
    red[g][el] = acc;
    __syncthreads();
    if (g == 0 && e < total) {
        const float sum = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
        const int r = (int)(e / cols), c = (int)(e - (int64_t)r * cols);
        const int orow = r < split ? r : r - split;
        const int ocol = r < split ? c : c + cols;
        jobs.out[j][(int64_t)orow * jobs.ldo[j] + ocol] = sum;
    }
}

// one job's block, four consecutive elements per lane (16-byte slab loads, a
// quarter of the workgroups; columns a multiple of 4): every element keeps
// slab_reduce_kernel's groups and order, so the results are identical
__device__ __forceinline__ void slab_reduce_block4(const SlabJobs& jobs, int j, float4 (*red)[SR_E]) {
    const float* __restrict__ slab = jobs.slab[j];
    const int S = jobs.S[j], cols = jobs.cols[j], split = jobs.split[j];
    const int64_t total = (int64_t)jobs.rows[j] * cols;   // a multiple of 4
    const int el = threadIdx.x % SR_E, g = threadIdx.x / SR_E;
    const int64_t e = ((int64_t)(blockIdx.x - jobs.first[j]) * SR_E + el) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < total) {
        int s = g;
        for (; s + (SR_U - 1) * SR_G < S; s += SR_U * SR_G) {
            float4 v[SR_U];
#pragma unroll
            for (int u = 0; u < SR_U; ++u) v[u] = *reinterpret_cast<const float4*>(slab + (int64_t)(s + u * SR_G) * total + e);
#pragma unroll
            for (int u = 0; u < SR_U; ++u) {
                acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
            }
        }
        for (; s < S; s += SR_G) {
            const float4 v = *reinterpret_cast<const float4*>(slab + (int64_t)s * total + e);
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
    }
    red[g][el] = acc;
    __syncthreads();
    if (g == 0 && e < total) {
        const float4 a = red[0][el], b = red[1][el], c = red[2][el], d = red[3][el];
        const float sum[4] = {((a.x + b.x) + c.x) + d.x, ((a.y + b.y) + c.y) + d.y, ((a.z + b.z) + c.z) + d.z,
                              ((a.w + b.w) + c.w) + d.w};
        const int r = (int)(e / cols), c0 = (int)(e - (int64_t)r * cols);
        const int orow = r < split ? r : r - split;
        const int ocol = r < split ? c0 : c0 + cols;
        float* dst = jobs.out[j] + (int64_t)orow * jobs.ldo[j] + ocol;
#pragma unroll
        for (int u = 0; u < 4; ++u) dst[u] = sum[u];
    }
}

__global__ __launch_bounds__(SR_E * SR_G) void slab_reduce_multi_kernel(SlabJobs jobs) {
    __shared__ float4 red[SR_G][SR_E];
    int j = 0;
    while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.first[j + 1]) ++j;
    if (jobs.vec4[j]) slab_reduce_block4(jobs, j, red);
    else slab_reduce_block1(jobs, j, reinterpret_cast<float (*)[SR_E]>(red));
}

// ---------------------------------------------------------------------------
// bf16-operand GEMMs staged by LDS-DMA (global_load_lds_dwordx4).
// Both operands bf16 in HBM, either both k-contiguous ("NT": C = A B^T, the
// forward PQ / conv5 and the input gradients with pre-transposed weights) or
// both i-contiguous ("TN": C = A^T B, the weight gradients, K = M rows split
// over workgroups). 128 x BN x 64 tiles, 4 waves (2 x 2), two LDS stages: the
// next stage's DMA is issued before the current stage's MFMAs and retired by
// one vmcnt(0) + barrier per stage (cdna_hip_programming.md §5.5 T3+T4, 2-phase).
// The LDS destination of a DMA is lane-linear, so the bank swizzles are
// applied to each lane's SOURCE address:
//   NT image [row][64 k] (128-B rows): 16-B chunk c of row r at c ^ (r & 7) —
//      the 16-row ds_read_b128 fragment reads are conflict-free.
//   TN image [k][TILE] (2*TILE-B rows): chunk c of k-row r at c ^ swz(r) —
//      the ds_read_b64_tr_b16 transposed fragment reads (T10) of 8 consecutive
//      k-rows per 32-lane half are conflict-free. TN fragments take k-rows
//      {4g + q} and {16 + 4g + q} (g = lane / 16, q = 0..3) for MFMA k-slots
//      8g + q and 8g + 4 + q: the same permutation on both operands, so the
//      sum over k is unchanged.
constexpr int G2_BM = 128, G2_BK = 64;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int tn_swz(int r, int tile) {
    return tile >= 128 ? 2 * (r & 7) : 2 * ((r >> 1) & 3);
}

__device__ __forceinline__ void dma16(const bf16* g, bf16* lds_base) {
    __builtin_amdgcn_global_load_lds(static_cast<const void*>(g), (lds_void*)(lds_base), 16, 0, 0);
}

// NT operand tile: rows [r0, r0+TILE) (clamped to rows-1), k [k0, k0+64).
template <int TILE>
__device__ __forceinline__ void stage_nt(const bf16* __restrict__ p, int64_t ld, int r0, int rows, int k0,
                                         bf16* img, int wave, int lane) {
    constexpr int INST = TILE * 128 / 1024;  // 1 KB per wave-instruction
#pragma unroll
    for (int u = 0; u < INST / 4; ++u) {
        const int inst = wave * (INST / 4) + u;
        const int row = inst * 8 + (lane >> 3);
        const int c = (lane & 7) ^ (row & 7);
        const int gr = min(r0 + row, rows - 1);
        dma16(p + (int64_t)gr * ld + k0 + 8 * c, img + inst * 512);
    }
}

// TN operand tile: k-rows [k0, k0+64) (clamped to kend-1), columns [c0, c0+TILE)
// (16-B chunks clamped to the last full chunk of the `cols` wide rows).
template <int TILE>
__device__ __forceinline__ void stage_tn(const bf16* __restrict__ p, int64_t ld, int c0, int cols, int k0,
                                         int kend, bf16* img, int wave, int lane) {
    constexpr int CPR = TILE / 8;            // chunks per row
    constexpr int RPI = 64 / CPR;            // rows per wave-instruction
    constexpr int INST = 64 / RPI;
#pragma unroll
    for (int u = 0; u < INST / 4; ++u) {
        const int inst = wave * (INST / 4) + u;
        const int row = inst * RPI + lane / CPR;
        const int c = (lane % CPR) ^ tn_swz(row, TILE);
        const int gk = min(k0 + row, kend - 1);
        const int gc = min(c0 + 8 * c, cols - 8);
        dma16(p + (int64_t)gk * ld + gc, img + inst * 512);
    }
}

__device__ __forceinline__ bf16x8 frag_nt(const bf16* img, int row, int chunk) {
    return *reinterpret_cast<const bf16x8*>(img + row * 64 + ((chunk ^ (row & 7)) << 3));
}

template <int TILE>
__device__ __forceinline__ bf16x8 frag_tn(const bf16* img, int s, int col0, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int chunk = (col0 >> 3) + (p >> 1);
    const int r1 = 32 * s + 4 * g + q, r2 = r1 + 16;
    const bf16* a1 = img + r1 * TILE + ((chunk ^ tn_swz(r1, TILE)) << 3) + 4 * (p & 1);
    const bf16* a2 = img + r2 * TILE + ((chunk ^ tn_swz(r2, TILE)) << 3) + 4 * (p & 1);
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)const_cast<bf16*>(a1));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)const_cast<bf16*>(a2));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}

template <bool TN, int BM, int BN, int EPI>
__global__ __launch_bounds__(GB_THREADS, 2) void gemm_lds_kernel(
    const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb, int M, int N, int K,
    int kchunk, int ka, float* __restrict__ C, int64_t ldc, float* __restrict__ part, const float* __restrict__ addend,
    int64_t ldd, const uint8_t* __restrict__ aux8 = nullptr, EpiEdge ex = EpiEdge{}) {
    static_assert(BM == G2_BM || (EPI != EPI_STATS && EPI != EPI_STATS16), "stats rows are per 128-row tile");
    constexpr int WN = BN >= 128 ? 2 : 1;
    constexpr int WM = 4 / WN;
    constexpr int TM = BM / WM / 16;
    constexpr int TN_ = BN / WN / 16;
    constexpr int STAGE = (BM + BN) * G2_BK;  // bf16 elements per stage
    __shared__ __attribute__((aligned(16))) bf16 lds[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int nJ = (N + BN - 1) / BN;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    // tile order in groups of two row tiles: the 4 consecutive tiles an XCD
    // takes (xcd_remap) form a 2 x 2 square, so each A row panel and each B
    // column panel of a K-chunk is fetched by half as many XCDs as in row-major
    // order (which shares A panels but sends every B panel to all eight)
    const int nI = (M + BM - 1) / BM;
    int ti, tj;
    {
        const int gsz = 2 * nJ, grp = L / gsz, first = grp * 2, gm = min(nI - first, 2), r = L - grp * gsz;
        ti = first + r % gm;
        tj = r / gm;
    }
    const int i0 = ti * BM, j0 = tj * BN;
    const int kbeg = blockIdx.y * kchunk;
    const int kend = min(K, kbeg + kchunk);
    const int nk = kend > kbeg ? (kend - kbeg + G2_BK - 1) / G2_BK : 0;

    f32x4 acc[TM][TN_];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN_; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto stage = [&](int t, int buf) {
        bf16* img = lds + buf * STAGE;
        const int k0 = kbeg + t * G2_BK;
        if (TN) {
            stage_tn<BM>(A, lda, i0, M, k0, kend, img, wave, lane);
            stage_tn<BN>(B, ldb, j0, N, k0, kend, img + BM * G2_BK, wave, lane);
        } else {
            stage_nt<BM>(A, lda, i0, M, k0 % ka, img, wave, lane);  // ka < K: A reused (split weight)
            stage_nt<BN>(B, ldb, j0, N, k0, img + BM * G2_BK, wave, lane);
        }
    };
    if (nk > 0) stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
        const int cur = t & 1;
        if (t + 1 < nk) stage(t + 1, cur ^ 1);
        bf16* img = lds + cur * STAGE;
        if (TN && kbeg + (t + 1) * G2_BK > kend) {
            // partial last stage: k-rows past kend hold clamped copies -> zero them
            // (uniform branch: every wave takes it or none)
            const int valid = kend - kbeg - t * G2_BK;
            for (int e = tid; e < (G2_BK - valid) * (BM + BN) / 8; e += GB_THREADS) {
                const int per_a = (G2_BK - valid) * BM / 8;
                bf16x8 z = {};
                if (e < per_a) {
                    *reinterpret_cast<bf16x8*>(img + valid * BM + e * 8) = z;
                } else {
                    *reinterpret_cast<bf16x8*>(img + BM * G2_BK + valid * BN + (e - per_a) * 8) = z;
                }
            }
            __syncthreads();
        }
        const bf16* As = img;
        const bf16* Bs = img + BM * G2_BK;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 af[TM], bfv[TN_];
#pragma unroll
            for (int a = 0; a < TM; ++a) {
                if (TN) af[a] = frag_tn<BM>(As, s, wm * TM * 16 + a * 16, lane);
                else af[a] = frag_nt(As, wm * TM * 16 + a * 16 + (lane & 15), s * 4 + (lane >> 4));
            }
#pragma unroll
            for (int b = 0; b < TN_; ++b) {
                if (TN) bfv[b] = frag_tn<BN>(Bs, s, wn * TN_ * 16 + b * 16, lane);
                else bfv[b] = frag_nt(Bs, wn * TN_ * 16 + b * 16 + (lane & 15), s * 4 + (lane >> 4));
            }
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN_; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfv[b], acc[a][b], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    float* out = C;
    if (EPI == EPI_SLAB) out = C + (int64_t)blockIdx.y * M * N;
    if (EPI == EPI_STATS || EPI == EPI_STATS16) {
        // BatchNorm column partials from the fp32 accumulators
        const int cb = j0 + wn * TN_ * 16 + (lane & 15);
        const int rb = i0 + wm * TM * 16 + (lane >> 4) * 4;
        float s1[TN_], s2[TN_];
#pragma unroll
        for (int b = 0; b < TN_; ++b) { s1[b] = 0.f; s2[b] = 0.f; }
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int b = 0; b < TN_; ++b) {
                    const bool ok = rb + a * 16 + r < M && cb + b * 16 < N;
                    const float v = ok ? acc[a][b][r] : 0.f;
                    s1[b] += v;
                    s2[b] = fmaf(v, v, s2[b]);
                }
        float* red = reinterpret_cast<float*>(lds);  // [WM][BN][2]
#pragma unroll
        for (int b = 0; b < TN_; ++b) {
            float a1 = s1[b], a2 = s2[b];
            a1 += __shfl_xor(a1, 16);
            a2 += __shfl_xor(a2, 16);
            a1 += __shfl_xor(a1, 32);
            a2 += __shfl_xor(a2, 32);
            if (lane < 16) {
                const int jl = wn * TN_ * 16 + b * 16 + lane;
                red[(wm * BN + jl) * 2 + 0] = a1;
                red[(wm * BN + jl) * 2 + 1] = a2;
            }
        }
        __syncthreads();
        for (int jl = tid; jl < BN; jl += GB_THREADS) {
            const int j = j0 + jl;
            if (j >= N) continue;
            float t1 = 0.f, t2 = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) { t1 += red[(w * BN + jl) * 2]; t2 += red[(w * BN + jl) * 2 + 1]; }
            part[(int64_t)ti * 2 * N + j] = t1;
            part[(int64_t)ti * 2 * N + N + j] = t2;
        }
    }

    // Output through LDS: the fp32 tile goes row-major into the idle stage
    // buffers (in NR row rounds when it does not fit at once), then each thread
    // moves 16-byte row pieces (4 fp32 or 8 bf16 outputs per store) instead of
    // scalar stores of 16-lane column fragments.
    constexpr int LDT = BN + 4;
    constexpr int LDSB = 2 * STAGE * (int)sizeof(bf16);
    constexpr int NR = BM * LDT * 4 <= LDSB ? 1 : 2;
    constexpr int RR = BM / NR;
    static_assert(RR * LDT * 4 <= LDSB && WM % NR == 0, "epilogue tile must fit the stage buffers");
    constexpr int VO = (EPI == EPI_STATS16 || EPI == EPI_DZ2 || EPI == EPI_H1BWD) ? 8 : 4;  // outputs per 16-B store
    // EPI_EDZ (EdgeConv backward, dgx_gemm_edge_dz_bf16): the product + addend is
    // the gradient dY of the previous block's output; instead of storing it the
    // epilogue applies that block's LeakyReLU' / BN-backward input: dz = dY *
    // LReLU'(a ysel + b), stored as packed dz|slot words (the selected slot in the
    // 6 low mantissa bits, dgx_edge_bwd_dz_packed_f32's format) with the per-tile
    // column partials (sum dz, sum dz * yhat) — no dY round trip, no dz pass.
    // ex.PQ = ysel (ld ex.ldpq), aux8 = the forward's slots (same ld).
    float e1[4], e2[4];
    if constexpr (EPI == EPI_EDZ) {
#pragma unroll
        for (int u = 0; u < 4; ++u) { e1[u] = 0.f; e2[u] = 0.f; }
    }
    constexpr int CPR = BN / VO;
    float* tile = reinterpret_cast<float*>(lds);
    const bool vec_out = (ldc % VO) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                         (EPI != EPI_ACCUM || !addend ||
                          ((ldd % 4) == 0 && (reinterpret_cast<uintptr_t>(addend) & 15) == 0));
    // EPI_DZ2 (BN2 backward of the PositionEmbedding edge MLP, dense over edge
    // rows i = p*k + s): dZ2 = c1 z + c0 + [arg[p] == s] a2 dz[p], bf16 out;
    // part = [c0 | c1 | a2] (3 N), addend = dz (M/k x N), ldd = k, aux8 = arg.
    // A thread's output columns are fixed (GB_THREADS % CPR == 0), so its
    // constants are loaded once
    float k0[8], k1[8], a2[8];
    if constexpr (EPI == EPI_DZ2) {
        static_assert(GB_THREADS % CPR == 0, "fixed columns per thread");
        const int jc = min(j0 + (tid % CPR) * VO, N - 8);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            *reinterpret_cast<float4*>(k0 + 4 * h) = *reinterpret_cast<const float4*>(part + jc + 4 * h);
            *reinterpret_cast<float4*>(k1 + 4 * h) = *reinterpret_cast<const float4*>(part + N + jc + 4 * h);
            *reinterpret_cast<float4*>(a2 + 4 * h) = *reinterpret_cast<const float4*>(part + 2 * N + jc + 4 * h);
        }
    }
#pragma unroll
    for (int q = 0; q < NR; ++q) {
        __syncthreads();  // K loop / stats / previous round done with the buffers
        if (wm / (WM / NR) == q) {
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int b = 0; b < TN_; ++b)
                        tile[(wm * TM * 16 - q * RR + a * 16 + (lane >> 4) * 4 + r) * LDT + wn * TN_ * 16 + b * 16 +
                             (lane & 15)] = acc[a][b][r];
        }
        if constexpr (EPI == EPI_H1BWD) {
            // g = dH1 * LReLU'(a1 (P_j + Q_i) + b1) stored bf16 + BN1-backward column
            // partials; the rows' ids, P_j and Q_i pieces are loaded for all of this
            // round's iterations before the tile is ready (latency overlap)
            constexpr int IT = RR * CPR / GB_THREADS;
            static_assert(RR * CPR % GB_THREADS == 0 && GB_THREADS % CPR == 0, "whole iterations, fixed columns");
            const int jc = min(j0 + (tid % CPR) * VO, N - 8);
            float pv[IT][8], qv[IT][8];
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int e = tid + it * GB_THREADS;
                const int rr = e / CPR;
                const int64_t row = min((int64_t)(i0 + q * RR + rr), (int64_t)M - 1);
                const int64_t pi = row / ex.k;
                const int64_t pj = (pi / ex.N) * ex.N + ex.idx[row];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    *reinterpret_cast<float4*>(pv[it] + 4 * h) =
                        *reinterpret_cast<const float4*>(ex.PQ + pj * ex.ldpq + jc + 4 * h);
                    *reinterpret_cast<float4*>(qv[it] + 4 * h) =
                        *reinterpret_cast<const float4*>(ex.PQ + pi * ex.ldpq + N + jc + 4 * h);
                }
            }
            float ea[8], eb[8], em[8], ei[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                *reinterpret_cast<float4*>(ea + 4 * h) = *reinterpret_cast<const float4*>(ex.scale + jc + 4 * h);
                *reinterpret_cast<float4*>(eb + 4 * h) = *reinterpret_cast<const float4*>(ex.shift + jc + 4 * h);
                *reinterpret_cast<float4*>(em + 4 * h) = *reinterpret_cast<const float4*>(ex.mean + jc + 4 * h);
                *reinterpret_cast<float4*>(ei + 4 * h) = *reinterpret_cast<const float4*>(ex.invstd + jc + 4 * h);
            }
            __syncthreads();
            float t1[8], t2[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) { t1[u] = 0.f; t2[u] = 0.f; }
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int e = tid + it * GB_THREADS;
                const int rr = e / CPR, c = (e - rr * CPR) * VO;
                const int64_t i = i0 + q * RR + rr;
                const int j = j0 + c;
                if (i >= M || j + 8 > N) continue;
                const float* src = tile + rr * LDT + c;
                bf16x8 h;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const float y = pv[it][u] + qv[it][u];
                    const float z = fmaf(ea[u], y, eb[u]);
                    const float g = src[u] * (z > 0.f ? 1.f : ex.slope);
                    t1[u] += g;
                    t2[u] = fmaf(g, (y - em[u]) * ei[u], t2[u]);
                    h[u] = (bf16)g;
                }
                *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(out) + i * ldc + j) = h;
            }
            // column partials: the GB_THREADS / CPR threads of each column group
            __syncthreads();
            float* red = tile;  // [GB_THREADS][16]
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                red[tid * 16 + u] = t1[u];
                red[tid * 16 + 8 + u] = t2[u];
            }
            __syncthreads();
            for (int o = tid; o < 2 * BN; o += GB_THREADS) {
                const int which = o / BN, col = o - which * BN;  // col within the tile
                const int grp = col / VO, u = col - grp * VO;
                float acc_s = 0.f;
                for (int r = grp; r < GB_THREADS; r += CPR) acc_s += red[r * 16 + which * 8 + u];
                if (j0 + col < N) part[((int64_t)ti * 2 + which) * N + j0 + col] = acc_s;
            }
            continue;
        }
        if constexpr (EPI == EPI_EDZ) {
            constexpr int IT = RR * CPR / GB_THREADS;
            static_assert(RR * CPR % GB_THREADS == 0 && GB_THREADS % CPR == 0, "whole iterations, fixed columns");
            const int jc = min(j0 + (tid % CPR) * VO, N - 4);
            float yv[IT][4], av[IT][4];
            uint32_t sw[IT];
#pragma unroll
            for (int it = 0; it < IT; ++it) {   // loads of this round's rows issued before the tile is ready
                const int e = tid + it * GB_THREADS;
                const int64_t row = min((int64_t)(i0 + q * RR + e / CPR), (int64_t)M - 1);
                *reinterpret_cast<float4*>(yv[it]) = *reinterpret_cast<const float4*>(ex.PQ + row * ex.ldpq + jc);
                *reinterpret_cast<float4*>(av[it]) = *reinterpret_cast<const float4*>(addend + row * ldd + jc);
                sw[it] = *reinterpret_cast<const uint32_t*>(aux8 + row * ex.ldpq + jc);
            }
            float ea[4], eb[4], em[4], ei[4];
            *reinterpret_cast<float4*>(ea) = *reinterpret_cast<const float4*>(ex.scale + jc);
            *reinterpret_cast<float4*>(eb) = *reinterpret_cast<const float4*>(ex.shift + jc);
            *reinterpret_cast<float4*>(em) = *reinterpret_cast<const float4*>(ex.mean + jc);
            *reinterpret_cast<float4*>(ei) = *reinterpret_cast<const float4*>(ex.invstd + jc);
            __syncthreads();
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int e = tid + it * GB_THREADS;
                const int rr = e / CPR, c = (e - rr * CPR) * VO;
                const int64_t i = i0 + q * RR + rr;
                const int j = j0 + c;
                if (i >= M || j + 4 > N) continue;
                const float* src = tile + rr * LDT + c;
                uint32_t w[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float g = src[u] + av[it][u];   // dY, as EPI_ACCUM forms it
                    const float z = fmaf(ea[u], yv[it][u], eb[u]);
                    const float d = g * (z > 0.f ? 1.f : ex.slope);
                    e1[u] += d;
                    e2[u] = fmaf(d, (yv[it][u] - em[u]) * ei[u], e2[u]);
                    w[u] = (__float_as_uint(d) & ~63u) | ((sw[it] >> (8 * u)) & 0xffu);
                }
                *reinterpret_cast<uint4*>(out + i * ldc + j) = make_uint4(w[0], w[1], w[2], w[3]);
            }
            if (q == NR - 1) {   // column partials of the tile: the GB_THREADS / CPR threads of each column group
                __syncthreads();
                float* red = tile;  // [GB_THREADS][8]
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    red[tid * 8 + u] = e1[u];
                    red[tid * 8 + 4 + u] = e2[u];
                }
                __syncthreads();
                for (int o = tid; o < 2 * BN; o += GB_THREADS) {
                    const int which = o / BN, col = o - which * BN;
                    const int grp = col / VO, u = col - grp * VO;
                    float acc_s = 0.f;
                    for (int r = grp; r < GB_THREADS; r += CPR) acc_s += red[r * 8 + which * 4 + u];
                    if (j0 + col < N) part[((int64_t)ti * 2 + which) * N + j0 + col] = acc_s;
                }
            }
            continue;
        }
        if constexpr (EPI == EPI_DZ2) {
            // the rows' dz / slot pieces are loaded for all of this round's
            // iterations at once, before the tile is ready (latency overlap)
            constexpr int IT = RR * CPR / GB_THREADS;
            static_assert(RR * CPR % GB_THREADS == 0, "whole iterations");
            float dd[IT][8];
            uint2 aw[IT];
            const int64_t kk = ldd;
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int e = tid + it * GB_THREADS;
                const int rr = e / CPR, c = (e - rr * CPR) * VO;
                const int64_t i = min(i0 + q * RR + rr, M - 1);
                const int j = min(j0 + c, N - 8);
                const int64_t pnt = i / kk;
                *reinterpret_cast<float4*>(dd[it]) = *reinterpret_cast<const float4*>(addend + pnt * N + j);
                *reinterpret_cast<float4*>(dd[it] + 4) = *reinterpret_cast<const float4*>(addend + pnt * N + j + 4);
                aw[it] = *reinterpret_cast<const uint2*>(aux8 + pnt * N + j);
            }
            __syncthreads();
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int e = tid + it * GB_THREADS;
                const int rr = e / CPR, c = (e - rr * CPR) * VO;
                const int64_t i = i0 + q * RR + rr;
                const int j = j0 + c;
                if (i >= M || j + 8 > N) continue;
                const int sl = (int)(i - (i / kk) * kk);
                const float* src = tile + rr * LDT + c;
                bf16x8 h;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int slot = (int)(((u < 4 ? aw[it].x : aw[it].y) >> (8 * (u & 3))) & 0xffu);
                    const float v = fmaf(k1[u], src[u], k0[u]);
                    h[u] = (bf16)(slot == sl ? v + a2[u] * dd[it][u] : v);
                }
                *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(out) + i * ldc + j) = h;
            }
            continue;
        }
        __syncthreads();
        for (int e = tid; e < RR * CPR; e += GB_THREADS) {
            const int rr = e / CPR, c = (e - rr * CPR) * VO;
            const int i = i0 + q * RR + rr, j = j0 + c;
            if (i >= M || j >= N) continue;
            const float* src = tile + rr * LDT + c;
            if (vec_out && j + VO <= N) {
                if constexpr (EPI == EPI_STATS16) {
                    const float4 u = *reinterpret_cast<const float4*>(src);
                    const float4 w = *reinterpret_cast<const float4*>(src + 4);
                    bf16x8 h = {(bf16)u.x, (bf16)u.y, (bf16)u.z, (bf16)u.w, (bf16)w.x, (bf16)w.y, (bf16)w.z, (bf16)w.w};
                    *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(out) + (int64_t)i * ldc + j) = h;
                } else {
                    float4 v = *reinterpret_cast<const float4*>(src);
                    float4* dst = reinterpret_cast<float4*>(out + (int64_t)i * ldc + j);
                    if (EPI == EPI_ACCUM) {
                        const float4 o = addend ? *reinterpret_cast<const float4*>(addend + (int64_t)i * ldd + j) : *dst;
                        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
                    }
                    *dst = v;
                }
            } else {
                for (int u = 0; u < VO && j + u < N; ++u) {
                    const float v = src[u];
                    if (EPI == EPI_STATS16) {
                        reinterpret_cast<bf16*>(out)[(int64_t)i * ldc + j + u] = (bf16)v;
                    } else {
                        float* dst = out + (int64_t)i * ldc + j + u;
                        if (EPI == EPI_ACCUM) *dst = (addend ? addend[(int64_t)i * ldd + j + u] : *dst) + v;
                        else *dst = v;
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// 256 x 256 NT tile for the large GEMMs (conv5 forward Z = Xcat W5^T, K = 512,
// and its input gradient dX = dZ W5, K = emb; models/dgcnn.py:74-78, 100-102).
// 8 waves (2 along M x 4 along N), each owning a 128 x 64 sub-tile = 8 x 4
// blocks of v_mfma_f32_16x16x32_bf16 (128 accumulator registers), K-steps of 64.
// Operands move by LDS-DMA (global_load_lds_dwordx4) into rings sized by where
// they come from: A (the activation stream, read once from HBM) has 3 slots and
// is fetched two K-steps ahead; B (the weight, L2-resident) has 2 slots and is
// fetched one K-step ahead. 3 x 32 + 2 x 32 KiB = the whole 160 KiB of LDS. Each
// K-step is four MFMA phases (one C quadrant x K = 64 = 16 MFMAs, fragments read
// where they change); the next K-steps' DMA is issued in pieces across the
// phases, B(t+1) before A(t+2), so the K-step ends on a COUNTED vmcnt (A(t+2)
// stays in flight) and a raw s_barrier: no drain of the DMA queue in the loop.
// LDS image per operand: [row][64 k] bf16, 128-B rows; 16-B chunk c of row r at
// position c ^ ((r >> 1) & 7): a ds_read_b128 lane group (16 rows, one chunk)
// then covers the 16 (row parity, position) slots of a 256-B bank row once —
// conflict-free (the swizzle is applied to each lane's SOURCE address, the DMA
// destination being lane-linear).
constexpr int G3_BM = 256, G3_BN = 256, G3_BK = 64, G3_THREADS = 512;
constexpr int G3_TILE = G3_BM * G3_BK;  // bf16 elements of one operand's K-step image (32 KiB)
constexpr int G3_ASLOTS = 3, G3_BSLOTS = 2;

__device__ __forceinline__ int g3_pos(int row, int c) { return c ^ ((row >> 1) & 7); }

// Half h (rows [128h, 128h + 128)) of one operand's K-step image: 16 KiB = 16
// wave-instructions; wave w issues instructions 2w, 2w + 1.
__device__ __forceinline__ void g3_stage_half(const bf16* __restrict__ src, int64_t ld, int r0, int rows, int kc,
                                              bf16* img, int h, int wave, int lane) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int inst = h * 16 + wave * 2 + u;  // 1 KiB = 8 rows per instruction
        const int row = inst * 8 + (lane >> 3);
        const int pos = lane & 7;
        const int c = pos ^ ((row >> 1) & 7);   // the chunk this lane's DMA lands at `pos`
        const int gr = min(r0 + row, rows - 1);
        dma16(src + (int64_t)gr * ld + kc + 8 * c, img + inst * 512);
    }
}

__device__ __forceinline__ bf16x8 g3_frag(const bf16* img, int row, int chunk) {
    return *reinterpret_cast<const bf16x8*>(img + row * 64 + (g3_pos(row, chunk) << 3));
}

template <int EPI>
__global__ __launch_bounds__(G3_THREADS, 1) void gemm256_nt_kernel(
    const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb, int M, int N, int K, int ka,
    float* __restrict__ C, int64_t ldc, float* __restrict__ part, const float* __restrict__ addend, int64_t ldd) {
    // A ring (3 slots) | B ring (2 slots): one array (a second __shared__ object
    // can make hipcc wait for the DMA queue before every ds_read)
    __shared__ __attribute__((aligned(16))) bf16 lds[(G3_ASLOTS + G3_BSLOTS) * G3_TILE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int nJ = (N + G3_BN - 1) / G3_BN;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int ti = L / nJ, tj = L - ti * nJ;
    const int i0 = ti * G3_BM, j0 = tj * G3_BN;
    const int nk = K / G3_BK;
    bf16* const aring = lds;
    bf16* const bring = lds + G3_ASLOTS * G3_TILE;

    f32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto stageA = [&](int t, int h) {
        if (t < nk) g3_stage_half(A, lda, i0, M, (t * G3_BK) % ka, aring + (t % G3_ASLOTS) * G3_TILE, h, wave, lane);
    };
    auto stageB = [&](int t, int h) {
        if (t < nk) g3_stage_half(B, ldb, j0, N, t * G3_BK, bring + (t % G3_BSLOTS) * G3_TILE, h, wave, lane);
    };
    // prologue: A(0), B(0), then A(1) left in flight (4 DMA per thread per operand K-step)
    stageA(0, 0); stageA(0, 1);
    stageB(0, 0); stageB(0, 1);
    stageA(1, 0); stageA(1, 1);
    if (nk > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    const int fr = lane & 15, fq = lane >> 4;
    for (int t = 0; t < nk; ++t) {
        const bf16* As = aring + (t % G3_ASLOTS) * G3_TILE;
        const bf16* Bs = bring + (t % G3_BSLOTS) * G3_TILE;
        bf16x8 bfr[2][2][2];  // [col half][col block][k sub-step]
        bf16x8 afr[4][2];     // [row block of the row half][k sub-step]
        // quadrant order (row half, col half): (0,0) (0,1) (1,1) (1,0): A read twice, B once
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int rh = q >> 1;
            const int ch = (q == 1 || q == 2) ? 1 : 0;
            if (q == 0) {
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
#pragma unroll
                        for (int s = 0; s < 2; ++s)
                            bfr[h][b][s] = g3_frag(Bs, wc * 64 + h * 32 + b * 16 + fr, s * 4 + fq);
            }
            if (q == 0 || q == 2) {
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int s = 0; s < 2; ++s)
                        afr[a][s] = g3_frag(As, wr * 128 + rh * 64 + a * 16 + fr, s * 4 + fq);
            }
            // next K-steps' DMA: B(t+1) in phases 0-1, then A(t+2) in phases 2-3
            if (q < 2) stageB(t + 1, q);
            else stageA(t + 2, q - 2);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc[rh * 4 + a][ch * 2 + b] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[a][s], bfr[ch][b][s], acc[rh * 4 + a][ch * 2 + b],
                                                                    0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
        // A(t+1) and B(t+1) landed (A(t+2) may stay in flight), and every wave is
        // done reading the slots the next K-step's DMA overwrites
        if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }

    // ---- epilogue
    // accumulator (a, b)[r]: row wr*128 + a*16 + fq*4 + r, column wc*64 + b*16 + fr
    if (EPI == EPI_STATS || EPI == EPI_STATS16) {
        // BatchNorm column partials of this wave's 128 rows from the fp32 sums:
        // partial row 2*ti + wr (128-row granularity, dgx_gemm_stats_rows)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            float s1 = 0.f, s2 = 0.f;
            const int col = j0 + wc * 64 + b * 16 + fr;
#pragma unroll
            for (int a = 0; a < 8; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const bool ok = i0 + wr * 128 + a * 16 + fq * 4 + r < M && col < N;
                    const float v = ok ? acc[a][b][r] : 0.f;
                    s1 += v;
                    s2 = fmaf(v, v, s2);
                }
            s1 += __shfl_xor(s1, 16);
            s2 += __shfl_xor(s2, 16);
            s1 += __shfl_xor(s1, 32);
            s2 += __shfl_xor(s2, 32);
            const int prow = 2 * ti + wr;
            if (fq == 0 && col < N && i0 + wr * 128 < M) {
                part[(int64_t)prow * 2 * N + col] = s1;
                part[(int64_t)prow * 2 * N + N + col] = s2;
            }
        }
    }
    // Output through LDS in 4 rounds of 64 rows x 256 columns (fp32, padded
    // rows): waves holding those rows write their accumulators, then every
    // thread moves 16-byte row pieces (4 fp32 / 8 bf16 outputs per store).
    constexpr int LDT = G3_BN + 4;
    constexpr int VO = EPI == EPI_STATS16 ? 8 : 4;
    constexpr int CPR = G3_BN / VO;
    float* tile = reinterpret_cast<float*>(lds);
    const bool vec_out = (ldc % VO) == 0 && (reinterpret_cast<uintptr_t>(C) & 15) == 0 &&
                         (EPI != EPI_ACCUM || !addend ||
                          ((ldd % 4) == 0 && (reinterpret_cast<uintptr_t>(addend) & 15) == 0));
#pragma unroll
    for (int rnd = 0; rnd < 4; ++rnd) {
        // round rnd holds rows [64 rnd, 64 rnd + 64): wave half wr = rnd >> 1, row blocks 4*(rnd&1) .. +4
        if (wr == (rnd >> 1)) {
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        tile[(a * 16 + fq * 4 + r) * LDT + wc * 64 + b * 16 + fr] = acc[(rnd & 1) * 4 + a][b][r];
        }
        __syncthreads();
        for (int e = tid; e < 64 * CPR; e += G3_THREADS) {
            const int rr = e / CPR, c = (e - rr * CPR) * VO;
            const int i = i0 + rnd * 64 + rr, j = j0 + c;
            if (i >= M || j >= N) continue;
            const float* src = tile + rr * LDT + c;
            if (vec_out && j + VO <= N) {
                if constexpr (EPI == EPI_STATS16) {
                    const float4 u = *reinterpret_cast<const float4*>(src);
                    const float4 w = *reinterpret_cast<const float4*>(src + 4);
                    bf16x8 h = {(bf16)u.x, (bf16)u.y, (bf16)u.z, (bf16)u.w, (bf16)w.x, (bf16)w.y, (bf16)w.z, (bf16)w.w};
                    *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(C) + (int64_t)i * ldc + j) = h;
                } else {
                    float4 v = *reinterpret_cast<const float4*>(src);
                    float4* dst = reinterpret_cast<float4*>(C + (int64_t)i * ldc + j);
                    if (EPI == EPI_ACCUM) {
                        const float4 o = addend ? *reinterpret_cast<const float4*>(addend + (int64_t)i * ldd + j) : *dst;
                        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
                    }
                    *dst = v;
                }
            } else {
                for (int u = 0; u < VO && j + u < N; ++u) {
                    const float v = src[u];
                    if (EPI == EPI_STATS16) {
                        reinterpret_cast<bf16*>(C)[(int64_t)i * ldc + j + u] = (bf16)v;
                    } else {
                        float* dst = C + (int64_t)i * ldc + j + u;
                        if (EPI == EPI_ACCUM) *dst = (addend ? addend[(int64_t)i * ldd + j + u] : *dst) + v;
                        else *dst = v;
                    }
                }
            }
        }
        __syncthreads();
    }
}

template <int EPI>
int launch_gemm256(const bf16* A, int64_t lda, const bf16* B, int64_t ldb, int M, int N, int K, int ka, float* C,
                   int64_t ldc, float* part, const float* addend, int64_t ldd, hipStream_t st) {
    const int nI = (M + G3_BM - 1) / G3_BM, nJ = (N + G3_BN - 1) / G3_BN;
    hipLaunchKernelGGL((gemm256_nt_kernel<EPI>), dim3((unsigned)(nI * nJ)), dim3(G3_THREADS), 0, st, A, lda, B, ldb,
                       M, N, K, ka, C, ldc, part, addend, ldd);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

template <bool TN, int BN, int EPI>
int launch_gemm_lds(const bf16* A, int64_t lda, const bf16* B, int64_t ldb, int M, int N, int K, int ka, int splits,
                    float* C, int64_t ldc, float* part, const float* addend, int64_t ldd, hipStream_t st) {
    int kchunk = (K + splits - 1) / splits;
    kchunk = (kchunk + G2_BK - 1) / G2_BK * G2_BK;
    const int sp = (K + kchunk - 1) / kchunk;
    const int nJ = (N + BN - 1) / BN;
    // skinny outputs (few 128-row tiles): 64-row tiles double the workgroups so
    // two share each CU and hide each other's load latency
    constexpr bool can_half = EPI != EPI_STATS && EPI != EPI_STATS16;
    const bool half = can_half && ((M + G2_BM - 1) / G2_BM) * nJ * sp < 512;
    if constexpr (can_half) {
        if (half) {
            const int nI = (M + 63) / 64;
            dim3 grid((unsigned)(nI * nJ), (unsigned)(EPI == EPI_SLAB ? sp : 1));
            hipLaunchKernelGGL((gemm_lds_kernel<TN, 64, BN, EPI>), grid, dim3(GB_THREADS), 0, st, A, lda, B, ldb, M,
                               N, K, EPI == EPI_SLAB ? kchunk : K, ka, C, ldc, part, addend, ldd);
            return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
        }
    }
    {
        const int nI = (M + G2_BM - 1) / G2_BM;
        dim3 grid((unsigned)(nI * nJ), (unsigned)(EPI == EPI_SLAB ? sp : 1));
        hipLaunchKernelGGL((gemm_lds_kernel<TN, G2_BM, BN, EPI>), grid, dim3(GB_THREADS), 0, st, A, lda, B, ldb, M,
                           N, K, EPI == EPI_SLAB ? kchunk : K, ka, C, ldc, part, addend, ldd);
    }
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

// Weight operands for the bf16 GEMMs, one launch per layer: `nt` = [rows][K]
// (the GEMM's B for X W^T), `tn` = its transpose (the B for dY W). For an
// EdgeConv weight W (Co, 2C) (reference conv weight, dgcnn.py:55) the rows are
// the stacked halves [W1; W2] (2Co, C); for conv5 W (Co, K) as is.
// 32 x 32 tiles through LDS, so both the row-major copy and the transpose are
// written with coalesced (row-contiguous) stores; 4 independent elements per
// thread (64 x 64 tiles left ~150 workgroups with 16 dependent trips each for
// DGCNN's weights: 11.5 us per step for 2.8 MB)
constexpr int WP_T = 32;
__global__ __launch_bounds__(256) void weight_prep_kernel(const float* __restrict__ W, int Co, int C, int stacked,
                                                          bf16* __restrict__ nt, bf16* __restrict__ tn) {
    __shared__ bf16 tile[WP_T][WP_T + 2];
    const int rows = stacked ? 2 * Co : Co;
    const int r0 = blockIdx.y * WP_T, c0 = blockIdx.x * WP_T;
    const int t = threadIdx.x;
#pragma unroll
    for (int e = t; e < WP_T * WP_T; e += 256) {
        const int rr = e / WP_T, cc = e - rr * WP_T;
        const int r = r0 + rr, c = c0 + cc;
        if (r < rows && c < C) {
            const float v = stacked ? W[(int64_t)(r % Co) * 2 * C + (r / Co) * C + c] : W[(int64_t)r * C + c];
            const bf16 h = (bf16)v;
            nt[(int64_t)r * C + c] = h;
            tile[rr][cc] = h;
        }
    }
    __syncthreads();
#pragma unroll
    for (int e = t; e < WP_T * WP_T; e += 256) {
        const int cc = e / WP_T, rr = e - cc * WP_T;
        const int r = r0 + rr, c = c0 + cc;
        if (r < rows && c < C) tn[(int64_t)c * rows + r] = tile[rr][cc];
    }
}

constexpr int WP_MAXJ_S = 8;
// fp32 stacked EdgeConv weights [W1; W2] (2 Co x C) of several blocks in one
// launch (the parity mode's GEMM operands; the reference layout is [W1 | W2],
// Co x 2C): job j owns blocks [first[j], first[j+1]), 256 elements each.
struct WeightStackJobs {
    const float* W[WP_MAXJ_S];
    float* out[WP_MAXJ_S];
    int Co[WP_MAXJ_S], C[WP_MAXJ_S], first[WP_MAXJ_S + 1];
    int n;
};
__global__ __launch_bounds__(256) void weight_stack_multi_kernel(WeightStackJobs jobs) {
    int j = 0;
    while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.first[j + 1]) ++j;
    const int Co = jobs.Co[j], C = jobs.C[j];
    const int64_t e = (int64_t)(blockIdx.x - jobs.first[j]) * 256 + threadIdx.x;
    if (e >= (int64_t)2 * Co * C) return;
    const int r = (int)(e / C), c = (int)(e - (int64_t)r * C);
    jobs.out[j][e] = jobs.W[j][(int64_t)(r % Co) * 2 * C + (r / Co) * C + c];
}

// Several weights in one launch (the EdgeConv blocks of one forward): job j
// owns blocks [first[j], first[j+1]) of the 1-D grid, tiles row-major in it.
constexpr int WP_MAXJ = 8;
struct WeightPrepJobs {
    const float* W[WP_MAXJ];
    bf16* nt[WP_MAXJ];
    bf16* tn[WP_MAXJ];
    int Co[WP_MAXJ], C[WP_MAXJ], stacked[WP_MAXJ], first[WP_MAXJ + 1];
    int n;
};
__global__ __launch_bounds__(256) void weight_prep_multi_kernel(WeightPrepJobs jobs) {
    __shared__ bf16 tile[WP_T][WP_T + 2];
    __shared__ bf16 tlo[WP_T][WP_T + 2];
    int j = 0;
    while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.first[j + 1]) ++j;
    const int Co = jobs.Co[j], C = jobs.C[j], stacked = jobs.stacked[j] & 1, split = jobs.stacked[j] & 2;
    const int tsplit = jobs.stacked[j] & 4;   // tn rows are [hi | lo] too (C x 2 rows)
    const float* __restrict__ W = jobs.W[j];
    const int rows = stacked ? 2 * Co : Co;
    const int ldn = split ? 2 * C : C;  // split: nt rows are [hi | lo], lo = bf16(w - hi)
    const int ldt = tsplit ? 2 * rows : rows;
    const int ntc = (C + WP_T - 1) / WP_T;
    const int b = blockIdx.x - jobs.first[j];
    const int r0 = (b / ntc) * WP_T, c0 = (b % ntc) * WP_T;
    const int t = threadIdx.x;
#pragma unroll
    for (int e = t; e < WP_T * WP_T; e += 256) {
        const int rr = e / WP_T, cc = e - rr * WP_T;
        const int r = r0 + rr, c = c0 + cc;
        if (r < rows && c < C) {
            const float v = stacked ? W[(int64_t)(r % Co) * 2 * C + (r / Co) * C + c] : W[(int64_t)r * C + c];
            const bf16 h = (bf16)v;
            const bf16 l = (bf16)(v - (float)h);
            jobs.nt[j][(int64_t)r * ldn + c] = h;
            if (split) jobs.nt[j][(int64_t)r * ldn + C + c] = l;
            tile[rr][cc] = h;
            tlo[rr][cc] = l;
        }
    }
    __syncthreads();
#pragma unroll
    for (int e = t; e < WP_T * WP_T; e += 256) {
        const int cc = e / WP_T, rr = e - cc * WP_T;
        const int r = r0 + rr, c = c0 + cc;
        if (r < rows && c < C) {
            jobs.tn[j][(int64_t)c * ldt + r] = tile[rr][cc];
            if (tsplit) jobs.tn[j][(int64_t)c * ldt + rows + r] = tlo[rr][cc];
        }
    }
}

// fp32 -> (hi, lo) bf16 planes: hi = bf16(x), lo = bf16(x - hi) (16 significant
// bits together): the operands of the fp32 mode's 3-pass GEMMs
// hi.W_hi + hi.W_lo + lo.W_hi (dgx_split_bf16)
__global__ __launch_bounds__(256) void split_bf16_kernel(const float* __restrict__ src, int64_t lds, int64_t rows,
                                                         int cols, bf16* __restrict__ hi, bf16* __restrict__ lo,
                                                         int64_t ldo) {
    const int64_t n4 = (int64_t)rows * (cols / 4);
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256) {
        const int64_t r = e / (cols / 4);
        const int c = (int)(e - r * (cols / 4)) * 4;
        const float4 v = *reinterpret_cast<const float4*>(src + r * lds + c);
        const bf16x4 h = {(bf16)v.x, (bf16)v.y, (bf16)v.z, (bf16)v.w};
        const bf16x4 l = {(bf16)(v.x - (float)h[0]), (bf16)(v.y - (float)h[1]), (bf16)(v.z - (float)h[2]),
                          (bf16)(v.w - (float)h[3])};
        if (hi) *reinterpret_cast<bf16x4*>(hi + r * ldo + c) = h;
        *reinterpret_cast<bf16x4*>(lo + r * ldo + c) = l;
    }
}

template <typename TA, bool AIC, typename TB, bool BIC, int BN, int EPI>
int launch_gemm(const void* A, int64_t lda, const void* B, int64_t ldb, int M, int N, int K, int splits,
                int vec_a, int vec_b, float* C, int64_t ldc, float* part, hipStream_t st) {
    const int nI = (M + GB_BM - 1) / GB_BM, nJ = (N + BN - 1) / BN;
    int kchunk = (K + splits - 1) / splits;
    kchunk = (kchunk + GB_BK - 1) / GB_BK * GB_BK;
    const int sp = (K + kchunk - 1) / kchunk;
    dim3 grid((unsigned)(nI * nJ), (unsigned)(EPI == EPI_SLAB ? sp : 1));
    hipLaunchKernelGGL((gemm_bf16_kernel<TA, AIC, TB, BIC, BN, EPI>), grid, dim3(GB_THREADS), 0, st,
                       static_cast<const TA*>(A), lda, static_cast<const TB*>(B), ldb, M, N, K,
                       EPI == EPI_SLAB ? kchunk : K, vec_a, vec_b, C, ldc, part);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

// Weight gradient with a narrow second operand (layer 1: dW = dPQ^T X, X has
// 3 channels): C slab[y][i][j] = sum over k in split y of A[k][i] B[k][j], A bf16
// (i contiguous), B fp32 rounded to bf16 like every operand of the bf16 GEMMs,
// fp32 accumulation. One thread per output row i, the split's B rows staged in
// LDS; the MFMA tile path would pad N to 64 columns (95 % idle at N = 3).
constexpr int AS_ROWS = 256;
template <int NB>
__global__ __launch_bounds__(256) void atb_small_kernel(const bf16* __restrict__ A, int64_t lda,
                                                        const float* __restrict__ B, int64_t ldb, int M, int N,
                                                        int K, int kchunk, float* __restrict__ slab) {
    __shared__ float bs[AS_ROWS][NB];
    const int kbeg = blockIdx.x * kchunk, kend = min(K, kbeg + kchunk);
    float* out = slab + (int64_t)blockIdx.x * M * N;
    for (int i0 = 0; i0 < M; i0 += 256) {
        const int i = i0 + threadIdx.x;
        float acc[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[j] = 0.f;
        for (int k0 = kbeg; k0 < kend; k0 += AS_ROWS) {
            const int nk = min(AS_ROWS, kend - k0);
            __syncthreads();
            for (int e = threadIdx.x; e < AS_ROWS * NB; e += 256) {
                const int kk = e / NB, j = e - kk * NB;
                bs[kk][j] = (kk < nk && j < N) ? (float)(bf16)B[(int64_t)(k0 + kk) * ldb + j] : 0.f;
            }
            __syncthreads();
            if (i < M) {
                const bf16* a = A + (int64_t)k0 * lda + i;
#pragma unroll 8
                for (int kk = 0; kk < nk; ++kk) {
                    const float av = (float)a[(int64_t)kk * lda];
#pragma unroll
                    for (int j = 0; j < NB; ++j) acc[j] = fmaf(av, bs[kk][j], acc[j]);
                }
            }
        }
        if (i < M)
            for (int j = 0; j < N; ++j) out[(int64_t)i * N + j] = acc[j];
    }
}

bool aligned_to(const void* p, int bytes) { return (reinterpret_cast<uintptr_t>(p) % bytes) == 0; }

// Exact fp32 GEMM for a short reduction (K <= 16): C (M x N) = X (M x K) W^T
// with W (N x K), every output an fmaf chain over k in order. Used for the
// layer-1 per-point GEMM on raw coordinates (K = 3, dgcnn.py:55 / layers.py:17):
// bf16 rounding of xyz there is the largest single error term of the bf16 mode
// (edge values y = P_j + Q_i of close neighbours nearly cancel in BN), and the
// work (2*M*N*K flops) is a few microseconds of HBM writes, not a GEMM.
// Block = 16 rows (2048 blocks at cfg2: 64 rows left a quarter of the CUs idle,
// 9.8 -> 8.8 us, r04r); W and the rows' X staged in LDS; each thread writes 4
// consecutive columns (16-B stores along the row).
#ifndef SK_ROWS_DEF
#define SK_ROWS_DEF 16
#endif
constexpr int SK_ROWS = SK_ROWS_DEF;
constexpr int SK_MAXK = 16;
// split != 0: W is a conv weight in the reference layout (N/2, 2K) = [W1 | W2]
// and row n of the product's weight is W1[n] (n < N/2) or W2[n - N/2]: the
// EdgeConv block's [W1; W2] without a separate reshuffle (torch.cat) launch.
__global__ __launch_bounds__(256) void smallk_gemm_kernel(const float* __restrict__ X, int64_t ldx,
                                                          const float* __restrict__ W, int M, int N, int K,
                                                          float* __restrict__ C, int64_t ldc, int split) {
    extern __shared__ float sk[];  // W [N][K] | X [SK_ROWS][K]
    float* ws = sk;
    float* xs = sk + N * K;
    const int r0 = blockIdx.x * SK_ROWS;
    const int rows = min(SK_ROWS, M - r0);
    const int half = N >> 1;
    for (int e = threadIdx.x; e < N * K; e += 256) {
        const int n = e / K, c = e - n * K;
        ws[e] = split ? W[(n < half ? n : n - half) * 2 * K + (n < half ? 0 : K) + c] : W[e];
    }
    for (int e = threadIdx.x; e < rows * K; e += 256) {
        const int r = e / K, c = e - r * K;
        xs[e] = X[(int64_t)(r0 + r) * ldx + c];
    }
    __syncthreads();
    const int nq = N >> 2;  // N % 4 == 0 (checked by the launcher)
    for (int e = threadIdx.x; e < rows * nq; e += 256) {
        const int r = e / nq, j = (e - r * nq) * 4;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < K; ++c) {
            const float xv = xs[r * K + c];
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] = fmaf(xv, ws[(j + u) * K + c], acc[u]);
        }
        *reinterpret_cast<float4*>(C + (int64_t)(r0 + r) * ldc + j) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    }
}

}  // namespace

extern "C" {

int dgx_gemm_smallk_f32(const float* X, int64_t ldx, const float* W, int M, int N, int K, float* C, int64_t ldc,
                        void* stream) {
    if (!X || !W || !C || M < 1 || N < 4 || K < 1 || ldx < K || ldc < N) return DGX_EINVAL;
    if (K > SK_MAXK || N % 4 || ldc % 4 || reinterpret_cast<uintptr_t>(C) % 16) return DGX_EUNSUPPORTED;
    if ((size_t)(N + SK_ROWS) * K * sizeof(float) > 64 * 1024) return DGX_EUNSUPPORTED;
    const size_t lds = (size_t)(N + SK_ROWS) * K * sizeof(float);
    hipLaunchKernelGGL(smallk_gemm_kernel, dim3((M + SK_ROWS - 1) / SK_ROWS), dim3(256), lds, dgx_stream(stream), X,
                       ldx, W, M, N, K, C, ldc, 0);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_gemm_smallk_split_f32(const float* X, int64_t ldx, const float* Wref, int M, int Co, int K, float* C,
                              int64_t ldc, void* stream) {
    const int N = 2 * Co;
    if (!X || !Wref || !C || M < 1 || Co < 2 || K < 1 || ldx < K || ldc < N) return DGX_EINVAL;
    if (K > SK_MAXK || N % 4 || ldc % 4 || reinterpret_cast<uintptr_t>(C) % 16) return DGX_EUNSUPPORTED;
    if ((size_t)(N + SK_ROWS) * K * sizeof(float) > 64 * 1024) return DGX_EUNSUPPORTED;
    const size_t lds = (size_t)(N + SK_ROWS) * K * sizeof(float);
    hipLaunchKernelGGL(smallk_gemm_kernel, dim3((M + SK_ROWS - 1) / SK_ROWS), dim3(256), lds, dgx_stream(stream), X,
                       ldx, Wref, M, N, K, C, ldc, 1);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_gemm_stats_rows(int M) { return (M + GB_BM - 1) / GB_BM; }

int dgx_gemm_splits(int M, int N, int K) {
    // split-K factor of a SLAB GEMM: about 2 workgroups per CU (256 CUs), each
    // split at least 8 K-steps deep
    if (N <= 4) {  // atb_small_kernel: one block per split, 64+ rows each, ~2 blocks per CU
        const int s = (K + 63) / 64;
        return s < 1 ? 1 : (s > 512 ? 512 : s);
    }
    const int BN = N > 64 ? 128 : 64;
    const int tiles = ((M + GB_BM - 1) / GB_BM) * ((N + BN - 1) / BN);
    int s = (512 + tiles - 1) / tiles;
    const int maxs = (K + 8 * GB_BK - 1) / (8 * GB_BK);
    if (s > maxs) s = maxs;
    return s < 1 ? 1 : s;
}

int dgx_gemm_bf16(const void* A, int a_bf16, int a_ic, int64_t lda, const void* B, int b_bf16, int b_ic,
                  int64_t ldb, int M, int N, int K, int epi, int splits, float* C, int64_t ldc, float* partials,
                  void* stream) {
    if (!A || !B || !C || M < 0 || N < 0 || K < 0 || lda < 1 || ldb < 1 || ldc < 1 || splits < 1)
        return DGX_EINVAL;
    if (epi == EPI_STATS && !partials) return DGX_EINVAL;
    if (M == 0 || N == 0) return DGX_OK;
    if (epi == EPI_SLAB) ldc = N;  // slabs are dense [splits][M][N]
    hipStream_t st = dgx_stream(stream);
    const int va = a_bf16 ? 8 : 4, vb = b_bf16 ? 8 : 4;
    const int vec_a = (lda % va == 0) && aligned_to(A, 16);
    const int vec_b = (ldb % vb == 0) && aligned_to(B, 16);
    const bool wide = N > 64;
#define DGX_GEMM(TA, AIC, TB, BIC, E)                                                                          \
    return wide ? launch_gemm<TA, AIC, TB, BIC, 128, E>(A, lda, B, ldb, M, N, K, splits, vec_a, vec_b, C, ldc, \
                                                        partials, st)                                          \
                : launch_gemm<TA, AIC, TB, BIC, 64, E>(A, lda, B, ldb, M, N, K, splits, vec_a, vec_b, C, ldc,  \
                                                       partials, st)
    // the operand layouts the engine uses; others are rejected
    if (!a_bf16 && !a_ic && !b_bf16 && !b_ic) {  // X W^T: forward PQ, conv5
        if (epi == EPI_STORE) DGX_GEMM(float, false, float, false, EPI_STORE);
        if (epi == EPI_STATS) DGX_GEMM(float, false, float, false, EPI_STATS);
    }
    if (!a_ic && !b_bf16 && b_ic) {  // dPQ Wcat / dZ W5: input gradients
        if (!a_bf16 && epi == EPI_ACCUM) DGX_GEMM(float, false, float, true, EPI_ACCUM);
        if (!a_bf16 && epi == EPI_STORE) DGX_GEMM(float, false, float, true, EPI_STORE);
        if (a_bf16 && epi == EPI_ACCUM) DGX_GEMM(bf16, false, float, true, EPI_ACCUM);
        if (a_bf16 && epi == EPI_STORE) DGX_GEMM(bf16, false, float, true, EPI_STORE);
    }
    if (a_ic && b_ic && !b_bf16 && epi == EPI_SLAB) {  // dPQ^T X / dZ^T X: weight gradients
        if (a_bf16 && N <= 4) {  // same split geometry (kchunk, slab count) as launch_gemm
            int kchunk = (K + splits - 1) / splits;
            kchunk = (kchunk + GB_BK - 1) / GB_BK * GB_BK;
            const int sp = (K + kchunk - 1) / kchunk;
            hipLaunchKernelGGL(atb_small_kernel<4>, dim3((unsigned)sp), dim3(256), 0, st, static_cast<const bf16*>(A),
                               lda, static_cast<const float*>(B), ldb, M, N, K, kchunk, C);
            return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
        }
        if (a_bf16) DGX_GEMM(bf16, true, float, true, EPI_SLAB);
        DGX_GEMM(float, true, float, true, EPI_SLAB);
    }
#undef DGX_GEMM
    return DGX_EUNSUPPORTED;
}

int dgx_gemm_dz2_bf16(const void* H1, const void* W2, int M, int N, int K, const float* dz, const uint8_t* arg,
                      const float* consts, int k, void* dZ2, void* stream) {
    if (!H1 || !W2 || !dz || !arg || !consts || !dZ2 || M < 1 || N < 1 || K < 1 || k < 1 || M % k) return DGX_EINVAL;
    if (!aligned_to(H1, 16) || !aligned_to(W2, 16) || !aligned_to(dz, 16) || !aligned_to(consts, 16) ||
        !aligned_to(dZ2, 16) || reinterpret_cast<uintptr_t>(arg) % 8 || K % G2_BK || N % 8)
        return DGX_EUNSUPPORTED;
    const bf16* a = static_cast<const bf16*>(H1);
    const bf16* b = static_cast<const bf16*>(W2);
    float* out = static_cast<float*>(dZ2);
    hipStream_t st = dgx_stream(stream);
    const int nI = (M + G2_BM - 1) / G2_BM;
    if (N > 64) {
        const int nJ = (N + 127) / 128;
        hipLaunchKernelGGL((gemm_lds_kernel<false, G2_BM, 128, EPI_DZ2>), dim3((unsigned)(nI * nJ)), dim3(GB_THREADS),
                           0, st, a, (int64_t)K, b, (int64_t)K, M, N, K, K, K, out, (int64_t)N, const_cast<float*>(consts),
                           dz, (int64_t)k, arg);
    } else {
        const int nJ = (N + 63) / 64;
        hipLaunchKernelGGL((gemm_lds_kernel<false, G2_BM, 64, EPI_DZ2>), dim3((unsigned)(nI * nJ)), dim3(GB_THREADS),
                           0, st, a, (int64_t)K, b, (int64_t)K, M, N, K, K, K, out, (int64_t)N, const_cast<float*>(consts),
                           dz, (int64_t)k, arg);
    }
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_gemm_h1bwd_rows(int M) { return M < 1 ? DGX_EINVAL : (M + G2_BM - 1) / G2_BM; }

int dgx_gemm_h1bwd_bf16(const void* dZ2, const void* W2t, int M, int N, int K, const float* PQ, int ldpq,
                        const int32_t* idx, int Np, int k, const float* scale, const float* shift, const float* mean,
                        const float* invstd, float slope, void* g, float* partials, int nrows, void* stream) {
    if (!dZ2 || !W2t || !PQ || !idx || !scale || !shift || !mean || !invstd || !g || !partials) return DGX_EINVAL;
    if (M < 1 || N < 1 || K < 1 || Np < 1 || k < 1 || M % k || ldpq < 2 * N) return DGX_EINVAL;
    if (nrows != (M + G2_BM - 1) / G2_BM) return DGX_EINVAL;
    if (N != 64 || K % G2_BK || ldpq % 4 || !aligned_to(dZ2, 16) || !aligned_to(W2t, 16) || !aligned_to(PQ, 16) ||
        !aligned_to(g, 16) || !aligned_to(scale, 16) || !aligned_to(shift, 16) || !aligned_to(mean, 16) ||
        !aligned_to(invstd, 16))
        return DGX_EUNSUPPORTED;
    EpiEdge ex{PQ, ldpq, idx, Np, k, scale, shift, mean, invstd, slope};
    const int nI = (M + G2_BM - 1) / G2_BM;
    hipLaunchKernelGGL((gemm_lds_kernel<false, G2_BM, 64, EPI_H1BWD>), dim3((unsigned)nI), dim3(GB_THREADS), 0,
                       dgx_stream(stream), static_cast<const bf16*>(dZ2), (int64_t)K, static_cast<const bf16*>(W2t),
                       (int64_t)K, M, N, K, K, K, static_cast<float*>(g), (int64_t)N, partials, nullptr, (int64_t)0,
                       nullptr, ex);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

// BM of the EPI_EDZ launch: 64-row tiles when 128-row ones would leave fewer
// than 512 workgroups (launch_gemm_lds's skinny rule)
inline int edz_bm(int M, int N) {
    const int bn = N > 64 ? 128 : 64;
    return (int64_t)((M + G2_BM - 1) / G2_BM) * ((N + bn - 1) / bn) < 512 ? 64 : G2_BM;
}

int dgx_gemm_edge_dz_rows(int M, int N) {
    if (M < 1 || N < 1) return DGX_EINVAL;
    return (M + edz_bm(M, N) - 1) / edz_bm(M, N);
}

int dgx_gemm_edge_dz_bf16(const void* A, int64_t lda, const void* W, int64_t ldw, int M, int N, int K,
                          const float* addend, int64_t ldd, const float* ysel, const uint8_t* arg, const float* scale,
                          const float* shift, const float* mean, const float* invstd, float slope, float* dz,
                          float* partials, int nrows, void* stream) {
    if (!A || !W || !addend || !ysel || !arg || !scale || !shift || !mean || !invstd || !dz || !partials)
        return DGX_EINVAL;
    if (M < 1 || N < 1 || K < 1 || nrows != dgx_gemm_edge_dz_rows(M, N)) return DGX_EINVAL;
    if (N % 8 || N > 128 || K % G2_BK || ldd % 4 || !aligned_to(A, 16) || !aligned_to(W, 16) || lda % 8 ||
        ldw % 8 || !aligned_to(addend, 16) || !aligned_to(ysel, 16) || !aligned_to(arg, 4) || !aligned_to(dz, 16) ||
        !aligned_to(scale, 16) || !aligned_to(shift, 16) || !aligned_to(mean, 16) || !aligned_to(invstd, 16))
        return DGX_EUNSUPPORTED;
    EpiEdge ex{};
    ex.PQ = ysel;
    ex.ldpq = N;
    ex.scale = scale;
    ex.shift = shift;
    ex.mean = mean;
    ex.invstd = invstd;
    ex.slope = slope;
    const bf16* a = static_cast<const bf16*>(A);
    const bf16* b = static_cast<const bf16*>(W);
    hipStream_t st = dgx_stream(stream);
    const int bm = edz_bm(M, N);
    const int nI = (M + bm - 1) / bm;
#define DGX_EDZ(BMV, BNV)                                                                                        \
    hipLaunchKernelGGL((gemm_lds_kernel<false, BMV, BNV, EPI_EDZ>), dim3((unsigned)(nI * ((N + BNV - 1) / BNV))), \
                       dim3(GB_THREADS), 0, st, a, lda, b, ldw, M, N, K, K, K, dz, (int64_t)N, partials, addend, ldd, \
                       arg, ex)
    if (N > 64) {
        if (bm == 64) DGX_EDZ(64, 128);
        else DGX_EDZ(G2_BM, 128);
    } else {
        if (bm == 64) DGX_EDZ(64, 64);
        else DGX_EDZ(G2_BM, 64);
    }
#undef DGX_EDZ
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_gemm_lds_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, int tn, int M, int N, int K,
                      int a_k, int epi, int splits, float* C, int64_t ldc, float* partials, const float* addend,
                      int64_t ldd, void* stream) {
    if (!A || !B || !C || M < 0 || N < 0 || K < 0 || splits < 1) return DGX_EINVAL;
    if (a_k == 0) a_k = K;
    if (a_k != K && (tn || a_k < G2_BK || a_k % G2_BK || K % a_k)) return DGX_EUNSUPPORTED;
    if ((epi == EPI_STATS || epi == EPI_STATS16) && !partials) return DGX_EINVAL;
    if (M == 0 || N == 0) return DGX_OK;
    // DMA staging moves 16-B chunks: rows 16-B aligned, whole chunks per row
    if (!aligned_to(A, 16) || !aligned_to(B, 16) || lda % 8 || ldb % 8) return DGX_EUNSUPPORTED;
    if (tn ? (M < 8 || N < 8 || M % 8 || N % 8 || epi != EPI_SLAB) : (K % G2_BK || epi == EPI_SLAB))
        return DGX_EUNSUPPORTED;
    if (epi == EPI_SLAB) ldc = N;
    hipStream_t st = dgx_stream(stream);
    const bf16* a = static_cast<const bf16*>(A);
    const bf16* b = static_cast<const bf16*>(B);
    const bool wide = N > 64;
    if (tn)
        return wide ? launch_gemm_lds<true, 128, EPI_SLAB>(a, lda, b, ldb, M, N, K, K, splits, C, ldc, partials,
                                                           nullptr, 0, st)
                    : launch_gemm_lds<true, 64, EPI_SLAB>(a, lda, b, ldb, M, N, K, K, splits, C, ldc, partials, nullptr,
                                                          0, st);
    // large NT GEMMs (conv5 forward and input gradient): 256 x 256 tiles when
    // they fill the chip (>= 256 tiles) and every tile is whole along N and K
    const bool big = (int64_t)((M + G3_BM - 1) / G3_BM) * ((N + G3_BN - 1) / G3_BN) >= 256 && N % G3_BN == 0 &&
                     K % G3_BK == 0 && a_k % G3_BK == 0;
    if (big) {
        if (epi == EPI_STORE) return launch_gemm256<EPI_STORE>(a, lda, b, ldb, M, N, K, a_k, C, ldc, partials, addend,
                                                              ldd, st);
        if (epi == EPI_ACCUM) return launch_gemm256<EPI_ACCUM>(a, lda, b, ldb, M, N, K, a_k, C, ldc, partials, addend,
                                                              ldd, st);
        if (epi == EPI_STATS) return launch_gemm256<EPI_STATS>(a, lda, b, ldb, M, N, K, a_k, C, ldc, partials, addend,
                                                              ldd, st);
        if (epi == EPI_STATS16)
            return launch_gemm256<EPI_STATS16>(a, lda, b, ldb, M, N, K, a_k, C, ldc, partials, addend, ldd, st);
    }
#define DGX_G2(E)                                                                                              \
    return wide ? launch_gemm_lds<false, 128, E>(a, lda, b, ldb, M, N, K, a_k, 1, C, ldc, partials, addend, ldd, \
                                                 st)                                                          \
                : launch_gemm_lds<false, 64, E>(a, lda, b, ldb, M, N, K, a_k, 1, C, ldc, partials, addend, ldd, st)
    if (epi == EPI_STORE) DGX_G2(EPI_STORE);
    if (epi == EPI_ACCUM) DGX_G2(EPI_ACCUM);
    if (epi == EPI_STATS) DGX_G2(EPI_STATS);
    if (epi == EPI_STATS16) DGX_G2(EPI_STATS16);
#undef DGX_G2
    return DGX_EUNSUPPORTED;
}

int dgx_split_bf16(const float* src, int64_t lds, int64_t rows, int cols, void* hi, void* lo, int64_t ldo,
                   void* stream) {
    if (!src || !lo || rows < 0 || cols < 1 || lds < cols || ldo < cols) return DGX_EINVAL;
    if (cols % 4 || lds % 4 || ldo % 4 || !aligned_to(src, 16) || !aligned_to(lo, 8) || (hi && !aligned_to(hi, 8)))
        return DGX_EUNSUPPORTED;
    if (rows == 0) return DGX_OK;
    const int64_t n4 = rows * (cols / 4);
    const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 8192);
    hipLaunchKernelGGL(split_bf16_kernel, dim3(grid), dim3(256), 0, dgx_stream(stream), src, lds, rows, cols,
                       static_cast<bf16*>(hi), static_cast<bf16*>(lo), ldo);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_weight_prep_bf16(const float* W, int Co, int C, int stacked, void* nt, void* tn, void* stream) {
    if (!W || !nt || !tn || Co < 1 || C < 1) return DGX_EINVAL;
    const int rows = stacked ? 2 * Co : Co;
    const dim3 grid((unsigned)((C + WP_T - 1) / WP_T), (unsigned)((rows + WP_T - 1) / WP_T));
    hipLaunchKernelGGL(weight_prep_kernel, grid, dim3(256), 0, dgx_stream(stream), W, Co, C, stacked,
                       static_cast<bf16*>(nt), static_cast<bf16*>(tn));
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_weight_stack_multi_f32(int n, const float* const* W, const int* Co, const int* C, float* const* out,
                               void* stream) {
    if (n < 1 || n > WP_MAXJ_S || !W || !Co || !C || !out) return DGX_EINVAL;
    WeightStackJobs jobs;
    jobs.n = n;
    int blocks = 0;
    for (int j = 0; j < n; ++j) {
        if (!W[j] || !out[j] || Co[j] < 1 || C[j] < 1) return DGX_EINVAL;
        jobs.W[j] = W[j];
        jobs.out[j] = out[j];
        jobs.Co[j] = Co[j];
        jobs.C[j] = C[j];
        jobs.first[j] = blocks;
        blocks += (int)(((int64_t)2 * Co[j] * C[j] + 255) / 256);
    }
    jobs.first[n] = blocks;
    hipLaunchKernelGGL(weight_stack_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, dgx_stream(stream), jobs);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_weight_prep_multi_bf16(int n, const float* const* W, const int* Co, const int* C, const int* stacked,
                               void* const* nt, void* const* tn, void* stream) {
    if (n < 1 || n > WP_MAXJ || !W || !Co || !C || !stacked || !nt || !tn) return DGX_EINVAL;
    WeightPrepJobs jobs = {};
    jobs.n = n;
    int blocks = 0;
    for (int j = 0; j < n; ++j) {
        if (!W[j] || !nt[j] || !tn[j] || Co[j] < 1 || C[j] < 1) return DGX_EINVAL;
        jobs.W[j] = W[j];
        jobs.nt[j] = static_cast<bf16*>(nt[j]);
        jobs.tn[j] = static_cast<bf16*>(tn[j]);
        jobs.Co[j] = Co[j];
        jobs.C[j] = C[j];
        jobs.stacked[j] = stacked[j];
        jobs.first[j] = blocks;
        const int rows = (stacked[j] & 1) ? 2 * Co[j] : Co[j];
        blocks += ((rows + WP_T - 1) / WP_T) * ((C[j] + WP_T - 1) / WP_T);
    }
    jobs.first[n] = blocks;
    hipLaunchKernelGGL(weight_prep_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, dgx_stream(stream), jobs);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_slab_reduce_multi_f32(int n, const float* const* slab, const int* S, const int* rows, const int* cols,
                              const int* split, float* const* out, const int64_t* ldo, void* stream) {
    if (n < 1 || n > SRM_MAXJ || !slab || !S || !rows || !cols || !split || !out || !ldo) return DGX_EINVAL;
    SlabJobs jobs;
    jobs.n = n;
    int blocks = 0;
    for (int j = 0; j < n; ++j) {
        if (!slab[j] || !out[j] || S[j] < 1 || rows[j] < 0 || cols[j] < 0 || split[j] < 0 || split[j] > rows[j])
            return DGX_EINVAL;
        jobs.slab[j] = slab[j];
        jobs.out[j] = out[j];
        jobs.ldo[j] = ldo[j];
        jobs.S[j] = S[j];
        jobs.rows[j] = rows[j];
        jobs.cols[j] = cols[j];
        jobs.split[j] = split[j];
        // 4 consecutive elements per lane: whole 4-groups in one row, 16-byte slab loads
        jobs.vec4[j] = cols[j] % 4 == 0 && (reinterpret_cast<uintptr_t>(slab[j]) & 15) == 0;
        jobs.first[j] = blocks;
        const int64_t units = (int64_t)rows[j] * cols[j] / (jobs.vec4[j] ? 4 : 1);
        blocks += (int)((units + SR_E - 1) / SR_E);
    }
    jobs.first[n] = blocks;
    if (blocks == 0) return DGX_OK;
    hipLaunchKernelGGL(slab_reduce_multi_kernel, dim3((unsigned)blocks), dim3(SR_E * SR_G), 0, dgx_stream(stream),
                       jobs);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_slab_reduce_f32(const float* slab, int S, int rows, int cols, int split, float* out, int64_t ldo,
                        void* stream) {
    if (!slab || !out || S < 1 || rows < 0 || cols < 0 || split < 0 || split > rows) return DGX_EINVAL;
    const int64_t total = (int64_t)rows * cols;
    if (total == 0) return DGX_OK;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)((total + SR_E - 1) / SR_E)), dim3(SR_E * SR_G), 0,
                       dgx_stream(stream),
                       slab, S, rows, cols, split, out, ldo);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

}  // extern "C"
