// a1 — kNN for EdgeConv (replaces reference models/dgcnn.py:6-12).
//
// One fused pass per cloud, no N x N matrix in HBM:
//   * |x|^2 per point in the reference's exact fp32 summation order (sqnorm).
//   * Gram tiles on the f32 MFMA (v_mfma_f32_16x16x4_f32). Its result is
//     bit-for-bit the k-ordered fmaf chain (cdna_hip_programming.md §3), which
//     is exactly what MKL's sgemm does for the reference, so the
//     distances match the reference bit for bit.
//   * pd = fl(fl(2*dot - xx_j) - xx_i) (dgcnn.py:7-9) and a per-row top-k kept
//     in registers, 4 lanes per query, merged through LDS at the end.
//
// Workgroup = 4 waves x 16 queries = 64 queries of one cloud. Candidates stream
// through a double-buffered LDS chunk of 64 points laid out [j/16][c][j%16] so
// the MFMA A operand read (lane l -> c = 4t + l/16, j = l%16) is a contiguous,
// conflict-free 256 B per wave.
#include <math.h>

#include "common.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifdef DGX_KNN_DEBUG
__device__ float* dgx_knn_dbg;
extern "C" int dgx_knn_set_debug(float* p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(dgx_knn_dbg), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif

namespace {

constexpr int KQ_WAVES = 4;
constexpr int KQ_QPW = 16;                    // queries per wave
constexpr int KQ_QPB = KQ_WAVES * KQ_QPW;     // queries per block
constexpr int KQ_JC = 64;                     // candidates per LDS chunk
constexpr int KQ_QCAP = 16;                   // per-lane pending-candidate FIFO

// ---------------------------------------------------------------- sqnorm ----
// |x_i|^2 with the rounding sequence of torch 2.10's CPU sum kernel, which the
// reference's `torch.sum(x**2, dim=1)` runs (dgcnn.py:8). Two building blocks
// (aten SumKernel.cpp): a 4-level cascade with 16-element level-0 runs, and a
// 4-way interleaved row sum of cascades. Layout decides which applies; see
// oracle/knn_oracle.c for the statement pinned against the reference.
// Each thread owns one point; C <= 128 here, so at most 2 cascade runs.
__device__ __forceinline__ float cascade16(const float* e, int stride, int m) {
#pragma clang fp contract(off)
    float a0 = 0.f, a1 = 0.f;  // level 0 / level 1 (m <= 256 never reaches level 2)
    int i = 0;
    for (; i + 16 <= m; i += 16) {
        float run = a0;
        for (int j = 0; j < 16; ++j) run = run + e[(i + j) * stride];
        a1 = a1 + run;
        a0 = 0.f;
    }
    for (; i < m; ++i) a0 = a0 + e[i * stride];
    return a0 + a1;  // acc[0] += acc[1] (+ acc[2] + acc[3], both 0)
}

__device__ __forceinline__ float rowsum4(const float* e, int stride, int n) {
#pragma clang fp contract(off)
    const int si = n >> 2;
    float l0 = si > 0 ? cascade16(e + 0 * stride, 4 * stride, si) : 0.f;
    float l1 = si > 0 ? cascade16(e + 1 * stride, 4 * stride, si) : 0.f;
    float l2 = si > 0 ? cascade16(e + 2 * stride, 4 * stride, si) : 0.f;
    float l3 = si > 0 ? cascade16(e + 3 * stride, 4 * stride, si) : 0.f;
    for (int i = 4 * si; i < n; ++i) l0 = l0 + e[i * stride];
    return ((l0 + l1) + l2) + l3;
}

__device__ __forceinline__ float sqnorm_point(const float* __restrict__ p, int64_t sC, int C, int order,
                                              bool tail) {
#pragma clang fp contract(off)
    float sq[128];
    for (int c = 0; c < C; ++c) {
        float v = p[c * sC];
        sq[c] = v * v;
    }
    if (order == DGX_ORDER_VEC8X4) {
        if (C < 8) return rowsum4(sq, 1, C);
        const int vs = C >> 3;
        float fin = 0.f;
        for (int c = 8 * vs; c < C; ++c) fin = fin + sq[c];
        for (int l = 0; l < 8; ++l) fin = fin + rowsum4(sq + l, 8, vs);
        return fin;
    }
    return tail ? rowsum4(sq, 1, C) : cascade16(sq, 1, C);
}

__global__ __launch_bounds__(256) void sqnorm_kernel(const float* __restrict__ x, int64_t sB, int64_t sC,
                                                    int64_t sN, int B, int C, int N, int order,
                                                    float* __restrict__ xx) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)B * N) return;
    int b = (int)(t / N), n = (int)(t - (int64_t)b * N);
    xx[t] = sqnorm_point(x + b * sB + n * sN, sC, C, order, n >= (N & ~31));
}

// ------------------------------------------------------------- top-k list ----
// Sorted (desc) list in registers, static indexing only. Candidates reach a
// lane in ascending index order, so a strict '>' keeps earlier (smaller) indices
// ahead of equal values: canonical tie order for free.
template <int KMAX>
__device__ __forceinline__ void list_insert_ordered(float (&v)[KMAX], int (&id)[KMAX], float nv, int nj) {
    // Shift insert from the tail: slot q takes slot q-1 if the new value beats
    // v[q-1], else the new value if it beats v[q], else keeps its own. Every
    // compare uses the NEW value against the original list, so elements of
    // equal value keep their relative order (a carried-element bubble would
    // swap equal neighbours). One lane mask live per step.
    bool gt_cur = nv > v[KMAX - 1];
#pragma unroll
    for (int q = KMAX - 1; q > 0; --q) {
        const bool gt_prev = nv > v[q - 1];
        v[q] = gt_prev ? v[q - 1] : (gt_cur ? nv : v[q]);
        id[q] = gt_prev ? id[q - 1] : (gt_cur ? nj : id[q]);
        gt_cur = gt_prev;
    }
    v[0] = gt_cur ? nv : v[0];
    id[0] = gt_cur ? nj : id[0];
}

// Insert with the full canonical comparator (value desc, index asc): used when
// merging lists built from different candidate subsets.
template <int KMAX>
__device__ __forceinline__ void list_insert_canon(float (&v)[KMAX], int (&id)[KMAX], float nv, int nj) {
    float cv = nv;
    int cj = nj;
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
        bool s = cv > v[q] || (cv == v[q] && cj < id[q]);
        float tv = v[q];
        int tj = id[q];
        v[q] = s ? cv : tv;
        id[q] = s ? cj : tj;
        cv = s ? tv : cv;
        cj = s ? tj : cj;
    }
}

template <int NSTEP>
struct KnnSmem {
    static constexpr int CP = NSTEP * 4;
    static constexpr int CHUNK = KQ_JC * CP + KQ_JC;  // tile + xx
    static constexpr int MAIN = 2 * CHUNK + KQ_WAVES * 2 * KQ_QCAP * 64;
};

template <int NSTEP, int KMAX>
constexpr int knn_smem_floats() {
    // merge stage: per wave 2 slots x 16 lists x KMAX x (value, index)
    constexpr int merge = KQ_WAVES * 2 * KQ_QPW * KMAX * 2;
    return KnnSmem<NSTEP>::MAIN > merge ? KnnSmem<NSTEP>::MAIN : merge;
}

// ------------------------------------------------------------ knn kernel ----
template <int NSTEP, int KMAX, bool CMAJOR>
__global__ __launch_bounds__(256, 2) void knn_kernel(const float* __restrict__ x, int64_t sB, int64_t sC,
                                                    int64_t sN, const float* __restrict__ xx, int B, int C,
                                                    int N, int k, int nqb, int64_t* __restrict__ idx64,
                                                    int32_t* __restrict__ idx32, float* __restrict__ vals) {
#pragma clang fp contract(off)
    constexpr int CP = NSTEP * 4;
    constexpr int CHUNK = KnnSmem<NSTEP>::CHUNK;
    __shared__ float smem[knn_smem_floats<NSTEP, KMAX>()];

    int b, qb;
    if (!dgx_xcd_cloud_map(blockIdx.x, B, nqb, b, qb)) return;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int g = lane >> 4;     // which quarter of the candidates this lane sees
    const int ql = lane & 15;
    const int q = qb * KQ_QPB + wave * KQ_QPW + ql;
    const float* __restrict__ xb = x + b * sB;
    const float* __restrict__ xxb = xx + (int64_t)b * N;

    // B operand (queries) stays in registers: lane holds x[q][4t + g].
    float bq[NSTEP];
#pragma unroll
    for (int t = 0; t < NSTEP; ++t) {
        int c = 4 * t + g;
        bq[t] = (q < N && c < C) ? xb[c * sC + q * sN] : 0.f;
    }
    const float xxq = q < N ? xxb[q] : 0.f;

    auto load_chunk = [&](int buf, int j0) {
        float* dst = smem + buf * CHUNK;
        for (int e = tid; e < KQ_JC * CP; e += 256) {
            int jj, c;
            if (CMAJOR) { jj = e % KQ_JC; c = e / KQ_JC; }
            else { c = e % CP; jj = e / CP; }
            int j = j0 + jj;
            float v = (c < C && j < N) ? xb[c * sC + j * sN] : 0.f;
            dst[(jj >> 4) * (CP * 16) + c * 16 + (jj & 15)] = v;
        }
        if (tid < KQ_JC) {
            int j = j0 + tid;
            dst[KQ_JC * CP + tid] = j < N ? xxb[j] : 0.f;
        }
    };

    // List of KMAX slots; the first KMAX-k hold +inf sentinels that nothing can
    // displace, so the live top-k always sits in slots [KMAX-k, KMAX) and the
    // lane's own admission value is simply the last slot (no dynamic indexing).
    const int kpad = KMAX - k;
    float lv[KMAX];
    int li[KMAX];
#pragma unroll
    for (int t = 0; t < KMAX; ++t) { lv[t] = t < kpad ? INFINITY : -INFINITY; li[t] = 0x7fffffff; }

    // Candidates that pass the filter wait in a per-lane FIFO in LDS and are
    // inserted in batches, so an insertion round (5*KMAX VALU ops for the
    // whole wave) is paid once per admitted candidate of the busiest lane,
    // not once per candidate. The filter is the max of the 4 lanes' k-th
    // values of this query (each is a lower bound of the row's final k-th);
    // '>=' keeps equal values, whose order is settled canonically at the merge.
    float* qv = smem + 2 * CHUNK + wave * (2 * KQ_QCAP * 64);
    int* qj = reinterpret_cast<int*>(qv + KQ_QCAP * 64);
    int cnt = 0;
    float thr = -INFINITY;
    auto flush = [&]() {
#pragma unroll 1
        for (int t = 0; __any(t < cnt); ++t) {
            float v = -INFINITY;
            int j = 0x7fffffff;
            if (t < cnt) { v = qv[t * 64 + lane]; j = qj[t * 64 + lane]; }
            list_insert_ordered<KMAX>(lv, li, v >= thr ? v : -INFINITY, j);
        }
        cnt = 0;
        float kth = lv[KMAX - 1];
        kth = fmaxf(kth, __shfl_xor(kth, 16));
        kth = fmaxf(kth, __shfl_xor(kth, 32));
        thr = kth;
    };

    const int nch = (N + KQ_JC - 1) / KQ_JC;
    load_chunk(0, 0);
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
        const int cur = ch & 1;
        if (ch + 1 < nch) load_chunk(cur ^ 1, (ch + 1) * KQ_JC);
        const float* __restrict__ tile = smem + cur * CHUNK;
#pragma unroll 1
        for (int s = 0; s < KQ_JC / 16; ++s) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            const float* __restrict__ ts = tile + s * (CP * 16);
#pragma unroll
            for (int t = 0; t < NSTEP; ++t)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ts[t * 64 + lane], bq[t], acc, 0, 0, 0);
            // lane holds candidates j = jb + r (r = 0..3) of query q
            const int jb = ch * KQ_JC + s * 16 + 4 * g;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float xc = tile[KQ_JC * CP + s * 16 + 4 * g + r];
                float two_dot = 2.0f * acc[r];
                float tq = two_dot - xc;
                float v = tq - xxq;
                bool pass = (jb + r < N) && v >= thr && v > -INFINITY;
                if (pass) { qv[cnt * 64 + lane] = v; qj[cnt * 64 + lane] = jb + r; }
                cnt += pass ? 1 : 0;
            }
            if (__any(cnt > KQ_QCAP - 4)) flush();
        }
        __syncthreads();
    }
    flush();
    __syncthreads();

#ifdef DGX_KNN_DEBUG
    if (q < N && dgx_knn_dbg) {
        float* d = dgx_knn_dbg + (((int64_t)b * N + q) * 4 + g) * KMAX * 2;
        for (int t = 0; t < KMAX; ++t) { d[t] = lv[t]; d[KMAX + t] = (float)li[t]; }
    }
#endif
    // Merge the 4 partial lists of each query (lanes ql, ql+16, ql+32, ql+48):
    // g1 -> g0 and g3 -> g2, then g2 -> g0. Scratch per wave: 2 slots x 16
    // lists, element-major ([t][list]) so a wave's accesses are conflict-free.
    float* mv = smem + wave * (2 * KQ_QPW * KMAX * 2);
    int* mi = reinterpret_cast<int*>(mv + 2 * KQ_QPW * KMAX);
    constexpr int NL = 2 * KQ_QPW;
    if (g & 1) {
        const int L = (g >> 1) * KQ_QPW + ql;
#pragma unroll
        for (int t = 0; t < KMAX; ++t) { mv[t * NL + L] = lv[t]; mi[t * NL + L] = li[t]; }
    }
    __syncthreads();
    if (!(g & 1)) {
        const int L = (g >> 1) * KQ_QPW + ql;
#pragma unroll 1
        for (int t = kpad; t < KMAX; ++t) list_insert_canon<KMAX>(lv, li, mv[t * NL + L], mi[t * NL + L]);
    }
    __syncthreads();
    if (g == 2) {
#pragma unroll
        for (int t = 0; t < KMAX; ++t) { mv[t * NL + ql] = lv[t]; mi[t * NL + ql] = li[t]; }
    }
    __syncthreads();
    if (g == 0) {
#pragma unroll 1
        for (int t = kpad; t < KMAX; ++t) list_insert_canon<KMAX>(lv, li, mv[t * NL + ql], mi[t * NL + ql]);
        if (q < N) {
            const int64_t row = ((int64_t)b * N + q) * k - kpad;
#pragma unroll
            for (int t = 0; t < KMAX; ++t) {
                if (t >= kpad) {
                    if (idx64) idx64[row + t] = li[t];
                    if (idx32) idx32[row + t] = li[t];
                    if (vals) vals[row + t] = lv[t];
                }
            }
        }
    }
}

template <int NSTEP, int KMAX>
int launch_knn(const float* x, int64_t sB, int64_t sC, int64_t sN, const float* xx, int B, int C, int N,
               int k, int64_t* idx64, int32_t* idx32, float* vals, hipStream_t st) {
    const int nqb = (N + KQ_QPB - 1) / KQ_QPB;
    dim3 grid(dgx_xcd_cloud_grid(B, nqb)), block(256);
    if (sN == 1)
        hipLaunchKernelGGL((knn_kernel<NSTEP, KMAX, true>), grid, block, 0, st, x, sB, sC, sN, xx, B, C, N, k,
                           nqb, idx64, idx32, vals);
    else
        hipLaunchKernelGGL((knn_kernel<NSTEP, KMAX, false>), grid, block, 0, st, x, sB, sC, sN, xx, B, C, N, k,
                           nqb, idx64, idx32, vals);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

template <int NSTEP>
int dispatch_k(const float* x, int64_t sB, int64_t sC, int64_t sN, const float* xx, int B, int C, int N, int k,
               int64_t* idx64, int32_t* idx32, float* vals, hipStream_t st) {
    if (k <= 16) return launch_knn<NSTEP, 16>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
    if (k <= 20) return launch_knn<NSTEP, 20>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
    if (k <= 32) return launch_knn<NSTEP, 32>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
    if (k <= 40) return launch_knn<NSTEP, 40>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
    return launch_knn<NSTEP, 64>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
}

}  // namespace

extern "C" {

int dgx_sqnorm_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int C, int N, int order, float* xx,
                   void* stream) {
    if (!x || !xx || B < 0 || C < 1 || N < 0) return DGX_EINVAL;
    int64_t total = (int64_t)B * N;
    if (total == 0) return DGX_OK;
    int grid = (int)((total + 255) / 256);
    hipLaunchKernelGGL(sqnorm_kernel, dim3(grid), dim3(256), 0, dgx_stream(stream), x, sB, sC, sN, B, C, N, order,
                       xx);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

size_t dgx_knn_workspace_bytes(int B, int N) { return (size_t)B * (size_t)N * sizeof(float); }

int dgx_knn_select_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, const float* xx, int B, int C, int N,
                       int k, int64_t* idx64, int32_t* idx32, float* vals, void* stream) {
    if (!x || !xx || B < 0 || C < 1 || N < 1 || k < 1 || k > N) return DGX_EINVAL;
    if (!idx64 && !idx32) return DGX_EINVAL;
    if (C > 128 || k > 64) return DGX_EUNSUPPORTED;
    if (B == 0) return DGX_OK;
    hipStream_t st = dgx_stream(stream);
    if (C <= 4) return dispatch_k<1>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
    if (C <= 12) return dispatch_k<3>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
    if (C <= 32) return dispatch_k<8>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
    if (C <= 64) return dispatch_k<16>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
    return dispatch_k<32>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, st);
}

int dgx_knn_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int C, int N, int k, int order,
                int64_t* idx64, int32_t* idx32, void* workspace, size_t workspace_bytes, void* stream) {
    if (!x || B < 0 || C < 1 || N < 1 || k < 1 || k > N) return DGX_EINVAL;
    if (!idx64 && !idx32) return DGX_EINVAL;
    if (C > 128 || k > 64) return DGX_EUNSUPPORTED;
    if (workspace_bytes < dgx_knn_workspace_bytes(B, N) || !workspace) return DGX_EINVAL;
    if (B == 0) return DGX_OK;
    float* xx = static_cast<float*>(workspace);
    int rc = dgx_sqnorm_f32(x, sB, sC, sN, B, C, N, order, xx, stream);
    if (rc != DGX_OK) return rc;
    return dgx_knn_select_f32(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, nullptr, stream);
}

}  // extern "C"
