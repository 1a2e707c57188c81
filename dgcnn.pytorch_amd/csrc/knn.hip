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
// through an LDS chunk laid out [j/16][c][j%16] (padded, see knn_tile_stride)
// so the MFMA A operand read (lane l -> c = 4t + l/16, j = l%16) and the chunk
// stores are bank-conflict-free.
#include <math.h>
#include <stdlib.h>

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

// Squares staged in LDS ([c][thread], conflict-free) instead of a private
// array (which would live in scratch memory).
constexpr int SQ_THREADS = 64;

__device__ __forceinline__ float sqnorm_point(const float* __restrict__ p, int64_t sC, int C, int order,
                                              bool tail, float* sq) {
#pragma clang fp contract(off)
    for (int c0 = 0; c0 < C; c0 += 16) {  // 16 loads in flight per thread
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = c0 + u < C ? p[(c0 + u) * sC] : 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (c0 + u < C) sq[(c0 + u) * SQ_THREADS] = v[u] * v[u];
    }
    if (order == DGX_ORDER_VEC8X4) {
        if (C < 8) return rowsum4(sq, SQ_THREADS, C);
        const int vs = C >> 3;
        float fin = 0.f;
        for (int c = 8 * vs; c < C; ++c) fin = fin + sq[c * SQ_THREADS];
        for (int l = 0; l < 8; ++l) fin = fin + rowsum4(sq + l * SQ_THREADS, 8 * SQ_THREADS, vs);
        return fin;
    }
    return tail ? rowsum4(sq, SQ_THREADS, C) : cascade16(sq, SQ_THREADS, C);
}

__global__ __launch_bounds__(SQ_THREADS) void sqnorm_kernel(const float* __restrict__ x, int64_t sB, int64_t sC,
                                                            int64_t sN, int B, int C, int N, int order,
                                                            float* __restrict__ xx) {
    __shared__ float sq[128 * SQ_THREADS];
    int64_t t = (int64_t)blockIdx.x * SQ_THREADS + threadIdx.x;
    if (t >= (int64_t)B * N) return;
    int b = (int)(t / N), n = (int)(t - (int64_t)b * N);
    xx[t] = sqnorm_point(x + b * sB + n * sN, sC, C, order, n >= (N & ~31), sq + threadIdx.x);
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

// Candidate chunk per LDS fill: JC candidates x CP channels, <= 16 KB, a
// multiple of 32 candidates (tiles are processed in pairs), and JC*CP a
// multiple of the 256 threads so each thread prefetches exactly PF floats of
// the next chunk into registers.
template <int CP>
struct KnnGeom {
    static constexpr int JC = CP <= 4 ? 1024 : (CP <= 12 ? 320 : (CP <= 32 ? 128 : (CP <= 64 ? 64 : 32)));
    static constexpr int PF = JC * CP / 256;
    static constexpr int XPF = (JC + 255) / 256;
};

// Per-lane list length for k <= KB: a quarter of k plus a margin. Each lane
// sees a quarter of the candidates; the true top-k splits ~Binomial(k, 1/4)
// over the 4 lanes, so a lane needing more than KL slots is rare. When it
// happens the row is flagged and recomputed exactly (knn_fix_kernel).
template <int KB>
struct KnnList {
    // KL ~ k/4 + 5 standard deviations of Binomial(k, 1/4): a flagged row
    // (~1e-6 per row for random point order at k = 20) costs one fix-up.
    static constexpr int KL = KB <= 16 ? 13 : (KB <= 20 ? 16 : (KB <= 32 ? 20 : (KB <= 40 ? 24 : 34)));
    static constexpr int RPL = (KB + 3) / 4;   // output ranks per lane
};

// Candidate tile image: 16 candidates x CP channels per tile, channel rows of
// 17 floats (16 + 1 pad) and tiles KT_SKEW floats apart beyond CP*17: the
// channel-fastest stores of a point-major chunk and the candidate-fastest
// stores of a channel-major one both hit 64 distinct banks, and the MFMA
// A-operand read (lane -> channel 4t + lane/16, candidate lane%16) is
// conflict-free (odd row stride).
constexpr int KT_ROW = 17;
constexpr int KT_SKEW = 16;
template <int CP>
constexpr int knn_tile_stride() { return CP * KT_ROW + KT_SKEW; }

template <int NSTEP>
constexpr int knn_smem_floats() {
    constexpr int CP = NSTEP * 4;
    constexpr int JC = KnnGeom<CP>::JC;
    return (JC / 16) * knn_tile_stride<CP>() + JC + KQ_WAVES * 2 * KQ_QCAP * 64;  // tile | xx | per-wave FIFOs
}

// Canonical order: value descending, then index ascending.
__device__ __forceinline__ bool canon_better(float av, int aj, float bv, int bj) {
    return av > bv || (av == bv && aj < bj);
}

// ------------------------------------------------------------ knn kernel ----
template <int NSTEP, int KB, bool CMAJOR>
__global__ __launch_bounds__(256, 2) void knn_kernel(const float* __restrict__ x, int64_t sB, int64_t sC,
                                                    int64_t sN, const float* __restrict__ xx, int B, int C,
                                                    int N, int k, int nqb, int64_t* __restrict__ idx64,
                                                    int32_t* __restrict__ idx32, float* __restrict__ vals) {
#pragma clang fp contract(off)
    constexpr int CP = NSTEP * 4;
    constexpr int JC = KnnGeom<CP>::JC;
    constexpr int PF = KnnGeom<CP>::PF;
    constexpr int XPF = KnnGeom<CP>::XPF;
    constexpr int KL = KnnList<KB>::KL;
    constexpr int RPL = KnnList<KB>::RPL;
    __shared__ __attribute__((aligned(16))) float smem[knn_smem_floats<NSTEP>()];
    float* tile = smem;                 // [JC/16][CP][16]
    constexpr int TS = knn_tile_stride<CP>();
    float* xxs = smem + (JC / 16) * TS;  // [JC]
    float* qbase = xxs + JC;            // per wave: [KQ_QCAP][64] float2 (value, index)

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

    // Next-chunk prefetch in registers: issued before the current chunk's
    // compute, written to LDS after it (load latency hidden by the MFMAs).
    float pf[PF], pfx[XPF];
    auto load_regs = [&](int j0) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int e = tid + u * 256;
            int jj, c;
            if (CMAJOR) { jj = e % JC; c = e / JC; }
            else { c = e % CP; jj = e / CP; }
            const int j = j0 + jj;
            pf[u] = (c < C && j < N) ? xb[c * sC + j * sN] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < XPF; ++u) {
            const int jj = tid + u * 256;
            pfx[u] = (jj < JC && j0 + jj < N) ? xxb[j0 + jj] : 0.f;
        }
    };
    auto store_regs = [&]() {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int e = tid + u * 256;
            int jj, c;
            if (CMAJOR) { jj = e % JC; c = e / JC; }
            else { c = e % CP; jj = e / CP; }
            tile[(jj >> 4) * TS + c * KT_ROW + (jj & 15)] = pf[u];
        }
#pragma unroll
        for (int u = 0; u < XPF; ++u) {
            const int jj = tid + u * 256;
            if (jj < JC) xxs[jj] = pfx[u];
        }
    };

    // Each lane keeps the KL best of ITS candidates (sorted, registers, static
    // indexing). Admission filter thr = max(own KL-th, T) where T = min over
    // the query's 4 lanes of their m-th value, m = ceil(k/4): 4 lanes x m
    // candidates >= T exist, so T never exceeds the row's final k-th value.
    // '>=' keeps equal values; their order is settled canonically at the merge.
    const int m = (k + 3) >> 2;
    float lv[KL];
    int li[KL];
#pragma unroll
    for (int t = 0; t < KL; ++t) { lv[t] = -INFINITY; li[t] = 0x7fffffff; }

    // Candidates that pass the filter wait in a per-lane FIFO in LDS and are
    // inserted in batches, so an insertion round (5*KL VALU ops for the whole
    // wave) is paid once per admitted candidate of the busiest lane.
    float2* fifo = reinterpret_cast<float2*>(qbase) + wave * (KQ_QCAP * 64);
    int cnt = 0;
    float thr = -INFINITY;
    auto flush = [&]() {
        float2 cur = cnt > 0 ? fifo[lane] : make_float2(-INFINITY, __int_as_float(0x7fffffff));
#pragma unroll 1
        for (int t = 0; __any(t < cnt); ++t) {
            const float2 nxt = (t + 1 < cnt) ? fifo[(t + 1) * 64 + lane]
                                             : make_float2(-INFINITY, __int_as_float(0x7fffffff));
            list_insert_ordered<KL>(lv, li, cur.x >= thr ? cur.x : -INFINITY, __float_as_int(cur.y));
            cur = nxt;
        }
        cnt = 0;
        float tm = lv[0];
#pragma unroll
        for (int t = 1; t < KL; ++t) tm = (t == m - 1) ? lv[t] : tm;
        tm = fminf(tm, __shfl_xor(tm, 16));
        tm = fminf(tm, __shfl_xor(tm, 32));
        thr = fmaxf(tm, lv[KL - 1]);
    };

    auto consider = [&](float dot, float xc, int j, bool valid) {
        float two_dot = 2.0f * dot;
        float tq = two_dot - xc;
        float v = tq - xxq;
        const bool pass = valid && v >= thr;
        if (pass) fifo[cnt * 64 + lane] = make_float2(v, __int_as_float(j));
        cnt += pass ? 1 : 0;
    };

    const int nch = (N + JC - 1) / JC;
    load_regs(0);
    store_regs();
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
        if (ch + 1 < nch) load_regs((ch + 1) * JC);
        const int jend = min(JC, N - ch * JC);
        // tiles in pairs: two independent MFMA chains in flight
#pragma unroll 1
        for (int s = 0; s < (jend + 15) / 16; s += 2) {
            f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
            const float* __restrict__ ts = tile + s * TS + (lane >> 4) * KT_ROW + (lane & 15);
#pragma unroll
            for (int t = 0; t < NSTEP; ++t) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ts[t * 4 * KT_ROW], bq[t], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ts[TS + t * 4 * KT_ROW], bq[t], acc1, 0, 0, 0);
            }
            // lane holds candidates j = jb + r (r = 0..3) and jb + 16 + r of query q
            const int jl = s * 16 + 4 * g;
            const int jb = ch * JC + jl;
            const float4 xc0 = *reinterpret_cast<const float4*>(xxs + jl);
            const float4 xc1 = *reinterpret_cast<const float4*>(xxs + jl + 16);
            const int lim = N - jb;
            consider(acc0[0], xc0.x, jb + 0, 0 < lim);
            consider(acc0[1], xc0.y, jb + 1, 1 < lim);
            consider(acc0[2], xc0.z, jb + 2, 2 < lim);
            consider(acc0[3], xc0.w, jb + 3, 3 < lim);
            consider(acc1[0], xc1.x, jb + 16, 16 < lim);
            consider(acc1[1], xc1.y, jb + 17, 17 < lim);
            consider(acc1[2], xc1.z, jb + 18, 18 < lim);
            consider(acc1[3], xc1.w, jb + 19, 19 < lim);
            if (__any(cnt > KQ_QCAP - 8)) flush();
        }
        __syncthreads();
        if (ch + 1 < nch) {
            store_regs();
            __syncthreads();
        }
    }
    flush();

#ifdef DGX_KNN_DEBUG
    if (q < N && dgx_knn_dbg) {
        float* d = dgx_knn_dbg + (((int64_t)b * N + q) * 4 + g) * KL * 2;
        for (int t = 0; t < KL; ++t) { d[t] = lv[t]; d[KL + t] = (float)li[t]; }
    }
#endif
    // Merge the query's 4 lists (lanes ql, ql+16, ql+32, ql+48) by k rounds of
    // a canonical arg-max over the 4 list heads; the winning lane pops its
    // head. Rank r ends up in lane r % 4.
    const float last = lv[KL - 1];
    float ov[RPL];
    int oj[RPL];
    float hv = -INFINITY;
#pragma unroll
    for (int r = 0; r < KB; ++r) {
        if (r < k) {
            hv = lv[0];
            int hj = li[0];
            float pv = __shfl_xor(hv, 16);
            int pj = __shfl_xor(hj, 16);
            if (canon_better(pv, pj, hv, hj)) { hv = pv; hj = pj; }
            pv = __shfl_xor(hv, 32);
            pj = __shfl_xor(hj, 32);
            if (canon_better(pv, pj, hv, hj)) { hv = pv; hj = pj; }
            const bool pop = li[0] == hj && lv[0] == hv;
#pragma unroll
            for (int t = 0; t < KL - 1; ++t) {
                lv[t] = pop ? lv[t + 1] : lv[t];
                li[t] = pop ? li[t + 1] : li[t];
            }
            lv[KL - 1] = pop ? -INFINITY : lv[KL - 1];
            li[KL - 1] = pop ? 0x7fffffff : li[KL - 1];
            if ((r & 3) == g) { ov[r >> 2] = hv; oj[r >> 2] = hj; }
        }
    }
    // hv is now the merged k-th value. A lane whose list was full and whose
    // last kept value reaches it may have dropped a member of the true top-k:
    // mark the row for the exact fix-up pass.
    int flag = (last != -INFINITY && last >= hv) ? 1 : 0;
    flag |= __shfl_xor(flag, 16);
    flag |= __shfl_xor(flag, 32);
    if (q < N) {
        const int64_t row = ((int64_t)b * N + q) * k;
#pragma unroll
        for (int t = 0; t < RPL; ++t) {
            const int r = 4 * t + g;
            if (r < k) {
                // flagged: rank 0 = -1 marker, rank 1 = bits of the merged k-th
                // value (a lower bound of the true k-th) for the fix-up pass
                const int j = !flag ? oj[t] : (r == 0 ? -1 : (r == 1 ? __float_as_int(hv) : oj[t]));
                if (idx64) idx64[row + r] = j;
                if (idx32) idx32[row + r] = j;
                if (vals) vals[row + r] = ov[t];
            }
        }
    }
}

// Exact recompute of the rows knn_kernel flagged (rank 0 = -1, rank 1 = the
// bits of T0, the merged k-th value: at least k candidates reach T0). One block
// per 256 consecutive rows scans their markers; for each flagged row the block
// recomputes all N distances (the same k-ordered fmaf chain the MFMA performs,
// the same rounding sequence), collects the candidates >= T0 (normally k plus
// the few the overflowing list dropped) and ranks them canonically in one
// all-pairs pass. If more than FIX_CAP reach T0 (mass ties), wave 0 extracts
// the top-k from all N by k rounds of a canonical arg-max instead.
constexpr int FIX_MAXN = 12288;
constexpr int FIX_CB = 16;    // channels loaded per batch (loads in flight)
constexpr int FIX_CAP = 1024;

__global__ __launch_bounds__(256) void knn_fix_kernel(const float* __restrict__ x, int64_t sB, int64_t sC,
                                                      int64_t sN, const float* __restrict__ xx, int B, int C,
                                                      int N, int k, int64_t* __restrict__ idx64,
                                                      int32_t* __restrict__ idx32, float* __restrict__ vals) {
#pragma clang fp contract(off)
    __shared__ float pd[FIX_MAXN];
    __shared__ float cv[FIX_CAP];
    __shared__ int cj[FIX_CAP];
    __shared__ float xq[128];
    __shared__ int rows[256];
    __shared__ int nrows, ncand;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t total = (int64_t)B * N;
    const int64_t r0 = (int64_t)blockIdx.x * 256;
    if (tid == 0) nrows = 0;
    __syncthreads();
    if (r0 + tid < total) {
        const int64_t at = (r0 + tid) * k;
        const bool flagged = idx64 ? idx64[at] < 0 : idx32[at] < 0;
        if (flagged) rows[atomicAdd(&nrows, 1)] = tid;
    }
    __syncthreads();
    const int nr = nrows;
    for (int i = 0; i < nr; ++i) {
        const int64_t row = r0 + rows[i];
        const int b = (int)(row / N), q = (int)(row - (int64_t)b * N);
        const float* __restrict__ xb = x + b * sB;
        const float* __restrict__ xxb = xx + (int64_t)b * N;
        float t0 = -INFINITY;
        if (k > 1) t0 = __int_as_float(idx64 ? (int)idx64[row * k + 1] : idx32[row * k + 1]);
        if (tid < C) xq[tid] = xb[tid * sC + q * sN];
        if (tid == 0) ncand = 0;
        __syncthreads();
        const float xxq = xxb[q];
        auto keep = [&](int j, float v) {
            pd[j] = v;
            if (v >= t0) {
                const int s = atomicAdd(&ncand, 1);
                if (s < FIX_CAP) { cv[s] = v; cj[s] = j; }
            }
        };
        for (int j0 = tid; j0 < N; j0 += 512) {
            const int ja = j0, jb = j0 + 256;
            float da = 0.f, db = 0.f;
            for (int c0 = 0; c0 < C; c0 += FIX_CB) {
                float va[FIX_CB], vb[FIX_CB];
#pragma unroll
                for (int u = 0; u < FIX_CB; ++u) {
                    const int c = c0 + u;
                    va[u] = c < C ? xb[c * sC + ja * sN] : 0.f;
                    vb[u] = (c < C && jb < N) ? xb[c * sC + jb * sN] : 0.f;
                }
#pragma unroll
                for (int u = 0; u < FIX_CB; ++u) {
                    if (c0 + u < C) {
                        da = fmaf(va[u], xq[c0 + u], da);
                        db = fmaf(vb[u], xq[c0 + u], db);
                    }
                }
            }
            const float ta = 2.0f * da, tb = 2.0f * db;
            const float ua = ta - xxb[ja];
            keep(ja, ua - xxq);
            if (jb < N) {
                const float ub = tb - xxb[jb];
                keep(jb, ub - xxq);
            }
        }
        __syncthreads();
        const int n = ncand;
        if (n <= FIX_CAP) {
            for (int t = tid; t < n; t += 256) {
                const float v = cv[t];
                const int j = cj[t];
                int rank = 0;
                for (int u = 0; u < n; ++u) rank += canon_better(cv[u], cj[u], v, j) ? 1 : 0;
                if (rank < k) {
                    if (idx64) idx64[row * k + rank] = j;
                    if (idx32) idx32[row * k + rank] = j;
                    if (vals) vals[row * k + rank] = v;
                }
            }
        } else if (wave == 0) {
            for (int r = 0; r < k; ++r) {
                float bv = -INFINITY;
                int bj = 0x7fffffff;
                for (int j = lane; j < N; j += 64)
                    if (canon_better(pd[j], j, bv, bj)) { bv = pd[j]; bj = j; }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const float pv = __shfl_xor(bv, o);
                    const int pj = __shfl_xor(bj, o);
                    if (canon_better(pv, pj, bv, bj)) { bv = pv; bj = pj; }
                }
                if (lane == 0) {
                    pd[bj] = -INFINITY;  // taken: finite candidates always outrank it
                    if (idx64) idx64[row * k + r] = bj;
                    if (idx32) idx32[row * k + r] = bj;
                    if (vals) vals[row * k + r] = bv;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        __syncthreads();
    }
}

template <int NSTEP, int KB>
int launch_knn(const float* x, int64_t sB, int64_t sC, int64_t sN, const float* xx, int B, int C, int N,
               int k, int64_t* idx64, int32_t* idx32, float* vals, hipStream_t st) {
    const int nqb = (N + KQ_QPB - 1) / KQ_QPB;
    dim3 grid(dgx_xcd_cloud_grid(B, nqb)), block(256);
    if (sN == 1)
        hipLaunchKernelGGL((knn_kernel<NSTEP, KB, true>), grid, block, 0, st, x, sB, sC, sN, xx, B, C, N, k,
                           nqb, idx64, idx32, vals);
    else
        hipLaunchKernelGGL((knn_kernel<NSTEP, KB, false>), grid, block, 0, st, x, sB, sC, sN, xx, B, C, N, k,
                           nqb, idx64, idx32, vals);
    if (hipGetLastError() != hipSuccess) return DGX_ELAUNCH;
    static const bool nofix = getenv("DGX_KNN_NOFIX") != nullptr;  // diagnostics: leave flagged rows marked
    if (nofix) return DGX_OK;
    const int64_t rows = (int64_t)B * N;
    hipLaunchKernelGGL(knn_fix_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, x, sB, sC, sN, xx,
                       B, C, N, k, idx64, idx32, vals);
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
    int grid = (int)((total + SQ_THREADS - 1) / SQ_THREADS);
    hipLaunchKernelGGL(sqnorm_kernel, dim3(grid), dim3(SQ_THREADS), 0, dgx_stream(stream), x, sB, sC, sN, B, C, N, order,
                       xx);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

size_t dgx_knn_workspace_bytes(int B, int N) { return (size_t)B * (size_t)N * sizeof(float); }

int dgx_knn_select_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, const float* xx, int B, int C, int N,
                       int k, int64_t* idx64, int32_t* idx32, float* vals, void* stream) {
    if (!x || !xx || B < 0 || C < 1 || N < 1 || k < 1 || k > N) return DGX_EINVAL;
    if (!idx64 && !idx32) return DGX_EINVAL;
    if (C > 128 || k > 64 || N > FIX_MAXN) return DGX_EUNSUPPORTED;
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
    if (C > 128 || k > 64 || N > FIX_MAXN) return DGX_EUNSUPPORTED;
    if (workspace_bytes < dgx_knn_workspace_bytes(B, N) || !workspace) return DGX_EINVAL;
    if (B == 0) return DGX_OK;
    float* xx = static_cast<float*>(workspace);
    int rc = dgx_sqnorm_f32(x, sB, sC, sN, B, C, N, order, xx, stream);
    if (rc != DGX_OK) return rc;
    return dgx_knn_select_f32(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, nullptr, stream);
}

}  // extern "C"
