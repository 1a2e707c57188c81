// a1 — kNN for EdgeConv (replaces reference models/dgcnn.py:6-12).
//
// One fused pass per cloud, no N x N matrix in HBM:
//   * |x|^2 per point in the reference's exact fp32 summation order (sqnorm).
//   * Gram tiles on the f32 MFMA (v_mfma_f32_16x16x4f32). Its result is
//     bit-for-bit the k-ordered fmaf chain (cdna_hip_programming.md §3), which
//     is exactly what MKL's sgemm does for the reference, so the
//     distances match the reference bit for bit.
//   * pd = fl(fl(2*dot - xx_j) - xx_i) (dgcnn.py:7-9) and a per-row top-k kept
//     in registers: 8 lanes per query (4 lanes x 2 candidate halves), merged
//     at the end.
//
// Two launches per call:
//   knn_image_kernel  one pass over x: |x|^2 in the reference's order and an
//                     MFMA A-operand "image" of each cloud (16-candidate tiles,
//                     lane-ordered so a wave fetches a tile with 16-B loads).
//   knn_kernel        workgroup = 4 waves = 2 wave groups x 2 candidate halves
//                     (even / odd tiles); a wave serves QG groups of 16 queries
//                     (QG = 2 at C > 64: two independent MFMA chains per image
//                     tile). Each wave keeps its queries' operands in registers
//                     and streams its half of the cloud's image straight from L2
//                     through a two-slot register ring; no LDS staging, no
//                     barrier until the final merge. Each query's candidates are
//                     dealt over 8 register lists (4 lanes x 2 halves) with an
//                     admission bound shared through LDS; 3-channel clouds first
//                     run a values-only pre-pass that seeds that bound. A (rare)
//                     row whose list overflowed is recomputed exactly by the
//                     same block at the end (knn_fix_row).
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include <type_traits>

#include "common.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int KQ_GROUPS = 2;                    // query groups of 16 per block
constexpr int KQ_HALVES = 2;                    // candidate halves: waves per query group
constexpr int KQ_WAVES = KQ_GROUPS * KQ_HALVES;
constexpr int KQ_THREADS = 64 * KQ_WAVES;
constexpr int KQ_QPW = 16;                      // queries per wave
constexpr int KQ_QPB = KQ_GROUPS * KQ_QPW;      // queries per block
constexpr int KQ_QCAP = 16;                     // per-lane pending-candidate FIFO
// register-ring depth (operand units in flight) of the selection kernel: four
// at NSTEP = 16 while the lists leave the registers for it (k <= 20: 128 VGPRs,
// 4 waves per SIMD; from k = 32 on the two extra slots would spill)
#ifndef KNN_RING
#define KNN_RING(ns, kb) (((ns) == 16 && (kb) <= 20) ? 4 : 2)
#endif
constexpr int KQ_LISTS = 4 * KQ_HALVES;         // top-k lists (lanes) per query
static_assert(KQ_HALVES == 2, "the threshold exchange and the final merge pair two halves");

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

// Sum of the C squares sq[c*stride] in the rounding order `order` selects.
__device__ __forceinline__ float sqnorm_sum(const float* sq, int stride, int C, int order, bool tail) {
#pragma clang fp contract(off)
    if (order == DGX_ORDER_VEC8X4) {
        if (C < 8) return rowsum4(sq, stride, C);
        const int vs = C >> 3;
        float fin = 0.f;
        for (int c = 8 * vs; c < C; ++c) fin = fin + sq[c * stride];
        for (int l = 0; l < 8; ++l) fin = fin + rowsum4(sq + l * stride, 8 * stride, vs);
        return fin;
    }
    return tail ? rowsum4(sq, stride, C) : cascade16(sq, stride, C);
}

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
    return sqnorm_sum(sq, SQ_THREADS, C, order, tail);
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
    // For a sorted list the new slot q value is median(v[q-1], v[q], nv): one
    // v_med3_f32 per slot (ties keep the value, the ids follow the compares).
    bool gt_cur = nv > v[KMAX - 1];
#pragma unroll
    for (int q = KMAX - 1; q > 0; --q) {
        const bool gt_prev = nv > v[q - 1];
        v[q] = __builtin_amdgcn_fmed3f(v[q - 1], v[q], nv);
        id[q] = gt_prev ? id[q - 1] : (gt_cur ? nj : id[q]);
        gt_cur = gt_prev;
    }
    v[0] = gt_cur ? nv : v[0];
    id[0] = gt_cur ? nj : id[0];
}

// Per-lane list length for k <= KB. A query's candidates are dealt over
// KQ_LISTS = 8 lanes (interleaved by index, see knn_row), so the true top-k
// splits ~Binomial(k, 1/8) over its lists; KL is where that distribution's
// upper tail drops to ~2e-6 per lane. A lane needing more than KL slots flags
// its row, which is recomputed exactly (knn_fix_row).
template <int KB>
struct KnnList {
    // (KL 10 / 11 at KB 20 measured with the in-block fix-up: 87 -> 98 / 87 us
    // at C = 64, 154 -> 184 / 167 us at C = 128 — the rows they flag cost more
    // than the shorter insertion rounds save)
    static constexpr int KL = KB <= 16 ? 10 : (KB <= 20 ? 12 : (KB <= 32 ? 15 : (KB <= 40 ? 17 : 23)));
    static constexpr int RPL = (KB + 3) / 4;   // ranks per lane of a wave's 4-list merge
};

// Tile row of candidate c (0..15): c = 4r + g goes to row 4g + r, so MFMA
// output lane group g holds candidates g, g+4, g+8, g+12 of the tile. Index
// classes are interleaved over a query's lists, so neighbours that sit close
// together in a cloud's index order still spread over its 8 lists.
__device__ __forceinline__ int knn_row(int c) { return ((c & 3) << 2) | (c >> 2); }
__device__ __forceinline__ int knn_cand(int row) { return ((row & 3) << 2) | (row >> 2); }  // inverse (an involution)

// ------------------------------------------------------------ operand image --
// The MFMA A operand of every 16-candidate tile, in lane order: for tile s of
// cloud b, lane l = 16*kk + i holds channels 4t + kk (t = 0..NSTEP-1) of
// candidate 16 s + knn_cand(i), NSTEP floats per lane. Within a tile the
// floats are CHUNK-MAJOR when NSTEP % 4 == 0: 16-byte chunk u = t / 4 of lane l
// at chunk index u*64 + l,
//     img[(b*ntile + s)*64*NSTEP + ((t/4)*64 + l)*4 + t%4]
// so each 16-byte wave load (one chunk u of all 64 lanes) is 1 KiB of
// contiguous bytes = 8 whole 128-B lines. (Lane-major NSTEP floats per lane —
// the layout before r09 — made every such load touch 32 lines for 16 B each
// of the lane's 64 / 128 B: 4x the L1 tag traffic of the bytes used, which
// capped the operand stream.) NSTEP = 1 / 3: lane-major, l*NSTEP + t. A wave
// fetches a whole tile straight from L2, without staging through LDS or
// synchronising with other waves. Zero rows pad N to a multiple of 16 and zero channels pad C to
// 4*NSTEP (they add exact zeros to the fmaf chain). xximg holds |x_j|^2 in the
// same row order: xximg[(b*ntile + s)*16 + i]. A query's own operand (the B
// side) is read from the same image.
// offset of float t of image lane l inside its tile
template <int NSTEP>
__device__ __forceinline__ int img_off(int l, int t) {
    if constexpr (NSTEP % 4 == 0) return ((t >> 2) * 64 + l) * 4 + (t & 3);
    else return l * NSTEP + t;
}

// lane l's floats t0 .. t0+V-1 of a tile (t0 % 4 == 0 in the chunk-major form)
template <int NSTEP, int V>
__device__ __forceinline__ void ld_lane(const float* __restrict__ tile, int l, int t0, float (&r)[V]) {
    if constexpr (NSTEP % 4 == 0) {
        static_assert(V % 4 == 0, "whole chunks");
#pragma unroll
        for (int u = 0; u < V / 4; ++u) {
            const float4 q = *reinterpret_cast<const float4*>(tile + (((t0 >> 2) + u) * 64 + l) * 4);
            r[4 * u] = q.x;
            r[4 * u + 1] = q.y;
            r[4 * u + 2] = q.z;
            r[4 * u + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int u = 0; u < V; ++u) r[u] = tile[l * NSTEP + t0 + u];
    }
}

constexpr int KI_TILES = 1;  // tiles per image-builder block
// One pass over x per layer: the operand image, the |x|^2 image and xx itself
// (|x_i|^2 in the reference's rounding order, sqnorm_sum on the staged row).
template <int NSTEP>
__global__ __launch_bounds__(256) void knn_image_kernel(const float* __restrict__ x, int64_t sB, int64_t sC,
                                                        int64_t sN, int B, int C, int N, int order, int ntile,
                                                        int tgroups, float* __restrict__ xx,
                                                        float* __restrict__ img, float* __restrict__ xximg) {
#pragma clang fp contract(off)
    constexpr int CP = NSTEP * 4;
    constexpr int P = 16 * KI_TILES;
    __shared__ float rows[P][CP + 1];
    __shared__ float nrm[P];
    const int b = blockIdx.x / tgroups;
    const int s0 = (blockIdx.x - b * tgroups) * KI_TILES;
    const int t = threadIdx.x;
    const float* __restrict__ xb = x + b * sB;
    for (int e = t; e < P * CP; e += 256) {
        int p, c;
        if (sN == 1) { c = e / P; p = e - c * P; }   // candidate-fastest: unit stride along n
        else { p = e / CP; c = e - p * CP; }          // channel-fastest
        const int n = s0 * 16 + p;
        rows[p][c] = (n < N && c < C) ? xb[c * sC + n * sN] : 0.f;
    }
    __syncthreads();
    const int ntl = min(KI_TILES, ntile - s0);
    float* __restrict__ dst = img + ((int64_t)b * ntile + s0) * 64 * NSTEP;
    for (int e = t; e < ntl * 64 * NSTEP; e += 256) {   // coalesced stores in image order
        const int tl = e / (64 * NSTEP);
        const int r = e - tl * 64 * NSTEP;
        int l, st;
        if constexpr (NSTEP % 4 == 0) {   // chunk-major: r = ((st/4)*64 + l)*4 + st%4
            l = (r >> 2) & 63;
            st = ((r >> 8) << 2) | (r & 3);
        } else {
            l = r / NSTEP;
            st = r - l * NSTEP;
        }
        dst[e] = rows[tl * 16 + knn_cand(l & 15)][4 * st + (l >> 4)];
    }
    __syncthreads();
    if (t < P) {  // each thread squares its own row in place, then sums it in the reference order
        const int n = s0 * 16 + t;
        float v = 0.f;
        if (n < N) {
            for (int c = 0; c < C; ++c) rows[t][c] = rows[t][c] * rows[t][c];
            v = sqnorm_sum(&rows[t][0], 1, C, order, n >= (N & ~31));
            xx[(int64_t)b * N + n] = v;
        }
        nrm[t] = v;
    }
    __syncthreads();
    if (t < P && s0 + t / 16 < ntile) xximg[((int64_t)b * ntile + s0) * 16 + t] = nrm[(t & ~15) + knn_cand(t & 15)];
}

inline int knn_nstep(int C) { return C <= 4 ? 1 : (C <= 12 ? 3 : (C <= 32 ? 8 : (C <= 64 ? 16 : 32))); }
inline int knn_ntile(int N) { return (N + 15) / 16; }

constexpr int FIX_MAXN = 12288;  // largest N (the fix-up's tie bitmap)
constexpr int FX_CAP = 256;      // candidates above T0 ranked directly by the fix-up

// Canonical order: value descending, then index ascending.
__device__ __forceinline__ bool canon_better(float av, int aj, float bv, int bj) {
    return av > bv || (av == bv && aj < bj);
}

template <int V>
__device__ __forceinline__ void ld_vec(const float* __restrict__ p, float (&r)[V]) {
    if constexpr (V % 4 == 0) {
#pragma unroll
        for (int u = 0; u < V; u += 4) {
            const float4 q = *reinterpret_cast<const float4*>(p + u);
            r[u] = q.x;
            r[u + 1] = q.y;
            r[u + 2] = q.z;
            r[u + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int u = 0; u < V; ++u) r[u] = p[u];
    }
}

// ------------------------------------------------------------- fix-up ----
// Exact recompute of one flagged query row qf of cloud b by the whole block
// (called block-uniformly after the merge). T0 = the merged k-th value of the
// row's lists: at least k candidates reach it, so the true k-th value is >= T0.
// Every distance is recomputed by the same MFMA chain on the same operands as
// the main stream (the query's doubled operand replicated over the 16 output
// columns; wave w takes tiles w, w+4, ...), so the values are identical.
//   n_gt = #{v > T0}. If n_gt >= k the top-k is among them: rank them
//   canonically (all-pairs) when they fit FX_CAP. If n_gt < k the k-th value is
//   T0 itself: the n_gt candidates above it, then the k - n_gt smallest indices
//   with v == T0 (a bitmap of ties, scanned in index order). With more than
//   FX_CAP candidates above T0 (mass ties) the row is extracted by k rounds of a
//   canonical arg-max over re-streamed values (slow, correct).
template <int NSTEP>
__device__ void knn_fix_row(float* fixa, const float* __restrict__ ib, const float* __restrict__ xib,
                            const float* __restrict__ xxb, int N, int k, int qf, float t0, int64_t row,
                            int64_t* __restrict__ idx64, int32_t* __restrict__ idx32, float* __restrict__ vals) {
#pragma clang fp contract(off)
    float* cv = fixa;
    int* cj = reinterpret_cast<int*>(fixa + FX_CAP);
    int* cnt = reinterpret_cast<int*>(fixa + 2 * FX_CAP);       // [0]: candidates above T0
    float* bestv = fixa + 2 * FX_CAP + 4;                        // [KQ_WAVES]: arg-max path per-wave values
    uint32_t* bits = reinterpret_cast<uint32_t*>(fixa + 2 * FX_CAP + 8);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, ql = lane & 15;
    const int ntile = (N + 15) >> 4, nw = (N + 31) >> 5;
    if (tid == 0) cnt[0] = 0;
    for (int w = tid; w < nw; w += KQ_THREADS) bits[w] = 0u;
    float bq[NSTEP];
    ld_lane<NSTEP, NSTEP>(ib + (int64_t)(qf >> 4) * 64 * NSTEP, g * 16 + knn_row(qf & 15), 0, bq);
#pragma unroll
    for (int t = 0; t < NSTEP; ++t) bq[t] *= 2.0f;
    const float xxq = xxb[qf];
    __syncthreads();
    // act(v, j) on every candidate; lanes with ql == 0 hold column 0 (all columns are the same query)
    auto stream = [&](auto&& act) {
        for (int s = wave; s < ntile; s += KQ_WAVES) {
            float a[NSTEP];
            ld_lane<NSTEP, NSTEP>(ib + (int64_t)s * 64 * NSTEP, lane, 0, a);
            const float4 xc = *reinterpret_cast<const float4*>(xib + s * 16 + 4 * g);
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < NSTEP; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], bq[t], acc, 0, 0, 0);
            if (ql == 0) {
                const int j0 = s * 16 + g;
                const float xcv[4] = {xc.x, xc.y, xc.z, xc.w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = j0 + 4 * r;
                    const float tq = acc[r] - xcv[r];
                    if (j < N) act(tq - xxq, j);
                }
            }
        }
    };
    stream([&](float v, int j) {
        if (v > t0) {
            const int sl = atomicAdd(&cnt[0], 1);
            if (sl < FX_CAP) { cv[sl] = v; cj[sl] = j; }
        } else if (v == t0) {
            atomicOr(&bits[j >> 5], 1u << (j & 31));
        }
    });
    __syncthreads();
    const int ngt = cnt[0];
    auto put = [&](int rank, int j, float v) {
        if (idx64) idx64[row * k + rank] = j;
        if (idx32) idx32[row * k + rank] = j;
        if (vals) vals[row * k + rank] = v;
    };
    if (ngt <= FX_CAP) {
        for (int t = tid; t < ngt; t += KQ_THREADS) {
            const float v = cv[t];
            const int j = cj[t];
            int rank = 0;
            for (int u = 0; u < ngt; ++u) rank += canon_better(cv[u], cj[u], v, j) ? 1 : 0;
            if (rank < k) put(rank, j, v);
        }
        if (ngt < k && wave == 0) {  // ranks ngt..k-1: ties at T0 in index order
            const int per = (nw + 63) >> 6;
            const int w0 = min(lane * per, nw), w1 = min(w0 + per, nw);
            int c = 0;
            for (int w = w0; w < w1; ++w) c += __popc(bits[w]);
            int inc = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(inc, o);
                if (lane >= o) inc += y;
            }
            int rank = ngt + inc - c;
            for (int w = w0; w < w1 && rank < k; ++w) {
                uint32_t m = bits[w];
                while (m && rank < k) {
                    const int bit = __ffs(m) - 1;
                    m &= m - 1;
                    put(rank++, (w << 5) + bit, t0);
                }
            }
        }
    } else {
        // mass ties above T0: rank r = the canonically best candidate worse than rank r-1
        float pv = INFINITY;
        int pj = -1;
        for (int r = 0; r < k; ++r) {
            float bv = -INFINITY;
            int bj = 0x7fffffff;
            stream([&](float v, int j) {
                if (canon_better(pv, pj, v, j) && canon_better(v, j, bv, bj)) { bv = v; bj = j; }
            });
#pragma unroll
            for (int o = 16; o < 64; o <<= 1) {
                const float ov = __shfl_xor(bv, o);
                const int oj = __shfl_xor(bj, o);
                if (canon_better(ov, oj, bv, bj)) { bv = ov; bj = oj; }
            }
            __syncthreads();  // previous round's picks are read
            if (lane == 0) { bestv[wave] = bv; cj[wave] = bj; }
            __syncthreads();
            pv = bestv[0];
            pj = cj[0];
#pragma unroll
            for (int w = 1; w < KQ_WAVES; ++w)
                if (canon_better(bestv[w], cj[w], pv, pj)) { pv = bestv[w]; pj = cj[w]; }
            if (tid == 0) put(r, pj, pv);
        }
    }
    __syncthreads();  // the fix-up area is free for the next row
}

// ------------------------------------------------------------ knn kernel ----
// Block = KQ_GROUPS wave groups x 2 candidate halves, one wave each; a wave
// serves QG groups of 16 queries (QG = 2: 32 queries per wave, 64 per block).
// A wave streams the tiles s = h, h+2, h+4, ... of its cloud's image with its
// loads two units ahead (see the operand stream below). With QG = 2 every
// image tile feeds two independent MFMA chains (one per query group), so a
// wave keeps the matrix pipe busy through the f32 MFMA's dependent latency
// and each tile is fetched once per 32 queries. The only block-wide
// synchronisation is the final merge.
template <int KB, int QG>
constexpr int knn_smem_floats_qg() {
    constexpr int qpb = KQ_GROUPS * KQ_QPW * QG;
    constexpr int stream = KQ_HALVES * qpb                              // published admission bounds
                           + KQ_WAVES * QG * KQ_QCAP * 64 * 2;          // FIFO (value, index) pairs
    constexpr int merge = KQ_HALVES * qpb * KB * 2 + 2 * qpb;          // half lists | k-th | flags
    constexpr int fix = merge + 2 * FX_CAP + 8 + FIX_MAXN / 32;         // ... | fix-up candidates, counters, tie bitmap
    return stream > fix ? stream : fix;
}

template <int NSTEP, int KB, int QG>
__global__ __launch_bounds__(KQ_THREADS, QG == 1 ? (KB <= 40 ? 4 : 2) : (KB <= 40 ? 2 : 1))
void knn_kernel(const float* __restrict__ img, const float* __restrict__ xximg, const float* __restrict__ xx, int B,
                int N, int k, int nqb, int64_t* __restrict__ idx64, int32_t* __restrict__ idx32,
                float* __restrict__ vals
#ifdef DGX_KNN_STATS
                , uint32_t* __restrict__ stats
#endif
                ) {
#pragma clang fp contract(off)
    constexpr int KL = KnnList<KB>::KL;
    constexpr int RPL = KnnList<KB>::RPL;
    constexpr int QPW = KQ_QPW * QG;           // queries per wave
    constexpr int QPB = KQ_GROUPS * QPW;       // queries per block
    __shared__ __attribute__((aligned(16))) float smem[knn_smem_floats_qg<KB, QG>()];
    float* pub = smem;                         // [KQ_HALVES][QPB] admission bounds
    // per (wave, group) [KQ_QCAP][64] pending (value, index) pairs: one 8-byte
    // LDS store per considered candidate and a single address computation
    float2* fifo = reinterpret_cast<float2*>(smem + KQ_HALVES * QPB);

    int b, qb;
    if (!dgx_xcd_cloud_map(blockIdx.x, B, nqb, b, qb)) return;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    // wave-uniform in a scalar register: the half's tile count and every
    // "unit is live" test become scalar branches
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave % KQ_GROUPS;  // wave group: queries grp*QPW ..
    const int h = wave / KQ_GROUPS;    // candidate half: tiles h, h + 2, h + 4, ...
    const int g = lane >> 4;           // MFMA output rows 4g..4g+3 of a tile
    const int ql = lane & 15;
    const int ntile = (N + 15) >> 4;
    const float* __restrict__ ib = img + (int64_t)b * ntile * 64 * NSTEP;
    const float* __restrict__ xib = xximg + (int64_t)b * ntile * 16;
    const int m = (k + KQ_LISTS - 1) / KQ_LISTS;
    const int m4 = (k + 3) / 4;

    // Per query group: one struct per group, every access by name (an array
    // indexed by the group number is not split into registers: its selects
    // became scratch loads).
    struct Grp {
        int qq, q;               // query within the block / within the cloud
        float bq[NSTEP];         // B operand: x[q][4t + g], doubled
        float xxq, tseed, thr;
        float lv[KL];            // the lane's sorted list (value desc, index asc)
        int li[KL];
        float2* fq;              // the lane's FIFO of admitted candidates (LDS, stride 64)
        int cnt;
        f32x4 acc;
        float last;
        float ov[RPL];           // merged ranks 4t + g of the wave's 4 lists
        int oj[RPL];
        int rk[RPL];             // final ranks after the half merge
    };
    Grp G0, G1;
    auto each = [&](auto&& fn) {
        fn(G0, 0);
        if constexpr (QG == 2) fn(G1, 1);
    };

    each([&](Grp& S, int e) {
        S.qq = grp * QPW + e * KQ_QPW + ql;
        S.q = qb * QPB + S.qq;
        // B operand from the query's own image row (zero channels beyond C;
        // q >= N reads a zero row). 2 x the query operand: every product and
        // partial sum of the fmaf chain doubles exactly, so the MFMA returns
        // fl(2 * dot) (dgcnn.py:7) directly.
        const int qs = min(S.q, N - 1);
        ld_lane<NSTEP, NSTEP>(ib + (int64_t)(qs >> 4) * 64 * NSTEP, g * 16 + knn_row(qs & 15), 0, S.bq);
#pragma unroll
        for (int t = 0; t < NSTEP; ++t) S.bq[t] *= 2.0f;
        S.xxq = S.q < N ? xx[(int64_t)b * N + S.q] : 0.f;
        // admission seed: a lower bound of the row's k-th value in this
        // kernel's exact arithmetic (the 3-channel pre-pass below), so
        // candidates below it can never enter the top-k; -inf without one
        S.tseed = -INFINITY;
        S.thr = S.tseed;
#pragma unroll
        for (int t = 0; t < KL; ++t) { S.lv[t] = -INFINITY; S.li[t] = 0x7fffffff; }
        S.fq = fifo + (wave * QG + e) * (KQ_QCAP * 64) + lane;
        S.cnt = 0;
    });
    // Each lane keeps, per group, the KL best of ITS candidates (sorted,
    // registers, static indexing). Admission filter thr = max(own KL-th, T)
    // where T = min over the query's 8 lists of their m-th value, m = ceil(k/8):
    // 8 lists x m candidates >= T exist, so T never exceeds the row's final k-th
    // value. The other half's 4 lists contribute through `pub` — a value
    // published at its last flush; lists only improve, so a stale value is
    // still a lower bound. '>=' keeps equal values; their order is settled
    // canonically at the merge. Candidates that pass wait in the lane's FIFO
    // and are inserted in batches, so an insertion round (5*KL VALU ops for
    // the whole wave) is paid once per admitted candidate of the busiest lane.
    if (tid < KQ_HALVES * QPB) pub[tid] = -INFINITY;
    static_assert(KnnList<KB>::KL >= (KB + 3) / 4, "lists must hold the m4-th value");
    __syncthreads();
    if constexpr (NSTEP == 1 && QG == 1) {
        // Admission pre-pass (3-channel clouds, where one MFMA makes a whole
        // tile and the selection VALU is the cost): each lane first streams its
        // candidates once keeping only the m = ceil(k/8) best VALUES (one
        // v_med3 per slot, no indices, no FIFO). 8 lists x m candidates reach
        // T = min over the query's 8 lists of their m-th value, so T is a lower
        // bound of the row's k-th value in this kernel's own arithmetic — the
        // main pass then admits only the few candidates above it instead of
        // inserting everything while its bound climbs from -inf.
        constexpr int MM = (KB + KQ_LISTS - 1) / KQ_LISTS;
        float p[MM];
#pragma unroll
        for (int t = 0; t < MM; ++t) p[t] = -INFINITY;
        const int ntl0 = (ntile - h + KQ_HALVES - 1) / KQ_HALVES;
        auto put = [&](float v) {
#pragma unroll
            for (int t = MM - 1; t > 0; --t) p[t] = __builtin_amdgcn_fmed3f(p[t - 1], p[t], v);
            p[0] = fmaxf(p[0], v);
        };
        // tiles in chunks of PC, the next chunk's operands in flight while this
        // one is selected (one L2 latency per chunk, not per tile); only the
        // cloud's last tile can hold padding rows (j >= N: excluded)
        constexpr int PC = 4;
        float av[2][PC];
        float4 xv[2][PC];
        auto fetch = [&](int buf, int tl0) {
#pragma unroll
            for (int c = 0; c < PC; ++c) {
                const int s = h + KQ_HALVES * min(tl0 + c, ntl0 - 1);
                av[buf][c] = ib[(int64_t)s * 64 + lane];
                xv[buf][c] = *reinterpret_cast<const float4*>(xib + s * 16 + 4 * g);
            }
        };
        if (ntl0 > 0) fetch(0, 0);
#pragma unroll 1
        for (int tl0 = 0; tl0 < ntl0; tl0 += 2 * PC) {
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const int base = tl0 + half * PC;
                fetch(half ^ 1, base + PC);
                if (base < ntl0) {
#pragma unroll
                    for (int c = 0; c < PC; ++c) {
                        const int tl = base + c;
                        const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(av[half][c], G0.bq[0],
                                                                             f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                        const float4 xc4 = xv[half][c];
                        float v0 = (d[0] - xc4.x) - G0.xxq, v1 = (d[1] - xc4.y) - G0.xxq;
                        float v2 = (d[2] - xc4.z) - G0.xxq, v3 = (d[3] - xc4.w) - G0.xxq;
                        const int s = h + KQ_HALVES * tl;
                        if (tl >= ntl0 || (s + 1) * 16 > N) {   // wave-uniform: past the end / the padded tile
                            const int j0 = tl < ntl0 ? s * 16 + g : N;
                            v0 = j0 < N ? v0 : -INFINITY;
                            v1 = j0 + 4 < N ? v1 : -INFINITY;
                            v2 = j0 + 8 < N ? v2 : -INFINITY;
                            v3 = j0 + 12 < N ? v3 : -INFINITY;
                        }
                        put(v0);
                        put(v1);
                        put(v2);
                        put(v3);
                    }
                }
            }
        }
        // (an exact k-th of the 8 lists' values by counting measured slower:
        // 61 vs 57 us at cfg2, the count costs more than the admissions it saves)
        float tm = p[0];
#pragma unroll
        for (int t = 1; t < MM; ++t) tm = (t == m - 1) ? p[t] : tm;
        tm = fminf(tm, __shfl_xor(tm, 16));
        tm = fminf(tm, __shfl_xor(tm, 32));
        if (g == 0) pub[h * QPB + G0.qq] = tm;
        __syncthreads();
        const float T = fminf(tm, pub[(1 - h) * QPB + G0.qq]);
        if (G0.q < N) G0.tseed = fmaxf(G0.tseed, T);
        G0.thr = G0.tseed;
    }
#ifdef DGX_KNN_STATS
    uint32_t n_rounds = 0, n_flush = 0;
#endif
    auto cmax = [&]() { return QG == 2 ? max(G0.cnt, G1.cnt) : G0.cnt; };
    auto flush = [&]() {
#ifdef DGX_KNN_STATS
        ++n_flush;
#endif
        // branch-free rounds: slots past a lane's count read stale entries and
        // are replaced by -inf, so every round is the same straight-line code;
        // the groups' lists are independent (two interleaved dependency chains)
        float2 c0 = G0.fq[0], c1 = make_float2(0.f, 0.f);
        float cv0 = G0.cnt > 0 ? c0.x : -INFINITY, cv1 = 0.f;
        int cj0 = __float_as_int(c0.y), cj1 = 0;
        if constexpr (QG == 2) {
            c1 = G1.fq[0];
            cv1 = G1.cnt > 0 ? c1.x : -INFINITY;
            cj1 = __float_as_int(c1.y);
        }
        const int cm = cmax();
        // fully unrolled with an early exit: no loop-carried copies of the list
#pragma unroll
        for (int t = 0; t < KQ_QCAP; ++t) {
            if (!__any(t < cm)) break;
#ifdef DGX_KNN_STATS
            ++n_rounds;
#endif
            const int nx = min(t + 1, KQ_QCAP - 1);
            const float2 n0 = G0.fq[nx * 64];
            const float nv0 = t + 1 < G0.cnt ? n0.x : -INFINITY;
            const int nj0 = __float_as_int(n0.y);
            list_insert_ordered<KL>(G0.lv, G0.li, cv0 >= G0.thr ? cv0 : -INFINITY, cj0);
            cv0 = nv0;
            cj0 = nj0;
            if constexpr (QG == 2) {
                const float2 n1 = G1.fq[nx * 64];
                const float nv1 = t + 1 < G1.cnt ? n1.x : -INFINITY;
                const int nj1 = __float_as_int(n1.y);
                list_insert_ordered<KL>(G1.lv, G1.li, cv1 >= G1.thr ? cv1 : -INFINITY, cj1);
                cv1 = nv1;
                cj1 = nj1;
            }
        }
        each([&](Grp& S, int) {
            S.cnt = 0;
            // admission bound: max of (own 4 lists' min m4-th value: 4*m4 >= k
            // candidates reach it) and (all 8 lists' min m-th value: 8*m >= k)
            float tm = S.lv[0], t4 = S.lv[0];
#pragma unroll
            for (int t = 1; t < KL; ++t) {
                tm = (t == m - 1) ? S.lv[t] : tm;
                t4 = (t == m4 - 1) ? S.lv[t] : t4;
            }
            tm = fminf(tm, __shfl_xor(tm, 16));
            tm = fminf(tm, __shfl_xor(tm, 32));
            t4 = fminf(t4, __shfl_xor(t4, 16));
            t4 = fminf(t4, __shfl_xor(t4, 32));
            if (g == 0) __hip_atomic_store(pub + h * QPB + S.qq, tm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const float tp = __hip_atomic_load(pub + (1 - h) * QPB + S.qq, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
            S.thr = fmaxf(fmaxf(fmaxf(t4, fminf(tm, tp)), S.lv[KL - 1]), S.tseed);
        });
    };

    // TAIL: the cloud's last tile when N % 16 != 0 (wave-uniform), the only
    // one whose rows can be padding (j >= N)
    auto consider = [&](Grp& S, float dot, float xc, int j, auto tail) {
        const float tq = dot - xc;  // dot is already 2 x (query operand doubled)
        const float v = tq - S.xxq;
        const bool pass = (!decltype(tail)::value || j < N) && v >= S.thr;
        // unconditional store: a rejected candidate's slot is reused by the
        // next one (a tile adds at most 4 entries to a FIFO holding <= QCAP-4)
        S.fq[S.cnt * 64] = make_float2(v, __int_as_float(j));
        S.cnt += pass ? 1 : 0;
    };

    // Operand stream: units of SW MFMA k-steps (half a tile at NSTEP = 16, a
    // quarter tile at NSTEP = 32, a whole tile below) through a RING-slot
    // register ring; the load of unit u+RING is issued as soon as unit u's
    // MFMAs have read their slot, so a unit's L2 latency hides behind RING-1
    // units of MFMA + selection work. (With two slots at NSTEP = 16 the wave
    // waited for its next tile right after issuing it: SQ_WAIT_INST_ANY was
    // 52 % of the wave cycles, r04j_pmc_cfg2.json.)
    constexpr int SW = NSTEP <= 8 ? NSTEP : 8;
    constexpr int SPT = NSTEP / SW;          // units per tile
    constexpr int RING = KNN_RING(NSTEP, KB);
    constexpr int UB = RING > SPT ? RING : SPT;   // units per loop trip (static ring slots)
    static_assert(NSTEP % SW == 0 && UB % SPT == 0 && UB % RING == 0, "unit split");
    const int ntl = (ntile - h + KQ_HALVES - 1) / KQ_HALVES;  // this half's tiles: h + 2*tl
    const int nunits = ntl * SPT;
    float a[RING][SW];
    float4 xq[RING];
#pragma unroll
    for (int r = 0; r < RING; ++r) xq[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    // Every load is unconditional (a unit past the end re-reads this half's
    // last tile, unused): with a data-dependent skip the compiler cannot count
    // the loads in flight and drains them all (vmcnt(0)) every trip. sl = u %
    // SPT is a compile-time constant at every call.
    // NSTEP <= 16: the loads of a unit are pinned as one group (sched_barrier)
    // so the prologue and the loop issue them in the same order; the wait
    // insertion then counts the ring's real distance at each trip's head
    // instead of draining it (vmcnt(0)). C = 64 90.5 -> 89.8 us, 4-cloud
    // shard 38.5 -> 37.8 us per call (r09q); at C = 128 (two groups) +1 %: off
    constexpr bool PIN = NSTEP <= 16;
    auto load = [&](int slot, int u, int sl) {
        const int s = min(h + KQ_HALVES * (u / SPT), ntile - 1);
        if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
        ld_lane<NSTEP, SW>(ib + (int64_t)s * 64 * NSTEP, lane, sl * SW, a[slot]);
        if (sl == 0) xq[slot] = *reinterpret_cast<const float4*>(xib + s * 16 + 4 * g);
        if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
    };
#pragma unroll
    for (int r = 0; r < RING; ++r) load(r, r, r % SPT);
    float4 xc = xq[0];
    float probe_sum = 0.f;
    (void)probe_sum;
#pragma unroll 1
    for (int u = 0; u < nunits; u += UB) {
#pragma unroll
        for (int ub = 0; ub < UB; ++ub) {
            const int slot = ub % RING, sl = ub % SPT;
            // every unit of a trip runs: a unit past the end (only in the last
            // trip, when nunits % UB != 0) re-reads the half's last tile and its
            // candidates fail the j < N test (its tile index is past the cloud, so
            // the TAIL form of consider runs). A wave-uniform `live` test here made
            // the trip's control flow conditional and the compiler drained every
            // operand load in flight (s_waitcnt vmcnt(0)) at each trip's start.
#ifndef KNN_LIVE_TEST
            constexpr bool live = true;
#else
            const bool live = UB == SPT || u + ub < nunits;   // (A/B builds only)
#endif
            if (live) {
                if (sl == 0) {
                    each([&](Grp& S, int) { S.acc = f32x4{0.f, 0.f, 0.f, 0.f}; });
                    xc = xq[slot];
                }
                // the groups' chains interleaved: independent MFMAs back to back,
                // issued at raised wave priority so a wave entering its chain
                // goes ahead of the other waves' selection VALU (r09h: C = 128
                // 146 -> 140 us, C = 64 92 -> 91 us per call)
#ifndef KNN_PRIO
#define KNN_PRIO 1
#endif
#if KNN_PRIO
                __builtin_amdgcn_s_setprio(KNN_PRIO);
#endif
#pragma unroll
                for (int t = 0; t < SW; ++t)
                    each([&](Grp& S, int) {
                        S.acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[slot][t], S.bq[sl * SW + t], S.acc, 0, 0, 0);
                    });
#if KNN_PRIO
                __builtin_amdgcn_s_setprio(0);
#endif
            }
#ifndef KNN_PROBE_NOLOAD
            load(slot, u + ub + RING, (ub + RING) % SPT);
#endif
            if (live && sl == SPT - 1) {
                // lane holds rows 4g..4g+3 = candidates g, g+4, g+8, g+12 of the tile
                const int st = h + KQ_HALVES * ((u + ub) / SPT);
                const int j0 = st * 16 + g;
                auto cons4 = [&](auto tail) {
                    each([&](Grp& S, int) {
                        consider(S, S.acc[0], xc.x, j0, tail);
                        consider(S, S.acc[1], xc.y, j0 + 4, tail);
                        consider(S, S.acc[2], xc.z, j0 + 8, tail);
                        consider(S, S.acc[3], xc.w, j0 + 12, tail);
                    });
                };
                // (the two-group kernel keeps the check everywhere: its split
                // code measured 2 us slower, r04u)
#ifdef KNN_PROBE_NOSEL   // timing probe (A/B builds only): the Gram stream without the selection
                each([&](Grp& S, int) { probe_sum += S.acc[0] + S.acc[1] + S.acc[2] + S.acc[3] + xc.x; });
                (void)j0;
#else
                if (QG == 2 || (st + 1) * 16 > N) cons4(std::true_type{});
                else cons4(std::false_type{});
                if (__any(cmax() > KQ_QCAP - 4)) flush();
#endif
            }
        }
    }
#if defined(KNN_PROBE_NOSEL) || defined(KNN_PROBE_NOLOAD)
    // timing probes (A/B builds only; wrong results): skip the merge and fix-up
    if (probe_sum == 1234.5f && vals) vals[tid] = probe_sum;
    return;
#endif
    flush();

    // Merge the wave's 4 lists of each query (lanes ql, ql+16, ql+32, ql+48)
    // by k rounds of a canonical arg-max over the 4 list heads; the winning
    // lane pops its head. Rank r ends up in lane r % 4. The groups' merges are
    // independent and interleaved.
    each([&](Grp& S, int) { S.last = S.lv[KL - 1]; });
#pragma unroll
    for (int r = 0; r < KB; ++r) {
        if (r < k) {
            each([&](Grp& S, int) {
                float hv = S.lv[0];
                int hj = S.li[0];
                float pv = __shfl_xor(hv, 16);
                int pj = __shfl_xor(hj, 16);
                if (canon_better(pv, pj, hv, hj)) { hv = pv; hj = pj; }
                pv = __shfl_xor(hv, 32);
                pj = __shfl_xor(hj, 32);
                if (canon_better(pv, pj, hv, hj)) { hv = pv; hj = pj; }
                const bool pop = S.li[0] == hj && S.lv[0] == hv;
#pragma unroll
                for (int t = 0; t < KL - 1; ++t) {
                    S.lv[t] = pop ? S.lv[t + 1] : S.lv[t];
                    S.li[t] = pop ? S.li[t + 1] : S.li[t];
                }
                S.lv[KL - 1] = pop ? -INFINITY : S.lv[KL - 1];
                S.li[KL - 1] = pop ? 0x7fffffff : S.li[KL - 1];
                if ((r & 3) == g) { S.ov[r >> 2] = hv; S.oj[r >> 2] = hj; }
            });
        }
    }

    // Merge the two halves: each half's sorted top-k goes to LDS; an element's
    // final rank is its rank in its own list plus the number of elements of the
    // other list that are canonically better (binary search). The halves hold
    // disjoint candidates, so the ranks 0..k-1 are taken exactly once.
    __syncthreads();  // every wave is done with its FIFO
    float2* lists = reinterpret_cast<float2*>(smem);         // [KQ_HALVES][QPB][KB]
    float* kth = smem + KQ_HALVES * QPB * KB * 2;            // [QPB] merged k-th value
    int* flg = reinterpret_cast<int*>(kth + QPB);            // [QPB] row needs the fix-up
    each([&](Grp& S, int) {
#pragma unroll
        for (int t = 0; t < RPL; ++t) {
            const int r = 4 * t + g;
            if (r < k) lists[(h * QPB + S.qq) * KB + r] = make_float2(S.ov[t], __int_as_float(S.oj[t]));
        }
    });
    if (tid < QPB) {
        kth[tid] = -INFINITY;
        flg[tid] = 0;
    }
    __syncthreads();
    each([&](Grp& S, int) {
        const float2* other = lists + ((1 - h) * QPB + S.qq) * KB;
#pragma unroll
        for (int t = 0; t < RPL; ++t) {
            const int r = 4 * t + g;
            S.rk[t] = k;
            if (r < k) {
                int lo = 0, hi = k;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    const float2 o = other[mid];
                    if (canon_better(o.x, __float_as_int(o.y), S.ov[t], S.oj[t])) lo = mid + 1;
                    else hi = mid;
                }
                S.rk[t] = r + lo;
                if (S.rk[t] == k - 1) kth[S.qq] = S.ov[t];
            }
        }
    });
    __syncthreads();
    each([&](Grp& S, int) {
        // A lane whose list was full and whose last kept value reaches the merged
        // k-th may have dropped a member of the true top-k: mark the row for the
        // exact fix-up pass.
        const float kv = kth[S.qq];
        if (S.last != -INFINITY && S.last >= kv) flg[S.qq] = 1;
        // fewer than k candidates reached the seed (the merged k-th is then a -inf
        // pad): only a seed that is not a value of this kernel's arithmetic does
        // that; the exact fix-up from T0 = -inf repairs the row
        if (!(kv >= S.tseed)) flg[S.qq] = 1;
    });
    __syncthreads();
    each([&](Grp& S, int) {
        if (S.q < N && flg[S.qq] == 0) {  // flagged rows are written by the fix-up below
            const int64_t row = ((int64_t)b * N + S.q) * k;
#pragma unroll
            for (int t = 0; t < RPL; ++t) {
                const int r = S.rk[t];
                if (r < k) {
                    if (idx64) idx64[row + r] = S.oj[t];
                    if (idx32) idx32[row + r] = S.oj[t];
                    if (vals) vals[row + r] = S.ov[t];
                }
            }
        }
    });
#ifdef DGX_KNN_STATS
    {   // diagnostics build only: per (block, wave) insertion rounds, flushes, flagged rows (vector stores)
        int nf = 0;
        for (int f = 0; f < QPB; ++f) nf += (flg[f] != 0 && qb * QPB + f < N) ? 1 : 0;
        if (lane == 0 && stats != nullptr) {
            uint32_t* st = stats + ((int64_t)blockIdx.x * KQ_WAVES + wave) * 4;
            st[0] = n_rounds; st[1] = n_flush; st[2] = wave == 0 ? (uint32_t)nf : 0u; st[3] = 1u;
        }
    }
#endif
    // the block's flagged rows (rare), one at a time; flg / kth are block-uniform LDS reads
    float* fixa = smem + KQ_HALVES * QPB * KB * 2 + 2 * QPB;
    for (int f = 0; f < QPB; ++f) {
        const int qf = qb * QPB + f;
        if (flg[f] != 0 && qf < N)
            knn_fix_row<NSTEP>(fixa, ib, xib, xx + (int64_t)b * N, N, k, qf, kth[f], (int64_t)b * N + qf, idx64,
                               idx32, vals);
    }
}

#ifdef DGX_KNN_STATS
uint32_t* g_knn_stats = nullptr;   // diagnostics build: device buffer set by dgx_knn_stats_buffer
#endif

// image floats per cloud, then |x|^2 image floats per cloud
inline size_t knn_image_floats(int C, int N) { return (size_t)knn_ntile(N) * 64 * knn_nstep(C); }
inline size_t knn_xximg_floats(int N) { return (size_t)knn_ntile(N) * 16; }

// ------------------------------------- apply + next block's kNN image ----
// An EdgeConv block's output x_l = LeakyReLU(a ysel + b) (dgcnn.py:84-98) is
// the next block's kNN input (dgcnn.py:88: knn(x_l) on the contiguous (B,C,N)
// tensor, ORDER_STRIDED). This kernel writes x_l (fp32 concat slice + its bf16
// twin, as dgx_bn_lrelu_apply_f32 does) AND what knn_image_kernel would build
// from it — the MFMA operand image, |x|^2 and the |x|^2 image — so the next
// kNN skips its image pass. One point per TPP = C/4 lanes (4 channels each);
// |x|^2 in the reference's cascade order (C a multiple of 16, no tail points:
// N % 32 == 0): lane 4r gathers run r's 16 squares (channels 16r..16r+15) and
// sums them in order, lane 0 adds the runs in order (sqnorm_sum's cascade16).
template <int CO>
__global__ __launch_bounds__(256) void apply_image_kernel(const float* __restrict__ ysel, int M, int N,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift, float slope,
                                                          float* __restrict__ out, int ldo, __bf16* __restrict__ out16,
                                                          float* __restrict__ xx, float* __restrict__ img,
                                                          float* __restrict__ xximg) {
#pragma clang fp contract(off)
    constexpr int NSTEP = CO / 4, TPP = CO / 4, PPB = 256 / TPP, RUNS = CO / 16;
    static_assert(CO % 16 == 0 && TPP <= 64, "whole 16-channel runs, one point inside a wave");
    const int q = threadIdx.x % TPP;
    const int64_t i = (int64_t)blockIdx.x * PPB + threadIdx.x / TPP;   // point row b*N + n
    const bool ok = i < M;
    const int64_t ic = ok ? i : M - 1;
    const float4 y = *reinterpret_cast<const float4*>(ysel + ic * CO + 4 * q);
    const float4 a = *reinterpret_cast<const float4*>(scale + 4 * q);
    const float4 c = *reinterpret_cast<const float4*>(shift + 4 * q);
    float v[4] = {lrelu(fmaf(a.x, y.x, c.x), slope), lrelu(fmaf(a.y, y.y, c.y), slope),
                  lrelu(fmaf(a.z, y.z, c.z), slope), lrelu(fmaf(a.w, y.w, c.w), slope)};
    const int b = (int)(ic / N), n = (int)(ic - (int64_t)b * N);
    const int ntile = N >> 4, st = n >> 4, ii = knn_row(n & 15);
    if (ok) {
        *reinterpret_cast<float4*>(out + i * ldo + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
        if (out16) {
            typedef __bf16 h4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<h4*>(out16 + i * ldo + 4 * q) = h4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
        }
        // image lane 16 u + ii of tile st holds channels 4 t + u: here t = q
        float* __restrict__ ib = img + ((int64_t)b * ntile + st) * 64 * NSTEP;
#pragma unroll
        for (int u = 0; u < 4; ++u) ib[img_off<NSTEP>(16 * u + ii, q)] = v[u];
    }
    float sq[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) sq[u] = v[u] * v[u];
    // run r = lanes 4r .. 4r+3 of the point: lane 4r collects the 16 squares
    const int lane = threadIdx.x & 63;
    float g[16];
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int u = 0; u < 4; ++u) g[4 * h + u] = __shfl(sq[u], lane + h, 64);
    float run = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) run = run + g[e];
    float runs[RUNS];
#pragma unroll
    for (int r = 0; r < RUNS; ++r) runs[r] = __shfl(run, lane + 4 * r, 64);
    if (ok && q == 0) {
        float a1 = 0.f;
#pragma unroll
        for (int r = 0; r < RUNS; ++r) a1 = a1 + runs[r];
        const float w = 0.f + a1;   // cascade16's a0 + a1 (a0 = 0: no partial run)
        xx[i] = w;
        xximg[((int64_t)b * ntile + st) * 16 + ii] = w;
    }
}

template <int NSTEP>
int launch_prepare(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int C, int N, int order, float* xx,
                   float* img, float* xximg, hipStream_t st) {
    const int ntile = knn_ntile(N);
    const int tgroups = (ntile + KI_TILES - 1) / KI_TILES;
    hipLaunchKernelGGL(knn_image_kernel<NSTEP>, dim3((unsigned)(B * tgroups)), dim3(256), 0, st, x, sB, sC, sN, B, C,
                       N, order, ntile, tgroups, xx, img, xximg);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

#ifndef KNN_QG2_C64_MINN
#define KNN_QG2_C64_MINN (1 << 30)
#endif
// query groups per wave: two where the MFMA chain dominates (C > 64; C = 64
// only on large clouds), one where the selection does (k <= 40: two groups'
// lists must fit in registers)
inline int knn_qg(int nstep, int kb, int N) {
    if (kb > 40) return 1;
    if (nstep >= 32) return 2;
    if (nstep == 16 && N >= KNN_QG2_C64_MINN) return 2;
    return 1;
}

// Grids of fewer than 512 workgroups at 32 queries per workgroup (few clouds:
// a strong-scaling shard) keep one query group per wave at C = 128 too: the
// two-group kernel would leave three quarters of the CUs idle (4 clouds: C = 128
// selection 93 -> 66 us, r05b). Splitting each group's candidates over four
// waves instead (knn_split_kernel, r05a/b) measured slower at every C.
inline bool knn_small(int B, int N) { return (int64_t)B * ((N + KQ_QPB - 1) / KQ_QPB) < 512; }

template <int NSTEP, int KB, int QG>
int launch_knn_qg(const float* xx, int B, int N, int k, int64_t* idx64, int32_t* idx32, float* vals,
                  const float* img, const float* xximg, hipStream_t st) {
    const int nqb = (N + KQ_QPB * QG - 1) / (KQ_QPB * QG);
    hipLaunchKernelGGL((knn_kernel<NSTEP, KB, QG>), dim3(dgx_xcd_cloud_grid(B, nqb)), dim3(KQ_THREADS), 0, st, img,
                       xximg, xx, B, N, k, nqb, idx64, idx32, vals
#ifdef DGX_KNN_STATS
                       , g_knn_stats
#endif
                       );
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

template <int NSTEP, int KB>
int launch_knn(const float* x, int64_t sB, int64_t sC, int64_t sN, const float* xx, int B, int C, int N,
               int k, int64_t* idx64, int32_t* idx32, float* vals, const float* img, const float* xximg,
               hipStream_t st) {
    // two query groups per wave where the MFMA chain dominates (C > 64, k <= 40:
    // the lists of two groups fit in registers); one where the selection does
    if constexpr (KB <= 40 && NSTEP >= 16) {
        if (knn_qg(NSTEP, KB, N) == 2 && !knn_small(B, N))
            return launch_knn_qg<NSTEP, KB, 2>(xx, B, N, k, idx64, idx32, vals, img, xximg, st);
    }
    return launch_knn_qg<NSTEP, KB, 1>(xx, B, N, k, idx64, idx32, vals, img, xximg, st);
}

template <int NSTEP>
int dispatch_k(const float* x, int64_t sB, int64_t sC, int64_t sN, const float* xx, int B, int C, int N, int k,
               int64_t* idx64, int32_t* idx32, float* vals, const float* img, const float* xximg, hipStream_t st) {
#define DGX_KNN_K(KBV) \
    return launch_knn<NSTEP, KBV>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, img, xximg, st)
    if (k <= 16) DGX_KNN_K(16);
    if (k <= 20) DGX_KNN_K(20);
    if (k <= 32) DGX_KNN_K(32);
    if (k <= 40) DGX_KNN_K(40);
    DGX_KNN_K(64);
#undef DGX_KNN_K
}

}  // namespace

extern "C" {

#ifdef DGX_KNN_STATS
// diagnostics build only (tools/knn_stats.py): per (block, wave) of the next
// selection launch, {insertion rounds, flushes, flagged rows, 1} as uint32
void dgx_knn_stats_buffer(void* dev) { g_knn_stats = static_cast<uint32_t*>(dev); }
#endif

const char* dgx_knn_kernel_name(int C, int k, int N) {
    // the selection kernel dgx_knn_select_f32 launches for (C, k, N) on grids of at least
    // 512 workgroups (knn_small: fewer clouds keep one query group per wave), as profilers print it
    struct Names {
        char s[5][5][2][40];
        Names() {
            static const int NS[5] = {1, 3, 8, 16, 32};
            static const int KBS[5] = {16, 20, 32, 40, 64};
            for (int a = 0; a < 5; ++a)
                for (int b = 0; b < 5; ++b)
                    for (int q = 0; q < 2; ++q)
                        snprintf(s[a][b][q], sizeof(s[a][b][q]), "knn_kernel<%d, %d, %d>", NS[a], KBS[b], q + 1);
        }
    };
    static const Names names;  // thread-safe one-time initialisation
    if (C < 1 || C > 128 || k < 1 || k > 64 || N < 1) return "";
    const int ns = knn_nstep(C);
    const int a = ns == 1 ? 0 : ns == 3 ? 1 : ns == 8 ? 2 : ns == 16 ? 3 : 4;
    const int b = k <= 16 ? 0 : k <= 20 ? 1 : k <= 32 ? 2 : k <= 40 ? 3 : 4;
    static const int KBS[5] = {16, 20, 32, 40, 64};
    return names.s[a][b][knn_qg(ns, KBS[b], N) - 1];
}

int dgx_bn_lrelu_apply_knn_image_f32(const float* ysel, int B, int N, int Co, const float* scale,
                                     const float* shift, float slope, float* out, int ldo, void* out_bf16, float* xx,
                                     void* image, size_t image_bytes, void* stream) {
    if (!ysel || !scale || !shift || !out || !xx || !image || B < 1 || N < 1 || ldo < Co) return DGX_EINVAL;
    if ((Co != 64 && Co != 128) || N % 32 != 0) return DGX_EUNSUPPORTED;
    if (image_bytes < dgx_knn_image_bytes(B, Co, N)) return DGX_EINVAL;
    if (ldo % 4 || reinterpret_cast<uintptr_t>(out) % 16 || reinterpret_cast<uintptr_t>(ysel) % 16 ||
        reinterpret_cast<uintptr_t>(scale) % 16 || reinterpret_cast<uintptr_t>(shift) % 16 ||
        reinterpret_cast<uintptr_t>(out_bf16) % 8 || reinterpret_cast<uintptr_t>(image) % 16)
        return DGX_EUNSUPPORTED;
    float* img = static_cast<float*>(image);
    float* xximg = img + (size_t)B * knn_image_floats(Co, N);
    const int M = B * N;
    hipStream_t st = dgx_stream(stream);
    if (Co == 64)
        hipLaunchKernelGGL(apply_image_kernel<64>, dim3((M + 15) / 16), dim3(256), 0, st, ysel, M, N, scale, shift,
                           slope, out, ldo, static_cast<__bf16*>(out_bf16), xx, img, xximg);
    else
        hipLaunchKernelGGL(apply_image_kernel<128>, dim3((M + 7) / 8), dim3(256), 0, st, ysel, M, N, scale, shift,
                           slope, out, ldo, static_cast<__bf16*>(out_bf16), xx, img, xximg);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

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

size_t dgx_knn_image_bytes(int B, int C, int N) {
    if (B < 0 || C < 1 || N < 1) return 0;
    // operand image | |x|^2 image
    return (size_t)B * (knn_image_floats(C, N) + knn_xximg_floats(N)) * sizeof(float);
}

size_t dgx_knn_workspace_bytes(int B, int C, int N) {
    if (B < 0 || C < 1 || N < 1) return 0;
    // |x|^2 (B*N floats, rounded up to 16 bytes) | operand image
    return ((((size_t)B * N + 3) & ~(size_t)3) * sizeof(float)) + dgx_knn_image_bytes(B, C, N);
}

int dgx_knn_prepare_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int C, int N, int order,
                        float* xx, void* image, size_t image_bytes, void* stream) {
    if (!x || !xx || B < 0 || C < 1 || N < 1) return DGX_EINVAL;
    if (C > 128) return DGX_EUNSUPPORTED;
    if (B == 0) return DGX_OK;
    if (!image || image_bytes < dgx_knn_image_bytes(B, C, N)) return DGX_EINVAL;
    if ((reinterpret_cast<uintptr_t>(image) & 15) != 0) return DGX_EINVAL;  // 16-byte operand loads
    float* img = static_cast<float*>(image);
    float* xximg = img + (size_t)B * knn_image_floats(C, N);
    hipStream_t st = dgx_stream(stream);
    switch (knn_nstep(C)) {
        case 1: return launch_prepare<1>(x, sB, sC, sN, B, C, N, order, xx, img, xximg, st);
        case 3: return launch_prepare<3>(x, sB, sC, sN, B, C, N, order, xx, img, xximg, st);
        case 8: return launch_prepare<8>(x, sB, sC, sN, B, C, N, order, xx, img, xximg, st);
        case 16: return launch_prepare<16>(x, sB, sC, sN, B, C, N, order, xx, img, xximg, st);
        default: return launch_prepare<32>(x, sB, sC, sN, B, C, N, order, xx, img, xximg, st);
    }
}

}  // extern "C"

namespace {
int knn_select(const float* x, int64_t sB, int64_t sC, int64_t sN, const float* xx, int B, int C, int N, int k,
               int64_t* idx64, int32_t* idx32, float* vals, const void* image, size_t image_bytes, void* stream) {
    if (!x || !xx || B < 0 || C < 1 || N < 1 || k < 1 || k > N) return DGX_EINVAL;
    if (!idx64 && !idx32) return DGX_EINVAL;
    if (C > 128 || k > 64 || N > FIX_MAXN) return DGX_EUNSUPPORTED;
    if (B == 0) return DGX_OK;
    if (!image || image_bytes < dgx_knn_image_bytes(B, C, N)) return DGX_EINVAL;
    if ((reinterpret_cast<uintptr_t>(image) & 15) != 0) return DGX_EINVAL;
    const float* img = static_cast<const float*>(image);
    const float* xximg = img + (size_t)B * knn_image_floats(C, N);
    hipStream_t st = dgx_stream(stream);
    switch (knn_nstep(C)) {
        case 1: return dispatch_k<1>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, img, xximg, st);
        case 3: return dispatch_k<3>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, img, xximg, st);
        case 8: return dispatch_k<8>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, img, xximg, st);
        case 16: return dispatch_k<16>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, img, xximg, st);
        default: return dispatch_k<32>(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, img, xximg, st);
    }
}
}  // namespace

extern "C" {

int dgx_knn_select_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, const float* xx, int B, int C, int N,
                       int k, int64_t* idx64, int32_t* idx32, float* vals, const void* image, size_t image_bytes,
                       void* stream) {
    return knn_select(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, vals, image, image_bytes, stream);
}

int dgx_knn_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int C, int N, int k, int order,
                int64_t* idx64, int32_t* idx32, void* workspace, size_t workspace_bytes, void* stream) {
    if (!x || B < 0 || C < 1 || N < 1 || k < 1 || k > N) return DGX_EINVAL;
    if (!idx64 && !idx32) return DGX_EINVAL;
    if (C > 128 || k > 64 || N > FIX_MAXN) return DGX_EUNSUPPORTED;
    if (workspace_bytes < dgx_knn_workspace_bytes(B, C, N) || !workspace) return DGX_EINVAL;
    if (B == 0) return DGX_OK;
    float* xx = static_cast<float*>(workspace);
    float* image = xx + (((size_t)B * N + 3) & ~(size_t)3);  // 16-byte aligned after xx
    const size_t ib = dgx_knn_image_bytes(B, C, N);
    int rc = dgx_knn_prepare_f32(x, sB, sC, sN, B, C, N, order, xx, image, ib, stream);
    if (rc != DGX_OK) return rc;
    return dgx_knn_select_f32(x, sB, sC, sN, xx, B, C, N, k, idx64, idx32, nullptr, image, ib, stream);
}

}  // extern "C"
