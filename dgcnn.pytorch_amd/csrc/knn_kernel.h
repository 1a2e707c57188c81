// Selection kernel of the a1 kNN (csrc/knn.hip): shared by knn.hip and the
// per-NS instantiation units knn_ns*.hip (compiled in parallel).
#pragma once
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include <type_traits>

#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Phase clock marks for tools/knn_lab.hip (compiled out of the library): wave
// lane 0 records the cycle counter at phase boundaries into DGX_KNN_LAB_BUF.
#ifdef DGX_KNN_LAB
#define KNN_MARK(i)                                                                                   \
    do {                                                                                              \
        if ((threadIdx.x & 63) == 0)                                                                  \
            DGX_KNN_LAB_BUF[((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 32 + (i)] = \
                (long long)clock64();                                                                 \
    } while (0)
#else
#define KNN_MARK(i) do { } while (0)
#endif

namespace dgx_knn {

constexpr int KT = 32;                // candidates per tile = queries per block (32x32 MFMA)
constexpr int KP = 4;                  // candidate parts = waves per block (part p: tiles p, p+KP, ...)
constexpr int KQ_THREADS = 64 * KP;
constexpr int KQ_LISTS = 2 * KP;       // top-k lists per query: 2 lane halves x KP parts

// ------------------------------------------------------------ operand image --
// MFMA operands of v_mfma_f32_32x32x2_f32 for 32-candidate tiles: step t of a
// tile covers channels 2t, 2t+1; lane l holds A[row l & 31][k l >> 5] =
// x[32 s + (l & 31)][2 t + (l >> 5)]. A cloud's image is NS = ceil(C/2) (rounded
// to 2, 4, 8, ...) steps per tile; steps are grouped in float4 chunks of 4
// (two for NS = 2) laid out [tile][chunk][lane][4], so one wave-instruction
// loads a whole chunk — 1 KiB contiguous. Zero rows pad N to a multiple of 32
// and zero channels pad C to 2 NS (exact zeros in the fmaf chain). The query
// side (B operand, B[k l >> 5][col l & 31]) of a 32-query block is the same
// tile's image. xximg holds |x_j|^2 per tile in row order: xximg[(b ntile + s) 32 + row].
inline int knn_ns(int C) { return C <= 4 ? 2 : (C <= 8 ? 4 : (C <= 16 ? 8 : (C <= 32 ? 16 : (C <= 64 ? 32 : 64)))); }
inline int knn_ntile(int N) { return (N + KT - 1) / KT; }

template <int NS>
__host__ __device__ __forceinline__ int64_t img_at(int64_t s, int l, int t) {
    if constexpr (NS == 2) return (s * 64 + l) * 2 + t;
    else return ((s * (NS / 4) + (t >> 2)) * 64 + l) * 4 + (t & 3);
}

constexpr int FIX_MAXN = 12288;  // largest N (the fix-up's tie bitmap)
constexpr int FX_CAP = 256;      // candidates above T0 ranked directly by the fix-up

// Canonical order: value descending, then index ascending.
__device__ __forceinline__ bool canon_better(float av, int aj, float bv, int bj) {
    return av > bv || (av == bv && aj < bj);
}

// row of accumulator register r in lane half hh (v_mfma 32x32 C/D layout)
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// ------------------------------------------------------------- fix-up ----
// Exact recompute of one flagged query row qf of cloud b by the whole block
// (called block-uniformly after the merge). T0 = the merged k-th value of the
// row's lists: at least k candidates reach it, so the true k-th value is >= T0.
// Every distance is recomputed by the same MFMA chain on the same operands as
// the main stream (the query's doubled operand replicated over the 32 output
// columns; wave w takes tiles w, w+4, ...), so the values are identical.
//   n_gt = #{v > T0}. If n_gt >= k the top-k is among them: rank them
//   canonically (all-pairs) when they fit FX_CAP. If n_gt < k the k-th value is
//   T0 itself: the n_gt candidates above it, then the k - n_gt smallest indices
//   with v == T0 (a bitmap of ties, scanned in index order). With more than
//   FX_CAP candidates above T0 (mass ties) the row is extracted by k rounds of a
//   canonical arg-max over re-streamed values (slow, correct).
template <int NS>
__device__ void knn_fix_row(float* fixa, const float* __restrict__ ib, const float* __restrict__ xs, int N, int k,
                            int qf, float xxq, float t0, int64_t row, int64_t* __restrict__ idx64,
                            int32_t* __restrict__ idx32, float* __restrict__ vals) {
#pragma clang fp contract(off)
    float* cv = fixa;
    int* cj = reinterpret_cast<int*>(fixa + FX_CAP);
    int* cnt = reinterpret_cast<int*>(fixa + 2 * FX_CAP);       // [0]: candidates above T0
    float* bestv = fixa + 2 * FX_CAP + 4;                        // [KP]: arg-max path per-wave values
    uint32_t* bits = reinterpret_cast<uint32_t*>(fixa + 2 * FX_CAP + 8);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5;
    const int ntile = (N + KT - 1) / KT, nw = (N + 31) >> 5;
    if (tid == 0) cnt[0] = 0;
    for (int w = tid; w < nw; w += KQ_THREADS) bits[w] = 0u;
    float bq[NS];   // the query's doubled operand in every column: B[k][*] = 2 x[qf][2t + k]
#pragma unroll
    for (int t = 0; t < NS; ++t) bq[t] = 2.0f * ib[img_at<NS>(qf >> 5, hh * 32 + (qf & 31), t)];
    __syncthreads();
    // act(v, j) on every candidate; the lanes of column 0 (lanes 0, 32) hold the tile's 32 rows
    auto stream = [&](auto&& act) __attribute__((always_inline)) {
        for (int s = wave; s < ntile; s += KP) {
            f32x16 acc = {};
#pragma unroll
            for (int t = 0; t < NS; ++t)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ib[img_at<NS>(s, lane, t)], bq[t], acc, 0, 0, 0);
            if ((lane & 31) == 0) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int j = s * KT + acc_row(r, hh);
                    if (j < N) act((acc[r] - xs[j]) - xxq, j);
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
    auto put = [&](int rank, int j, float v) __attribute__((always_inline)) {
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
            {   // lanes 0 and 32 hold the candidates
                const float ov = __shfl_xor(bv, 32);
                const int oj = __shfl_xor(bj, 32);
                if (canon_better(ov, oj, bv, bj)) { bv = ov; bj = oj; }
            }
            __syncthreads();  // previous round's picks are read
            if (lane == 0) { bestv[wave] = bv; cj[wave] = bj; }
            __syncthreads();
            pv = bestv[0];
            pj = cj[0];
#pragma unroll
            for (int w = 1; w < KP; ++w)
                if (canon_better(bestv[w], cj[w], pv, pj)) { pv = bestv[w]; pj = cj[w]; }
            if (tid == 0) put(r, pj, pv);
        }
    }
    __syncthreads();  // the fix-up area is free for the next row
}

// ------------------------------------------------------------ knn kernel ----
// Block = 32 queries (tile qb of the cloud: the B operand, doubled, in
// registers) x KP candidate parts, one wave each: wave p streams tiles p,
// p + KP, ... through a RING-slot register ring of UNIT-step operand units. A
// tile's MFMA chain gives each lane 16 candidates of its query (rows
// acc_row(r, hh)); the cloud's |x|^2 image is staged once per block in LDS.
// The only block-wide synchronisation is the final merge.
template <int NS>
struct KnnStream {
    static constexpr int UNIT = NS <= 8 ? NS : 8;          // MFMA steps per ring unit
    static constexpr int NU = NS / UNIT;                   // units per tile
    static constexpr int RING = 4;                         // ring slots: loads run RING-1 units ahead
    static constexpr int TT = RING / NU > 2 ? RING / NU : 2;   // tiles per loop trip (static slots, 2 accumulators)
    // NS = 64: the query operand (64 VGPRs) is read from LDS one unit ahead instead
    // of held in registers, which keeps the kernel within 256 VGPRs for every k
    static constexpr bool BQL = NS == 64;
};

// Per-lane list depth KL for k <= KB. A query's candidates are dealt over
// KQ_LISTS = 8 lists (2 lane halves x 4 parts, interleaved by index), so its
// true top-k splits ~Binomial(k, 1/8) over them; KL is where the chance that a
// list holds >= KL of them drops below ~5e-4 per row. Such a row (the list may
// have dropped a member) is recomputed exactly (knn_fix_row).
template <int KB>
struct KnnList {
    static constexpr int KL = KB <= 16 ? 9 : (KB <= 20 ? 10 : (KB <= 32 ? 13 : (KB <= 40 ? 15 : 20)));
};
// A lane's candidate log: compacted (to <= KL entries, the lane's own top-KL
// bounding it) whenever a chunk of candidates leaves it holding more than
// KL + KH; the KH slots of headroom make compactions rare once the lane's list
// has settled. Chunk = one unit's candidates (16 / NU), at most 8.
constexpr int KH = 8;
template <int NS>
constexpr int knn_chunk() { return 16 / KnnStream<NS>::NU > 8 ? 8 : 16 / KnnStream<NS>::NU; }
template <int NS, int KB>
constexpr int knn_qcap() { return KnnList<KB>::KL + KH + knn_chunk<NS>(); }

// LDS after [pub KP x KT | xs ntile x KT | bqs]: the final stage's small arrays
// (Tq, row flags, overflow flags, survivor counts, staged rows), then the candidate logs
// while streaming and ranking, which the fix-up's scratch aliases afterwards
// the final bound counts each list's top-(m + 2) values (8 (m + 2) > k, so the
// k-th of their union is tighter than the lists' smallest m-th value)
template <int KB>
constexpr int knn_mm() { return (KB + KQ_LISTS - 1) / KQ_LISTS + 2 < KnnList<KB>::KL ? (KB + KQ_LISTS - 1) / KQ_LISTS + 2 : KnnList<KB>::KL; }
template <int KB>
constexpr int knn_small_floats() { return 18 * KT + 4 + KT * KB + KT * KQ_LISTS * knn_mm<KB>() + KT; }
template <int NS, int KB>
constexpr int knn_f_floats() {
    constexpr int SMALL_FLOATS = knn_small_floats<KB>();
    constexpr int logs = KP * knn_qcap<NS, KB>() * 64 * 2;
    constexpr int fix = 2 * FX_CAP + 8 + FIX_MAXN / 32;
    return SMALL_FLOATS + (logs > fix ? logs : fix);
}
template <int NS, int KB>
inline size_t knn_lds_bytes(int N) {
    return ((size_t)KP * KT + (size_t)knn_ntile(N) * KT + (NS == 64 ? 64 * NS : 0) + knn_f_floats<NS, KB>()) * 4;
}

template <int NS, int KB>
__global__ __launch_bounds__(KQ_THREADS, 2)
void knn_kernel(const float* __restrict__ img, const float* __restrict__ xximg, const float* __restrict__ xx, int B,
                int N, int k, int nqb, int64_t* __restrict__ idx64, int32_t* __restrict__ idx32,
                float* __restrict__ vals) {
#pragma clang fp contract(off)
    using SP = KnnStream<NS>;
    constexpr int UNIT = SP::UNIT, NU = SP::NU, RING = SP::RING;
    constexpr bool BQL = SP::BQL;
    constexpr int QCAP = knn_qcap<NS, KB>();
    constexpr int KL = KnnList<KB>::KL;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    int b, qb;
    if (!dgx_xcd_cloud_map(blockIdx.x, B, nqb, b, qb)) return;
    KNN_MARK(0);
    const int ntile = (N + KT - 1) / KT;
    float* pub = smem;                 // [KP][KT] published admission bounds
    float* xs = smem + KP * KT;        // [ntile][KT] the cloud's |x|^2 in tile row order
    float* bqs = xs + ntile * KT;      // [NS/4][64][4] the doubled query operand (BQL only)
    float* F = bqs + (BQL ? 64 * NS : 0);
    constexpr int SMALL_FLOATS = knn_small_floats<KB>();
    float* small = F;
    float2* logs = reinterpret_cast<float2*>(F + SMALL_FLOATS);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    // wave-uniform in a scalar register: the part's tile count and every "unit
    // is live" test become scalar branches
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hh = lane >> 5;          // lane half: accumulator rows acc_row(r, hh)
    const int ql = lane & 31;          // the lane's query within the block
    const float* __restrict__ ib = img + (int64_t)b * ntile * 64 * NS;
    const float* __restrict__ xib = xximg + (int64_t)b * ntile * KT;
    const int q = qb * KT + ql;
    const int m = (k + KQ_LISTS - 1) / KQ_LISTS;   // every list's m-th value: 8 m >= k candidates reach their min

    for (int e = tid * 4; e < ntile * KT; e += KQ_THREADS * 4)
        *reinterpret_cast<float4*>(xs + e) = *reinterpret_cast<const float4*>(xib + e);
    if (tid < KP * KT) pub[tid] = -INFINITY;
    // B operand: the block's query tile, doubled — every product and partial sum
    // of the fmaf chain doubles exactly, so the MFMA returns fl(2 * dot) (dgcnn.py:7)
    float bq[BQL ? 1 : NS];
    if constexpr (NS == 2) {
        const float2 v = *reinterpret_cast<const float2*>(ib + img_at<2>(qb, lane, 0));
        bq[0] = 2.0f * v.x;
        bq[1] = 2.0f * v.y;
    } else if constexpr (BQL) {
        // the whole block shares the query tile: staged once, doubled, in LDS
        const float4* src = reinterpret_cast<const float4*>(ib + (int64_t)qb * 64 * NS);
        for (int e = tid; e < 16 * NS; e += KQ_THREADS) {
            const float4 v = src[e];
            reinterpret_cast<float4*>(bqs)[e] = make_float4(2.0f * v.x, 2.0f * v.y, 2.0f * v.z, 2.0f * v.w);
        }
    } else {
#pragma unroll
        for (int c = 0; c < NS / 4; ++c) {
            const float4 v = *reinterpret_cast<const float4*>(ib + img_at<NS>(qb, lane, 4 * c));
            bq[4 * c] = 2.0f * v.x;
            bq[4 * c + 1] = 2.0f * v.y;
            bq[4 * c + 2] = 2.0f * v.z;
            bq[4 * c + 3] = 2.0f * v.w;
        }
    }
    const float xxq = q < N ? xx[(int64_t)b * N + q] : 0.f;
    // admission seed: a lower bound of the row's k-th value in this kernel's
    // exact arithmetic (the 3-channel pre-pass below); -inf without one
    float tseed = -INFINITY;
    const int ntl = (ntile - wave + KP - 1) / KP;   // this part's tiles: wave + KP * tl
    __syncthreads();
    KNN_MARK(1);
    auto tile_xc = [&](int s, float (&xc)[16]) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 v = *reinterpret_cast<const float4*>(xs + s * KT + 8 * g + 4 * hh);
            xc[4 * g] = v.x;
            xc[4 * g + 1] = v.y;
            xc[4 * g + 2] = v.z;
            xc[4 * g + 3] = v.w;
        }
    };
    if constexpr (NS == 2) {
        // Admission pre-pass (3-channel clouds, where one tile is two MFMAs and the
        // selection VALU is the cost): each lane streams its candidates once keeping
        // only the m = ceil(k/8) best VALUES (one v_med3 per slot, no indices, no
        // FIFO). 8 lists x m candidates reach T = min over the query's 8 lists of
        // their m-th value, so T is a lower bound of the row's k-th value in this
        // kernel's own arithmetic — the main pass then admits only the few
        // candidates above it instead of inserting everything while its bound
        // climbs from -inf.
        constexpr int MM = (KB + KQ_LISTS - 1) / KQ_LISTS;
        float p[MM];
#pragma unroll
        for (int t = 0; t < MM; ++t) p[t] = -INFINITY;
        auto put = [&](float v) __attribute__((always_inline)) {
#pragma unroll
            for (int t = MM - 1; t > 0; --t) p[t] = __builtin_amdgcn_fmed3f(p[t - 1], p[t], v);
            p[0] = fmaxf(p[0], v);
        };
        constexpr int PC = 4;   // tiles per chunk: the next chunk's operands in flight
        float2 av[2][PC];
        auto fetch = [&](int buf, int tl0) __attribute__((always_inline)) {
#pragma unroll
            for (int c = 0; c < PC; ++c) {
                const int s = wave + KP * min(tl0 + c, ntl - 1);
                av[buf][c] = *reinterpret_cast<const float2*>(ib + img_at<2>(s, lane, 0));
            }
        };
        if (ntl > 0) fetch(0, 0);
#pragma unroll 1
        for (int tl0 = 0; tl0 < ntl; tl0 += 2 * PC) {
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const int base = tl0 + half * PC;
                fetch(half ^ 1, base + PC);
#pragma unroll
                for (int c = 0; c < PC; ++c) {
                    const int tl = base + c;
                    if (tl < ntl) {   // wave-uniform
                        f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[half][c].x, bq[0], f32x16{}, 0, 0, 0);
                        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[half][c].y, bq[1], acc, 0, 0, 0);
                        const int s = wave + KP * tl;
                        float xc[16];
                        tile_xc(s, xc);
                        const bool tail = (s + 1) * KT > N;
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            float v = (acc[r] - xc[r]) - xxq;
                            if (tail && s * KT + acc_row(r, hh) >= N) v = -INFINITY;
                            put(v);
                        }
                    }
                }
            }
        }
        float tm = p[0];
#pragma unroll
        for (int t = 1; t < MM; ++t) tm = (t == m - 1) ? p[t] : tm;
        tm = fminf(tm, __shfl_xor(tm, 32));
        if (hh == 0) pub[wave * KT + ql] = tm;
        __syncthreads();
        float T = pub[ql];
#pragma unroll
        for (int w = 1; w < KP; ++w) T = fminf(T, pub[w * KT + ql]);
        __syncthreads();   // every wave has read the pre-pass bounds before the main pass publishes
        if (q < N) tseed = T;
    }
    KNN_MARK(2);

    // Selection state of a lane (one of the query's 8 candidate lists: 2 lane
    // halves x KP parts). Admitted candidates are appended to the lane's LOG (LDS,
    // index order, never sorted); `tl` holds the top KL logged VALUES (one v_med3
    // per slot per entry, no index bookkeeping while streaming). Admission and
    // the log's compaction use adm = max(thr, tl[KL-1]):
    //   thr = max(seed, T), T = min over the query's 8 lists of their m-th value
    //   (m = ceil(k/8): 8 m >= k candidates reach T, a lower bound of the row's
    //   k-th value; read through `pub`, where a stale entry is still a bound);
    //   tl[KL-1]: a candidate below the lane's own KL-th value is in the top-k
    //   only if the lane holds >= KL members, and then the row is flagged at the
    //   end and recomputed (knn_fix_row).
    // At the end the survivors (>= the final T) of the 8 logs are ranked by
    // counting.
#ifdef DGX_KNN_LAB
    long long lab_flush = 0, lab_nflush = 0;   // in-stream fold/compact cycles / count
#endif
    float thr = tseed;
    float tl[KL];
#pragma unroll
    for (int t = 0; t < KL; ++t) tl[t] = -INFINITY;
    float adm = thr;  // admission threshold max(thr, tl[KL-1]); NaN once the log overflowed
    float2* fq = logs + wave * (QCAP * 64) + lane;   // this lane's log: entry e at fq[64 e]
    int cnt = 0;      // entries in the log
    int done = 0;     // entries folded into tl
    bool ovf = false; // the log could not hold the lane's candidates: the row is recomputed
    // (the round loops below stay rolled: every inlined copy of an unrolled one
    // would cost ~QCAP x KL instructions of I-cache in the stream loop)
    auto fold = [&]() __attribute__((always_inline)) {
        // rounds = the busiest lane's new entries; lanes past their count fold -inf
#pragma unroll 1
        for (int t = 0; t < QCAP; ++t) {
            if (!__any(done + t < cnt)) break;
            const float v = done + t < cnt ? fq[min(done + t, QCAP - 1) * 64].x : -INFINITY;
#pragma unroll
            for (int u = KL - 1; u > 0; --u) tl[u] = __builtin_amdgcn_fmed3f(tl[u - 1], tl[u], v);
            tl[0] = fmaxf(tl[0], v);
        }
        done = cnt;
        float tm = tl[0];
#pragma unroll
        for (int t = 1; t < KL; ++t) tm = (t == m - 1) ? tl[t] : tm;
        tm = fminf(tm, __shfl_xor(tm, 32));
        if (hh == 0) __hip_atomic_store(pub + wave * KT + ql, tm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        float T = tm;
#pragma unroll
        for (int w = 0; w < KP; ++w)
            if (w != wave)
                T = fminf(T, __hip_atomic_load(pub + w * KT + ql, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        thr = fmaxf(thr, T);
        adm = ovf ? __builtin_nanf("") : fmaxf(thr, tl[KL - 1]);   // NaN: admits nothing
    };
    auto compact = [&]() __attribute__((always_inline)) {
        // keep the entries >= adm, in order (write position <= read position)
        int w = 0;
#pragma unroll 1
        for (int t = 0; t < QCAP; ++t) {
            if (!__any(t < cnt)) break;
            const float2 e = fq[t * 64];
            fq[w * 64] = e;
            w += (t < cnt && e.x >= adm) ? 1 : 0;
        }
        cnt = w;
        done = w;
        if (cnt > KL + KH) {   // ties at the KL-th value fill the log: stop admitting, recompute the row
            ovf = true;
            adm = __builtin_nanf("");
            cnt = 0;
            done = 0;
        }
    };
    // TAIL: the cloud's last tile when N % 32 != 0 (wave-uniform), the only one
    // whose rows can be padding (j >= N)
#ifdef DGX_KNN_LAB_NOSEL
    float lab_sink = 0.f;   // lab variant: the stream alone (the sink keeps the MFMAs live)
    auto consider = [&](float dot, float xc, int j, float th, auto tail) __attribute__((always_inline)) {
        lab_sink = fmaxf(lab_sink, dot - xc);
    };
    auto consider_real = [&](float dot, float xc, int j, float th, auto tail) __attribute__((always_inline)) {
#else
    auto consider = [&](float dot, float xc, int j, float th, auto tail) __attribute__((always_inline)) {
#endif
        const float tq = dot - xc;   // dot is already 2 x (query operand doubled)
        const float v = tq - xxq;
        const bool pass = (!decltype(tail)::value || j < N) && v >= th;
        // unconditional store: a rejected candidate's slot is reused by the
        // next one (a unit adds at most 16 / NU entries to a log holding <= KL)
        fq[cnt * 64] = make_float2(v, __int_as_float(j));
        cnt += pass ? 1 : 0;
    };

    if (ntl > 0) {
        // Software pipeline over the part's tiles: the MFMA chain of tile i runs
        // into one accumulator while the candidates of tile i-1 (the other one)
        // are filtered into the FIFO in the same scheduling region, so the
        // selection VALU issues in the shadow of the dependent MFMAs. Operand
        // units stream through a RING-slot register ring, each loaded RING-1
        // units ahead; a sched_barrier keeps every load at the head of its unit
        // (the scheduler otherwise sinks the loads behind the chain, leaving no
        // distance). Every load is unconditional (past the end it re-reads this
        // part's last tile, unused), so the compiler counts the loads in flight
        // exactly. TT tiles per trip keep the ring slot and accumulator static.
        constexpr int TT = SP::TT;
        float a[RING][UNIT];
        f32x16 acc[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[1][r] = __builtin_nanf("");   // "tile -1": every compare fails
        auto load = [&](int slot, int gu, int sl) __attribute__((always_inline)) {
            const int s = wave + KP * min(gu / NU, ntl - 1);
            if constexpr (NS == 2) {
                const float2 v = *reinterpret_cast<const float2*>(ib + img_at<2>(s, lane, 0));
                a[slot][0] = v.x;
                a[slot][1] = v.y;
            } else {
#pragma unroll
                for (int c = 0; c < UNIT / 4; ++c) {
                    const float4 v = *reinterpret_cast<const float4*>(ib + img_at<NS>(s, lane, sl * UNIT + 4 * c));
                    a[slot][4 * c] = v.x;
                    a[slot][4 * c + 1] = v.y;
                    a[slot][4 * c + 2] = v.z;
                    a[slot][4 * c + 3] = v.w;
                }
            }
        };
#pragma unroll
        for (int r = 0; r < RING - 1; ++r) load(r, r, r % NU);
        float bqr[2][BQL ? UNIT : 1];   // BQL: the query operand of this unit and the next
        auto load_bq = [&](int slot, int sl) __attribute__((always_inline)) {
            if constexpr (BQL) {
#pragma unroll
                for (int c = 0; c < UNIT / 4; ++c) {
                    const float4 v = *reinterpret_cast<const float4*>(bqs + ((sl * UNIT / 4 + c) * 64 + lane) * 4);
                    bqr[slot][4 * c] = v.x;
                    bqr[slot][4 * c + 1] = v.y;
                    bqr[slot][4 * c + 2] = v.z;
                    bqr[slot][4 * c + 3] = v.w;
                }
            }
        };
        load_bq(0, 0);
        constexpr int CPN = 16 / NU;   // candidates of the previous tile filtered per unit
        constexpr int CH = knn_chunk<NS>();   // ... in chunks of CH between log checks
#pragma unroll 1
        for (int tl0 = 0; tl0 < ntl; tl0 += TT) {
#pragma unroll
            for (int t2 = 0; t2 < TT; ++t2) {
                const int i = tl0 + t2;
                const bool live = i < ntl;          // wave-uniform
                // every trip runs the same straight-line MFMA code (past the end on the
                // clamped last tile, unused): no accumulator phi copies at unit ends
                f32x16& cur = acc[t2 & 1];
                f32x16& prv = acc[(t2 & 1) ^ 1];
                const int jb = (wave + KP * (i - 1)) * KT + 4 * hh;   // previous tile's rows
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int pos = t2 * NU + u;
                    load((pos + RING - 1) % RING, i * NU + u + RING - 1, (u + RING - 1) % NU);
                    load_bq((pos + 1) & 1, (u + 1) % NU);
                    __builtin_amdgcn_sched_barrier(0);
                    // |x_j|^2 of this unit's CPN rows of the previous tile: rows
                    // acc_row(r, hh) for r in [u CPN, (u+1) CPN) come in runs of 4
                    // (2 for CPN = 2), contiguous in the tile's xs row order
                    float xcu[CPN];
                    {
                        {
                            const float* xr = xs + (wave + KP * min(max(i - 1, 0), ntl - 1)) * KT + 4 * hh;
                            if constexpr (CPN == 2) {
                                const float2 v = *reinterpret_cast<const float2*>(xr + acc_row(u * CPN, 0));
                                xcu[0] = v.x;
                                xcu[1] = v.y;
                            } else {
#pragma unroll
                                for (int g4 = 0; g4 < CPN / 4; ++g4) {
                                    const float4 v = *reinterpret_cast<const float4*>(xr + acc_row(u * CPN + 4 * g4, 0));
                                    xcu[4 * g4] = v.x;
                                    xcu[4 * g4 + 1] = v.y;
                                    xcu[4 * g4 + 2] = v.z;
                                    xcu[4 * g4 + 3] = v.w;
                                }
                            }
                        }
#pragma unroll
                        for (int t = 0; t < UNIT; ++t)
                            cur = __builtin_amdgcn_mfma_f32_32x32x2f32(a[pos % RING][t],
                                                                       BQL ? bqr[pos & 1][t] : bq[u * UNIT + t],
                                                                       t == 0 && u == 0 ? f32x16{} : cur, 0, 0, 0);
                        // branch-free for i = 0 too (the NaN-filled accumulator admits
                        // nothing) and past the part's end (a NaN bound admits nothing,
                        // not even a +inf value)
                        const float adm_live = live ? adm : __builtin_nanf("");
#pragma unroll
                        for (int c = 0; c < CH; ++c) {
                            const int r = u * CPN + c;
                            consider(prv[r], xcu[c], jb + acc_row(r, 0), adm_live, std::false_type{});
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    // the log holds <= KL + KH + CH entries after a chunk: compact it
                    // when it has no room for the next one
                    auto check = [&]() __attribute__((always_inline)) {
                        if (__any(cnt > KL + KH)) {
#ifdef DGX_KNN_LAB
                            const long long f0 = clock64();
#endif
                            fold();
                            compact();
#ifdef DGX_KNN_LAB
                            lab_flush += clock64() - f0;
                            ++lab_nflush;
#endif
                        }
                    };
                    check();
                    // the unit's further chunks (16-candidate units: NU = 1)
#pragma unroll
                    for (int ch = 1; ch < CPN / CH; ++ch) {
                        const float adm_live = live ? adm : __builtin_nanf("");
#pragma unroll
                        for (int c = 0; c < CH; ++c) {
                            const int r = u * CPN + ch * CH + c;
                            consider(prv[r], xcu[ch * CH + c], jb + acc_row(r, 0), adm_live, std::false_type{});
                        }
                        check();
                    }
                }
                // fold the previous tile's admissions: publish the bound early
                if (live && i > 0 && __any(cnt > done)) fold();
            }
        }
        // the part's last tile: the only one that can hold padding rows (j >= N)
        {
            const int s = wave + KP * (ntl - 1);
            const f32x16 last = ((ntl - 1) & 1) ? acc[1] : acc[0];
            float xc[16];
            tile_xc(s, xc);
            const int jb = s * KT + 4 * hh;
            auto tile16 = [&](auto tail) __attribute__((always_inline)) {
                // in chunks of CH candidates, the log compacted between them as in the stream
#pragma unroll
                for (int u = 0; u < 16 / CH; ++u) {
#pragma unroll
                    for (int c = 0; c < CH; ++c) {
                        const int r = u * CH + c;
                        consider(last[r], xc[r], jb + acc_row(r, 0), adm, tail);
                    }
                    if (u + 1 < 16 / CH && __any(cnt > KL + KH)) {
                        fold();
                        compact();
                    }
                }
            };
            if ((s + 1) * KT > N) tile16(std::true_type{});
            else tile16(std::false_type{});
        }
    }
#ifdef DGX_KNN_LAB
#ifdef DGX_KNN_LAB_NOSEL
    if (lab_sink == 12345.f) DGX_KNN_LAB_BUF[0] = 1;
#endif
    if ((threadIdx.x & 63) == 0) {
        DGX_KNN_LAB_BUF[((int64_t)blockIdx.x * KP + wave) * 32 + 24] = lab_flush;
        DGX_KNN_LAB_BUF[((int64_t)blockIdx.x * KP + wave) * 32 + 25] = lab_nflush;
    }
#endif
    KNN_MARK(3);
    if (__any(cnt > done)) fold();
    KNN_MARK(4);

    // Final threshold of the row. Every list published its final m-th value, so
    // min over the 8 lists (and the seed) bounds the row's k-th value from below;
    // tighter: the k-th largest of the 8 lists' top-m2 values (m2 = min(m + 2, KL):
    // 8 m2 > k distinct candidates), counted by the octet of lanes of the query
    // (tid = 8 query + list). Tq = the larger of the two. Every top-k member of a list that is
    // not flagged below is in its log and >= Tq. Each lane then keeps its
    // survivors (v >= Tq) in place as 64-bit canonical keys: (order-preserving
    // bits of v) << 32 | ~j, so "canonically better" (value desc, index asc) is
    // one unsigned compare; the octet ranks list g's survivors against all 8
    // lists by counting: rank r < k is row slot r, staged in LDS.
    float* kth = small;                                        // [KT] the row's Tq
    int* flg = reinterpret_cast<int*>(small + KT);             // [KP] per wave: flagged rows of its 8 queries
    int* scnt = reinterpret_cast<int*>(small + 2 * KT + 4);    // [KT][8] survivors per list
    float* klv = small + 10 * KT + 4;                          // [KT][8] each list's KL-th value
    int* ostage = reinterpret_cast<int*>(small + 18 * KT + 4); // [KT][KB] the rows' indices by rank
    constexpr int MM = knn_mm<KB>();
    float* tlq = small + 18 * KT + 4 + KT * KB;                // [KT][8][MM] each list's top-MM values
    float* t2q = tlq + KT * KQ_LISTS * MM;                     // [KT] k-th of the lists' top-m values
    {
        float* d = tlq + (ql * KQ_LISTS + wave * 2 + hh) * MM;
#pragma unroll
        for (int t = 0; t < MM; ++t) d[t] = tl[t];
    }
    KNN_MARK(5);
    __syncthreads();   // every list's final m-th value and top-MM values are published
    KNN_MARK(6);
    const int qm = tid >> 3, g = tid & 7;                      // octet role: query qm, list g
    {
        // count, for each of list g's top-m values, the values >= it over the 8
        // lists' top-m; the largest one reaching k is a valid bound
        const float* tq = tlq + qm * KQ_LISTS * MM;
        const int m2 = min(m + 2, KL);
        float mine[MM];
#pragma unroll
        for (int t = 0; t < MM; ++t) mine[t] = tq[g * MM + t];
        int cnt_ge[MM];
#pragma unroll
        for (int t = 0; t < MM; ++t) cnt_ge[t] = 0;
#pragma unroll
        for (int l = 0; l < KQ_LISTS; ++l) {
#pragma unroll
            for (int u = 0; u < MM; ++u) {
                const float o = u < m2 ? tq[l * MM + u] : -INFINITY;
#pragma unroll
                for (int t = 0; t < MM; ++t) cnt_ge[t] += o >= mine[t] ? 1 : 0;
            }
        }
        float best = -INFINITY;
#pragma unroll
        for (int t = 0; t < MM; ++t)
            if (t < m2 && cnt_ge[t] >= k) best = fmaxf(best, mine[t]);
        best = fmaxf(best, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(best), 0xB1, 0xf, 0xf, false)));
        best = fmaxf(best, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(best), 0x4E, 0xf, 0xf, false)));
        best = fmaxf(best, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(best), 0x141, 0xf, 0xf, false)));
        if (g == 0) t2q[qm] = best;
    }
    KNN_MARK(7);
    __syncthreads();
    KNN_MARK(8);
    {
        float Tq = pub[ql];
#pragma unroll
        for (int w = 1; w < KP; ++w) Tq = fminf(Tq, pub[w * KT + ql]);
        Tq = fmaxf(fmaxf(Tq, tseed), t2q[ql]);
        uint64_t* fk = reinterpret_cast<uint64_t*>(fq);
        int sc = 0;
#pragma unroll 1
        for (int t = 0; t < QCAP; ++t) {
            if (!__any(t < cnt)) break;
            const float2 e = fq[t * 64];
            const float v = e.x + 0.0f;   // -0 -> +0: keys order like the float compare
            const uint32_t u = __float_as_uint(v);
            const uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
            fk[sc * 64] = ((uint64_t)ord << 32) | (uint32_t)~__float_as_uint(e.y);
            sc += (t < cnt && e.x >= Tq) ? 1 : 0;
        }
        const int li = ql * KQ_LISTS + wave * 2 + hh;
        scnt[li] = sc;
        klv[li] = ovf ? INFINITY : tl[KL - 1];   // an overflowed list flags its row below
        if (wave == 0 && hh == 0) kth[ql] = Tq;
    }
    KNN_MARK(9);
    __syncthreads();
    KNN_MARK(10);
    {
        const uint64_t* lg = reinterpret_cast<const uint64_t*>(logs);
        auto col = [&](int l) __attribute__((always_inline)) {   // list l of query qm
            return lg + (l >> 1) * (QCAP * 64) + (l & 1) * 32 + qm;
        };
        int sl[KQ_LISTS];
        int c = 0, ns = 0;
#pragma unroll
        for (int l = 0; l < KQ_LISTS; ++l) {
            sl[l] = scnt[qm * KQ_LISTS + l];
            c += sl[l];
            ns = l == g ? sl[l] : ns;
        }
        const int qr = qb * KT + qm;
#ifdef DGX_KNN_LAB
        {   // survivors per row (c, counted by octet leaders) and per list (ns), summed over the wave
            int sc_ = (g == 0 && qr < N) ? c : 0, sn_ = qr < N ? ns : 0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                sc_ += __shfl_xor(sc_, o);
                sn_ += __shfl_xor(sn_, o);
            }
            if (lane == 0) {
                DGX_KNN_LAB_BUF[((int64_t)blockIdx.x * KP + wave) * 32 + 26] = sc_;
                DGX_KNN_LAB_BUF[((int64_t)blockIdx.x * KP + wave) * 32 + 27] = sn_;
            }
        }
#endif
        // the k-th value of the row (rank k - 1), for the flag test below
        uint64_t kkey = 0ull;
        if (qr < N && c >= k) {
            // EPL own survivors per sweep against every survivor of the row, two
            // independent LDS reads per trip (padding keys 0 are never better)
            constexpr int EPL = 4;
            const uint64_t* mine = col(g);
            for (int i0 = 0; i0 < ns; i0 += EPL) {
                uint64_t key[EPL];
                int rk[EPL];
#pragma unroll
                for (int i = 0; i < EPL; ++i) {
                    key[i] = i0 + i < ns ? mine[(i0 + i) * 64] : ~0ull;
                    rk[i] = 0;
                }
#pragma unroll
                for (int l = 0; l < KQ_LISTS; ++l) {
                    const uint64_t* o = col(l);
                    for (int u = 0; u < sl[l]; u += 2) {
                        const uint64_t o0 = o[u * 64];
                        const uint64_t o1 = u + 1 < sl[l] ? o[(u + 1) * 64] : 0ull;
#pragma unroll
                        for (int i = 0; i < EPL; ++i) rk[i] += (o0 > key[i] ? 1 : 0) + (o1 > key[i] ? 1 : 0);
                    }
                }
#pragma unroll
                for (int i = 0; i < EPL; ++i) {
                    if (i0 + i < ns && rk[i] < k) {
                        ostage[qm * KB + rk[i]] = (int)~(uint32_t)key[i];
                        if (vals) {
                            const uint32_t ord = (uint32_t)(key[i] >> 32);
                            vals[((int64_t)b * N + qr) * k + rk[i]] =
                                __uint_as_float((ord & 0x80000000u) ? (ord & 0x7fffffffu) : ~ord);
                        }
                    }
                    if (i0 + i < ns && rk[i] == k - 1) kkey = key[i];
                }
            }
        }
        KNN_MARK(11);
        // octet max: every lane gets the k-th key (0 when the row has < k survivors)
        auto omax = [&](uint64_t v, auto ctrl) __attribute__((always_inline)) {
            constexpr int C = decltype(ctrl)::value;
            const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, C, 0xf, 0xf, false);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), C, 0xf, 0xf, false);
            const uint64_t o = ((uint64_t)hi << 32) | lo;
            return o > v ? o : v;
        };
        kkey = omax(kkey, std::integral_constant<int, 0xB1>{});    // quad_perm [1,0,3,2]: lane ^ 1
        kkey = omax(kkey, std::integral_constant<int, 0x4E>{});    // quad_perm [2,3,0,1]: lane ^ 2
        kkey = omax(kkey, std::integral_constant<int, 0x141>{});   // row_half_mirror: the other quad
        // A list whose KL-th value reaches the row's k-th value may have dropped a
        // member (it admitted and kept only values >= its KL-th): the row goes to
        // the exact fix-up, as does a row with fewer than k survivors.
        const uint32_t kord = (uint32_t)(kkey >> 32);
        const float kv = __uint_as_float((kord & 0x80000000u) ? (kord & 0x7fffffffu) : ~kord);
        const float lk = klv[qm * KQ_LISTS + g];
        const bool mine_bad = c < k || (lk != -INFINITY && lk >= kv);
        {   // the wave's 8 row flags (octet o = lanes 8o..8o+7) as one byte
            const uint64_t bm = __ballot(mine_bad && qr < N);
            uint32_t m8 = 0;
#pragma unroll
            for (int o = 0; o < 8; ++o) m8 |= ((bm >> (8 * o)) & 0xffull) != 0 ? (1u << o) : 0u;
            if (lane == 0) flg[wave] = (int)m8;
        }
    }
    KNN_MARK(12);
    __syncthreads();
    KNN_MARK(13);
    {   // the block's rows are consecutive in the output: 32 k entries, written
        // coalesced (flagged rows are left to the fix-up)
        uint32_t fm = 0;
#pragma unroll
        for (int w = 0; w < KP; ++w) fm |= (uint32_t)flg[w] << (8 * w);
        const int nrow = min(KT, N - qb * KT);
        const int64_t base = ((int64_t)b * N + qb * KT) * k;
        for (int e = tid; e < nrow * k; e += KQ_THREADS) {
            const int r = e / k, s2 = e - r * k;
            if ((fm >> r) & 1u) continue;
            const int j = ostage[r * KB + s2];
            if (idx64) idx64[base + e] = j;
            if (idx32) idx32[base + e] = j;
        }
    }
    KNN_MARK(14);
    // the block's flagged rows (rare), one at a time; flg / kth are block-uniform LDS reads
    float* fixa = F + SMALL_FLOATS;   // aliases the logs, done with
#ifdef DGX_KNN_LAB
    int nfix = 0;
#endif
    uint32_t fmask = 0;   // block-uniform: the flagged rows of the block
#pragma unroll
    for (int w = 0; w < KP; ++w) fmask |= (uint32_t)flg[w] << (8 * w);
    fmask = __builtin_amdgcn_readfirstlane(fmask);
    while (fmask != 0u) {
        const int f = __ffs(fmask) - 1;
        fmask &= fmask - 1u;
        const int qf = qb * KT + f;
        knn_fix_row<NS>(fixa, ib, xs, N, k, qf, xx[(int64_t)b * N + qf], kth[f], (int64_t)b * N + qf, idx64, idx32,
                        vals);
#ifdef DGX_KNN_LAB
        ++nfix;
#endif
    }
    KNN_MARK(15);
#ifdef DGX_KNN_LAB
    if ((threadIdx.x & 63) == 0) DGX_KNN_LAB_BUF[((int64_t)blockIdx.x * KP + wave) * 32 + 28] = nfix;
#endif
}

template <int NS, int KB>
int launch_knn(const float* xx, int B, int N, int k, int64_t* idx64, int32_t* idx32, float* vals, const float* img,
               const float* xximg, hipStream_t st) {
    const int nqb = knn_ntile(N);
    hipLaunchKernelGGL((knn_kernel<NS, KB>), dim3(dgx_xcd_cloud_grid(B, nqb)), dim3(KQ_THREADS),
                       (knn_lds_bytes<NS, KB>(N)), st, img, xximg, xx, B, N, k, nqb, idx64, idx32, vals);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

template <int NS>
int dispatch_k(const float* xx, int B, int N, int k, int64_t* idx64, int32_t* idx32, float* vals, const float* img,
               const float* xximg, hipStream_t st) {
#define DGX_KNN_K(KBV) return launch_knn<NS, KBV>(xx, B, N, k, idx64, idx32, vals, img, xximg, st)
    if (k <= 16) DGX_KNN_K(16);
    if (k <= 20) DGX_KNN_K(20);
    if (k <= 32) DGX_KNN_K(32);
    if (k <= 40) DGX_KNN_K(40);
    DGX_KNN_K(64);
#undef DGX_KNN_K
}

}  // namespace dgx_knn
