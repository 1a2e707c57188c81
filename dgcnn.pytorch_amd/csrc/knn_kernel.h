// Selection kernel of the a1 kNN (csrc/knn.hip): shared by knn.hip and the
// per-NS instantiation units knn_ns*.hip (compiled in parallel).
#pragma once
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include <type_traits>

#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace dgx_knn {

constexpr int KT = 32;                 // candidates per tile = queries per block (32x32 MFMA)
constexpr int KP = 4;                  // candidate parts = waves per block (part p: tiles p, p+KP, ...)
constexpr int KQ_THREADS = 64 * KP;
constexpr int KQ_LISTS = 2 * KP;       // top-k lists per query: 2 lane halves x KP parts
constexpr int KQ_QCAP = 16;            // per-lane pending-candidate FIFO (a half tile adds <= 8)

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
// KQ_LISTS = 8 lists (2 lane halves x 4 parts, interleaved by index), so the
// true top-k splits ~Binomial(k, 1/8) over its lists; KL is where that
// distribution's upper tail drops to ~2e-6 per list. A lane needing more than
// KL slots flags its row, which is recomputed exactly (knn_fix_row).
template <int KB>
struct KnnList {
    static constexpr int KL = KB <= 16 ? 10 : (KB <= 20 ? 12 : (KB <= 32 ? 15 : (KB <= 40 ? 17 : 23)));
    static constexpr int RPL = (KB + 1) / 2;   // ranks per lane of a wave's 2-list merge
};

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
    auto stream = [&](auto&& act) {
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
    static constexpr int UNIT = NS <= 8 ? NS : (NS == 64 ? 16 : 8);   // MFMA steps per ring unit
    static constexpr int NU = NS / UNIT;                               // units per tile
    static constexpr int RING = NS == 64 ? 2 : 4;                      // units in flight
    static constexpr int UB = RING > NU ? RING : NU;                   // units per loop trip (static slots)
    static_assert(UB % RING == 0 && UB % NU == 0, "unit split");
};

// LDS after [pub KP x KT | xs ntile x KT]: the FIFO while streaming, then the
// merge lists, k-th values, flags and the fix-up's scratch
template <int KB>
constexpr int knn_f_floats() {
    constexpr int fifo = KP * KQ_QCAP * 64 * 2;
    constexpr int fix = KP * KT * KB * 2 + 2 * KT + 2 * FX_CAP + 8 + FIX_MAXN / 32;
    return fifo > fix ? fifo : fix;
}
template <int KB>
inline size_t knn_lds_bytes(int N) { return ((size_t)KP * KT + (size_t)knn_ntile(N) * KT + knn_f_floats<KB>()) * 4; }

template <int NS, int KB>
__global__ __launch_bounds__(KQ_THREADS, 2)
void knn_kernel(const float* __restrict__ img, const float* __restrict__ xximg, const float* __restrict__ xx, int B,
                int N, int k, int nqb, int64_t* __restrict__ idx64, int32_t* __restrict__ idx32,
                float* __restrict__ vals) {
#pragma clang fp contract(off)
    constexpr int KL = KnnList<KB>::KL;
    constexpr int RPL = KnnList<KB>::RPL;
    using SP = KnnStream<NS>;
    constexpr int UNIT = SP::UNIT, NU = SP::NU, RING = SP::RING, UB = SP::UB;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    int b, qb;
    if (!dgx_xcd_cloud_map(blockIdx.x, B, nqb, b, qb)) return;
    const int ntile = (N + KT - 1) / KT;
    float* pub = smem;                 // [KP][KT] published admission bounds
    float* xs = smem + KP * KT;        // [ntile][KT] the cloud's |x|^2 in tile row order
    float* F = xs + ntile * KT;
    float2* fifo = reinterpret_cast<float2*>(F);
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
    const int m2 = (k + 1) / 2;                    // the wave's two lists' m2-th: 2 m2 >= k

    for (int e = tid * 4; e < ntile * KT; e += KQ_THREADS * 4)
        *reinterpret_cast<float4*>(xs + e) = *reinterpret_cast<const float4*>(xib + e);
    if (tid < KP * KT) pub[tid] = -INFINITY;
    // B operand: the block's query tile, doubled — every product and partial sum
    // of the fmaf chain doubles exactly, so the MFMA returns fl(2 * dot) (dgcnn.py:7)
    float bq[NS];
    if constexpr (NS == 2) {
        const float2 v = *reinterpret_cast<const float2*>(ib + img_at<2>(qb, lane, 0));
        bq[0] = 2.0f * v.x;
        bq[1] = 2.0f * v.y;
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
        auto put = [&](float v) {
#pragma unroll
            for (int t = MM - 1; t > 0; --t) p[t] = __builtin_amdgcn_fmed3f(p[t - 1], p[t], v);
            p[0] = fmaxf(p[0], v);
        };
        constexpr int PC = 4;   // tiles per chunk: the next chunk's operands in flight
        float2 av[2][PC];
        auto fetch = [&](int buf, int tl0) {
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

    // Each lane keeps the KL best of ITS candidates (sorted, registers, static
    // indexing). Admission filter thr = max(own KL-th, t2, T, seed): t2 = the
    // wave's two lists' min m2-th value (2 m2 >= k candidates reach it), T = the
    // query's 8 lists' min m-th value (the other parts' through `pub`, a value
    // published at their last flush: lists only improve, so a stale value is
    // still a lower bound). '>=' keeps equal values; their order is settled
    // canonically at the merge. Candidates that pass wait in the lane's FIFO
    // and are inserted in batches, so an insertion round (5*KL VALU ops for the
    // whole wave) is paid once per admitted candidate of the busiest lane.
    float thr = tseed;
    float lv[KL];
    int li[KL];
#pragma unroll
    for (int t = 0; t < KL; ++t) { lv[t] = -INFINITY; li[t] = 0x7fffffff; }
    float2* fq = fifo + wave * (KQ_QCAP * 64) + lane;
    int cnt = 0;
    auto flush = [&]() {
        // branch-free rounds: slots past a lane's count read stale entries and
        // are replaced by -inf, so every round is the same straight-line code
        float2 c0 = fq[0];
        float cv = cnt > 0 ? c0.x : -INFINITY;
        int cj = __float_as_int(c0.y);
        // fully unrolled with an early exit: no loop-carried copies of the list
#pragma unroll
        for (int t = 0; t < KQ_QCAP; ++t) {
            if (!__any(t < cnt)) break;
            const int nx = min(t + 1, KQ_QCAP - 1);
            const float2 n0 = fq[nx * 64];
            const float nv = t + 1 < cnt ? n0.x : -INFINITY;
            const int nj = __float_as_int(n0.y);
            list_insert_ordered<KL>(lv, li, cv >= thr ? cv : -INFINITY, cj);
            cv = nv;
            cj = nj;
        }
        cnt = 0;
        float tm = lv[0], t2 = lv[0];
#pragma unroll
        for (int t = 1; t < KL; ++t) {
            tm = (t == m - 1) ? lv[t] : tm;
            t2 = (t == m2 - 1) ? lv[t] : t2;
        }
        if (m2 > KL) t2 = -INFINITY;   // the two lists cannot certify k candidates
        tm = fminf(tm, __shfl_xor(tm, 32));
        t2 = fminf(t2, __shfl_xor(t2, 32));
        if (hh == 0) __hip_atomic_store(pub + wave * KT + ql, tm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        float T = tm;
#pragma unroll
        for (int w = 0; w < KP; ++w)
            if (w != wave)
                T = fminf(T, __hip_atomic_load(pub + w * KT + ql, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        thr = fmaxf(fmaxf(fmaxf(t2, T), lv[KL - 1]), tseed);
    };
    // TAIL: the cloud's last tile when N % 32 != 0 (wave-uniform), the only one
    // whose rows can be padding (j >= N)
    auto consider = [&](float dot, float xc, int j, auto tail) {
        const float tq = dot - xc;   // dot is already 2 x (query operand doubled)
        const float v = tq - xxq;
        const bool pass = (!decltype(tail)::value || j < N) && v >= thr;
        // unconditional store: a rejected candidate's slot is reused by the
        // next one (a half tile adds at most 8 entries to a FIFO holding <= QCAP-8)
        fq[cnt * 64] = make_float2(v, __int_as_float(j));
        cnt += pass ? 1 : 0;
    };

    if (ntl > 0) {
        // Every load is unconditional (a unit past the end re-reads this part's
        // last tile, unused): with a data-dependent skip the compiler cannot count
        // the loads in flight and drains them all (vmcnt(0)) every trip.
        float a[RING][UNIT];
        auto load = [&](int slot, int u, int sl) {
            const int s = wave + KP * min(u / NU, ntl - 1);
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
        const int nunits = ntl * NU;
#pragma unroll
        for (int r = 0; r < RING; ++r) load(r, r, r % NU);
        f32x16 acc = {};
#pragma unroll 1
        for (int u = 0; u < nunits; u += UB) {
#pragma unroll
            for (int ub = 0; ub < UB; ++ub) {
                const int slot = ub % RING, sl = ub % NU;
                const bool live = UB == NU || u + ub < nunits;   // wave-uniform
                if (live) {
                    if (sl == 0) acc = f32x16{};
#pragma unroll
                    for (int t = 0; t < UNIT; ++t)
                        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[slot][t], bq[sl * UNIT + t], acc, 0, 0, 0);
                }
                load(slot, u + ub + RING, (ub + RING) % NU);
                if (live && sl == NU - 1) {
                    const int s = wave + KP * ((u + ub) / NU);
                    float xc[16];
                    tile_xc(s, xc);
                    const int jb = s * KT + 4 * hh;
                    auto half = [&](int r0, auto tail) {
#pragma unroll
                        for (int r = r0; r < r0 + 8; ++r) consider(acc[r], xc[r], jb + acc_row(r, 0), tail);
                        if (__any(cnt > KQ_QCAP - 8)) flush();
                    };
                    if ((s + 1) * KT > N) {
                        half(0, std::true_type{});
                        half(8, std::true_type{});
                    } else {
                        half(0, std::false_type{});
                        half(8, std::false_type{});
                    }
                }
            }
        }
    }
    flush();

    // Merge the wave's 2 lists of each query (lanes ql, ql + 32) by k rounds of a
    // canonical arg-max over the 2 list heads; the winning lane pops its head.
    // Rank r ends up in lane half r % 2.
    const float last = lv[KL - 1];
    float ov[RPL];
    int oj[RPL];
#pragma unroll
    for (int t = 0; t < RPL; ++t) { ov[t] = -INFINITY; oj[t] = 0x7fffffff; }
#pragma unroll
    for (int r = 0; r < KB; ++r) {
        if (r < k) {
            float hv = lv[0];
            int hj = li[0];
            const float pv = __shfl_xor(hv, 32);
            const int pj = __shfl_xor(hj, 32);
            if (canon_better(pv, pj, hv, hj)) { hv = pv; hj = pj; }
            const bool pop = li[0] == hj && lv[0] == hv;
#pragma unroll
            for (int t = 0; t < KL - 1; ++t) {
                lv[t] = pop ? lv[t + 1] : lv[t];
                li[t] = pop ? li[t + 1] : li[t];
            }
            lv[KL - 1] = pop ? -INFINITY : lv[KL - 1];
            li[KL - 1] = pop ? 0x7fffffff : li[KL - 1];
            if ((r & 1) == hh) { ov[r >> 1] = hv; oj[r >> 1] = hj; }
        }
    }

    // Merge the parts: each part's sorted top-k goes to LDS; an element's final
    // rank is its rank in its own list plus, for every other part, the number of
    // that part's elements that are canonically better (binary search). The
    // parts hold disjoint candidates, so the ranks 0..k-1 are taken exactly once.
    __syncthreads();  // every wave is done with its FIFO
    float2* lists = reinterpret_cast<float2*>(F);    // [KP][KT][KB]
    float* kth = F + KP * KT * KB * 2;               // [KT] merged k-th value
    int* flg = reinterpret_cast<int*>(kth + KT);     // [KT] row needs the fix-up
#pragma unroll
    for (int t = 0; t < RPL; ++t) {
        const int r = 2 * t + hh;
        if (r < k) lists[(wave * KT + ql) * KB + r] = make_float2(ov[t], __int_as_float(oj[t]));
    }
    if (tid < KT) {
        kth[tid] = -INFINITY;
        flg[tid] = 0;
    }
    __syncthreads();
    int rk[RPL];
#pragma unroll
    for (int t = 0; t < RPL; ++t) {
        const int r = 2 * t + hh;
        rk[t] = k;
        if (r < k) {
            int tot = r;
#pragma unroll
            for (int w = 0; w < KP; ++w) {
                if (w == wave) continue;
                const float2* other = lists + (w * KT + ql) * KB;
                int lo = 0, hi = k;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    const float2 o = other[mid];
                    if (canon_better(o.x, __float_as_int(o.y), ov[t], oj[t])) lo = mid + 1;
                    else hi = mid;
                }
                tot += lo;
            }
            rk[t] = tot;
            if (tot == k - 1) kth[ql] = ov[t];
        }
    }
    __syncthreads();
    {
        // A lane whose list was full and whose last kept value reaches the merged
        // k-th may have dropped a member of the true top-k: mark the row for the
        // exact fix-up pass. Fewer than k candidates reaching the seed (the merged
        // k-th is then a -inf pad) marks it too.
        const float kv = kth[ql];
        if (last != -INFINITY && last >= kv) flg[ql] = 1;
        if (!(kv >= tseed)) flg[ql] = 1;
    }
    __syncthreads();
    if (q < N && flg[ql] == 0) {  // flagged rows are written by the fix-up below
        const int64_t row = ((int64_t)b * N + q) * k;
#pragma unroll
        for (int t = 0; t < RPL; ++t) {
            const int r = rk[t];
            if (r < k) {
                if (idx64) idx64[row + r] = oj[t];
                if (idx32) idx32[row + r] = oj[t];
                if (vals) vals[row + r] = ov[t];
            }
        }
    }
    // the block's flagged rows (rare), one at a time; flg / kth are block-uniform LDS reads
    float* fixa = F + KP * KT * KB * 2 + 2 * KT;
    for (int f = 0; f < KT; ++f) {
        const int qf = qb * KT + f;
        if (flg[f] != 0 && qf < N)
            knn_fix_row<NS>(fixa, ib, xs, N, k, qf, xx[(int64_t)b * N + qf], kth[f], (int64_t)b * N + qf, idx64,
                            idx32, vals);
    }
}

template <int NS, int KB>
int launch_knn(const float* xx, int B, int N, int k, int64_t* idx64, int32_t* idx32, float* vals, const float* img,
               const float* xximg, hipStream_t st) {
    const int nqb = knn_ntile(N);
    hipLaunchKernelGGL((knn_kernel<NS, KB>), dim3(dgx_xcd_cloud_grid(B, nqb)), dim3(KQ_THREADS),
                       knn_lds_bytes<KB>(N), st, img, xximg, xx, B, N, k, nqb, idx64, idx32, vals);
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
