// a1 — kNN of coordinate clouds (C <= 3: the xyz kNN of DGCNN's first block,
// PositionEmbedding and compute_hog_1x1; reference models/dgcnn.py:6-12,
// models/layers.py:45, models/model_partseg.py:26) on a uniform cell grid.
//
// The dense selection (knn.hip) streams all N candidates past every query;
// at N = 1024, k = 20 a query's 20 nearest points lie within ~1.3 cells of a
// grid holding ~2 points per cell, so one launch here:
//   build    every workgroup sorts its cloud into a cell grid in LDS (bounding
//            box -> grid -> per-wave cell histograms -> a stable, deterministic
//            counting sort: identical arrays in every workgroup of the cloud);
//            sorted points carry (x0, x1, x2, |x|^2) and ~(original index).
//   queries  64 queries per workgroup, consecutive in cell order (so a wave's
//            queries are neighbours), 4 lanes per query. A values-only pre-pass
//            over the 3x3x3 cells around the query gives T, a lower bound of the
//            query's k-th value; the main pass streams the 5x5x5 cells, admitting
//            candidates at or above the bound into per-lane sorted lists of
//            64-bit keys (value-major, index-minor: canonical order by
//            construction, no tie cases), then one lane per query merges the 4
//            lists.
//   exact    a query is finished only if its k-th value exceeds every value a
//            point outside the visited cells can have (the distance from the
//            query to the visited box, minus rounding margins); otherwise — or if
//            a lane's list may have dropped a top-k member — the whole wave
//            recomputes that query over all N points from the k-th value found
//            (a lower bound of the true one). The output never depends on the
//            grid: it is the canonical top-k of the reference's values.
// Values are the reference's arithmetic bit for bit:
//   dot = fmaf(x2, 2q2, fmaf(x1, 2q1, x0 * 2q0))   (the MFMA chain of knn.hip,
//         doubled query: exact), v = (dot - |x_j|^2) - |x_q|^2,
//   |x|^2 = (x0^2 + x1^2) + x2^2 — for C <= 3 torch's strided cascade and its
//         vectorised row sum both reduce to this order (knn.hip sqnorm_sum).
#include <math.h>
#include <stdint.h>

#include "common.h"

namespace {

constexpr int KG_THREADS = 256;
constexpr int KG_LPQ = 4;                        // lanes per query
constexpr int KG_QPW = DGX_WAVE / KG_LPQ;        // 16 queries per wave
constexpr int KG_QPB = KG_THREADS / KG_LPQ;      // 64 queries per workgroup
constexpr int KG_WAVES = KG_THREADS / DGX_WAVE;
constexpr int KG_MAXN = 4096;                    // LDS: 20 B per point
constexpr int KG_QCAP = 8;                       // per-lane admitted-candidate FIFO
constexpr int KG_FXCAP = 256;                    // keys ranked directly by the exact fix

// larger key = better: value-major (sortable float bits), then smaller index
__device__ __forceinline__ uint32_t kg_fkey(float v) {
    v = v + 0.0f;   // -0 -> +0: equal values must have equal keys
    const uint32_t u = __float_as_uint(v);
    return u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
}
__device__ __forceinline__ float kg_keyf(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}
__device__ __forceinline__ uint64_t kg_key(float v, uint32_t nid) { return ((uint64_t)kg_fkey(v) << 32) | nid; }

// per-lane list length: a query's candidates are dealt over 4 lanes, each keeps
// KL >= ceil(KB/4) of its best; a lane holding more than KL of the final top-k
// is detected after the merge and the query recomputed exactly
template <int KB>
struct KgList {
    static constexpr int M = (KB + KG_LPQ - 1) / KG_LPQ;   // 4 M >= k: min over lanes of M-th bounds the k-th
    static constexpr int KL = KB <= 8 ? KB : (KB <= 16 ? 12 : (KB <= 20 ? 14 : (KB <= 32 ? 18 : (KB <= 40 ? 22 : 30))));
};

// geometry of one cloud's grid (identical in every thread: same inputs, same arithmetic)
struct KgGrid {
    float lo[3], inv[3], h[3];
    int G[3];
    int nc;
};

__device__ __forceinline__ int kg_cell_axis(const KgGrid& g, int a, float x) {
    const int c = (int)((x - g.lo[a]) * g.inv[a]);   // NaN / negative -> clamped below
    return min(g.G[a] - 1, max(0, c));
}

// scratch layout (bytes) of one workgroup for N points, cell cap NCMAX, list length KL
struct KgLds {
    size_t pts, nid, cst, scr, total;
};
__host__ __device__ inline KgLds kg_lds(int N, int ncmax, int KL) {
    KgLds l;
    l.pts = 0;
    l.nid = l.pts + (size_t)N * 16;
    l.cst = l.nid + (size_t)N * 4;
    l.scr = l.cst + (((size_t)(ncmax + 1) * 4 + 15) & ~(size_t)15);
    size_t hist = (size_t)KG_WAVES * ncmax * 4;
    size_t fifo = (size_t)KG_QCAP * KG_THREADS * 8;
    size_t lists = (size_t)KG_THREADS * KL * 8;
    size_t s = hist > fifo ? hist : fifo;
    if (lists > s) s = lists;
    l.total = l.scr + s + 128;   // + 32 reduction words
    return l;
}

// cells per cloud: ~PPC points per cell, PPC = max(2, k/10) (the 5x5x5 box then
// covers the k-th neighbour of a uniform cloud; measured in a simulation of the
// kernel's visiting order: 2 % of queries need the exact fix at k 20)
__host__ __device__ inline int kg_cells_target(int N, int k) {
    const float ppc = fmaxf(2.0f, (float)k / 10.0f);
    return max(1, (int)((float)N / ppc));
}
__host__ __device__ inline int kg_ncmax(int N, int k) {
    const int t = kg_cells_target(N, k);
    return t + t / 4 + 8;
}

template <int CC>
__device__ __forceinline__ void kg_load(const float* __restrict__ xb, int64_t sC, int64_t sN, int p, float (&v)[3]) {
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = c < CC ? xb[c * sC + (int64_t)p * sN] : 0.f;
}

__device__ __forceinline__ float kg_wave_min(float v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float kg_wave_max(float v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

__device__ __forceinline__ uint64_t kg_max64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint64_t kg_min64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t kg_shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((uint32_t)v, m), hi = __shfl_xor((uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

// sorted (descending) list insert, every compare against the original list: slot
// q takes slot q-1 if the new key beats it, else the new key if it beats slot q
template <int KL>
__device__ __forceinline__ void kg_insert(uint64_t (&L)[KL], uint64_t key) {
    bool gt_cur = key > L[KL - 1];
#pragma unroll
    for (int q = KL - 1; q > 0; --q) {
        const bool gt_prev = key > L[q - 1];
        L[q] = gt_prev ? L[q - 1] : (gt_cur ? key : L[q]);
        gt_cur = gt_prev;
    }
    L[0] = gt_cur ? key : L[0];
}

template <int CC, int KB>
__global__ __launch_bounds__(KG_THREADS) void knn_grid_kernel(const float* __restrict__ x, int64_t sB, int64_t sC,
                                                             int64_t sN, int B, int N, int k, int nqb,
                                                             int64_t* __restrict__ idx64, int32_t* __restrict__ idx32,
                                                             float* __restrict__ vals) {
#pragma clang fp contract(off)
    constexpr int KL = KgList<KB>::KL;
    constexpr int M = KgList<KB>::M;
    extern __shared__ __attribute__((aligned(16))) unsigned char kg_smem[];
    int b, qb;
    if (!dgx_xcd_cloud_map(blockIdx.x, B, nqb, b, qb)) return;
    const int ncmax = kg_ncmax(N, k);
    const KgLds lay = kg_lds(N, ncmax, KL);
    float4* pts = reinterpret_cast<float4*>(kg_smem + lay.pts);
    uint32_t* nid = reinterpret_cast<uint32_t*>(kg_smem + lay.nid);
    int* cst = reinterpret_cast<int*>(kg_smem + lay.cst);
    unsigned char* scr = kg_smem + lay.scr;
    float* red = reinterpret_cast<float*>(kg_smem + lay.total - 128);   // [0, 24) bounding box, [24, 28) scan
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float* __restrict__ xb = x + (int64_t)b * sB;

    // ---- build: load the cloud once (registers), bounding box ------------------
    // wave w owns the index quarter [p_beg, p_end); its lane holds points
    // p_beg + 64 i + lane, i < PPT (the order the stable scatter needs)
    constexpr int PPT = KG_MAXN / KG_THREADS;
    const int q4 = (N + KG_WAVES - 1) / KG_WAVES;
    const int p_beg = min(N, wave * q4), p_end = min(N, p_beg + q4);
    float px[PPT][3];
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int p = p_beg + 64 * i + lane;
        if (p < p_end) {
            kg_load<CC>(xb, sC, sN, p, px[i]);
#pragma unroll
            for (int a = 0; a < 3; ++a) { mn[a] = fminf(mn[a], px[i][a]); mx[a] = fmaxf(mx[a], px[i][a]); }
        } else {
            px[i][0] = px[i][1] = px[i][2] = 0.f;
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) { mn[a] = kg_wave_min(mn[a]); mx[a] = kg_wave_max(mx[a]); }
    if (lane == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) { red[wave * 6 + a] = mn[a]; red[wave * 6 + 3 + a] = mx[a]; }
    }
    __syncthreads();
    float gmn[3], gmx[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        gmn[a] = red[a];
        gmx[a] = red[3 + a];
        for (int w = 1; w < KG_WAVES; ++w) {
            gmn[a] = fminf(gmn[a], red[w * 6 + a]);
            gmx[a] = fmaxf(gmx[a], red[w * 6 + 3 + a]);
        }
    }
    // ---- build: grid ----------------------------------------------------------
    KgGrid g;
    {
        float ext[3], emax = 0.f;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            ext[a] = gmx[a] - gmn[a];
            if (!(ext[a] > 0.f) || !isfinite(ext[a])) ext[a] = 0.f;
            emax = fmaxf(emax, ext[a]);
        }
        bool act[3];
        int nact = 0;
        float vol = 1.f;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            act[a] = ext[a] > 1e-6f * emax && ext[a] > 1e-30f;
            if (act[a]) { ++nact; vol *= ext[a]; }
        }
        const int tgt = kg_cells_target(N, k);
        float hh = nact == 0 ? 1.f : (nact == 1 ? vol / tgt : (nact == 2 ? sqrtf(vol / tgt) : cbrtf(vol / tgt)));
        if (!(hh > 0.f) || !isfinite(hh)) hh = emax > 0.f ? emax : 1.f;
        g.nc = ncmax + 1;
        for (int it = 0; it < 64; ++it) {
            int nc = 1;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                g.G[a] = act[a] ? min(64, max(1, (int)ceilf(ext[a] / hh))) : 1;
                nc *= g.G[a];
            }
            g.nc = nc;
            if (nc <= ncmax) break;
            hh *= 1.1f;
        }
        if (g.nc > ncmax) {   // degenerate extents: one cell (the exact fix covers every query)
#pragma unroll
            for (int a = 0; a < 3; ++a) { g.G[a] = 1; act[a] = false; }
            g.nc = 1;
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            g.lo[a] = gmn[a];
            g.inv[a] = act[a] ? (float)g.G[a] / ext[a] : 0.f;
            g.h[a] = act[a] ? ext[a] / (float)g.G[a] : 0.f;
        }
    }
    const int nc = g.nc;
    // ---- build: per-wave cell histograms (wave w counts its index quarter) ----
    int* hist = reinterpret_cast<int*>(scr);   // [KG_WAVES][nc]
    for (int i = tid; i < KG_WAVES * nc; i += KG_THREADS) hist[i] = 0;
    auto cell_of = [&](const float (&v)[3]) {
        return (kg_cell_axis(g, 2, v[2]) * g.G[1] + kg_cell_axis(g, 1, v[1])) * g.G[0] + kg_cell_axis(g, 0, v[0]);
    };
    int pc[PPT];
#pragma unroll
    for (int i = 0; i < PPT; ++i) pc[i] = cell_of(px[i]);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PPT; ++i)
        if (p_beg + 64 * i + lane < p_end) atomicAdd(&hist[wave * nc + pc[i]], 1);
    __syncthreads();
    // ---- build: scan -> cell starts and each wave's first slot per cell ------
    {
        const int cpt = (nc + KG_THREADS - 1) / KG_THREADS;
        const int c0 = min(nc, tid * cpt), c1 = min(nc, c0 + cpt);
        int s = 0;
        for (int c = c0; c < c1; ++c)
            for (int w = 0; w < KG_WAVES; ++w) s += hist[w * nc + c];
        int inc = s;   // inclusive scan over the block: waves, then across waves
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        int* wsum = reinterpret_cast<int*>(red) + 24;
        __syncthreads();
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        int run = inc - s;
        for (int w = 0; w < wave; ++w) run += wsum[w];
        for (int c = c0; c < c1; ++c) {
            cst[c] = run;
            for (int w = 0; w < KG_WAVES; ++w) {
                const int t = hist[w * nc + c];
                hist[w * nc + c] = run;
                run += t;
            }
        }
        if (tid == 0) cst[nc] = N;
    }
    __syncthreads();
    // ---- build: stable scatter (index order inside each wave's quarter) -------
    {
        const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
        int nbits = 1;
        while ((1 << nbits) < nc) ++nbits;
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            if (p_beg + 64 * i >= p_end) break;   // wave-uniform
            const int p = p_beg + 64 * i + lane;
            const bool ok = p < p_end;
            const int c = pc[i];
            // lanes of this chunk with the same cell: match over the cell's bits
            uint64_t peers = __ballot(ok);
            for (int bit = 0; bit < nbits; ++bit) {
                const uint64_t m = __ballot(ok && ((c >> bit) & 1));
                peers &= ((c >> bit) & 1) ? m : ~m;
            }
            const int rank = __popcll(peers & lt);
            const int base = ok ? hist[wave * nc + c] : 0;
            if (ok) {
                const float xx = (px[i][0] * px[i][0] + px[i][1] * px[i][1]) + px[i][2] * px[i][2];
                pts[base + rank] = make_float4(px[i][0], px[i][1], px[i][2], xx);
                nid[base + rank] = ~(uint32_t)p;
                if (rank == 0) hist[wave * nc + c] = base + __popcll(peers);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();
#ifdef DGX_KG_STAGE   // diagnostics build only: time the kernel's stages by early exits
    if (DGX_KG_STAGE == 1) {
        if (tid == 0 && pts[0].x == 12345.f) vals[0] = pts[1].y;
        return;
    }
#endif

    // ---- queries ---------------------------------------------------------------
    const int qi = lane >> 2, l = lane & 3;
    const int qpos = qb * KG_QPB + wave * KG_QPW + qi;   // sorted position of this lane's query
    const bool qok = qpos < N;
    const float4 qv = pts[qok ? qpos : 0];
    const uint32_t qn = nid[qok ? qpos : 0];
    const float q2[3] = {2.f * qv.x, 2.f * qv.y, 2.f * qv.z};
    const float xxq = qv.w;
    int qc[3];
    {
        const float v[3] = {qv.x, qv.y, qv.z};
#pragma unroll
        for (int a = 0; a < 3; ++a) qc[a] = kg_cell_axis(g, a, v[a]);
    }
    auto value = [&](const float4& c) {
        float d = c.x * q2[0];
        if (CC > 1) d = fmaf(c.y, q2[1], d);
        if (CC > 2) d = fmaf(c.z, q2[2], d);
        return (d - c.w) - xxq;
    };
    // visit the box of cells within R of the query's cell: rows (dy, dz), each a
    // contiguous run of positions; a query's 4 lanes deal the concatenation
    // round-robin. fn(p, live) is called wave-uniformly (live: lane has an item).
    auto row_range = [&](int R, int ri, int& p0, int& n) {   // row ri of the box: (dy, dz) in [-R, R]^2
        const int w = 2 * R + 1;
        const int z = qc[2] + ri / w - R, y = qc[1] + ri % w - R;
        p0 = 0;
        n = 0;
        if (qok && z >= 0 && z < g.G[2] && y >= 0 && y < g.G[1]) {
            const int row = (z * g.G[1] + y) * g.G[0];
            p0 = cst[row + max(0, qc[0] - R)];
            n = cst[row + min(g.G[0] - 1, qc[0] + R) + 1] - p0;
        }
    };
    // two items per step (both loads in flight together); the next row's range
    // is read while the current row is processed
    auto visit_box = [&](int R, auto&& fn) {
        int base = 0;
        const int nr = (2 * R + 1) * (2 * R + 1);
        int pn, nn;
        row_range(R, 0, pn, nn);
        for (int ri = 0; ri < nr; ++ri) {
            const int p0 = pn, n = nn;
            if (ri + 1 < nr) row_range(R, ri + 1, pn, nn);
            const int first = (l - base) & 3;
            const int trips = n > first ? (n - first + 3) >> 2 : 0;
            base += n;
            for (int t = 0;; t += 2) {
                const bool la = t < trips, lb = t + 1 < trips;
                if (!__any(la)) break;
                fn(p0 + first + 4 * t, la, p0 + first + 4 * t + 4, lb);
            }
        }
    };
    // distance from the query to the outside of the visited box (infinite on a
    // side at the grid edge: no point lies beyond it), less the cell-assignment
    // rounding margin
    auto coverage = [&](int R) {
        float cov = INFINITY;
        const float v[3] = {qv.x, qv.y, qv.z};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (g.G[a] <= 1) continue;
            const float dl = qc[a] - R > 0 ? v[a] - (g.lo[a] + (float)(qc[a] - R) * g.h[a]) : INFINITY;
            const float du = qc[a] + R < g.G[a] - 1 ? (g.lo[a] + (float)(qc[a] + R + 1) * g.h[a]) - v[a] : INFINITY;
            cov = fminf(cov, fminf(dl, du) - 1e-5f * (g.h[a] * (float)g.G[a]));
        }
        return cov;
    };

    // pre-pass (values only) over the 3x3x3 box: each lane's M best values;
    // T = min over the query's 4 lanes of their M-th is a lower bound of the
    // query's k-th value (4 M >= k candidates reach it)
    float pm[M];
#pragma unroll
    for (int t = 0; t < M; ++t) pm[t] = -INFINITY;
    auto put_m = [&](float v) {
#pragma unroll
        for (int t = M - 1; t > 0; --t) pm[t] = __builtin_amdgcn_fmed3f(pm[t - 1], pm[t], v);
        pm[0] = fmaxf(pm[0], v);
    };
    visit_box(1, [&](int pa, bool la, int pb, bool lb) {
        const float4 ca = pts[la ? pa : 0], cb = pts[lb ? pb : 0];
        if (la) put_m(value(ca));
        if (lb) put_m(value(cb));
    });
    float tm = pm[M - 1];
    tm = fminf(tm, __shfl_xor(tm, 1));
    tm = fminf(tm, __shfl_xor(tm, 2));
    const uint64_t tseed = tm == -INFINITY ? 0ull : ((uint64_t)kg_fkey(tm) << 32);
#ifdef DGX_KG_STAGE
    if (DGX_KG_STAGE == 2) {
        if (tm == 12345.f) vals[tid] = tm;
        return;
    }
#endif

    // main pass over the 5x5x5 box
    uint64_t Ls[KL];
#pragma unroll
    for (int t = 0; t < KL; ++t) Ls[t] = 0ull;
    uint64_t thr = tseed;
    uint64_t* fifo = reinterpret_cast<uint64_t*>(scr);   // [KG_QCAP][KG_THREADS]
    int cnt = 0;
    auto flush = [&]() {
#pragma unroll
        for (int t = 0; t < KG_QCAP; ++t) {
            if (!__any(t < cnt)) break;
            const uint64_t key = fifo[t * KG_THREADS + tid];
            if (t < cnt && key > thr) kg_insert<KL>(Ls, key);
        }
        cnt = 0;
        // shared bound: min over the 4 lanes of their M-th key; own bound: the list tail
        uint64_t mth = Ls[M - 1];
        mth = kg_min64(mth, kg_shfl_xor64(mth, 1));
        mth = kg_min64(mth, kg_shfl_xor64(mth, 2));
        thr = kg_max64(thr, kg_max64(mth, Ls[KL - 1]));
    };
    visit_box(2, [&](int pa, bool la, int pb, bool lb) {
        const int qa = la ? pa : 0, qb2 = lb ? pb : 0;
        const float4 ca = pts[qa], cb = pts[qb2];
        const uint32_t na = nid[qa], nb = nid[qb2];
        if (la) {
            const uint64_t key = kg_key(value(ca), na);
            fifo[cnt * KG_THREADS + tid] = key;
            cnt += key > thr ? 1 : 0;
        }
        if (lb) {
            const uint64_t key = kg_key(value(cb), nb);
            fifo[cnt * KG_THREADS + tid] = key;
            cnt += key > thr ? 1 : 0;
        }
        if (__any(cnt >= KG_QCAP - 1)) flush();   // room for the next step's two
    });
    flush();
#ifdef DGX_KG_STAGE
    if (DGX_KG_STAGE == 3) {
        if (Ls[0] == 12345ull) vals[tid] = 1.f;
        return;
    }
#endif

    // merge the query's 4 lists (lane l == 0, through LDS), check exactness
    __syncthreads();   // every wave is done with the FIFO region
    uint64_t* lists = reinterpret_cast<uint64_t*>(scr);   // [KG_THREADS][KL]
#pragma unroll
    for (int t = 0; t < KL; ++t) lists[tid * KL + t] = Ls[t];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint64_t kth = 0ull;
    int nvalid = 0;
    if (l == 0 && qok) {
        const uint64_t* L0 = lists + tid * KL;
        int p[4] = {0, 0, 0, 0};
        uint64_t h0 = L0[0], h1 = L0[KL], h2 = L0[2 * KL], h3 = L0[3 * KL];
        const int64_t row = ((int64_t)b * N + (int64_t)(~qn)) * k;
        for (int r = 0; r < k; ++r) {
            const uint64_t a01 = kg_max64(h0, h1), a23 = kg_max64(h2, h3);
            const uint64_t best = kg_max64(a01, a23);
            if (best == 0ull) break;
            const int w = best == h0 ? 0 : (best == h1 ? 1 : (best == h2 ? 2 : 3));
            const int np = ++p[w];
            const uint64_t nx = np < KL ? L0[w * KL + np] : 0ull;
            h0 = w == 0 ? nx : h0;
            h1 = w == 1 ? nx : h1;
            h2 = w == 2 ? nx : h2;
            h3 = w == 3 ? nx : h3;
            const int j = (int)~(uint32_t)best;
            if (idx64) idx64[row + r] = j;
            if (idx32) idx32[row + r] = j;
            if (vals) vals[row + r] = kg_keyf((uint32_t)(best >> 32));
            kth = best;
            nvalid = r + 1;
        }
    }
    // broadcast the query's k-th key to its 4 lanes
    {
        const int src = lane & ~3;
        kth = ((uint64_t)(uint32_t)__shfl((uint32_t)(kth >> 32), src) << 32) | (uint32_t)__shfl((uint32_t)kth, src);
        nvalid = __shfl(nvalid, src);
    }
    // a lane whose full list reaches the k-th may have dropped a top-k member
    bool flag = KL < k && Ls[KL - 1] != 0ull && Ls[KL - 1] >= kth;
    if (l == 0) {
        if (nvalid < k) {
            flag = true;
        } else {
            // every unvisited point is at least cov away: its value is at most
            // -cov^2 (+ the rounding of the reference's formula); the k-th
            // found must beat that
            const float cov = coverage(2);
            const float vk = kg_keyf((uint32_t)(kth >> 32));
            if (!(cov == INFINITY)) {
                const float c2 = cov > 0.f ? cov * cov : 0.f;
                const float margin = 1e-5f * (fabsf(xxq) + 4.f * fmaxf(fabsf(vk), c2)) + 1e-30f;
                if (!(vk > -c2 + margin)) flag = true;
            }
        }
    }
    flag = flag && qok;
    flag = flag || __shfl_xor(flag, 1);   // per query: the OR of its 4 lanes
    flag = flag || __shfl_xor(flag, 2);
    // ---- exact fix of flagged queries: the whole wave, over all N points ------
    uint64_t fl = __ballot(flag && l == 0);
#ifdef DGX_KG_STAGE
    if (DGX_KG_STAGE == 4) {
        if (lane == 0 && vals) vals[blockIdx.x * 4 + wave] = (float)__popcll(fl);   // flagged queries per wave
        return;
    }
#endif
    __syncthreads();   // lists region becomes the fix scratch
    uint64_t* fx = reinterpret_cast<uint64_t*>(scr) + wave * (KG_FXCAP + 1);   // [KG_FXCAP] keys | count
    int* fcnt = reinterpret_cast<int*>(fx + KG_FXCAP);
    while (fl) {
        const int src = __ffsll((long long)fl) - 1;
        fl &= fl - 1;
        // the flagged query's operands, from its lane
        const float fq0 = __shfl(q2[0], src), fq1 = __shfl(q2[1], src), fq2 = __shfl(q2[2], src);
        const float fxx = __shfl(xxq, src);
        const uint32_t fqn = __shfl(qn, src);
        const uint64_t t0 = ((uint64_t)(uint32_t)__shfl((uint32_t)(kth >> 32), src) << 32) |
                            (uint32_t)__shfl((uint32_t)kth, src);
        const bool have_t0 = __shfl(nvalid, src) >= k;
        const uint64_t T0 = have_t0 ? t0 : 0ull;   // a lower bound of the true k-th key
        auto fkey = [&](int p) {
            const float4 c = pts[p];
            float d = c.x * fq0;
            if (CC > 1) d = fmaf(c.y, fq1, d);
            if (CC > 2) d = fmaf(c.z, fq2, d);
            return kg_key((d - c.w) - fxx, nid[p]);
        };
        if (lane == 0) *fcnt = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int p = lane; p < N; p += 64) {
            const uint64_t key = fkey(p);
            if (key >= T0) {
                const int s = atomicAdd(fcnt, 1);
                if (s < KG_FXCAP) fx[s] = key;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int n = *fcnt;
        const int64_t row = ((int64_t)b * N + (int64_t)(~fqn)) * k;
        auto put = [&](int r, uint64_t key) {
            const int j = (int)~(uint32_t)key;
            if (idx64) idx64[row + r] = j;
            if (idx32) idx32[row + r] = j;
            if (vals) vals[row + r] = kg_keyf((uint32_t)(key >> 32));
        };
        if (n <= KG_FXCAP) {
            for (int e = lane; e < n; e += 64) {   // rank = number of better keys (keys are distinct)
                const uint64_t key = fx[e];
                int r = 0;
                for (int u = 0; u < n; ++u) r += fx[u] > key ? 1 : 0;
                if (r < k) put(r, key);
            }
        } else {
            // more than KG_FXCAP keys reach the bound: k rounds of a wave arg-max
            uint64_t prev = ~0ull;
            for (int r = 0; r < k; ++r) {
                uint64_t best = 0ull;
                for (int p = lane; p < N; p += 64) {
                    const uint64_t key = fkey(p);
                    if (key < prev) best = kg_max64(best, key);
                }
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) best = kg_max64(best, kg_shfl_xor64(best, o));
                if (lane == 0) put(r, best);
                prev = best;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int CC, int KB>
int launch_grid(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int N, int k, int64_t* idx64,
                int32_t* idx32, float* vals, hipStream_t st) {
    const int nqb = (N + KG_QPB - 1) / KG_QPB;
    const KgLds lay = kg_lds(N, kg_ncmax(N, k), KgList<KB>::KL);
    if (lay.total > 160 * 1024) return DGX_EUNSUPPORTED;
    hipLaunchKernelGGL((knn_grid_kernel<CC, KB>), dim3(dgx_xcd_cloud_grid(B, nqb)), dim3(KG_THREADS), lay.total, st,
                       x, sB, sC, sN, B, N, k, nqb, idx64, idx32, vals);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

template <int CC>
int dispatch_grid(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int N, int k, int64_t* idx64,
                  int32_t* idx32, float* vals, hipStream_t st) {
    if (k <= 8) return launch_grid<CC, 8>(x, sB, sC, sN, B, N, k, idx64, idx32, vals, st);
    if (k <= 16) return launch_grid<CC, 16>(x, sB, sC, sN, B, N, k, idx64, idx32, vals, st);
    if (k <= 20) return launch_grid<CC, 20>(x, sB, sC, sN, B, N, k, idx64, idx32, vals, st);
    if (k <= 32) return launch_grid<CC, 32>(x, sB, sC, sN, B, N, k, idx64, idx32, vals, st);
    if (k <= 40) return launch_grid<CC, 40>(x, sB, sC, sN, B, N, k, idx64, idx32, vals, st);
    return launch_grid<CC, 64>(x, sB, sC, sN, B, N, k, idx64, idx32, vals, st);
}

}  // namespace

extern "C" {

int dgx_knn_grid_ok(int C, int N, int k) {
    return C >= 1 && C <= 3 && N >= 1 && N <= KG_MAXN && k >= 1 && k <= 64 && k <= N ? 1 : 0;
}

const char* dgx_knn_grid_kernel_name(int C, int k) {
    static const char* names[3][6] = {
        {"knn_grid_kernel<1, 8>", "knn_grid_kernel<1, 16>", "knn_grid_kernel<1, 20>", "knn_grid_kernel<1, 32>",
         "knn_grid_kernel<1, 40>", "knn_grid_kernel<1, 64>"},
        {"knn_grid_kernel<2, 8>", "knn_grid_kernel<2, 16>", "knn_grid_kernel<2, 20>", "knn_grid_kernel<2, 32>",
         "knn_grid_kernel<2, 40>", "knn_grid_kernel<2, 64>"},
        {"knn_grid_kernel<3, 8>", "knn_grid_kernel<3, 16>", "knn_grid_kernel<3, 20>", "knn_grid_kernel<3, 32>",
         "knn_grid_kernel<3, 40>", "knn_grid_kernel<3, 64>"}};
    if (C < 1 || C > 3 || k < 1 || k > 64) return "";
    const int kb = k <= 8 ? 0 : k <= 16 ? 1 : k <= 20 ? 2 : k <= 32 ? 3 : k <= 40 ? 4 : 5;
    return names[C - 1][kb];
}

int dgx_knn_grid_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int C, int N, int k,
                     int64_t* idx64, int32_t* idx32, float* vals, void* stream) {
    if (!x || B < 0 || C < 1 || N < 1 || k < 1 || k > N) return DGX_EINVAL;
    if (!idx64 && !idx32) return DGX_EINVAL;
    if (!dgx_knn_grid_ok(C, N, k)) return DGX_EUNSUPPORTED;
    if (B == 0) return DGX_OK;
    hipStream_t st = dgx_stream(stream);
    switch (C) {
        case 1: return dispatch_grid<1>(x, sB, sC, sN, B, N, k, idx64, idx32, vals, st);
        case 2: return dispatch_grid<2>(x, sB, sC, sN, B, N, k, idx64, idx32, vals, st);
        default: return dispatch_grid<3>(x, sB, sC, sN, B, N, k, idx64, idx32, vals, st);
    }
}

}  // extern "C"
