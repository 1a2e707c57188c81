/*
 * TEST INFRASTRUCTURE ONLY — the CPU oracle for the kNN hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker. The product path (dgx/, libdgx.so)
 * never links or calls it.
 *
 * Restates, in plain C with the exact fp32 rounding sequence of the reference's
 * CPU arithmetic, reference models/dgcnn.py:6-12:
 *
 *     inner = -2 * matmul(x^T, x)                      (dgcnn.py:7)
 *     xx    = sum(x**2, dim=1, keepdim=True)           (dgcnn.py:8)
 *     pd    = -xx - inner - xx^T                       (dgcnn.py:9)
 *     idx   = pd.topk(k, dim=-1)[1]                    (dgcnn.py:11)
 *
 * Rounding facts pinned against the reference itself (tests/golden/, made by
 * tests/golden/make_goldens.py from the reference's own knn on this host):
 *   - dot_ij is a sequential fp32 FMA chain over c = 0..C-1 (MKL sgemm, C <= 256).
 *   - xx_i follows torch 2.10's CPU sum kernel (aten SumKernel.cpp), whose
 *     order depends on the layout torch sees for x**2:
 *       cascade(e)  : 4-level cascade, 16 elements per level-0 run (multi_row_sum)
 *       rowsum(e)   : 4 interleaved accumulators (e[i] -> i%4), each a cascade;
 *                     leftover e[4*floor(n/4)..] added to accumulator 0; then
 *                     ((a0+a1)+a2)+a3 (row_sum, ILP 4)
 *       ORDER_STRIDED  (N contiguous, a (B,C,N) contiguous tensor): points in
 *                      full 32-point blocks use cascade(all C channels), the
 *                      rest rowsum(all C channels) (vectorized_outer_sum); N >= 8.
 *       ORDER_VEC8X4   (C contiguous, e.g. the permute(0,2,1) view main_cls.py:91
 *                      feeds): C >= 8: lane l = rowsum over the C/8 full 8-wide
 *                      vectors; result = ((0 + tail channels in order) + lane 0)
 *                      + ... + lane 7 (vectorized_inner_sum); C < 8: rowsum.
 *   - pd_ij = fl( fl(2*dot_ij - xx_j) - xx_i ).
 *   - topk tie order in the reference is arbitrary; the oracle returns the
 *     canonical order (pd descending, index ascending).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORDER_STRIDED 0
#define ORDER_VEC8X4 1

/* torch multi_row_sum for one row: levels of 16 */
static float cascade(const float* e, int m) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int i = 0;
    while (i + 16 <= m) {
        for (int j = 0; j < 16; ++j, ++i) acc[0] = acc[0] + e[i];
        for (int l = 1; l < 4; ++l) {
            acc[l] = acc[l] + acc[l - 1];
            acc[l - 1] = 0.f;
            if ((i & (15 << (4 * l))) != 0) break;
        }
    }
    for (; i < m; ++i) acc[0] = acc[0] + e[i];
    for (int l = 1; l < 4; ++l) acc[0] = acc[0] + acc[l];
    return acc[0];
}

/* torch row_sum, ILP 4 */
static float rowsum(const float* e, int n) {
    int si = n / 4;
    float lanes[4];
    float tmp[1024];
    for (int k = 0; k < 4; ++k) {
        for (int t = 0; t < si; ++t) tmp[t] = e[k + 4 * t];
        lanes[k] = si > 0 ? cascade(tmp, si) : 0.f;
    }
    for (int i = 4 * si; i < n; ++i) lanes[0] = lanes[0] + e[i];
    return ((lanes[0] + lanes[1]) + lanes[2]) + lanes[3];
}

static float sqnorm_one(const float* x, int64_t sC, int C, int order, int tail) {
    float sq[4096];
    for (int c = 0; c < C; ++c) {
        float v = x[c * sC];
        sq[c] = v * v;
    }
    if (order == ORDER_VEC8X4) {
        if (C < 8) return rowsum(sq, C);
        int vs = C / 8;
        float lane_elems[512];
        float fin = 0.f;
        for (int c = 8 * vs; c < C; ++c) fin = fin + sq[c];
        for (int l = 0; l < 8; ++l) {
            for (int v = 0; v < vs; ++v) lane_elems[v] = sq[8 * v + l];
            fin = fin + rowsum(lane_elems, vs);
        }
        return fin;
    }
    return tail ? rowsum(sq, C) : cascade(sq, C);
}

/* xx[b*N+n] for x given by element strides (sB, sC, sN). */
void oracle_sqnorm(const float* x, int64_t sB, int64_t sC, int64_t sN,
                   int B, int C, int N, int order, float* xx) {
    if (C > 4096) return;
    const int nvec = N & ~31;
    for (int b = 0; b < B; ++b)
        for (int n = 0; n < N; ++n)
            xx[(int64_t)b * N + n] = sqnorm_one(x + b * sB + n * sN, sC, C, order, n >= nvec);
}

static inline float pd_elem(const float* xb, int64_t sC, int64_t sN, int C,
                            int i, int j, float xxi, float xxj) {
    float d = 0.f;
    const float* xi = xb + i * sN;
    const float* xj = xb + j * sN;
    for (int c = 0; c < C; ++c) d = fmaf(xi[c * sC], xj[c * sC], d);
    volatile float two_dot = 2.0f * d;         /* exact: -2*dot negated */
    volatile float t = two_dot - xxj;          /* (-xx_j) - inner       */
    volatile float r = t - xxi;                /* ... - xx_i            */
    return r;
}

/* Full (B,N,N) negated squared-distance matrix, reference dgcnn.py:7-9. */
void oracle_pairwise(const float* x, int64_t sB, int64_t sC, int64_t sN,
                     int B, int C, int N, int order, float* pd) {
    float* xx = (float*)malloc(sizeof(float) * (size_t)B * N);
    oracle_sqnorm(x, sB, sC, sN, B, C, N, order, xx);
    for (int b = 0; b < B; ++b) {
        const float* xb = x + b * sB;
        const float* xxb = xx + (int64_t)b * N;
        #pragma omp parallel for schedule(static)
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j)
                pd[((int64_t)b * N + i) * N + j] = pd_elem(xb, sC, sN, C, i, j, xxb[i], xxb[j]);
    }
    free(xx);
}

/* canonical "a ranks before b": larger value first, then smaller index */
static inline int ranks_before(float va, int ia, float vb, int ib) {
    return va > vb || (va == vb && ia < ib);
}

/*
 * kNN, reference dgcnn.py:6-12, canonical tie order. idx (B,N,k) int64 local
 * indices 0..N-1; vals (B,N,k) the selected pd values (may be NULL).
 * Returns 0, or -1 when k is out of range (torch.topk raises for k > N).
 */
int oracle_knn(const float* x, int64_t sB, int64_t sC, int64_t sN,
               int B, int C, int N, int k, int order,
               int64_t* idx, float* vals) {
    if (k < 1 || k > N || C > 4096) return -1;
    float* xx = (float*)malloc(sizeof(float) * (size_t)B * N);
    oracle_sqnorm(x, sB, sC, sN, B, C, N, order, xx);
    for (int b = 0; b < B; ++b) {
        const float* xb = x + b * sB;
        const float* xxb = xx + (int64_t)b * N;
        #pragma omp parallel for schedule(dynamic, 16)
        for (int i = 0; i < N; ++i) {
            float* bv = (float*)malloc(sizeof(float) * k);
            int* bi = (int*)malloc(sizeof(int) * k);
            int cnt = 0;
            for (int j = 0; j < N; ++j) {
                float v = pd_elem(xb, sC, sN, C, i, j, xxb[i], xxb[j]);
                if (cnt == k && !ranks_before(v, j, bv[k - 1], bi[k - 1])) continue;
                int p = cnt < k ? cnt++ : k - 1;
                while (p > 0 && ranks_before(v, j, bv[p - 1], bi[p - 1])) {
                    bv[p] = bv[p - 1];
                    bi[p] = bi[p - 1];
                    --p;
                }
                bv[p] = v;
                bi[p] = j;
            }
            int64_t row = ((int64_t)b * N + i) * k;
            for (int t = 0; t < k; ++t) {
                idx[row + t] = bi[t];
                if (vals) vals[row + t] = bv[t];
            }
            free(bv);
            free(bi);
        }
    }
    free(xx);
    return 0;
}
