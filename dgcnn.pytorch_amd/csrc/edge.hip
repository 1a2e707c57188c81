// a2 — edge features (reference models/dgcnn.py:15-44, get_graph_feature).
//
// Materialises the reference's edge tensor for API callers (PositionEmbedding,
// user code): out(b, c, n, kk) = x_j for c < C and x_i for c >= C, with the
// knn_only / disp_only variants and the paper's / test.ipynb:131 form
// (x_j - x_i, x_i) (DGX_GF_DIFFCAT), plus its backward (scatter-add into dx).
// DGCNN's own blocks never call this: they gather straight from P/Q
// (edgeconv.hip).
#include <math.h>

#include "common.h"

namespace {

// ------------------------------------------------------- graph feature -----
__global__ void graph_feature_kernel(const float* __restrict__ x, int64_t sB, int64_t sC, int64_t sN, int B,
                                     int C, int N, const int32_t* __restrict__ idx, int k, int mode,
                                     float* __restrict__ out) {
    const int64_t per_b = (mode == DGX_GF_CAT || mode == DGX_GF_DIFFCAT ? 2LL : 1LL) * C * N * k;
    const int64_t total = per_b * B;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        int64_t r = t;
        int b = (int)(r / per_b);
        r -= (int64_t)b * per_b;
        const float* xb = x + b * sB;
        const int32_t* ib = idx + (int64_t)b * N * k;
        if (mode == DGX_GF_KNN_ONLY) {  // (B,N,k,C)
            int c = (int)(r % C);
            int64_t nk = r / C;
            int n = (int)(nk / k), kk = (int)(nk - (int64_t)n * k);
            out[t] = xb[c * sC + (int64_t)ib[(int64_t)n * k + kk] * sN];
        } else {                         // (B,C',N,k)
            int kk = (int)(r % k);
            int64_t cn = r / k;
            int n = (int)(cn % N);
            int c2 = (int)(cn / N);
            int j = ib[(int64_t)n * k + kk];
            if (mode == DGX_GF_DISP || (mode == DGX_GF_DIFFCAT && c2 < C)) {
                out[t] = xb[c2 * sC + (int64_t)j * sN] - xb[c2 * sC + (int64_t)n * sN];
            } else {
                out[t] = c2 < C ? xb[c2 * sC + (int64_t)j * sN] : xb[(c2 - C) * sC + (int64_t)n * sN];
            }
        }
    }
}

// dx (B,C,N) contiguous += grad of graph_feature
__global__ void graph_feature_bwd_kernel(const float* __restrict__ dout, int B, int C, int N,
                                         const int32_t* __restrict__ idx, int k, int mode,
                                         float* __restrict__ dx) {
    const int64_t total = (int64_t)B * C * N;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        int n = (int)(t % N);
        int64_t bc = t / N;
        int c = (int)(bc % C);
        int b = (int)(bc / C);
        const int32_t* row = idx + ((int64_t)b * N + n) * k;
        float* dxb = dx + (int64_t)b * C * N;
        float centre = 0.f;
        if (mode == DGX_GF_KNN_ONLY) {
            const float* d = dout + (((int64_t)b * N + n) * k) * C + c;
            for (int kk = 0; kk < k; ++kk) atomicAdd(dxb + (int64_t)c * N + row[kk], d[(int64_t)kk * C]);
        } else {
            const bool two = mode == DGX_GF_CAT || mode == DGX_GF_DIFFCAT;
            const int Cp = two ? 2 * C : C;
            const float* d = dout + (((int64_t)b * Cp + c) * N + n) * k;
            for (int kk = 0; kk < k; ++kk) {
                float g = d[kk];
                atomicAdd(dxb + (int64_t)c * N + row[kk], g);
                if (mode == DGX_GF_DISP || mode == DGX_GF_DIFFCAT) centre -= g;
            }
            if (two) {
                const float* dc = dout + (((int64_t)b * Cp + C + c) * N + n) * k;
                for (int kk = 0; kk < k; ++kk) centre += dc[kk];
            }
        }
        if (centre != 0.f) atomicAdd(dxb + (int64_t)c * N + n, centre);
    }
}

// The same gradient without atomics: one thread per (b, c, j) sums j's
// in-edges from the reverse kNN graph (dgx_graph_reverse: CSR rows of edge ids
// (i << 6) | slot, ascending) in that fixed order, then the centre terms of
// j's own row — every dx element has one writer and a fixed summation order.
__global__ void graph_feature_bwd_csr_kernel(const float* __restrict__ dout, int B, int C, int N, int k, int mode,
                                             const int32_t* __restrict__ rowptr, const int32_t* __restrict__ edges,
                                             float* __restrict__ dx) {
    const int64_t total = (int64_t)B * C * N;
    const bool two = mode == DGX_GF_CAT || mode == DGX_GF_DIFFCAT;
    const int Cp = two ? 2 * C : C;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int n = (int)(t % N);
        const int64_t bc = t / N;
        const int c = (int)(bc % C);
        const int b = (int)(bc / C);
        const int64_t j = (int64_t)b * N + n;
        const int32_t beg = rowptr[j], end = rowptr[j + 1];
        float acc = 0.f;
        for (int32_t e = beg; e < end; ++e) {
            const int32_t id = edges[e];
            const int64_t i = id >> 6;   // global point of the edge's source
            const int s = id & 63;
            if (mode == DGX_GF_KNN_ONLY) acc += dout[(i * k + s) * C + c];
            else acc += dout[(((int64_t)b * Cp + c) * N + (i - (int64_t)b * N)) * k + s];
        }
        float centre = 0.f;
        if (mode != DGX_GF_KNN_ONLY) {
            const float* d = dout + (((int64_t)b * Cp + c) * N + n) * k;
            if (mode == DGX_GF_DISP || mode == DGX_GF_DIFFCAT)
                for (int kk = 0; kk < k; ++kk) centre -= d[kk];
            if (two) {
                const float* dc = dout + (((int64_t)b * Cp + C + c) * N + n) * k;
                for (int kk = 0; kk < k; ++kk) centre += dc[kk];
            }
        }
        dx[(int64_t)b * C * N + (int64_t)c * N + n] += acc + centre;
    }
}

inline int grid_for(int64_t total, int block) {
    int64_t g = (total + block - 1) / block;
    return (int)(g < 8192 ? (g < 1 ? 1 : g) : 8192);
}

}  // namespace

extern "C" {

const char* dgx_version(void) { return "dgx 0.1.0 (gfx950)"; }

const char* dgx_strerror(int code) {
    switch (code) {
        case DGX_OK: return "ok";
        case DGX_EINVAL: return "invalid argument";
        case DGX_EUNSUPPORTED: return "unsupported shape";
        case DGX_ELAUNCH: return "kernel launch failed";
        default: return "unknown error";
    }
}

int dgx_graph_feature_f32(const float* x, int64_t sB, int64_t sC, int64_t sN, int B, int C, int N,
                          const int32_t* idx, int k, int mode, float* out, void* stream) {
    if (!x || !idx || !out || B < 0 || C < 1 || N < 1 || k < 1 || mode < 0 || mode > 3) return DGX_EINVAL;
    int64_t total = (int64_t)B * C * N * k * (mode == DGX_GF_CAT || mode == DGX_GF_DIFFCAT ? 2 : 1);
    if (total == 0) return DGX_OK;
    hipLaunchKernelGGL(graph_feature_kernel, dim3(grid_for(total, 256)), dim3(256), 0, dgx_stream(stream), x, sB, sC,
                       sN, B, C, N, idx, k, mode, out);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_graph_feature_bwd_csr_f32(const float* dout, int B, int C, int N, int k, int mode, const int32_t* rowptr,
                                  const int32_t* edges, float* dx, void* stream) {
    if (!dout || !rowptr || !edges || !dx || B < 0 || C < 1 || N < 1 || k < 1 || k > 64 || mode < 0 || mode > 3)
        return DGX_EINVAL;
    const int64_t total = (int64_t)B * C * N;
    if (total == 0) return DGX_OK;
    hipLaunchKernelGGL(graph_feature_bwd_csr_kernel, dim3(grid_for(total, 256)), dim3(256), 0, dgx_stream(stream),
                       dout, B, C, N, k, mode, rowptr, edges, dx);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_graph_feature_bwd_f32(const float* dout, int B, int C, int N, const int32_t* idx, int k, int mode,
                              float* dx, void* stream) {
    if (!dout || !idx || !dx || B < 0 || C < 1 || N < 1 || k < 1 || mode < 0 || mode > 3) return DGX_EINVAL;
    int64_t total = (int64_t)B * C * N;
    if (total == 0) return DGX_OK;
    hipLaunchKernelGGL(graph_feature_bwd_kernel, dim3(grid_for(total, 256)), dim3(256), 0, dgx_stream(stream), dout,
                       B, C, N, idx, k, mode, dx);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

}  // extern "C"
