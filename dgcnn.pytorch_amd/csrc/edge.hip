// a2/a3/a8 — edge features and the decomposed EdgeConv block.
//
// Reference (models/dgcnn.py:15-44, 54-98): every block materialises the edge
// tensor (B,2C,N,k), runs Conv2d(2C,Co,1) + BatchNorm2d + LeakyReLU over all
// B*N*k edges and takes max over k. Because the conv is linear and 1x1,
//     y(i,j) = W1 x_j + W2 x_i = P_j + Q_i,   P = X W1^T, Q = X W2^T,
// so the engine runs a per-point GEMM (k times fewer flops, done by the
// caller) and these kernels do the rest straight from P/Q:
//   gather   : per (i,o) max_k P_j (min_k where gamma_o < 0), argument, sum_k P_j
//              and BN partial sums over every edge value — no edge tensor.
//   finalize : batch statistics -> affine (a,b), running stats.
//   apply    : LeakyReLU(a*ysel + b) into the caller's concat buffer.
// max_k LReLU(a y + b) = LReLU(a max_k y + b) for a >= 0 (min for a < 0) since
// both maps are monotone; sign(a) = sign(gamma).
//
// Backward follows BN's train-mode gradient: for every edge
//   dy_e = a*dz_e + c0 + c1*y_e,   dz_e nonzero only at the selected edge,
// so dQ_i = a*dz_i + k*c0 + c1*sum_k y_ik and dP_j needs the reverse kNN graph
// (in-edges of j): built as a CSR here, gathered per point (deterministic
// except for the order of in-edges, i.e. fp32 summation order only).
#include <math.h>

#include "common.h"

namespace {

constexpr int EG_PTS = 16;   // points per wave in the gather kernels
constexpr int EG_WAVES = 4;

__device__ __forceinline__ float lrelu(float v, float slope) { return v > 0.f ? v : v * slope; }

// ------------------------------------------------------- graph feature -----
__global__ void graph_feature_kernel(const float* __restrict__ x, int64_t sB, int64_t sC, int64_t sN, int B,
                                     int C, int N, const int32_t* __restrict__ idx, int k, int mode,
                                     float* __restrict__ out) {
    const int64_t per_b = (mode == DGX_GF_CAT ? 2LL : 1LL) * C * N * k;
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
            if (mode == DGX_GF_DISP) {
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
            const int Cp = mode == DGX_GF_CAT ? 2 * C : C;
            const float* d = dout + (((int64_t)b * Cp + c) * N + n) * k;
            for (int kk = 0; kk < k; ++kk) {
                float g = d[kk];
                atomicAdd(dxb + (int64_t)c * N + row[kk], g);
                if (mode == DGX_GF_DISP) centre -= g;
            }
            if (mode == DGX_GF_CAT) {
                const float* dc = dout + (((int64_t)b * Cp + C + c) * N + n) * k;
                for (int kk = 0; kk < k; ++kk) centre += dc[kk];
            }
        }
        if (centre != 0.f) atomicAdd(dxb + (int64_t)c * N + n, centre);
    }
}

// ---------------------------------------------------- EdgeConv forward -----
// grid: (dgx_xcd_cloud_grid(B, tiles), ceil(Co/64)); block 256 = 4 waves.
// A block covers EG_WAVES*EG_PTS points of one cloud for 64 channels; each
// lane owns one channel, each wave walks its points one by one (the idx row
// of a point is wave-uniform -> scalar loads; P rows are 256 B coalesced).
template <bool EVAL>
__global__ __launch_bounds__(256) void edge_gather_kernel(
    const float* __restrict__ PQ, int ldpq, const int32_t* __restrict__ idx, int B, int N, int k, int Co,
    int tiles, const float* __restrict__ gamma_or_scale, const float* __restrict__ shift, float slope,
    float* __restrict__ ysel, uint8_t* __restrict__ arg, float* __restrict__ sumP, float* __restrict__ partials,
    float* __restrict__ out, int ldo) {
    __shared__ float red[2][EG_WAVES][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int o = blockIdx.y * 64 + lane;
    const bool ok = o < Co;
    int b, tile;
    const bool valid = dgx_xcd_cloud_map(blockIdx.x, B, tiles, b, tile);
    float acc1 = 0.f, acc2 = 0.f;
    if (valid) {
        const float sgn = ok ? gamma_or_scale[o] : 1.f;
        const bool take_min = sgn < 0.f;
        const float* __restrict__ Pb = PQ + (int64_t)b * N * ldpq;
        const int n0 = tile * (EG_WAVES * EG_PTS) + wave * EG_PTS;
        for (int p = 0; p < EG_PTS; ++p) {
            const int n = n0 + p;
            if (n >= N) break;
            const int64_t i = (int64_t)b * N + n;
            const int32_t* __restrict__ row = idx + i * k;
            float best = 0.f, s = 0.f, s2 = 0.f;
            int barg = 0;
            if (ok) {
                for (int kk = 0; kk < k; ++kk) {
                    const float v = Pb[(int64_t)row[kk] * ldpq + o];
                    const bool better = kk == 0 || (take_min ? v < best : v > best);
                    best = better ? v : best;
                    barg = better ? kk : barg;
                    s += v;
                    s2 = fmaf(v, v, s2);
                }
                const float q = PQ[i * ldpq + Co + o];
                const float y = best + q;
                if (EVAL) {
                    out[i * ldo + o] = lrelu(fmaf(sgn, y, shift[o]), slope);
                } else {
                    ysel[i * Co + o] = y;
                    arg[i * Co + o] = (uint8_t)barg;
                    sumP[i * Co + o] = s;
                    // sum over the k edge values y = P_j + q, and of y^2
                    acc1 += fmaf((float)k, q, s);
                    acc2 += s2 + q * fmaf(2.f, s, (float)k * q);
                }
            }
        }
    }
    if (EVAL) return;
    red[0][wave][lane] = acc1;
    red[1][wave][lane] = acc2;
    __syncthreads();
    if (wave == 0 && ok) {
        float t1 = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
        float t2 = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
        partials[(int64_t)blockIdx.x * 2 * Co + o] = t1;
        partials[(int64_t)blockIdx.x * 2 * Co + Co + o] = t2;
    }
}

__global__ void bn_finalize_kernel(const float* __restrict__ partials, int nblk, int Co, double count,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ rmean, float* __restrict__ rvar, double momentum,
                                   double eps, float* __restrict__ scale, float* __restrict__ shift,
                                   float* __restrict__ mean_out, float* __restrict__ invstd_out) {
    int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= Co) return;
    double s1 = 0.0, s2 = 0.0;
    for (int i = 0; i < nblk; ++i) {
        s1 += (double)partials[(int64_t)i * 2 * Co + o];
        s2 += (double)partials[(int64_t)i * 2 * Co + Co + o];
    }
    double mean = s1 / count;
    double var = s2 / count - mean * mean;
    if (var < 0.0) var = 0.0;
    double invstd = 1.0 / sqrt(var + eps);
    double g = gamma ? (double)gamma[o] : 1.0;
    double bt = beta ? (double)beta[o] : 0.0;
    double a = g * invstd;
    scale[o] = (float)a;
    shift[o] = (float)(bt - mean * a);
    if (mean_out) mean_out[o] = (float)mean;
    if (invstd_out) invstd_out[o] = (float)invstd;
    if (rmean) rmean[o] = (float)((1.0 - momentum) * (double)rmean[o] + momentum * mean);
    if (rvar) {
        double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
        rvar[o] = (float)((1.0 - momentum) * (double)rvar[o] + momentum * unbiased);
    }
}

__global__ void bn_eval_affine_kernel(int Co, const float* __restrict__ gamma, const float* __restrict__ beta,
                                      const float* __restrict__ rmean, const float* __restrict__ rvar,
                                      double eps, float* __restrict__ scale, float* __restrict__ shift) {
    int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= Co) return;
    float invstd = 1.0f / sqrtf(rvar[o] + (float)eps);
    float a = (gamma ? gamma[o] : 1.f) * invstd;
    scale[o] = a;
    shift[o] = (beta ? beta[o] : 0.f) - rmean[o] * a;
}

__global__ void bn_lrelu_apply_kernel(const float* __restrict__ ysel, int M, int Co,
                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                      float slope, float* __restrict__ out, int ldo) {
    const int64_t total = (int64_t)M * Co;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        int o = (int)(t % Co);
        int64_t i = t / Co;
        out[i * ldo + o] = lrelu(fmaf(scale[o], ysel[t], shift[o]), slope);
    }
}

// --------------------------------------------------- EdgeConv backward -----
// dz at the selected edge and partial (sum dz, sum dz*yhat); grid (nblk, ceil(Co/64)).
__global__ __launch_bounds__(256) void edge_bwd_dz_kernel(const float* __restrict__ dY, int lddy,
                                                          const float* __restrict__ ysel, int M, int Co,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, float slope,
                                                          float* __restrict__ dz, float* __restrict__ partials,
                                                          int rows_per_blk) {
    __shared__ float red[2][EG_WAVES][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int o = blockIdx.y * 64 + lane;
    const bool ok = o < Co;
    float acc1 = 0.f, acc2 = 0.f;
    if (ok) {
        const float a = scale[o], sh = shift[o], mu = mean[o], is = invstd[o];
        const int64_t i0 = (int64_t)blockIdx.x * rows_per_blk;
        for (int r = wave; r < rows_per_blk; r += EG_WAVES) {
            const int64_t i = i0 + r;
            if (i >= M) break;
            const float y = ysel[i * Co + o];
            const float z = fmaf(a, y, sh);
            const float d = dY[i * lddy + o] * (z > 0.f ? 1.f : slope);
            dz[i * Co + o] = d;
            acc1 += d;
            acc2 = fmaf(d, (y - mu) * is, acc2);
        }
    }
    red[0][wave][lane] = acc1;
    red[1][wave][lane] = acc2;
    __syncthreads();
    if (wave == 0 && ok) {
        partials[(int64_t)blockIdx.x * 2 * Co + o] = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
        partials[(int64_t)blockIdx.x * 2 * Co + Co + o] =
            red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
    }
}

__global__ void bn_bwd_finalize_kernel(const float* __restrict__ partials, int nblk, int Co, double count,
                                       const float* __restrict__ scale, const float* __restrict__ mean,
                                       const float* __restrict__ invstd, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, float* __restrict__ c0,
                                       float* __restrict__ c1, int accumulate) {
    int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= Co) return;
    double s1 = 0.0, s2 = 0.0;
    for (int i = 0; i < nblk; ++i) {
        s1 += (double)partials[(int64_t)i * 2 * Co + o];
        s2 += (double)partials[(int64_t)i * 2 * Co + Co + o];
    }
    if (dbeta) dbeta[o] = (float)(accumulate ? (double)dbeta[o] + s1 : s1);
    if (dgamma) dgamma[o] = (float)(accumulate ? (double)dgamma[o] + s2 : s2);
    const double a = scale[o], mu = mean[o], is = invstd[o];
    const double g1 = s1 / count, g2 = s2 / count;
    c0[o] = (float)(a * (-g1 + g2 * mu * is));
    c1[o] = (float)(-a * g2 * is);
}

// ----------------------------------------------------- reverse kNN graph ----
__global__ void rev_count_kernel(const int32_t* __restrict__ idx, int B, int N, int k, int32_t* __restrict__ cnt) {
    const int64_t E = (int64_t)B * N * k;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        int64_t i = e / k;
        int b = (int)(i / N);
        atomicAdd(cnt + (int64_t)b * N + idx[e], 1);
    }
}

// single-block exclusive scan of M counts -> rowptr (M+1); cursor = rowptr copy
__global__ __launch_bounds__(1024) void rev_scan_kernel(const int32_t* __restrict__ cnt, int M,
                                                        int32_t* __restrict__ rowptr,
                                                        int32_t* __restrict__ cursor) {
    __shared__ int32_t part[1024];
    const int t = threadIdx.x;
    const int per = (M + 1023) / 1024;
    const int lo = t * per, hi = min(M, lo + per);
    int32_t s = 0;
    for (int i = lo; i < hi; ++i) s += cnt[i];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        int32_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int32_t run = t == 0 ? 0 : part[t - 1];
    for (int i = lo; i < hi; ++i) {
        rowptr[i] = run;
        cursor[i] = run;
        run += cnt[i];
    }
    if (t == 1023) rowptr[M] = part[1023];
}

__global__ void rev_fill_kernel(const int32_t* __restrict__ idx, int B, int N, int k, int32_t* __restrict__ cursor,
                                int32_t* __restrict__ edges) {
    const int64_t E = (int64_t)B * N * k;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        int64_t i = e / k;
        int kk = (int)(e - i * k);
        int b = (int)(i / N);
        int pos = atomicAdd(cursor + (int64_t)b * N + idx[e], 1);
        edges[pos] = (int32_t)((i << 6) | kk);
    }
}

// dPQ for every point: one wave per point, lanes over 64 channels.
__global__ __launch_bounds__(256) void edge_bwd_scatter_kernel(
    const float* __restrict__ PQ, int ldpq, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ edges,
    const uint8_t* __restrict__ arg, const float* __restrict__ dz, const float* __restrict__ sumP, int B, int N,
    int k, int Co, int tiles, const float* __restrict__ scale, const float* __restrict__ c0,
    const float* __restrict__ c1, float* __restrict__ dPQ) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int o = blockIdx.y * 64 + lane;
    int b, tile;
    if (!dgx_xcd_cloud_map(blockIdx.x, B, tiles, b, tile)) return;
    if (o >= Co) return;
    const float a = scale[o], k0 = c0[o], k1 = c1[o];
    const int n0 = tile * (EG_WAVES * EG_PTS) + wave * EG_PTS;
    for (int p = 0; p < EG_PTS; ++p) {
        const int n = n0 + p;
        if (n >= N) break;
        const int64_t j = (int64_t)b * N + n;
        const int beg = rowptr[j], end = rowptr[j + 1];
        float sq = 0.f, sd = 0.f;
        for (int t = beg; t < end; ++t) {
            const int32_t e = edges[t];
            const int64_t i = e >> 6;
            const int kk = e & 63;
            sq += PQ[i * ldpq + Co + o];
            sd += (arg[i * Co + o] == kk) ? dz[i * Co + o] : 0.f;
        }
        const float deg = (float)(end - beg);
        const float pj = PQ[j * ldpq + o], qj = PQ[j * ldpq + Co + o];
        dPQ[j * 2 * Co + o] = fmaf(a, sd, fmaf(k0, deg, k1 * fmaf(deg, pj, sq)));
        const float kf = (float)k;
        dPQ[j * 2 * Co + Co + o] = fmaf(a, dz[j * Co + o], fmaf(k0, kf, k1 * fmaf(kf, qj, sumP[j * Co + o])));
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
    if (!x || !idx || !out || B < 0 || C < 1 || N < 1 || k < 1 || mode < 0 || mode > 2) return DGX_EINVAL;
    int64_t total = (int64_t)B * C * N * k * (mode == DGX_GF_CAT ? 2 : 1);
    if (total == 0) return DGX_OK;
    hipLaunchKernelGGL(graph_feature_kernel, dim3(grid_for(total, 256)), dim3(256), 0, dgx_stream(stream), x, sB, sC,
                       sN, B, C, N, idx, k, mode, out);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_graph_feature_bwd_f32(const float* dout, int B, int C, int N, const int32_t* idx, int k, int mode,
                              float* dx, void* stream) {
    if (!dout || !idx || !dx || B < 0 || C < 1 || N < 1 || k < 1 || mode < 0 || mode > 2) return DGX_EINVAL;
    int64_t total = (int64_t)B * C * N;
    if (total == 0) return DGX_OK;
    hipLaunchKernelGGL(graph_feature_bwd_kernel, dim3(grid_for(total, 256)), dim3(256), 0, dgx_stream(stream), dout,
                       B, C, N, idx, k, mode, dx);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_partials_blocks(int B, int N, int Co) {
    (void)Co;
    const int tiles = (N + EG_WAVES * EG_PTS - 1) / (EG_WAVES * EG_PTS);
    return dgx_xcd_cloud_grid(B, tiles);
}

int dgx_edge_fwd_gather_f32(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int Co,
                            const float* gamma, float* ysel, uint8_t* arg, float* sumP, float* partials,
                            int nblk_hint, void* stream) {
    if (!PQ || !idx || !gamma || !ysel || !arg || !sumP || !partials) return DGX_EINVAL;
    if (B < 1 || N < 1 || k < 1 || k > 64 || Co < 1 || ldpq < 2 * Co) return DGX_EINVAL;
    const int tiles = (N + EG_WAVES * EG_PTS - 1) / (EG_WAVES * EG_PTS);
    const int gx = dgx_xcd_cloud_grid(B, tiles);
    if (nblk_hint != gx) return DGX_EINVAL;
    dim3 grid(gx, (Co + 63) / 64);
    hipLaunchKernelGGL((edge_gather_kernel<false>), grid, dim3(256), 0, dgx_stream(stream), PQ, ldpq, idx, B, N, k,
                       Co, tiles, gamma, (const float*)nullptr, 0.f, ysel, arg, sumP, partials, (float*)nullptr, 0);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_fwd_eval_f32(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int Co,
                          const float* scale, const float* shift, float slope, float* out, int ldo, void* stream) {
    if (!PQ || !idx || !scale || !shift || !out) return DGX_EINVAL;
    if (B < 1 || N < 1 || k < 1 || Co < 1 || ldpq < 2 * Co || ldo < Co) return DGX_EINVAL;
    const int tiles = (N + EG_WAVES * EG_PTS - 1) / (EG_WAVES * EG_PTS);
    dim3 grid(dgx_xcd_cloud_grid(B, tiles), (Co + 63) / 64);
    hipLaunchKernelGGL((edge_gather_kernel<true>), grid, dim3(256), 0, dgx_stream(stream), PQ, ldpq, idx, B, N, k,
                       Co, tiles, scale, shift, slope, (float*)nullptr, (uint8_t*)nullptr, (float*)nullptr,
                       (float*)nullptr, out, ldo);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_bn_finalize_f32(const float* partials, int nblk, int Co, double count, const float* gamma,
                        const float* beta, float* running_mean, float* running_var, double momentum, double eps,
                        float* scale, float* shift, float* mean, float* invstd, void* stream) {
    if (!partials || nblk < 1 || Co < 1 || count <= 0.0 || !scale || !shift) return DGX_EINVAL;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((Co + 255) / 256), dim3(256), 0, dgx_stream(stream), partials, nblk,
                       Co, count, gamma, beta, running_mean, running_var, momentum, eps, scale, shift, mean, invstd);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_bn_eval_affine_f32(int Co, const float* gamma, const float* beta, const float* running_mean,
                           const float* running_var, double eps, float* scale, float* shift, void* stream) {
    if (Co < 1 || !running_mean || !running_var || !scale || !shift) return DGX_EINVAL;
    hipLaunchKernelGGL(bn_eval_affine_kernel, dim3((Co + 255) / 256), dim3(256), 0, dgx_stream(stream), Co, gamma,
                       beta, running_mean, running_var, eps, scale, shift);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_bn_lrelu_apply_f32(const float* ysel, int M, int Co, const float* scale, const float* shift, float slope,
                           float* out, int ldo, void* stream) {
    if (!ysel || !scale || !shift || !out || M < 0 || Co < 1 || ldo < Co) return DGX_EINVAL;
    int64_t total = (int64_t)M * Co;
    if (total == 0) return DGX_OK;
    hipLaunchKernelGGL(bn_lrelu_apply_kernel, dim3(grid_for(total, 256)), dim3(256), 0, dgx_stream(stream), ysel, M,
                       Co, scale, shift, slope, out, ldo);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_bwd_dz_f32(const float* dY, int lddy, const float* ysel, int M, int Co, const float* scale,
                        const float* shift, const float* mean, const float* invstd, float slope, float* dz,
                        float* partials, int nblk_hint, void* stream) {
    if (!dY || !ysel || !scale || !shift || !mean || !invstd || !dz || !partials) return DGX_EINVAL;
    if (M < 1 || Co < 1 || lddy < Co || nblk_hint < 1) return DGX_EINVAL;
    const int rows = (M + nblk_hint - 1) / nblk_hint;
    dim3 grid(nblk_hint, (Co + 63) / 64);
    hipLaunchKernelGGL(edge_bwd_dz_kernel, grid, dim3(256), 0, dgx_stream(stream), dY, lddy, ysel, M, Co, scale,
                       shift, mean, invstd, slope, dz, partials, rows);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_bn_bwd_finalize_f32(const float* partials, int nblk, int Co, double count, const float* scale,
                            const float* mean, const float* invstd, float* dgamma, float* dbeta, float* c0,
                            float* c1, int accumulate, void* stream) {
    if (!partials || nblk < 1 || Co < 1 || count <= 0.0 || !scale || !mean || !invstd || !c0 || !c1)
        return DGX_EINVAL;
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((Co + 255) / 256), dim3(256), 0, dgx_stream(stream), partials,
                       nblk, Co, count, scale, mean, invstd, dgamma, dbeta, c0, c1, accumulate);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

size_t dgx_graph_reverse_workspace_bytes(int B, int N, int k) {
    (void)k;
    return 2 * (size_t)B * (size_t)N * sizeof(int32_t);
}

int dgx_graph_reverse(const int32_t* idx, int B, int N, int k, int32_t* rowptr, int32_t* edges, void* workspace,
                      size_t workspace_bytes, void* stream) {
    if (!idx || !rowptr || !edges || !workspace || B < 1 || N < 1 || k < 1 || k > 64) return DGX_EINVAL;
    if (workspace_bytes < dgx_graph_reverse_workspace_bytes(B, N, k)) return DGX_EINVAL;
    const int64_t M = (int64_t)B * N;
    if (M >= (1LL << 25)) return DGX_EUNSUPPORTED;
    hipStream_t st = dgx_stream(stream);
    int32_t* cnt = static_cast<int32_t*>(workspace);
    int32_t* cursor = cnt + M;
    if (hipMemsetAsync(cnt, 0, M * sizeof(int32_t), st) != hipSuccess) return DGX_ELAUNCH;
    const int64_t E = M * k;
    hipLaunchKernelGGL(rev_count_kernel, dim3(grid_for(E, 256)), dim3(256), 0, st, idx, B, N, k, cnt);
    hipLaunchKernelGGL(rev_scan_kernel, dim3(1), dim3(1024), 0, st, cnt, (int)M, rowptr, cursor);
    hipLaunchKernelGGL(rev_fill_kernel, dim3(grid_for(E, 256)), dim3(256), 0, st, idx, B, N, k, cursor, edges);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_bwd_scatter_f32(const float* PQ, int ldpq, const int32_t* idx, const int32_t* rowptr,
                             const int32_t* edges, const uint8_t* arg, const float* dz, const float* sumP, int B,
                             int N, int k, int Co, const float* scale, const float* c0, const float* c1, float* dPQ,
                             void* stream) {
    (void)idx;
    if (!PQ || !rowptr || !edges || !arg || !dz || !sumP || !scale || !c0 || !c1 || !dPQ) return DGX_EINVAL;
    if (B < 1 || N < 1 || k < 1 || k > 64 || Co < 1 || ldpq < 2 * Co) return DGX_EINVAL;
    const int tiles = (N + EG_WAVES * EG_PTS - 1) / (EG_WAVES * EG_PTS);
    dim3 grid(dgx_xcd_cloud_grid(B, tiles), (Co + 63) / 64);
    hipLaunchKernelGGL(edge_bwd_scatter_kernel, grid, dim3(256), 0, dgx_stream(stream), PQ, ldpq, rowptr, edges, arg,
                       dz, sumP, B, N, k, Co, tiles, scale, c0, c1, dPQ);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

}  // extern "C"
