// a3/a8 — the decomposed EdgeConv block (reference models/dgcnn.py:54-98).
//
// Reference, per block: edge tensor (B,2C,N,k) -> Conv2d(2C,Co,1) -> BN2d ->
// LeakyReLU -> max over k. Because the conv is linear and 1x1,
//     y(i,j) = W1 x_j + W2 x_i = P_j + Q_i,   P = X W1^T, Q = X W2^T,
// so the caller runs a per-point GEMM (k times fewer flops) into PQ (M x 2Co)
// and these kernels do the rest without ever forming an edge tensor:
//
//   gather    per (i,o): max_k P_j (min_k where gamma_o < 0 — BN's affine is
//             decreasing there), its slot, sum_k P_j, and partial sums of y and
//             y^2 over all B*N*k edge values (BN batch statistics).
//   finalize  statistics -> (a, b) affine, running stats (nn.BatchNorm rules).
//   apply     LeakyReLU(a*ysel + b) into the caller's concat buffer.
//   max_k LReLU(a y + b) = LReLU(a max_k y + b) for a >= 0 (min for a < 0).
//
// Backward follows BN's train-mode gradient: for every edge
//   dy_e = a*dz_e + c0 + c1*y_e   (dz_e nonzero only at the selected edge),
// so dQ_i = a*dz_i + k*c0 + c1*(sum_k P + k*Q_i) and dP_j sums over the
// in-edges of j (reverse kNN graph, built per cloud as a CSR).
//
// Memory layout / LDS tiling: a workgroup owns (cloud b, channel slice of CS
// channels, part of the points). It stages the cloud's whole slice of the
// gathered operand (P forward; Q and packed dz|slot backward) in LDS once, then
// every neighbour access is an LDS read: HBM/L2 traffic per block is the
// compulsory M*Co*(bytes) instead of M*k*Co*(bytes).
#include <math.h>
#include <stdlib.h>

#include <algorithm>

#include "common.h"

namespace {

constexpr int EC_THREADS = 512;
constexpr int EC_LDS_BYTES = 64 * 1024;   // operand slices per workgroup (2 workgroups per CU)
constexpr int GF_IPT = 8;                    // idx ints per thread per pass
constexpr int GF_ICAP = GF_IPT * EC_THREADS;

// V consecutive floats from LDS in one ds_read (b32 / b64 / b128).
template <int V>
__device__ __forceinline__ void lds_vec(const float* __restrict__ p, float (&r)[V]) {
    if constexpr (V == 1) {
        r[0] = p[0];
    } else if constexpr (V == 2) {
        const float2 t = *reinterpret_cast<const float2*>(p);
        r[0] = t.x;
        r[1] = t.y;
    } else {
#pragma unroll
        for (int u = 0; u < V; u += 4) {
            const float4 t = *reinterpret_cast<const float4*>(p + u);
            r[u] = t.x;
            r[u + 1] = t.y;
            r[u + 2] = t.z;
            r[u + 3] = t.w;
        }
    }
}

// V consecutive floats / bytes to or from HBM in 16/8-byte accesses (the
// caller guarantees V-alignment of the element offset and of the row stride).
template <int V>
__device__ __forceinline__ void gld_vec(const float* __restrict__ p, float (&r)[V]) {
    if constexpr (V == 1) {
        r[0] = p[0];
    } else if constexpr (V == 2) {
        const float2 t = *reinterpret_cast<const float2*>(p);
        r[0] = t.x;
        r[1] = t.y;
    } else {
#pragma unroll
        for (int u = 0; u < V; u += 4) {
            const float4 t = *reinterpret_cast<const float4*>(p + u);
            r[u] = t.x;
            r[u + 1] = t.y;
            r[u + 2] = t.z;
            r[u + 3] = t.w;
        }
    }
}
template <int V>
__device__ __forceinline__ void gst_vec(float* __restrict__ p, const float (&r)[V]) {
    if constexpr (V == 1) {
        p[0] = r[0];
    } else if constexpr (V == 2) {
        *reinterpret_cast<float2*>(p) = make_float2(r[0], r[1]);
    } else {
#pragma unroll
        for (int u = 0; u < V; u += 4)
            *reinterpret_cast<float4*>(p + u) = make_float4(r[u], r[u + 1], r[u + 2], r[u + 3]);
    }
}
template <int V>
__device__ __forceinline__ void gst_u8(uint8_t* __restrict__ p, const int (&r)[V]) {
    if constexpr (V == 1) {
        p[0] = (uint8_t)r[0];
    } else if constexpr (V == 2) {
        *reinterpret_cast<uint16_t*>(p) = (uint16_t)(r[0] | (r[1] << 8));
    } else {
#pragma unroll
        for (int u = 0; u < V; u += 4)
            *reinterpret_cast<uint32_t*>(p + u) =
                (uint32_t)r[u] | ((uint32_t)r[u + 1] << 8) | ((uint32_t)r[u + 2] << 16) | ((uint32_t)r[u + 3] << 24);
    }
}

template <int V>
__device__ __forceinline__ void gst_bf16(__bf16* __restrict__ p, const float (&r)[V]) {
    typedef __bf16 h4 __attribute__((ext_vector_type(4)));
    if constexpr (V % 4 == 0) {
#pragma unroll
        for (int u = 0; u < V; u += 4) *reinterpret_cast<h4*>(p + u) = h4{(__bf16)r[u], (__bf16)r[u + 1],
                                                                          (__bf16)r[u + 2], (__bf16)r[u + 3]};
    } else {
#pragma unroll
        for (int u = 0; u < V; ++u) p[u] = (__bf16)r[u];
    }
}

// Work split inside a channel slice of CS channels: TPP threads per point,
// V = CS / TPP consecutive channels per thread (one vector LDS read per
// neighbour), PP_MAX points per pass.
template <int CS>
struct SliceSplit {
    static constexpr int TPP = CS >= 4 ? 4 : CS;
    static constexpr int V = CS / TPP;
    static constexpr int PP_MAX = EC_THREADS / TPP;
};

// ------------------------------------------------------------- forward -----
// grid (B * nparts, ceil(Co / CS)); partial-stat row = blockIdx.x.
// Stage rows [0,N) x columns [col0, col0+CS) of a row-major matrix (row stride
// ld floats) into LDS [N][CS]; 16-byte loads when the slice is 16-byte aligned.
// With `dir` each column is multiplied by the sign of dir[col] (+-1, exact),
// so the forward gather's per-channel max-or-min becomes a plain max.
// SWZ (CS = 8 only): the two 16-byte halves of row n are stored swapped when
// bit 2 of n is set, so 16-byte reads of one half from random rows spread over
// all eight 16-byte bank groups instead of the four that 32-byte rows map one
// half to (fewer LDS bank conflicts in the backward scatter's gathers).
template <int CS, int THREADS, bool SWZ = false>
__device__ __forceinline__ void stage_slice(float* __restrict__ dst, const float* __restrict__ src, int64_t ld,
                                            int N, int col0, int ncols, bool vec4,
                                            const float* __restrict__ dir = nullptr) {
    static_assert(!SWZ || CS == 8, "swizzled rows are 2 x 16 bytes");
    const int t = threadIdx.x;
    auto sgn = [&](int c) { return (dir && col0 + c < ncols && dir[col0 + c] < 0.f) ? -1.f : 1.f; };
    constexpr int Q = CS >= 4 ? CS / 4 : 1;
    static_assert(THREADS % Q == 0, "a thread stages one column group");
    if (CS % 4 == 0 && vec4 && col0 + CS <= ncols) {
        const int qt = t % Q;  // this thread's column group, the same on every trip
        const float4 sg = make_float4(sgn(4 * qt), sgn(4 * qt + 1), sgn(4 * qt + 2), sgn(4 * qt + 3));
        const int total = N * Q;
        int e = t;
        for (; e + 3 * THREADS < total; e += 4 * THREADS) {  // 4 independent 16-byte loads in flight
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int ee = e + u * THREADS, n = ee / Q;
                v[u] = *reinterpret_cast<const float4*>(src + (int64_t)n * ld + col0 + 4 * qt);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int ee = e + u * THREADS;
                const int pos = SWZ ? (ee ^ ((ee >> 3) & 1)) : ee;  // ee = 2n + q: q ^ bit 2 of n
                reinterpret_cast<float4*>(dst)[pos] =
                    make_float4(v[u].x * sg.x, v[u].y * sg.y, v[u].z * sg.z, v[u].w * sg.w);
            }
        }
        for (; e < total; e += THREADS) {
            const int n = e / Q;
            const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)n * ld + col0 + 4 * qt);
            const int pos = SWZ ? (e ^ ((e >> 3) & 1)) : e;
            reinterpret_cast<float4*>(dst)[pos] = make_float4(v.x * sg.x, v.y * sg.y, v.z * sg.z, v.w * sg.w);
        }
    } else {
        for (int e = t; e < N * CS; e += THREADS) {
            const int n = e / CS, c = e - n * CS;
            const int pos = SWZ ? n * CS + (c ^ (((n >> 2) & 1) << 2)) : e;
            dst[pos] = (col0 + c < ncols) ? src[(int64_t)n * ld + col0 + c] * sgn(c) : 0.f;
        }
    }
}

template <int CS, bool EVAL>
__global__ __launch_bounds__(EC_THREADS) void edge_gather_lds_kernel(
    const float* __restrict__ PQ, int ldpq, const int32_t* __restrict__ idx, int B, int N, int k, int Co, int nparts,
    const float* __restrict__ sel_sign, const float* __restrict__ shift, float slope, float* __restrict__ ysel,
    uint8_t* __restrict__ arg, float* __restrict__ sumP, float* __restrict__ partials, float* __restrict__ out,
    int ldo) {
    constexpr int TPP = SliceSplit<CS>::TPP, V = SliceSplit<CS>::V;
    extern __shared__ float lds[];  // [N][CS] slice of P | idx rows of a pass; then the stat reduction
    int b, part, slice;
    if (!dgx_xcd_slice_map(blockIdx.x, B, nparts, (Co + CS - 1) / CS, b, part, slice)) return;
    const int o0 = slice * CS;
    const int prow = b * nparts + part;  // partial-stat row
    const int t = threadIdx.x;
    const int64_t base = (int64_t)b * N;
    const int per = (N + nparts - 1) / nparts;
    const int n_beg = part * per, n_end = min(N, n_beg + per);
    // P slice with each channel's sign of the BN scale folded in: max over k of
    // dir*P is max_k P (dir = +1) or -min_k P (dir = -1), one compare per value
    stage_slice<CS, EC_THREADS>(lds, PQ + base * ldpq, ldpq, N, o0, Co, (ldpq % 4) == 0 && (o0 % 4) == 0, sel_sign);

    // Pass = PP consecutive points; their idx rows (PP*k ints, contiguous in
    // HBM) are staged in LDS, the next pass's rows prefetched into registers
    // while the current pass computes.
    const int PP = min(SliceSplit<CS>::PP_MAX, GF_ICAP / k);
    int* gbuf = reinterpret_cast<int*>(lds + N * CS);
    const int npass = n_end > n_beg ? (n_end - n_beg + PP - 1) / PP : 0;
    const int gtot = PP * k;
    int pre[GF_IPT];
    auto load_rows = [&](int p) {
        const int64_t r0 = (base + n_beg + (int64_t)p * PP) * k;
        const int lim = (min(n_end, n_beg + (p + 1) * PP) - n_beg - p * PP) * k;
#pragma unroll
        for (int u = 0; u < GF_IPT; ++u) {
            const int e = t + u * EC_THREADS;
            pre[u] = (e < gtot && e < lim) ? idx[r0 + e] : 0;
        }
    };
    auto store_rows = [&]() {
#pragma unroll
        for (int u = 0; u < GF_IPT; ++u) {
            const int e = t + u * EC_THREADS;
            if (e < gtot) gbuf[e] = pre[u];
        }
    };

    const int tp = t % TPP, pl = t / TPP;
    const int c0 = tp * V;          // first channel of this thread within the slice
    float sgn[V], dir[V], shv[V];  // sel value (scale in EVAL), its sign +-1, shift
    bool okc[V];
#pragma unroll
    for (int u = 0; u < V; ++u) {
        okc[u] = o0 + c0 + u < Co;
        sgn[u] = okc[u] ? sel_sign[o0 + c0 + u] : 1.f;
        dir[u] = sgn[u] < 0.f ? -1.f : 1.f;
        shv[u] = (EVAL && okc[u]) ? shift[o0 + c0 + u] : 0.f;
    }
    // whole-vector HBM accesses when all V channels exist and rows stay aligned
    const bool vec = okc[V - 1] && (Co % 4) == 0 && (ldpq % 4) == 0;
    float acc1[V], acc2[V];
#pragma unroll
    for (int u = 0; u < V; ++u) { acc1[u] = 0.f; acc2[u] = 0.f; }
    if (npass > 0) load_rows(0);
    __syncthreads();  // slice staged
    if (npass > 0) store_rows();
    __syncthreads();
    for (int p = 0; p < npass; ++p) {
        if (p + 1 < npass) load_rows(p + 1);
        const int n = n_beg + p * PP + pl;
        if (pl < PP && n < n_end && okc[0]) {
            const int64_t i = base + n;
            const int* __restrict__ row = gbuf + pl * k;
            float qv[V];  // HBM read issued before the neighbour loop
            if (vec) {
                gld_vec<V>(PQ + i * ldpq + Co + o0 + c0, qv);
            } else {
#pragma unroll
                for (int u = 0; u < V; ++u) qv[u] = okc[u] ? PQ[i * ldpq + Co + o0 + c0 + u] : 0.f;
            }
            float best[V], s[V], s2[V];
            int barg[V];
#pragma unroll
            for (int u = 0; u < V; ++u) {
                best[u] = -INFINITY;
                s[u] = 0.f;
                s2[u] = 0.f;
                barg[u] = 0;
            }
            // values are dir*P: strict '>' keeps the first extremal slot
            auto take = [&](int j, int kk) {
                float v[V];
                lds_vec<V>(lds + j * CS + c0, v);
#pragma unroll
                for (int u = 0; u < V; ++u) {
                    const bool better = v[u] > best[u];
                    best[u] = better ? v[u] : best[u];
                    barg[u] = better ? kk : barg[u];
                    s[u] += v[u];
                    s2[u] = fmaf(v[u], v[u], s2[u]);
                }
            };
            int kk = 0;
            for (; kk + 4 <= k; kk += 4) {
                const int j0 = row[kk], j1 = row[kk + 1], j2 = row[kk + 2], j3 = row[kk + 3];
                take(j0, kk);
                take(j1, kk + 1);
                take(j2, kk + 2);
                take(j3, kk + 3);
            }
            for (; kk < k; ++kk) take(row[kk], kk);
            float yv[V];
#pragma unroll
            for (int u = 0; u < V; ++u) {
                const float q = qv[u];
                best[u] *= dir[u];  // back to P: the selected P_j (exact sign flips)
                s[u] *= dir[u];
                yv[u] = best[u] + q;
                if (EVAL) {
                    yv[u] = lrelu(fmaf(sgn[u], yv[u], shv[u]), slope);
                } else if (okc[u]) {
                    acc1[u] += fmaf((float)k, q, s[u]);                      // sum_k y
                    acc2[u] += s2[u] + q * fmaf(2.f, s[u], (float)k * q);    // sum_k y^2
                }
            }
            const int oc = o0 + c0;
            if (vec && !EVAL) {
                gst_vec<V>(ysel + i * Co + oc, yv);
                gst_vec<V>(sumP + i * Co + oc, s);
                gst_u8<V>(arg + i * Co + oc, barg);
            } else if (vec && (ldo % 4) == 0) {
                gst_vec<V>(out + i * ldo + oc, yv);
            } else {
#pragma unroll
                for (int u = 0; u < V; ++u) {
                    if (!okc[u]) continue;
                    if (EVAL) {
                        out[i * ldo + oc + u] = yv[u];
                    } else {
                        ysel[i * Co + oc + u] = yv[u];
                        arg[i * Co + oc + u] = (uint8_t)barg[u];
                        sumP[i * Co + oc + u] = s[u];
                    }
                }
            }
        }
        __syncthreads();
        if (p + 1 < npass) {
            store_rows();
            __syncthreads();
        }
    }
    if (EVAL) return;
    // reduce over the threads that share a channel: red[(2u + s)][thread]
    float* red = lds;
#pragma unroll
    for (int u = 0; u < V; ++u) {
        red[(2 * u) * EC_THREADS + t] = acc1[u];
        red[(2 * u + 1) * EC_THREADS + t] = acc2[u];
    }
    __syncthreads();
    if (t < CS && o0 + t < Co) {
        const int tpc = t / V, uc = t % V;
        float r1 = 0.f, r2 = 0.f;
        for (int w = tpc; w < EC_THREADS; w += TPP) {
            r1 += red[(2 * uc) * EC_THREADS + w];
            r2 += red[(2 * uc + 1) * EC_THREADS + w];
        }
        partials[(int64_t)prow * 2 * Co + o0 + t] = r1;
        partials[(int64_t)prow * 2 * Co + Co + o0 + t] = r2;
    }
}

// one wave per channel (4 channels per block): fp64 sums of the partial rows
// (fp32 per-block partials, or fp64 global sums after a SyncBatchNorm
// all-reduce), lanes strided over the rows then a shuffle tree — no barriers
template <typename T>
__global__ __launch_bounds__(256) void bn_finalize_kernel(const T* __restrict__ partials, int nrows, int Co,
                                                          double count, const float* __restrict__ gamma,
                                                          const float* beta, const float* rmean,
                                                          const float* rvar, double momentum, double eps,
                                                          float* __restrict__ scale, float* __restrict__ shift,
                                                          float* __restrict__ mean_out,
                                                          float* __restrict__ invstd_out,
                                                          const int64_t* nbt,
                                                          float* rmean_new, float* rvar_new, int64_t* nbt_new) {
    const int t = threadIdx.x & 63, o = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (nbt && o == 0 && t == 0) *nbt_new = *nbt + 1;  // BatchNorm.num_batches_tracked, no extra launch
    if (o >= Co) return;
    double s1 = 0.0, s2 = 0.0;
    for (int i = t; i < nrows; i += 64) {
        s1 += (double)partials[(int64_t)i * 2 * Co + o];
        s2 += (double)partials[(int64_t)i * 2 * Co + Co + o];
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
        s1 += __shfl_xor(s1, m);
        s2 += __shfl_xor(s2, m);
    }
    if (t != 0) return;
    // count < 0: the element count follows the sums on the device (SyncBatchNorm:
    // all-reduced with them, never read back to the host)
    if (count < 0.0) count = (double)partials[(int64_t)nrows * 2 * Co];
    // momentum < 0: nn.BatchNorm's cumulative average (momentum=None), factor
    // 1 / (num_batches_tracked + 1) read here instead of on the host (the
    // counter input is only read: the caller passes a separate nbt_new)
    if (momentum < 0.0) momentum = nbt ? 1.0 / (double)(*nbt + 1) : 0.0;
    const double mean = s1 / count;
    double var = s2 / count - mean * mean;
    if (var < 0.0) var = 0.0;
    const double invstd = 1.0 / sqrt(var + eps);
    const double a = (gamma ? (double)gamma[o] : 1.0) * invstd;
    scale[o] = (float)a;
    shift[o] = (float)((beta ? (double)beta[o] : 0.0) - mean * a);
    if (mean_out) mean_out[o] = (float)mean;
    if (invstd_out) invstd_out[o] = (float)invstd;
    if (rmean) rmean_new[o] = (float)((1.0 - momentum) * (double)rmean[o] + momentum * mean);
    if (rvar) {
        const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
        rvar_new[o] = (float)((1.0 - momentum) * (double)rvar[o] + momentum * unbiased);
    }
}

__global__ void bn_eval_affine_kernel(int Co, const float* __restrict__ gamma, const float* __restrict__ beta,
                                      const float* __restrict__ rmean, const float* __restrict__ rvar,
                                      double eps, float* __restrict__ scale, float* __restrict__ shift) {
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= Co) return;
    const float invstd = 1.0f / sqrtf(rvar[o] + (float)eps);
    const float a = (gamma ? gamma[o] : 1.f) * invstd;
    scale[o] = a;
    shift[o] = (beta ? beta[o] : 0.f) - rmean[o] * a;
}

// out16 (optional): the same values rounded to bf16 (RNE) at the same
// position of a bf16 twin of the output buffer — the GEMM operand copy of the
// concat buffer, written here so no conversion pass re-reads HBM.
__global__ void bn_lrelu_apply_kernel(const float* __restrict__ ysel, int M, int Co,
                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                      float slope, float* __restrict__ out, int ldo, __bf16* __restrict__ out16) {
    const int64_t total = (int64_t)M * Co;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int o = (int)(t % Co);
        const int64_t i = t / Co;
        const float v = lrelu(fmaf(scale[o], ysel[t], shift[o]), slope);
        out[i * ldo + o] = v;
        if (out16) out16[i * ldo + o] = (__bf16)v;
    }
}

// 4 channels per thread (Co, ldo multiples of 4): 16-byte loads and stores,
// 8-byte bf16 twin stores.
__global__ void bn_lrelu_apply4_kernel(const float* __restrict__ ysel, int M, int Co,
                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                       float slope, float* __restrict__ out, int ldo, __bf16* __restrict__ out16) {
    const int cq = Co >> 2;
    const int64_t total = (int64_t)M * cq;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int o = (int)(t % cq) * 4;
        const int64_t i = t / cq;
        const float4 y = *reinterpret_cast<const float4*>(ysel + i * Co + o);
        const float4 a = *reinterpret_cast<const float4*>(scale + o);
        const float4 b = *reinterpret_cast<const float4*>(shift + o);
        float v[4] = {lrelu(fmaf(a.x, y.x, b.x), slope), lrelu(fmaf(a.y, y.y, b.y), slope),
                      lrelu(fmaf(a.z, y.z, b.z), slope), lrelu(fmaf(a.w, y.w, b.w), slope)};
        gst_vec<4>(out + i * ldo + o, v);
        if (out16) gst_bf16<4>(out16 + i * ldo + o, v);
    }
}

// ------------------------------------------------------------ backward -----
// dz = dL/dz at the selected edge (z = BN(y)), fp32, and per-row-block
// partials (sum dz, sum dz*yhat). grid (nrows, ceil(Co/64)).
__global__ __launch_bounds__(256) void edge_bwd_dz_kernel(
    const float* __restrict__ dY, int lddy, const float* __restrict__ ysel, int M, int Co,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ invstd, float slope, float* __restrict__ dz, float* __restrict__ partials,
    int rows_per_blk, const uint8_t* __restrict__ arg) {
    __shared__ float red[2][4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int o = blockIdx.y * 64 + lane;
    const bool ok = o < Co;
    float acc1 = 0.f, acc2 = 0.f;
    if (ok) {
        const float a = scale[o], sh = shift[o], mu = mean[o], is = invstd[o];
        const int64_t i0 = (int64_t)blockIdx.x * rows_per_blk;
        // DZ_U rows per wave per iteration, loads issued together (the pass is
        // latency-bound with one row in flight); accumulation order unchanged
        constexpr int DZ_U = 4;
        for (int r0 = wave; r0 < rows_per_blk; r0 += 4 * DZ_U) {
            float yv[DZ_U], gv[DZ_U];
            uint32_t sv[DZ_U];
#pragma unroll
            for (int u = 0; u < DZ_U; ++u) {
                const int64_t i = min(i0 + r0 + 4 * u, (int64_t)M - 1);
                yv[u] = ysel[i * Co + o];
                gv[u] = dY[i * lddy + o];
                sv[u] = arg ? arg[i * Co + o] : 0u;
            }
#pragma unroll
            for (int u = 0; u < DZ_U; ++u) {
                const int64_t i = i0 + r0 + 4 * u;
                if (r0 + 4 * u >= rows_per_blk || i >= M) break;
                const float z = fmaf(a, yv[u], sh);
                const float d = gv[u] * (z > 0.f ? 1.f : slope);
                // packed form: the selected slot replaces the low 6 mantissa bits
                // (18 significant bits left; the scatter reads one word per edge)
                dz[i * Co + o] = arg ? __uint_as_float((__float_as_uint(d) & ~63u) | sv[u]) : d;
                acc1 += d;
                acc2 = fmaf(d, (yv[u] - mu) * is, acc2);
            }
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

// The same dz and partials for a CHANNEL-major dY (B, Co, N) — the gradient of
// a (B, C, N) module output that the engine keeps point-major (PositionEmbedding's
// edge stage, layers.py:52): block = (cloud, 64-point tile) x 64-channel tile,
// dY tile loaded along n (coalesced), transposed through LDS, then lanes =
// channels as in edge_bwd_dz_kernel. Partial row = blockIdx.x.
__global__ __launch_bounds__(256) void edge_bwd_dz_cm_kernel(
    const float* __restrict__ dY, const float* __restrict__ ysel, int N, int Co, int ntn,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ invstd, float slope, float* __restrict__ dz, float* __restrict__ partials) {
    __shared__ float t[64][65];
    __shared__ float red[2][4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x / ntn, n0 = (blockIdx.x - b * ntn) * 64, c0 = blockIdx.y * 64;
    for (int r = wave; r < 64; r += 4) {
        const int c = c0 + r, n = n0 + lane;
        t[r][lane] = (c < Co && n < N) ? dY[((int64_t)b * Co + c) * N + n] : 0.f;
    }
    __syncthreads();
    const int o = c0 + lane;
    const bool ok = o < Co;
    float acc1 = 0.f, acc2 = 0.f;
    if (ok) {
        const float a = scale[o], sh = shift[o], mu = mean[o], is = invstd[o];
        for (int rr = wave; rr < 64 && n0 + rr < N; rr += 4) {
            const int64_t i = (int64_t)b * N + n0 + rr;
            const float y = ysel[i * Co + o];
            const float z = fmaf(a, y, sh);
            const float d = t[lane][rr] * (z > 0.f ? 1.f : slope);
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

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const T* __restrict__ partials, int nrows,
                                                              int Co, double count, const float* __restrict__ scale,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ c0, float* __restrict__ c1,
                                                              int accumulate) {
    const int t = threadIdx.x & 63, o = blockIdx.x * 4 + (threadIdx.x >> 6);   // one wave per channel
    if (o >= Co) return;
    double s1 = 0.0, s2 = 0.0;
    for (int i = t; i < nrows; i += 64) {
        s1 += (double)partials[(int64_t)i * 2 * Co + o];
        s2 += (double)partials[(int64_t)i * 2 * Co + Co + o];
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
        s1 += __shfl_xor(s1, m);
        s2 += __shfl_xor(s2, m);
    }
    if (t != 0) return;
    if (count < 0.0) count = (double)partials[(int64_t)nrows * 2 * Co];   // device-side count, as above
    if (dbeta) dbeta[o] = (float)(accumulate ? (double)dbeta[o] + s1 : s1);
    if (dgamma) dgamma[o] = (float)(accumulate ? (double)dgamma[o] + s2 : s2);
    const double a = scale[o], mu = mean[o], is = invstd[o];
    const double g1 = s1 / count, g2 = s2 / count;
    c0[o] = (float)(a * (-g1 + g2 * mu * is));
    c1[o] = (float)(-a * g2 * is);
}

// Reverse graph, parallel form: P workgroups per cloud, workgroup p owns the
// targets j in [p*R, p*R + R). It reads the cloud's whole index list (L2
// resident), counts its own targets' in-edges and the edges that land before
// its range (its global list offset), places edge ids with LDS atomics, then
// orders every list by a rank sort (rank = number of smaller ids in the same
// list: independent LDS reads, no serial chain), so the lists come out
// ascending and the backward's summation order is deterministic. A workgroup
// whose range holds more than RG_CAP edges (degenerate clouds, e.g. all points
// equal) places them in HBM and sorts each list there instead.
constexpr int RG_THREADS = 512;
#ifndef RG_CAP_DEF
#define RG_CAP_DEF 12288
#endif
#ifndef RG_MIN_WG
#define RG_MIN_WG 512
#endif
constexpr int RG_CAP = RG_CAP_DEF;
constexpr int RG_U = 8;  // independent index loads in flight per thread

__device__ __forceinline__ int32_t block_sum_rg(int32_t v, int32_t* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    int32_t t = 0;
    for (int u = 0; u < RG_THREADS / 64; ++u) t += red[u];
    return t;
}

// Several graphs (the kNN graphs of a DGCNN's blocks, same B, N, k) in one
// launch: blockIdx.x = graph * (B * P) + cloud * P + range.
constexpr int RG_MAX_GRAPHS = 8;
struct RevGraphJobs {
    const int32_t* idx[RG_MAX_GRAPHS];
    int32_t* rowptr[RG_MAX_GRAPHS];
    int32_t* edges[RG_MAX_GRAPHS];
};

__global__ __launch_bounds__(RG_THREADS) void rev_graph_par_kernel(RevGraphJobs jobs, int G, int B, int N, int k,
                                                                   int P, int cap) {
    extern __shared__ int32_t rg[];
    // (graph, cloud) items with all P ranges of one item on one XCD
    // (dgx_xcd_cloud_map): the item's index list, which every range scans twice,
    // is fetched into that XCD's L2 once instead of once per range
    int item, p;
    if (!dgx_xcd_cloud_map(blockIdx.x, G * B, P, item, p)) return;
    const int gi = item / B, b = item - gi * B;
    const int32_t* __restrict__ idx = jobs.idx[gi];
    int32_t* __restrict__ rowptr = jobs.rowptr[gi];
    int32_t* __restrict__ edges = jobs.edges[gi];
    const int R = (N + P - 1) / P;
    int32_t* cnt = rg;                 // [R] in-degree -> fill cursor
    int32_t* start = cnt + R;          // [R] local list starts
    int32_t* red = start + R;          // [RG_THREADS / 64 + 2]
    int32_t* list = red + RG_THREADS / 64 + 2;   // [cap] edge ids
    int32_t* ltg = list + cap;                    // [cap] local target of each slot
    const int t = threadIdx.x;
    const int j0 = p * R, j1 = min(N, j0 + R), nr = max(0, j1 - j0);
    const int64_t base = (int64_t)b * N;
    const int32_t* __restrict__ ib = idx + base * k;
    const int E = N * k;
    const int32_t ebase = (int32_t)(base * k);
    for (int r = t; r < nr; r += RG_THREADS) cnt[r] = 0;
    __syncthreads();
    int32_t before = 0;
    // the cloud's index list is read in batches of RG_U independent loads per
    // thread (a dependent load per iteration would leave the loop latency-bound)
    for (int e0 = 0; e0 < E; e0 += RG_U * RG_THREADS) {
        int32_t jv[RG_U];
#pragma unroll
        for (int u = 0; u < RG_U; ++u) {
            const int e = e0 + u * RG_THREADS + t;
            jv[u] = e < E ? ib[e] : INT32_MAX;
        }
#pragma unroll
        for (int u = 0; u < RG_U; ++u) {
            const int j = jv[u];
            if (j < j0) ++before;
            else if (j < j1) atomicAdd(&cnt[j - j0], 1);
        }
    }
    before = block_sum_rg(before, red);
    // exclusive scan of cnt over the range: thread-contiguous chunks + block scan of chunk sums
    const int per = (nr + RG_THREADS - 1) / RG_THREADS;
    const int lo = min(nr, t * per), hi = min(nr, lo + per);
    int32_t s = 0;
    for (int r = lo; r < hi; ++r) s += cnt[r];
    // block exclusive scan of s (wave scan + wave totals)
    const int lane = t & 63, w = t >> 6;
    int32_t inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t v = __shfl_up(inc, o);
        if (lane >= o) inc += v;
    }
    __syncthreads();
    if (lane == 63) red[w] = inc;
    __syncthreads();
    int32_t wofs = 0;
    for (int u = 0; u < w; ++u) wofs += red[u];
    int32_t total = 0;
    for (int u = 0; u < RG_THREADS / 64; ++u) total += red[u];
    int32_t run = wofs + inc - s;
    for (int r = lo; r < hi; ++r) {
        const int32_t c = cnt[r];
        rowptr[base + j0 + r] = ebase + before + run;
        start[r] = run;
        cnt[r] = run;  // fill cursor
        run += c;
    }
    if (b == B - 1 && p == P - 1 && t == 0) rowptr[base + N] = (int32_t)((base + N) * k);
    __syncthreads();
    const bool in_lds = total <= cap;
    int32_t* out = in_lds ? list : edges + ebase + before;
    for (int e0 = 0; e0 < E; e0 += RG_U * RG_THREADS) {
        int32_t jv[RG_U];
#pragma unroll
        for (int u = 0; u < RG_U; ++u) {
            const int e = e0 + u * RG_THREADS + t;
            jv[u] = e < E ? ib[e] : INT32_MAX;
        }
#pragma unroll
        for (int u = 0; u < RG_U; ++u) {
            const int j = jv[u];
            if (j >= j0 && j < j1) {
                const int e = e0 + u * RG_THREADS + t;
                const int32_t pos = atomicAdd(&cnt[j - j0], 1);
                out[pos] = ((int32_t)(base + e / k) << 6) | (e % k);
                if (in_lds) ltg[pos] = j - j0;
            }
        }
    }
    __syncthreads();
    if (in_lds) {
        int32_t* dst = edges + ebase + before;
        for (int q = t; q < total; q += RG_THREADS) {
            const int32_t a = list[q];
            const int r = ltg[q];
            const int32_t beg = start[r], end = cnt[r];
            int32_t rank = 0;
            for (int32_t u = beg; u < end; ++u) rank += list[u] < a ? 1 : 0;
            dst[beg + rank] = a;
        }
    } else {
        for (int r = t; r < nr; r += RG_THREADS) {  // degenerate range: insertion sort in HBM
            const int32_t beg = start[r], end = cnt[r];
            for (int32_t a = beg + 1; a < end; ++a) {
                const int32_t v = out[a];
                int32_t q = a - 1;
                while (q >= beg && out[q] > v) { out[q + 1] = out[q]; --q; }
                out[q + 1] = v;
            }
        }
    }
}

// dPQ for every point: grid (B * nparts, ceil(Co / CS)), CS <= 8 channels per
// slice, one point per thread with all CS channels, so the per-edge work
// (edge-id decode, LDS addresses) is shared by CS channels. LDS holds the
// cloud's Q slice and dz slice (fp32, exact) and the selected slots (u8, the
// forward's arg) — 9 bytes per (point, channel) — plus the block's points in
// descending in-degree order: the in-degree of feature-space kNN graphs is
// skewed (hubs), and a wave's trip count is its largest in-degree, so waves
// take points of similar degree. Every point still sums its in-edges in its
// CSR (ascending edge id) order: results do not depend on the schedule.
//   dP_j = a * sum_{in-edges (i,s) of j, s = slot_i} dz_i
//          + deg_j c0 + c1 (deg_j P_j + sum_in Q_i)
//   dQ_i = a dz_i + k c0 + c1 (k Q_i + sum_k P_j)
constexpr int BW_EB = 16;         // in-edge ids loaded per batch
constexpr int BW_BUCKETS = 64;    // degree buckets of the in-block order
constexpr int BW_LDS_BYTES = 72 * 1024;  // Q | dz | slot slices (two workgroups per CU)

template <int CS>
__device__ __forceinline__ void lds_slots(const uint8_t* __restrict__ p, uint32_t (&w)[(CS + 3) / 4]) {
    if constexpr (CS == 16) {
        const uint4 t = *reinterpret_cast<const uint4*>(p);
        w[0] = t.x;
        w[1] = t.y;
        w[2] = t.z;
        w[3] = t.w;
    } else if constexpr (CS == 8) {
        const uint2 t = *reinterpret_cast<const uint2*>(p);
        w[0] = t.x;
        w[1] = t.y;
    } else if constexpr (CS == 4) {
        w[0] = *reinterpret_cast<const uint32_t*>(p);
    } else if constexpr (CS == 2) {
        w[0] = *reinterpret_cast<const uint16_t*>(p);
    } else {
        w[0] = p[0];
    }
}

// BN backward finalize folded into the scatter's prologue (no separate
// dgx_bn_bwd_finalize launch): every workgroup reduces the dz kernel's partial
// rows for its own CS channels in one fixed order (so all of a slice's
// workgroups hold bit-identical c0 / c1), the slice's first workgroup writes
// dgamma, dbeta, c0, c1. partials == nullptr: c0 / c1 are inputs.
struct BnBwdFin {
    const float* partials;   // (nrows, 2, Co): sum dz | sum dz*yhat
    int nrows;
    double count;
    const float* mean;
    const float* invstd;
    int eval;                // running-statistics forward: c0 = c1 = 0
    float* dgamma;
    float* dbeta;
    float* c0;
    float* c1;
};
constexpr int BW_FIN_LDS = 16 * 2 * 8 * sizeof(double) + 2 * 8 * sizeof(float);   // per-wave sums | c0 c1

// The scatter's per-channel constants a (BN scale), k0 = c0, k1 = c1 for the
// workgroup's CS channels: read, or (fin.partials) finalized from the dz
// pass's partial rows. scratch: BW_FIN_LDS bytes of LDS, 8-byte aligned.
template <int CS>
__device__ __forceinline__ void scatter_consts(const BnBwdFin& fin, int b, int part, int o0, int Co,
                                               const float* __restrict__ scale, const float* __restrict__ c0,
                                               const float* __restrict__ c1, void* scratch, float (&a)[CS],
                                               float (&k0)[CS], float (&k1)[CS]) {
    const int t = threadIdx.x;
    if (fin.partials) {
        // thread t sums rows g, g + G, ... of channel o0 + t % CS (fp64), lanes of a
        // wave with the same channel combine by xor shuffles, then the waves in order
        static_assert(CS <= 8 && EC_THREADS / 64 <= 16, "finalize scratch");
        double* wsum = reinterpret_cast<double*>(scratch);   // [wave][2][CS]
        float* kc = reinterpret_cast<float*>(wsum + 16 * 2 * 8);        // [2][CS]
        const int c = t % CS, g = t / CS;
        constexpr int G = EC_THREADS / CS;
        const int o = o0 + c;
        double s1 = 0.0, s2 = 0.0;
        if (o < Co) {
            const float* __restrict__ pp = fin.partials + o;
            int r = g;
            for (; r + 3 * G < fin.nrows; r += 4 * G) {   // 8 independent loads in flight
                float v1[4], v2[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    v1[u] = pp[(int64_t)(r + u * G) * 2 * Co];
                    v2[u] = pp[(int64_t)(r + u * G) * 2 * Co + Co];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    s1 += (double)v1[u];
                    s2 += (double)v2[u];
                }
            }
            for (; r < fin.nrows; r += G) {
                s1 += (double)pp[(int64_t)r * 2 * Co];
                s2 += (double)pp[(int64_t)r * 2 * Co + Co];
            }
        }
#pragma unroll
        for (int m = CS; m < 64; m <<= 1) {
            s1 += __shfl_xor(s1, m);
            s2 += __shfl_xor(s2, m);
        }
        const int lane = t & 63, wv = t >> 6;
        if (lane < CS) {
            wsum[(wv * 2) * CS + lane] = s1;
            wsum[(wv * 2 + 1) * CS + lane] = s2;
        }
        __syncthreads();
        if (t < CS) {
            double r1 = 0.0, r2 = 0.0;
            for (int w = 0; w < EC_THREADS / 64; ++w) {
                r1 += wsum[(w * 2) * CS + t];
                r2 += wsum[(w * 2 + 1) * CS + t];
            }
            float v0 = 0.f, v1 = 0.f;
            if (o0 + t < Co) {
                const double av = scale[o0 + t], mu = fin.mean[o0 + t], is = fin.invstd[o0 + t];
                const double g1 = r1 / fin.count, g2 = r2 / fin.count;
                if (!fin.eval) {
                    v0 = (float)(av * (-g1 + g2 * mu * is));
                    v1 = (float)(-av * g2 * is);
                }
                if (b == 0 && part == 0) {
                    if (fin.dbeta) fin.dbeta[o0 + t] = (float)r1;
                    if (fin.dgamma) fin.dgamma[o0 + t] = (float)r2;
                    fin.c0[o0 + t] = v0;
                    fin.c1[o0 + t] = v1;
                }
            }
            kc[t] = v0;
            kc[CS + t] = v1;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < CS; ++u) {
            a[u] = scale[min(o0 + u, Co - 1)];
            k0[u] = kc[u];
            k1[u] = kc[CS + u];
        }
    } else {
#pragma unroll
        for (int u = 0; u < CS; ++u) {
            const int o = min(o0 + u, Co - 1);
            a[u] = scale[o];
            k0[u] = c0[o];
            k1[u] = c1[o];
        }
    }
}

// SPLIT (with OUT16): dPQ as split bf16 planes, out_split = planes after the
// first (1: lo; 2: lo, hi) — a separate instantiation, so the bf16 and fp32
// forms' code is untouched by the extra stores
// TPP > 1 (few-cloud shards): TPP consecutive lanes share a point, each taking
// every TPP-th in-edge, their sums combined by an xor-shuffle tree (a fixed
// order: deterministic), so a block of 512 threads covers 512 / TPP points
// with short per-lane edge chains instead of 512 points' worth of threads of
// which most are idle at 64 points per block
template <int CS, bool OUT16, bool PACKED, bool SPLIT = false, int TPP = 1>
__global__ __launch_bounds__(EC_THREADS, 4) void edge_bwd_scatter_kernel(
    const float* __restrict__ PQ, int ldpq, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ edges,
    const float* __restrict__ dz, const uint8_t* __restrict__ arg, const float* __restrict__ sumP, int B, int N,
    int k, int Co, int nparts, const float* __restrict__ scale, const float* __restrict__ c0,
    const float* __restrict__ c1, void* __restrict__ dPQv, BnBwdFin fin, int out_split, int idcap) {
    static_assert(CS == 1 || CS == 2 || CS == 4 || CS == 8 || CS == 16, "slice width");
    constexpr int SW = (CS + 3) / 4;  // slot words per row
    float* __restrict__ dPQ = static_cast<float*>(dPQv);
    __bf16* __restrict__ dPQh = static_cast<__bf16*>(dPQv);
    // [N][CS] Q | [N][CS] dz | [N][CS] u8 slot (not PACKED) | order u16 [per] | buckets
    // PACKED: dz words carry the slot in their low 6 bits (dgx_edge_bwd_dz_packed_f32)
    extern __shared__ float lds[];
    float* qs = lds;
    float* ds = lds + N * CS;
    uint8_t* ss = reinterpret_cast<uint8_t*>(ds + N * CS);
    uint16_t* order = reinterpret_cast<uint16_t*>(PACKED ? ss : ss + ((N * CS + 15) & ~15));
    int b, part, slice;
    if (!dgx_xcd_slice_map(blockIdx.x, B, nparts, (Co + CS - 1) / CS, b, part, slice)) return;
    const int o0 = slice * CS;
    const int t = threadIdx.x;
    const int64_t base = (int64_t)b * N;
    const int per = (N + nparts - 1) / nparts;
    const int n_beg = part * per, n_end = min(N, n_beg + per);
    const int np = max(0, n_end - n_beg);
    int* bucket = reinterpret_cast<int*>(order + ((per + 7) & ~7));
    const bool full = o0 + CS <= Co;
    if (t < BW_BUCKETS) bucket[t] = 0;
    constexpr bool SWZ = CS == 8;
    // the part's in-edge ids (a contiguous CSR range) staged in LDS as 16-bit
    // (local source << 6 | slot) words when they fit idcap (block-uniform;
    // idcap > 0 only for N <= 1024): the in-edge loop then waits on LDS instead
    // of dependent global id batches
    const int32_t ibase = (int32_t)base;
    uint16_t* lid = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(bucket + BW_BUCKETS) + BW_FIN_LDS);
    int32_t e_lo = 0;
    bool idl = false;
    if (idcap > 0 && np > 0) {
        e_lo = rowptr[base + n_beg];
        const int32_t e_cnt = rowptr[base + n_end] - e_lo;
        idl = e_cnt <= idcap;
        if (idl)
            for (int e = t; e < e_cnt; e += EC_THREADS) {
                const int32_t w = edges[e_lo + e];
                lid[e] = (uint16_t)((((w >> 6) - ibase) << 6) | (w & 63));
            }
    }
    stage_slice<CS, EC_THREADS, SWZ>(qs, PQ + base * ldpq + Co, ldpq, N, o0, Co, (ldpq % 4) == 0 && (Co % 4) == 0);
    stage_slice<CS, EC_THREADS, SWZ>(ds, dz + base * Co, Co, N, o0, Co, (Co % 4) == 0);
    // row n of a swizzled slice: halves at 4 * (h ^ bit 2 of n)
    auto lds_row = [&](const float* __restrict__ arr, int n, float (&r)[CS]) {
        if constexpr (SWZ) {
            const int sw = ((n >> 2) & 1) << 2;
            const float4 a = *reinterpret_cast<const float4*>(arr + n * CS + sw);
            const float4 b = *reinterpret_cast<const float4*>(arr + n * CS + (4 ^ sw));
            r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
            r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
        } else {
            lds_vec<CS>(arr + n * CS, r);
        }
    };
    const uint8_t* __restrict__ ab = PACKED ? nullptr : arg + base * Co + o0;
    if (PACKED) {
    } else if (full && (Co % CS) == 0) {
        for (int n = t; n < N; n += EC_THREADS) {
            uint32_t w[SW];
            if constexpr (CS == 16) {
                *reinterpret_cast<uint4*>(ss + n * CS) = *reinterpret_cast<const uint4*>(ab + (int64_t)n * Co);
            } else if constexpr (CS == 8) {
                const uint2 v = *reinterpret_cast<const uint2*>(ab + (int64_t)n * Co);
                w[0] = v.x;
                w[1] = v.y;
                *reinterpret_cast<uint2*>(ss + n * CS) = make_uint2(w[0], w[1]);
            } else if constexpr (CS == 4) {
                *reinterpret_cast<uint32_t*>(ss + n * CS) = *reinterpret_cast<const uint32_t*>(ab + (int64_t)n * Co);
            } else if constexpr (CS == 2) {
                *reinterpret_cast<uint16_t*>(ss + n * CS) = *reinterpret_cast<const uint16_t*>(ab + (int64_t)n * Co);
            } else {
                ss[n] = ab[(int64_t)n * Co];
            }
            (void)w;
        }
    } else {
        for (int e = t; e < N * CS; e += EC_THREADS) {
            const int n = e / CS, c = e - n * CS;
            ss[e] = o0 + c < Co ? ab[(int64_t)n * Co + c] : (uint8_t)255;
        }
    }
    __syncthreads();  // buckets zeroed
    // in-block order: counting sort of the block's points by in-degree, descending
    for (int r = t; r < np; r += EC_THREADS) {
        const int64_t j = base + n_beg + r;
        const int deg = rowptr[j + 1] - rowptr[j];
        atomicAdd(&bucket[BW_BUCKETS - 1 - min(deg, BW_BUCKETS - 1)], 1);
    }
    __syncthreads();
    if (t < 64) {  // exclusive scan of the 64 bucket counts (one wave)
        const int c = bucket[t];
        int inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(inc, o);
            if (t >= o) inc += v;
        }
        bucket[t] = inc - c;
    }
    __syncthreads();
    for (int r = t; r < np; r += EC_THREADS) {
        const int64_t j = base + n_beg + r;
        const int deg = rowptr[j + 1] - rowptr[j];
        order[atomicAdd(&bucket[BW_BUCKETS - 1 - min(deg, BW_BUCKETS - 1)], 1)] = (uint16_t)r;
    }
    float a[CS], k0[CS], k1[CS];
    scatter_consts<CS>(fin, b, part, o0, Co, scale, c0, c1, bucket + BW_BUCKETS, a, k0, k1);
    const bool vec = full && (CS % 4) == 0 && (Co % 4) == 0 && (ldpq % 4) == 0;
    const float kf = (float)k;
    __syncthreads();
    // boustrophedon deal of the degree-sorted points: pass 2p takes ranks
    // t, pass 2p+1 ranks from the far end, so a thread's in-degree total (and a
    // wave's longest lane) is balanced instead of wave 0 holding every hub
    static_assert(TPP == 1 || TPP == 2 || TPP == 4 || TPP == 8, "lanes per point");
    constexpr int PPB = EC_THREADS / TPP;   // points per pass
    const int pl = t / TPP, sub = t % TPP;
    for (int it = 0; it * PPB < np; ++it) {
        const int r = it * PPB + ((it & 1) ? PPB - 1 - pl : pl);
        if (r >= np) continue;   // the TPP lanes of a point skip together
        const int n = n_beg + order[r];
        const int64_t j = base + n;
        const int32_t beg = rowptr[j], end = rowptr[j + 1];
        float pjv[CS], spv[CS];  // HBM reads issued before the edge loop hides their latency
        if (vec) {
            gld_vec<CS>(PQ + j * ldpq + o0, pjv);
            gld_vec<CS>(sumP + j * Co + o0, spv);
        } else {
#pragma unroll
            for (int u = 0; u < CS; ++u) {
                pjv[u] = o0 + u < Co ? PQ[j * ldpq + o0 + u] : 0.f;
                spv[u] = o0 + u < Co ? sumP[j * Co + o0 + u] : 0.f;
            }
        }
        float sq[CS], sd[CS];
#pragma unroll
        for (int u = 0; u < CS; ++u) { sq[u] = 0.f; sd[u] = 0.f; }
        auto edge = [&](int il, uint32_t slot) {
            float q[CS];
            lds_row(qs, il, q);
#pragma unroll
            for (int u = 0; u < CS; ++u) sq[u] += q[u];
            float d[CS];
            lds_row(ds, il, d);
            if constexpr (PACKED) {
#pragma unroll
                for (int u = 0; u < CS; ++u) {
                    const uint32_t wd = __float_as_uint(d[u]);
                    sd[u] += (wd & 63u) == slot ? __uint_as_float(wd & ~63u) : 0.f;
                }
            } else {
                uint32_t w[SW];
                lds_slots<CS>(ss + il * CS, w);
#pragma unroll
                for (int u = 0; u < CS; ++u) sd[u] += ((w[u >> 2] >> (8 * (u & 3))) & 0xffu) == slot ? d[u] : 0.f;
            }
        };
        if constexpr (TPP > 1) {
            // this lane's in-edges beg + sub + TPP * v, EB at a time; then the
            // point's sums over its TPP lanes
            constexpr int EB = BW_EB / TPP > 2 ? BW_EB / TPP : 2;
            for (int32_t u0 = beg + sub; u0 < end; u0 += TPP * EB) {
                int32_t ids[EB];
#pragma unroll
                for (int v = 0; v < EB; ++v) ids[v] = u0 + TPP * v < end ? edges[u0 + TPP * v] : 0;
#pragma unroll
                for (int v = 0; v < EB; ++v)
                    if (u0 + TPP * v < end) edge((ids[v] >> 6) - ibase, (uint32_t)(ids[v] & 63));
            }
#pragma unroll
            for (int m = 1; m < TPP; m <<= 1)
#pragma unroll
                for (int u = 0; u < CS; ++u) {
                    sq[u] += __shfl_xor(sq[u], m);
                    sd[u] += __shfl_xor(sd[u], m);
                }
        } else if (idl) {   // ids from LDS, EB at a time
            for (int32_t u0 = beg; u0 < end; u0 += BW_EB) {
                uint32_t ids[BW_EB];
#pragma unroll
                for (int v = 0; v < BW_EB; ++v) ids[v] = u0 + v < end ? lid[u0 + v - e_lo] : 0u;
#pragma unroll
                for (int v = 0; v < BW_EB; ++v)
                    if (u0 + v < end) edge((int)(ids[v] >> 6), ids[v] & 63u);
            }
        } else {
            // in-edge ids EB at a time, all loads issued before the first is used
            // (prefetching the next batch as well measured slower)
            for (int32_t u0 = beg; u0 < end; u0 += BW_EB) {
                int32_t ids[BW_EB];
#pragma unroll
                for (int v = 0; v < BW_EB; ++v) ids[v] = u0 + v < end ? edges[u0 + v] : 0;
#pragma unroll
                for (int v = 0; v < BW_EB; ++v)
                    if (u0 + v < end) edge((ids[v] >> 6) - ibase, (uint32_t)(ids[v] & 63));
            }
        }
        const float deg = (float)(end - beg);
        float qn[CS], dn[CS];
        lds_row(qs, n, qn);
        lds_row(ds, n, dn);
        if constexpr (PACKED) {
#pragma unroll
            for (int u = 0; u < CS; ++u) dn[u] = __uint_as_float(__float_as_uint(dn[u]) & ~63u);
        }
        float dp[CS], dq[CS];
#pragma unroll
        for (int u = 0; u < CS; ++u) {
            dp[u] = fmaf(a[u], sd[u], fmaf(k0[u], deg, k1[u] * fmaf(deg, pjv[u], sq[u])));
            dq[u] = fmaf(a[u], dn[u], fmaf(k0[u], kf, k1[u] * fmaf(kf, qn[u], spv[u])));
        }
        if (TPP > 1 && sub != 0) continue;   // one lane of the point stores
        if constexpr (SPLIT) {
            // the fp32 mode's split planes: hi = bf16(v) here, lo = bf16(v - hi) at
            // + B*N*2Co (dgx_split_bf16's rounding), the 3-pass GEMMs' operands
            const int64_t lo_off = (int64_t)B * N * 2 * Co;
            float dph[CS], dpl[CS], dqh[CS], dql[CS];
#pragma unroll
            for (int u = 0; u < CS; ++u) {
                dph[u] = (float)(__bf16)dp[u];
                dpl[u] = dp[u] - dph[u];
                dqh[u] = (float)(__bf16)dq[u];
                dql[u] = dq[u] - dqh[u];
            }
            // out_split 2: hi again at + 2 B*N*2Co, so [hi; lo; hi] is one row-stacked
            // operand of the 3-pass weight gradient (one TN GEMM over 3 B*N rows)
            const int np = out_split >= 2 ? 2 : 1;
            if (vec) {
                for (int pl = 0; pl < np; ++pl) {
                    gst_bf16<CS>(dPQh + 2 * pl * lo_off + j * 2 * Co + o0, dph);
                    gst_bf16<CS>(dPQh + 2 * pl * lo_off + j * 2 * Co + Co + o0, dqh);
                }
                gst_bf16<CS>(dPQh + lo_off + j * 2 * Co + o0, dpl);
                gst_bf16<CS>(dPQh + lo_off + j * 2 * Co + Co + o0, dql);
            } else {
#pragma unroll
                for (int u = 0; u < CS; ++u) {
                    if (o0 + u >= Co) continue;
                    for (int pl = 0; pl < np; ++pl) {
                        dPQh[2 * pl * lo_off + j * 2 * Co + o0 + u] = (__bf16)dph[u];
                        dPQh[2 * pl * lo_off + j * 2 * Co + Co + o0 + u] = (__bf16)dqh[u];
                    }
                    dPQh[lo_off + j * 2 * Co + o0 + u] = (__bf16)dpl[u];
                    dPQh[lo_off + j * 2 * Co + Co + o0 + u] = (__bf16)dql[u];
                }
            }
        } else if (OUT16 && vec) {
            gst_bf16<CS>(dPQh + j * 2 * Co + o0, dp);
            gst_bf16<CS>(dPQh + j * 2 * Co + Co + o0, dq);
        } else if (vec) {
            gst_vec<CS>(dPQ + j * 2 * Co + o0, dp);
            gst_vec<CS>(dPQ + j * 2 * Co + Co + o0, dq);
        } else {
#pragma unroll
            for (int u = 0; u < CS; ++u) {
                if (o0 + u >= Co) continue;
                if (OUT16) {
                    dPQh[j * 2 * Co + o0 + u] = (__bf16)dp[u];
                    dPQh[j * 2 * Co + Co + o0 + u] = (__bf16)dq[u];
                } else {
                    dPQ[j * 2 * Co + o0 + u] = dp[u];
                    dPQ[j * 2 * Co + Co + o0 + u] = dq[u];
                }
            }
        }
    }
}

// ---- push form of the scatter (dgx_edge_bwd_scatter_push_f32) ------------
// The a * sum_{selected edges -> j} dz term is pushed from the sources instead
// of pulled over the in-edges: each (point i, channel c) of the cloud adds its
// dz_i[c] to the accumulator of j = idx[i][arg_i[c]] (exactly one target per
// source and channel), so the in-edge loop reads only the Q row (no dz row, no
// slot compare per channel). The accumulators are 64-bit fixed point in units
// of 2^(emax - 172), emax the channel's largest biased exponent over the cloud:
// every term is an integer below 2^46 and the sum of N <= 65535 of them stays
// below 2^62, so the LDS atomics add exactly and the sum does not depend on the
// order they land in (deterministic; the exact sum rounded once to fp32). A
// channel holding an inf / NaN dz makes its sums NaN.
__device__ __forceinline__ unsigned long long fx_term(uint32_t bits, int emax) {
    const int E = (bits >> 23) & 0xff;
    const uint32_t m = (bits & 0x7fffffu) | (E ? 0x800000u : 0u);
    const int sh = max(E, 1) - emax + 22;  // <= 22
    const unsigned long long mag =
        sh >= 0 ? (unsigned long long)m << sh : (sh > -32 ? (unsigned long long)(m >> -sh) : 0ull);
    return (bits >> 31) ? 0ull - mag : mag;
}
__device__ __forceinline__ float fx_value(unsigned long long s, int emax) {
    return ldexpf((float)(long long)s, emax - 172);
}

constexpr int BP_U = 16;  // source (point, channel) pairs per thread per batch of the push

template <int CS, bool OUT16, bool PACKED>
__global__ __launch_bounds__(EC_THREADS, 4) void edge_bwd_push_kernel(
    const float* __restrict__ PQ, int ldpq, const int32_t* __restrict__ idx, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ edges, const float* __restrict__ dz, const uint8_t* __restrict__ arg,
    const float* __restrict__ sumP, int B, int N, int k, int Co, int nparts, const float* __restrict__ scale,
    const float* __restrict__ c0, const float* __restrict__ c1, void* __restrict__ dPQv, BnBwdFin fin,
    uint32_t skip) {   // skip: phase-timing probe (tools/push_lab.py), 0 in production
    static_assert(CS == 1 || CS == 2 || CS == 4 || CS == 8, "slice width");
    static_assert(EC_THREADS % CS == 0, "a thread keeps one channel");
    float* __restrict__ dPQ = static_cast<float*>(dPQv);
    __bf16* __restrict__ dPQh = static_cast<__bf16*>(dPQv);
    int b, part, slice;
    if (!dgx_xcd_slice_map(blockIdx.x, B, nparts, (Co + CS - 1) / CS, b, part, slice)) return;
    const int o0 = slice * CS;
    const int t = threadIdx.x, lane = t & 63;
    const int64_t base = (int64_t)b * N;
    const int per = (N + nparts - 1) / nparts;
    const int per8 = (per + 7) & ~7;
    const int n_beg = part * per, n_end = min(N, n_beg + per);
    const int np = max(0, n_end - n_beg);
    // [N][CS] Q | [per8][CS] u64 accumulators | [per8] u16 order | buckets | emax, bad | finalize scratch
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* qs = lds;
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(lds + ((N * CS + 3) & ~3));
    uint16_t* order = reinterpret_cast<uint16_t*>(acc + per8 * CS);
    int* bucket = reinterpret_cast<int*>(order + per8);
    int* emx = bucket + BW_BUCKETS;
    int* badc = emx + 8;
    void* scratch = badc + 8;
    const bool full = o0 + CS <= Co;
    constexpr bool SWZ = CS == 8;
    for (int e = t; e < per8 * CS / 2; e += EC_THREADS) reinterpret_cast<uint4*>(acc)[e] = make_uint4(0, 0, 0, 0);
    if (t < BW_BUCKETS) bucket[t] = 0;
    if (t < 8) {
        emx[t] = 1;
        badc[t] = 0;
    }
    auto lds_row = [&](const float* __restrict__ arr, int n, float (&r)[CS]) {
        if constexpr (SWZ) {
            const int sw = ((n >> 2) & 1) << 2;
            const float4 x = *reinterpret_cast<const float4*>(arr + n * CS + sw);
            const float4 y = *reinterpret_cast<const float4*>(arr + n * CS + (4 ^ sw));
            r[0] = x.x; r[1] = x.y; r[2] = x.z; r[3] = x.w;
            r[4] = y.x; r[5] = y.y; r[6] = y.z; r[7] = y.w;
        } else {
            lds_vec<CS>(arr + n * CS, r);
        }
    };
    // the thread's channel is the same on every trip of the (point, channel) loops
    const int cc = t % CS;
    const bool cvalid = o0 + cc < Co;
    const uint32_t* __restrict__ dzw = reinterpret_cast<const uint32_t*>(dz) + base * Co + o0 + cc;
    const int total = N * CS;
    constexpr int CHUNK = BP_U * EC_THREADS;
    uint32_t w[BP_U];
    auto load_w = [&](int p0) {
#pragma unroll
        for (int u = 0; u < BP_U; ++u) {
            const int p = p0 + u * EC_THREADS;
            w[u] = cvalid && p < total ? dzw[(uint32_t)((p / CS) * Co)] : 0u;   // 32-bit offsets: saddr loads
        }
    };
    // the first chunk of dz words and in-degrees are loaded before the Q slice
    // is staged, so their latency hides behind the staging
    load_w(t);
    const int deg0 = t < np ? rowptr[base + n_beg + t + 1] - rowptr[base + n_beg + t] : 0;
    if (!(skip & 8))
        stage_slice<CS, EC_THREADS, SWZ>(qs, PQ + base * ldpq + Co, ldpq, N, o0, Co,
                                         (ldpq % 4) == 0 && (Co % 4) == 0);
    // pass 1: the channel's largest exponent and whether it holds a non-finite dz
    int em = 1, bad = 0;
    for (int p0 = t; !(skip & 1);) {
#pragma unroll
        for (int u = 0; u < BP_U; ++u) {
            const int E = (w[u] >> 23) & 0xff;
            bad |= E == 0xff;
            em = max(em, E == 0xff ? 1 : E);
        }
        p0 += CHUNK;
        if (p0 >= total) break;
        load_w(p0);
    }
#pragma unroll
    for (int m = CS; m < 64; m <<= 1) {
        em = max(em, __shfl_xor(em, m));
        bad |= __shfl_xor(bad, m);
    }
    __syncthreads();  // accumulators, buckets, emx zeroed
    if (lane < CS) {
        atomicMax(&emx[lane], em);
        if (bad) atomicOr(&badc[lane], 1);
    }
    // in-block order: counting sort of the block's points by in-degree, descending
    for (int r = t; r < np; r += EC_THREADS) {
        const int64_t j = base + n_beg + r;
        const int deg = r == t ? deg0 : rowptr[j + 1] - rowptr[j];
        atomicAdd(&bucket[BW_BUCKETS - 1 - min(deg, BW_BUCKETS - 1)], 1);
    }
    __syncthreads();
    if (t < 64) {  // exclusive scan of the 64 bucket counts (one wave)
        const int c = bucket[t];
        int inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(inc, o);
            if (t >= o) inc += v;
        }
        bucket[t] = inc - c;
    }
    // pass 2: push every source's selected dz into its target's accumulator
    // (a single chunk is still in registers from pass 1)
    if (cvalid && !(skip & 2)) {
        const int ec = emx[cc];
        const int32_t* __restrict__ ib = idx + base * k;
        const uint8_t* __restrict__ ab = PACKED ? nullptr : arg + base * Co + o0 + cc;
        for (int p0 = t; p0 < total; p0 += CHUNK) {
            if (total > CHUNK) load_w(p0);
            int j[BP_U];   // the slot, then the target
#pragma unroll
            for (int u = 0; u < BP_U; ++u) {
                const int p = p0 + u * EC_THREADS;
                if constexpr (PACKED) j[u] = (int)(w[u] & 63u);
                else j[u] = p < total ? ab[(uint32_t)((p / CS) * Co)] : 0;
            }
#pragma unroll
            for (int u = 0; u < BP_U; ++u) {
                const int p = p0 + u * EC_THREADS;
                j[u] = p < total ? ib[(uint32_t)((p / CS) * k + j[u])] : -1;
            }
#pragma unroll
            for (int u = 0; u < BP_U; ++u) {
                const uint32_t v = PACKED ? (w[u] & ~63u) : w[u];
                if (j[u] >= n_beg && j[u] < n_end && ((v >> 23) & 0xff) != 0xff && !(skip & 16))
                    atomicAdd(&acc[(j[u] - n_beg) * CS + cc], fx_term(v, ec));
            }
        }
    }
    __syncthreads();  // bucket offsets
    for (int r = t; r < np; r += EC_THREADS) {
        const int64_t j = base + n_beg + r;
        const int deg = rowptr[j + 1] - rowptr[j];
        order[atomicAdd(&bucket[BW_BUCKETS - 1 - min(deg, BW_BUCKETS - 1)], 1)] = (uint16_t)r;
    }
    float a[CS], k0[CS], k1[CS];
    scatter_consts<CS>(fin, b, part, o0, Co, scale, c0, c1, scratch, a, k0, k1);
    const bool vec = full && (CS % 4) == 0 && (Co % 4) == 0 && (ldpq % 4) == 0;
    const float kf = (float)k;
    const int32_t ibase = (int32_t)base;
    __syncthreads();  // order, accumulators, emx / bad complete
    int ex[CS];
    bool nan_c[CS];
#pragma unroll
    for (int u = 0; u < CS; ++u) {
        ex[u] = emx[u];
        nan_c[u] = badc[u] != 0;
    }
    // boustrophedon deal of the degree-sorted points (as edge_bwd_scatter_kernel)
    for (int it = 0; it * EC_THREADS < np; ++it) {
        const int r = it * EC_THREADS + ((it & 1) ? EC_THREADS - 1 - t : t);
        if (r >= np) continue;
        const int rl = order[r];
        const int n = n_beg + rl;
        const int64_t j = base + n;
        const int32_t beg = rowptr[j], end = rowptr[j + 1];
        float pjv[CS], spv[CS], dn[CS];  // HBM reads issued before the edge loop hides their latency
        if (vec) {
            gld_vec<CS>(PQ + j * ldpq + o0, pjv);
            gld_vec<CS>(sumP + j * Co + o0, spv);
            gld_vec<CS>(dz + j * Co + o0, dn);
        } else {
#pragma unroll
            for (int u = 0; u < CS; ++u) {
                pjv[u] = o0 + u < Co ? PQ[j * ldpq + o0 + u] : 0.f;
                spv[u] = o0 + u < Co ? sumP[j * Co + o0 + u] : 0.f;
                dn[u] = o0 + u < Co ? dz[j * Co + o0 + u] : 0.f;
            }
        }
        float sq[CS];
#pragma unroll
        for (int u = 0; u < CS; ++u) sq[u] = 0.f;
        for (int32_t u0 = beg; u0 < ((skip & 4) ? beg : end); u0 += BW_EB) {
            int32_t ids[BW_EB];
#pragma unroll
            for (int v = 0; v < BW_EB; ++v) ids[v] = u0 + v < end ? edges[u0 + v] : 0;
#pragma unroll
            for (int v = 0; v < BW_EB; ++v)
                if (u0 + v < end) {
                    float q[CS];
                    lds_row(qs, (ids[v] >> 6) - ibase, q);
#pragma unroll
                    for (int u = 0; u < CS; ++u) sq[u] += q[u];
                }
        }
        const float deg = (float)(end - beg);
        float qn[CS], sd[CS];
        lds_row(qs, n, qn);
#pragma unroll
        for (int u = 0; u < CS; ++u) {
            sd[u] = nan_c[u] ? __builtin_nanf("") : fx_value(acc[rl * CS + u], ex[u]);
            if constexpr (PACKED) dn[u] = __uint_as_float(__float_as_uint(dn[u]) & ~63u);
        }
        float dp[CS], dq[CS];
#pragma unroll
        for (int u = 0; u < CS; ++u) {
            dp[u] = fmaf(a[u], sd[u], fmaf(k0[u], deg, k1[u] * fmaf(deg, pjv[u], sq[u])));
            dq[u] = fmaf(a[u], dn[u], fmaf(k0[u], kf, k1[u] * fmaf(kf, qn[u], spv[u])));
        }
        if (OUT16 && vec) {
            gst_bf16<CS>(dPQh + j * 2 * Co + o0, dp);
            gst_bf16<CS>(dPQh + j * 2 * Co + Co + o0, dq);
        } else if (vec) {
            gst_vec<CS>(dPQ + j * 2 * Co + o0, dp);
            gst_vec<CS>(dPQ + j * 2 * Co + Co + o0, dq);
        } else {
#pragma unroll
            for (int u = 0; u < CS; ++u) {
                if (o0 + u >= Co) continue;
                if (OUT16) {
                    dPQh[j * 2 * Co + o0 + u] = (__bf16)dp[u];
                    dPQh[j * 2 * Co + Co + o0 + u] = (__bf16)dq[u];
                } else {
                    dPQ[j * 2 * Co + o0 + u] = dp[u];
                    dPQ[j * 2 * Co + Co + o0 + u] = dq[u];
                }
            }
        }
    }
}

// push-scatter LDS bytes: Q slice | accumulators | order | buckets | emax, bad | finalize scratch
inline size_t push_lds_bytes(int N, int cs, int parts) {
    const size_t per8 = (size_t)(((N + parts - 1) / parts + 7) & ~7);
    return (((size_t)N * cs + 3) & ~(size_t)3) * sizeof(float) + per8 * cs * 8 + per8 * sizeof(uint16_t) +
           BW_BUCKETS * sizeof(int) + 16 * sizeof(int) + BW_FIN_LDS;
}

// scatter LDS bytes for N points at CS channels (Q | dz | slot | order | buckets;
// no slot array when the dz words carry the slots)
inline size_t scatter_lds_bytes(int N, int cs, int parts, bool packed, int idcap = 0) {
    const int per = (N + parts - 1) / parts;
    return (size_t)2 * N * cs * sizeof(float) + (packed ? 0 : (((size_t)N * cs + 15) & ~(size_t)15)) +
           (size_t)((per + 7) & ~7) * sizeof(uint16_t) + BW_BUCKETS * sizeof(int) + BW_FIN_LDS +
           (size_t)((idcap + 7) & ~7) * sizeof(uint16_t);
}

inline int grid_for(int64_t total, int block) {
    int64_t g = (total + block - 1) / block;
    return (int)(g < 8192 ? (g < 1 ? 1 : g) : 8192);
}

// channels per LDS slice: the cloud's slice (words_per_elem x N x CS floats)
// must fit EC_LDS_BYTES
inline int slice_channels(int N, int words_per_elem) {
    int cs = 32;
    while (cs > 1 && (size_t)words_per_elem * N * cs * sizeof(float) > (size_t)EC_LDS_BYTES) cs >>= 1;
    return cs;
}

// split the points of a cloud over `parts` workgroups so the grid reaches ~2
// workgroups per CU (each restages the slice: redundancy = parts)
inline int point_parts(int B, int slices, int N) {
    int parts = 1;
    while ((int64_t)B * slices * parts < 512 && parts * 64 < N) parts <<= 1;
    return parts;
}

template <bool EVAL>
int launch_gather(int cs, dim3 grid, size_t lds, hipStream_t st, const float* PQ, int ldpq, const int32_t* idx, int B,
                  int N,
                  int k, int Co, int nparts, const float* sel, const float* shift, float slope, float* ysel,
                  uint8_t* arg, float* sumP, float* partials, float* out, int ldo) {
#define DGX_GATHER_CASE(CSV)                                                                                      \
    case CSV:                                                                                                    \
        hipLaunchKernelGGL((edge_gather_lds_kernel<CSV, EVAL>), grid, dim3(EC_THREADS), lds, st, PQ, ldpq, idx, B, \
                           N, k, Co, nparts, sel, shift, slope, ysel, arg, sumP, partials, out, ldo);             \
        break;
    switch (cs) {
        DGX_GATHER_CASE(32)
        DGX_GATHER_CASE(16)
        DGX_GATHER_CASE(8)
        DGX_GATHER_CASE(4)
        DGX_GATHER_CASE(2)
        DGX_GATHER_CASE(1)
        default: return DGX_EUNSUPPORTED;
    }
#undef DGX_GATHER_CASE
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

struct GatherGeom {
    int cs, slices, parts;
    size_t lds;
};

inline GatherGeom gather_geom(int B, int N, int Co) {
    GatherGeom g;
    g.cs = slice_channels(N, 1);
    g.slices = (Co + g.cs - 1) / g.cs;
    g.parts = point_parts(B, g.slices, N);
    size_t stage = (size_t)N * g.cs * sizeof(float) + GF_ICAP * sizeof(int);
    const int v = g.cs >= 4 ? g.cs / 4 : 1;
    size_t red = (size_t)2 * v * EC_THREADS * sizeof(float);
    g.lds = stage > red ? stage : red;
    return g;
}

}  // namespace

extern "C" {

int dgx_edge_partials_rows(int B, int N, int Co) {
    if (B < 1 || N < 1 || Co < 1) return DGX_EINVAL;
    return B * gather_geom(B, N, Co).parts;
}

int dgx_edge_fwd_gather_f32(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int Co,
                            const float* gamma, float* ysel, uint8_t* arg, float* sumP, float* partials, int nrows,
                            void* stream) {
    if (!PQ || !idx || !gamma || !ysel || !arg || !sumP || !partials) return DGX_EINVAL;
    if (B < 1 || N < 1 || k < 1 || k > 64 || Co < 1 || ldpq < 2 * Co) return DGX_EINVAL;
    const GatherGeom g = gather_geom(B, N, Co);
    if (nrows != B * g.parts) return DGX_EINVAL;
    // beyond EC_LDS_BYTES (N > 16384) a one-channel slice takes up to the CU's 160 KiB (one workgroup per CU)
    if (g.lds > (size_t)160 * 1024) return DGX_EUNSUPPORTED;
    return launch_gather<false>(g.cs, dim3(dgx_xcd_cloud_grid(B, g.parts * g.slices)), g.lds, dgx_stream(stream), PQ,
                                ldpq, idx, B, N, k, Co,
                                g.parts, gamma, nullptr, 0.f, ysel, arg, sumP, partials, nullptr, 0);
}

int dgx_edge_fwd_eval_f32(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int Co,
                          const float* scale, const float* shift, float slope, float* out, int ldo, void* stream) {
    if (!PQ || !idx || !scale || !shift || !out) return DGX_EINVAL;
    if (B < 1 || N < 1 || k < 1 || Co < 1 || ldpq < 2 * Co || ldo < Co) return DGX_EINVAL;
    const GatherGeom g = gather_geom(B, N, Co);
    if (g.lds > (size_t)160 * 1024) return DGX_EUNSUPPORTED;
    return launch_gather<true>(g.cs, dim3(dgx_xcd_cloud_grid(B, g.parts * g.slices)), g.lds, dgx_stream(stream), PQ,
                               ldpq, idx, B, N, k, Co,
                               g.parts, scale, shift, slope, nullptr, nullptr, nullptr, nullptr, out, ldo);
}

int dgx_bn_finalize_out_f32(const float* partials, int nrows, int Co, double count, const float* gamma,
                            const float* beta, const float* running_mean, const float* running_var, double momentum,
                            double eps, float* scale, float* shift, float* mean, float* invstd,
                            const int64_t* num_batches_tracked, float* running_mean_new, float* running_var_new,
                            int64_t* num_batches_tracked_new, void* stream) {
    if (!partials || nrows < 1 || Co < 1 || count <= 0.0 || !scale || !shift) return DGX_EINVAL;
    if ((running_mean && !running_mean_new) || (running_var && !running_var_new) ||
        (num_batches_tracked && !num_batches_tracked_new))
        return DGX_EINVAL;
    // cumulative average: every block reads the counter, so it may not be updated in place
    if (momentum < 0.0 && num_batches_tracked && num_batches_tracked == num_batches_tracked_new) return DGX_EINVAL;
    hipLaunchKernelGGL(bn_finalize_kernel<float>, dim3((Co + 3) / 4), dim3(256), 0, dgx_stream(stream), partials, nrows, Co,
                       count, gamma, beta, running_mean, running_var, momentum, eps, scale, shift, mean, invstd,
                       num_batches_tracked, running_mean_new, running_var_new, num_batches_tracked_new);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_bn_finalize_f32(const float* partials, int nrows, int Co, double count, const float* gamma,
                        const float* beta, float* running_mean, float* running_var, double momentum, double eps,
                        float* scale, float* shift, float* mean, float* invstd, int64_t* num_batches_tracked,
                        void* stream) {
    return dgx_bn_finalize_out_f32(partials, nrows, Co, count, gamma, beta, running_mean, running_var, momentum, eps,
                                   scale, shift, mean, invstd, num_batches_tracked, running_mean, running_var,
                                   num_batches_tracked, stream);
}

int dgx_bn_finalize_out_f64(const double* sums, int nrows, int Co, double count, const float* gamma,
                            const float* beta, const float* running_mean, const float* running_var, double momentum,
                            double eps, float* scale, float* shift, float* mean, float* invstd,
                            const int64_t* num_batches_tracked, float* running_mean_new, float* running_var_new,
                            int64_t* num_batches_tracked_new, void* stream) {
    if (!sums || nrows < 1 || Co < 1 || count == 0.0 || !scale || !shift) return DGX_EINVAL;
    if ((running_mean && !running_mean_new) || (running_var && !running_var_new) ||
        (num_batches_tracked && !num_batches_tracked_new))
        return DGX_EINVAL;
    // cumulative average: every block reads the counter, so it may not be updated in place
    if (momentum < 0.0 && num_batches_tracked && num_batches_tracked == num_batches_tracked_new) return DGX_EINVAL;
    hipLaunchKernelGGL(bn_finalize_kernel<double>, dim3((Co + 3) / 4), dim3(256), 0, dgx_stream(stream), sums, nrows, Co,
                       count, gamma, beta, running_mean, running_var, momentum, eps, scale, shift, mean, invstd,
                       num_batches_tracked, running_mean_new, running_var_new, num_batches_tracked_new);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_bn_finalize_f64(const double* sums, int nrows, int Co, double count, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, double momentum, double eps, float* scale,
                        float* shift, float* mean, float* invstd, int64_t* num_batches_tracked, void* stream) {
    return dgx_bn_finalize_out_f64(sums, nrows, Co, count, gamma, beta, running_mean, running_var, momentum, eps,
                                   scale, shift, mean, invstd, num_batches_tracked, running_mean, running_var,
                                   num_batches_tracked, stream);
}

int dgx_bn_eval_affine_f32(int Co, const float* gamma, const float* beta, const float* running_mean,
                           const float* running_var, double eps, float* scale, float* shift, void* stream) {
    if (Co < 1 || !running_mean || !running_var || !scale || !shift) return DGX_EINVAL;
    hipLaunchKernelGGL(bn_eval_affine_kernel, dim3((Co + 255) / 256), dim3(256), 0, dgx_stream(stream), Co, gamma,
                       beta, running_mean, running_var, eps, scale, shift);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_bn_lrelu_apply_f32(const float* ysel, int M, int Co, const float* scale, const float* shift, float slope,
                           float* out, int ldo, void* out_bf16, void* stream) {
    if (!ysel || !scale || !shift || !out || M < 0 || Co < 1 || ldo < Co) return DGX_EINVAL;
    const int64_t total = (int64_t)M * Co;
    if (total == 0) return DGX_OK;
    const bool v4 = Co % 4 == 0 && ldo % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(ysel) % 16 == 0 && reinterpret_cast<uintptr_t>(scale) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(shift) % 16 == 0 && reinterpret_cast<uintptr_t>(out_bf16) % 8 == 0;
    if (v4)
        hipLaunchKernelGGL(bn_lrelu_apply4_kernel, dim3(grid_for(total / 4, 256)), dim3(256), 0, dgx_stream(stream),
                           ysel, M, Co, scale, shift, slope, out, ldo, static_cast<__bf16*>(out_bf16));
    else
        hipLaunchKernelGGL(bn_lrelu_apply_kernel, dim3(grid_for(total, 256)), dim3(256), 0, dgx_stream(stream), ysel,
                           M, Co, scale, shift, slope, out, ldo, static_cast<__bf16*>(out_bf16));
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_bwd_dz_f32(const float* dY, int lddy, const float* ysel, int M, int Co, const float* scale,
                        const float* shift, const float* mean, const float* invstd, float slope, float* dz,
                        float* partials, int nrows, void* stream) {
    if (!dY || !ysel || !scale || !shift || !mean || !invstd || !dz || !partials) return DGX_EINVAL;
    if (M < 1 || Co < 1 || lddy < Co || nrows < 1) return DGX_EINVAL;
    const int rows = (M + nrows - 1) / nrows;
    hipLaunchKernelGGL(edge_bwd_dz_kernel, dim3(nrows, (Co + 63) / 64), dim3(256), 0, dgx_stream(stream), dY, lddy,
                       ysel, M, Co, scale, shift, mean, invstd, slope, dz, partials, rows, nullptr);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_bwd_dz_packed_f32(const float* dY, int lddy, const float* ysel, const uint8_t* arg, int M, int Co,
                               const float* scale, const float* shift, const float* mean, const float* invstd,
                               float slope, float* dz_packed, float* partials, int nrows, void* stream) {
    if (!dY || !ysel || !arg || !scale || !shift || !mean || !invstd || !dz_packed || !partials) return DGX_EINVAL;
    if (M < 1 || Co < 1 || lddy < Co || nrows < 1) return DGX_EINVAL;
    const int rows = (M + nrows - 1) / nrows;
    hipLaunchKernelGGL(edge_bwd_dz_kernel, dim3(nrows, (Co + 63) / 64), dim3(256), 0, dgx_stream(stream), dY, lddy,
                       ysel, M, Co, scale, shift, mean, invstd, slope, dz_packed, partials, rows, arg);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_edge_bwd_dz_cm_rows(int B, int N) {
    if (B < 1 || N < 1) return DGX_EINVAL;
    return B * ((N + 63) / 64);
}

int dgx_edge_bwd_dz_cm_f32(const float* dY, const float* ysel, int B, int N, int Co, const float* scale,
                           const float* shift, const float* mean, const float* invstd, float slope, float* dz,
                           float* partials, int nrows, void* stream) {
    if (!dY || !ysel || !scale || !shift || !mean || !invstd || !dz || !partials) return DGX_EINVAL;
    if (B < 1 || N < 1 || Co < 1 || nrows != dgx_edge_bwd_dz_cm_rows(B, N)) return DGX_EINVAL;
    const int ntn = (N + 63) / 64;
    hipLaunchKernelGGL(edge_bwd_dz_cm_kernel, dim3(B * ntn, (Co + 63) / 64), dim3(256), 0, dgx_stream(stream), dY,
                       ysel, N, Co, ntn, scale, shift, mean, invstd, slope, dz, partials);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_bn_bwd_finalize_f32(const float* partials, int nrows, int Co, double count, const float* scale,
                            const float* mean, const float* invstd, float* dgamma, float* dbeta, float* c0,
                            float* c1, int accumulate, void* stream) {
    if (!partials || nrows < 1 || Co < 1 || count <= 0.0 || !scale || !mean || !invstd || !c0 || !c1)
        return DGX_EINVAL;
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<float>, dim3((Co + 3) / 4), dim3(256), 0, dgx_stream(stream), partials, nrows,
                       Co, count, scale, mean, invstd, dgamma, dbeta, c0, c1, accumulate);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_bn_bwd_finalize_f64(const double* sums, int nrows, int Co, double count, const float* scale,
                            const float* mean, const float* invstd, float* dgamma, float* dbeta, float* c0,
                            float* c1, int accumulate, void* stream) {
    if (!sums || nrows < 1 || Co < 1 || count == 0.0 || !scale || !mean || !invstd || !c0 || !c1)
        return DGX_EINVAL;
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<double>, dim3((Co + 3) / 4), dim3(256), 0, dgx_stream(stream), sums, nrows, Co,
                       count, scale, mean, invstd, dgamma, dbeta, c0, c1, accumulate);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_graph_reverse_multi(int n, const int32_t* const* idx, int B, int N, int k, int32_t* const* rowptr,
                            int32_t* const* edges, void* stream) {
    if (n < 1 || n > RG_MAX_GRAPHS || !idx || !rowptr || !edges || B < 1 || N < 1 || k < 1 || k > 64)
        return DGX_EINVAL;
    if ((int64_t)B * N >= (1LL << 25)) return DGX_EUNSUPPORTED;
    RevGraphJobs jobs{};
    for (int g = 0; g < n; ++g) {
        if (!idx[g] || !rowptr[g] || !edges[g]) return DGX_EINVAL;
        jobs.idx[g] = idx[g];
        jobs.rowptr[g] = rowptr[g];
        jobs.edges[g] = edges[g];
    }
    // workgroups per cloud: enough (over all graphs) to fill the chip, and few
    // enough that the cloud's index list is not re-scanned more than needed
    // (every workgroup of a cloud scans it twice); a range's edges (about
    // N*k/P) stay well inside the LDS list capacity
    int P = 1;
    while (P < N && ((int64_t)n * B * P < RG_MIN_WG || (int64_t)N * k / P > RG_CAP / 2)) P *= 2;
    const int R = (N + P - 1) / P;
    // list capacity 1.75x a range's mean edge count (two workgroups per CU at
    // cfg2); a range beyond it (degenerate clouds) sorts its lists in HBM
    const int cap = (int)std::min<int64_t>(RG_CAP, std::max<int64_t>(1024, 7 * ((int64_t)N * k / P) / 4));
    const size_t lds = ((size_t)2 * R + RG_THREADS / 64 + 2 + 2 * (size_t)cap) * sizeof(int32_t);
    if (lds > 160 * 1024) return DGX_EUNSUPPORTED;
    hipLaunchKernelGGL(rev_graph_par_kernel, dim3((unsigned)dgx_xcd_cloud_grid(n * B, P)), dim3(RG_THREADS), lds,
                       dgx_stream(stream), jobs, n, B, N, k, P, cap);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_graph_reverse(const int32_t* idx, int B, int N, int k, int32_t* rowptr, int32_t* edges, void* stream) {
    return dgx_graph_reverse_multi(1, &idx, B, N, k, &rowptr, &edges, stream);
}

namespace {
int launch_scatter(const float* PQ, int ldpq, const int32_t* rowptr, const int32_t* edges, const float* dz,
                   const uint8_t* arg, const float* sumP, int B, int N, int k, int Co, const float* scale,
                   const float* c0, const float* c1, void* dPQ, int out_bf16, bool packed, void* stream,
                   const BnBwdFin& fin = BnBwdFin{}) {
    if (!PQ || !rowptr || !edges || !dz || (!packed && !arg) || !sumP || !scale || !c0 || !c1 || !dPQ)
        return DGX_EINVAL;
    if (fin.partials && (fin.nrows < 1 || fin.count <= 0.0 || !fin.mean || !fin.invstd)) return DGX_EINVAL;
    if (B < 1 || N < 1 || k < 1 || k > 64 || Co < 1 || ldpq < 2 * Co) return DGX_EINVAL;
    if (out_bf16 < 0 || out_bf16 > 3) return DGX_EINVAL;   // 2: split planes (hi, lo), 3: (hi, lo, hi)
    if (N > 65535) return DGX_EUNSUPPORTED;
    // slice channels: 9 (8 packed) bytes per (point, channel) within BW_LDS_BYTES
    // (16 measured slower: one workgroup per CU; 4 slower: per-edge work over fewer channels)
    const size_t per_pc = packed ? 8 : 9;
    int cs = 8;
    while (cs > 1 && per_pc * N * cs > (size_t)BW_LDS_BYTES) cs >>= 1;
    // LDS-staged in-edge ids (16-bit words: N <= 1024, packed dz words): at most
    // SCATTER_IDL_CS channels per slice so the slices, the ids (capacity 1.75x a
    // part's mean in-edge count; a part beyond it reads its ids from HBM) and
    // the rest fit two workgroups per CU. Measured and kept OFF (r09g, cfg2
    // step, mean scatter launch): 4-channel slices with LDS ids 59.3 us vs 54.9
    // for the 8-channel HBM-id form (the narrower slices cost more than the id
    // latency saves; with ids synthesised instead of loaded, r09e, the 8-channel
    // form ran 43.8 us, but 8-channel slices leave LDS for ~6.5 K of a part's
    // ~10 K ids, so most parts fall back: 55.3 us). -DSCATTER_IDL_CS=4 / 8 A/B.
#ifndef SCATTER_IDL_CS
#define SCATTER_IDL_CS 0
#endif
    const bool idl = SCATTER_IDL_CS > 0 && packed && N <= 1024 && k <= 64;
    if (idl) cs = std::min(cs, SCATTER_IDL_CS);
    const int slices = (Co + cs - 1) / cs;
    int parts = point_parts(B, slices, N);
    // a cloud whose one-channel slices exceed BW_LDS_BYTES (N > 9216) takes up to
    // the CU's 160 KiB (one workgroup per CU; more point parts shrink the order
    // array): N <= 20000 packed, 17900 unpacked
    while (scatter_lds_bytes(N, cs, parts, packed) > (size_t)160 * 1024 && parts * 64 < N) parts *= 2;
    int idcap = 0;
    if (idl) {
        const int per = (N + parts - 1) / parts;
        idcap = (int)std::min<int64_t>(7 * (int64_t)per * k / 4, (int64_t)per * k * 2);
        const size_t room = (size_t)80 * 1024;   // two workgroups per CU
        const size_t fixed = scatter_lds_bytes(N, cs, parts, packed);
        if (fixed + 16 * sizeof(uint16_t) > room) idcap = 0;
        else idcap = std::min<int>(idcap, (int)((room - fixed) / sizeof(uint16_t)) & ~7);
    }
    const dim3 grid(dgx_xcd_cloud_grid(B, parts * slices));
    const size_t lds = scatter_lds_bytes(N, cs, parts, packed, idcap);
    if (lds > (size_t)160 * 1024) return DGX_EUNSUPPORTED;
    hipStream_t st = dgx_stream(stream);
#define DGX_SCATTER_LAUNCH_T(CSV, O16, PK, SP, TP)                                                                  \
    hipLaunchKernelGGL((edge_bwd_scatter_kernel<CSV, O16, PK, SP, TP>), grid, dim3(EC_THREADS), lds, st, PQ, ldpq,     \
                       rowptr, edges, dz, arg, sumP, B, N, k, Co, parts, scale, c0, c1, dPQ, fin, out_bf16 - 1, idcap)
#define DGX_SCATTER_LAUNCH(CSV, O16, PK, SP) DGX_SCATTER_LAUNCH_T(CSV, O16, PK, SP, 1)
#define DGX_SCATTER_CASE(CSV)                                                \
    case CSV:                                                               \
        if (packed) {                                                       \
            if (out_bf16 >= 2) DGX_SCATTER_LAUNCH(CSV, true, true, true);   \
            else if (out_bf16) DGX_SCATTER_LAUNCH(CSV, true, true, false);  \
            else DGX_SCATTER_LAUNCH(CSV, false, true, false);               \
        } else {                                                            \
            if (out_bf16 >= 2) DGX_SCATTER_LAUNCH(CSV, true, false, true);  \
            else if (out_bf16) DGX_SCATTER_LAUNCH(CSV, true, false, false); \
            else DGX_SCATTER_LAUNCH(CSV, false, false, false);              \
        }                                                                   \
        break;
    // packed dz|slot words at 8-channel slices: TPP lanes per point
    // (edge_bwd_scatter_kernel): 2 for parts of 256+ points, up to
    // SCATTER_SMALL_TPP while a part's points x lanes fit the block (few-cloud
    // shards, whose grids are widened by point parts). cfg2 (r09o, mean of the
    // step's 4 bf16 launches): 1 lane 56.2 us, 2 lanes 52.5, 4 lanes 57.8;
    // 4-cloud shard (r09m): 1 lane 20.3, 4 lanes 14.1, 8 lanes 14.4 us
#ifndef SCATTER_SMALL_TPP
#define SCATTER_SMALL_TPP 4
#endif
    const int per_pts = (N + parts - 1) / parts;
    int tpp = 2;
    while (tpp < SCATTER_SMALL_TPP && per_pts * 2 * tpp <= EC_THREADS) tpp *= 2;
#ifdef SCATTER_FORCE_TPP   // (A/B builds) the same lanes per point at any part size
    tpp = SCATTER_FORCE_TPP;
#endif
    if (tpp > 1 && cs == 8 && packed) {
#define DGX_SCATTER_TPP(O16, SP)                                             \
    if (tpp >= 8) DGX_SCATTER_LAUNCH_T(8, O16, true, SP, 8);                 \
    else if (tpp == 4) DGX_SCATTER_LAUNCH_T(8, O16, true, SP, 4);            \
    else DGX_SCATTER_LAUNCH_T(8, O16, true, SP, 2);
        if (out_bf16 >= 2) { DGX_SCATTER_TPP(true, true) }
        else if (out_bf16) { DGX_SCATTER_TPP(true, false) }
        else { DGX_SCATTER_TPP(false, false) }
#undef DGX_SCATTER_TPP
        return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
    }
    switch (cs) {
        DGX_SCATTER_CASE(8)
        DGX_SCATTER_CASE(4)
        DGX_SCATTER_CASE(2)
        DGX_SCATTER_CASE(1)
        default: return DGX_EUNSUPPORTED;
    }
#undef DGX_SCATTER_CASE
#undef DGX_SCATTER_LAUNCH
#undef DGX_SCATTER_LAUNCH_T
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

// slice width and point parts of the push scatter: the fewest re-staged Q
// slices (parts / cs) whose LDS fits two workgroups per CU (80 KiB), else one
// (160 KiB); parts also brings the grid to ~2 workgroups per CU (point_parts)
bool push_geometry(int B, int N, int Co, int& cs_out, int& parts_out) {
    for (const size_t budget : {(size_t)80 * 1024, (size_t)160 * 1024}) {
        int best_cs = 0, best_parts = 0;
        for (int cs = 8; cs >= 1; cs >>= 1) {
            const int slices = (Co + cs - 1) / cs;
            int parts = point_parts(B, slices, N);
            while (push_lds_bytes(N, cs, parts) > budget && parts * 64 < N) parts *= 2;
            if (push_lds_bytes(N, cs, parts) > budget) continue;
            if (!best_cs || (int64_t)parts * best_cs < (int64_t)best_parts * cs) {
                best_cs = cs;
                best_parts = parts;
            }
        }
        if (best_cs) {
            cs_out = best_cs;
            parts_out = best_parts;
            return true;
        }
    }
    return false;
}

int launch_push(const float* PQ, int ldpq, const int32_t* idx, const int32_t* rowptr, const int32_t* edges,
                const float* dz, const uint8_t* arg, const float* sumP, int B, int N, int k, int Co,
                const float* scale, const float* c0, const float* c1, void* dPQ, int out_bf16, bool packed,
                void* stream, const BnBwdFin& fin) {
    if (!PQ || !idx || !rowptr || !edges || !dz || (!packed && !arg) || !sumP || !scale || !c0 || !c1 || !dPQ)
        return DGX_EINVAL;
    if (fin.partials && (fin.nrows < 1 || fin.count <= 0.0 || !fin.mean || !fin.invstd)) return DGX_EINVAL;
    if (B < 1 || N < 1 || k < 1 || k > 64 || Co < 1 || ldpq < 2 * Co) return DGX_EINVAL;
    if (out_bf16 < 0 || out_bf16 > 1) return out_bf16 <= 3 ? DGX_EUNSUPPORTED : DGX_EINVAL;
    if (N > 65535) return DGX_EUNSUPPORTED;
    int cs = 0, parts = 0;
    if (!push_geometry(B, N, Co, cs, parts)) return DGX_EUNSUPPORTED;
#ifdef DGX_PUSH_LAB
    // phase-timing probe of tools/push_lab.py: only in a lab build (-DDGX_PUSH_LAB),
    // never in the product library, where a stray variable would drop phases
    const char* probe = getenv("DGX_PUSH_SKIP");
    const uint32_t skip = probe ? (uint32_t)strtoul(probe, nullptr, 0) : 0u;
#else
    const uint32_t skip = 0u;
#endif
    const int slices = (Co + cs - 1) / cs;
    const dim3 grid(dgx_xcd_cloud_grid(B, parts * slices));
    const size_t lds = push_lds_bytes(N, cs, parts);
    hipStream_t st = dgx_stream(stream);
#define DGX_PUSH_LAUNCH(CSV, O16, PK)                                                                              \
    hipLaunchKernelGGL((edge_bwd_push_kernel<CSV, O16, PK>), grid, dim3(EC_THREADS), lds, st, PQ, ldpq, idx, rowptr, \
                       edges, dz, arg, sumP, B, N, k, Co, parts, scale, c0, c1, dPQ, fin, skip)
#define DGX_PUSH_CASE(CSV)                                      \
    case CSV:                                                   \
        if (packed) {                                           \
            if (out_bf16) DGX_PUSH_LAUNCH(CSV, true, true);     \
            else DGX_PUSH_LAUNCH(CSV, false, true);             \
        } else {                                                \
            if (out_bf16) DGX_PUSH_LAUNCH(CSV, true, false);    \
            else DGX_PUSH_LAUNCH(CSV, false, false);            \
        }                                                       \
        break;
    switch (cs) {
        DGX_PUSH_CASE(8)
        DGX_PUSH_CASE(4)
        DGX_PUSH_CASE(2)
        DGX_PUSH_CASE(1)
        default: return DGX_EUNSUPPORTED;
    }
#undef DGX_PUSH_CASE
#undef DGX_PUSH_LAUNCH
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}
}  // namespace

int dgx_edge_bwd_scatter_f32(const float* PQ, int ldpq, const int32_t* rowptr, const int32_t* edges,
                             const float* dz, const uint8_t* arg, const float* sumP, int B, int N, int k, int Co,
                             const float* scale, const float* c0, const float* c1, void* dPQ, int out_bf16,
                             void* stream) {
    return launch_scatter(PQ, ldpq, rowptr, edges, dz, arg, sumP, B, N, k, Co, scale, c0, c1, dPQ, out_bf16, false,
                          stream);
}

int dgx_edge_bwd_scatter_fin_f32(const float* PQ, int ldpq, const int32_t* rowptr, const int32_t* edges,
                                 const float* dz, const uint8_t* arg, const float* sumP, int B, int N, int k, int Co,
                                 const float* partials, int nrows, double count, const float* scale,
                                 const float* mean, const float* invstd, int eval, float* dgamma, float* dbeta,
                                 float* c0, float* c1, void* dPQ, int out_bf16, int packed, void* stream) {
    if (!partials) return DGX_EINVAL;
    const BnBwdFin fin{partials, nrows, count, mean, invstd, eval, dgamma, dbeta, c0, c1};
    return launch_scatter(PQ, ldpq, rowptr, edges, dz, packed ? nullptr : arg, sumP, B, N, k, Co, scale, c0, c1, dPQ,
                          out_bf16, packed != 0, stream, fin);
}

int dgx_edge_bwd_scatter_packed_f32(const float* PQ, int ldpq, const int32_t* rowptr, const int32_t* edges,
                                    const float* dz_packed, const float* sumP, int B, int N, int k, int Co,
                                    const float* scale, const float* c0, const float* c1, void* dPQ, int out_bf16,
                                    void* stream) {
    return launch_scatter(PQ, ldpq, rowptr, edges, dz_packed, nullptr, sumP, B, N, k, Co, scale, c0, c1, dPQ,
                          out_bf16, true, stream);
}

int dgx_edge_bwd_scatter_push_f32(const float* PQ, int ldpq, const int32_t* idx, const int32_t* rowptr,
                                  const int32_t* edges, const float* dz, const uint8_t* arg, const float* sumP, int B,
                                  int N, int k, int Co, const float* partials, int nrows, double count,
                                  const float* scale, const float* mean, const float* invstd, int eval, float* dgamma,
                                  float* dbeta, float* c0, float* c1, void* dPQ, int out_bf16, int packed,
                                  void* stream) {
    const BnBwdFin fin{partials, nrows, count, mean, invstd, eval, dgamma, dbeta, c0, c1};
    return launch_push(PQ, ldpq, idx, rowptr, edges, dz, packed ? nullptr : arg, sumP, B, N, k, Co, scale, c0, c1,
                       dPQ, out_bf16, packed != 0, stream, fin);
}

}  // extern "C"
