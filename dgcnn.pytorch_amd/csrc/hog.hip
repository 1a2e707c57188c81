// compute_hog_1x1 on the device (reference models/model_partseg.py:15-92):
// per-point dominant direction of the k-neighbourhood (SVD) and the 9-bin x
// 2-angle histogram of its neighbours' directions, with no host round trip.
//
// Reference behaviour reproduced bug-for-bug: the neighbourhoods
// are rows of x.contiguous().view(B*N, 3) addressed with LOCAL kNN ids, i.e. the
// (B, 3, N) buffer reinterpreted as rows of 3 floats, and the direction table
// is read back with the same local ids. Every id is < N, so only cloud 0's N
// neighbourhoods ever feed the histograms: hog_axis_kernel does those N SVDs
// (the reference does B*N and uses N of them), hog_hist_kernel bins all B*N
// points against that table.
//
// Arithmetic follows the reference op by op, on the device the reference runs
// each stage on (`sem`, DGX_HOG_*):
//   * the neighbourhood mean runs on x's device (model_partseg.py:32): on the
//     host, torch's CPU sum (ILP-4 row sum) then div_(k); on a GPU, torch's
//     reduce kernel (one thread per output, four accumulators over items
//     i = l mod 4 with the tail items dealt to accumulators 0, 1, ... in order,
//     combined ((a0 + a1) + a2) + a3) then MeanOps' multiply by the factor
//     float(outputs) / numel (DGX_HOG_MEAN_DEVICE);
//   * the SVD in fp64 exactly as numpy's dgesdd path (svd3.h), rounded to fp32;
//     magnitude = fp32 sqrt of the fp32 singular value;
//   * the votes run where v and s were moved (model_partseg.py:42-47: the GPU
//     unless use_cpu without LOCAL_RANK). Host: acos / atan from fp64 (the host
//     libm's, but for rare last-ulp cases), `/ pi` and `/ 20` as true
//     divisions, torch's CPU sums and FMA-accumulated norm. GPU
//     (DGX_HOG_VOTES_DEVICE): ocml acosf / atanf (the functions torch's HIP
//     kernels call), division by a Python scalar as a multiply by its fp32
//     reciprocal (torch's div_true_kernel_cuda), .int() as v_cvt_i32_f32 (NaN
//     -> 0, saturating), the reduce kernel's order for the bin sums and the
//     norm (NormTwoOps: acc + x*x, contracted to an FMA).
// .int() truncation, votes and bin sums in reference order; L2 normalisation
// with eps 1e-12. Compiled without FMA contraction so each fp op rounds once
// (the norm's FMA is explicit).
#pragma clang fp contract(off)

#include "common.h"
#include "svd3.h"

#define HOG_MAX_K 64

// torch's CPU sum over a strided dim of length k (the reference's .mean(dim=2)
// and .sum(dim=2), SumKernel.cpp row_sum): four interleaved partial sums over
// the first 4*(k/4) items, the remainder added to partial 0, then
// ((p0 + p1) + p2) + p3. slot(l, j) enumerates partial l's items in order.
__device__ __forceinline__ int ilp_count(int k, int l) { return k / 4 + (l == 0 ? k % 4 : 0); }
__device__ __forceinline__ int ilp_item(int k, int l, int j) { return j < k / 4 ? 4 * j + l : 4 * (k / 4) + (j - k / 4); }
// torch's GPU reduce kernel (Reduce.cuh thread_reduce_impl, vt0 = 4) over a
// non-innermost dim of length k: accumulator l takes items l, l+4, ... of the
// 4*(k/4) head, then tail item 4*(k/4)+t goes to accumulator t.
__device__ __forceinline__ int gpu_count(int k, int l) { return k / 4 + (l < k % 4 ? 1 : 0); }
__device__ __forceinline__ int gpu_item(int k, int l, int j) { return 4 * j + l; }
template <bool DEV>
__device__ __forceinline__ int red_count(int k, int l) { return DEV ? gpu_count(k, l) : ilp_count(k, l); }
template <bool DEV>
__device__ __forceinline__ int red_item(int k, int l, int j) { return DEV ? gpu_item(k, l, j) : ilp_item(k, l, j); }

// One thread per point n of cloud 0: axis[n] = (v0, v1, v2, sqrt(sigma0)).
// DMEAN: the mean as torch's GPU kernel takes it (sum in the reduce kernel's
// order, times mfac = float(outputs) / numel); else CPU (ILP-4 sum / k).
template <bool DMEAN>
__global__ __launch_bounds__(64) void hog_axis_kernel(const float* __restrict__ x, const int64_t* __restrict__ idx,
                                                      int N, int k, float mfac, float4* __restrict__ axis) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const float* rows = x;  // view(B*N, 3) of the contiguous (B, 3, N) buffer
    const int64_t* nb = idx + (int64_t)n * k;
    float mean[3] = {0.f, 0.f, 0.f};
    for (int l = 0; l < 4; ++l) {
        float p[3] = {0.f, 0.f, 0.f};
        for (int j = 0; j < red_count<DMEAN>(k, l); ++j) {
            const float* r = rows + 3 * nb[red_item<DMEAN>(k, l, j)];
            for (int c = 0; c < 3; ++c) p[c] += r[c];
        }
        for (int c = 0; c < 3; ++c) mean[c] = l == 0 ? p[c] : mean[c] + p[c];
    }
    // CPU: mean = sum.div_(k); GPU: MeanOps::project, sum * factor
    for (int c = 0; c < 3; ++c) mean[c] = DMEAN ? mean[c] * mfac : mean[c] / (float)k;
    svd3::real A[HOG_MAX_K * 3];
    for (int s = 0; s < k; ++s) {
        const float* r = rows + 3 * nb[s];
        for (int c = 0; c < 3; ++c) A[s * 3 + c] = (svd3::real)(r[c] - mean[c]);
    }
    svd3::real s0, v[3];
    svd3::dominant_right_vector(A, k, &s0, v);
    const float sf = (float)s0;
    // np.sqrt of the fp32 singular value: fp64 sqrt rounded once to fp32 is the
    // correctly rounded fp32 sqrt
    axis[n] = make_float4((float)v[0], (float)v[1], (float)v[2], (float)sqrt((double)sf));
}

// Floor-mod as torch.remainder (exact for these small integer / half values).
__device__ __forceinline__ float fmod_floor(float a, float m) {
    float r = fmodf(a, m);
    if (r != 0.f && (r < 0.f) != (m < 0.f)) r += m;
    return r;
}

template <bool DEV>
__device__ __forceinline__ float to_cell(float deg) {
    // .int() truncates toward zero; cells < 0 get +180 (model_partseg.py:62-64).
    // Host: x86's cvttss2si gives INT_MIN for NaN / out-of-range. GPU:
    // v_cvt_i32_f32 gives 0 for NaN and saturates.
    float c;
    if (DEV) c = deg != deg ? 0.f : (deg >= 2147483648.f ? 2147483647.f : (deg <= -2147483648.f ? -2147483648.f
                                                                                                 : truncf(deg)));
    else c = (deg != deg || fabsf(deg) >= 2147483648.f) ? -2147483648.f : truncf(deg);
    return c < 0.f ? c + 180.f : c;
}

// One thread per (cloud, point): out[b, n, bin, angle] (B, N, 9, 2).
// DVOTE: the vote ops as torch's GPU kernels evaluate them (see the header).
template <bool DVOTE>
__global__ __launch_bounds__(256) void hog_hist_kernel(const float4* __restrict__ axis,
                                                       const int64_t* __restrict__ idx, int BN, int k,
                                                       float* __restrict__ out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= BN) return;
    const float pi = 3.14159265358979323846f;  // np.pi as the fp32 scalar operand
    // the GPU's division by a Python scalar: a * (1.0f / float(scalar))
    const float inv_pi = 1.0f / pi, inv20 = 1.0f / 20.0f;
    const int64_t* nb = idx + (int64_t)p * k;
    float F[2][9], S[2][9];  // bin sums: first votes into bin c, second votes from bin c
    for (int l = 0; l < 4; ++l) {
        float f[2][9], sv[2][9];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int c = 0; c < 9; ++c) f[a][c] = sv[a][c] = 0.f;
        for (int j = 0; j < red_count<DVOTE>(k, l); ++j) {
            const float4 g = axis[nb[red_item<DVOTE>(k, l, j)]];
            float cell[2];
            if (DVOTE) {   // ocml acosf / atanf, * 180 then * (1 / pi)
                cell[0] = to_cell<true>(acosf(g.z) * 180.f * inv_pi);
                cell[1] = to_cell<true>(atanf(g.y / g.x) * 180.f * inv_pi);
            } else {
                // acos / atan rounded from fp64 (the host libm results, correctly rounded
                // but for rare last-ulp cases), then * 180 and / pi as two fp32 ops
                const float zen = (float)acos((double)g.z);
                const float azi = (float)atan((double)(g.y / g.x));
                cell[0] = to_cell<false>(zen * 180.f / pi);
                cell[1] = to_cell<false>(azi * 180.f / pi);
            }
            const float m = g.w;
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const float q = DVOTE ? cell[a] * inv20 : cell[a] / 20.f;
                const float bin = fmod_floor(floorf(q - 0.5f), 9.f);
                const float r1 = m * fmod_floor(20.f * (fmod_floor(bin + 1.f, 9.f) + 0.5f) - cell[a], 180.f);
                const float r2 = m * fmod_floor(cell[a] - 20.f * (bin + 0.5f), 180.f);
                const float first = DVOTE ? r1 * inv20 : r1 / 20.f;
                const float second = DVOTE ? r2 * inv20 : r2 / 20.f;
                const int b = (int)bin;
#pragma unroll
                for (int c = 0; c < 9; ++c) {
                    f[a][c] += b == c ? first : 0.f;
                    sv[a][c] += b == c ? second : 0.f;
                }
            }
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int c = 0; c < 9; ++c) {
                F[a][c] = l == 0 ? f[a][c] : F[a][c] + f[a][c];
                S[a][c] = l == 0 ? sv[a][c] : S[a][c] + sv[a][c];
            }
    }
    float h[9][2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        float ss = 0.f;
#pragma unroll
        for (int c = 0; c < 9; ++c) {
            // histogram[c] = (0 + F_c) + S_{c-1} (loop c adds F_c, loop c-1 adds S_{c-1})
            h[c][a] = c == 0 ? (0.f + S[a][8]) + F[a][0] : (0.f + S[a][c - 1]) + F[a][c];
            if (!DVOTE) ss = fmaf(h[c][a], h[c][a], ss);  // torch's CPU norm accumulates with FMA
        }
        if (DVOTE) {   // the GPU reduce order over the 9 bins: items 0,4,8 | 1,5 | 2,6 | 3,7
            float acc[4];
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                acc[l] = 0.f;
#pragma unroll
                for (int c = l; c < 9; c += 4) acc[l] = fmaf(h[c][a], h[c][a], acc[l]);
            }
            ss = ((acc[0] + acc[1]) + acc[2]) + acc[3];
        }
        const float den = fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
        for (int c = 0; c < 9; ++c) h[c][a] = h[c][a] / den;
    }
    float2* o = reinterpret_cast<float2*>(out + (int64_t)p * 18);
#pragma unroll
    for (int c = 0; c < 9; ++c) o[c] = make_float2(h[c][0], h[c][1]);
}

extern "C" {

int dgx_hog_1x1_sem_f32(const float* x, const int64_t* idx, int B, int N, int k, int sem, float* axis, float* out,
                        void* stream) {
    if (!x || !idx || !axis || !out || B < 0 || N < 1 || k < 1 || k > N) return DGX_EINVAL;
    if (sem & ~(DGX_HOG_MEAN_DEVICE | DGX_HOG_VOTES_DEVICE)) return DGX_EINVAL;
    if (k < 5 || k > HOG_MAX_K) return DGX_EUNSUPPORTED;  // svd3.h restates dgesdd's M >> N path only
    if (B == 0) return DGX_OK;
    hipStream_t st = dgx_stream(stream);
    // MeanOps' factor: static_cast<float>(num_outputs) / numel (an int64 promoted to float)
    const int64_t nout = (int64_t)B * N * 3;
    const float mfac = (float)nout / (float)(nout * k);
    if (sem & DGX_HOG_MEAN_DEVICE)
        hipLaunchKernelGGL(hog_axis_kernel<true>, dim3((N + 63) / 64), dim3(64), 0, st, x, idx, N, k, mfac,
                           reinterpret_cast<float4*>(axis));
    else
        hipLaunchKernelGGL(hog_axis_kernel<false>, dim3((N + 63) / 64), dim3(64), 0, st, x, idx, N, k, mfac,
                           reinterpret_cast<float4*>(axis));
    DGX_CHECK_LAUNCH();
    const int BN = B * N;
    if (sem & DGX_HOG_VOTES_DEVICE)
        hipLaunchKernelGGL(hog_hist_kernel<true>, dim3((BN + 255) / 256), dim3(256), 0, st,
                           reinterpret_cast<const float4*>(axis), idx, BN, k, out);
    else
        hipLaunchKernelGGL(hog_hist_kernel<false>, dim3((BN + 255) / 256), dim3(256), 0, st,
                           reinterpret_cast<const float4*>(axis), idx, BN, k, out);
    DGX_CHECK_LAUNCH();
    return DGX_OK;
}

int dgx_hog_1x1_f32(const float* x, const int64_t* idx, int B, int N, int k, float* axis, float* out,
                    void* stream) {
    return dgx_hog_1x1_sem_f32(x, idx, B, N, k, 0, axis, out, stream);
}

}  // extern "C"
