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
// Arithmetic follows the reference op by op as torch's CPU kernels evaluate it
// (the golden fixture's device): neighbourhood mean = fp32 sum in torch's CPU
// order / k;
// SVD in fp64 exactly as numpy's dgesdd path (svd3.h), rounded to fp32;
// magnitude = fp32 sqrt of the fp32 singular value; angle * 180 / pi as two
// fp32 ops; .int() truncation; votes and bin sums in reference order; L2
// normalisation with eps 1e-12. Compiled without FMA contraction so each fp op
// rounds once, as on the reference's host.
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

// One thread per point n of cloud 0: axis[n] = (v0, v1, v2, sqrt(sigma0)).
__global__ __launch_bounds__(64) void hog_axis_kernel(const float* __restrict__ x, const int64_t* __restrict__ idx,
                                                      int N, int k, float4* __restrict__ axis) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const float* rows = x;  // view(B*N, 3) of the contiguous (B, 3, N) buffer
    const int64_t* nb = idx + (int64_t)n * k;
    float mean[3] = {0.f, 0.f, 0.f};
    for (int l = 0; l < 4; ++l) {
        float p[3] = {0.f, 0.f, 0.f};
        for (int j = 0; j < ilp_count(k, l); ++j) {
            const float* r = rows + 3 * nb[ilp_item(k, l, j)];
            for (int c = 0; c < 3; ++c) p[c] += r[c];
        }
        for (int c = 0; c < 3; ++c) mean[c] = l == 0 ? p[c] : mean[c] + p[c];
    }
    for (int c = 0; c < 3; ++c) mean[c] = mean[c] / (float)k;  // mean = sum.div_(k) on CPU
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

__device__ __forceinline__ float to_cell(float deg) {
    // .int() truncates toward zero; cells < 0 get +180 (model_partseg.py:62-64)
    // (x86's cvttss2si gives INT_MIN for NaN / out-of-range, as on the reference's host)
    const float c = (deg != deg || fabsf(deg) >= 2147483648.f) ? -2147483648.f : truncf(deg);
    return c < 0.f ? c + 180.f : c;
}

// One thread per (cloud, point): out[b, n, bin, angle] (B, N, 9, 2).
__global__ __launch_bounds__(256) void hog_hist_kernel(const float4* __restrict__ axis,
                                                       const int64_t* __restrict__ idx, int BN, int k,
                                                       float* __restrict__ out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= BN) return;
    const float pi = 3.14159265358979323846f;  // np.pi as the fp32 scalar operand
    const int64_t* nb = idx + (int64_t)p * k;
    float F[2][9], S[2][9];  // bin sums: first votes into bin c, second votes from bin c
    for (int l = 0; l < 4; ++l) {
        float f[2][9], sv[2][9];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int c = 0; c < 9; ++c) f[a][c] = sv[a][c] = 0.f;
        for (int j = 0; j < ilp_count(k, l); ++j) {
            const float4 g = axis[nb[ilp_item(k, l, j)]];
            // acos / atan rounded from fp64 (the host libm results, correctly rounded
            // but for rare last-ulp cases), then * 180 and / pi as two fp32 ops
            const float zen = (float)acos((double)g.z);
            const float azi = (float)atan((double)(g.y / g.x));
            const float cell[2] = {to_cell(zen * 180.f / pi), to_cell(azi * 180.f / pi)};
            const float m = g.w;
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const float bin = fmod_floor(floorf(cell[a] / 20.f - 0.5f), 9.f);
                const float first = m * fmod_floor(20.f * (fmod_floor(bin + 1.f, 9.f) + 0.5f) - cell[a], 180.f) / 20.f;
                const float second = m * fmod_floor(cell[a] - 20.f * (bin + 0.5f), 180.f) / 20.f;
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
            ss = fmaf(h[c][a], h[c][a], ss);  // torch's CPU norm accumulates with FMA
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

int dgx_hog_1x1_f32(const float* x, const int64_t* idx, int B, int N, int k, float* axis, float* out,
                    void* stream) {
    if (!x || !idx || !axis || !out || B < 0 || N < 1 || k < 1 || k > N) return DGX_EINVAL;
    if (k < 5 || k > HOG_MAX_K) return DGX_EUNSUPPORTED;  // svd3.h restates dgesdd's M >> N path only
    if (B == 0) return DGX_OK;
    hipStream_t st = dgx_stream(stream);
    hipLaunchKernelGGL(hog_axis_kernel, dim3((N + 63) / 64), dim3(64), 0, st, x, idx, N, k,
                       reinterpret_cast<float4*>(axis));
    DGX_CHECK_LAUNCH();
    const int BN = B * N;
    hipLaunchKernelGGL(hog_hist_kernel, dim3((BN + 255) / 256), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(axis), idx, BN, k, out);
    DGX_CHECK_LAUNCH();
    return DGX_OK;
}

}  // extern "C"
