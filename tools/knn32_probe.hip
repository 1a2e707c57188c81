// Probe (not product): the Gram stream of a kNN selection kernel on
// v_mfma_f32_32x32x2_f32 (32 queries per wave, 32-candidate tiles, 16
// candidates per lane per tile) against the current 16x16x4 layout's rate.
// Variants: mode 0 = MFMA chain only (values folded into a running max),
// mode 1 = + a FIFO admission pass (2 subs, compare, 8-byte LDS store, count).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/knn32_probe.hip -o /tmp/knn32_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int NS, int P, int MODE, int UNIT>
__global__ __launch_bounds__(64 * P) void probe(const float* __restrict__ img, const float* __restrict__ xximg,
                                                int N, float thr0, float* __restrict__ out) {
    constexpr int QCAP = 24;
    __shared__ float2 fifo[MODE == 1 ? P * QCAP * 64 : 1];
    const int ntile = N / 32;
    const int nqb = ntile;
    const int b = blockIdx.x / nqb, qs = blockIdx.x % nqb;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
    const float* ib = img + (size_t)b * ntile * 64 * NS;
    const float* xib = xximg + (size_t)b * ntile * 32;
    float bq[NS];
#pragma unroll
    for (int t = 0; t < NS; ++t) bq[t] = 2.f * ib[((size_t)qs * 64 + lane) * NS + t];
    const float xxq = xib[qs * 32 + (lane & 31)];
    float best = -1e30f;
    int cnt = 0;
    float2* fq = fifo + (wave * QCAP) * 64 + lane;
    const float thr = thr0;
    constexpr int NU = NS / UNIT;
    float a[2][UNIT];
    auto load = [&](int slot, int tl, int u) {
        const int s = wave + P * (tl < ntile / P ? tl : ntile / P - 1);
        const float4* p = reinterpret_cast<const float4*>(ib + ((size_t)s * 64 + lane) * NS + u * UNIT);
        if constexpr (UNIT % 4 == 0) {
#pragma unroll
            for (int v = 0; v < UNIT / 4; ++v) {
                float4 q = p[v];
                a[slot][4 * v] = q.x; a[slot][4 * v + 1] = q.y; a[slot][4 * v + 2] = q.z; a[slot][4 * v + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int v = 0; v < UNIT; ++v) a[slot][v] = ib[((size_t)s * 64 + lane) * NS + u * UNIT + v];
        }
    };
    const int ntl = ntile / P;
    load(0, 0, 0);
    int slot = 0;
    for (int tl = 0; tl < ntl; ++tl) {
        f32x16 acc = {};
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int nu = u + 1 < NU ? u + 1 : 0;
            const int ntl2 = u + 1 < NU ? tl : tl + 1;
            load(slot ^ 1, ntl2, nu);
#pragma unroll
            for (int t = 0; t < UNIT; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[slot][t], bq[u * UNIT + t], acc, 0, 0, 0);
            slot ^= 1;
        }
        const int s = wave + P * tl;
        float xc[16];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 q = *reinterpret_cast<const float4*>(xib + s * 32 + 8 * m + 4 * h);
            xc[4 * m] = q.x; xc[4 * m + 1] = q.y; xc[4 * m + 2] = q.z; xc[4 * m + 3] = q.w;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float v = (acc[r] - xc[r]) - xxq;
            if constexpr (MODE == 0) {
                best = fmaxf(best, v);
            } else {
                const int j = s * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                fq[cnt * 64] = make_float2(v, __int_as_float(j));
                cnt += v >= thr ? 1 : 0;
            }
        }
        if constexpr (MODE == 1) {
            if (__any(cnt > QCAP - 16)) {
                for (int i = 0; i < cnt; ++i) best = fmaxf(best, fq[i * 64].x);
                cnt = 0;
            }
        }
    }
    out[blockIdx.x * 64 * P + threadIdx.x] = best + (float)cnt;
}

template <int NS, int P, int MODE, int UNIT>
float run(int B, int N, const float* img, const float* xximg, float* out, float thr) {
    const int grid = B * (N / 32);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe<NS, P, MODE, UNIT>), dim3(grid), dim3(64 * P), 0, 0, img, xximg, N, thr, out);
    CHECK(hipEventRecord(e0));
    const int reps = 20;
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((probe<NS, P, MODE, UNIT>), dim3(grid), dim3(64 * P), 0, 0, img, xximg, N, thr, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps * 1e3f;
}

int main() {
    const int B = 32, N = 1024;
    const size_t maxns = 64;
    std::vector<float> h((size_t)B * (N / 32) * 64 * maxns);
    for (auto& v : h) v = (float)(rand() % 1000) / 1000.f;
    std::vector<float> hx((size_t)B * N);
    for (auto& v : hx) v = (float)(rand() % 1000) / 100.f;
    float *img, *xximg, *out;
    CHECK(hipMalloc(&img, h.size() * 4));
    CHECK(hipMalloc(&xximg, hx.size() * 4));
    CHECK(hipMalloc(&out, (size_t)B * N * 64 * 8 * 4));
    CHECK(hipMemcpy(img, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(xximg, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    const double pairs = (double)B * N * N;
    auto rep = [&](const char* name, int C, float us) {
        printf("%-34s C=%3d  %8.2f us  %6.1f TF/s  (%.3f of 157.3)\n", name, C, us, 2.0 * pairs * C / (us * 1e-6) / 1e12,
               2.0 * pairs * C / (us * 1e-6) / 1e12 / 157.3);
    };
    rep("mfma-only NS=2  P=4", 3, run<2, 4, 0, 2>(B, N, img, xximg, out, 0.f));
    rep("fifo      NS=2  P=4 thr=hi", 3, run<2, 4, 1, 2>(B, N, img, xximg, out, 1e30f));
    rep("mfma-only NS=32 P=4 unit8", 64, run<32, 4, 0, 8>(B, N, img, xximg, out, 0.f));
    rep("mfma-only NS=32 P=4 unit16", 64, run<32, 4, 0, 16>(B, N, img, xximg, out, 0.f));
    rep("fifo      NS=32 P=4 unit8 thr=hi", 64, run<32, 4, 1, 8>(B, N, img, xximg, out, 1e30f));
    rep("mfma-only NS=32 P=2 unit8", 64, run<32, 2, 0, 8>(B, N, img, xximg, out, 0.f));
    rep("mfma-only NS=64 P=4 unit16", 128, run<64, 4, 0, 16>(B, N, img, xximg, out, 0.f));
    rep("mfma-only NS=64 P=4 unit8", 128, run<64, 4, 0, 8>(B, N, img, xximg, out, 0.f));
    rep("fifo      NS=64 P=4 unit16 thr=hi", 128, run<64, 4, 1, 16>(B, N, img, xximg, out, 1e30f));
    CHECK(hipDeviceSynchronize());
    return 0;
}
