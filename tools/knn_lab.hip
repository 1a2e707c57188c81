// kNN selection lab (not product): times knn_kernel at the cfg2/cfg3 layer
// shapes and splits each wave's time into phases from the KNN_MARK clock marks
// (knn_kernel.h, compiled in only here with DGX_KNN_LAB).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/knn_lab.hip -o tools/knn_lab [-D...]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define DGX_KNN_LAB
__device__ long long* g_lab;
#define DGX_KNN_LAB_BUF g_lab
#include "../dgcnn.pytorch_amd/csrc/knn_kernel.h"

using namespace dgx_knn;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static const char* kPhase[9] = {"xs+seed", "prepass", "stream", "flush", "2-merge", "barrier", "rank", "write", "fixup"};

template <int NS, int KB>
void run_case(const char* name, int B, int N, int C, int k, bool cube, int reps) {
    const int ntile = knn_ntile(N);
    std::mt19937 rng(1234 + C + N);
    std::uniform_real_distribution<float> uni(0.f, 1.f);
    std::normal_distribution<float> nrm(0.f, 1.f);
    std::vector<float> x((size_t)B * N * C);
    for (auto& v : x) v = cube ? uni(rng) : std::max(0.f, nrm(rng));
    std::vector<float> img((size_t)B * ntile * 64 * NS, 0.f), xximg((size_t)B * ntile * KT, 0.f), xx((size_t)B * N);
    for (int b = 0; b < B; ++b)
        for (int n = 0; n < N; ++n) {
            const float* p = &x[((size_t)b * N + n) * C];
            float s = 0.f;
            for (int c = 0; c < C; ++c) s += p[c] * p[c];
            xx[(size_t)b * N + n] = s;
            xximg[((size_t)b * ntile + n / KT) * KT + n % KT] = s;
            for (int t = 0; t < NS; ++t)
                for (int h = 0; h < 2; ++h) {
                    const int c = 2 * t + h;
                    img[(size_t)b * ntile * 64 * NS + img_at<NS>(n / KT, h * 32 + n % KT, t)] = c < C ? p[c] : 0.f;
                }
        }
    float *dimg, *dxximg, *dxx;
    int32_t* didx;
    long long* dlab;
    const int grid = dgx_xcd_cloud_grid(B, ntile);
    const size_t nlab = (size_t)grid * KP * 16;
    CHECK(hipMalloc(&dimg, img.size() * 4));
    CHECK(hipMalloc(&dxximg, xximg.size() * 4));
    CHECK(hipMalloc(&dxx, xx.size() * 4));
    CHECK(hipMalloc(&didx, (size_t)B * N * k * 4));
    CHECK(hipMalloc(&dlab, nlab * 8));
    CHECK(hipMemcpy(dimg, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dxximg, xximg.data(), xximg.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dxx, xx.data(), xx.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemset(dlab, 0, nlab * 8));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_lab), &dlab, sizeof(dlab)));
    auto launch = [&]() {
        if (launch_knn<NS, KB>(dxx, B, N, k, nullptr, didx, nullptr, dimg, dxximg, 0) != DGX_OK) {
            printf("launch failed\n");
            exit(1);
        }
    };
    for (int w = 0; w < 3; ++w) launch();
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    for (int w = 0; w < reps; ++w) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> lab(nlab);
    CHECK(hipMemcpy(lab.data(), dlab, nlab * 8, hipMemcpyDeviceToHost));
    std::vector<int32_t> idx((size_t)B * N * k);
    CHECK(hipMemcpy(idx.data(), didx, idx.size() * 4, hipMemcpyDeviceToHost));
    uint64_t h = 1469598103934665603ull;
    for (int32_t v : idx) h = (h ^ (uint32_t)v) * 1099511628211ull;
    double ph[9] = {0};
    double tot = 0, fl = 0, nfl = 0;
    long long fix = 0;
    int nw = 0;
    for (int blk = 0; blk < grid; ++blk) {
        const long long* m0 = &lab[(size_t)blk * KP * 16];
        if (m0[0] == 0) continue;   // padding block
        fix += m0[15];
        for (int w = 0; w < KP; ++w) {
            const long long* m = m0 + w * 16;
            for (int i = 0; i < 9; ++i) ph[i] += (double)(m[i + 1] - m[i]);
            tot += (double)(m[9] - m[0]);
            fl += (double)m[12];
            nfl += (double)m[13];
            ++nw;
        }
    }
    const double flops = 2.0 * B * (double)N * N * C;
    printf("%-16s NS=%2d KB=%2d  %8.2f us  %6.1f TF/s  fixrows=%lld  hash=%016llx\n", name, NS, KB, ms / reps * 1e3,
           flops / (ms / reps * 1e-3) / 1e12, fix, (unsigned long long)h);
    printf("   cycles/wave: total %.0f |", tot / nw);
    for (int i = 0; i < 9; ++i) printf(" %s %.0f", kPhase[i], ph[i] / nw);
    printf(" | in-stream flushes %.2f taking %.0f\n", nfl / nw, fl / nw);
    CHECK(hipFree(dimg));
    CHECK(hipFree(dxximg));
    CHECK(hipFree(dxx));
    CHECK(hipFree(didx));
    CHECK(hipFree(dlab));
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    run_case<2, 20>("C3 N1024 k20", 32, 1024, 3, 20, true, reps);
    run_case<32, 20>("C64 N1024 k20", 32, 1024, 64, 20, false, reps);
    run_case<64, 20>("C128 N1024 k20", 32, 1024, 128, 20, false, reps);
    run_case<2, 40>("C3 N2048 k40", 32, 2048, 3, 40, true, reps);
    run_case<32, 40>("C64 N2048 k40", 32, 2048, 64, 40, false, reps);
    return 0;
}
