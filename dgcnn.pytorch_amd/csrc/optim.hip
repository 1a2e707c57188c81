// Multi-tensor SGD: torch.optim.SGD's update (momentum, dampening, weight
// decay, Nesterov, maximize) over a list of fp32 parameters in ONE launch.
//
// torch's fused SGD (multi_tensor_apply, 65536-element chunks, one workgroup
// per chunk) runs a DGCNN's ~0.6 M parameters on ~22 workgroups: 28 us per
// train step at cfg2, latency-bound. Here each tensor is cut into 1024-element
// pieces, one workgroup per piece (the piece's tensor is found by a
// workgroup-uniform search of the piece offsets), four consecutive elements
// per thread with 16-byte accesses where aligned. Per element, in torch's
// order (torch/optim/sgd.py):
//   g = maximize ? -grad : grad;  g = g + wd * p
//   buf = first ? g : momentum * buf + (1 - dampening) * g
//   g = nesterov ? g + momentum * buf : buf;   p = p - lr * g
#include "common.h"

namespace {

constexpr int SGD_MAX = 48;   // tensors per launch (kernel argument block)

struct SgdJobs {
    float* p[SGD_MAX];
    const float* g[SGD_MAX];
    float* m[SGD_MAX];
    int64_t numel[SGD_MAX];
    int blk[SGD_MAX + 1];   // first workgroup of each tensor, blk[n] = grid
    int n;
};

constexpr int SGD_PIECE = 1024;   // elements per workgroup (256 threads x 4)

__device__ __forceinline__ float sgd_elem(float pv, float g, float* m, int64_t i, float lr, float wd, float mom,
                                          float damp, int nesterov, int maximize, int first) {
    if (maximize) g = -g;
    if (wd != 0.f) g = g + wd * pv;
    if (mom != 0.f) {
        const float b = first ? g : mom * m[i] + (1.f - damp) * g;
        m[i] = b;
        g = nesterov ? g + mom * b : b;
    }
    return pv - lr * g;
}

__global__ __launch_bounds__(256) void sgd_kernel(SgdJobs J, float lr, float wd, float mom, float damp, int nesterov,
                                                  int maximize, int first) {
    int lo = 0, hi = J.n - 1;   // the tensor t with blk[t] <= blockIdx.x < blk[t + 1] (workgroup-uniform)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (J.blk[mid] <= (int)blockIdx.x) lo = mid;
        else hi = mid - 1;
    }
    float* __restrict__ p = J.p[lo];
    const float* __restrict__ gr = J.g[lo];
    float* __restrict__ m = J.m[lo];
    const int64_t n = J.numel[lo];
    const int64_t i0 = (int64_t)(blockIdx.x - J.blk[lo]) * SGD_PIECE + 4 * threadIdx.x;
    const bool vec = i0 + 3 < n && ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(gr) |
                                     reinterpret_cast<uintptr_t>(m)) & 15) == 0;
    if (vec) {
        const float4 pv = *reinterpret_cast<const float4*>(p + i0);
        const float4 gv = *reinterpret_cast<const float4*>(gr + i0);
        float4 o;
        o.x = sgd_elem(pv.x, gv.x, m, i0, lr, wd, mom, damp, nesterov, maximize, first);
        o.y = sgd_elem(pv.y, gv.y, m, i0 + 1, lr, wd, mom, damp, nesterov, maximize, first);
        o.z = sgd_elem(pv.z, gv.z, m, i0 + 2, lr, wd, mom, damp, nesterov, maximize, first);
        o.w = sgd_elem(pv.w, gv.w, m, i0 + 3, lr, wd, mom, damp, nesterov, maximize, first);
        *reinterpret_cast<float4*>(p + i0) = o;
    } else {
        for (int64_t i = i0; i < min(n, i0 + 4); ++i)
            p[i] = sgd_elem(p[i], gr[i], m, i, lr, wd, mom, damp, nesterov, maximize, first);
    }
}

}  // namespace

extern "C" {

int dgx_sgd_step_f32(int n, float* const* params, const float* const* grads, float* const* momentum_bufs,
                     const int64_t* numels, float lr, float weight_decay, float momentum, float dampening,
                     int nesterov, int maximize, int first, void* stream) {
    if (n < 0 || n > SGD_MAX || (n > 0 && (!params || !grads || !numels))) return DGX_EINVAL;
    if (momentum != 0.f && !momentum_bufs) return DGX_EINVAL;
    if (n == 0) return DGX_OK;
    SgdJobs J{};
    J.n = n;
    J.blk[0] = 0;
    for (int t = 0; t < n; ++t) {
        if (!params[t] || !grads[t] || numels[t] < 0 || (momentum != 0.f && !momentum_bufs[t])) return DGX_EINVAL;
        J.p[t] = params[t];
        J.g[t] = grads[t];
        J.m[t] = momentum != 0.f ? momentum_bufs[t] : nullptr;
        J.numel[t] = numels[t];
        const int64_t pieces = (numels[t] + SGD_PIECE - 1) / SGD_PIECE;
        if ((int64_t)J.blk[t] + pieces > (1LL << 30)) return DGX_EUNSUPPORTED;
        J.blk[t + 1] = J.blk[t] + (int)pieces;
    }
    if (J.blk[n] == 0) return DGX_OK;
    hipLaunchKernelGGL(sgd_kernel, dim3((unsigned)J.blk[n]), dim3(256), 0, dgx_stream(stream), J, lr, weight_decay,
                       momentum, dampening, nesterov, maximize, first);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

}  // extern "C"
