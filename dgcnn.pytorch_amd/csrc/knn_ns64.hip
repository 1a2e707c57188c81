// Instantiation unit of the kNN selection kernel for NS = 64 MFMA steps per
// tile (knn_kernel.h), compiled apart so the kernel variants build in parallel.
#include "knn_kernel.h"

namespace dgx_knn {
template int dispatch_k<64>(const float* xx, int B, int N, int k, int64_t* idx64, int32_t* idx32, float* vals,
                             const float* img, const float* xximg, hipStream_t st);
}  // namespace dgx_knn
