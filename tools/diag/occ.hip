// Occupancy check for the kNN kernels (diagnostic, not part of the library).
#include "../../dgcnn.pytorch_amd/csrc/knn.hip"
#include <cstdio>
int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("lds/block %zu lds/CU %zu optin %zu CUs %d\n", p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor,
           p.sharedMemPerBlockOptin, p.multiProcessorCount);
    int n = -1;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, knn_kernel<16, 20, false>, KQ_THREADS, 0);
    printf("knn<16,20,false> blocks/CU %d\n", n);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, knn_kernel<32, 20, false>, KQ_THREADS, 0);
    printf("knn<32,20,false> blocks/CU %d\n", n);
    hipFuncAttributes a;
    hipFuncGetAttributes(&a, reinterpret_cast<const void*>(knn_kernel<16, 20, false>));
    printf("attr: shared %zu regs %d maxthreads %d local %zu\n", a.sharedSizeBytes, a.numRegs, a.maxThreadsPerBlock, a.localSizeBytes);
    return 0;
}
