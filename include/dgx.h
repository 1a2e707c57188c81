/*
 * dgx — MI355X-native EdgeConv engine, C ABI (libdgx.so).
 *
 * The reference (QasimKhan5x/dgcnn.pytorch) is pure Python; its "operator API"
 * for the hot path is the set of functions in models/dgcnn.py that every model
 * binds by name (models/layers.py:6, models/model_partseg.py:11). Each entry
 * point below replaces one step of that path and cites the reference lines it
 * stands in for. The Python mirror (dgcnn.pytorch_amd/models/dgcnn.py) binds
 * these through ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - All pointers are DEVICE pointers (HBM) except where noted; the ABI never
 *     allocates, never synchronises, and enqueues on `stream` (a hipStream_t).
 *   - Tensors are described by element strides, so permuted views work
 *     (main_cls.py:91 feeds x as a permute(0,2,1) view).
 *   - "point-major" buffers are (M = B*N rows) x (channels) with a row stride ld.
 *   - Return value: DGX_OK or a negative DGX_E* code; never throws.
 */
#ifndef DGX_H
#define DGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DGX_OK 0
#define DGX_EINVAL (-1)       /* bad shape / argument                          */
#define DGX_EUNSUPPORTED (-2) /* shape outside what the kernels are built for */
#define DGX_ELAUNCH (-3)      /* hipLaunch / runtime error                     */

/* torch CPU reduction order of sum(x**2, dim=1) that the distances must follow */
#define DGX_ORDER_STRIDED 0 /* N-contiguous x: cascade over 16-channel blocks  */
#define DGX_ORDER_VEC8X4 1  /* C-contiguous x: 4x8 vector accumulators         */

/* get_graph_feature output modes, reference models/dgcnn.py:37-44 */
#define DGX_GF_CAT 0      /* (B,2C,N,k): [x_j ; x_i]          dgcnn.py:42-44 */
#define DGX_GF_DISP 1     /* (B,C,N,k):  x_j - x_i            dgcnn.py:39-40 */
#define DGX_GF_KNN_ONLY 2 /* (B,N,k,C):  x_j                  dgcnn.py:37-38 */
#define DGX_GF_DIFFCAT 3  /* (B,2C,N,k): (x_j - x_i, x_i)    test.ipynb:131 (the paper's form) */

const char* dgx_version(void);
const char* dgx_strerror(int code);

/* ---- a1: kNN, replaces models/dgcnn.py:6-12 (knn) -------------------------
 * x: fp32 (B,C,N) with element strides (sB,sC,sN). For every point i returns
 * the k points j with the largest pd_ij = (2 x_i.x_j - |x_j|^2) - |x_i|^2,
 * rounded exactly as the reference's CPU arithmetic (FMA chain over c,
 * `order` for |x|^2), sorted by pd descending, ties by index ascending.
 * Outputs local indices 0..N-1 into idx64 (B,N,k) int64 and/or idx32 (either
 * may be NULL). Workspace: dgx_knn_workspace_bytes(B,C,N), 16-byte aligned.
 * Supports C <= 128, 1 <= k <= min(N, 64). */
size_t dgx_knn_workspace_bytes(int B, int C, int N);
int dgx_knn_f32(const float* x, int64_t sB, int64_t sC, int64_t sN,
                int B, int C, int N, int k, int order,
                int64_t* idx64, int32_t* idx32,
                void* workspace, size_t workspace_bytes, void* stream);

/* The stages of dgx_knn_f32, separately. dgx_sqnorm_f32: |x_i|^2 in the
 * reference's rounding order into xx (B*N fp32, dgcnn.py:8).
 * dgx_knn_prepare_f32: the same xx plus the MFMA operand image of x in
 * `image` (16-byte aligned, dgx_knn_image_bytes(B,C,N)) in one pass over x.
 * dgx_knn_select_f32: the fused distance + top-k pass (dgcnn.py:7-11) over a
 * prepared image and its xx; vals (B,N,k), nullable, receives the selected pd
 * values (what pd.topk(k)[0] would hold). */
size_t dgx_knn_image_bytes(int B, int C, int N);
/* Name of the selection kernel dgx_knn_select_f32 launches for (C, k, N), as
 * rocprofv3 prints it (host-side query; lets profiles be matched to the
 * kernels that actually ran). "" for unsupported (C, k, N). */
const char* dgx_knn_kernel_name(int C, int k, int N);
/* dgx_bn_lrelu_apply_f32 for an EdgeConv block whose output feeds the next
 * block's kNN (dgcnn.py:84-98, the feature-space knn of x_l): writes
 * out = LeakyReLU(scale*ysel + shift) (+ its bf16 twin) AND the next kNN's
 * prepared operands — |x|^2 in the reference's strided-layout order into xx
 * (B*N) and the operand image (dgx_knn_image_bytes(B, Co, N)) — so that kNN
 * runs dgx_knn_select_f32 directly (no dgx_knn_prepare_f32 pass).
 * Co in {64, 128}, N % 32 == 0; else DGX_EUNSUPPORTED. */
int dgx_bn_lrelu_apply_knn_image_f32(const float* ysel, int B, int N, int Co,
                                     const float* scale, const float* shift, float slope,
                                     float* out, int ldo, void* out_bf16, float* xx,
                                     void* image, size_t image_bytes, void* stream);
int dgx_sqnorm_f32(const float* x, int64_t sB, int64_t sC, int64_t sN,
                   int B, int C, int N, int order, float* xx, void* stream);
int dgx_knn_prepare_f32(const float* x, int64_t sB, int64_t sC, int64_t sN,
                        int B, int C, int N, int order, float* xx,
                        void* image, size_t image_bytes, void* stream);
int dgx_knn_select_f32(const float* x, int64_t sB, int64_t sC, int64_t sN,
                       const float* xx, int B, int C, int N, int k,
                       int64_t* idx64, int32_t* idx32, float* vals,
                       const void* image, size_t image_bytes, void* stream);

/* The same kNN for every shape the fused selection kernel is not built for
 * (C > 128, k > 64, N > 12288; the reference, dgcnn.py:6-12, takes any C,
 * k <= N and N): |x|^2 in the reference's order for any C, the Gram chain on
 * dgx_gemm_f32 (one fp32 MFMA accumulation chain per output, c in order), and
 * an exact radix select + bitonic sort per query row — identical values and
 * canonical order. x needs sN == 1 or sC == 1; k <= 8192. Workspace:
 * dgx_knn_generic_workspace_bytes(B,C,N) (|x|^2 + one chunk of dot rows). */
size_t dgx_knn_generic_workspace_bytes(int B, int C, int N);
int dgx_knn_generic_f32(const float* x, int64_t sB, int64_t sC, int64_t sN,
                        int B, int C, int N, int k, int order,
                        int64_t* idx64, int32_t* idx32, float* vals,
                        void* workspace, size_t workspace_bytes, void* stream);

/* ---- a2: edge features, replaces models/dgcnn.py:15-44 (get_graph_feature)
 * after the knn call: idx (B,N,k) int32 local indices. out is contiguous in
 * the layout of `mode` (see DGX_GF_*). */
int dgx_graph_feature_f32(const float* x, int64_t sB, int64_t sC, int64_t sN,
                          int B, int C, int N, const int32_t* idx, int k,
                          int mode, float* out, void* stream);
/* Backward of dgx_graph_feature_f32 (autograd of dgcnn.py:31-44): adds into
 * dx (B,C,N) contiguous. Uses float atomics (summation order not fixed); the
 * CSR form below is the deterministic one, this one serves k > 64. */
int dgx_graph_feature_bwd_f32(const float* dout, int B, int C, int N,
                              const int32_t* idx, int k, int mode, float* dx,
                              void* stream);
/* The same gradient, deterministic: every dx element summed by one thread
 * over the point's in-edges in the reverse graph's order (rowptr / edges from
 * dgx_graph_reverse of the same idx, k <= 64), then its own row's centre
 * terms; no atomics. */
int dgx_graph_feature_bwd_csr_f32(const float* dout, int B, int C, int N, int k,
                                  int mode, const int32_t* rowptr, const int32_t* edges,
                                  float* dx, void* stream);

/* ---- a3: decomposed EdgeConv block, replaces
 *   get_graph_feature -> Conv2d(2C,Co,1,bias=False) -> BatchNorm2d -> LeakyReLU
 *   -> max(dim=-1)                        (models/dgcnn.py:54-73, 84-98)
 * With W = [W1 | W2] (Co x 2C), the conv on edge (i,j) is P_j + Q_i where
 * P = X W1^T, Q = X W2^T (point-major, computed by the caller's GEMM into one
 * buffer PQ (M x 2Co, row stride ldpq): columns [0,Co) = P, [Co,2Co) = Q).
 * idx: (B,N,k) int32 local neighbour indices from dgx_knn_*; M = B*N.
 *
 * Forward (training BN), three launches:
 *   dgx_edge_fwd_gather: per (i,o) max_k P (min_k where gamma[o] < 0: BN's
 *     affine is decreasing there), its slot `arg`, sum_k P `sumP`, and
 *     per-row partial (sum y, sum y^2) over all B*N*k edge outputs y = P_j+Q_i
 *     into partials (nrows x 2 x Co), nrows = dgx_edge_partials_rows(B,N,Co).
 *   dgx_bn_finalize: batch mean/var (biased) -> scale a, shift b, mean,
 *     invstd; running stats updated with unbiased var (nn.BatchNorm rules).
 *   dgx_bn_lrelu_apply: out[i,o] = LeakyReLU(a_o * ysel[i,o] + b_o), written
 *     with row stride ldo (straight into the caller's concat buffer,
 *     models/dgcnn.py:100). */
int dgx_edge_partials_rows(int B, int N, int Co);
int dgx_edge_fwd_gather_f32(const float* PQ, int ldpq, const int32_t* idx,
                            int B, int N, int k, int Co, const float* gamma,
                            float* ysel, uint8_t* arg, float* sumP,
                            float* partials, int nrows, void* stream);
int dgx_bn_finalize_f32(const float* partials, int nrows, int Co, double count,
                        const float* gamma, const float* beta,
                        float* running_mean, float* running_var,
                        double momentum, double eps,
                        float* scale, float* shift, float* mean, float* invstd,
                        int64_t* num_batches_tracked, void* stream);
/* dgx_bn_finalize_f32 writing the updated running statistics (and the
 * incremented batch counter) to separate *_new outputs instead of in place —
 * the form a functional op (torch.library) needs: no private copy of the
 * buffers is made first. dgx_bn_finalize_f32 = this with *_new = the inputs.
 * momentum < 0 selects nn.BatchNorm's cumulative average (momentum=None,
 * torch/nn/modules/batchnorm.py): factor 1 / (*num_batches_tracked + 1) read on
 * the device; the counter must then not alias num_batches_tracked_new. */
int dgx_bn_finalize_out_f32(const float* partials, int nrows, int Co, double count,
                            const float* gamma, const float* beta,
                            const float* running_mean, const float* running_var,
                            double momentum, double eps, float* scale, float* shift,
                            float* mean, float* invstd, const int64_t* num_batches_tracked,
                            float* running_mean_new, float* running_var_new,
                            int64_t* num_batches_tracked_new, void* stream);
int dgx_bn_finalize_out_f64(const double* sums, int nrows, int Co, double count,
                            const float* gamma, const float* beta,
                            const float* running_mean, const float* running_var,
                            double momentum, double eps, float* scale, float* shift,
                            float* mean, float* invstd, const int64_t* num_batches_tracked,
                            float* running_mean_new, float* running_var_new,
                            int64_t* num_batches_tracked_new, void* stream);
/* The same finalize from fp64 column sums (nrows x 2 x Co doubles): the global
 * sums of a SyncBatchNorm all-reduce (main_partseg_dist.py:189), kept in fp64
 * into var = E[y^2] - E[y]^2. count < 0: the element count is the double that
 * follows the sums on the device (all-reduced with them; no host read). */
int dgx_bn_finalize_f64(const double* sums, int nrows, int Co, double count,
                        const float* gamma, const float* beta,
                        float* running_mean, float* running_var,
                        double momentum, double eps,
                        float* scale, float* shift, float* mean, float* invstd,
                        int64_t* num_batches_tracked, void* stream);
int dgx_bn_lrelu_apply_f32(const float* ysel, int M, int Co, const float* scale,
                           const float* shift, float slope, float* out, int ldo,
                           void* out_bf16, void* stream);
/* Eval-mode forward in one launch: out = LeakyReLU(a*sel + b), a,b from
 * running stats (dgx_bn_eval_affine_f32). */
int dgx_bn_eval_affine_f32(int Co, const float* gamma, const float* beta,
                           const float* running_mean, const float* running_var,
                           double eps, float* scale, float* shift, void* stream);
int dgx_edge_fwd_eval_f32(const float* PQ, int ldpq, const int32_t* idx,
                          int B, int N, int k, int Co, const float* scale,
                          const float* shift, float slope, float* out, int ldo,
                          void* stream);

/* Backward of the block (autograd of dgcnn.py:84-98 through BN train mode):
 *   dgx_edge_bwd_dz: dz = dY * LeakyReLU'(z) at the selected edge (M x Co
 *     fp32; the edge is the forward's arg slot), and per-row partials (sum dz,
 *     sum dz*yhat) -> dgx_bn_bwd_finalize: dgamma, dbeta (accumulate != 0
 *     adds to them) and the per-channel affine c0 + c1*y of BN's input grad.
 *   dgx_graph_reverse: reverse kNN graph: rowptr (M+1), edges (M*k), edge id
 *     = (i << 6) | slot, lists sorted (deterministic summation order).
 *   dgx_edge_bwd_scatter: dPQ (M x 2Co): dP_j = a*sum_{selected edges->j} dz +
 *     sum_{edges->j}(c0 + c1*y_e),  dQ_i = a*dz_i + k*c0 + c1*sum_k y_ik.
 * The caller's GEMMs then form dX += dPQ [W1;W2] and dW = dPQ^T X. */
int dgx_edge_bwd_dz_f32(const float* dY, int lddy, const float* ysel,
                        int M, int Co, const float* scale,
                        const float* shift, const float* mean,
                        const float* invstd, float slope, float* dz,
                        float* partials, int nrows, void* stream);
/* dgx_edge_bwd_dz_f32 with the forward's selected slot (arg, M x Co u8) packed
 * into each dz word's low 6 mantissa bits (18 significant bits of dz left):
 * the input of dgx_edge_bwd_scatter_packed_f32, which then reads one LDS word
 * per in-edge and channel instead of a dz word plus a slot byte. Used by the
 * bf16 precision mode (its dPQ is rounded to bf16 afterwards); the fp32 parity
 * mode keeps exact dz. Partials are from the unpacked dz. */
int dgx_edge_bwd_dz_packed_f32(const float* dY, int lddy, const float* ysel,
                               const uint8_t* arg, int M, int Co, const float* scale,
                               const float* shift, const float* mean, const float* invstd,
                               float slope, float* dz_packed, float* partials, int nrows,
                               void* stream);
/* dgx_edge_bwd_dz_f32 for a channel-major dY (B x Co x N, the layout of the
 * gradient of a (B, C, N) module output): same dz (M x Co, point-major) and
 * partials, nrows = dgx_edge_bwd_dz_cm_rows(B, N). */
int dgx_edge_bwd_dz_cm_rows(int B, int N);
int dgx_edge_bwd_dz_cm_f32(const float* dY, const float* ysel, int B, int N, int Co,
                           const float* scale, const float* shift, const float* mean,
                           const float* invstd, float slope, float* dz, float* partials,
                           int nrows, void* stream);
int dgx_bn_bwd_finalize_f32(const float* partials, int nrows, int Co,
                            double count, const float* scale, const float* mean,
                            const float* invstd, float* dgamma, float* dbeta,
                            float* c0, float* c1, int accumulate, void* stream);
/* fp64-sums form (SyncBatchNorm backward, after the all-reduce). */
int dgx_bn_bwd_finalize_f64(const double* sums, int nrows, int Co,
                            double count, const float* scale, const float* mean,
                            const float* invstd, float* dgamma, float* dbeta,
                            float* c0, float* c1, int accumulate, void* stream);
int dgx_graph_reverse(const int32_t* idx, int B, int N, int k,
                      int32_t* rowptr, int32_t* edges, void* stream);
/* The reverse graphs of n <= 8 kNN graphs of the same (B, N, k) — a
 * DGCNN's blocks — in one launch (the graphs' workgroups share the chip). */
int dgx_graph_reverse_multi(int n, const int32_t* const* idx, int B, int N, int k,
                            int32_t* const* rowptr, int32_t* const* edges, void* stream);
/* dPQ output (out_bf16): 0 fp32, 1 bf16, 2 split bf16 planes — hi = bf16(v)
 * at dPQ, lo = bf16(v - hi) at dPQ + B*N*2Co elements — or 3: (hi, lo, hi),
 * hi again at dPQ + 2*B*N*2Co (the fp32 mode's 3-pass GEMM operands; the pull
 * forms below, not the push form). */
int dgx_edge_bwd_scatter_f32(const float* PQ, int ldpq, const int32_t* rowptr,
                             const int32_t* edges, const float* dz,
                             const uint8_t* arg, const float* sumP, int B, int N,
                             int k, int Co, const float* scale, const float* c0,
                             const float* c1, void* dPQ, int out_bf16,
                             void* stream);
/* dgx_bn_bwd_finalize_f32 + dgx_edge_bwd_scatter_f32 in ONE launch: every
 * workgroup reduces the dz pass's partial rows (nrows x 2 x Co) for its own
 * channels in a fixed order (fp64) and the channel slice's first workgroup
 * writes dgamma, dbeta (not accumulated), c0, c1 (c0 = c1 = 0 when eval != 0).
 * packed != 0: dz holds dgx_edge_bwd_dz_packed_f32 words (arg unused). */
int dgx_edge_bwd_scatter_fin_f32(const float* PQ, int ldpq, const int32_t* rowptr,
                                 const int32_t* edges, const float* dz, const uint8_t* arg,
                                 const float* sumP, int B, int N, int k, int Co,
                                 const float* partials, int nrows, double count,
                                 const float* scale, const float* mean, const float* invstd,
                                 int eval, float* dgamma, float* dbeta, float* c0, float* c1,
                                 void* dPQ, int out_bf16, int packed, void* stream);
/* The same dPQ from packed dz|slot words (dgx_edge_bwd_dz_packed_f32). */
int dgx_edge_bwd_scatter_packed_f32(const float* PQ, int ldpq, const int32_t* rowptr,
                                    const int32_t* edges, const float* dz_packed,
                                    const float* sumP, int B, int N, int k, int Co,
                                    const float* scale, const float* c0, const float* c1,
                                    void* dPQ, int out_bf16, void* stream);
/* The same dPQ with the selected-edge term pushed from the sources: each
 * (point i, channel c) adds dz_i[c] to j = idx[i][slot] (idx: the forward's
 * B x N x k kNN graph), summed exactly in 64-bit fixed point (LDS atomics,
 * order-independent, rounded once to fp32), so the in-edge loop reads Q rows
 * only. All modes in one entry: partials != NULL finalizes the BN backward as
 * dgx_edge_bwd_scatter_fin_f32 (else c0 / c1 are inputs, eval ignored);
 * packed != 0 reads dgx_edge_bwd_dz_packed_f32 words (arg unused). A channel
 * whose dz holds inf / NaN gets NaN in every dP of the channel. */
int dgx_edge_bwd_scatter_push_f32(const float* PQ, int ldpq, const int32_t* idx,
                                  const int32_t* rowptr, const int32_t* edges, const float* dz,
                                  const uint8_t* arg, const float* sumP, int B, int N, int k,
                                  int Co, const float* partials, int nrows, double count,
                                  const float* scale, const float* mean, const float* invstd,
                                  int eval, float* dgamma, float* dbeta, float* c0, float* c1,
                                  void* dPQ, int out_bf16, int packed, void* stream);

/* ---- a4: pointwise Conv1x1 + BatchNorm + LeakyReLU, replaces conv5 of
 * models/dgcnn.py:74-78, 100-102 (cat(x1..x4) -> Conv2d(512,emb,1) -> BN ->
 * LeakyReLU -> view(B,emb,N)). The caller's GEMM gives Z = X W^T point-major
 * (M x C, row stride ldz); these passes finish the block:
 *   dgx_colstats: per-row-block (sum z, sum z^2), nrows = dgx_colstats_rows(M)
 *     -> dgx_bn_finalize_f32 (shared with a3) gives scale/shift/mean/invstd.
 *   dgx_pointconv_apply: out (B,C,N) = LeakyReLU(a z + b), LDS-transposed.
 *   dgx_pointconv_bwd: dz = dout * LeakyReLU'(a z + b) (dout (B,C,N)) into
 *     dz (M x C) + partials (nrows = dgx_pointconv_bwd_rows(B,N)) ->
 *     dgx_bn_bwd_finalize_f32 -> c0, c1.
 *   dgx_pointconv_input_grad: dZ = a*dz + c0 + c1*z as fp32 or bf16 (bf16 != 0).
 *   dgx_to_bf16: strided fp32 -> dense bf16 (RNE) operand copy. */
int dgx_colstats_rows(int64_t M);
int dgx_colstats_f32(const float* Z, int ldz, int64_t M, int C, float* partials,
                     int nrows, void* stream);
int dgx_pointconv_apply_f32(const float* Z, int ldz, int B, int N, int C,
                              const float* scale, const float* shift,
                              float slope, float* out, void* stream);
int dgx_pointconv_bwd_rows(int B, int N);
int dgx_pointconv_bwd_f32(const float* dout, const float* Z, int ldz, int B,
                            int N, int C, const float* scale,
                            const float* shift, const float* mean,
                            const float* invstd, float slope, float* dz,
                            float* partials, void* stream);
int dgx_pointconv_input_grad(const float* dz, const float* Z, int ldz, int64_t M,
                         int C, const float* scale, const float* c0,
                         const float* c1, void* dZ, int bf16, void* stream);
int dgx_to_bf16(const float* src, int64_t ld, int64_t rows, int cols, void* dst,
                void* stream);
/* conv5 with a bf16 Z (precision "bf16": dgx_gemm_lds_bf16 epi 4 stores Z as
 * bf16 (M x C, row stride C) with the BN statistics taken from the fp32
 * accumulators — what autocast stores for a conv output).
 *   dgx_pointconv_apply_bf16: out (B,C,N) = LeakyReLU(scale*z + shift).
 *   dgx_pointconv_bwd_bf16 pass 0: partials[dgx_pointconv_bf16_rows(B,N)][2][C]
 *     = per 512-point tile (sum d, sum d*zhat), d = dout * LeakyReLU'(scale*z + shift), zhat =
 *     (z - mean) * invstd; -> dgx_bn_bwd_finalize_f32 -> c0, c1.
 *   pass 1: dZ (bf16, M x C) = scale*d + c0 + c1*z — the GEMM operand of
 *     dW5 = dZ^T X and dX = dZ W5. Replace the reference's autograd of
 *     conv5 + BatchNorm2d + LeakyReLU (dgcnn.py:74-78, 102). */
int dgx_pointconv_bf16_rows(int B, int N);
int dgx_pointconv_apply_bf16(const void* Z, int B, int N, int C, const float* scale,
                             const float* shift, float slope, float* out, void* stream);
int dgx_pointconv_bwd_bf16(const float* dout, const void* Z, int B, int N, int C,
                           const float* scale, const float* shift, const float* mean,
                           const float* invstd, float slope, const float* c0,
                           const float* c1, float* partials, void* dZ, int pass,
                           void* stream);
/* The same two passes for an fp32 Z (dense M x C, C % 4 == 0; fp32 mode with
 * the 3-pass split-bf16 conv5 GEMMs): pass 0 partials as dgx_pointconv_bwd_bf16
 * (dgx_pointconv_bf16_rows rows); pass 1 writes dZ = scale*d + c0 + c1*z (fp32
 * arithmetic, the value dgx_pointconv_input_grad computes) as its split-bf16
 * planes dZ_hi = bf16(dZ), dZ_lo = bf16(dZ - dZ_hi) (dgx_split_bf16), the
 * operands of the split GEMMs — no fp32 dz or dZ round trip. */
int dgx_pointconv_bwd_split_f32(const float* dout, const float* Z, int B, int N, int C,
                                const float* scale, const float* shift, const float* mean,
                                const float* invstd, float slope, const float* c0,
                                const float* c1, float* partials, void* dZ_hi, void* dZ_lo,
                                int pass, void* stream);

/* ---- a3/a4/a8: the Conv2d(1x1) GEMMs of the chain, bf16 MFMA ----------------
 * Replace the reference's per-edge conv GEMMs (models/dgcnn.py:55-73, K11) and
 * conv5 (dgcnn.py:74-78, 100-102, K15) plus their autograd dgrad/wgrad, in the
 * decomposed per-point form:
 *   C[i][j] = sum_k opA(i,k) * opB(j,k),  i < M, j < N, k < K
 *   opA(i,k) = A[i*lda + k] (a_ic = 0) or A[k*lda + i] (a_ic = 1), same for B.
 * A/B are fp32 (x_bf16 = 0) or bf16 (1); operands are rounded to bf16 (RNE)
 * when staged, products accumulate in fp32, C is fp32 with row stride ldc.
 * epi: 0 store, 1 accumulate (C += ...), 2 store + column statistics
 * (4, dgx_gemm_lds_bf16 only: as 2 but C is stored bf16)
 * (partials[dgx_gemm_stats_rows(M)][2][N] = per 128-row block sum, sum of
 * squares; feeds dgx_bn_finalize_f32), 3 split-K slabs: C is a dense
 * [splits][M][N] workspace (ldc ignored), summed by dgx_slab_reduce_f32.
 * Supported layouts: (fp32 KC, fp32 KC) epi 0/2; (fp32|bf16 KC, fp32 IC)
 * epi 0/1; (fp32|bf16 IC, fp32 IC) epi 3. Others: DGX_EUNSUPPORTED. */
int dgx_gemm_stats_rows(int M);
int dgx_gemm_splits(int M, int N, int K);
int dgx_gemm_bf16(const void* A, int a_bf16, int a_ic, int64_t lda,
                  const void* B, int b_bf16, int b_ic, int64_t ldb,
                  int M, int N, int K, int epi, int splits,
                  float* C, int64_t ldc, float* partials, void* stream);
/* fp32 MFMA GEMM of the parity mode (v_mfma_f32_16x16x4_f32, exact products,
 * fp32 accumulation): the same C[i][j] = sum_k opA(i,k) opB(j,k) contract as
 * dgx_gemm_bf16 with fp32 operands read in place (a_ic / b_ic: i- / j-
 * contiguous), epi 0 store, 1 accumulate (C = addend + .. when addend is
 * given, else C += ..), 3 split-K slabs (C = splits x M x N, summed by
 * dgx_slab_reduce_f32). Replaces the fp32 Conv(1x1) GEMMs of reference
 * models/dgcnn.py:54-78 and models/layers.py:17-24 and their dgrad / wgrad. */
int dgx_gemm_f32(const float* A, int a_ic, int lda, const float* B, int b_ic, int ldb, int M, int N, int K, int epi,
                 int splits, float* C, int64_t ldc, const float* addend, int64_t ldd, void* stream);
int dgx_gemm_f32_splits(int M, int N, int K);
/* Exact fp32 GEMM for a short reduction: C (M x N, row stride ldc) = X W^T,
 * X (M x K, row stride ldx), W (N x K) dense; each output an fmaf chain over
 * k = 0..K-1. K <= 16, N % 4 == 0, 16-byte aligned C rows. The layer-1
 * per-point GEMM on raw xyz (dgcnn.py:55, layers.py:17: K = 3), kept exact in
 * every precision mode. */
int dgx_gemm_smallk_f32(const float* X, int64_t ldx, const float* W, int M, int N, int K,
                        float* C, int64_t ldc, void* stream);
/* dgx_gemm_smallk_f32 with the weight given as the reference's conv weight
 * (Co, 2K) = [W1 | W2] (models/dgcnn.py:55): C (M, 2Co) = X [W1; W2]^T, the
 * EdgeConv PQ of the 3-channel block without a reshuffled weight copy. */
int dgx_gemm_smallk_split_f32(const float* X, int64_t ldx, const float* Wref, int M, int Co,
                              int K, float* C, int64_t ldc, void* stream);
/* out[orow][ocol] = sum_s slab[s][r][c] (fixed order: deterministic); rows
 * r >= split land at (r - split, c + cols): the [W1;W2] -> [W1 | W2] weight
 * un-stacking (reference conv weight layout (Co, 2C, 1, 1)). */
int dgx_slab_reduce_f32(const float* slab, int S, int rows, int cols, int split,
                        float* out, int64_t ldo, void* stream);
/* dgx_slab_reduce_f32 for n <= 8 independent slabs in one launch (job j:
 * slab[j], S[j], rows[j], cols[j], split[j] -> out[j] with row stride ldo[j];
 * host arrays of length n): the weight gradients of one backward pass reduced
 * together at its end, each element summed in dgx_slab_reduce_f32's order. */
int dgx_slab_reduce_multi_f32(int n, const float* const* slab, const int* S, const int* rows, const int* cols,
                              const int* split, float* const* out, const int64_t* ldo, void* stream);
/* The same GEMMs with bf16 operands in HBM, staged by LDS-DMA
 * (global_load_lds) into swizzled LDS images. tn = 0: C = A B^T with A (M,K)
 * and B (N,K) k-contiguous, K % 64 == 0, epi 0/1/2. tn = 1: C = A^T B with A
 * (K,M), B (K,N) row-major (the weight gradients), M, N multiples of 8, epi 3
 * (split-K slabs). lda, ldb multiples of 8, 16-byte aligned bases; anything
 * else returns DGX_EUNSUPPORTED (callers then use dgx_gemm_bf16). With epi 1
 * and addend != NULL: C = addend (row stride ldd) + A B^T (C need not hold data).
 * a_k (tn = 0): A's k extent; 0 or K for a plain GEMM, K/2 for a split weight
 * B = [W_hi | W_lo] (N x K, W_lo = bf16(W - W_hi)): C = A W_hi^T + A W_lo^T,
 * i.e. the weight operand carries 16 significant bits (a_k % 64 == 0). */
/* EdgeConv backward, bf16 mode: block l's input-gradient GEMM dY_{l-1} =
 * addend + A W^T (A = dPQ_l (M x K) bf16, W = [W1;W2]^T (N x K) bf16, addend =
 * the incoming gradient of the concat slice, ld ldd) whose epilogue applies
 * block l-1's LeakyReLU' instead of storing dY: dz = dY * LReLU'(scale*ysel +
 * shift) written as packed dz|slot words (dgx_edge_bwd_dz_packed_f32's format,
 * arg = block l-1's selected slots) with per-tile column partials (sum dz,
 * sum dz*yhat), nrows = dgx_gemm_edge_dz_rows(M, N) — no dY round trip and no
 * separate dz pass. N <= 128, N % 8 == 0, K % 64 == 0. */
int dgx_gemm_edge_dz_rows(int M, int N);
int dgx_gemm_edge_dz_bf16(const void* A, int64_t lda, const void* W, int64_t ldw, int M, int N, int K,
                          const float* addend, int64_t ldd, const float* ysel, const uint8_t* arg,
                          const float* scale, const float* shift, const float* mean,
                          const float* invstd, float slope, float* dz, float* partials, int nrows,
                          void* stream);
int dgx_gemm_lds_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, int tn,
                      int M, int N, int K, int a_k, int epi, int splits, float* C,
                      int64_t ldc, float* partials, const float* addend,
                      int64_t ldd, void* stream);
/* fp32 (rows x cols, row stride lds) -> two bf16 planes (row stride ldo): hi =
 * bf16(x) (nullable: skip), lo = bf16(x - hi) — x with 16 significant bits as
 * hi + lo. The operands of the fp32 parity mode's 3-pass GEMMs (hi.W_hi +
 * hi.W_lo + lo.W_hi on the bf16 MFMA, ~2^-16 relative per product) that stand
 * in for the f32-MFMA conv5 GEMMs (dgcnn.py:74-78, 100-102). cols, lds, ldo
 * multiples of 4, 16-byte aligned src. */
int dgx_split_bf16(const float* src, int64_t lds, int64_t rows, int cols, void* hi, void* lo, int64_t ldo,
                   void* stream);
/* bf16 weight operands per step: nt = [rows][C], tn = its transpose. stacked
 * != 0: W is an EdgeConv weight (Co, 2C) (dgcnn.py:55) and rows = 2Co are
 * [W1; W2]; else W is (Co, C) (conv5, dgcnn.py:74). */
int dgx_weight_prep_bf16(const float* W, int Co, int C, int stacked, void* nt,
                         void* tn, void* stream);
/* dgx_weight_prep_bf16 for n <= 8 weights in one launch (host arrays of
 * length n: one job per EdgeConv block of a forward). stacked[j] bit 0: an
 * EdgeConv weight as above; bit 1: nt is the split form [rows][2C] = [hi | lo]
 * (lo = bf16(w - hi)) for dgx_gemm_lds_bf16's a_k = C; tn stays hi only
 * unless bit 2 (value 4) is set: then tn is [C][2 rows] = [hi^T | lo^T]. */
int dgx_weight_prep_multi_bf16(int n, const float* const* W, const int* Co, const int* C, const int* stacked,
                               void* const* nt, void* const* tn, void* stream);
/* fp32 stacked weights [W1; W2] (2 Co x C, row-major) of n <= 8 EdgeConv
 * weights W (Co x 2C, the reference's [W1 | W2]) in one launch: the fp32
 * parity mode's GEMM operands for all blocks of a forward / backward. */
int dgx_weight_stack_multi_f32(int n, const float* const* W, const int* Co, const int* C, float* const* out,
                               void* stream);

/* ---- a6: PositionEmbedding's per-edge MLP, replaces
 *   get_graph_feature -> conv1 (Conv2d 2C->C1, BN, LeakyReLU, per edge)
 *   -> conv2 (Conv2d C1->C2, BN, LeakyReLU) -> max(dim=-1)
 *                                             (models/layers.py:45-52, 17-22)
 * Edge rows e = i*k + s (i = global point, s = slot), E = B*N*k. conv1 is
 * decomposed as in a3 (PQ = X [W1;W2]^T, y_e = P_j + Q_i, BN1 statistics from
 * dgx_edge_fwd_gather_f32); conv2 is the caller's GEMM Z2 = H1 W^T over the E
 * edge rows (BN2 statistics from its epilogue / dgx_colstats_f32).
 *   dgx_edge_mlp_h1: H1 (E x C1) = LeakyReLU(a1 (P_j + Q_i) + b1), fp32 or
 *     bf16 (out_bf16 != 0: the GEMM operand).
 *   dgx_edge_mlp_max: ysel (M x C2) = max_s Z2 (min where a2 < 0), arg = the
 *     first extremal slot; then dgx_bn_lrelu_apply_f32 gives the output.
 * Backward: dgx_edge_bwd_dz_f32 + dgx_bn_bwd_finalize_f32 on (ysel, arg) ->
 *   dgx_edge_mlp_dz: dZ2 (E x C2) = a2 dz [s == slot] + c0 + c1 Z2 (dense BN2
 *     backward; Z2/dZ2 both fp32 or both bf16);
 *   caller's GEMMs dH1 = dZ2 W2, dW2 = dZ2^T H1;
 *   dgx_edge_mlp_h1_bwd: dH1 *= LeakyReLU'(z1) in place + partials (sum g,
 *     sum g*yhat) [dgx_edge_mlp_h1_bwd_rows][2][C1] -> dgx_bn_bwd_finalize_f32;
 *   dgx_edge_mlp_scatter: dPQ (M x 2C1) fp32, dQ_i = sum over i's edges and
 *     dP_j = sum over j's in-edges (dgx_graph_reverse) of a1 g + c0 + c1 y
 *     (sumP = sum_k P_j per point, as dgx_edge_fwd_gather_f32 writes it).
 * Edge-MLP kernels need C1 % 8 == 0 (and C1/4 dividing 256), C2 % 8 == 0 and
 * 16-byte aligned rows. */
int dgx_edge_mlp_h1_f32(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int C1,
                        const float* scale, const float* shift, float slope, void* H1, int out_bf16, void* stream);
int dgx_edge_mlp_max_f32(const void* Z, int z_bf16, int B, int N, int k, int C2, const float* scale, float* ysel,
                         uint8_t* arg, void* stream);
int dgx_edge_mlp_dz_f32(const float* dz, const uint8_t* arg, const void* Z, int bf16, int B, int N, int k, int C2,
                        const float* scale, const float* c0, const float* c1, void* dZ, void* stream);
int dgx_edge_mlp_h1_bwd_rows(int B, int N, int k, int C1);
int dgx_edge_mlp_h1_bwd_f32(float* dH, const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int C1,
                            const float* scale, const float* shift, const float* mean, const float* invstd,
                            float slope, float* partials, int nrows, void* stream);
/* Fused bf16 forward of the edge MLP (h1, conv2, max over k and BN2 statistics
 * in one kernel; z2 is never stored): W2d = bf16(dir2[c] * W2[c][:]) with
 * dir2 = sign(gamma2) (+-1), so the kernel maximises dir2*z2; ysel/arg as the
 * unfused max-over-k entry writes them (ysel in z2's sign), partials [nrows][2][C2] (sum z2,
 * sum z2^2) with nrows = dgx_edge_mlp_fused_rows(B, N) for BN2; h1 (E x C1
 * bf16) is written when H1 != NULL (the backward's operand). C1 = 64,
 * C2 in {64, 128}, k <= 64, 16-byte aligned operands. */
int dgx_edge_mlp_fused_rows(int B, int N);
/* Its backward partner: dZ2 (E x C2 bf16) = c1 (H1 W2^T) + c0 + [arg == s] a2 dz
 * for edge rows e = p*k + s, z2 recomputed on the MFMA from h1 (E x C1 bf16,
 * K = C1 % 64 == 0) and W2 (C2 x C1 bf16) with the BN2 backward in the
 * epilogue; consts = [c0 | c1 | a2] (3 x C2 fp32), dz / arg (E/k x C2). */
/* ... and the conv2 input gradient with the LReLU + BN1 backward in its
 * epilogue: dH1 = dZ2 W2 (dZ2 E x C2 bf16, W2t = W2^T as C1 x C2 bf16) never
 * leaves the tile; g = dH1 * LReLU'(a1 (P_j + Q_i) + b1) is stored bf16 (E x
 * C1) and the BN1-backward column partials [nrows][2][C1] (sum g, sum g*yhat,
 * nrows = dgx_gemm_h1bwd_rows(E)) feed dgx_bn_bwd_finalize. C1 = 64. The
 * scatter then reads g bf16 (dgx_edge_mlp_scatter_f32, g_bf16 = 1). */
int dgx_gemm_h1bwd_rows(int M);
int dgx_gemm_h1bwd_bf16(const void* dZ2, const void* W2t, int M, int N, int K, const float* PQ, int ldpq,
                        const int32_t* idx, int Np, int k, const float* scale, const float* shift, const float* mean,
                        const float* invstd, float slope, void* g, float* partials, int nrows, void* stream);
int dgx_gemm_dz2_bf16(const void* H1, const void* W2, int M, int N, int K, const float* dz, const uint8_t* arg,
                      const float* consts, int k, void* dZ2, void* stream);
int dgx_edge_mlp_fused_fwd_bf16(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int C1, int C2,
                                const float* scale1, const float* shift1, float slope1, const void* W2d,
                                const float* dir2, float* ysel, uint8_t* arg, float* partials, int nrows, void* H1,
                                void* stream);
/* bf16 mode, backward of the same stage (autograd of layers.py:48-52): with
 * dz = dgx_edge_bwd_dz_f32 of the max's output gradient and consts2 =
 * [c0 | c1 | a2] (BN2 backward, 3*C2 floats), per edge row e = (i, s):
 *   z2 = W2 h1_e (h1 rebuilt from P_j, Q_i as the forward did), dZ2 = c1 z2 + c0
 *   + [arg_i == s] a2 dz_i (bf16), dH1 = W2^T dZ2, g = dH1 LReLU'(z1) -> gE
 *   (E x C1 bf16), BN1-backward partials part1 (nrows x 2 x C1) and dW2 =
 *   sum_e dZ2_e h1_e^T per block in dw2slab (nrows x C2 x C1; reduce with
 *   dgx_slab_reduce_f32). z2, dZ2, dH1 and h1 never reach HBM. W2: bf16
 *   (C2 x C1). C1 = 64, C2 = 128, k <= 64; nrows = dgx_edge_mlp_fused_bwd_rows. */
int dgx_edge_mlp_fused_bwd_rows(int B, int N);
int dgx_edge_mlp_fused_bwd_bf16(const float* PQ, int ldpq, const int32_t* idx, int B, int N, int k, int C1, int C2,
                                const float* scale1, const float* shift1, const float* mean1, const float* invstd1,
                                float slope1, const void* W2, const float* dz, const uint8_t* arg,
                                const float* consts2, void* gE, float* part1, float* dw2slab, int nrows,
                                void* stream);
int dgx_edge_mlp_scatter_f32(const void* g, int g_bf16, const float* PQ, int ldpq, const float* sumP,
                             const int32_t* rowptr, const int32_t* edges, int B, int N, int k, int C1,
                             const float* scale, const float* c0, const float* c1, float* dPQ, void* stream);

/* ---- f1: compute_hog_1x1 on the device, replaces models/model_partseg.py:26-92
 * after the kNN call (the D2H copy, np.linalg.svd on B*N k x 3 matrices, the H2D
 * copy and the histogram votes). x: contiguous (B, 3, N) fp32; idx: (B, N, k)
 * int64 LOCAL ids (the engine kNN's output, as knn() returns it). Reproduces the
 * reference's local-id gather: neighbourhoods are rows of the
 * (B*N, 3) view of x, so only cloud 0's N SVDs are used; axis (N x 4 fp32
 * scratch) receives (v0 v1 v2 sqrt(sigma0)) of the dominant right singular
 * vector (LAPACK dgesdd's sign, csrc/svd3.h); out: (B, N, 18) = (B, N, 9 bins,
 * 2 angles) L2-normalised histograms. 5 <= k <= 64 (DGX_EUNSUPPORTED else). */
int dgx_hog_1x1_f32(const float* x, const int64_t* idx, int B, int N, int k, float* axis, float* out,
                    void* stream);
/* The same, with the arithmetic of the device each reference stage runs on for
 * the caller's configuration (`sem`, a mask): DGX_HOG_MEAN_DEVICE — x is a GPU
 * tensor, so the neighbourhood mean (model_partseg.py:32) is torch's GPU mean
 * (reduce-kernel order, times float(outputs)/numel); DGX_HOG_VOTES_DEVICE — v and
 * s were moved to the GPU (model_partseg.py:42-47: LOCAL_RANK set or use_cpu
 * False), so the angle / vote / bin-sum / normalize ops (:58-90) are torch's
 * GPU kernels (ocml acosf / atanf, scalar division as a reciprocal multiply,
 * reduce-kernel sum and norm order). sem 0 = dgx_hog_1x1_f32 (every stage as
 * torch's CPU kernels, the reference's use_cpu run on a host cloud). */
#define DGX_HOG_MEAN_DEVICE 1
#define DGX_HOG_VOTES_DEVICE 2
int dgx_hog_1x1_sem_f32(const float* x, const int64_t* idx, int B, int N, int k, int sem, float* axis, float* out,
                        void* stream);

/* ---- f2: attention in Net (nn.Transformer / nn.MultiheadAttention), replaces the
 * scaled_dot_product_attention call inside torch.nn.functional.
 * multi_head_attention_forward for every attention of models/model_partseg.py:
 * 167-171 (nn.Transformer, 1 encoder + 1 decoder layer: 3 attentions per call,
 * called twice at 187-188) and 190 (nn.MultiheadAttention). O = dropout(softmax(
 * scale Q K^T)) V per (b, h) without an Nq x Nk buffer. dtype 0 = fp16, 1 = bf16
 * operands (fp32 accumulation and softmax), 2 = fp32 operands given as two bf16
 * planes hi = bf16(x), lo = bf16(x - hi) at +sP elements (three MFMAs per
 * product; O is then fp32). Element (b, n, h, d) of an operand plane at
 * b*sB + n*sN + h*sH + d (strides in elements, 16-byte aligned rows: the
 * (B, N, E) in-projection output viewed as (B, N, H, D)). D in {64, 128}.
 * lse: (B*H*Nq) fp32 log2-sum-exp of the scaled scores, kept for the backward.
 * Dropout (0 <= p < 1) on the attention weights from a counter-based hash of
 * (row, key, seed), regenerated by the backward; kept weights scaled 1/(1-p).
 * seed_dev: when non-NULL, the seed is read from this device word at run time
 * instead of `seed` (a device-generator draw: HIP-graph replays see new seeds). */
int dgx_attn_fwd(int dtype, const void* q, int64_t qsP, int64_t qsB, int64_t qsN, int64_t qsH, const void* k,
                 int64_t ksP, int64_t ksB, int64_t ksN, int64_t ksH, const void* v, int64_t vsP, int64_t vsB,
                 int64_t vsN, int64_t vsH, void* o, int64_t osB, int64_t osN, int64_t osH, float* lse, int B, int H,
                 int Nq, int Nk, int D, float scale, float dropout_p, uint64_t seed, const uint64_t* seed_dev,
                 void* stream);
/* Gradients of dgx_attn_fwd (same operands, seed and p). dout: dO in the
 * operand format (planes at +gsP for dtype 2) with O's (sB, sN, sH); dout32:
 * dO in fp32 (dtype 2 only, for delta = rowsum(dO . O)); dq/dk/dv fp32 with
 * their own strides; delta: (B*H*Nq) fp32 scratch. No atomics (bitwise
 * reproducible). */
int dgx_attn_bwd(int dtype, const void* q, int64_t qsP, int64_t qsB, int64_t qsN, int64_t qsH, const void* k,
                 int64_t ksP, int64_t ksB, int64_t ksN, int64_t ksH, const void* v, int64_t vsP, int64_t vsB,
                 int64_t vsN, int64_t vsH, const void* o, const void* dout, int64_t gsP, int64_t osB, int64_t osN,
                 int64_t osH, const float* dout32, const float* lse, float* delta, int B, int H, int Nq, int Nk, int D,
                 float scale, float dropout_p, uint64_t seed, const uint64_t* seed_dev, float* dq, int64_t dqsB,
                 int64_t dqsN, int64_t dqsH,
                 float* dk, int64_t dksB, int64_t dksN, int64_t dksH, float* dv, int64_t dvsB, int64_t dvsN,
                 int64_t dvsH, void* stream);
/* The keep mask (rows = B*H*Nq, Nk) the kernels draw for (p, seed), u8 0/1. */
int dgx_attn_dropout_mask(int64_t rows, int Nk, float dropout_p, uint64_t seed, uint8_t* out, void* stream);


/* ---- training-step utility: torch.optim.SGD's update (lr, momentum,
 * dampening, weight_decay, nesterov, maximize) over n <= 48 fp32 tensors in
 * one launch (torch's fused form runs ~22 workgroups for a DGCNN's ~0.6 M
 * parameters); first != 0 sets the momentum buffers to the step's gradient
 * (torch's first step). torch/optim/sgd.py's arithmetic in fp32 (last-bit
 * differences from FMA contraction possible). */
int dgx_sgd_step_f32(int n, float* const* params, const float* const* grads, float* const* momentum_bufs,
                     const int64_t* numels, float lr, float weight_decay, float momentum, float dampening,
                     int nesterov, int maximize, int first, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DGX_H */
