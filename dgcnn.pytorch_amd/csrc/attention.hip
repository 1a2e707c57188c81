// Fused multi-head attention for Net's nn.Transformer / nn.MultiheadAttention
// (reference models/model_partseg.py:167-171, 187-191):
// softmax(Q Kᵀ / sqrt(D)) with dropout on the attention weights, times V, and
// its backward, without materialising the (B, H, Nq, Nk) score matrix.
//
// Operands are 16-bit (fp16 or bf16: v_mfma_f32_16x16x32_{f16,bf16}), every sum
// and the softmax are fp32. The fp32 mode splits each fp32 operand into two
// bf16 planes, x = hi + lo (hi = bf16(x), lo = bf16(x - hi)), and every product
// into hi.hi + hi.lo + lo.hi (three MFMAs; the dropped lo.lo term is ~2^-16
// relative), P and dS likewise: ~16-bit-mantissa products for fp32 parity. Layout: element (b, n, h, d) of Q/K/V/O/dO at
// b*sB + n*sN + h*sH + d (d contiguous) — the (B, N, E) projections of
// nn.MultiheadAttention (batch_first) viewed as (B, N, H, D) without a copy.
//
// Forward (attn_fwd_kernel): a block = 4 waves x 32 queries of one (b, h); the
// block streams 64-key K/V tiles through LDS (register-staged: the next tile's
// global loads are in flight during the current tile's math). Scores are
// computed transposed, Sᵀ = K Qᵀ, so a lane holds one query's scores (the
// row max/sum is in-lane plus two cross-lane steps) and the Sᵀ accumulators
// are directly the B operand of Oᵀ = Vᵀ Pᵀ; Vᵀ fragments come from LDS through
// ds_read_b64_tr_b16 (gfx950 transposing LDS read). Online softmax in the
// exp2 domain; the log-sum-exp of every row is kept for the backward.
//
// Backward: delta = rowsum(dO ∘ O) (attn_delta_kernel); dQ by a query-owned
// pass (attn_bwd_dq_kernel: Sᵀ, dPᵀ = V dOᵀ, dSᵀ, dQᵀ += Kᵀ dSᵀ) and dK, dV by
// a key-owned pass (attn_bwd_dkv_kernel: S = Q Kᵀ, dP = dO Vᵀ, dVᵀ += dOᵀ P,
// dKᵀ += Qᵀ dS). No atomics: each output element is summed by one wave in a
// fixed order, so gradients are bitwise reproducible.
//
// Dropout: element (row = (b*H + h)*Nq + q, key) is kept iff
// hash(row, key, seed) >= p * 2^32; kept weights are scaled by 1 / (1 - p).
// The same function regenerates the mask in the backward and in
// dgx_attn_dropout_mask (tests). It is not torch's Philox stream: the
// distribution matches nn.Dropout, the individual draws do not.
#include "common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T>
struct Mma;
template <>
struct Mma<_Float16> {
    static __device__ __forceinline__ f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                      0, 0, 0);
    }
    static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
        const _Float16 a = (_Float16)lo, b = (_Float16)hi;
        return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
    }
};
template <>
struct Mma<__bf16> {
    static __device__ __forceinline__ f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
    }
    static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
        const __bf16 a = (__bf16)lo, b = (__bf16)hi;
        return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
    }
};

constexpr int AT_THREADS = 256;
constexpr int AT_QW = 32;        // queries per wave (two 16-row MFMA tiles), forward and dQ pass
constexpr int AT_QB = 4 * AT_QW; // queries per block
constexpr int AT_KT = 64;        // keys per streamed K/V tile
constexpr int AT_KW = 16;        // keys per wave, dK/dV pass
constexpr int AT_KB = 4 * AT_KW; // keys per block, dK/dV pass
constexpr int AT_QT = 64;        // queries per streamed Q/dO tile, dK/dV pass
constexpr float AT_DS_SCALE = 256.f;  // dS enters its MFMA scaled by 2^8 (no fp16 subnormals), undone exactly

// LDS row stride in 32-bit words for a D-wide 16-bit tile: D/2 + 8 (== 8 mod 64
// for D = 128, 40 for D = 64) puts the 8 rows x 4 column chunks of a 32-lane
// half of a transposed read on distinct banks; the 16-row b128 reads are 2-way.
template <int D>
constexpr int at_rsw() { return D / 2 + 8; }

__device__ __forceinline__ uint32_t at_hash(uint32_t row, uint32_t col, uint32_t s0, uint32_t s1) {
    uint32_t h = (row * 0x9E3779B1u + s0) ^ (col * 0x85EBCA77u) ^ s1;
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}

__device__ __forceinline__ bool at_keep(uint32_t row, uint32_t col, uint32_t p32, uint32_t s0, uint32_t s1) {
    return at_hash(row, col, s0, s1) >= p32;
}

// A row-major 16-bit tile [rows][D] in LDS (row stride RSW words).
// Row read: lane (row r, k chunk) -> 8 consecutive elements (b128).
template <int RSW>
__device__ __forceinline__ s16x8 lds_row8(const uint32_t* t, int row, int col) {
    return *reinterpret_cast<const s16x8*>(t + row * RSW + col / 2);
}

// Transposed read (ds_read_b64_tr_b16): the 16x16x32 operand whose row index is
// a COLUMN of the tile and whose k index runs over tile rows r0 + {4g..4g+3,
// 16+4g..16+4g+3}: lane (g, i) gets t[r0 + 4g + q][c0 + i] (q = 0..3) and
// t[r0 + 16 + 4g + q][c0 + i]. Lane 4q+p of a 16-lane group supplies the
// address of row q, columns 4p..4p+3 of its 4-row block.
template <int RSW>
__device__ __forceinline__ s16x8 lds_tr8(const uint32_t* t, int r0, int c0, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const uint32_t* a0 = t + (r0 + 4 * g + q) * RSW + (c0 + 4 * p) / 2;
    const uint32_t* a1 = a0 + 16 * RSW;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// The B operand of a product summing over the 32 rows {4g+r, 16+4g+r} of two
// accumulator tiles (lane = column): elements 0..3 from tile a, 4..7 from b.
// NP = 2 (split fp32): plane 0 = bf16(x), plane 1 = bf16(x - plane 0).
template <typename T, int NP>
__device__ __forceinline__ void pack_acc(const f32x4& a, const f32x4& b, s16x8 (&out)[NP]) {
    float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = Mma<T>::pack(x[2 * i], x[2 * i + 1]);
    out[0] = __builtin_bit_cast(s16x8, make_uint4(w[0], w[1], w[2], w[3]));
    if constexpr (NP == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float h0 = __uint_as_float(w[i] << 16), h1 = __uint_as_float(w[i] & 0xffff0000u);
            w[i] = Mma<T>::pack(x[2 * i] - h0, x[2 * i + 1] - h1);
        }
        out[1] = __builtin_bit_cast(s16x8, make_uint4(w[0], w[1], w[2], w[3]));
    }
}

// c += a b over the planes: hi.hi (+ hi.lo + lo.hi when split; lo.lo ~ 2^-16 is dropped)
template <typename T, int NP>
__device__ __forceinline__ f32x4 mmp(const s16x8 (&a)[NP], const s16x8 (&b)[NP], f32x4 c) {
    if constexpr (NP == 2) {
        c = Mma<T>::run(a[0], b[1], c);
        c = Mma<T>::run(a[1], b[0], c);
    }
    return Mma<T>::run(a[0], b[0], c);
}

// Register-staged copy of a [64][D] 16-bit tile (rows from `row0`, row stride
// sN elements) into LDS: issue() loads into registers, commit() writes them.
template <int D>
struct TileStage {
    static constexpr int CH = D / 8;                   // 16-byte chunks per row
    static constexpr int NLD = 64 * CH / AT_THREADS;   // chunks per thread
    uint4 r[NLD];
    __device__ __forceinline__ void issue(const uint16_t* base, int64_t sN, int row0, int nrows) {
#pragma unroll
        for (int u = 0; u < NLD; ++u) {
            const int e = threadIdx.x + AT_THREADS * u;
            const int row = e / CH, ch = e - row * CH;
            r[u] = row0 + row < nrows ? *reinterpret_cast<const uint4*>(base + (int64_t)(row0 + row) * sN + 8 * ch)
                                      : make_uint4(0u, 0u, 0u, 0u);
        }
    }
    __device__ __forceinline__ void commit(uint32_t* t) const {
        constexpr int RSW = at_rsw<D>();
#pragma unroll
        for (int u = 0; u < NLD; ++u) {
            const int e = threadIdx.x + AT_THREADS * u;
            const int row = e / CH, ch = e - row * CH;
            *reinterpret_cast<uint4*>(t + row * RSW + 4 * ch) = r[u];
        }
    }
};

__device__ __forceinline__ float wmax16(float v) {  // max over lanes l, l^16, l^32, l^48
    v = fmaxf(v, __shfl_xor(v, 16));
    return fmaxf(v, __shfl_xor(v, 32));
}
__device__ __forceinline__ float wsum16(float v) {
    v += __shfl_xor(v, 16);
    return v + __shfl_xor(v, 32);
}

// One operand: planes at p, p + sP; element (b, n, h, d) at b*sB + n*sN + h*sH + d.
struct AtOp {
    const uint16_t* p;
    int64_t sP, sB, sN, sH;
    __device__ __forceinline__ const uint16_t* at(int pl, int b, int h) const { return p + pl * sP + b * sB + h * sH; }
};

struct AtArgs {
    AtOp q, k, v, dout;                 // dout shares O's (sB, sN, sH)
    const void* o;                      // forward output as stored (16-bit, or fp32 when split)
    const float* dout32;                // split mode: dO in fp32 (for delta)
    int64_t osB, osN, osH;
    float *lse, *delta;
    int H, Nq, Nk;
    float scale_log2;   // log2(e) * scale
    float scale;        // the softmax scale
    uint32_t p32;       // dropout threshold (0: no dropout)
    float rdrop;        // 1 / (1 - p)
    uint32_t s0, s1;    // dropout seed
    const uint64_t* seedp;  // when set: the seed is read here (device-drawn, graph-replay safe)
};

// the dropout seed of this launch: from device memory when given (a seed drawn
// by the device generator: every HIP-graph replay reads the new draw)
__device__ __forceinline__ void at_seed(const AtArgs& a, uint32_t& s0, uint32_t& s1) {
    if (a.seedp) {
        const uint64_t v = *a.seedp;
        s0 = (uint32_t)v, s1 = (uint32_t)(v >> 32);
    } else {
        s0 = a.s0, s1 = a.s1;
    }
}

template <int D, int NP>
constexpr int at_lds_bytes_qk() { return 2 * NP * 64 * at_rsw<D>() * 4; }

// ---------------------------------------------------------------- forward --
template <typename T, int D, bool DROP, int NP>
__global__ __launch_bounds__(AT_THREADS, NP == 2 ? 1 : 2) void attn_fwd_kernel(AtArgs a, void* __restrict__ out) {
    uint32_t sd0, sd1;
    at_seed(a, sd0, sd1);
    constexpr int RSW = at_rsw<D>();
    constexpr int KS = D / 32, DB = D / 16, TW = 64 * RSW;
    extern __shared__ __attribute__((aligned(16))) uint32_t at_lds[];
    uint32_t* kl = at_lds;             // [NP][64][RSW]
    uint32_t* vl = at_lds + NP * TW;   // [NP][64][RSW]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, c = lane & 15;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
    const int q0 = blockIdx.x * AT_QB + wave * AT_QW;

    s16x8 qf[2][KS][NP];  // B operand of Sᵀ = K Qᵀ: lane (g, c) holds Q[q0 + 16qt + c][32ks + 8g .. +7]
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
        const int q = min(q0 + 16 * qt + c, a.Nq - 1);
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) {
            const uint16_t* qp = a.q.at(pl, b, h) + (int64_t)q * a.q.sN;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) qf[qt][ks][pl] = *reinterpret_cast<const s16x8*>(qp + 32 * ks + 8 * g);
        }
    }
    f32x4 o[2][DB];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int db = 0; db < DB; ++db) o[qt][db] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
    const uint32_t row0 = (uint32_t)bh * (uint32_t)a.Nq + (uint32_t)q0;

    TileStage<D> ks_[NP], vs_[NP];
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
        ks_[pl].issue(a.k.at(pl, b, h), a.k.sN, 0, a.Nk);
        vs_[pl].issue(a.v.at(pl, b, h), a.v.sN, 0, a.Nk);
    }
    for (int kv0 = 0; kv0 < a.Nk; kv0 += AT_KT) {
        __syncthreads();  // the previous tile's LDS reads are done
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) {
            ks_[pl].commit(kl + pl * TW);
            vs_[pl].commit(vl + pl * TW);
        }
        __syncthreads();
        if (kv0 + AT_KT < a.Nk) {  // next tile in flight during this one's math
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) {
                ks_[pl].issue(a.k.at(pl, b, h), a.k.sN, kv0 + AT_KT, a.Nk);
                vs_[pl].issue(a.v.at(pl, b, h), a.v.sN, kv0 + AT_KT, a.Nk);
            }
        }
        f32x4 s[2][4];
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) s[qt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                s16x8 kf[NP];
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) kf[pl] = lds_row8<RSW>(kl + pl * TW, 16 * kt + c, 32 * ks + 8 * g);
#pragma unroll
                for (int qt = 0; qt < 2; ++qt) s[qt][kt] = mmp<T, NP>(kf, qf[qt][ks], s[qt][kt]);
            }
        // online softmax, lane = query 16qt + c, registers = keys 16kt + 4g + r
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
            float mx = m[qt];
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = kv0 + 16 * kt + 4 * g + r;
                    const float v = key < a.Nk ? s[qt][kt][r] * a.scale_log2 : -INFINITY;
                    s[qt][kt][r] = v;
                    mx = fmaxf(mx, v);
                }
            mx = wmax16(mx);
            const float alpha = __builtin_amdgcn_exp2f(m[qt] - mx);
            m[qt] = mx;
            float rs = 0.f;
            const uint32_t row = row0 + 16 * qt + c;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float p = __builtin_amdgcn_exp2f(s[qt][kt][r] - mx);
                    rs += p;
                    if constexpr (DROP) {
                        const int key = kv0 + 16 * kt + 4 * g + r;
                        s[qt][kt][r] = at_keep(row, (uint32_t)key, a.p32, sd0, sd1) ? p : 0.f;
                    } else {
                        s[qt][kt][r] = p;
                    }
                }
            l[qt] = l[qt] * alpha + wsum16(rs);
#pragma unroll
            for (int db = 0; db < DB; ++db) o[qt][db] *= alpha;
        }
        // Oᵀ += Vᵀ Pᵀ over two 32-key steps
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            s16x8 pf0[NP], pf1[NP];
            pack_acc<T, NP>(s[0][2 * st], s[0][2 * st + 1], pf0);
            pack_acc<T, NP>(s[1][2 * st], s[1][2 * st + 1], pf1);
#pragma unroll
            for (int db = 0; db < DB; ++db) {
                s16x8 vf[NP];
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) vf[pl] = lds_tr8<RSW>(vl + pl * TW, 32 * st, 16 * db, lane);
                o[0][db] = mmp<T, NP>(vf, pf0, o[0][db]);
                o[1][db] = mmp<T, NP>(vf, pf1, o[1][db]);
            }
        }
    }
    // O[q][16db + 4g + r] = o / l (x 1/(1-p)); lse in the exp2 domain of the scaled scores
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
        const int q = q0 + 16 * qt + c;
        if (q < a.Nq) {
            const float inv = (DROP ? a.rdrop : 1.f) / l[qt];
            const int64_t off = b * a.osB + h * a.osH + (int64_t)q * a.osN;
#pragma unroll
            for (int db = 0; db < DB; ++db) {
                if constexpr (NP == 2) {
                    *reinterpret_cast<float4*>(static_cast<float*>(out) + off + 16 * db + 4 * g) =
                        make_float4(o[qt][db][0] * inv, o[qt][db][1] * inv, o[qt][db][2] * inv, o[qt][db][3] * inv);
                } else {
                    const uint32_t w0 = Mma<T>::pack(o[qt][db][0] * inv, o[qt][db][1] * inv);
                    const uint32_t w1 = Mma<T>::pack(o[qt][db][2] * inv, o[qt][db][3] * inv);
                    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(out) + off + 16 * db + 4 * g) =
                        make_uint2(w0, w1);
                }
            }
            if (g == 0) a.lse[(int64_t)bh * a.Nq + q] = m[qt] + __log2f(l[qt]);
        }
    }
}

// delta[row] = sum_d dO . O (fp32), one 16-lane group per row, 16-byte loads;
// fmt 0 f16, 1 bf16, 2 f32.
__device__ __forceinline__ float h2f(uint32_t w, int hi, int fmt) {
    const uint16_t u = (uint16_t)(w >> (16 * hi));
    return fmt == 1 ? __uint_as_float((uint32_t)u << 16) : (float)__builtin_bit_cast(_Float16, u);
}

template <int D>
__global__ __launch_bounds__(256) void attn_delta_kernel(AtArgs a, int B, int fmt) {
    const int64_t rowg = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const int i = threadIdx.x & 15;
    const int64_t rows = (int64_t)B * a.H * a.Nq;
    float acc = 0.f;
    if (rowg < rows) {
        const int64_t bh = rowg / a.Nq, q = rowg - bh * a.Nq;
        const int b = (int)(bh / a.H), h = (int)(bh - (int64_t)b * a.H);
        const int64_t off = b * a.osB + h * a.osH + q * a.osN;
        if (fmt == 2) {  // fp32: 4 per load
            const float* op = static_cast<const float*>(a.o) + off;
            const float* gp = a.dout32 + off;
            for (int d = 4 * i; d < D; d += 64) {
                const float4 x = *reinterpret_cast<const float4*>(op + d);
                const float4 y = *reinterpret_cast<const float4*>(gp + d);
                acc = fmaf(x.x, y.x, fmaf(x.y, y.y, fmaf(x.z, y.z, fmaf(x.w, y.w, acc))));
            }
        } else {  // 16-bit: 8 per load
            const uint16_t* op = static_cast<const uint16_t*>(a.o) + off;
            const uint16_t* gp = a.dout.p + off;
            for (int d = 8 * i; d < D; d += 128) {
                const uint4 x = *reinterpret_cast<const uint4*>(op + d);
                const uint4 y = *reinterpret_cast<const uint4*>(gp + d);
                const uint32_t xw[4] = {x.x, x.y, x.z, x.w}, yw[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    acc = fmaf(h2f(xw[u], 0, fmt), h2f(yw[u], 0, fmt), fmaf(h2f(xw[u], 1, fmt), h2f(yw[u], 1, fmt), acc));
            }
        }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 16);
    if (rowg < rows && i == 0) a.delta[rowg] = acc;
}

// ------------------------------------------------------------- backward dQ --
template <typename T, int D, bool DROP, int NP>
__global__ __launch_bounds__(AT_THREADS, (D == 128 || NP == 2) ? 1 : 2) void attn_bwd_dq_kernel(
    AtArgs a, float* __restrict__ dq, int64_t dsB, int64_t dsN, int64_t dsH) {
    uint32_t sd0, sd1;
    at_seed(a, sd0, sd1);
    constexpr int RSW = at_rsw<D>();
    constexpr int KS = D / 32, DB = D / 16, TW = 64 * RSW;
    extern __shared__ __attribute__((aligned(16))) uint32_t at_lds[];
    uint32_t* kl = at_lds;
    uint32_t* vl = at_lds + NP * TW;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, c = lane & 15;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
    const int q0 = blockIdx.x * AT_QB + wave * AT_QW;

    s16x8 qf[2][KS][NP], gf[2][KS][NP];
    float lse[2], dl[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
        const int q = min(q0 + 16 * qt + c, a.Nq - 1);
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) {
            const uint16_t* qp = a.q.at(pl, b, h) + (int64_t)q * a.q.sN;
            const uint16_t* gp = a.dout.at(pl, b, h) + (int64_t)q * a.osN;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                qf[qt][ks][pl] = *reinterpret_cast<const s16x8*>(qp + 32 * ks + 8 * g);
                gf[qt][ks][pl] = *reinterpret_cast<const s16x8*>(gp + 32 * ks + 8 * g);
            }
        }
        lse[qt] = a.lse[(int64_t)bh * a.Nq + q];
        dl[qt] = a.delta[(int64_t)bh * a.Nq + q];
    }
    f32x4 acc[2][DB];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int db = 0; db < DB; ++db) acc[qt][db] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint32_t row0 = (uint32_t)bh * (uint32_t)a.Nq + (uint32_t)q0;

    TileStage<D> ks_[NP], vs_[NP];
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
        ks_[pl].issue(a.k.at(pl, b, h), a.k.sN, 0, a.Nk);
        vs_[pl].issue(a.v.at(pl, b, h), a.v.sN, 0, a.Nk);
    }
    for (int kv0 = 0; kv0 < a.Nk; kv0 += AT_KT) {
        __syncthreads();
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) {
            ks_[pl].commit(kl + pl * TW);
            vs_[pl].commit(vl + pl * TW);
        }
        __syncthreads();
        if (kv0 + AT_KT < a.Nk) {
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) {
                ks_[pl].issue(a.k.at(pl, b, h), a.k.sN, kv0 + AT_KT, a.Nk);
                vs_[pl].issue(a.v.at(pl, b, h), a.v.sN, kv0 + AT_KT, a.Nk);
            }
        }
        f32x4 s[2][4], dp[2][4];
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) s[qt][kt] = dp[qt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                s16x8 kf[NP], vf[NP];
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) {
                    kf[pl] = lds_row8<RSW>(kl + pl * TW, 16 * kt + c, 32 * ks + 8 * g);
                    vf[pl] = lds_row8<RSW>(vl + pl * TW, 16 * kt + c, 32 * ks + 8 * g);
                }
#pragma unroll
                for (int qt = 0; qt < 2; ++qt) {
                    s[qt][kt] = mmp<T, NP>(kf, qf[qt][ks], s[qt][kt]);
                    dp[qt][kt] = mmp<T, NP>(vf, gf[qt][ks], dp[qt][kt]);
                }
            }
        // dSᵀ = P (dP (keep / (1-p)) - delta), scaled by 2^8 for the MFMA
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
            const uint32_t row = row0 + 16 * qt + c;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = kv0 + 16 * kt + 4 * g + r;
                    const float p = key < a.Nk ? __builtin_amdgcn_exp2f(s[qt][kt][r] * a.scale_log2 - lse[qt]) : 0.f;
                    float d = dp[qt][kt][r];
                    if constexpr (DROP) d = at_keep(row, (uint32_t)key, a.p32, sd0, sd1) ? d * a.rdrop : 0.f;
                    s[qt][kt][r] = p * (d - dl[qt]) * AT_DS_SCALE;
                }
        }
        // dQᵀ += Kᵀ dSᵀ
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            s16x8 d0[NP], d1[NP];
            pack_acc<T, NP>(s[0][2 * st], s[0][2 * st + 1], d0);
            pack_acc<T, NP>(s[1][2 * st], s[1][2 * st + 1], d1);
#pragma unroll
            for (int db = 0; db < DB; ++db) {
                s16x8 kf[NP];
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) kf[pl] = lds_tr8<RSW>(kl + pl * TW, 32 * st, 16 * db, lane);
                acc[0][db] = mmp<T, NP>(kf, d0, acc[0][db]);
                acc[1][db] = mmp<T, NP>(kf, d1, acc[1][db]);
            }
        }
    }
    const float f = a.scale / AT_DS_SCALE;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
        const int q = q0 + 16 * qt + c;
        if (q < a.Nq) {
            float* dp_ = dq + b * dsB + h * dsH + (int64_t)q * dsN;
#pragma unroll
            for (int db = 0; db < DB; ++db)
                *reinterpret_cast<float4*>(dp_ + 16 * db + 4 * g) =
                    make_float4(acc[qt][db][0] * f, acc[qt][db][1] * f, acc[qt][db][2] * f, acc[qt][db][3] * f);
        }
    }
}

// ---------------------------------------------------------- backward dK, dV --
template <typename T, int D, bool DROP, int NP>
__global__ __launch_bounds__(AT_THREADS, NP == 2 ? 1 : 2) void attn_bwd_dkv_kernel(
    AtArgs a, float* __restrict__ dk, int64_t ksB, int64_t ksN, int64_t ksH, float* __restrict__ dv, int64_t vsB,
    int64_t vsN, int64_t vsH) {
    uint32_t sd0, sd1;
    at_seed(a, sd0, sd1);
    constexpr int RSW = at_rsw<D>();
    constexpr int KS = D / 32, DB = D / 16, TW = 64 * RSW;
    extern __shared__ __attribute__((aligned(16))) uint32_t at_lds[];
    uint32_t* ql = at_lds;              // [NP][64][RSW]
    uint32_t* gl = at_lds + NP * TW;    // [NP][64][RSW]
    float* lsel = reinterpret_cast<float*>(at_lds + 2 * NP * TW);
    float* dll = lsel + AT_QT;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, c = lane & 15;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
    const int key = blockIdx.x * AT_KB + wave * AT_KW + c;  // this lane's key (column of S)

    s16x8 kf[KS][NP], vf[KS][NP];  // B operands: lane (g, c) holds K/V[key][32ks + 8g .. +7]
    {
        const int kk = min(key, a.Nk - 1);
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) {
            const uint16_t* kp = a.k.at(pl, b, h) + (int64_t)kk * a.k.sN;
            const uint16_t* vp = a.v.at(pl, b, h) + (int64_t)kk * a.v.sN;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                kf[ks][pl] = *reinterpret_cast<const s16x8*>(kp + 32 * ks + 8 * g);
                vf[ks][pl] = *reinterpret_cast<const s16x8*>(vp + 32 * ks + 8 * g);
            }
        }
    }
    f32x4 ak[DB], av[DB];
#pragma unroll
    for (int db = 0; db < DB; ++db) ak[db] = av[db] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool kvalid = key < a.Nk;

    TileStage<D> qs_[NP], gs_[NP];
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
        qs_[pl].issue(a.q.at(pl, b, h), a.q.sN, 0, a.Nq);
        gs_[pl].issue(a.dout.at(pl, b, h), a.osN, 0, a.Nq);
    }
    for (int qv0 = 0; qv0 < a.Nq; qv0 += AT_QT) {
        __syncthreads();
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) {
            qs_[pl].commit(ql + pl * TW);
            gs_[pl].commit(gl + pl * TW);
        }
        if (threadIdx.x < AT_QT) {
            const int q = qv0 + threadIdx.x;
            // padded rows: P = exp2(-inf) = 0 and delta 0, so they add nothing
            lsel[threadIdx.x] = q < a.Nq ? a.lse[(int64_t)bh * a.Nq + q] : INFINITY;
            dll[threadIdx.x] = q < a.Nq ? a.delta[(int64_t)bh * a.Nq + q] : 0.f;
        }
        __syncthreads();
        if (qv0 + AT_QT < a.Nq) {
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) {
                qs_[pl].issue(a.q.at(pl, b, h), a.q.sN, qv0 + AT_QT, a.Nq);
                gs_[pl].issue(a.dout.at(pl, b, h), a.osN, qv0 + AT_QT, a.Nq);
            }
        }
        f32x4 s[4], dp[4];  // [query tile]: lane = key, registers = queries 16qt + 4g + r
#pragma unroll
        for (int qt = 0; qt < 4; ++qt) s[qt] = dp[qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int qt = 0; qt < 4; ++qt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                s16x8 qa[NP], ga[NP];
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) {
                    qa[pl] = lds_row8<RSW>(ql + pl * TW, 16 * qt + c, 32 * ks + 8 * g);
                    ga[pl] = lds_row8<RSW>(gl + pl * TW, 16 * qt + c, 32 * ks + 8 * g);
                }
                s[qt] = mmp<T, NP>(qa, kf[ks], s[qt]);
                dp[qt] = mmp<T, NP>(ga, vf[ks], dp[qt]);
            }
#pragma unroll
        for (int qt = 0; qt < 4; ++qt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int qi = 16 * qt + 4 * g + r;
                const float p = kvalid ? __builtin_amdgcn_exp2f(s[qt][r] * a.scale_log2 - lsel[qi]) : 0.f;
                float d = dp[qt][r], pd = p;
                if constexpr (DROP) {
                    const uint32_t row = (uint32_t)bh * (uint32_t)a.Nq + (uint32_t)(qv0 + qi);
                    const bool kp = at_keep(row, (uint32_t)key, a.p32, sd0, sd1);
                    d = kp ? d * a.rdrop : 0.f;
                    pd = kp ? p : 0.f;
                }
                dp[qt][r] = p * (d - dll[qi]) * AT_DS_SCALE;  // dS
                s[qt][r] = pd;                                // P with the dropout mask (1/(1-p) at the end)
            }
        // dVᵀ += dOᵀ P, dKᵀ += Qᵀ dS over two 32-query steps
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            s16x8 pf[NP], df[NP];
            pack_acc<T, NP>(s[2 * st], s[2 * st + 1], pf);
            pack_acc<T, NP>(dp[2 * st], dp[2 * st + 1], df);
#pragma unroll
            for (int db = 0; db < DB; ++db) {
                s16x8 gt[NP], qtr[NP];
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) {
                    gt[pl] = lds_tr8<RSW>(gl + pl * TW, 32 * st, 16 * db, lane);
                    qtr[pl] = lds_tr8<RSW>(ql + pl * TW, 32 * st, 16 * db, lane);
                }
                av[db] = mmp<T, NP>(gt, pf, av[db]);
                ak[db] = mmp<T, NP>(qtr, df, ak[db]);
            }
        }
    }
    if (kvalid) {
        const float fk = a.scale / AT_DS_SCALE, fv = DROP ? a.rdrop : 1.f;
        float* kp = dk + b * ksB + h * ksH + (int64_t)key * ksN;
        float* vp = dv + b * vsB + h * vsH + (int64_t)key * vsN;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            *reinterpret_cast<float4*>(kp + 16 * db + 4 * g) =
                make_float4(ak[db][0] * fk, ak[db][1] * fk, ak[db][2] * fk, ak[db][3] * fk);
            *reinterpret_cast<float4*>(vp + 16 * db + 4 * g) =
                make_float4(av[db][0] * fv, av[db][1] * fv, av[db][2] * fv, av[db][3] * fv);
        }
    }
}

__global__ void attn_mask_kernel(int64_t rows, int Nk, uint32_t p32, uint32_t s0, uint32_t s1,
                                 uint8_t* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rows * Nk) return;
    const int64_t row = e / Nk;
    const int col = (int)(e - row * Nk);
    out[e] = at_keep((uint32_t)row, (uint32_t)col, p32, s0, s1) ? 1 : 0;
}

// ------------------------------------------------------------------ host ----
struct Drop {
    uint32_t p32;
    float rdrop;
    bool on;
};

Drop drop_params(float p) {
    Drop d{0u, 1.f, false};
    if (p > 0.f) {
        const double t = (double)p * 4294967296.0;
        d.p32 = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
        d.rdrop = 1.f / (1.f - p);
        d.on = true;
    }
    return d;
}

// 16-byte operand rows: pointer and every stride a multiple of 8 elements
bool op_ok(const void* p, int64_t sP, int64_t sB, int64_t sN, int64_t sH) {
    return p && (reinterpret_cast<uintptr_t>(p) & 15) == 0 && sP % 8 == 0 && sB % 8 == 0 && sN % 8 == 0 &&
           sH % 8 == 0;
}

// Launch kernel K<T, D, DROP, NP> for (dtype, D, dropout): dtype 0 fp16, 1 bf16, 2 split fp32 (bf16 planes).
#define DGX_ATTN_DISPATCH(LAUNCH)                                                  \
    do {                                                                           \
        if (dtype == 0) {                                                          \
            if (D == 128) { if (dr.on) LAUNCH(_Float16, 128, true, 1); else LAUNCH(_Float16, 128, false, 1); } \
            else { if (dr.on) LAUNCH(_Float16, 64, true, 1); else LAUNCH(_Float16, 64, false, 1); }            \
        } else if (dtype == 1) {                                                   \
            if (D == 128) { if (dr.on) LAUNCH(__bf16, 128, true, 1); else LAUNCH(__bf16, 128, false, 1); }     \
            else { if (dr.on) LAUNCH(__bf16, 64, true, 1); else LAUNCH(__bf16, 64, false, 1); }                \
        } else {                                                                   \
            if (D == 128) { if (dr.on) LAUNCH(__bf16, 128, true, 2); else LAUNCH(__bf16, 128, false, 2); }     \
            else { if (dr.on) LAUNCH(__bf16, 64, true, 2); else LAUNCH(__bf16, 64, false, 2); }                \
        }                                                                          \
    } while (0)

}  // namespace

extern "C" {

int dgx_attn_fwd(int dtype, const void* q, int64_t qsP, int64_t qsB, int64_t qsN, int64_t qsH, const void* k,
                 int64_t ksP, int64_t ksB, int64_t ksN, int64_t ksH, const void* v, int64_t vsP, int64_t vsB,
                 int64_t vsN, int64_t vsH, void* o, int64_t osB, int64_t osN, int64_t osH, float* lse, int B, int H,
                 int Nq, int Nk, int D, float scale, float dropout_p, uint64_t seed, const uint64_t* seed_dev,
                 void* stream) {
    if (!o || !lse || B < 0 || H < 1 || Nq < 0 || Nk < 1 || !(scale > 0.f)) return DGX_EINVAL;
    if (!(dropout_p >= 0.f && dropout_p < 1.f)) return DGX_EINVAL;
    if (dtype < 0 || dtype > 2 || (D != 64 && D != 128)) return DGX_EUNSUPPORTED;
    if (!op_ok(q, qsP, qsB, qsN, qsH) || !op_ok(k, ksP, ksB, ksN, ksH) || !op_ok(v, vsP, vsB, vsN, vsH) ||
        (reinterpret_cast<uintptr_t>(o) & 15) != 0 || osB % 4 != 0 || osN % 4 != 0 || osH % 4 != 0)
        return DGX_EINVAL;
    if (B == 0 || Nq == 0) return DGX_OK;
    const Drop dr = drop_params(dropout_p);
    AtArgs a{};
    a.q = AtOp{static_cast<const uint16_t*>(q), qsP, qsB, qsN, qsH};
    a.k = AtOp{static_cast<const uint16_t*>(k), ksP, ksB, ksN, ksH};
    a.v = AtOp{static_cast<const uint16_t*>(v), vsP, vsB, vsN, vsH};
    a.osB = osB, a.osN = osN, a.osH = osH;
    a.lse = lse, a.H = H, a.Nq = Nq, a.Nk = Nk;
    a.scale_log2 = scale * 1.4426950408889634f, a.scale = scale;
    a.p32 = dr.p32, a.rdrop = dr.rdrop, a.s0 = (uint32_t)seed, a.s1 = (uint32_t)(seed >> 32);
    a.seedp = seed_dev;
    const dim3 grid((Nq + AT_QB - 1) / AT_QB, B * H);
    hipStream_t st = dgx_stream(stream);
#define DGX_ATTN_FWD(T, DV, DR, NPV)                                                                      \
    hipLaunchKernelGGL((attn_fwd_kernel<T, DV, DR, NPV>), grid, dim3(AT_THREADS), (at_lds_bytes_qk<DV, NPV>()), \
                       st, a, o)
    DGX_ATTN_DISPATCH(DGX_ATTN_FWD);
#undef DGX_ATTN_FWD
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_attn_bwd(int dtype, const void* q, int64_t qsP, int64_t qsB, int64_t qsN, int64_t qsH, const void* k,
                 int64_t ksP, int64_t ksB, int64_t ksN, int64_t ksH, const void* v, int64_t vsP, int64_t vsB,
                 int64_t vsN, int64_t vsH, const void* o, const void* dout, int64_t gsP, int64_t osB, int64_t osN,
                 int64_t osH, const float* dout32, const float* lse, float* delta, int B, int H, int Nq, int Nk, int D,
                 float scale, float dropout_p, uint64_t seed, const uint64_t* seed_dev, float* dq, int64_t dqsB,
                 int64_t dqsN, int64_t dqsH,
                 float* dk, int64_t dksB, int64_t dksN, int64_t dksH, float* dv, int64_t dvsB, int64_t dvsN,
                 int64_t dvsH, void* stream) {
    if (!o || !lse || !delta || !dq || !dk || !dv || B < 0 || H < 1 || Nq < 0 || Nk < 1 || !(scale > 0.f))
        return DGX_EINVAL;
    if (!(dropout_p >= 0.f && dropout_p < 1.f)) return DGX_EINVAL;
    if (dtype < 0 || dtype > 2 || (D != 64 && D != 128)) return DGX_EUNSUPPORTED;
    if (dtype == 2 && !dout32) return DGX_EINVAL;
    if (!op_ok(q, qsP, qsB, qsN, qsH) || !op_ok(k, ksP, ksB, ksN, ksH) || !op_ok(v, vsP, vsB, vsN, vsH) ||
        !op_ok(dout, gsP, osB, osN, osH) || (reinterpret_cast<uintptr_t>(o) & 15) != 0)
        return DGX_EINVAL;
    if ((reinterpret_cast<uintptr_t>(dq) | reinterpret_cast<uintptr_t>(dk) | reinterpret_cast<uintptr_t>(dv)) & 15 ||
        dqsN % 4 || dqsH % 4 || dksN % 4 || dksH % 4 || dvsN % 4 || dvsH % 4 || dqsB % 4 || dksB % 4 || dvsB % 4)
        return DGX_EINVAL;
    if (B == 0 || Nq == 0) return DGX_OK;
    const Drop dr = drop_params(dropout_p);
    AtArgs a{};
    a.q = AtOp{static_cast<const uint16_t*>(q), qsP, qsB, qsN, qsH};
    a.k = AtOp{static_cast<const uint16_t*>(k), ksP, ksB, ksN, ksH};
    a.v = AtOp{static_cast<const uint16_t*>(v), vsP, vsB, vsN, vsH};
    a.dout = AtOp{static_cast<const uint16_t*>(dout), gsP, osB, osN, osH};
    a.o = o, a.dout32 = dout32;
    a.osB = osB, a.osN = osN, a.osH = osH;
    a.lse = const_cast<float*>(lse), a.delta = delta, a.H = H, a.Nq = Nq, a.Nk = Nk;
    a.scale_log2 = scale * 1.4426950408889634f, a.scale = scale;
    a.p32 = dr.p32, a.rdrop = dr.rdrop, a.s0 = (uint32_t)seed, a.s1 = (uint32_t)(seed >> 32);
    a.seedp = seed_dev;
    hipStream_t st = dgx_stream(stream);
    const int64_t rows = (int64_t)B * H * Nq;
    const unsigned dblocks = (unsigned)((rows * 16 + 255) / 256);
    if (D == 128) hipLaunchKernelGGL((attn_delta_kernel<128>), dim3(dblocks), dim3(256), 0, st, a, B, dtype);
    else hipLaunchKernelGGL((attn_delta_kernel<64>), dim3(dblocks), dim3(256), 0, st, a, B, dtype);
    DGX_CHECK_LAUNCH();
    const dim3 gq((Nq + AT_QB - 1) / AT_QB, B * H), gk((Nk + AT_KB - 1) / AT_KB, B * H);
#define DGX_ATTN_BWD(T, DV, DR, NPV)                                                                          \
    do {                                                                                                      \
        hipLaunchKernelGGL((attn_bwd_dq_kernel<T, DV, DR, NPV>), gq, dim3(AT_THREADS),                        \
                           (at_lds_bytes_qk<DV, NPV>()), st, a, dq, dqsB, dqsN, dqsH);                        \
        hipLaunchKernelGGL((attn_bwd_dkv_kernel<T, DV, DR, NPV>), gk, dim3(AT_THREADS),                       \
                           (at_lds_bytes_qk<DV, NPV>() + 2 * AT_QT * 4), st, a, dk, dksB, dksN, dksH, dv, dvsB, \
                           dvsN, dvsH);                                                                       \
    } while (0)
    DGX_ATTN_DISPATCH(DGX_ATTN_BWD);
#undef DGX_ATTN_BWD
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

int dgx_attn_dropout_mask(int64_t rows, int Nk, float dropout_p, uint64_t seed, uint8_t* out, void* stream) {
    if (!out || rows < 0 || Nk < 1 || !(dropout_p >= 0.f && dropout_p < 1.f)) return DGX_EINVAL;
    if (rows == 0) return DGX_OK;
    const Drop dr = drop_params(dropout_p);
    const int64_t n = rows * Nk;
    hipLaunchKernelGGL(attn_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, dgx_stream(stream), rows, Nk,
                       dr.on ? dr.p32 : 0u, (uint32_t)seed, (uint32_t)(seed >> 32), out);
    return hipGetLastError() == hipSuccess ? DGX_OK : DGX_ELAUNCH;
}

}  // extern "C"
