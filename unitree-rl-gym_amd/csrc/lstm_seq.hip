// lstm_seq.hip — the recurrent memory of rsl_rl's ActorCriticRecurrent (one-layer
// LSTM, torch gate order i, f, g, o) as two sequence kernels for gfx950, part of
// libppomlp.so (include/ppo_mlp.h, "recurrent memory").
//
// rsl_rl v1.0.2 trains the LSTM on trajectories split at dones and zero-padded to T
// (split_and_pad_trajectories: a data-dependent trajectory count, a host sync per
// mini-batch).  The same outputs come from running every env's T steps densely and
// zeroing (h, c) before step t whenever the env was done at t-1: a padded trajectory
// that starts after a done starts from the zero state the rollout saved there.  So
// these kernels take a [T, B] reset mask instead of padded trajectories: fixed shapes,
// no host sync, capturable in a HIP graph.
//
// Layout: one workgroup of 4H threads owns EB envs for all T steps; thread j owns gate
// column j (its row of W_hh in registers); the envs' h and c live in LDS across steps.
// The input projection x W_ih^T + b is one GEMM over all T*B rows beforehand (gx).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "../../include/ppo_mlp.h"
#include "pmlp_noise.h"

namespace {

// envs per workgroup: 8, or 4 when that leaves fewer than two workgroups per CU (the
// update's 2048-env mini-batches: a step is latency-bound, so more resident workgroups)
constexpr int EB_MAX = 8;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// Per step every thread issues the NEXT step's global inputs (gx, reset flags; in the
// backward dh_out, c, c_prev, gates) before this step's work, so one load round trip is
// in flight behind each step instead of exposed in it; the EB envs' dot products run
// interleaved (EB independent FMA chains).

// forward over T steps: gact [T,B,4H] (activated gates), c_out [T,B,H], h_out [T,B,H];
// each of gact / c_out / h_out / h_last / c_last may be null.
// IP == 0: the gate pre-activations come as gx [T,B,4H] (x W_ih^T + b, a GEMM beforehand).
// IP > 0: the input projection is fused in: x [T,B,I] (I <= IP) is staged through LDS per
// step and thread j adds b_ih[j] + b_hh[j] + x . W_ih[j] (its W_ih row in registers) --
// no [T,B,4H] gx round trip through HBM; xh (optional) receives [x | h_prev | 1] per row,
// the operand of the weight gradients (h_prev: the state the step starts from, after a
// reset).
struct FwdArgs {
    int T, B, I;
    const float* gx;
    const float* x;
    const float* wih;
    const float* bih;
    const float* bhh;
    const float* whh;
    const float* h0;
    const float* c0;
    const uint8_t* reset;
    float* h_out;
    float* c_out;
    float* gact;
    float* h_last;
    float* c_last;
    float* xh;
    float* h_save;  // (optional) copies of h0 / c0 as read: the rollout storage's saved state
    float* c_save;
};

template <int H, int EB, int IP>
__global__ __launch_bounds__(4 * H) void k_lstm_fwd(FwdArgs a) {
    constexpr int G = 4 * H;
    constexpr int PE = EB / 4;  // (env, unit) elements per thread in the elementwise phases (EB*H / 4H)
    constexpr int XS = IP > 0 ? IP : 4;
    constexpr int XPT = IP > 0 ? (EB * IP + G - 1) / G : 1;  // staged x elements per thread
    __shared__ __attribute__((aligned(16))) float hs[EB][H];
    __shared__ float cs[EB][H];
    __shared__ float ga[EB][G];
    __shared__ __attribute__((aligned(16))) float xs[EB][XS];
    const int T = a.T, B = a.B, I = a.I;
    const int j = threadIdx.x;
    const int e0 = blockIdx.x * EB;
    float w[H];
#pragma unroll
    for (int k = 0; k < H; k += 4) {
        const float4 v = *reinterpret_cast<const float4*>(a.whh + (size_t)j * H + k);
        w[k] = v.x; w[k + 1] = v.y; w[k + 2] = v.z; w[k + 3] = v.w;
    }
    float wi[IP > 0 ? IP : 1];
    float bj = 0.f;
    if constexpr (IP > 0) {
#pragma unroll
        for (int i = 0; i < IP; ++i) wi[i] = i < I ? a.wih[(size_t)j * I + i] : 0.f;
        bj = (a.bih ? a.bih[j] : 0.f) + (a.bhh ? a.bhh[j] : 0.f);
    }
#pragma unroll
    for (int p = 0; p < PE; ++p) {
        const int i = j + p * G, e = i / H, k = i % H, ge = e0 + e;
        const float hv = (ge < B && a.h0) ? a.h0[(size_t)ge * H + k] : 0.f;
        const float cv = (ge < B && a.c0) ? a.c0[(size_t)ge * H + k] : 0.f;
        hs[e][k] = hv;
        cs[e][k] = cv;
        if (ge < B && a.h_save) a.h_save[(size_t)ge * H + k] = hv;
        if (ge < B && a.c_save) a.c_save[(size_t)ge * H + k] = cv;
    }
    const int kind = j / H;  // 0 i, 1 f, 2 g (tanh), 3 o
    float gxn[IP > 0 ? 1 : EB];
    float xn[XPT];
    bool rsn[PE];
    auto fetch = [&](int t) {
        if constexpr (IP == 0) {
#pragma unroll
            for (int e = 0; e < EB; ++e) {
                const int ge = e0 + e;
                gxn[e] = ge < B ? a.gx[((size_t)t * B + ge) * G + j] : 0.f;
            }
        } else {
#pragma unroll
            for (int p = 0; p < XPT; ++p) {
                const int q = j + p * G, e = q / IP, i = q % IP, ge = e0 + e;
                xn[p] = (q < EB * IP && ge < B && i < I) ? a.x[((size_t)t * B + ge) * I + i] : 0.f;
            }
        }
#pragma unroll
        for (int p = 0; p < PE; ++p) {
            const int ge = e0 + (j + p * G) / H;
            rsn[p] = a.reset && ge < B && a.reset[(size_t)t * B + ge];
        }
    };
    fetch(0);
    __syncthreads();
    const int RL = I + H + 1;  // xh row
    for (int t = 0; t < T; ++t) {
        float acc[EB];
        bool rs[PE];
        if constexpr (IP == 0) {
#pragma unroll
            for (int e = 0; e < EB; ++e) acc[e] = gxn[e];
        } else {
#pragma unroll
            for (int p = 0; p < XPT; ++p) {
                const int q = j + p * G;
                if (q < EB * IP) xs[q / IP][q % IP] = xn[p];
            }
#pragma unroll
            for (int e = 0; e < EB; ++e) acc[e] = bj;
        }
#pragma unroll
        for (int p = 0; p < PE; ++p) rs[p] = rsn[p];
        if (t + 1 < T) fetch(t + 1);
        if (a.reset) {
#pragma unroll
            for (int p = 0; p < PE; ++p) {
                const int i = j + p * G, e = i / H, k = i % H;
                if (rs[p]) { hs[e][k] = 0.f; cs[e][k] = 0.f; }
            }
        }
        if (IP > 0 || a.reset) __syncthreads();
        if constexpr (IP > 0) {
            if (a.xh) {
                for (int q = j; q < EB * RL; q += G) {
                    const int e = q / RL, c = q % RL, ge = e0 + e;
                    if (ge < B)
                        a.xh[((size_t)t * B + ge) * RL + c] = c < I ? xs[e][c] : (c < I + H ? hs[e][c - I] : 1.f);
                }
            }
            // input projection: env pairs, two interleaved FMA chains from the bias
#pragma unroll
            for (int e = 0; e < EB; e += 2) {
#pragma unroll
                for (int i4 = 0; i4 < IP / 4; ++i4) {
                    const float4 xa = reinterpret_cast<const float4*>(xs[e])[i4];
                    const float4 xb = reinterpret_cast<const float4*>(xs[e + 1])[i4];
                    acc[e] = fmaf(xa.x, wi[4 * i4], acc[e]);
                    acc[e + 1] = fmaf(xb.x, wi[4 * i4], acc[e + 1]);
                    acc[e] = fmaf(xa.y, wi[4 * i4 + 1], acc[e]);
                    acc[e + 1] = fmaf(xb.y, wi[4 * i4 + 1], acc[e + 1]);
                    acc[e] = fmaf(xa.z, wi[4 * i4 + 2], acc[e]);
                    acc[e + 1] = fmaf(xb.z, wi[4 * i4 + 2], acc[e + 1]);
                    acc[e] = fmaf(xa.w, wi[4 * i4 + 3], acc[e]);
                    acc[e + 1] = fmaf(xb.w, wi[4 * i4 + 3], acc[e + 1]);
                }
                asm volatile("" ::: "memory");
            }
        }
        // env pairs: two interleaved FMA chains (the compiler barrier keeps one pair's LDS
        // reads in flight at a time instead of hoisting all EB*H/4 of them)
#pragma unroll
        for (int e = 0; e < EB; e += 2) {
#pragma unroll
            for (int k4 = 0; k4 < H / 4; ++k4) {
                const float4 ha = reinterpret_cast<const float4*>(hs[e])[k4];
                const float4 hb = reinterpret_cast<const float4*>(hs[e + 1])[k4];
                acc[e] = fmaf(ha.x, w[4 * k4], acc[e]);
                acc[e + 1] = fmaf(hb.x, w[4 * k4], acc[e + 1]);
                acc[e] = fmaf(ha.y, w[4 * k4 + 1], acc[e]);
                acc[e + 1] = fmaf(hb.y, w[4 * k4 + 1], acc[e + 1]);
                acc[e] = fmaf(ha.z, w[4 * k4 + 2], acc[e]);
                acc[e + 1] = fmaf(hb.z, w[4 * k4 + 2], acc[e + 1]);
                acc[e] = fmaf(ha.w, w[4 * k4 + 3], acc[e]);
                acc[e + 1] = fmaf(hb.w, w[4 * k4 + 3], acc[e + 1]);
            }
            asm volatile("" ::: "memory");
        }
        if (kind == 2) {  // (wave-uniform for H >= 64; a branch, not both functions per env)
#pragma unroll
            for (int e = 0; e < EB; ++e) acc[e] = tanhf(acc[e]);
        } else {
#pragma unroll
            for (int e = 0; e < EB; ++e) acc[e] = sigm(acc[e]);
        }
#pragma unroll
        for (int e = 0; e < EB; ++e) {
            const int ge = e0 + e;
            ga[e][j] = acc[e];
            if (a.gact && ge < B) a.gact[((size_t)t * B + ge) * G + j] = acc[e];
        }
        __syncthreads();
#pragma unroll
        for (int p = 0; p < PE; ++p) {
            const int i = j + p * G, e = i / H, k = i % H, ge = e0 + e;
            if (ge >= B) continue;
            const float ig = ga[e][k], fg = ga[e][H + k], gg = ga[e][2 * H + k], og = ga[e][3 * H + k];
            const float c = fg * cs[e][k] + ig * gg;
            const float h = og * tanhf(c);
            cs[e][k] = c;
            hs[e][k] = h;
            const size_t o = ((size_t)t * B + ge) * H + k;
            if (a.h_out) a.h_out[o] = h;
            if (a.c_out) a.c_out[o] = c;
        }
        __syncthreads();
    }
#pragma unroll
    for (int p = 0; p < PE; ++p) {
        const int i = j + p * G, e = i / H, k = i % H, ge = e0 + e;
        if (ge >= B) continue;
        if (a.h_last) a.h_last[(size_t)ge * H + k] = hs[e][k];
        if (a.c_last) a.c_last[(size_t)ge * H + k] = cs[e][k];
    }
}

// backward through time: dh_out [T,B,H] -> dgx [T,B,4H] (gradient of the gate
// pre-activations, i.e. of gx and of the biases).  No gradient flows into h0/c0 or
// across a reset (the state was replaced by zeros there).
template <int H, int EB>
__global__ __launch_bounds__(4 * H) void k_lstm_bwd(int T, int B, const float* __restrict__ whh,
                                                    const float* __restrict__ c0, const uint8_t* __restrict__ reset,
                                                    const float* __restrict__ c_out, const float* __restrict__ gact,
                                                    const float* __restrict__ dh_out, float* __restrict__ dgx) {
    constexpr int G = 4 * H;
    constexpr int PE = EB / 4;
    __shared__ float dhn[EB][H], dcn[EB][H];
    __shared__ __attribute__((aligned(16))) float dgs[EB][G];
    __shared__ float red[4][EB][H];
    const int tid = threadIdx.x;
    const int e0 = blockIdx.x * EB;
    // thread (k, q): column k of W_hh over the gate rows q*H .. q*H+H-1
    const int k_own = tid % H, q = tid / H;
    float w[H];
#pragma unroll
    for (int jj = 0; jj < H; ++jj) w[jj] = whh[(size_t)(q * H + jj) * H + k_own];
#pragma unroll
    for (int p = 0; p < PE; ++p) {
        const int i = tid + p * G, e = i / H, k = i % H;
        dhn[e][k] = 0.f;
        dcn[e][k] = 0.f;
    }
    // step inputs of the thread's (env, unit) elements
    struct In {
        float dh, c, cp, ig, fg, gg, og;
        bool rs;
    };
    In nx[PE];
    auto fetch = [&](int t) {
#pragma unroll
        for (int p = 0; p < PE; ++p) {
            const int i = tid + p * G, e = i / H, k = i % H, ge = e0 + e;
            In& v = nx[p];
            if (ge >= B) {
                v = In{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, false};
                continue;
            }
            const size_t row = (size_t)t * B + ge;
            v.rs = reset && reset[row];
            v.dh = dh_out[row * H + k];
            v.c = c_out[row * H + k];
            v.cp = t > 0 ? c_out[(row - B) * H + k] : (c0 ? c0[(size_t)ge * H + k] : 0.f);
            const float* a = gact + row * G;
            v.ig = a[k]; v.fg = a[H + k]; v.gg = a[2 * H + k]; v.og = a[3 * H + k];
        }
    };
    fetch(T - 1);
    __syncthreads();
    for (int t = T - 1; t >= 0; --t) {
        In cur[PE];
#pragma unroll
        for (int p = 0; p < PE; ++p) cur[p] = nx[p];
        if (t > 0) fetch(t - 1);
        // gate gradients of step t, (env, unit) pairs
#pragma unroll
        for (int p = 0; p < PE; ++p) {
            const int i = tid + p * G, e = i / H, k = i % H, ge = e0 + e;
            if (ge >= B) {
#pragma unroll
                for (int g = 0; g < 4; ++g) dgs[e][g * H + k] = 0.f;
                continue;
            }
            const In& v = cur[p];
            const size_t row = (size_t)t * B + ge;
            const float dh = v.dh + dhn[e][k];
            const float cp = v.rs ? 0.f : v.cp;
            const float tc = tanhf(v.c);
            const float dc = dcn[e][k] + dh * v.og * (1.f - tc * tc);
            const float d_i = dc * v.gg * v.ig * (1.f - v.ig);
            const float d_f = dc * cp * v.fg * (1.f - v.fg);
            const float d_g = dc * v.ig * (1.f - v.gg * v.gg);
            const float d_o = dh * tc * v.og * (1.f - v.og);
            dgs[e][k] = d_i; dgs[e][H + k] = d_f; dgs[e][2 * H + k] = d_g; dgs[e][3 * H + k] = d_o;
            float* o = dgx + row * G;
            o[k] = d_i; o[H + k] = d_f; o[2 * H + k] = d_g; o[3 * H + k] = d_o;
            dcn[e][k] = v.rs ? 0.f : dc * v.fg;  // into c_{t-1} (none across a reset)
        }
        __syncthreads();
        // dh_{t-1} = dG W_hh: four partial sums over gate-row quarters, then a fixed-order add
        float acc[EB];
#pragma unroll
        for (int e = 0; e < EB; ++e) acc[e] = 0.f;
#pragma unroll
        for (int e = 0; e < EB; e += 2) {
#pragma unroll
            for (int j4 = 0; j4 < H / 4; ++j4) {
                const float4 da = reinterpret_cast<const float4*>(&dgs[e][q * H])[j4];
                const float4 db = reinterpret_cast<const float4*>(&dgs[e + 1][q * H])[j4];
                acc[e] = fmaf(da.x, w[4 * j4], acc[e]);
                acc[e + 1] = fmaf(db.x, w[4 * j4], acc[e + 1]);
                acc[e] = fmaf(da.y, w[4 * j4 + 1], acc[e]);
                acc[e + 1] = fmaf(db.y, w[4 * j4 + 1], acc[e + 1]);
                acc[e] = fmaf(da.z, w[4 * j4 + 2], acc[e]);
                acc[e + 1] = fmaf(db.z, w[4 * j4 + 2], acc[e + 1]);
                acc[e] = fmaf(da.w, w[4 * j4 + 3], acc[e]);
                acc[e + 1] = fmaf(db.w, w[4 * j4 + 3], acc[e + 1]);
            }
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int e = 0; e < EB; ++e) red[q][e][k_own] = acc[e];
        __syncthreads();
#pragma unroll
        for (int p = 0; p < PE; ++p) {
            const int i = tid + p * G, e = i / H, k = i % H;
            const float s = (red[0][e][k] + red[1][e][k]) + (red[2][e][k] + red[3][e][k]);
            dhn[e][k] = cur[p].rs ? 0.f : s;
        }
        __syncthreads();
    }
}


// ---------------------------------------------------------------- MFMA form --
// The update's dense sequences on the matrix cores (H = 64, I <= 64): a workgroup of 4
// waves owns E = 16 envs for all T steps; per step the gate pre-activations of its 16
// envs are ONE [16 x 128] . [128 x 256] product, [x_t | h_{t-1}] . [W_ih | W_hh]^T, on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation from the fp32 bias.  Precision: every
// operand is split into bf16 hi + lo (v = hi + lo to ~2^-16 relative) and the product is
// hi.hi + hi.lo + lo.hi (SPLIT = 3), near fp32 (SPLIT = 1, the plain bf16 product, was 5e-2
// off on the pretrained policies' action means: not shipped).
// The cell update, c and h stay in the lanes (fp32); the weight fragments are loaded once;
// h_{t-1} and x_t sit in a double-buffered LDS operand, one barrier per step.  Outputs as
// k_lstm_fwd (fp32).
// The backward runs the same way: the gate gradients (fp32, in the lane) go to dgx and, as
// bf16 (hi, lo), to an LDS operand for dh_{t-1} = dG . W_hh, whose 16 x 16 result tile of
// wave w is exactly the lane's own (env, unit) pairs.
constexpr int ME = 16, MH = 64, MG = 256, MKX = 64;  // envs per workgroup, hidden, gates, x slots
constexpr int MLDA = MKX + MH + 8;                   // LDS row stride of [x | h] (bf16): 272 B
constexpr int MLDG = MG + 8;                         // LDS row stride of dG (bf16): 528 B

typedef __bf16 mbf16;
typedef mbf16 mbf16x8 __attribute__((ext_vector_type(8)));
typedef mbf16 mbf16x4 __attribute__((ext_vector_type(4)));
typedef float mfloatx4 __attribute__((ext_vector_type(4)));

// activations of the MFMA kernels: v_exp_f32 + v_rcp_f32 (a few ulp; tanh to ~1e-7 absolute)
__device__ __forceinline__ float fsig(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float ftanh(float x) { return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f; }

__device__ __forceinline__ void split_bf16(float v, mbf16& hi, mbf16& lo) {
    hi = (mbf16)v;
    lo = (mbf16)(v - (float)hi);
}

struct MFwdArgs {
    int T, B, I;
    const float *x, *wih, *bih, *bhh, *whh, *h0, *c0;
    const uint8_t* reset;
    float *h_out, *c_out, *gact, *xh;
    float *h_save, *c_save;  // optional: the state the sequence starts from (the rollout's storage slot)
};

// Eight waves (512 threads, two waves per SIMD): wave w owns units 8w .. 8w + 7 as two
// 16-column tiles, [i | f] and [g | o] (8 units each), so a step is 24 MFMAs per wave (a
// 4-wave form with the four gate tiles of 16 units per wave ran 68 vs 59 us at H1 scale).
// A lane (column j) holds i, g (j < 8) or f, o (j >= 8) of unit 8w + (j & 7) for its 4 rows;
// the partner lane j ^ 8 (DPP row_ror:8, one VALU move per value) supplies the other two
// gates, and each lane updates 2 of the 4 (env, unit) pairs (j < 8: rows 0, 1; else 2, 3).
__device__ __forceinline__ float ror8(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
}

// Up to two independent sequences per launch (the actor's and the critic's memory: a
// 2,048-env mini-batch is 128 workgroups, half the CUs, so one launch of both fills them):
// blockIdx.y selects the job; a job with fewer workgroups than the grid's x leaves the rest.
struct MFwdBatch { MFwdArgs m[2]; };

// tiles: consecutive 16-env tiles per workgroup, run one after the other on the weight
// fragments loaded once (the rollout's single steps: the fragments' 128 KB of loads per
// workgroup otherwise dominate a T = 1 launch); each tile's arithmetic is the same
template <int SPLIT>
__global__ __launch_bounds__(512) void k_lstm_fwd_mfma8(MFwdBatch ab, int tiles) {
    constexpr int NP = SPLIT == 3 ? 2 : 1;  // operand parts (hi, lo)
    __shared__ __attribute__((aligned(16))) mbf16 A[NP][2][ME * MLDA];
    const MFwdArgs a = ab.m[blockIdx.y];
    const int T = a.T, B = a.B, I = a.I, RL = I + MH + 1;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int ebase = blockIdx.x * ME * tiles;
    if (ebase >= B) return;  // (whole workgroup)
    const int j = lane & 15, rg = lane >> 4;  // column in the tile; row group (envs 4 rg .. 4 rg + 3)
    const int hj = j >> 3;                    // 0: this column holds i / g, 1: f / o
    const int uu = 8 * w + (j & 7);           // this lane's unit
    // weight fragments: tile t (0: [i | f], 1: [g | o]), k-step s
    mbf16x8 wf[NP][2][4];
    float bias[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const int r = (2 * tt + hj) * MH + uu;
        bias[tt] = a.bih[r] + a.bhh[r];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = s * 32 + 8 * rg + e;
                const float v = k < MKX ? (k < I ? a.wih[(size_t)r * I + k] : 0.f) : a.whh[(size_t)r * MH + (k - MKX)];
                mbf16 hi, lo;
                split_bf16(v, hi, lo);
                wf[0][tt][s][e] = hi;
                if constexpr (NP == 2) wf[NP - 1][tt][s][e] = lo;
            }
    }
    // a tile's t = 0 inputs (state, reset, x), loaded for tile q + 1 while tile q computes (the
    // rollout's multi-tile steps: each tile otherwise waits one full round trip on them);
    // unconditional loads at clamped addresses, masked where used
    const bool xs = tid < 256;
    const int xe = (tid & 255) >> 4, xk = (tid & 15) * 4;
    float pf_h[2], pf_c[2], pf_x[4];
    uint8_t pf_r[2], pf_rn[2];  // resets at t = 0 and at t = 1 (rload(1))
    const uint8_t* rbase = a.reset ? a.reset : (const uint8_t*)a.x;  // masked when absent
    // (absent h0 / c0 / reset: a load of x[0], masked -- no branch, which would put a vmcnt(0)
    // behind every load)
    const float* h0p = a.h0 ? a.h0 : a.x;
    const float* c0p = a.c0 ? a.c0 : a.x;
    auto in_load = [&](int e0n) {
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            const int gc = min(e0n + 4 * rg + 2 * hj + pp, B - 1);
            const float hv = h0p[a.h0 ? (size_t)gc * MH + uu : 0];
            const float cv = c0p[a.c0 ? (size_t)gc * MH + uu : 0];
            const uint8_t r0 = rbase[a.reset ? gc : 0];
            pf_h[pp] = a.h0 ? hv : 0.f;
            pf_c[pp] = a.c0 ? cv : 0.f;
            pf_r[pp] = a.reset ? r0 : (uint8_t)0;
            pf_rn[pp] = rbase[(size_t)min(1, T - 1) * B + gc];
        }
        const int gx = min(e0n + xe, B - 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) pf_x[i] = a.x[(size_t)gx * I + min(xk + i, I - 1)];
    };
    in_load(ebase);
    for (int q = 0; q < tiles; ++q) {
    const int e0 = ebase + q * ME;
    if (e0 >= B) break;   // (uniform)
    if (q) __syncthreads();  // the previous tile's last reads of A are done
    auto put = [&](int buf, int idx, float v) {  // operand element (hi, lo)
        mbf16 hi, lo;
        split_bf16(v, hi, lo);
        A[0][buf][idx] = hi;
        if constexpr (NP == 2) A[NP - 1][buf][idx] = lo;
    };
    // x staging by the first 256 threads: 4 floats each per step (16 envs x 64 slots).  x and
    // the resets are loaded two steps ahead (xr: step t + 1's, stored at the end of step t; xr2:
    // step t + 2's): vmcnt counts the per-step stores too and retires in order, so a load issued
    // after step t's stores and used one step later waited for those stores as well
    float xr[4], xr2[4];
    auto xload = [&](int t, float (&dst)[4]) {
        const int gc = min(e0 + xe, B - 1);
        const size_t tc = (size_t)min(t, T - 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[i] = a.x[(tc * B + gc) * I + min(xk + i, I - 1)];
    };
    auto xstore = [&](int buf, int t) {
        const int ge = e0 + xe;
#pragma unroll
        for (int i = 0; i < 4; ++i) xr[i] = (ge < B && xk + i < I) ? xr[i] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) put(buf, xe * MLDA + xk + i, xr[i]);
        if (a.xh && ge < B) {
            float* row = a.xh + ((size_t)t * B + ge) * RL;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (xk + i < I) row[xk + i] = xr[i];
            if (xk == 0) row[I + MH] = 1.f;
        }
    };
    // state of the lane's 2 (env, unit) pairs: rows 2 hj, 2 hj + 1 of its row group
    float c[2], hp[2];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
        const int p = 2 * hj + pp, ge = e0 + 4 * rg + p;
        const bool rs = a.reset && ge < B && pf_r[pp];
        const float h0 = ge < B ? pf_h[pp] : 0.f;
        const float c0 = ge < B ? pf_c[pp] : 0.f;
        hp[pp] = rs ? 0.f : h0;
        c[pp] = rs ? 0.f : c0;
        put(0, (4 * rg + p) * MLDA + MKX + uu, hp[pp]);
        if (a.h_save && ge < B) {
            a.h_save[(size_t)ge * MH + uu] = hp[pp];
            a.c_save[(size_t)ge * MH + uu] = c[pp];
        }
    }
    const bool has_reset = a.reset != nullptr;
    auto rload = [&](int t, uint8_t* r) {
        const size_t tc = (size_t)min(t, T - 1) * B;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) r[pp] = rbase[tc + min(e0 + 4 * rg + 2 * hj + pp, B - 1)];
    };
    uint8_t rnx[2] = {pf_rn[0], pf_rn[1]};  // reset(t + 1) at step t (rload(1), prefetched)
    uint8_t rnx2[2];                          // reset(t + 2)
    rload(2, rnx2);
    if (xs) {
#pragma unroll
        for (int i = 0; i < 4; ++i) xr[i] = pf_x[i];  // (xload(0), prefetched)
        xstore(0, 0);
        if (T > 1) xload(1, xr);
    }
    // the next tile's, in flight from here (not hoisted above this tile's last uses of the
    // prefetched values: vmcnt is in order, so those would then wait for these)
    __builtin_amdgcn_sched_barrier(0);
    if (q + 1 < tiles && e0 + ME < B) in_load(e0 + ME);
    __syncthreads();
    for (int t = 0; t < T; ++t) {
        const int cur = t & 1;
        bool rn[2];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            rn[pp] = has_reset && t + 1 < T && rnx[pp] != 0;
            rnx[pp] = rnx2[pp];
        }
        rload(t + 3, rnx2);
        if (xs) xload(t + 2, xr2);  // (clamped to T - 1 past the end)
        mfloatx4 acc[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int p = 0; p < 4; ++p) acc[tt][p] = bias[tt];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int o = j * MLDA + s * 32 + 8 * rg;
            const mbf16x8 ah = *(const mbf16x8*)(&A[0][cur][o]);
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wf[0][tt][s], acc[tt], 0, 0, 0);
            if constexpr (NP == 2) {
                const mbf16x8 al = *(const mbf16x8*)(&A[NP - 1][cur][o]);
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wf[NP - 1][tt][s], acc[tt], 0, 0, 0);
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, wf[0][tt][s], acc[tt], 0, 0, 0);
            }
        }
        // own rows and the partner's: own = rows 2 hj + pp, sent = the partner's own rows
        float ownA[2], ownB[2], rcvA[2], rcvB[2];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            ownA[pp] = hj ? acc[0][2 + pp] : acc[0][pp];
            ownB[pp] = hj ? acc[1][2 + pp] : acc[1][pp];
            rcvA[pp] = ror8(hj ? acc[0][pp] : acc[0][2 + pp]);
            rcvB[pp] = ror8(hj ? acc[1][pp] : acc[1][2 + pp]);
        }
        const int nxt = cur ^ 1;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            const int p = 2 * hj + pp, ge = e0 + 4 * rg + p;
            const float zi = hj ? rcvA[pp] : ownA[pp], zf = hj ? ownA[pp] : rcvA[pp];
            const float zg = hj ? rcvB[pp] : ownB[pp], zo = hj ? ownB[pp] : rcvB[pp];
            const float ig = fsig(zi), fg = fsig(zf), gg = ftanh(zg), og = fsig(zo);
            const float cn = fg * c[pp] + ig * gg;
            const float hn = og * ftanh(cn);
            if (ge < B) {
                const size_t row = (size_t)t * B + ge;
                if (a.gact) {
                    float* gr = a.gact + row * MG;
                    gr[uu] = ig; gr[MH + uu] = fg; gr[2 * MH + uu] = gg; gr[3 * MH + uu] = og;
                }
                if (a.c_out) a.c_out[row * MH + uu] = cn;
                if (a.h_out) a.h_out[row * MH + uu] = hn;
                if (a.xh) a.xh[row * RL + I + uu] = hp[pp];  // the state this step started from
            }
            c[pp] = rn[pp] ? 0.f : cn;  // a reset at t + 1 starts that step from zero
            hp[pp] = rn[pp] ? 0.f : hn;
            if (t + 1 < T) put(nxt, (4 * rg + p) * MLDA + MKX + uu, hp[pp]);
        }
        if (xs) {
            if (t + 1 < T) xstore(nxt, t + 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) xr[i] = xr2[i];
        }
        __syncthreads();
    }
    }  // tiles
}

struct MBwdArgs {
    int T, B;
    const float *whh, *c0;
    const uint8_t* reset;
    const float *c_out, *gact, *dh_out;
    float* dgx;        // optional: the gate gradients [T, B, 4H]
    const float* xh;   // DW: the forward's [x | h_prev | 1] rows [T, B, I + H + 1]
    int I;
    float* slab;       // DW: per workgroup [dW_ih (4H x I) | dW_hh (4H x H) | db (4H)], torch row order
};

// DW: the three weight gradients dG^T [x | h_prev | 1] accumulate inside the backward as well,
// on four more waves of the workgroup (512 threads): per step the workgroup's 16 envs are the
// K of a [256 gates x 16] . [16 x (I + H + 1)] product on v_mfma_f32_32x32x16_bf16 (split-bf16
// operands, fp32 accumulators held over all T steps; weight-gradient wave w owns gate-row tiles
// 2w, 2w + 1) beside the recurrence, written once per workgroup into its slab row
// (summed over workgroups by pmlp_reduce_slabs): no [T, B, 4H] dgx round trip and no
// separate 49k-row reduction GEMM.
constexpr int MXC = 128;  // xh columns covered (I + H + 1 <= 128)
typedef float mfloatx16 __attribute__((ext_vector_type(16)));

struct MBwdBatch { MBwdArgs m[2]; };  // as MFwdBatch

template <int SPLIT, bool DW>
__global__ __launch_bounds__(DW ? 512 : 256) void k_lstm_bwd_mfma(MBwdBatch ab) {
    constexpr int NP = SPLIT == 3 ? 2 : 1;
    const MBwdArgs a = ab.m[blockIdx.y];
    if ((int)blockIdx.x * ME >= a.B) return;  // (whole workgroup)
    __shared__ __attribute__((aligned(16))) mbf16 G[NP][2][ME * MLDG];
    // DW operands, transposed so a fragment is 8 consecutive envs (one 16-byte read):
    // GT[perm gate col][env], XT[xh col][env]
    __shared__ __attribute__((aligned(16))) mbf16 GT[DW ? NP : 1][2][DW ? MG * ME : 8];
    __shared__ __attribute__((aligned(16))) mbf16 XT[DW ? NP : 1][2][DW ? MXC * ME : 8];
    const int T = a.T, B = a.B;
    const int e0 = blockIdx.x * ME;
    if (DW && threadIdx.x >= 256) {
        // ---- DW: the weight-gradient waves (4..7), off the recurrence's critical path: per
        // step they stage that step's xh rows (transposed, split) and, after the step's
        // barrier, accumulate dG^T [x | h_prev | 1] from the gate gradients the recurrence
        // waves wrote.  Same number of barriers per step as the recurrence loop below.
        if constexpr (DW) {
            const int wt = threadIdx.x - 256, lane = wt & 63, ww = wt >> 6;
            // thread (column xc, env group xg) holds column xc of envs 8 xg .. 8 xg + 7: each
            // load instruction reads 64 consecutive columns of one row (coalesced)
            const int RL = a.I + MH + 1, nenv = min(ME, B - e0), nct = (RL + 31) / 32;
            const int xc = wt & (MXC - 1), xg = wt >> 7;
            // xr: step t's rows, xr2: step t - 1's (loaded two steps ahead)
            float xr[8], xr2[8];
            auto xload = [&](int t, float (&dst)[8]) {
                const float* src = a.xh + ((size_t)max(t, 0) * B + e0) * RL + min(xc, RL - 1);
#pragma unroll
                for (int k = 0; k < 8; ++k) dst[k] = src[(size_t)min(8 * xg + k, nenv - 1) * RL];
            };
            mfloatx16 dacc[8];
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) dacc[i][r] = 0.f;
            // columns >= RL stay 0.  Only those: columns < RL are written by the step stores below
            // from other waves, with no barrier between (a zero landing after one of them would
            // drop that column of the first step's operand)
            for (int i = wt; i < NP * 2 * MXC * ME; i += 256)
                if ((i % (MXC * ME)) / ME >= RL) (&XT[0][0][0])[i] = (mbf16)0.f;
            xload(T - 1, xr);
            xload(T - 2, xr2);
            for (int t = T - 1; t >= 0; --t) {
                const int buf = t & 1;
                if (xc < RL) {
                    mbf16x8 hi8, lo8;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        mbf16 hi, lo;
                        split_bf16(8 * xg + k < nenv ? xr[k] : 0.f, hi, lo);
                        hi8[k] = hi;
                        lo8[k] = lo;
                    }
                    *(mbf16x8*)(&XT[0][buf][xc * ME + 8 * xg]) = hi8;
                    if constexpr (NP == 2) *(mbf16x8*)(&XT[NP - 1][buf][xc * ME + 8 * xg]) = lo8;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) xr[k] = xr2[k];
                xload(t - 2, xr2);
                __syncthreads();
                // operands of the wave's 2 x 4 tiles, then the products pass by pass
                // (consecutive MFMAs on different accumulators)
                mbf16x8 ah[2], al[2], bh[4], bl[4];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    const int ao = ((2 * ww + mt) * 32 + (lane & 31)) * ME + 8 * (lane >> 5);
                    ah[mt] = *(const mbf16x8*)(&GT[0][buf][ao]);
                    if constexpr (NP == 2) al[mt] = *(const mbf16x8*)(&GT[NP - 1][buf][ao]);
                }
#pragma unroll
                for (int nt = 0; nt < MXC / 32; ++nt) {
                    const int bo = (nt * 32 + (lane & 31)) * ME + 8 * (lane >> 5);
                    bh[nt] = *(const mbf16x8*)(&XT[0][buf][bo]);
                    if constexpr (NP == 2) bl[nt] = *(const mbf16x8*)(&XT[NP - 1][buf][bo]);
                }
#pragma unroll
                for (int pass = 0; pass < (NP == 2 ? 3 : 1); ++pass)
#pragma unroll
                    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                        for (int nt = 0; nt < MXC / 32; ++nt)
                            if (nt < nct) {
                                const mbf16x8& A = pass == 2 ? al[mt] : ah[mt];
                                const mbf16x8& Bv = pass == 1 ? bl[nt] : bh[nt];
                                dacc[mt * 4 + nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, Bv, dacc[mt * 4 + nt], 0, 0, 0);
                            }
            }
            // this workgroup's partial weight gradients, torch row order
            const int I = a.I;
            float* sl = a.slab + (size_t)blockIdx.x * (size_t)MG * RL;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int nt = 0; nt < MXC / 32; ++nt) {
                    const int n = nt * 32 + (lane & 31);
                    if (nt >= nct || n >= RL) continue;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int gp = (2 * ww + mt) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);  // permuted
                        const int tr = ((gp >> 4) & 3) * MH + 16 * (gp >> 6) + (gp & 15);          // torch row
                        const float x = dacc[mt * 4 + nt][r];
                        if (n < I) sl[(size_t)tr * I + n] = x;
                        else if (n < I + MH) sl[(size_t)MG * I + (size_t)tr * MH + (n - I)] = x;
                        else sl[(size_t)MG * (I + MH) + tr] = x;
                    }
                }
        }
        return;
    }
    // ---- the recurrence waves (0..3)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int j = lane & 15, rg = lane >> 4, u = 16 * w + j;
    // B[k = permuted gate column][n = unit 16w + j] = W_hh[torch row of k][u], 8 k-steps of 32
    mbf16x8 wf[NP][8];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = s * 32 + 8 * rg + e;  // permuted column: wave kw, gate kq, unit kj
            const int kw = k >> 6, kq = (k >> 4) & 3, kj = k & 15;
            mbf16 hi, lo;
            split_bf16(a.whh[(size_t)(kq * MH + 16 * kw + kj) * MH + u], hi, lo);
            wf[0][s][e] = hi;
            if constexpr (NP == 2) wf[NP - 1][s][e] = lo;
        }
    // the step's global inputs for the lane's 4 (env, unit) pairs, loaded one step ahead
    struct In {
        float g[4][4], cv[4], cp[4], dh[4];
        uint8_t rs[4];
        bool cz;
    };
    // unconditional loads at clamped addresses (see the forward); rows past B are computed
    // and never stored, t < 0 is never used
    // (absent reset / c0 read valid memory and are masked where used; nothing here consumes
    // a loaded value, so the loads stay in flight across the step)
    const bool has_reset = a.reset != nullptr, has_c0 = a.c0 != nullptr;
    const uint8_t* rbase = has_reset ? a.reset : (const uint8_t*)a.c_out;
    auto load = [&](int t, In& v) {
        const int tt = max(t, 0);
        const float* cpb = tt > 0 ? a.c_out + (size_t)(tt - 1) * B * MH : (has_c0 ? a.c0 : a.c_out);
        v.cz = tt == 0 && !has_c0;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int gc = min(e0 + 4 * rg + p, B - 1);
            const size_t row = (size_t)tt * B + gc;
            v.rs[p] = rbase[row];
#pragma unroll
            for (int q = 0; q < 4; ++q) v.g[p][q] = a.gact[row * MG + q * MH + u];
            v.cv[p] = a.c_out[row * MH + u];
            v.cp[p] = cpb[(size_t)gc * MH + u];
            v.dh[p] = a.dh_out[row * MH + u];
        }
    };
    float dhn[4] = {0.f, 0.f, 0.f, 0.f}, dcn[4] = {0.f, 0.f, 0.f, 0.f};
    In nx, nx2;  // step t's inputs and step t - 1's, loaded two steps ahead
    load(T - 1, nx);
    load(T - 2, nx2);
    for (int t = T - 1; t >= 0; --t) {
        const int buf = t & 1;
        const In v = nx;
        nx = nx2;
        load(t - 2, nx2);
        mbf16x4 gth[4], gtl[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int ge = e0 + 4 * rg + p;
            const bool rs = has_reset && v.rs[p] != 0;
            const float cp = (rs || v.cz) ? 0.f : v.cp[p];
            const float ig = v.g[p][0], fg = v.g[p][1], gg = v.g[p][2], og = v.g[p][3];
            const float dh = v.dh[p] + dhn[p];
            const float tc = ftanh(v.cv[p]);
            const float dc = dcn[p] + dh * og * (1.f - tc * tc);
            float dg[4];
            dg[0] = dc * gg * ig * (1.f - ig);
            dg[1] = dc * cp * fg * (1.f - fg);
            dg[2] = dc * ig * (1.f - gg * gg);
            dg[3] = dh * tc * og * (1.f - og);
            dcn[p] = rs ? 0.f : dc * fg;  // into c_{t-1} (none across a reset)
            if (ge < B) {
                if (a.dgx) {
                    float* o = a.dgx + ((size_t)t * B + ge) * MG;
                    o[u] = dg[0]; o[MH + u] = dg[1]; o[2 * MH + u] = dg[2]; o[3 * MH + u] = dg[3];
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) dg[q] = 0.f;  // rows past B feed nothing
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                mbf16 hi, lo;
                split_bf16(dg[q], hi, lo);
                const int o = (4 * rg + p) * MLDG + 64 * w + 16 * q + j;
                G[0][buf][o] = hi;
                if constexpr (NP == 2) G[NP - 1][buf][o] = lo;
                if constexpr (DW) {
                    gth[q][p] = hi;
                    gtl[q][p] = lo;
                }
            }
        }
        if constexpr (DW) {  // dG^T: the lane's 4 envs of each gate column, one 8-byte run per part
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ot = (64 * w + 16 * q + j) * ME + 4 * rg;
                *(mbf16x4*)(&GT[0][buf][ot]) = gth[q];
                if constexpr (NP == 2) *(mbf16x4*)(&GT[NP - 1][buf][ot]) = gtl[q];
            }
        }
        __syncthreads();
        // dh_{t-1} = dG . W_hh for units 16w + j, envs 4 rg .. 4 rg + 3: this lane's own pairs;
        // six independent accumulator chains (k-step parity x product), summed at the end
        mfloatx4 acc[2][3];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int p = 0; p < 4; ++p) acc[m][k][p] = 0.f;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int o = j * MLDG + s * 32 + 8 * rg;
            const mbf16x8 ah = *(const mbf16x8*)(&G[0][buf][o]);
            acc[s & 1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wf[0][s], acc[s & 1][0], 0, 0, 0);
            if constexpr (NP == 2) {
                const mbf16x8 al = *(const mbf16x8*)(&G[NP - 1][buf][o]);
                acc[s & 1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wf[NP - 1][s], acc[s & 1][1], 0, 0, 0);
                acc[s & 1][2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, wf[0][s], acc[s & 1][2], 0, 0, 0);
            }
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const float d = (acc[0][0][p] + acc[1][0][p]) + ((acc[0][1][p] + acc[1][1][p]) + (acc[0][2][p] + acc[1][2][p]));
            dhn[p] = (has_reset && v.rs[p]) ? 0.f : d;
        }
    }
}

// ------------------------------------------------------------ recurrent heads --
// The MLP heads of ActorCriticRecurrent on the LSTM output (rsl_rl actor / critic:
// Linear(H, N0) -> ELU -> Linear(N0, N1)), fp32, for the fused recurrent optimizer step.
// A workgroup of 256 threads owns HR = 128 rows, two threads per row (each half of the row's
// units); the weights sit in LDS (every lane reads the same entry: broadcasts) and the row
// tiles are staged through LDS so every global access is coalesced.
//   forward:  y0 = elu(W0 h + b0) [M, N0], out = W1 y0 + b1 [M, N1]
//   backward: from dout [M, N1]: dz0 = (W1^T dout) * elu'(y0) (torch's form from the output:
//             1 for y0 > 0, else y0 + 1), dh = W0^T dz0 [M, H] (the LSTM's output gradient),
//             and per workgroup the partial sums of [dW0 | db0 | dW1 | db1] (the parameter
//             order of the Sequential's two Linears) into slab row blockIdx.x.
// LDS stays under 80 KB at H = 64 (two workgroups, 8 waves per CU).
constexpr int HR = 128, HT = 256, HN0 = 32, HN1 = 16;  // rows, threads per workgroup; max N0, N1
// the forward's rows / threads per workgroup (its split of a row never changes a result): 64 rows
// on 4 threads each fill twice the CUs at the rollout's 4,096-8,192 rows (15.6 -> 10.2 us) and
// gain 2 us at the update's 49,152 (profiles/round6/heads_fwd_tiling.txt)
#ifndef PMLP_HEADS_BWD_ROWS
#define PMLP_HEADS_BWD_ROWS 128
#endif
#ifndef PMLP_HEADS_FWD_ROWS
#define PMLP_HEADS_FWD_ROWS 64
#endif
#ifndef PMLP_HEADS_FWD_THREADS
#define PMLP_HEADS_FWD_THREADS 256
#endif

struct HeadJob {
    const float *h, *W0, *b0, *W1, *b1;
    float *y0, *out;        // forward outputs
    const float* dout;      // backward input
    float *dh, *slab;       // backward outputs
    int N0, N1;
};
struct HeadJobs {
    HeadJob j[2];
};

// Stage n consecutive floats (src[0..n), 0 < n <= U * HT) into LDS through put(i, v): every
// thread's loads are issued before any is stored (unrolled to U), unconditionally at clamped
// addresses (a load under a divergent branch gets a vmcnt(0) at the branch's end), so the
// round trips overlap instead of a load -> wait -> load chain per element.
template <int U, int NT = HT, typename F>
__device__ __forceinline__ void stage(const float* __restrict__ src, int n, F&& put) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[min((int)threadIdx.x + u * NT, n - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = threadIdx.x + u * NT;
        if (i < n) put(i, v[u]);
    }
}
// the h rows r0 .. r0 + R of [M, H] into an LDS tile of row stride LH (rows >= M zero), NT threads
template <int H, int LH, int R = HR, int NT = HT>
__device__ __forceinline__ void stage_rows(const float* __restrict__ h, int r0, int M, float* hs) {
    constexpr int U = R * H / 4 / NT;
    static_assert(U >= 1 && R * H / 4 == U * NT, "whole float4 loads per thread");
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = threadIdx.x + u * NT, r = i / (H / 4), c = (i % (H / 4)) * 4;
        v[u] = *(const float4*)(h + (size_t)min(r0 + r, M - 1) * H + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = threadIdx.x + u * NT, r = i / (H / 4), c = (i % (H / 4)) * 4;
        *(float4*)(hs + r * LH + c) = r0 + r < M ? v[u] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
// a [rows, N] row-major span (N <= 32 runtime) into an LDS tile of row stride L, zero past M
template <int UMAX, int L, int R = HR, int NT = HT>
__device__ __forceinline__ void stage_span(const float* __restrict__ src, int N, int r0, int M, float* t) {
    const int nr = min(R, M - r0);
    for (int i = threadIdx.x; i < R * N; i += NT) t[(i / N) * L + i % N] = 0.f;
    stage<UMAX, NT>(src + (size_t)r0 * N, nr * N, [&](int i, float v) { t[(i / N) * L + i % N] = v; });
}

// The same three stagings split into a load phase (registers) and a store phase (LDS), so a
// kernel issues every tile's loads before its first LDS store: one round trip for all of them
// instead of one per tile (each store phase ends a basic block the next loads cannot rise above).
template <int U, int NT>
__device__ __forceinline__ void flat_load(const float* __restrict__ src, int n, float (&v)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[min((int)threadIdx.x + u * NT, n - 1)];
}
template <int U, int NT, typename F>
__device__ __forceinline__ void flat_store(int n, const float (&v)[U], F&& put) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = threadIdx.x + u * NT;
        if (i < n) put(i, v[u]);
    }
}
template <int H, int R, int NT>
__device__ __forceinline__ void rows_load(const float* __restrict__ h, int r0, int M, float4 (&v)[R * H / 4 / NT]) {
    constexpr int U = R * H / 4 / NT;
    static_assert(U >= 1 && R * H / 4 == U * NT, "whole float4 loads per thread");
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = threadIdx.x + u * NT, r = i / (H / 4), c = (i % (H / 4)) * 4;
        v[u] = *(const float4*)(h + (size_t)min(r0 + r, M - 1) * H + c);
    }
}
template <int H, int LH, int R, int NT>
__device__ __forceinline__ void rows_store(int r0, int M, const float4 (&v)[R * H / 4 / NT], float* hs) {
#pragma unroll
    for (int u = 0; u < R * H / 4 / NT; ++u) {
        const int i = threadIdx.x + u * NT, r = i / (H / 4), c = (i % (H / 4)) * 4;
        *(float4*)(hs + r * LH + c) = r0 + r < M ? v[u] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
// stage_span's tile: UMAX * NT >= R * N, every (row, column < N) entry written once (0 past M)
template <int UMAX, int R, int NT>
__device__ __forceinline__ void span_load(const float* __restrict__ src, int N, int r0, int M, float (&v)[UMAX]) {
    const int n = min(R, M - r0) * N;
    const float* s = src + (size_t)r0 * N;
#pragma unroll
    for (int u = 0; u < UMAX; ++u) v[u] = s[min((int)threadIdx.x + u * NT, n - 1)];
}
template <int UMAX, int L, int R, int NT>
__device__ __forceinline__ void span_store(int N, int r0, int M, const float (&v)[UMAX], float* t) {
    const int n = min(R, M - r0) * N;
#pragma unroll
    for (int u = 0; u < UMAX; ++u) {
        const int i = threadIdx.x + u * NT;
        if (i < R * N) t[(i / N) * L + i % N] = i < n ? v[u] : 0.f;
    }
}

// pmlp_heads_forward_act: the rollout's pmlp_act in the heads' launch (job 0 the actor, job 1
// the critic): each actor workgroup samples its rows' actions from the mu tile still in LDS
// (act_quad: pmlp_act's arithmetic, the same bits) and writes the storage rows; the critic's
// workgroups write the values and privileged rows
struct HeadAct {
    const float *stdv, *obs, *cobs;
    int O, CO, A;
    const int64_t* draw;
    uint64_t seed;
    float *actions_out, *st_actions, *st_logp, *st_mu, *st_sigma, *st_value, *st_obs, *st_cobs;
};

// R rows per workgroup of NT threads, NT / R threads per row (each a share of the row's units;
// every unit's and output's sum runs in the same order whatever the split: bitwise one result)
// MF: y0 on the matrix cores (NT = 2 R, wave w owns rows 32w .. 32w + 31; see below)
template <int H, int R = HR, int NT = HT, bool ACT = false, bool MF = false>
__global__ __launch_bounds__(NT) void k_heads_fwd(HeadJobs jobs, int M, HeadAct ha = {}) {
    constexpr int PARTS = NT / R;
    static_assert(PARTS * R == NT && (PARTS == 2 || PARTS == 4), "2 or 4 threads per row");
    static_assert(!MF || (NT == 2 * R && R % 32 == 0 && H % 8 == 0), "MF: one 32-row tile per wave");
    const HeadJob& J = jobs.j[blockIdx.y];
    const int N0 = J.N0, N1 = J.N1, tid = threadIdx.x, r0 = blockIdx.x * R;
    const int row = tid & (R - 1), half = tid / R;
    constexpr int LH = H + 4, LY = HN0 + 1, LO = HN1 + 1;
    // h tile, then y0 + out (+ the log-density terms [R][16] with ACT)
    constexpr int HS0 = R * LH > R * (LY + LO) ? R * LH : R * (LY + LO);
    constexpr int HS = ACT && HS0 < R * (LY + LO + 16) ? R * (LY + LO + 16) : HS0;
    __shared__ __attribute__((aligned(16))) float hs[HS];
    __shared__ __attribute__((aligned(16))) float w0[HN0 * H];
    __shared__ float bb0[HN0], w1[HN1 * HN0], bb1[HN1];
    // MF: the lane's W0 operands straight into registers (W0 [N0, H] is L2-resident; from LDS at
    // a row stride of H floats every lane would read the same banks), in flight with the staging
    float4 wf[MF ? H / 8 : 1];
    if constexpr (MF) {
        const int lane = tid & 63;
        const float* wrow = J.W0 + min(lane & 31, N0 - 1) * H + 4 * (lane >> 5);  // (units past N0: discarded)
#pragma unroll
        for (int s = 0; s < H / 8; ++s) wf[s] = *(const float4*)(wrow + 8 * s);
    }
    {  // every tile's loads, then every LDS store
        constexpr int UW0 = MF ? 1 : HN0 * H / NT, UW1 = (HN1 * HN0 + NT - 1) / NT;
        float vw0[UW0], vw1[UW1];
        float4 vh[R * H / 4 / NT];
        if constexpr (!MF) flat_load<UW0, NT>(J.W0, N0 * H, vw0);
        flat_load<UW1, NT>(J.W1, N1 * N0, vw1);
        rows_load<H, R, NT>(J.h, r0, M, vh);
        const float b0v = J.b0[min(tid, N0 - 1)], b1v = J.b1[min(tid, N1 - 1)];
        if constexpr (!MF) flat_store<UW0, NT>(N0 * H, vw0, [&](int i, float v) { w0[i] = v; });
        flat_store<UW1, NT>(N1 * N0, vw1, [&](int i, float v) { w1[i] = v; });
        if (tid < N0) bb0[tid] = b0v;
        if (tid < N1) bb1[tid] = b1v;
        rows_store<H, LH, R, NT>(r0, M, vh, hs);
    }
    __syncthreads();
    if constexpr (MF) {
        // y0 on the matrix cores: wave w, rows 32w .. 32w + 31, all 32 units (one
        // v_mfma_f32_32x32x2_f32 tile; lane l: A = h[row l & 31][k], B = W0[unit l & 31][k] for
        // its k slot l >> 5).  Accumulator u takes k = u, u + 4, u + 8, ...: step s's
        // instruction holds k = u + 8s (slot 0) and u + 8s + 4 (slot 1), and an f32 MFMA is a
        // k-ordered fmaf chain -- the VALU form's four chains over k mod 4 with the bias at the
        // start of chain 0, and the same (z0 + z1) + (z2 + z3): the same bits.
        const int lane = tid & 63, w = tid >> 6, q = lane >> 5, jc = lane & 31;
        const float bj = jc < N0 ? bb0[jc] : 0.f;
        mfloatx16 acc[4];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            acc[0][r] = bj;
            acc[1][r] = acc[2][r] = acc[3][r] = 0.f;
        }
        const float* hrow = hs + (32 * w + jc) * LH + 4 * q;
#pragma unroll
        for (int s = 0; s < H / 8; ++s) {
            const float4 hv = *(const float4*)(hrow + 8 * s);
            const float4 wv = wf[s];
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(hv.x, wv.x, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(hv.y, wv.y, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(hv.z, wv.z, acc[2], 0, 0, 0);
            acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(hv.w, wv.w, acc[3], 0, 0, 0);
        }
        __syncthreads();  // every read of the h tile is done (hs takes y0)
        if (jc < N0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int rr = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * q;
                const float zz = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]);
                hs[rr * LY + jc] = zz > 0.f ? zz : expm1f(zz);
            }
        }
    } else {
        float hr[H];
#pragma unroll
        for (int k = 0; k < H; k += 4) {
            const float4 v = *(const float4*)(hs + row * LH + k);
            hr[k] = v.x; hr[k + 1] = v.y; hr[k + 2] = v.z; hr[k + 3] = v.w;
        }
        __syncthreads();  // (hs is reused for the y0 tile below)
        // y0: this thread's share of the units, one at a time (four FMA chains over k mod 4)
        const int nh = N0 / PARTS, jb = half * nh;
#pragma unroll 1
        for (int j = jb; j < jb + nh; ++j) {
            float z[4] = {bb0[j], 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H; k += 4) {
                const float4 w = *(const float4*)(w0 + j * H + k);
                z[0] = fmaf(w.x, hr[k], z[0]); z[1] = fmaf(w.y, hr[k + 1], z[1]);
                z[2] = fmaf(w.z, hr[k + 2], z[2]); z[3] = fmaf(w.w, hr[k + 3], z[3]);
            }
            const float zz = (z[0] + z[1]) + (z[2] + z[3]);
            hs[row * LY + j] = zz > 0.f ? zz : expm1f(zz);
        }
    }
    __syncthreads();
    // out: this thread's outputs i = half, half + PARTS, ... over the row's y0 (LDS)
    float* os = hs + R * LY;  // [R][LO]
#pragma unroll 1
    for (int i = half; i < N1; i += PARTS) {
        float a[4] = {bb1[i], 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int j = 0; j < N0; j += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = fmaf(w1[i * N0 + j + u], hs[row * LY + j + u], a[u]);
        }
        os[row * LO + i] = (a[0] + a[1]) + (a[2] + a[3]);
    }
    __syncthreads();
    for (int i = tid; i < R * N0; i += NT) {  // coalesced row-major stores
        const int r = i / N0, c = i - r * N0;
        if (r0 + r < M) J.y0[(size_t)(r0 + r) * N0 + c] = hs[r * LY + c];
    }
    for (int i = tid; i < R * N1; i += NT) {
        const int r = i / N1, c = i - r * N1;
        if (r0 + r < M) J.out[(size_t)(r0 + r) * N1 + c] = os[r * LO + c];
    }
    if constexpr (ACT) {
        const int nrow = min(R, M - r0);
        if (blockIdx.y == 0) {  // the actor: sampling, log-probability, the storage rows
            float* terms = hs + R * (LY + LO);  // [R][16]
            const uint32_t draw = (uint32_t)*ha.draw;
            const uint2 key = make_uint2((uint32_t)ha.seed, (uint32_t)(ha.seed >> 32));
            for (int q = tid; q < R * 4; q += NT) {
                const int rl = q >> 2, c = q & 3, k0 = 4 * c;
                if (rl >= nrow || k0 >= ha.A) continue;
                const int i = r0 + rl;
                float act[4], mu[4], sg[4], tm[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) mu[u] = k0 + u < ha.A ? os[rl * LO + k0 + u] : 0.f;
                act_quad(draw, key, (uint32_t)i, c, ha.A, ha.stdv, mu, act, sg, tm);
                const size_t o = (size_t)i * ha.A + k0;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k0 + u < ha.A) {
                        terms[rl * 16 + k0 + u] = tm[u];
                        ha.actions_out[o + u] = act[u];
                        ha.st_actions[o + u] = act[u];
                        ha.st_mu[o + u] = mu[u];
                        ha.st_sigma[o + u] = sg[u];
                    }
            }
            __syncthreads();
            if (tid < nrow) {
                float logp = 0.f;
                for (int k = 0; k < ha.A; ++k) logp += terms[tid * 16 + k];
                ha.st_logp[r0 + tid] = logp;
            }
            for (int q = tid; q < nrow * ha.O; q += NT) ha.st_obs[(size_t)r0 * ha.O + q] = ha.obs[(size_t)r0 * ha.O + q];
        } else {  // the critic: the values and the privileged rows
            if (tid < nrow) ha.st_value[r0 + tid] = os[tid * LO];
            if (ha.st_cobs)
                for (int q = tid; q < nrow * ha.CO; q += NT)
                    ha.st_cobs[(size_t)r0 * ha.CO + q] = ha.cobs[(size_t)r0 * ha.CO + q];
        }
    }
}

// R rows per workgroup of 2 R threads (the weight-gradient partial sums run over R-row halves:
// R sets the slab rows, pmlp_heads_blocks)
// MF: dW0 and dh on the matrix cores (see below)
template <int H, int R = HR, bool MF = false>
__global__ __launch_bounds__(2 * R) void k_heads_bwd(HeadJobs jobs, int M) {
    constexpr int NT = 2 * R;
    static_assert(!MF || R >= 128, "MF: dW1 on waves 0 and 1, db1 on wave 2");
    const HeadJob& J = jobs.j[blockIdx.y];
    const int N0 = J.N0, N1 = J.N1, tid = threadIdx.x, r0 = blockIdx.x * R;
    const int row = tid & (R - 1), half = tid / R;
    constexpr int LH = H + 4, LZ = HN0 + 4, LO = HN1 + 1;
    __shared__ __attribute__((aligned(16))) float hs[R * LH];   // h, then dW0 halves, then dh
    __shared__ __attribute__((aligned(16))) float zs[R * LZ];   // y0, then dz0
    __shared__ float ds[R * LO];                                 // dout
    __shared__ __attribute__((aligned(16))) float w0[HN0 * H];
    __shared__ float w1[HN1 * HN0];
    {  // every tile's loads, then every LDS store
        constexpr int UW0 = HN0 * H / NT, UW1 = (HN1 * HN0 + NT - 1) / NT;
        constexpr int UY = (R * HN0 + NT - 1) / NT, UD = (R * HN1 + NT - 1) / NT;
        float vw0[UW0], vw1[UW1], vy[UY], vd[UD];
        float4 vh[R * H / 4 / NT];
        flat_load<UW0, NT>(J.W0, N0 * H, vw0);
        flat_load<UW1, NT>(J.W1, N1 * N0, vw1);
        rows_load<H, R, NT>(J.h, r0, M, vh);
        span_load<UY, R, NT>(J.y0, N0, r0, M, vy);
        span_load<UD, R, NT>(J.dout, N1, r0, M, vd);
        flat_store<UW0, NT>(N0 * H, vw0, [&](int i, float v) { w0[i] = v; });
        flat_store<UW1, NT>(N1 * N0, vw1, [&](int i, float v) { w1[i] = v; });
        rows_store<H, LH, R, NT>(r0, M, vh, hs);
        span_store<UY, LZ, R, NT>(N0, r0, M, vy, zs);
        span_store<UD, LO, R, NT>(N1, r0, M, vd, ds);
    }
    __syncthreads();
    float* sl = J.slab + (size_t)blockIdx.x * (N0 * H + N0 + N1 * N0 + N1);
    // dW1 (+ db1) from the y0 and dout tiles, before y0 is overwritten
    if constexpr (MF) {
        // dW1 [i][j] as two v_mfma_f32_16x16x4_f32 tiles (j in 0..15, 16..31) on waves 0 and 1:
        // A[i][slot] = dout[r][i], B[slot][j] = y0[r][j], step s holding rows 4s .. 4s + 3 -- the
        // VALU form's chain over the rows in order.  db1 on wave 2 (adds, rows in order).
        const int lane = tid & 63, w = tid >> 6;
        if (w < 2) {
            mfloatx4 acc = {0.f, 0.f, 0.f, 0.f};
            const float* da = ds + (lane >> 4) * LO + (lane & 15);
            const float* yb = zs + (lane >> 4) * LZ + 16 * w + (lane & 15);
#pragma unroll 8
            for (int st = 0; st < R / 4; ++st)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(da[4 * st * LO], yb[4 * st * LZ], acc, 0, 0, 0);
            const int j = 16 * w + (lane & 15);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int i = 4 * (lane >> 4) + v;
                if (i < N1 && j < N0) sl[N0 * H + N0 + i * N0 + j] = acc[v];
            }
        } else if (w == 2 && lane < N1) {
            float b = 0.f;
#pragma unroll 8
            for (int r = 0; r < R; ++r) b += ds[r * LO + lane];
            sl[N0 * H + N0 + N1 * N0 + lane] = b;
        }
    } else {
        for (int t = tid; t < N1 * N0; t += NT) {
            const int i = t / N0, j = t - i * N0;
            float a = 0.f, b = 0.f;
#pragma unroll 8
            for (int r = 0; r < R; ++r) {
                const float d = ds[r * LO + i];
                a = fmaf(d, zs[r * LZ + j], a);
                b += d;
            }
            sl[N0 * H + N0 + t] = a;
            if (j == 0) sl[N0 * H + N0 + N1 * N0 + i] = b;
        }
    }
    // dz0 of this thread's half of the row's units (registers), W1^T dout over the rows of W1
    const int nh = N0 / 2, jb = half * nh;
    float dz[HN0 / 2];
#pragma unroll
    for (int u = 0; u < HN0 / 2; ++u) dz[u] = 0.f;
    for (int i = 0; i < N1; ++i) {
        const float di = ds[row * LO + i];
#pragma unroll
        for (int u = 0; u < HN0 / 2; ++u)
            if (u < nh) dz[u] = fmaf(w1[i * N0 + jb + u], di, dz[u]);
    }
#pragma unroll
    for (int u = 0; u < HN0 / 2; ++u) {
        if (u < nh) {
            const float y = zs[row * LZ + jb + u];
            dz[u] = y > 0.f ? dz[u] : dz[u] * (y + 1.f);
        }
    }
    __syncthreads();  // every read of the y0 tile is done
#pragma unroll
    for (int u = 0; u < HN0 / 2; ++u)
        if (u < nh) zs[row * LZ + jb + u] = dz[u];
    __syncthreads();
    if constexpr (MF) {
        // dW0 and dh as v_mfma_f32_32x32x2_f32 tiles: an f32 MFMA is a k-ordered fmaf chain, and
        // each chain below keeps the VALU form's order, so the bits are the same.
        //   dW0 [j][k], per half of the rows: A[j][slot] = dz[r][j], B[slot][k] = h[r][k], step s
        //   holding rows rb + 2s, rb + 2s + 1.  Item c = (k tile c % KT, half c / KT); wave w
        //   takes items w, w + NW, ..  The second half's tile goes through LDS and the first adds
        //   it, as db0's two halves (VALU) do.
        //   dh [row][k]: A[row][slot] = dz[row][j], B[slot][k] = W0[j][k], step s holding
        //   j = 2s, 2s + 1 (j < N0).
        constexpr int KT = H / 32, NW = NT / 64, NI = 2 * KT, IPW = (NI + NW - 1) / NW;
        constexpr int DT = (R / 32) * KT, DPW = (DT + NW - 1) / NW;
        static_assert(H % 32 == 0 && R % 64 == 0, "MF: 32 x 32 tiles, two row halves of whole steps");
        static_assert(KT * 1024 + HN0 <= R * LH, "the second halves' partials fit the h tile");
        const int lane = tid & 63, w = tid >> 6, q = lane >> 5, l32 = lane & 31;
        mfloatx16 dw[IPW];
#pragma unroll
        for (int it = 0; it < IPW; ++it) {
            const int c = w + it * NW;
#pragma unroll
            for (int r = 0; r < 16; ++r) dw[it][r] = 0.f;
            if (c < NI) {  // (wave-uniform)
                const int kt = c % KT, rb = (c / KT) * (R / 2);
                const float* za = zs + (rb + q) * LZ + l32;
                const float* hb = hs + (rb + q) * LH + 32 * kt + l32;
#pragma unroll 8
                for (int st = 0; st < R / 4; ++st)
                    dw[it] = __builtin_amdgcn_mfma_f32_32x32x2f32(za[2 * st * LZ], hb[2 * st * LH], dw[it], 0, 0, 0);
            }
        }
        float bsum = 0.f;  // db0: thread (unit row, half) over its half's rows in order
        if (row < N0) {
            const float* zr = zs + half * (R / 2) * LZ + row;
#pragma unroll 8
            for (int r = 0; r < R / 2; ++r) bsum += zr[r * LZ];
        }
        // dh: every operand is in LDS already (dz tile, W0)
        mfloatx16 dha[DPW];
#pragma unroll
        for (int it = 0; it < DPW; ++it) {
            const int c = w + it * NW;
#pragma unroll
            for (int r = 0; r < 16; ++r) dha[it][r] = 0.f;
            if (c < DT) {
                const int rt = c / KT, kt = c % KT;
                const float* za = zs + (32 * rt + l32) * LZ + q;
                const float* wb = w0 + q * H + 32 * kt + l32;
                for (int s4 = 0; s4 < N0 / 2; s4 += 4)  // (N0 % 8 == 0)
#pragma unroll
                    for (int st = s4; st < s4 + 4; ++st)
                        dha[it] = __builtin_amdgcn_mfma_f32_32x32x2f32(za[2 * st], wb[2 * st * H], dha[it], 0, 0, 0);
            }
        }
        __syncthreads();  // every read of the h tile is done: it takes the second halves
        float* part = hs;  // [KT][16][64] tiles in register order, then db0's second half [HN0]
#pragma unroll
        for (int it = 0; it < IPW; ++it) {
            const int c = w + it * NW;
            if (c < NI && c / KT == 1)
#pragma unroll
                for (int r = 0; r < 16; ++r) part[(c % KT) * 1024 + r * 64 + lane] = dw[it][r];
        }
        if (row < N0 && half == 1) part[KT * 1024 + row] = bsum;
        __syncthreads();
#pragma unroll
        for (int it = 0; it < IPW; ++it) {
            const int c = w + it * NW;
            if (c < NI && c / KT == 0) {
                const int kt = c % KT;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int j = (r & 3) + 8 * (r >> 2) + 4 * q;
                    const float a = dw[it][r] + part[kt * 1024 + r * 64 + lane];
                    if (j < N0) sl[(size_t)j * H + 32 * kt + l32] = a;
                }
            }
        }
        if (row < N0 && half == 0) sl[N0 * H + row] = bsum + part[KT * 1024 + row];
        __syncthreads();  // every read of the partials is done: the h tile takes dh (then
        // 16-byte coalesced stores; straight from the accumulators was slower, 41.1 vs 39.1 us)
#pragma unroll
        for (int it = 0; it < DPW; ++it) {
            const int c = w + it * NW;
            if (c < DT) {
                const int rt = c / KT, kt = c % KT;
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    hs[(32 * rt + (r & 3) + 8 * (r >> 2) + 4 * q) * LH + 32 * kt + l32] = dha[it][r];
            }
        }
    } else {
        // dW0 (+ db0 on k0 = 0): 4 x 4 tiles, each over one half of the rows; the second half's
        // partial goes through LDS (over the h tile) and the first adds it (fixed order)
        const int ntile = (N0 / 4) * (H / 4);  // one tile per thread pair and pass
        float* part = hs;  // [R][20]: the h tile, after its last read (dh overwrites it later)
        static_assert(R * 20 <= R * LH, "dW0 partials fit the h tile");
        for (int tb = 0; tb < ntile; tb += R) {
            float a[4][4] = {}, bs[4] = {};
            const int t = tb + row, j0 = 4 * (t / (H / 4)), k0 = 4 * (t % (H / 4));
            if (t < ntile) {
                const int rb = half * (R / 2);
    #pragma unroll 4
                for (int r = rb; r < rb + R / 2; ++r) {
                    const float4 z4 = *(const float4*)(zs + r * LZ + j0);
                    const float4 h4 = *(const float4*)(hs + r * LH + k0);
                    const float zz[4] = {z4.x, z4.y, z4.z, z4.w}, hh[4] = {h4.x, h4.y, h4.z, h4.w};
    #pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        bs[u] += zz[u];
    #pragma unroll
                        for (int v = 0; v < 4; ++v) a[u][v] = fmaf(zz[u], hh[v], a[u][v]);
                    }
                }
            }
            __syncthreads();  // every read of the h tile in this pass is done
            if (half == 1 && t < ntile) {
    #pragma unroll
                for (int u = 0; u < 4; ++u) {
    #pragma unroll
                    for (int v = 0; v < 4; ++v) part[row * 20 + 4 * u + v] = a[u][v];
                    part[row * 20 + 16 + u] = bs[u];
                }
            }
            __syncthreads();
            if (half == 0 && t < ntile) {
    #pragma unroll
                for (int u = 0; u < 4; ++u) {
    #pragma unroll
                    for (int v = 0; v < 4; ++v) a[u][v] += part[row * 20 + 4 * u + v];
                    bs[u] += part[row * 20 + 16 + u];
                    *(float4*)(sl + (size_t)(j0 + u) * H + k0) = make_float4(a[u][0], a[u][1], a[u][2], a[u][3]);
                }
                if (k0 == 0)
    #pragma unroll
                    for (int u = 0; u < 4; ++u) sl[N0 * H + j0 + u] = bs[u];
            }
            if (tb + R < ntile) {  // the next pass reads the h tile again: restage it
                __syncthreads();
                stage_rows<H, LH, R, NT>(J.h, r0, M, hs);
                __syncthreads();
            }
        }
        // dh: this thread's half of the row's H entries, over all N0 units (dz0 from the tile)
        {
            constexpr int HH = H / 2;
            const int kb = half * HH;
            float dh[HH];
    #pragma unroll
            for (int k = 0; k < HH; ++k) dh[k] = 0.f;
    #pragma unroll 1
            for (int j = 0; j < N0; ++j) {
                const float zj = zs[row * LZ + j];
    #pragma unroll
                for (int k = 0; k < HH; k += 4) {
                    const float4 w = *(const float4*)(w0 + j * H + kb + k);
                    dh[k] = fmaf(w.x, zj, dh[k]); dh[k + 1] = fmaf(w.y, zj, dh[k + 1]);
                    dh[k + 2] = fmaf(w.z, zj, dh[k + 2]); dh[k + 3] = fmaf(w.w, zj, dh[k + 3]);
                }
            }
            __syncthreads();  // every read of the h tile is done: it takes dh
    #pragma unroll
            for (int k = 0; k < HH; k += 4)
                *(float4*)(hs + row * LH + kb + k) = make_float4(dh[k], dh[k + 1], dh[k + 2], dh[k + 3]);
        }
    }
    __syncthreads();
    for (int i = tid; i < R * (H / 4); i += NT) {
        const int r = i / (H / 4), c = (i % (H / 4)) * 4;
        if (r0 + r < M) *(float4*)(J.dh + (size_t)(r0 + r) * H + c) = *(const float4*)(hs + r * LH + c);
    }
}

thread_local std::string g_err;

int fail(const std::string& m) {
    g_err = m;
    return -1;
}

template <int H, int IP>
int fwd_launch(const FwdArgs& a, hipStream_t s) {
    if ((a.B + EB_MAX - 1) / EB_MAX >= 512)
        hipLaunchKernelGGL((k_lstm_fwd<H, EB_MAX, IP>), dim3((a.B + EB_MAX - 1) / EB_MAX), dim3(4 * H), 0, s, a);
    else
        hipLaunchKernelGGL((k_lstm_fwd<H, 4, IP>), dim3((a.B + 3) / 4), dim3(4 * H), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_fwd: ") + hipGetErrorString(e));
}

template <int H>
int fwd_h(const FwdArgs& a, hipStream_t s) {
    if (!a.x) return fwd_launch<H, 0>(a, s);
    if (a.I <= 32) return fwd_launch<H, 32>(a, s);
    if (a.I <= 48) return fwd_launch<H, 48>(a, s);
    return fwd_launch<H, 64>(a, s);
}

template <int H>
int bwd_h(int T, int B, const float* whh, const float* c0, const uint8_t* reset, const float* c_out,
          const float* gact, const float* dh_out, float* dgx, hipStream_t s) {
    if ((B + EB_MAX - 1) / EB_MAX >= 512)
        hipLaunchKernelGGL((k_lstm_bwd<H, EB_MAX>), dim3((B + EB_MAX - 1) / EB_MAX), dim3(4 * H), 0, s, T, B, whh, c0,
                           reset, c_out, gact, dh_out, dgx);
    else
        hipLaunchKernelGGL((k_lstm_bwd<H, 4>), dim3((B + 3) / 4), dim3(4 * H), 0, s, T, B, whh, c0, reset, c_out, gact,
                           dh_out, dgx);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_bwd: ") + hipGetErrorString(e));
}

}  // namespace

PMLP_API const char* pmlp_lstm_last_error(void) { return g_err.c_str(); }

PMLP_API int pmlp_lstm_supported(int32_t hidden) { return hidden == 32 || hidden == 64 || hidden == 128; }

static int fwd_dispatch(const FwdArgs& a, int H, hipStream_t s) {
    switch (H) {
    case 32: return fwd_h<32>(a, s);
    case 64: return fwd_h<64>(a, s);
    case 128: return fwd_h<128>(a, s);
    default: return fail("pmlp_lstm_fwd: hidden size must be 32, 64 or 128");
    }
}

PMLP_API int pmlp_lstm_fwd(int32_t T, int32_t B, int32_t H, const float* gx, const float* whh, const float* h0,
                           const float* c0, const uint8_t* reset, float* h_out, float* c_out, float* gact,
                           float* h_last, float* c_last, void* stream) {
    if (T <= 0 || B <= 0 || !gx || !whh) return fail("pmlp_lstm_fwd: empty sequence or null gx/whh");
    if (((uintptr_t)whh & 15u) != 0) return fail("pmlp_lstm_fwd: whh must be 16-byte aligned");
    FwdArgs a{T, B, 0, gx, nullptr, nullptr, nullptr, nullptr, whh, h0, c0, reset, h_out, c_out, gact,
              h_last, c_last, nullptr, nullptr, nullptr};
    return fwd_dispatch(a, H, (hipStream_t)stream);
}

PMLP_API int pmlp_lstm_step(int32_t B, int32_t H, const float* gx, const float* whh, float* h, float* c,
                            float* h_save, float* c_save, void* stream) {
    if (B <= 0 || !gx || !whh || !h || !c) return fail("pmlp_lstm_step: empty batch or null gx/whh/h/c");
    if (((uintptr_t)whh & 15u) != 0) return fail("pmlp_lstm_step: whh must be 16-byte aligned");
    FwdArgs a{1, B, 0, gx, nullptr, nullptr, nullptr, nullptr, whh, h, c, nullptr, nullptr, nullptr, nullptr,
              h, c, nullptr, h_save, c_save};
    return fwd_dispatch(a, H, (hipStream_t)stream);
}

PMLP_API int pmlp_lstm_fwd_x(int32_t T, int32_t B, int32_t H, int32_t I, const float* x, const float* wih,
                             const float* bih, const float* bhh, const float* whh, const float* h0, const float* c0,
                             const uint8_t* reset, float* h_out, float* c_out, float* gact, float* h_last,
                             float* c_last, float* xh, void* stream) {
    if (T <= 0 || B <= 0 || !x || !wih || !whh) return fail("pmlp_lstm_fwd_x: empty sequence or null x/wih/whh");
    if (I <= 0 || I > 64) return fail("pmlp_lstm_fwd_x: input size must be 1..64");
    if (((uintptr_t)whh & 15u) != 0) return fail("pmlp_lstm_fwd_x: whh must be 16-byte aligned");
    FwdArgs a{T, B, I, nullptr, x, wih, bih, bhh, whh, h0, c0, reset, h_out, c_out, gact, h_last, c_last, xh,
              nullptr, nullptr};
    return fwd_dispatch(a, H, (hipStream_t)stream);
}

PMLP_API int pmlp_lstm_bwd(int32_t T, int32_t B, int32_t H, const float* whh, const float* c0, const uint8_t* reset,
                           const float* c_out, const float* gact, const float* dh_out, float* dgx, void* stream) {
    if (T <= 0 || B <= 0 || !whh || !c_out || !gact || !dh_out || !dgx)
        return fail("pmlp_lstm_bwd: empty sequence or null buffer");
    hipStream_t s = (hipStream_t)stream;
    switch (H) {
    case 32: return bwd_h<32>(T, B, whh, c0, reset, c_out, gact, dh_out, dgx, s);
    case 64: return bwd_h<64>(T, B, whh, c0, reset, c_out, gact, dh_out, dgx, s);
    case 128: return bwd_h<128>(T, B, whh, c0, reset, c_out, gact, dh_out, dgx, s);
    default: return fail("pmlp_lstm_bwd: hidden size must be 32, 64 or 128");
    }
}

// 16-env tiles per workgroup of a single step (the rollout's): PMLP_LSTM_STEP_TILES overrides
static int step_tiles(int B) {
    static const int env = [] {
        const char* v = std::getenv("PMLP_LSTM_STEP_TILES");
        return v ? std::atoi(v) : 0;
    }();
    if (env > 0) return env;
    // 128 workgroups per memory (2,048 envs a tile-row): the H1 x 8192 rollout 9.95 -> 9.59 ms at
    // 4 tiles, G1 x 4096 6.06 -> 5.93 ms at 2 (profiles/round6/lstm_step_tiles.txt)
    return std::max(1, std::min(4, B / 2048));
}

PMLP_API int pmlp_lstm_fwd_mfma(int32_t T, int32_t B, int32_t H, int32_t I, const float* x, const float* wih,
                                const float* bih, const float* bhh, const float* whh, const float* h0, const float* c0,
                                const uint8_t* reset, float* h_out, float* c_out, float* gact, float* xh, void* stream) {
    if (T <= 0 || B <= 0 || !x || !wih || !bih || !bhh || !whh) return fail("pmlp_lstm_fwd_mfma: empty sequence or null input");
    if (H != MH || I <= 0 || I > MKX) return fail("pmlp_lstm_fwd_mfma: hidden 64, input 1..64");
    MFwdBatch a{};
    a.m[0] = MFwdArgs{T, B, I, x, wih, bih, bhh, whh, h0, c0, reset, h_out, c_out, gact, xh, nullptr, nullptr};
    hipLaunchKernelGGL(k_lstm_fwd_mfma8<3>, dim3((B + ME - 1) / ME), dim3(512), 0, (hipStream_t)stream, a, 1);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_fwd_mfma: ") + hipGetErrorString(e));
}

PMLP_API int pmlp_lstm_bwd_mfma(int32_t T, int32_t B, int32_t H, const float* whh, const float* c0,
                                const uint8_t* reset, const float* c_out, const float* gact, const float* dh_out,
                                float* dgx, void* stream) {
    if (T <= 0 || B <= 0 || !whh || !c_out || !gact || !dh_out || !dgx) return fail("pmlp_lstm_bwd_mfma: null buffer");
    if (H != MH) return fail("pmlp_lstm_bwd_mfma: hidden 64");
    MBwdBatch a{};
    a.m[0] = MBwdArgs{T, B, whh, c0, reset, c_out, gact, dh_out, dgx, nullptr, 0, nullptr};
    hipLaunchKernelGGL((k_lstm_bwd_mfma<3, false>), dim3((B + ME - 1) / ME), dim3(256), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_bwd_mfma: ") + hipGetErrorString(e));
}

PMLP_API int32_t pmlp_lstm_bwd_dw_blocks(int32_t B) { return (B + ME - 1) / ME; }

PMLP_API int pmlp_lstm_bwd_dw_mfma(int32_t T, int32_t B, int32_t H, int32_t I, const float* whh, const float* c0,
                                   const uint8_t* reset, const float* c_out, const float* gact, const float* dh_out,
                                   const float* xh, float* slab, void* stream) {
    if (T <= 0 || B <= 0 || !whh || !c_out || !gact || !dh_out || !xh || !slab)
        return fail("pmlp_lstm_bwd_dw_mfma: null buffer");
    if (H != MH || I <= 0 || I + MH + 1 > MXC) return fail("pmlp_lstm_bwd_dw_mfma: hidden 64, I + 65 <= 128");
    MBwdBatch a{};
    a.m[0] = MBwdArgs{T, B, whh, c0, reset, c_out, gact, dh_out, nullptr, xh, I, slab};
    hipLaunchKernelGGL((k_lstm_bwd_mfma<3, true>), dim3((B + ME - 1) / ME), dim3(512), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_bwd_dw_mfma: ") + hipGetErrorString(e));
}

/* The recurrent policy's MLP heads (include/ppo_mlp.h, "recurrent heads"). */
static int heads_check(const char* w, int njobs, const pmlp_head_job* jobs, int M, int H, bool bwd) {
    if (njobs < 1 || njobs > 2 || !jobs || M <= 0) return fail(std::string(w) + ": 1..2 jobs, M > 0");
    if (H != 32 && H != 64 && H != 128) return fail(std::string(w) + ": H must be 32, 64 or 128");
    for (int i = 0; i < njobs; ++i) {
        const pmlp_head_job& J = jobs[i];
        if (J.N0 <= 0 || J.N0 > HN0 || J.N0 % 8 || J.N1 <= 0 || J.N1 > HN1)
            return fail(std::string(w) + ": 0 < N0 <= 32 (a multiple of 8), 0 < N1 <= 16");
        if (!J.h || !J.W0 || !J.W1 || ((uintptr_t)J.h & 15u) || ((uintptr_t)J.W0 & 15u))
            return fail(std::string(w) + ": null or unaligned h / W0 / W1");
        if (!bwd && (!J.b0 || !J.b1 || !J.y0 || !J.out)) return fail(std::string(w) + ": null b0 / b1 / y0 / out");
        if (bwd && (!J.y0 || !J.dout || !J.dh || !J.slab || ((uintptr_t)J.dh & 15u) || ((uintptr_t)J.slab & 15u)))
            return fail(std::string(w) + ": null or unaligned y0 / dout / dh / slab");
    }
    return 0;
}

static HeadJobs heads_pack(int njobs, const pmlp_head_job* jobs) {
    HeadJobs hj{};
    for (int i = 0; i < njobs; ++i) {
        const pmlp_head_job& J = jobs[i];
        hj.j[i] = HeadJob{J.h, J.W0, J.b0, J.W1, J.b1, J.y0, J.out, J.dout, J.dh, J.slab, J.N0, J.N1};
    }
    return hj;
}

PMLP_API int32_t pmlp_heads_blocks(int32_t M) { return (M + PMLP_HEADS_BWD_ROWS - 1) / PMLP_HEADS_BWD_ROWS; }

// the heads' products on the matrix cores (k_heads_fwd<.., MF>: y0, 64 rows x 128 threads;
// k_heads_bwd<.., MF>: dW0 and dh), the same bits as the VALU forms; PMLP_HEADS_MFMA=0 keeps the
// VALU forms (the forward at PMLP_HEADS_FWD_ROWS x _THREADS)
static bool heads_mfma() {
    static const bool on = [] {
        const char* e = getenv("PMLP_HEADS_MFMA");
        return !(e && e[0] == '0');
    }();
    return on;
}
constexpr int HFR_MF = 64, HFT_MF = 128;
// below this many rows the forward keeps the VALU form: at the rollout's 8,192 its 64-row x
// 256-thread workgroups fill the CUs better (10.2 against 11.2 us; the same bits either way)
constexpr int HF_MF_MIN_ROWS = 16384;

template <int H, bool ACT>
static void heads_fwd_launch(int njobs, const HeadJobs& hj, int M, const HeadAct& ha, hipStream_t s) {
    constexpr int FR = PMLP_HEADS_FWD_ROWS, FT = PMLP_HEADS_FWD_THREADS;
    if (heads_mfma() && M >= HF_MF_MIN_ROWS)
        hipLaunchKernelGGL((k_heads_fwd<H, HFR_MF, HFT_MF, ACT, true>), dim3((M + HFR_MF - 1) / HFR_MF, njobs),
                           dim3(HFT_MF), 0, s, hj, M, ha);
    else
        hipLaunchKernelGGL((k_heads_fwd<H, FR, FT, ACT>), dim3((M + FR - 1) / FR, njobs), dim3(FT), 0, s, hj, M, ha);
}

PMLP_API int pmlp_heads_forward(int32_t njobs, const pmlp_head_job* jobs, int32_t M, int32_t H, void* stream) {
    if (int e = heads_check("pmlp_heads_forward", njobs, jobs, M, H, false)) return e;
    const HeadJobs hj = heads_pack(njobs, jobs);
    hipStream_t s = (hipStream_t)stream;
    if (H == 32) heads_fwd_launch<32, false>(njobs, hj, M, HeadAct{}, s);
    else if (H == 64) heads_fwd_launch<64, false>(njobs, hj, M, HeadAct{}, s);
    else heads_fwd_launch<128, false>(njobs, hj, M, HeadAct{}, s);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_heads_forward: ") + hipGetErrorString(e));
}

PMLP_API int pmlp_heads_forward_act(const pmlp_head_job* jobs, int32_t M, int32_t H, const pmlp_head_act* act,
                                    void* stream) {
    if (int e = heads_check("pmlp_heads_forward_act", 2, jobs, M, H, false)) return e;
    if (!act || !act->stdv || !act->obs || !act->draw || !act->actions_out || !act->st_actions || !act->st_logp ||
        !act->st_mu || !act->st_sigma || !act->st_value || !act->st_obs || act->O <= 0 || act->A <= 0 ||
        act->A > 16 || act->A != jobs[0].N1 || jobs[1].N1 != 1 || (act->st_cobs && (!act->cobs || act->CO <= 0)))
        return fail("pmlp_heads_forward_act: null buffer, A != the actor's N1 (<= 16) or a critic N1 != 1");
    const HeadJobs hj = heads_pack(2, jobs);
    const HeadAct ha{act->stdv, act->obs, act->cobs, act->O, act->CO, act->A, act->draw, act->seed,
                     act->actions_out, act->st_actions, act->st_logp, act->st_mu, act->st_sigma, act->st_value,
                     act->st_obs, act->st_cobs};
    hipStream_t s = (hipStream_t)stream;
    if (H == 32) heads_fwd_launch<32, true>(2, hj, M, ha, s);
    else if (H == 64) heads_fwd_launch<64, true>(2, hj, M, ha, s);
    else heads_fwd_launch<128, true>(2, hj, M, ha, s);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_heads_forward_act: ") + hipGetErrorString(e));
}

PMLP_API int pmlp_heads_backward(int32_t njobs, const pmlp_head_job* jobs, int32_t M, int32_t H, void* stream) {
    if (int e = heads_check("pmlp_heads_backward", njobs, jobs, M, H, true)) return e;
    const HeadJobs hj = heads_pack(njobs, jobs);
    constexpr int BR = PMLP_HEADS_BWD_ROWS;
    const dim3 g((M + BR - 1) / BR, njobs);
    hipStream_t s = (hipStream_t)stream;
    const bool mf = heads_mfma();
    if (H == 32) hipLaunchKernelGGL(mf ? (k_heads_bwd<32, BR, true>) : (k_heads_bwd<32, BR>), g, dim3(2 * BR), 0, s, hj, M);
    else if (H == 64) hipLaunchKernelGGL(mf ? (k_heads_bwd<64, BR, true>) : (k_heads_bwd<64, BR>), g, dim3(2 * BR), 0, s, hj, M);
    else hipLaunchKernelGGL(mf ? (k_heads_bwd<128, BR, true>) : (k_heads_bwd<128, BR>), g, dim3(2 * BR), 0, s, hj, M);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_heads_backward: ") + hipGetErrorString(e));
}

/* One rollout step of a hidden-64 memory on the matrix cores (the 8-wave sequence kernel at
 * T = 1, the arithmetic of the update's pmlp_lstm_fwd_mfma): h, c [B, 64] are read and
 * overwritten in place (each (env, unit) by the lane that reads it), the input projection
 * is inside, and the state the step starts from goes to h_save / c_save when given. */
PMLP_API int pmlp_lstm_step_mfma(int32_t B, int32_t H, int32_t I, const float* x, const float* wih, const float* bih,
                                 const float* bhh, const float* whh, float* h, float* c, float* h_save, float* c_save,
                                 void* stream) {
    if (B <= 0 || !x || !wih || !bih || !bhh || !whh || !h || !c) return fail("pmlp_lstm_step_mfma: null input");
    if (H != MH || I <= 0 || I > MKX) return fail("pmlp_lstm_step_mfma: hidden 64, input 1..64");
    if ((h_save == nullptr) != (c_save == nullptr)) return fail("pmlp_lstm_step_mfma: h_save and c_save together");
    MFwdBatch a{};
    a.m[0] = MFwdArgs{1, B, I, x, wih, bih, bhh, whh, h, c, nullptr, h, c, nullptr, nullptr, h_save, c_save};
    const int nt = step_tiles(B);
    hipLaunchKernelGGL(k_lstm_fwd_mfma8<3>, dim3((B + ME * nt - 1) / (ME * nt)), dim3(512), 0, (hipStream_t)stream, a, nt);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_step_mfma: ") + hipGetErrorString(e));
}

/* Both memories of the fused recurrent step in one launch each way (include/ppo_mlp.h,
 * pmlp_lstm_job): the same kernels and arithmetic as pmlp_lstm_fwd_mfma /
 * pmlp_lstm_bwd_dw_mfma per job, the jobs side by side in the grid's y. */
static int lstm_jobs_check(const char* w, int njobs, const pmlp_lstm_job* jobs, int T, int B, int H, bool bwd) {
    if (njobs < 1 || njobs > 2 || !jobs || T <= 0 || B <= 0) return fail(std::string(w) + ": 1..2 jobs, T, B > 0");
    if (H != MH) return fail(std::string(w) + ": hidden 64");
    for (int i = 0; i < njobs; ++i) {
        const pmlp_lstm_job& J = jobs[i];
        if (J.I <= 0 || J.I > MKX || J.I + MH + 1 > MXC) return fail(std::string(w) + ": input 1..63");
        if (!J.w_hh || !J.c_out || !J.gact || !J.xh) return fail(std::string(w) + ": null w_hh / c_out / gact / xh");
        if (!bwd && (!J.x || !J.w_ih || !J.b_ih || !J.b_hh || !J.h_out)) return fail(std::string(w) + ": null forward input");
        if (bwd && (!J.dh_out || !J.slab)) return fail(std::string(w) + ": null dh_out / slab");
    }
    return 0;
}

PMLP_API int pmlp_lstm_fwd_mfma_jobs(int32_t njobs, const pmlp_lstm_job* jobs, int32_t T, int32_t B, int32_t H,
                                     const uint8_t* reset, void* stream) {
    if (int e = lstm_jobs_check("pmlp_lstm_fwd_mfma_jobs", njobs, jobs, T, B, H, false)) return e;
    MFwdBatch a{};
    for (int i = 0; i < njobs; ++i) {
        const pmlp_lstm_job& J = jobs[i];
        a.m[i] = MFwdArgs{T, B, J.I, J.x, J.w_ih, J.b_ih, J.b_hh, J.w_hh, J.h0, J.c0, reset,
                          J.h_out, J.c_out, J.gact, J.xh, nullptr, nullptr};
    }
    hipLaunchKernelGGL(k_lstm_fwd_mfma8<3>, dim3((B + ME - 1) / ME, njobs), dim3(512), 0, (hipStream_t)stream, a, 1);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_fwd_mfma_jobs: ") + hipGetErrorString(e));
}

PMLP_API int pmlp_lstm_bwd_dw_mfma_jobs(int32_t njobs, const pmlp_lstm_job* jobs, int32_t T, int32_t B, int32_t H,
                                        const uint8_t* reset, void* stream) {
    if (int e = lstm_jobs_check("pmlp_lstm_bwd_dw_mfma_jobs", njobs, jobs, T, B, H, true)) return e;
    MBwdBatch a{};
    for (int i = 0; i < njobs; ++i) {
        const pmlp_lstm_job& J = jobs[i];
        a.m[i] = MBwdArgs{T, B, J.w_hh, J.c0, reset, J.c_out, J.gact, J.dh_out, nullptr, J.xh, J.I, J.slab};
    }
    hipLaunchKernelGGL((k_lstm_bwd_mfma<3, true>), dim3((B + ME - 1) / ME, njobs), dim3(512), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_bwd_dw_mfma_jobs: ") + hipGetErrorString(e));
}

PMLP_API int pmlp_lstm_step_mfma_jobs(int32_t njobs, const pmlp_lstm_job* jobs, int32_t B, int32_t H, void* stream) {
    if (njobs < 1 || njobs > 2 || !jobs || B <= 0) return fail("pmlp_lstm_step_mfma_jobs: 1..2 jobs, B > 0");
    if (H != MH) return fail("pmlp_lstm_step_mfma_jobs: hidden 64");
    MFwdBatch a{};
    for (int i = 0; i < njobs; ++i) {
        const pmlp_lstm_job& J = jobs[i];
        if (J.I <= 0 || J.I > MKX || !J.x || !J.w_ih || !J.b_ih || !J.b_hh || !J.w_hh || !J.h_out || !J.c_out ||
            (J.h_save == nullptr) != (J.c_save == nullptr))
            return fail("pmlp_lstm_step_mfma_jobs: input 1..64, null input / state, h_save and c_save together");
        a.m[i] = MFwdArgs{1, B, J.I, J.x, J.w_ih, J.b_ih, J.b_hh, J.w_hh, J.h_out, J.c_out, nullptr,
                          J.h_out, J.c_out, nullptr, nullptr, J.h_save, J.c_save};
    }
    const int nt = step_tiles(B);
    hipLaunchKernelGGL(k_lstm_fwd_mfma8<3>, dim3((B + ME * nt - 1) / (ME * nt), njobs), dim3(512), 0, (hipStream_t)stream, a, nt);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_step_mfma_jobs: ") + hipGetErrorString(e));
}
