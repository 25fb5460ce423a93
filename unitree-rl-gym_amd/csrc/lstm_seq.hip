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

#include <cstdint>
#include <string>

#include "../../include/ppo_mlp.h"

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
