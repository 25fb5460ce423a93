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

constexpr int EB = 8;  // envs per workgroup

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// forward over T steps: gact [T,B,4H] (activated gates), c_out [T,B,H], h_out [T,B,H];
// each of gact / c_out / h_out / h_last / c_last may be null
template <int H>
__global__ __launch_bounds__(4 * H) void k_lstm_fwd(int T, int B, const float* __restrict__ gx,
                                                    const float* __restrict__ whh, const float* __restrict__ h0,
                                                    const float* __restrict__ c0, const uint8_t* __restrict__ reset,
                                                    float* __restrict__ h_out, float* __restrict__ c_out,
                                                    float* __restrict__ gact, float* h_last, float* c_last) {
    constexpr int G = 4 * H;
    __shared__ __attribute__((aligned(16))) float hs[EB][H];
    __shared__ float cs[EB][H];
    __shared__ float ga[EB][G];
    const int j = threadIdx.x;
    const int e0 = blockIdx.x * EB;
    float w[H];
#pragma unroll
    for (int k = 0; k < H; k += 4) {
        const float4 v = *reinterpret_cast<const float4*>(whh + (size_t)j * H + k);
        w[k] = v.x; w[k + 1] = v.y; w[k + 2] = v.z; w[k + 3] = v.w;
    }
    for (int i = j; i < EB * H; i += G) {
        const int e = i / H, k = i % H, ge = e0 + e;
        hs[e][k] = (ge < B && h0) ? h0[(size_t)ge * H + k] : 0.f;
        cs[e][k] = (ge < B && c0) ? c0[(size_t)ge * H + k] : 0.f;
    }
    __syncthreads();
    const int kind = j / H;  // 0 i, 1 f, 2 g (tanh), 3 o
    for (int t = 0; t < T; ++t) {
        if (reset) {
            for (int i = j; i < EB * H; i += G) {
                const int e = i / H, k = i % H, ge = e0 + e;
                if (ge < B && reset[(size_t)t * B + ge]) { hs[e][k] = 0.f; cs[e][k] = 0.f; }
            }
            __syncthreads();
        }
#pragma unroll 2
        for (int e = 0; e < EB; ++e) {
            const int ge = e0 + e;
            if (ge >= B) break;
            const size_t row = (size_t)t * B + ge;
            float acc = gx[row * G + j];
            const float4* h4 = reinterpret_cast<const float4*>(hs[e]);
#pragma unroll
            for (int k = 0; k < H / 4; ++k) {
                const float4 hv = h4[k];
                acc = fmaf(hv.x, w[4 * k], acc);
                acc = fmaf(hv.y, w[4 * k + 1], acc);
                acc = fmaf(hv.z, w[4 * k + 2], acc);
                acc = fmaf(hv.w, w[4 * k + 3], acc);
            }
            const float a = kind == 2 ? tanhf(acc) : sigm(acc);
            ga[e][j] = a;
            if (gact) gact[row * G + j] = a;
        }
        __syncthreads();
        for (int i = j; i < EB * H; i += G) {
            const int e = i / H, k = i % H, ge = e0 + e;
            if (ge >= B) continue;
            const float ig = ga[e][k], fg = ga[e][H + k], gg = ga[e][2 * H + k], og = ga[e][3 * H + k];
            const float c = fg * cs[e][k] + ig * gg;
            const float h = og * tanhf(c);
            cs[e][k] = c;
            hs[e][k] = h;
            const size_t o = ((size_t)t * B + ge) * H + k;
            if (h_out) h_out[o] = h;
            if (c_out) c_out[o] = c;
        }
        __syncthreads();
    }
    for (int i = j; i < EB * H; i += G) {
        const int e = i / H, k = i % H, ge = e0 + e;
        if (ge >= B) continue;
        if (h_last) h_last[(size_t)ge * H + k] = hs[e][k];
        if (c_last) c_last[(size_t)ge * H + k] = cs[e][k];
    }
}

// backward through time: dh_out [T,B,H] -> dgx [T,B,4H] (gradient of the gate
// pre-activations, i.e. of gx and of the biases).  No gradient flows into h0/c0 or
// across a reset (the state was replaced by zeros there).
template <int H>
__global__ __launch_bounds__(4 * H) void k_lstm_bwd(int T, int B, const float* __restrict__ whh,
                                                    const float* __restrict__ c0, const uint8_t* __restrict__ reset,
                                                    const float* __restrict__ c_out, const float* __restrict__ gact,
                                                    const float* __restrict__ dh_out, float* __restrict__ dgx) {
    constexpr int G = 4 * H;
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
    for (int i = tid; i < EB * H; i += G) {
        const int e = i / H, k = i % H;
        dhn[e][k] = 0.f;
        dcn[e][k] = 0.f;
    }
    __syncthreads();
    for (int t = T - 1; t >= 0; --t) {
        // gate gradients of step t, (env, unit) pairs
        for (int i = tid; i < EB * H; i += G) {
            const int e = i / H, k = i % H, ge = e0 + e;
            if (ge >= B) {
#pragma unroll
                for (int g = 0; g < 4; ++g) dgs[e][g * H + k] = 0.f;
                continue;
            }
            const size_t row = (size_t)t * B + ge;
            const bool rs = reset && reset[row];
            const float dh = dh_out[row * H + k] + dhn[e][k];
            const float c = c_out[row * H + k];
            const float cp = rs ? 0.f : (t > 0 ? c_out[(row - B) * H + k] : (c0 ? c0[(size_t)ge * H + k] : 0.f));
            const float* a = gact + row * G;
            const float ig = a[k], fg = a[H + k], gg = a[2 * H + k], og = a[3 * H + k];
            const float tc = tanhf(c);
            const float dc = dcn[e][k] + dh * og * (1.f - tc * tc);
            const float d_i = dc * gg * ig * (1.f - ig);
            const float d_f = dc * cp * fg * (1.f - fg);
            const float d_g = dc * ig * (1.f - gg * gg);
            const float d_o = dh * tc * og * (1.f - og);
            dgs[e][k] = d_i; dgs[e][H + k] = d_f; dgs[e][2 * H + k] = d_g; dgs[e][3 * H + k] = d_o;
            float* o = dgx + row * G;
            o[k] = d_i; o[H + k] = d_f; o[2 * H + k] = d_g; o[3 * H + k] = d_o;
            dcn[e][k] = rs ? 0.f : dc * fg;  // into c_{t-1} (none across a reset)
        }
        __syncthreads();
        // dh_{t-1} = dG W_hh: four partial sums over gate-row quarters, then a fixed-order add
#pragma unroll 2
        for (int e = 0; e < EB; ++e) {
            float acc = 0.f;
            const float4* d4 = reinterpret_cast<const float4*>(&dgs[e][q * H]);
#pragma unroll
            for (int jj = 0; jj < H / 4; ++jj) {
                const float4 dv = d4[jj];
                acc = fmaf(dv.x, w[4 * jj], acc);
                acc = fmaf(dv.y, w[4 * jj + 1], acc);
                acc = fmaf(dv.z, w[4 * jj + 2], acc);
                acc = fmaf(dv.w, w[4 * jj + 3], acc);
            }
            red[q][e][k_own] = acc;
        }
        __syncthreads();
        for (int i = tid; i < EB * H; i += G) {
            const int e = i / H, k = i % H, ge = e0 + e;
            const bool rs = ge < B && reset && reset[(size_t)t * B + ge];
            const float s = (red[0][e][k] + red[1][e][k]) + (red[2][e][k] + red[3][e][k]);
            dhn[e][k] = rs ? 0.f : s;
        }
        __syncthreads();
    }
}

thread_local std::string g_err;

int fail(const std::string& m) {
    g_err = m;
    return -1;
}

template <int H>
int fwd_h(int T, int B, const float* gx, const float* whh, const float* h0, const float* c0, const uint8_t* reset,
          float* h_out, float* c_out, float* gact, float* h_last, float* c_last, hipStream_t s) {
    hipLaunchKernelGGL(k_lstm_fwd<H>, dim3((B + EB - 1) / EB), dim3(4 * H), 0, s, T, B, gx, whh, h0, c0, reset, h_out,
                       c_out, gact, h_last, c_last);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_fwd: ") + hipGetErrorString(e));
}

template <int H>
int bwd_h(int T, int B, const float* whh, const float* c0, const uint8_t* reset, const float* c_out,
          const float* gact, const float* dh_out, float* dgx, hipStream_t s) {
    hipLaunchKernelGGL(k_lstm_bwd<H>, dim3((B + EB - 1) / EB), dim3(4 * H), 0, s, T, B, whh, c0, reset, c_out, gact,
                       dh_out, dgx);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("pmlp_lstm_bwd: ") + hipGetErrorString(e));
}

}  // namespace

PMLP_API const char* pmlp_lstm_last_error(void) { return g_err.c_str(); }

PMLP_API int pmlp_lstm_supported(int32_t hidden) { return hidden == 32 || hidden == 64 || hidden == 128; }

PMLP_API int pmlp_lstm_fwd(int32_t T, int32_t B, int32_t H, const float* gx, const float* whh, const float* h0,
                           const float* c0, const uint8_t* reset, float* h_out, float* c_out, float* gact,
                           float* h_last, float* c_last, void* stream) {
    if (T <= 0 || B <= 0 || !gx || !whh) return fail("pmlp_lstm_fwd: empty sequence or null gx/whh");
    if (((uintptr_t)whh & 15u) != 0) return fail("pmlp_lstm_fwd: whh must be 16-byte aligned");
    hipStream_t s = (hipStream_t)stream;
    switch (H) {
    case 32: return fwd_h<32>(T, B, gx, whh, h0, c0, reset, h_out, c_out, gact, h_last, c_last, s);
    case 64: return fwd_h<64>(T, B, gx, whh, h0, c0, reset, h_out, c_out, gact, h_last, c_last, s);
    case 128: return fwd_h<128>(T, B, gx, whh, h0, c0, reset, h_out, c_out, gact, h_last, c_last, s);
    default: return fail("pmlp_lstm_fwd: hidden size must be 32, 64 or 128");
    }
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
