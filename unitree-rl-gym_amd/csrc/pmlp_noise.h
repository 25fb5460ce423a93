// The rollout's policy noise and Gaussian log-density, shared by pmlp_act (ppo_mlp.hip), the
// fused rollout forward and the recurrent heads' fused sampling (lstm_seq.hip), so all of them
// compute the same bits: Philox4x32-10 keyed by the rollout seed, counter (draw, env row,
// action quad, 0x5050), Box-Muller pairs (rsl_rl ActorCritic.act: Normal(mu, std).sample()).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}
__device__ __forceinline__ float u01(uint32_t x) { return ((float)x + 0.5f) * 2.3283064365386963e-10f; }

static constexpr float kHalfLog2Pi = 0.91893853320467274f;  // log(sqrt(2 pi))

// pmlp_act's sampling of row i, actions 4c .. 4c + 3 (k < A): act = mu + sigma z and the
// Gaussian log-density term of each (the caller sums a row's terms into its log-probability)
__device__ __forceinline__ void act_quad(uint32_t draw, uint2 key, uint32_t i, int c, int A, const float* stdv,
                                         const float* mu, float act[4], float sg[4], float term[4]) {
    // (the library's default contraction, as pmlp_act has always been compiled)
    const uint4 r = philox4x32(make_uint4(draw, i, (uint32_t)c, 0x5050u), key);
    const float rad0 = sqrtf(-2.f * logf(u01(r.x))), rad1 = sqrtf(-2.f * logf(u01(r.z)));
    float z[4];
    sincospif(2.f * u01(r.y), &z[1], &z[0]);
    sincospif(2.f * u01(r.w), &z[3], &z[2]);
    z[0] *= rad0; z[1] *= rad0; z[2] *= rad1; z[3] *= rad1;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int k = 4 * c + u;
        if (k >= A) break;
        sg[u] = stdv[k];
        act[u] = mu[u] + sg[u] * z[u];
        const float d = act[u] - mu[u];
        term[u] = -(d * d) / (2.f * sg[u] * sg[u]) - logf(sg[u]) - kHalfLog2Pi;
    }
}
