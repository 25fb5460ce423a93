// leggedsim.hip — MI355X (gfx950) implementation of include/leggedsim.h.
//
// One wavefront (a 64-thread workgroup) owns one env.  The env's articulated
// state lives in LDS for the whole control step: `decimation` physics substeps
// and the post-physics stack run inside ONE launch, lanes spread over bodies,
// DOFs, constraint rows and observation entries.  HBM sees each env's state
// once in and once out per control step (SURVEY §8d algorithmic bytes).
//
// Substep (same algorithm as oracle/lgs_oracle.c, part B):
//   FK (lane per body, walks its own chain)  ->  spatial inertia / motion
//   subspace / RNEA bias per body  ->  subtree sums (lane per body, contiguous
//   DFS ranges)  ->  mass matrix (lane per lower-triangle entry) + bias  ->
//   left-looking Cholesky (lane per row)  ->  free velocity  ->  joint-limit and
//   contact rows (ballot compaction)  ->  Y = L^-1 J^T (lane per row)  ->
//   A = Y^T Y  ->  projected Gauss-Seidel (row owner lanes, readlane
//   broadcasts)  ->  qd' = qf + L^-T Y lambda  ->  integrate.
// Post-physics (legged_robot.py:673-709): lane 0 runs the scalar stack in the
// reference's order; observation/noise/reset draws are spread over lanes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/leggedsim.h"
#include "lgs_detmath.h"

// Diagnostic build only (-DLGS_PHASE_STAMPS): lane 0 accumulates s_memtime
// deltas per phase into a global [N][LGS_NPHASE] buffer.  Never in the real build.
#define LGS_NPHASE 24
#ifdef LGS_PHASE_STAMPS
__device__ unsigned long long* g_phase_buf;
#define STAMP(i)                                                                                 \
    do {                                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        unsigned long long _t;                                                                   \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");             \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        if (threadIdx.x == 0) {                                                                  \
            if ((i) > 0) s.stamps[(i)] += _t - s.tlast;                                          \
            s.tlast = _t;                                                                        \
        }                                                                                        \
    } while (0)
#define STAMP_FLUSH(e)                                                                           \
    do {                                                                                         \
        if (threadIdx.x < LGS_NPHASE && g_phase_buf)                                             \
            g_phase_buf[(size_t)(e) * LGS_NPHASE + threadIdx.x] = s.stamps[threadIdx.x];         \
    } while (0)
#define STAMP_INIT()                                                                             \
    do {                                                                                         \
        if (threadIdx.x < LGS_NPHASE) s.stamps[threadIdx.x] = 0;                                 \
        if (threadIdx.x == 0) {                                                                  \
            s.stamps[18] = _wt0; s.stamps[20] = _wr0;                                            \
            s.stamps[22] = _whw; s.stamps[23] = _wxcc;                                           \
        }                                                                                        \
    } while (0)
// the wave's timeline: shader-clock and 100 MHz real-time stamps at kernel entry and exit,
// and where it ran (HW_ID: SIMD / CU / SH / SE; XCC_ID), for tools/wave_timeline.py
#define STAMP_BEGIN()                                                                            \
    unsigned long long _wt0, _wr0;                                                               \
    unsigned _whw, _wxcc;                                                                        \
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_getreg_b32 %2, hwreg(HW_REG_HW_ID)\n\t"   \
                 "s_getreg_b32 %3, hwreg(HW_REG_XCC_ID)\n\ts_waitcnt lgkmcnt(0)"                    \
                 : "=s"(_wt0), "=s"(_wr0), "=s"(_whw), "=s"(_wxcc)::"memory")
#define STAMP_END()                                                                              \
    do {                                                                                         \
        unsigned long long _t, _r;                                                               \
        asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)"                    \
                     : "=s"(_t), "=s"(_r)::"memory");                                            \
        if (threadIdx.x == 0) { s.stamps[19] = _t; s.stamps[21] = _r; }                          \
    } while (0)
#else
#define STAMP_BEGIN() do {} while (0)
#define STAMP_END() do {} while (0)
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH(e) do {} while (0)
#define STAMP_INIT() do {} while (0)
#endif
// occupancy target of the 32-row (Go2) k_step: 4 waves/SIMD puts all 4096 envs in
// flight at once but caps VGPRs at 128 (spills); 2 keeps every value in registers
#ifndef LGS_WAVES_PER_EU
#define LGS_WAVES_PER_EU 4
#endif
// the 48-row (humanoid) variant: A stays in registers, so its LDS allows 3 waves/SIMD
#ifndef LGS_WAVES_PER_EU_48
#define LGS_WAVES_PER_EU_48 3
#endif
#define MAXB LGS_MAX_BODIES
#define MAXD LGS_MAX_DEPTH
// contact candidates per model: at most 32 chunks of 32 (the pre-filter's chunk masks)
#define LGS_MAX_CHUNKS 32
// slack of the contact pre-filter's bounding-sphere test (m): far above fp32 rounding
#define LGS_PREFILTER_MARGIN 1e-3f
#define WAVE 64
typedef float floatx16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------ errors --
static thread_local std::string g_err;
static int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIP_TRY(x)                                                                        \
    do {                                                                                  \
        hipError_t _e = (x);                                                              \
        if (_e != hipSuccess) return set_err(LGS_ERR_HIP, std::string(#x ": ") + hipGetErrorString(_e)); \
    } while (0)

// ------------------------------------------------------------ device math --
struct DevModel {
    int B, D, P;
    // the robot's own body / DOF counts.  B, D (and the kernel's template sizes) may be larger:
    // lgs_create_sim pads a model to its kernel's shape with inert bodies and DOFs (no mass, no
    // contact candidates, no torque; every product they enter is an exact zero), so the state,
    // torques, observations and body rows in memory use Br / Dr
    int Br, Dr;
    const int* parent;
    const int* dof;
    const int* subtree_end;
    const int* depth;
    const int* chain;
    const float* joint_rot;
    const float* joint_pos;
    const float* axis;
    const float* mass;
    const float* com;
    const float* inertia;
    const float* dof_lower;
    const float* dof_upper;
    const float* dof_velocity;
    const int* pt_body;
    const float* pt_pos;
    const float* pt_radius;
    // contact pre-filter (lgs_create_sim): per body a bounding sphere of its candidates
    // [cx cy cz rho rmax] (body frame; rho = max |p - c|, rmax = max radius, rho < 0: no
    // candidates), and per chunk of 32 candidates the bit mask of the bodies in it
    const float* bsph;
    const unsigned* chunk32;
    int nch32;
};

struct DevSim {
    float dt, gx, gy, gz;
    int iters;
    float contact_offset, rest_offset, max_depen, beta, ground_friction, armature;
    int clamp_qd, max_contacts, max_rows;
    // heightfield ground (lgs_set_heightfield); hf == nullptr: the z = 0 plane
    const int16_t* hf;
    int hf_rows, hf_cols;
    float hf_inv_hs, hf_vs, hf_border;
    // the map's slope bound (lgs_set_heightfield): 1 + G and 1/sqrt(1 + G^2), G = the largest
    // triangle gradient norm; the contact pre-filter's terrain margin
    float hf_slope1, hf_nmin;
    // self-collision (lgs_set_self_collision): n_selfp pair records of 16 floats,
    // [p0(3) p1(3) r body] of the first proxy then of the second; n_selfp == 0: off
    const float4* selfp;
    int n_selfp, max_self;
    // [8][LGS_NUM_CONTACT_STATS] capacity-drop counters, one row per XCD (lgs_get_contact_stats)
    unsigned long long* stats;
};

// a substep's capacity drops into the per-XCD counter row (rare: atomics only when nonzero,
// and no register holds a count across the substeps)
__device__ __forceinline__ void count_drops(const DevSim& sp, int lane, int k, int v) {
    if (lane == 0 && v > 0) atomicAdd(sp.stats + LGS_NUM_CONTACT_STATS * (blockIdx.x & 7u) + k, (unsigned long long)v);
}

struct DevState {
    float* root;     // [N,13]
    float* dofs;     // [N,D,2]
    float* cforce;   // [N,B,3]
    float* rbs;      // [N,B,13]
    const float* friction;    // [N]
    const float* added_mass;  // [N]
    const float* torques_in;  // [N,D] (lgs_simulate)
    float* vsim;              // [N,2] the step's base xy velocity before the all-env push draw (k_step_extras)
    unsigned* pushed;         // [3] "some env was pushed" per step parity (k_step sets, k_step_extras reads),
                              // then the step key of the last control step (a deferred step's consumer)
};

__device__ __forceinline__ float rl(float x, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
__device__ __forceinline__ int rli(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
// wave-uniform copy (SGPR) of a value that is identical in every lane
__device__ __forceinline__ float rfl(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }

// ---- envs per wave.  EPW = 1: one env per 64-lane wave.  EPW = 2: two envs per wave in
// lanes 0-31 and 32-63 (the Go2 variant: every per-env phase fits in 32 lanes, ROWS <= 32),
// so half as many waves carry the same envs and the lane-per-body / per-DOF / per-row
// phases use 2x the lanes.  hl = the lane within its env, hh = which env of the wave;
// bc(x, r) = x of lane r of this lane's env; hballot = the ballot of this lane's env.
template <int EPW> __device__ __forceinline__ int hl() { return EPW == 2 ? (int)(threadIdx.x & 31u) : (int)threadIdx.x; }
template <int EPW> __device__ __forceinline__ int hh() { return EPW == 2 ? (int)(threadIdx.x >> 5) : 0; }
// Broadcast with ds_bpermute (the LDS crossbar: one instruction, no SGPR round trip and
// no readlane hazard wait).  The source lane must be active: every call sits outside
// lane-divergent branches (only whole-env conditions, which keep the env's lanes together).  Two envs per wave: 0.230 -> 0.203 ms per Go2 4096-env step
// against two v_readlane + select; one env per wave: -1 % on H1 8192 against v_readlane.
template <int EPW> __device__ __forceinline__ float bc(float x, int r) {
    return __int_as_float(
        __builtin_amdgcn_ds_bpermute((int)(((EPW == 2 ? (threadIdx.x & 32u) : 0u) + (unsigned)r) << 2), __float_as_int(x)));
}
template <int EPW> __device__ __forceinline__ uint64_t hballot(bool p) {
    const uint64_t m = __ballot(p);
    if constexpr (EPW == 1) return m;
    else return (m >> (threadIdx.x & 32u)) & 0xffffffffull;
}

__device__ __forceinline__ void cross3(const float* a, const float* b, float* o) {
    float x = a[1] * b[2] - a[2] * b[1];
    float y = a[2] * b[0] - a[0] * b[2];
    float z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
__device__ __forceinline__ float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ void matvec(const float* R, const float* v, float* o) {
    float x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    float y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    float z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}
__device__ __forceinline__ void matmul(const float* A, const float* B, float* C) {
    float T[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = T[i];
}
__device__ __forceinline__ void quat_to_mat(const float* q, float* R) {
    float x = q[0], y = q[1], z = q[2], w = q[3];
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w);     R[2] = 2 * (x * z + y * w);
    R[3] = 2 * (x * y + z * w);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
    R[6] = 2 * (x * z - y * w);     R[7] = 2 * (y * z + x * w);     R[8] = 1 - 2 * (x * x + y * y);
}
__device__ __forceinline__ void mat_to_quat(const float* R, float* q) {
    float tr = R[0] + R[4] + R[8];
    if (tr > 0.f) {
        float s = sqrtf(tr + 1.f) * 2.f;
        q[3] = 0.25f * s; q[0] = (R[7] - R[5]) / s; q[1] = (R[2] - R[6]) / s; q[2] = (R[3] - R[1]) / s;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        float s = sqrtf(1.f + R[0] - R[4] - R[8]) * 2.f;
        q[3] = (R[7] - R[5]) / s; q[0] = 0.25f * s; q[1] = (R[1] + R[3]) / s; q[2] = (R[2] + R[6]) / s;
    } else if (R[4] > R[8]) {
        float s = sqrtf(1.f + R[4] - R[0] - R[8]) * 2.f;
        q[3] = (R[2] - R[6]) / s; q[0] = (R[1] + R[3]) / s; q[1] = 0.25f * s; q[2] = (R[5] + R[7]) / s;
    } else {
        float s = sqrtf(1.f + R[8] - R[0] - R[4]) * 2.f;
        q[3] = (R[3] - R[1]) / s; q[0] = (R[2] + R[6]) / s; q[1] = (R[5] + R[7]) / s; q[2] = 0.25f * s;
    }
}
__device__ __forceinline__ void axis_angle(const float* a, float ang, float* R) {
    float s, c;
    lgs_sincosf(ang, &s, &c);  // deterministic: the oracle's bits (lgs_detmath.h)
    float t = 1.f - c;
    float x = a[0], y = a[1], z = a[2];
    R[0] = t * x * x + c;     R[1] = t * x * y - s * z; R[2] = t * x * z + s * y;
    R[3] = t * x * y + s * z; R[4] = t * y * y + c;     R[5] = t * y * z - s * x;
    R[6] = t * x * z - s * y; R[7] = t * y * z + s * x; R[8] = t * z * z + c;
}
// spatial inertia (m, h, I6) applied to motion (w, v) -> force (n, f)
__device__ __forceinline__ void sin_apply(float m, const float* h, const float* I, const float* w, const float* v,
                                          float* n, float* f) {
    float Iw0 = I[0] * w[0] + I[3] * w[1] + I[4] * w[2];
    float Iw1 = I[3] * w[0] + I[1] * w[1] + I[5] * w[2];
    float Iw2 = I[4] * w[0] + I[5] * w[1] + I[2] * w[2];
    float hv[3], hw[3];
    cross3(h, v, hv);
    cross3(h, w, hw);
    n[0] = Iw0 + hv[0]; n[1] = Iw1 + hv[1]; n[2] = Iw2 + hv[2];
    f[0] = m * v[0] - hw[0]; f[1] = m * v[1] - hw[1]; f[2] = m * v[2] - hw[2];
}

// ----------------------------------------------------------- Philox RNG --
__host__ __device__ __forceinline__ float philox_uniform(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2,
                                                         uint32_t c3) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return (float)(c0 >> 8) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ float rand_range(float lo, float hi, float u) { return (hi - lo) * u + lo; }

// ------------------------------------------------------------- terrain --
// Ground height under (x, y) and the unit normal of the triangle there.  The
// heightfield cell (i, j) is split along its (i,j)-(i+1,j+1) diagonal
// (terrain_utils.convert_heightfield_to_trimesh); outside the map the edge samples
// continue.  Without a heightfield: the plane z = 0, normal +z.  Same arithmetic
// as oracle/lgs_oracle.c terrain_sample().
__device__ __forceinline__ float terrain_sample(const DevSim& sp, float x, float y, float* nrm) {
    if (!sp.hf) {
        nrm[0] = 0.f; nrm[1] = 0.f; nrm[2] = 1.f;
        return 0.f;
    }
    float u = (x + sp.hf_border) * sp.hf_inv_hs, v = (y + sp.hf_border) * sp.hf_inv_hs;
    u = fminf(fmaxf(u, 0.f), (float)(sp.hf_rows - 1));
    v = fminf(fmaxf(v, 0.f), (float)(sp.hf_cols - 1));
    const int i = min((int)u, sp.hf_rows - 2), j = min((int)v, sp.hf_cols - 2);
    const float fu = u - (float)i, fv = v - (float)j;
    const int16_t* h0 = sp.hf + (size_t)i * sp.hf_cols + j;
    const float h00 = (float)h0[0] * sp.hf_vs, h01 = (float)h0[1] * sp.hf_vs;
    const float h10 = (float)h0[sp.hf_cols] * sp.hf_vs, h11 = (float)h0[sp.hf_cols + 1] * sp.hf_vs;
    float du, dv;
    if (fu >= fv) { du = h10 - h00; dv = h11 - h10; }
    else { du = h11 - h01; dv = h01 - h00; }
    const float h = h00 + fu * du + fv * dv;
    const float gx = du * sp.hf_inv_hs, gy = dv * sp.hf_inv_hs;
    const float inv = 1.f / sqrtf(gx * gx + gy * gy + 1.f);
    nrm[0] = 0.f - gx * inv; nrm[1] = 0.f - gy * inv; nrm[2] = inv;
    return h;
}
// contact frame: t1 = normalise(e_x - n_x n), t2 = n x t1 (flat ground: +x, +y exactly)
__device__ __forceinline__ void contact_tangents(const float* n, float* t1, float* t2) {
    const float a0 = 1.f - n[0] * n[0], a1 = 0.f - n[0] * n[1], a2 = 0.f - n[0] * n[2];
    const float inv = 1.f / sqrtf(a0 * a0 + a1 * a1 + a2 * a2);
    t1[0] = a0 * inv; t1[1] = a1 * inv; t1[2] = a2 * inv;
    cross3(n, t1, t2);
}
__device__ __forceinline__ float clipf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// ------------------------------------------------------- self-collision --
// Closest points c1, c2 of the segments p1q1 and p2q2 (Ericson, Real-Time Collision
// Detection 5.1.9).  Same arithmetic as oracle/lgs_oracle.c seg_closest().
__device__ __forceinline__ void seg_closest(const float* p1, const float* q1, const float* p2, const float* q2,
                                            float* c1, float* c2) {
    const float d1[3] = {q1[0] - p1[0], q1[1] - p1[1], q1[2] - p1[2]};
    const float d2[3] = {q2[0] - p2[0], q2[1] - p2[1], q2[2] - p2[2]};
    const float r[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    const float a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    const float eps = 1e-12f;
    float s, t;
    if (a <= eps && e <= eps) {
        s = 0.f; t = 0.f;
    } else if (a <= eps) {
        s = 0.f; t = clipf(f / e, 0.f, 1.f);
    } else {
        const float c = dot3(d1, r);
        if (e <= eps) {
            t = 0.f; s = clipf(-c / a, 0.f, 1.f);
        } else {
            const float b = dot3(d1, d2);
            const float den = a * e - b * b;
            s = den != 0.f ? clipf((b * f - c * e) / den, 0.f, 1.f) : 0.f;
            t = (b * s + f) / e;
            if (t < 0.f) { t = 0.f; s = clipf(-c / a, 0.f, 1.f); }
            else if (t > 1.f) { t = 1.f; s = clipf((b - c) / a, 0.f, 1.f); }
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) { c1[k] = p1[k] + d1[k] * s; c2[k] = p2[k] + d2[k] * t; }
}
// friction frame of a self contact: t1 = normalise(e - (e.n) n) with e = x, or y when n is
// within 55 degrees of x; t2 = n x t1
__device__ __forceinline__ void self_tangents(const float* n, float* t1, float* t2) {
    float a0, a1, a2;
    if (fabsf(n[0]) < 0.57735f) { a0 = 1.f - n[0] * n[0]; a1 = 0.f - n[0] * n[1]; a2 = 0.f - n[0] * n[2]; }
    else { a0 = 0.f - n[1] * n[0]; a1 = 1.f - n[1] * n[1]; a2 = 0.f - n[1] * n[2]; }
    const float inv = 1.f / sqrtf(a0 * a0 + a1 * a1 + a2 * a2);
    t1[0] = a0 * inv; t1[1] = a1 * inv; t1[2] = a2 * inv;
    cross3(n, t1, t2);
}

// ------------------------------------------------------------ LDS layout --
// Model topology/geometry cached in LDS at kernel start: every chain walk and
// subtree test below is an LDS access instead of a dependent global load.
template <int D, int B>
struct ModelCache {
    int dof[B], depth[B], se[B], dofbody[D > 0 ? D : 1];
    unsigned anc[D > 0 ? D : 1];  // bit i: DOF i is an ancestor-or-self of DOF j (i <= j)
    unsigned char chain[B][MAXD];
    float jr[B][9], jp[B][3], ax[B][3], com[B][3], mass[B], in[B][6];
    float lo[D > 0 ? D : 1], hi[D > 0 ? D : 1], vl[D > 0 ? D : 1];
    float bs[B][5];                 // candidates' bounding sphere per body (DevModel::bsph)
    unsigned ch32[LGS_MAX_CHUNKS];  // bodies per chunk of 32 candidates (zero-padded)
};

// bodies with candidates in chunk ch of WAVE/EPW candidates
template <int EPW, int D, int B>
__device__ __forceinline__ unsigned chunk_bodies(const ModelCache<D, B>& mc, int ch) {
    return EPW == 2 ? mc.ch32[ch] : (mc.ch32[2 * ch] | mc.ch32[2 * ch + 1]);
}

template <int D, int B, int ROWS>
struct Smem {
    static constexpr int n = 6 + D;
    static constexpr int NP = (n % 2 == 0) ? n + 1 : n;     // odd row stride: conflict-free columns
    static constexpr int AS = (ROWS % 2 == 0) ? ROWS + 1 : ROWS;
    float root[16];
    float q[D], qd[D], tau[D], act[D];
    float R[B][9], p[B][3], aw[B][3], cw[B][3];
    union {
        struct {
            // per body, packed for 16-byte LDS reads in the subtree sums:
            // pk  = [m, h(3), I(6), fn(3), ff(3)]  (spatial inertia at O, bias force)
            // cpk = [cm, ch(3), cI(6), Fn(3), Ff(3)]  (the subtree sums of pk)
            __attribute__((aligned(16))) float pk[B][16];
            __attribute__((aligned(16))) float cpk[B][16];
            float Sw[B][3], Sv[B][3];
            __attribute__((aligned(16))) float Sd[D > 0 ? D : 1][8];  // per DOF: [Sw(3), Sv(3), 0, 0]
            float Fj[D][6];
        } dyn;
        struct {
            float Y[ROWS][NP];  // (A never leaves registers: MFMA tiles, columns per lane)
        } con;
        struct {  // FK scratch: per-DOF joint rotation R(axis, q)
            float Ra[D > 0 ? D : 1][9];
        } fk;
        struct {  // post-physics scratch
            float obs_tmp[LGS_MAX_OBS];
            float terms[LGS_MAX_REWARDS + 1];
            float misc[32];
        } post;
        struct {  // contact selection (step 8, before any constraint row is written)
            int pwin[B];              // per body: its first touching candidate so far (primary)
            int sec_body[ROWS / 4];   // ground contacts beyond the primaries, in candidate order
            float sec[ROWS / 4][7];   // point(3), separation, normal(3)
            int sc_ab[ROWS / 4][2];   // self contacts, in pair order
            float sc_tmp[ROWS / 4][7];  // point(3), separation, normal(3)
        } sel;
    } u;
    static constexpr int LP = (n + 3) / 4 * 4;  // 16-byte rows: uniform row reads are ds_read_b128
    __attribute__((aligned(16))) float L[n][LP];
    float Linv[n];
    float qf[n];
    float tgt[ROWS];
    int c_body[ROWS / 3];
    int c_body2[ROWS / 3];    // self contact: the second body (its force enters with a minus sign)
    float c_pt[ROWS / 3][3];
    float c_fr[ROWS / 3][9];  // contact frame: normal, tangent 1, tangent 2
    float c_sep[ROWS / 3];
    float cf[B][3];
    int flags[8];
#ifdef LGS_PHASE_STAMPS
    unsigned long long stamps[LGS_NPHASE];
    unsigned long long tlast;
#endif
};

// the whole workgroup fills the block's (shared) model cache
template <int D, int B>
__device__ __forceinline__ void load_model(ModelCache<D, B>& c, const DevModel& md) {
    const int lane = threadIdx.x;
    if (lane < B) {
        const int j = md.dof[lane];
        c.dof[lane] = j;
        c.depth[lane] = md.depth[lane];
        c.se[lane] = md.subtree_end[lane];
        c.mass[lane] = md.mass[lane];
        if (j >= 0) c.dofbody[j] = lane;
    }
    for (int i = lane; i < B * MAXD; i += WAVE) (&c.chain[0][0])[i] = (unsigned char)md.chain[i];
    for (int i = lane; i < 9 * B; i += WAVE) (&c.jr[0][0])[i] = md.joint_rot[i];
    for (int i = lane; i < 3 * B; i += WAVE) {
        (&c.jp[0][0])[i] = md.joint_pos[i];
        (&c.ax[0][0])[i] = md.axis[i];
        (&c.com[0][0])[i] = md.com[i];
    }
    for (int i = lane; i < 6 * B; i += WAVE) (&c.in[0][0])[i] = md.inertia[i];
    for (int i = lane; i < 5 * B; i += WAVE) (&c.bs[0][0])[i] = md.bsph[i];
    if (lane < LGS_MAX_CHUNKS) c.ch32[lane] = lane < md.nch32 ? md.chunk32[lane] : 0u;
    if (lane < D) {
        int bj = 0;
        for (int b = 0; b < B; ++b) bj = md.dof[b] == lane ? b : bj;
        unsigned am = 0u;
        for (int b = 0; b <= bj; ++b) {
            const int i = md.dof[b];
            if (i >= 0 && i <= lane && bj < md.subtree_end[b]) am |= 1u << i;
        }
        c.anc[lane] = am;
        c.lo[lane] = md.dof_lower[lane];
        c.hi[lane] = md.dof_upper[lane];
        c.vl[lane] = md.dof_velocity[lane];
    }
}

// -------------------------------------------------------------- substep --
// One physics substep of this block's env.  Preconditions: s.root/q/qd/tau hold
// the state and the torques, s.mc the model.  Postcondition: state integrated,
// s.cf = contact forces of this substep.  All 64 lanes must call it.
//
// Register-resident linear algebra (lane i < n owns row i of M / L):
//   mass matrix row assembled in-lane from the composites; right-looking
//   Cholesky with v_readlane broadcasts (per entry the same subtraction order
//   as the oracle's left-looking loop); triangular solves on register rows
//   (forward) and register columns (backward); Y = L^-1 J^T with L entries
//   broadcast by readlane; A = Y Y^T on the matrix cores
//   (v_mfma_f32_32x32x2_f32: exact fp32 fma chain over k); PGS with each lane
//   holding its column of A in registers.
// The linear algebra runs in the LEAVES-FIRST order: index p = n-1-i of the natural
// [base (6), joints in DFS order] order, i.e. every DOF after all of its descendants,
// so the Cholesky factor has no fill-in.  With CH > 0 every joint chain has CH DOFs
// hanging from the base (Go2: 4 x 3, G1 / H1_2: 2 x 6, H1: 2 x 5), and column k < D
// of L is nonzero only at rows k+1 .. k+pos(k) (the joint's ancestors on its chain,
// pos = its depth in the chain) and at the base rows D..n-1.  Structurally zero
// entries are exact zeros (no fill-in), so skipping them changes no result bit.
template <int D, int CH>
__host__ __device__ constexpr bool l_nz(int i, int k) {  // may L[i][k] (i > k) be nonzero?
    return CH == 0 || k >= D || i >= D || i <= k + (D - 1 - k) % CH;
}

// L L^T x = b for an env-uniform b (LDS), every lane computing the whole x from env-uniform
// LDS reads of L (leaves-first, structural zeros skipped: l_nz).  Forward then backward; per
// element the operations and their order of the lane-distributed solves in substep().
template <int D, int CH, int n, int LP>
__device__ __forceinline__ void uniform_back(const float* b, const float (*L)[LP], const float* Linv, float* xv) {
#pragma unroll
    for (int i = 0; i < n; ++i) xv[i] = b[i];
#pragma unroll
    for (int i = n - 1; i >= 0; --i) {
        float t = xv[i];
#pragma unroll
        for (int k = n - 1; k > i; --k)
            if (l_nz<D, CH>(k, i)) t = fmaf(-L[k][i], xv[k], t);
        xv[i] = t * Linv[i];
    }
}
template <int D, int CH, int n, int LP>
__device__ __forceinline__ void uniform_solve(const float* b, const float (*L)[LP], const float* Linv, float* xv) {
    float yv[n];
#pragma unroll
    for (int i = 0; i < n; ++i) {
        float t = b[i];
#pragma unroll
        for (int k = 0; k < i; ++k)
            if (l_nz<D, CH>(i, k)) t = fmaf(-L[i][k], yv[k], t);
        yv[i] = t * Linv[i];
    }
    // backward from the register vector (the same arithmetic as uniform_back)
#pragma unroll
    for (int i = n - 1; i >= 0; --i) {
        float t = yv[i];
#pragma unroll
        for (int k = n - 1; k > i; --k)
            if (l_nz<D, CH>(k, i)) t = fmaf(-L[k][i], xv[k], t);
        xv[i] = t * Linv[i];
    }
}

template <int D, int B, int ROWS, int CH, int EPW, bool PAD = false>
__device__ void substep(Smem<D, B, ROWS>* sm, const ModelCache<D, B>& mc, const DevModel& md, const DevSim& sp,
                        float added_mass, float shape_mu) {
    constexpr int n = 6 + D;
    Smem<D, B, ROWS>& s = sm[hh<EPW>()];
    // Opaque lane id: lane-derived addresses are recomputed each substep (a few VALU
    // ops) instead of being hoisted out of the decimation loop and held live across
    // every substep, which pushed the 4-waves/SIMD build into scratch.
    int lane = hl<EPW>();
    asm volatile("" : "+v"(lane));
    const float dt = sp.dt;
    const float idt = 1.0f / dt;  // every per-row / per-force division by dt is a multiply (as the oracle)

    STAMP(0);
    // ---- 1. forward kinematics: joint rotations lane per DOF, then lane b walks root..b
    if (lane < D) axis_angle(mc.ax[mc.dofbody[lane]], s.q[lane], s.u.fk.Ra[lane]);
    __syncthreads();
    if (lane < B) {
        float R[9], p[3], aw[3] = {0.f, 0.f, 0.f};
        quat_to_mat(s.root + 3, R);
        p[0] = s.root[0]; p[1] = s.root[1]; p[2] = s.root[2];
        const int d = mc.depth[lane];
        for (int l = 1; l <= d; ++l) {
            const int a = mc.chain[lane][l];
            float Rj[9], t[3];
            matmul(R, mc.jr[a], Rj);
            matvec(R, mc.jp[a], t);
            p[0] += t[0]; p[1] += t[1]; p[2] += t[2];
            const int j = mc.dof[a];
            if (j >= 0) {
                if (l == d) matvec(Rj, mc.ax[a], aw);
                matmul(Rj, s.u.fk.Ra[j], R);
            } else {
#pragma unroll
                for (int k = 0; k < 9; ++k) R[k] = Rj[k];
            }
        }
        float c[3];
        matvec(R, mc.com[lane], c);
#pragma unroll
        for (int k = 0; k < 9; ++k) s.R[lane][k] = R[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            s.p[lane][k] = p[k];
            s.aw[lane][k] = aw[k];
            s.cw[lane][k] = p[k] + c[k];
        }
    }
    __syncthreads();
    STAMP(1);
    const float O[3] = {s.p[0][0], s.p[0][1], s.p[0][2]};
    float w0[3] = {s.root[10], s.root[11], s.root[12]};
    float vO[3];
    {
        float rc[3] = {s.cw[0][0] - O[0], s.cw[0][1] - O[1], s.cw[0][2] - O[2]}, wxr[3];
        cross3(w0, rc, wxr);
        vO[0] = s.root[7] - wxr[0]; vO[1] = s.root[8] - wxr[1]; vO[2] = s.root[9] - wxr[2];
    }
    // ---- 2. per-body spatial inertia at O and motion subspace
    if (lane < B) {
        float m = mc.mass[lane], scale = 1.f;
        if (lane == 0 && added_mass != 0.f && m > 0.f) { scale = (m + added_mass) / m; m = m + added_mass; }
        const float* Il = mc.in[lane];
        float IL[9] = {Il[0] * scale, Il[3] * scale, Il[4] * scale, Il[3] * scale, Il[1] * scale,
                       Il[5] * scale, Il[4] * scale, Il[5] * scale, Il[2] * scale};
        float R[9], Rt[9], T[9], Iw[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) R[k] = s.R[lane][k];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) Rt[3 * i + j] = R[3 * j + i];
        matmul(R, IL, T);
        matmul(T, Rt, Iw);
        float r[3] = {s.cw[lane][0] - O[0], s.cw[lane][1] - O[1], s.cw[lane][2] - O[2]};
        float rr = dot3(r, r);
        s.u.dyn.pk[lane][0] = m;
        s.u.dyn.pk[lane][1 + 0] = m * r[0]; s.u.dyn.pk[lane][1 + 1] = m * r[1]; s.u.dyn.pk[lane][1 + 2] = m * r[2];
        s.u.dyn.pk[lane][4 + 0] = Iw[0] + m * (rr - r[0] * r[0]);
        s.u.dyn.pk[lane][4 + 1] = Iw[4] + m * (rr - r[1] * r[1]);
        s.u.dyn.pk[lane][4 + 2] = Iw[8] + m * (rr - r[2] * r[2]);
        s.u.dyn.pk[lane][4 + 3] = Iw[1] - m * r[0] * r[1];
        s.u.dyn.pk[lane][4 + 4] = Iw[2] - m * r[0] * r[2];
        s.u.dyn.pk[lane][4 + 5] = Iw[5] - m * r[1] * r[2];
        float rp[3] = {s.p[lane][0] - O[0], s.p[lane][1] - O[1], s.p[lane][2] - O[2]}, sv[3];
        float a[3] = {s.aw[lane][0], s.aw[lane][1], s.aw[lane][2]};
        cross3(rp, a, sv);
#pragma unroll
        for (int k = 0; k < 3; ++k) { s.u.dyn.Sw[lane][k] = a[k]; s.u.dyn.Sv[lane][k] = sv[k]; }
        const int jd = mc.dof[lane];
        if (jd >= 0) {
            float4* o = (float4*)s.u.dyn.Sd[jd];
            o[0] = make_float4(a[0], a[1], a[2], sv[0]);
            o[1] = make_float4(sv[1], sv[2], 0.f, 0.f);
        }
    }
    __syncthreads();
    STAMP(2);
    // ---- 3. velocity + bias acceleration down the chain, bias force per body
    if (lane < B) {
        float Vw[3] = {w0[0], w0[1], w0[2]}, Vv[3] = {vO[0], vO[1], vO[2]};
        float Aw[3] = {0.f, 0.f, 0.f}, Av[3] = {-sp.gx, -sp.gy, -sp.gz};
        const int d = mc.depth[lane];
        for (int l = 1; l <= d; ++l) {
            const int a = mc.chain[lane][l];
            const int j = mc.dof[a];
            if (j < 0) continue;
            const float qd = s.qd[j];
            float sw[3] = {s.u.dyn.Sw[a][0] * qd, s.u.dyn.Sw[a][1] * qd, s.u.dyn.Sw[a][2] * qd};
            float sv[3] = {s.u.dyn.Sv[a][0] * qd, s.u.dyn.Sv[a][1] * qd, s.u.dyn.Sv[a][2] * qd};
            float t1[3], t2[3], t3[3];
            cross3(Vw, sw, t1);
            cross3(Vw, sv, t2);
            cross3(Vv, sw, t3);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                Aw[k] += t1[k];
                Av[k] += t2[k] + t3[k];
                Vw[k] += sw[k];
                Vv[k] += sv[k];
            }
        }
        const float m = s.u.dyn.pk[lane][0];
        float h[3] = {s.u.dyn.pk[lane][1 + 0], s.u.dyn.pk[lane][1 + 1], s.u.dyn.pk[lane][1 + 2]};
        float I[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) I[k] = s.u.dyn.pk[lane][4 + k];
        float IAn[3], IAf[3], IVn[3], IVf[3], a1[3], a2[3], a3[3];
        sin_apply(m, h, I, Aw, Av, IAn, IAf);
        sin_apply(m, h, I, Vw, Vv, IVn, IVf);
        cross3(Vw, IVn, a1);
        cross3(Vv, IVf, a2);
        cross3(Vw, IVf, a3);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            s.u.dyn.pk[lane][10 + k] = IAn[k] + a1[k] + a2[k];
            s.u.dyn.pk[lane][13 + k] = IAf[k] + a3[k];
        }
    }
    __syncthreads();
    STAMP(3);
    // ---- 4. subtree (composite) sums: lane b adds its contiguous DFS range,
    // last to first (the oracle's order).  Loads of an iteration are independent;
    // unrolling lets them overlap the 16 add chains.
    if (lane < B) {
        const int end = mc.se[lane];
        float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0, a3 = a0;
#pragma unroll 4
        for (int k = end - 1; k >= lane; --k) {
            const float4* q = (const float4*)s.u.dyn.pk[k];
            const float4 b0 = q[0], b1 = q[1], b2 = q[2], b3 = q[3];
            a0.x += b0.x; a0.y += b0.y; a0.z += b0.z; a0.w += b0.w;
            a1.x += b1.x; a1.y += b1.y; a1.z += b1.z; a1.w += b1.w;
            a2.x += b2.x; a2.y += b2.y; a2.z += b2.z; a2.w += b2.w;
            a3.x += b3.x; a3.y += b3.y; a3.z += b3.z; a3.w += b3.w;
        }
        float4* o = (float4*)s.u.dyn.cpk[lane];
        o[0] = a0; o[1] = a1; o[2] = a2; o[3] = a3;
    }
    __syncthreads();
    // F_j = Ic(b_j) S_j (lane per DOF): the base block of M's row 6+j and, dotted
    // with S_i, every DOF-DOF entry of that row.
    if (lane < D) {
        const int bj = mc.dofbody[lane];
        float Sw[3] = {s.u.dyn.Sw[bj][0], s.u.dyn.Sw[bj][1], s.u.dyn.Sw[bj][2]};
        float Sv[3] = {s.u.dyn.Sv[bj][0], s.u.dyn.Sv[bj][1], s.u.dyn.Sv[bj][2]};
        float cn[3], cf[3];
        sin_apply(s.u.dyn.cpk[bj][0], (&s.u.dyn.cpk[bj][1]), (&s.u.dyn.cpk[bj][4]), Sw, Sv, cn, cf);
#pragma unroll
        for (int k = 0; k < 3; ++k) { s.u.dyn.Fj[lane][k] = cn[k]; s.u.dyn.Fj[lane][3 + k] = cf[k]; }
    }
    __syncthreads();
    STAMP(4);
    // ---- 5. row `lane` of the leaves-first mass matrix (lower triangle) into
    // registers, rhs = tau - C.  Lane i < D: joint jr = D-1-i (columns: itself and its
    // descendants); lane i >= D: base row r = n-1-i (columns: every joint, and the
    // base columns c >= r).
    float m[n];
    float x = 0.f;
#pragma unroll
    for (int c = 0; c < n; ++c) m[c] = 0.f;
    if (lane >= D && lane < n) {
        const int r = n - 1 - lane;
        const float* I = (&s.u.dyn.cpk[0][4]);
        const float* h = (&s.u.dyn.cpk[0][1]);
        const float cm0 = s.u.dyn.cpk[0][0];
        // M[r][6+j] = (F_j)_r
#pragma unroll
        for (int cp = 0; cp < D; ++cp) m[cp] = s.u.dyn.Fj[D - 1 - cp][r];
        // base block [[I, [h]x], [[h]x^T, m 1]], entries c >= r
        const float H[9] = {0.f, -h[2], h[1], h[2], 0.f, -h[0], -h[1], h[0], 0.f};
        const float I3[9] = {I[0], I[3], I[4], I[3], I[1], I[5], I[4], I[5], I[2]};
#pragma unroll
        for (int c = 0; c < 6; ++c) {  // c compile-time, r per lane: selects, no indexed registers
            const float* T = c < 3 ? I3 : H;
            const int cc = c < 3 ? c : c - 3;
            float val = r == 0 ? T[cc] : (r == 1 ? T[3 + cc] : (r == 2 ? T[6 + cc] : 0.f));
            if (c >= 3) val = r < 3 ? val : (r == c ? cm0 : 0.f);
            m[n - 1 - c] = c >= r ? val : 0.f;
        }
        x = -(r < 3 ? s.u.dyn.cpk[0][10 + r] : s.u.dyn.cpk[0][13 + r - 3]);
    } else if (lane < D) {
        const int jr = D - 1 - lane;
        const int bj = mc.dofbody[jr];
        float Sw[3] = {s.u.dyn.Sw[bj][0], s.u.dyn.Sw[bj][1], s.u.dyn.Sw[bj][2]};
        float Sv[3] = {s.u.dyn.Sv[bj][0], s.u.dyn.Sv[bj][1], s.u.dyn.Sv[bj][2]};
        // M[jr][jc] = S_jr . F_jc for jc a descendant-or-self of jr
#pragma unroll
        for (int cp = 0; cp < D; ++cp) {
            const int jc = D - 1 - cp;
            const float* F = s.u.dyn.Fj[jc];
            const float cn[3] = {F[0], F[1], F[2]}, cf[3] = {F[3], F[4], F[5]};
            float val = dot3(Sw, cn) + dot3(Sv, cf);
            if (jc == jr) val += (!PAD || jr < md.Dr) ? sp.armature : 1.f;  // (a padded model's inert DOF: M_jj = 1)
            m[cp] = ((mc.anc[jc] >> jr) & 1u) ? val : 0.f;
        }
        float Fn[3] = {s.u.dyn.cpk[bj][10 + 0], s.u.dyn.cpk[bj][10 + 1], s.u.dyn.cpk[bj][10 + 2]};
        float Ff[3] = {s.u.dyn.cpk[bj][13 + 0], s.u.dyn.cpk[bj][13 + 1], s.u.dyn.cpk[bj][13 + 2]};
        float C = dot3(Sw, Fn) + dot3(Sv, Ff);
        x = s.tau[jr] - C;
    }
    STAMP(5);
    // ---- 6. Cholesky, right-looking on register rows.  Entry (i,j) receives
    // -L_ik L_jk for k = 0..j-1 in ascending order, then / L_jj: the oracle's
    // left-looking arithmetic, operation for operation.
    // One IEEE reciprocal per pivot (wave-uniform); every division by L_kk here and
    // in the solves below is a multiplication by it (the oracle's arithmetic).  Lane k
    // keeps 1/L_kk in idg.
    float idg = 0.f;
    // With CH > 0 the joint pivots run level by level: the NC chains' pivots at depth t
    // (k = c*CH + t) are independent (column k is nonzero only on its own chain and the
    // base rows), so each pivot lane takes the square root and reciprocal of its own
    // diagonal and the NC reciprocals are broadcast together, one dependent
    // sqrt -> rcp -> broadcast -> fma step per level instead of per pivot.  Every base
    // row then receives the leg terms in LEVEL order (k = t, CH+t, 2CH+t, .. for
    // t = 0..CH-1); the oracle's cholesky() sums in that order for these instantiations
    // (orc_set_factor_chain).  The base pivots D..n-1 follow one by one.
    constexpr int K0 = CH > 0 ? D : 0;
    if constexpr (CH > 0) {
        constexpr int NC = D / CH;
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            int ln = lane;
            asm volatile("" : "+v"(ln));
            // the level's column entries, broadcast UNSCALED ahead of the square roots (off
            // the pivot chain); L_jk = raw * (1/L_kk) in the receiving lane is the product
            // lane j would form, so the same bits
            float raw[NC][n];
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int j = c * CH + t + 1; j < n; ++j)
                    if (l_nz<D, CH>(j, c * CH + t)) raw[c][j] = bc<EPW>(m[c * CH + t], j);
            float dg = 1.f;
#pragma unroll
            for (int c = 0; c < NC; ++c) dg = ln == c * CH + t ? m[c * CH + t] : dg;
            const float dl = sqrtf(fmaxf(dg, 1e-12f));
            const float il = 1.0f / dl;
            float ic[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) ic[c] = bc<EPW>(il, c * CH + t);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int k = c * CH + t;
                m[k] = ln == k ? dl : m[k] * ic[c];
                idg = ln == k ? il : idg;
            }
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int k = c * CH + t;
#pragma unroll
                for (int j = k + 1; j < n; ++j) {
                    if (!l_nz<D, CH>(j, k)) continue;
                    const float ljk = raw[c][j] * ic[c];
                    m[j] = fmaf(-m[k], ljk, m[j]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int k = K0; k < n; ++k) {
        // opaque per step: lane masks are recomputed here (one v_cmp each) instead of
        // being CSE'd across the factorisation and solves, where ~70 live mask SGPRs
        // spilled to VGPR lanes
        int ln = lane;
        asm volatile("" : "+v"(ln));
        // the column's entries broadcast unscaled, in flight with the diagonal's (as above)
        float raw[n];
#pragma unroll
        for (int j = k + 1; j < n; ++j)
            if (l_nz<D, CH>(j, k)) raw[j] = bc<EPW>(m[k], j);
        const float d = sqrtf(fmaxf(bc<EPW>(m[k], k), 1e-12f));
        const float inv = 1.0f / d;
        // Lanes above the diagonal (i < k, i < j) update their upper-triangle registers
        // too: nothing reads those (the L store, the solves and the broadcasts take the
        // lower triangle only), and no lane mask / select is spent per update.
        m[k] = ln == k ? d : m[k] * inv;
        idg = ln == k ? inv : idg;
#pragma unroll
        for (int j = k + 1; j < n; ++j) {
            if (!l_nz<D, CH>(j, k)) continue;  // L_jk == 0: no update (compile-time after unrolling)
            const float ljk = raw[j] * inv;
            m[j] = fmaf(-m[k], ljk, m[j]);  // fused, as the oracle's cholesky()
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // rows of L to LDS; lane j then holds column j (c[k] = L[k][j], k >= j)
    if (lane < n) {
#pragma unroll
        for (int c = 0; c < n; ++c)
            if (c <= lane) s.L[lane][c] = m[c];
        s.Linv[lane] = idg;
    }
    STAMP(6);
    // ---- 7. qdd = M^-1 rhs: forward on rows (registers), backward on columns
    if constexpr (EPW == 2) {
        // every lane solves the whole system from env-uniform LDS reads of L (no broadcast
        // chain: the L loads are independent of x and issue ahead; structural zeros
        // skipped), then keeps its own entry.  Per element the same operations in the same
        // order as the lane-distributed form below.
        if (lane < n) s.qf[lane] = x;  // (s.qf is scratch until the free velocity below)
        __syncthreads();
        float xv[n];
        uniform_solve<D, CH, n, Smem<D, B, ROWS>::LP>(s.qf, s.L, s.Linv, xv);
        x = 0.f;
#pragma unroll
        for (int i = 0; i < n; ++i) x = lane == i ? xv[i] : x;
        __syncthreads();
    } else {
#pragma unroll
    for (int i = 0; i < n; ++i) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        x = ln == i ? x * idg : x;
        const float xi = bc<EPW>(x, i);
        x = ln > i ? fmaf(-m[i], xi, x) : x;
    }
    __syncthreads();
    {
        float lc[n];
#pragma unroll
        for (int k = 0; k < n; ++k) lc[k] = (lane < n && k >= lane) ? s.L[k][lane] : 0.f;
#pragma unroll
        for (int i = n - 1; i >= 0; --i) {
            int ln = lane;
            asm volatile("" : "+v"(ln));
            x = ln == i ? x * idg : x;
            const float xi = bc<EPW>(x, i);
            x = ln < i ? fmaf(-lc[i], xi, x) : x;
        }
    }
    }
    // free velocity (classical velocity of the root origin after dt); lane i holds
    // qdd of natural index r = n-1-i, s.qf is in the natural order.  Lane b < B also runs
    // the contact pre-filter: body b's candidates may touch the ground only if their
    // bounding sphere (world centre C, radius rho, largest candidate radius rmax) reaches
    // within contact_offset + margin of it.  Plane: C_z - rho - rmax - rest.  Heightfield
    // (h piecewise linear with gradient norm <= G, normal n_z >= nmin): every candidate's
    // height above the triangle under it is >= C_z - h(C) - (1 + G) rho, so its separation
    // is >= nmin (C_z - h(C) - (1 + G) rho) - rmax - rest.  The test only skips candidates
    // that cannot be active: the selected contacts are the ones a full scan selects.
    uint32_t touch;
    {
        float wxv[3];
        cross3(w0, vO, wxv);
        const int r = n - 1 - lane;
        const int c = (r >= 0 ? r : 0) % 3;
        const float wl = c == 0 ? w0[0] : (c == 1 ? w0[1] : w0[2]);
        const float vl = c == 0 ? vO[0] : (c == 1 ? vO[1] : vO[2]);
        const float cl = c == 0 ? wxv[0] : (c == 1 ? wxv[1] : wxv[2]);
        if (lane < D) s.qf[r] = s.qd[r - 6] + dt * x;
        else if (lane < n - 3) s.qf[r] = vl + dt * (x + cl);
        else if (lane < n) s.qf[r] = wl + dt * x;
        bool may = false;
        if (lane < B) {
            s.u.sel.pwin[lane] = 0x7fffffff;
            const float* bs = mc.bs[lane];
            if (bs[3] >= 0.f) {
                float cw[3];
                matvec(s.R[lane], bs, cw);
                const float cz = cw[2] + s.p[lane][2];
                float gap;
                if (sp.hf) {
                    float nrm[3];
                    const float h = terrain_sample(sp, cw[0] + s.p[lane][0], cw[1] + s.p[lane][1], nrm);
                    gap = sp.hf_nmin * (cz - h - sp.hf_slope1 * bs[3]) - bs[4];
                } else {
                    gap = cz - bs[3] - bs[4];
                }
                may = gap - sp.rest_offset < sp.contact_offset + LGS_PREFILTER_MARGIN;
            }
        }
        // WAVE-uniform (two envs per wave: either env's bodies): the candidate loop below has a
        // barrier in it, so its trip through the chunks must not differ between the halves.  A
        // chunk run for the other env's bodies finds nothing the pre-filter ruled out (it only
        // skips candidates that cannot be active): the same contacts, bit for bit.
        const uint64_t mw = __ballot(may);
        touch = (uint32_t)mw | (uint32_t)(mw >> 32);
    }
    __syncthreads();
    STAMP(7);
    // ---- 8. constraint rows.  Fixed layout: contact slot c at rows 3c (normal), 3c+1,
    // 3c+2 (friction), c < CM; joint limit l at row 3*CM + l, l < LM, and the limits
    // beyond LM in the rows of the unused contact slots (3*nc ...).
    // Slot policy (the oracle's, oracle/lgs_oracle.c orc_substep_env): every touching
    // body first gets ONE slot for its first touching candidate (the primaries, in
    // candidate order: the feet's come first, Model.reorder_points), then the self
    // contacts take up to max_self slots (pair order), then the remaining touching ground
    // candidates fill what is left, in candidate order.  So two planted soles cannot
    // starve a knee, hip or pelvis on the ground of its contact row.  What does not fit
    // is counted (Drops, lgs_get_contact_stats).
    // Gauss-Seidel order: contacts ascending, then limits in DOF order.
    constexpr int CM = ROWS / 4, LM = ROWS - 3 * CM;
    const float beta = sp.beta;
    const int maxc = sp.max_contacts < CM ? sp.max_contacts : CM;
    int nc = 0, ncg = 0;  // contacts, of which the first ncg are ground contacts
    {
        // self contacts: lane per proxy pair, every pair tested; the first maxc in pair
        // order are staged
        int nsf = 0;
        if (sp.n_selfp > 0) {
            for (int base = 0; base < sp.n_selfp; base += WAVE / EPW) {
                const int q = base + lane;
                bool act = false;
                float pc[3] = {0.f, 0.f, 0.f}, nrm[3] = {0.f, 0.f, 1.f}, sep = 0.f;
                int ba = 0, bb = 0;
                if (q < sp.n_selfp) {
                    const float4* rec = sp.selfp + 4 * q;
                    const float4 r0 = rec[0], r1 = rec[1], r2 = rec[2], r3 = rec[3];
                    ba = __float_as_int(r1.w);
                    bb = __float_as_int(r3.w);
                    float Ra[9], Rb[9];
#pragma unroll
                    for (int t = 0; t < 9; ++t) { Ra[t] = s.R[ba][t]; Rb[t] = s.R[bb][t]; }
                    const float a0[3] = {r0.x, r0.y, r0.z}, a1[3] = {r0.w, r1.x, r1.y};
                    const float b0[3] = {r2.x, r2.y, r2.z}, b1[3] = {r2.w, r3.x, r3.y};
                    float pa0[3], pa1[3], pb0[3], pb1[3];
                    matvec(Ra, a0, pa0); matvec(Ra, a1, pa1); matvec(Rb, b0, pb0); matvec(Rb, b1, pb1);
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        pa0[k] += s.p[ba][k]; pa1[k] += s.p[ba][k];
                        pb0[k] += s.p[bb][k]; pb1[k] += s.p[bb][k];
                    }
                    float c1[3], c2[3];
                    seg_closest(pa0, pa1, pb0, pb1, c1, c2);
                    const float dx[3] = {c1[0] - c2[0], c1[1] - c2[1], c1[2] - c2[2]};
                    const float dist = sqrtf(dot3(dx, dx));
                    if (dist > 1e-9f) {
                        const float inv = 1.f / dist;
                        nrm[0] = dx[0] * inv; nrm[1] = dx[1] * inv; nrm[2] = dx[2] * inv;
                    }
                    const float ra = r1.z, rb = r3.z;
                    sep = dist - ra - rb - sp.rest_offset;
                    act = sep < sp.contact_offset;
#pragma unroll
                    for (int k = 0; k < 3; ++k) pc[k] = 0.5f * ((c1[k] - ra * nrm[k]) + (c2[k] + rb * nrm[k]));
                }
                const uint64_t mask = hballot<EPW>(act);
                const int slot = nsf + __popcll(mask & ((1ull << lane) - 1ull));
                if (act && slot < maxc) {
                    s.u.sel.sc_ab[slot][0] = ba; s.u.sel.sc_ab[slot][1] = bb;
                    float* t = s.u.sel.sc_tmp[slot];
                    t[0] = pc[0]; t[1] = pc[1]; t[2] = pc[2]; t[3] = sep;
                    t[4] = nrm[0]; t[5] = nrm[1]; t[6] = nrm[2];
                }
                nsf += __popcll(mask);
            }
        }
        // ground candidates: lane per candidate over the chunks that hold a body the
        // pre-filter kept.  A touching candidate is its body's primary when it is the
        // body's first touching candidate (LDS min of the candidate index over the chunks
        // so far: chunks run in index order); primaries go straight to their slots, the
        // others are staged in candidate order.
        int np = 0, nsec = 0;
        const int nch = (md.P + WAVE / EPW - 1) / (WAVE / EPW);
        for (int ch = 0; ch < nch; ++ch) {
            if (!(chunk_bodies<EPW>(mc, ch) & touch)) continue;  // (wave-uniform: touch above)
            const int k = ch * (WAVE / EPW) + lane;
            bool act = false;
            float c[3] = {0.f, 0.f, 0.f}, sep = 0.f, rad = 0.f, nrm[3] = {0.f, 0.f, 1.f};
            int b = 0;
            if (k < md.P) {
                b = md.pt_body[k];
                float pp[3] = {md.pt_pos[3 * k], md.pt_pos[3 * k + 1], md.pt_pos[3 * k + 2]};
                rad = md.pt_radius[k];
                float R[9];
#pragma unroll
                for (int t = 0; t < 9; ++t) R[t] = s.R[b][t];
                matvec(R, pp, c);
                c[0] += s.p[b][0]; c[1] += s.p[b][1]; c[2] += s.p[b][2];
                // signed distance of the point's sphere centre to the ground triangle's plane
                const float h = terrain_sample(sp, c[0], c[1], nrm);
                sep = (c[2] - h) * nrm[2] - rad - sp.rest_offset;
                act = sep < sp.contact_offset;
            }
            if (act) atomicMin(&s.u.sel.pwin[b], k);
            __syncthreads();
            const bool prim = act && s.u.sel.pwin[b] == k;
            const bool sec = act && !prim;
            const uint64_t pm = hballot<EPW>(prim), sm_ = hballot<EPW>(sec);
            const uint64_t below = (1ull << lane) - 1ull;
            const int ps = np + __popcll(pm & below), ss = nsec + __popcll(sm_ & below);
            const float pc[3] = {c[0] - rad * nrm[0], c[1] - rad * nrm[1], c[2] - rad * nrm[2]};
            if (prim && ps < maxc) {
                s.c_body[ps] = b;
                s.c_pt[ps][0] = pc[0]; s.c_pt[ps][1] = pc[1]; s.c_pt[ps][2] = pc[2];
                s.c_sep[ps] = sep;
                float t1[3] = {1.f, 0.f, 0.f}, t2[3] = {0.f, 1.f, 0.f};  // plane: +x, +y
                if (sp.hf) contact_tangents(nrm, t1, t2);
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    s.c_fr[ps][t] = nrm[t]; s.c_fr[ps][3 + t] = t1[t]; s.c_fr[ps][6 + t] = t2[t];
                }
            }
            if (sec && ss < maxc) {
                s.u.sel.sec_body[ss] = b;
                float* t = s.u.sel.sec[ss];
                t[0] = pc[0]; t[1] = pc[1]; t[2] = pc[2]; t[3] = sep;
                t[4] = nrm[0]; t[5] = nrm[1]; t[6] = nrm[2];
            }
            np += __popcll(pm);
            nsec += __popcll(sm_);
        }
        const int npg = np < maxc ? np : maxc;
        int nsc = nsf < sp.max_self ? nsf : sp.max_self;
        if (nsc > maxc - npg) nsc = maxc - npg;
        const int nsu = nsec < maxc - npg - nsc ? nsec : maxc - npg - nsc;
        ncg = npg + nsu;
        nc = ncg + nsc;
        count_drops(sp, lane, 0, np - npg);
        count_drops(sp, lane, 1, nsf - nsc);
        __syncthreads();
        if (lane < nsu) {  // staged ground contacts after the primaries
            const int slot = npg + lane;
            const float* t = s.u.sel.sec[lane];
            s.c_body[slot] = s.u.sel.sec_body[lane];
            s.c_pt[slot][0] = t[0]; s.c_pt[slot][1] = t[1]; s.c_pt[slot][2] = t[2];
            s.c_sep[slot] = t[3];
            const float nrm[3] = {t[4], t[5], t[6]};
            float t1[3] = {1.f, 0.f, 0.f}, t2[3] = {0.f, 1.f, 0.f};
            if (sp.hf) contact_tangents(nrm, t1, t2);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                s.c_fr[slot][k] = nrm[k]; s.c_fr[slot][3 + k] = t1[k]; s.c_fr[slot][6 + k] = t2[k];
            }
        } else if (lane >= CM && lane < CM + nsc) {  // then the self contacts
            const int j = lane - CM, slot = ncg + j;
            s.c_body[slot] = s.u.sel.sc_ab[j][0];
            s.c_body2[slot] = s.u.sel.sc_ab[j][1];
            const float* t = s.u.sel.sc_tmp[j];
            s.c_pt[slot][0] = t[0]; s.c_pt[slot][1] = t[1]; s.c_pt[slot][2] = t[2];
            s.c_sep[slot] = t[3];
            const float nrm[3] = {t[4], t[5], t[6]};
            float t1[3], t2[3];
            self_tangents(nrm, t1, t2);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                s.c_fr[slot][k] = nrm[k]; s.c_fr[slot][3 + k] = t1[k]; s.c_fr[slot][6 + k] = t2[k];
            }
        }
        __syncthreads();  // the staging (s.u.sel) is dead before the constraint rows (s.u.con) are written
    }
    // joint limits: the first max_limit in DOF order take the limit block, the next ones the
    // rows of the unused contact slots; the rest are counted (Drops::limits)
    int nlimit, nover;
    {
        bool lo_act = false, hi_act = false;
        float gap = 0.f;
        if (lane < D) {
            const float qj = s.q[lane], lo = mc.lo[lane], hi = mc.hi[lane];
            const float qn = qj + dt * s.qf[6 + lane];
            if (qn < lo) { lo_act = true; gap = qj - lo; }
            else if (qn > hi) { hi_act = true; gap = hi - qj; }
        }
        const bool act = lo_act || hi_act;
        const uint64_t mask = hballot<EPW>(act);
        const int slot = __popcll(mask & ((1ull << lane) - 1ull));
        int max_limit = sp.max_rows - 3 * sp.max_contacts;
        if (max_limit > LM) max_limit = LM;
        const int nl = __popcll(mask);
        nlimit = nl < max_limit ? nl : max_limit;
        nover = nl - nlimit < 3 * (maxc - nc) ? nl - nlimit : 3 * (maxc - nc);
        count_drops(sp, lane, 2, nl - nlimit - nover);
        if (act && slot < nlimit + nover) {
            const int r = slot < nlimit ? 3 * CM + slot : 3 * nc + (slot - nlimit);
            float* row = s.u.con.Y[r];
            for (int i = 0; i < n; ++i) row[i] = 0.f;
            row[6 + lane] = lo_act ? 1.f : -1.f;
            s.tgt[r] = gap >= 0.f ? -gap * idt : -beta * gap * idt;
        }
    }
    __syncthreads();
    STAMP(8);
    // contact rows (lane per row): J row into Y[r]
    if (lane < 3 * nc) {
        const int cc = lane / 3, dd = lane % 3;
        const float d[3] = {s.c_fr[cc][3 * dd], s.c_fr[cc][3 * dd + 1], s.c_fr[cc][3 * dd + 2]};
        const int b = s.c_body[cc];
        float pc[3] = {s.c_pt[cc][0], s.c_pt[cc][1], s.c_pt[cc][2]};
        float r[3] = {pc[0] - O[0], pc[1] - O[1], pc[2] - O[2]}, rxd[3];
        cross3(r, d, rxd);
        float* row = s.u.con.Y[lane];
        for (int i = 0; i < n; ++i) row[i] = 0.f;
        const bool self = cc >= ncg;
        if (!self) {  // ground: J(pc) d of body b; a self contact's base columns cancel to 0
            row[0] = rxd[0]; row[1] = rxd[1]; row[2] = rxd[2];
            row[3] = d[0]; row[4] = d[1]; row[5] = d[2];
        }
        const int dep = mc.depth[b];
        for (int l = 1; l <= dep; ++l) {
            const int a = mc.chain[b][l];
            const int j = mc.dof[a];
            if (j < 0) continue;
            float rp[3] = {pc[0] - s.p[a][0], pc[1] - s.p[a][1], pc[2] - s.p[a][2]}, t[3];
            float aw[3] = {s.aw[a][0], s.aw[a][1], s.aw[a][2]};
            cross3(aw, rp, t);
            row[6 + j] = dot3(d, t);
        }
        if (self) {  // minus J(pc) d of the second body (shared ancestors cancel exactly)
            const int b2 = s.c_body2[cc];
            const int dep2 = mc.depth[b2];
            for (int l = 1; l <= dep2; ++l) {
                const int a = mc.chain[b2][l];
                const int j = mc.dof[a];
                if (j < 0) continue;
                float rp[3] = {pc[0] - s.p[a][0], pc[1] - s.p[a][1], pc[2] - s.p[a][2]}, t[3];
                float aw[3] = {s.aw[a][0], s.aw[a][1], s.aw[a][2]};
                cross3(aw, rp, t);
                row[6 + j] = row[6 + j] - dot3(d, t);
            }
        }
        const float sep = s.c_sep[cc];
        s.tgt[lane] = dd != 0 ? 0.f : (sep >= 0.f ? -sep * idt : fminf(-beta * sep * idt, sp.max_depen));
    }
    __syncthreads();
    STAMP(9);
    // rows in use: the contacts' and the overflow limits' (3nc ...), the limit block's
    const bool used = (lane < 3 * nc + nover) || (lane >= 3 * CM && lane < 3 * CM + nlimit);
    // ---- 9. v = J qf ; Y = L^-1 J^T (lane r; L entries broadcast from their row lanes)
    float v = 0.f;
    float dg = 0.f;  // A_rr = |Y_r|^2 of this lane's row (the MFMA's fp32 chain, k ascending)
    {
        float y[n];
#pragma unroll
        for (int i = 0; i < n; ++i) y[i] = used ? s.u.con.Y[lane][i] : 0.f;
#pragma unroll
        for (int i = 0; i < n; ++i) v = fmaf(y[i], s.qf[i], v);
        // leaves-first order (register renaming only), then row i of L and 1/L_ii as
        // wave-uniform LDS reads (16-byte row loads on the LDS pipe) instead of ~170
        // v_readlane broadcasts on the VALU; structurally zero L entries are skipped
        float yp[n];
#pragma unroll
        for (int i = 0; i < n; ++i) yp[i] = y[n - 1 - i];
#pragma unroll
        for (int i = 0; i < n; ++i) {
            const float* Li = s.L[i];
            float t = yp[i];
#pragma unroll
            for (int k = 0; k < i; ++k)
                if (l_nz<D, CH>(i, k)) t = fmaf(-Li[k], yp[k], t);
            yp[i] = t * s.Linv[i];
            // pinned per row: with the sparse joint rows independent the scheduler
            // otherwise runs them all at once and spills at the 128-VGPR (4 waves/SIMD)
            // budget
            if (CH > 0) asm volatile("" : "+v"(yp[i]));
        }
#pragma unroll
        for (int i = 0; i < n; ++i) dg = fmaf(yp[i], yp[i], dg);
        if (lane < ROWS) {
#pragma unroll
            for (int i = 0; i < n; ++i) s.u.con.Y[lane][i] = yp[i];
        }
    }
    __syncthreads();
    STAMP(10);
    // ---- 10. A = Y Y^T on the matrix cores, 32x32 tiles, k = 2 per instruction.
    // Lane l feeds Y[row0 + (l&31)][2t + (l>>5)]; D element (row, col) is the fp32
    // fma chain over k ascending (the oracle's loop).  Unused rows are zero.
    // ---- 11. projected Gauss-Seidel.  Lane s holds column s of A (registers) and
    // v_s; per-row lambda are wave-uniform (SGPRs).  One contact = normal row,
    // then its friction pair against the post-normal velocities.
    static_assert(EPW == 1 || ROWS <= 32, "two envs per wave need one A tile per env");
    const int li = threadIdx.x & 31, lk = threadIdx.x >> 5;  // the tiles take the whole wave
    float acol[ROWS];
    if constexpr (ROWS <= 32 && EPW == 2) {
        // one tile per env, both fed by all 64 lanes; lane l of env h owns column l&31 of
        // that env's A: for env 0 its own accumulators hold rows (t&3)+8(t>>2) and lane
        // l+32's rows +4; for env 1 the other way round.  Each lane sends the other half the
        // accumulator it needs (one shuffle per element, as for one env).
        floatx16 acc0, acc1;
#pragma unroll
        for (int t = 0; t < 16; ++t) { acc0[t] = 0.f; acc1[t] = 0.f; }
#pragma unroll
        for (int st = 0; st < (n + 1) / 2; ++st) {
            const int kk = 2 * st + lk;
            const float a0 = (li < ROWS && kk < n) ? sm[0].u.con.Y[li][kk] : 0.f;
            const float a1 = (li < ROWS && kk < n) ? sm[1].u.con.Y[li][kk] : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, a0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, a1, acc1, 0, 0, 0);
        }
        const bool up = threadIdx.x >= 32;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int r0 = (t & 3) + 8 * (t >> 2);
            const float own = up ? acc1[t] : acc0[t];
            const float other = __shfl_xor(up ? acc0[t] : acc1[t], 32);
            if (r0 < ROWS) acol[r0] = up ? other : own;
            if (r0 + 4 < ROWS) acol[r0 + 4] = up ? own : other;
        }
        STAMP(11);
    } else if constexpr (ROWS <= 32) {
        // one tile; lane l < 32 owns column l: rows (t&3)+8(t>>2) from its own
        // accumulators, rows +4 from lane l+32's.
        floatx16 acc;
#pragma unroll
        for (int t = 0; t < 16; ++t) acc[t] = 0.f;
#pragma unroll
        for (int st = 0; st < (n + 1) / 2; ++st) {
            const int kk = 2 * st + lk;
            const float a = (li < ROWS && kk < n) ? s.u.con.Y[li][kk] : 0.f;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, acc, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int r0 = (t & 3) + 8 * (t >> 2);
            const float other = __shfl_xor(acc[t], 32);
            if (r0 < ROWS) acol[r0] = acc[t];
            if (r0 + 4 < ROWS) acol[r0 + 4] = other;
        }
        STAMP(11);
    } else {
        // up to 64 rows, one env: two 32-column blocks.  Lane l owns column l; for each row
        // block ti the wave computes the tiles (ti, 0) and (ti, 1) -- the symmetric one
        // too, so that every lane's column comes out of accumulators: in tile (ti, tj) lane
        // l holds column 32 tj + (l & 31), rows (t&3)+8(t>>2)+4(l>>5), and its partner
        // l ^ 32 the other half.  (A^T tile entries are the same products in the same order:
        // bit-identical to the mirrored tile.)  A never goes through LDS.
        const int hi_row = nlimit > 0 ? 3 * CM + nlimit : 3 * nc + nover;
        const int nt = (hi_row + 31) >> 5;
        const bool up = threadIdx.x >= 32;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acol[r] = 0.f;
#pragma unroll
        for (int ti = 0; ti < (ROWS + 31) / 32; ++ti) {
            if (ti >= nt) break;  // (uniform)
            floatx16 acc0, acc1;
#pragma unroll
            for (int t = 0; t < 16; ++t) { acc0[t] = 0.f; acc1[t] = 0.f; }
            const int ra = 32 * ti + li;
#pragma unroll
            for (int st = 0; st < (n + 1) / 2; ++st) {
                const int kk = 2 * st + lk;
                const float a = (ra < ROWS && kk < n) ? s.u.con.Y[ra][kk] : 0.f;
                const float b0 = (li < ROWS && kk < n) ? s.u.con.Y[li][kk] : 0.f;
                const float b1 = (32 + li < ROWS && kk < n) ? s.u.con.Y[32 + li][kk] : 0.f;
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
            }
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int r0 = 32 * ti + (t & 3) + 8 * (t >> 2);
                const float o0 = __shfl_xor(acc0[t], 32), o1 = __shfl_xor(acc1[t], 32);
                const float own = up ? acc1[t] : acc0[t], other = up ? o1 : o0;
                if (r0 < ROWS) acol[r0] = up ? other : own;
                if (r0 + 4 < ROWS) acol[r0 + 4] = up ? own : other;
            }
        }
        STAMP(11);
    }
    float lam = 0.f;  // one env per wave: lane r holds lambda_r (one VGPR; broadcast when read)
    // two envs per wave: every lane holds every lambda of its env (the values are uniform
    // over the env's lanes), so the sweep reads them from registers instead of broadcasts
    float lamv[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) lamv[r] = 0.f;
    {
        const float mu = 0.5f * (sp.ground_friction + shape_mu);  // ground contacts
        const float mus = shape_mu;  // self contacts: both shapes carry the env's friction
        float tg = used ? s.tgt[lane] : 0.f;
        // the diagonal comes from the lane's own row (above), not a 32-way select over
        // acol (32 lane masks, which spilled SGPRs into VGPR lanes)
        float inv = used ? 1.f / (dg + 1e-9f) : 0.f;
        if constexpr (EPW == 2) {
            // the sweep-invariant per-row constants broadcast once (256 VGPRs at 2 waves/SIMD
            // hold them): targets, 1/A_rr, a contact's normal-friction couplings.  The
            // dependency chain of a contact update then carries 3 broadcasts (v) instead of 12.
            float ptg[ROWS], pinv[ROWS], pa1[CM], pa2[CM];
#pragma unroll
            for (int r = 0; r < ROWS; ++r) { ptg[r] = 0.f; pinv[r] = 0.f; }
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                pa1[c] = 0.f; pa2[c] = 0.f;
                if (c < nc) {
                    const int r = 3 * c;
                    ptg[r] = bc<EPW>(tg, r);
                    pinv[r] = bc<EPW>(inv, r); pinv[r + 1] = bc<EPW>(inv, r + 1); pinv[r + 2] = bc<EPW>(inv, r + 2);
                    pa1[c] = bc<EPW>(acol[r], r + 1); pa2[c] = bc<EPW>(acol[r], r + 2);
                }
            }
#pragma unroll
            for (int l = 0; l < LM; ++l)
                if (l < nlimit) {
                    const int r = 3 * CM + l;
                    ptg[r] = bc<EPW>(tg, r);
                    pinv[r] = bc<EPW>(inv, r);
                }
            for (int it = 0; it < sp.iters; ++it) {
                // opaque row counts per sweep: the per-row guards are recomputed (one s_cmp
                // each) instead of held across the sweeps as hoisted lane masks (SGPR spills)
                int ncs = nc, ncgs = ncg, nls = nlimit, nos = nover;
                asm volatile("" : "+v"(ncs), "+v"(ncgs), "+v"(nls), "+v"(nos));
#pragma unroll
                for (int c = 0; c < CM; ++c) {
                    if (c < ncs) {
                        const int r = 3 * c;
                        const float lno = lamv[r], l1o = lamv[r + 1], l2o = lamv[r + 2];
                        const float vn = bc<EPW>(v, r), v1 = bc<EPW>(v, r + 1), v2 = bc<EPW>(v, r + 2);
                        const float ln = fmaxf(0.f, lno + (ptg[r] - vn) * pinv[r]);
                        const float dn = ln - lno;
                        v = fmaf(acol[r], dn, v);
                        const float v1n = fmaf(pa1[c], dn, v1);
                        const float v2n = fmaf(pa2[c], dn, v2);
                        const float lim = (c < ncgs ? mu : mus) * ln;
                        float l1 = l1o - v1n * pinv[r + 1];
                        float l2 = l2o - v2n * pinv[r + 2];
                        // cone test on squared norms (the oracle's): sqrt and division only
                        // when the impulse is projected onto the cone
                        const float n2 = l1 * l1 + l2 * l2;
                        if (n2 > lim * lim) {
                            const float nrm = sqrtf(n2);
                            const float sc = nrm > 0.f ? lim / nrm : 0.f;
                            l1 *= sc; l2 *= sc;
                        }
                        const float d1 = l1 - l1o, d2 = l2 - l2o;
                        v = fmaf(acol[r + 2], d2, fmaf(acol[r + 1], d1, v));
                        lamv[r] = ln; lamv[r + 1] = l1; lamv[r + 2] = l2;
                    }
                }
#pragma unroll
                for (int l = 0; l < LM; ++l) {
                    if (l < nls) {
                        const int r = 3 * CM + l;
                        const float lo = lamv[r];
                        const float ln = fmaxf(0.f, lo + (ptg[r] - bc<EPW>(v, r)) * pinv[r]);
                        v = fmaf(acol[r], ln - lo, v);
                        lamv[r] = ln;
                    }
                }
                if (nos > 0) {  // limits in the rows of unused contact slots (rare: their
                                  // constants are broadcast per use, no registers held for them;
                                  // opaque copies keep LICM from hoisting the 2 x 3CM invariant
                                  // broadcasts out of the sweep loop into live registers)
                    const float tgo = tg, invo = inv;
#pragma unroll
                    for (int r = 0; r < 3 * CM; ++r)
                        if (r >= 3 * ncs && r < 3 * ncs + nos) {
                            const float lo = lamv[r];
                            const float ln = fmaxf(0.f, lo + (bc<EPW>(tgo, r) - bc<EPW>(v, r)) * bc<EPW>(invo, r));
                            v = fmaf(acol[r], ln - lo, v);
                            lamv[r] = ln;
                        }
                }
            }
        } else
        for (int it = 0; it < sp.iters; ++it) {
            // Opaque per sweep: otherwise LICM hoists ~64 loop-invariant readlanes
            // (targets, 1/A_rr, normal-friction couplings) out of the sweep loop; with
            // the SGPRs full they occupy VGPRs and the kernel spills to scratch.
            asm volatile("" : "+v"(tg), "+v"(inv));
#pragma unroll
            for (int r = 0; r < ROWS; ++r) asm volatile("" : "+v"(acol[r]));
            // opaque lane id per sweep: the row masks (lane == r) are recomputed (one v_cmp
            // each) instead of held across the sweeps in SGPRs, which spilled
            int lid = lane;
            asm volatile("" : "+v"(lid));
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c < nc) {
                    const int r = 3 * c;
                    const float lno = bc<EPW>(lam, r), l1o = bc<EPW>(lam, r + 1), l2o = bc<EPW>(lam, r + 2);
                    const float vn = bc<EPW>(v, r), v1 = bc<EPW>(v, r + 1), v2 = bc<EPW>(v, r + 2);
                    const float ln = fmaxf(0.f, lno + (bc<EPW>(tg, r) - vn) * bc<EPW>(inv, r));
                    const float dn = ln - lno;
                    v = fmaf(acol[r], dn, v);
                    const float v1n = fmaf(bc<EPW>(acol[r], r + 1), dn, v1);
                    const float v2n = fmaf(bc<EPW>(acol[r], r + 2), dn, v2);
                    const float lim = (c < ncg ? mu : mus) * ln;
                    float l1 = l1o - v1n * bc<EPW>(inv, r + 1);
                    float l2 = l2o - v2n * bc<EPW>(inv, r + 2);
                    const float n2 = l1 * l1 + l2 * l2;
                    if (n2 > lim * lim) {
                        const float nrm = sqrtf(n2);
                        const float sc = nrm > 0.f ? lim / nrm : 0.f;
                        l1 *= sc; l2 *= sc;
                    }
                    const float d1 = l1 - l1o, d2 = l2 - l2o;
                    v = fmaf(acol[r + 2], d2, fmaf(acol[r + 1], d1, v));
                    lam = lid == r ? ln : (lid == r + 1 ? l1 : (lid == r + 2 ? l2 : lam));
                }
            }
#pragma unroll
            for (int l = 0; l < LM; ++l) {
                if (l < nlimit) {
                    const int r = 3 * CM + l;
                    const float lo = bc<EPW>(lam, r);
                    const float ln = fmaxf(0.f, lo + (bc<EPW>(tg, r) - bc<EPW>(v, r)) * bc<EPW>(inv, r));
                    v = fmaf(acol[r], ln - lo, v);
                    lam = lid == r ? ln : lam;
                }
            }
            if (nover > 0) {  // limits in the rows of unused contact slots
#pragma unroll
                for (int r = 0; r < 3 * CM; ++r)
                    if (r >= 3 * nc && r < 3 * nc + nover) {
                        const float lo = bc<EPW>(lam, r);
                        const float ln = fmaxf(0.f, lo + (bc<EPW>(tg, r) - bc<EPW>(v, r)) * bc<EPW>(inv, r));
                        v = fmaf(acol[r], ln - lo, v);
                        lam = lid == r ? ln : lam;
                    }
            }
        }
    }
    STAMP(12);
    // ---- 12. z = Y^T lambda ; dq = L^-T z (register columns) ; qd' = qf + dq
    // (the broadcasts stay outside the lane < n test: ds_bpermute reads nothing from a lane
    // that is switched off)
    float z = 0.f;
#pragma unroll
    for (int c = 0; c < CM; ++c)
        if (c < nc) {
            const float l0 = EPW == 2 ? lamv[3 * c] : bc<EPW>(lam, 3 * c);
            const float l1 = EPW == 2 ? lamv[3 * c + 1] : bc<EPW>(lam, 3 * c + 1);
            const float l2 = EPW == 2 ? lamv[3 * c + 2] : bc<EPW>(lam, 3 * c + 2);
            if (lane < n) {
                z = fmaf(s.u.con.Y[3 * c][lane], l0, z);
                z = fmaf(s.u.con.Y[3 * c + 1][lane], l1, z);
                z = fmaf(s.u.con.Y[3 * c + 2][lane], l2, z);
            }
        }
#pragma unroll
    for (int l = 0; l < LM; ++l)
        if (l < nlimit) {
            const float ll = EPW == 2 ? lamv[3 * CM + l] : bc<EPW>(lam, 3 * CM + l);
            if (lane < n) z = fmaf(s.u.con.Y[3 * CM + l][lane], ll, z);
        }
    if (nover > 0)
#pragma unroll
        for (int r = 0; r < 3 * CM; ++r)
            if (r >= 3 * nc && r < 3 * nc + nover) {
                const float ll = EPW == 2 ? lamv[r] : bc<EPW>(lam, r);
                if (lane < n) z = fmaf(s.u.con.Y[r][lane], ll, z);
            }
    if constexpr (EPW == 2) {  // the uniform backward solve of step 7
        __syncthreads();  // (every read of s.tgt / the limit rows is done: reuse s.tgt as scratch)
        if (lane < n) s.tgt[lane] = z;
        __syncthreads();
        float zv[n];
        uniform_back<D, CH, n, Smem<D, B, ROWS>::LP>(s.tgt, s.L, s.Linv, zv);
        z = 0.f;
#pragma unroll
        for (int i = 0; i < n; ++i) z = lane == i ? zv[i] : z;
    } else {
        float lc[n];
#pragma unroll
        for (int k = 0; k < n; ++k) lc[k] = (lane < n && k >= lane) ? s.L[k][lane] : 0.f;
#pragma unroll
        for (int i = n - 1; i >= 0; --i) {
            int ln = lane;
            asm volatile("" : "+v"(ln));
            z = ln == i ? z * idg : z;
            const float zi = bc<EPW>(z, i);
            z = ln < i ? fmaf(-lc[i], zi, z) : z;
        }
    }
    // back to the natural order: lane i < n holds qd' of index n-1-i
    float qn = (lane < n) ? s.qf[n - 1 - lane] + z : 0.f;
    if (sp.clamp_qd && lane < D) {
        const float lim = mc.vl[D - 1 - lane];
        if (lim > 0.f) qn = fminf(fmaxf(qn, -lim), lim);
    }
    // contact forces of this substep
    {
        float F[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < CM; ++c)
            if (c < nc) {
                const float ln = EPW == 2 ? lamv[3 * c] : bc<EPW>(lam, 3 * c);
                const float l1 = EPW == 2 ? lamv[3 * c + 1] : bc<EPW>(lam, 3 * c + 1);
                const float l2 = EPW == 2 ? lamv[3 * c + 2] : bc<EPW>(lam, 3 * c + 2);
                if (c >= ncg && s.c_body2[c] == lane) {  // self contact: the reaction on the second body
                    const float* fr = s.c_fr[c];
#pragma unroll
                    for (int t = 0; t < 3; ++t) F[t] -= (ln * fr[t] + l1 * fr[3 + t] + l2 * fr[6 + t]) * idt;
                }
                if (s.c_body[c] == lane) {
                    if (sp.hf || c >= ncg) {
                        const float* fr = s.c_fr[c];  // world force = ln n + l1 t1 + l2 t2
#pragma unroll
                        for (int t = 0; t < 3; ++t) F[t] += (ln * fr[t] + l1 * fr[3 + t] + l2 * fr[6 + t]) * idt;
                    } else {  // plane: the same numbers (n = z, t1 = x, t2 = y exactly)
                        F[0] += l1 * idt; F[1] += l2 * idt; F[2] += ln * idt;
                    }
                }
            }
        if (lane < B) { s.cf[lane][0] = F[0]; s.cf[lane][1] = F[1]; s.cf[lane][2] = F[2]; }
    }
    STAMP(13);
    // ---- 13. integrate
    const float qw0 = bc<EPW>(qn, n - 1), qw1 = bc<EPW>(qn, n - 2), qw2 = bc<EPW>(qn, n - 3);
    const float qv0 = bc<EPW>(qn, n - 4), qv1 = bc<EPW>(qn, n - 5), qv2 = bc<EPW>(qn, n - 6);
    __syncthreads();
    if (lane < D) {
        const int j = D - 1 - lane;
        s.qd[j] = qn;
        s.q[j] = s.q[j] + dt * qn;
    }
    if (lane == 0) {
        float* rt = s.root;
        rt[0] += dt * qv0; rt[1] += dt * qv1; rt[2] += dt * qv2;
        float* q = rt + 3;
        const float w[3] = {qw0, qw1, qw2};
        float dq[4];
        dq[0] = 0.5f * dt * (q[3] * w[0] + (w[1] * q[2] - w[2] * q[1]));
        dq[1] = 0.5f * dt * (q[3] * w[1] + (w[2] * q[0] - w[0] * q[2]));
        dq[2] = 0.5f * dt * (q[3] * w[2] + (w[0] * q[1] - w[1] * q[0]));
        dq[3] = 0.5f * dt * (-(w[0] * q[0] + w[1] * q[1] + w[2] * q[2]));
        float nn = 0.f;
        for (int k = 0; k < 4; ++k) { q[k] += dq[k]; nn += q[k] * q[k]; }
        nn = 1.f / sqrtf(nn);
        for (int k = 0; k < 4; ++k) q[k] *= nn;
        float R[9], c[3], wc[3];
        quat_to_mat(q, R);
        matvec(R, mc.com[0], c);
        cross3(w, c, wc);
        rt[10] = w[0]; rt[11] = w[1]; rt[12] = w[2];
        rt[7] = qv0 + wc[0]; rt[8] = qv1 + wc[1]; rt[9] = qv2 + wc[2];
    }
    __syncthreads();
    STAMP(14);
}

// Workgroups are dealt round-robin over the 8 XCDs (each with its own L2).  Map
// them so every XCD owns one contiguous env range: small per-env fields (reward,
// reset byte, commands, counters) then share cache lines within one L2 instead
// of being dirtied and written back by up to 8 (bijective for any grid size,
// MI355X guide §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_env(int b, int nwg) {
    const int xcd = b % 8, q = nwg / 8, r = nwg % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// rigid body states [B][13] of the block's env into global memory
template <int D, int B, int ROWS, int EPW>
__device__ void body_states(Smem<D, B, ROWS>& s, const ModelCache<D, B>& mc, float* rbs_out, int Br,
                            unsigned mask = 0u) {
    const int lane = hl<EPW>();
    if (lane < Br && (!mask || ((mask >> lane) & 1u))) {  // mask: the rows the task reads (0: all)
        float R[9], p[3], aw[3] = {0.f, 0.f, 0.f};
        quat_to_mat(s.root + 3, R);
        p[0] = s.root[0]; p[1] = s.root[1]; p[2] = s.root[2];
        const float O[3] = {p[0], p[1], p[2]};
        float c0[3];
        matvec(R, mc.com[0], c0);
        // the root COM offset as (O + R c) - O, the oracle's (and substep()'s) arithmetic
        float rc[3] = {(O[0] + c0[0]) - O[0], (O[1] + c0[1]) - O[1], (O[2] + c0[2]) - O[2]};
        float w[3] = {s.root[10], s.root[11], s.root[12]}, t[3];
        cross3(w, rc, t);
        float Vw[3] = {w[0], w[1], w[2]};
        float Vv[3] = {s.root[7] - t[0], s.root[8] - t[1], s.root[9] - t[2]};
        const int d = mc.depth[lane];
        for (int l = 1; l <= d; ++l) {
            const int a = mc.chain[lane][l];
            float Rj[9], tp[3];
            matmul(R, mc.jr[a], Rj);
            matvec(R, mc.jp[a], tp);
            p[0] += tp[0]; p[1] += tp[1]; p[2] += tp[2];
            const int j = mc.dof[a];
            if (j >= 0) {
                matvec(Rj, mc.ax[a], aw);
                float Ra[9];
                axis_angle(mc.ax[a], s.q[j], Ra);
                matmul(Rj, Ra, R);
                const float qd = s.qd[j];
                float rp[3] = {p[0] - O[0], p[1] - O[1], p[2] - O[2]}, sv[3];
                cross3(rp, aw, sv);
#pragma unroll
                for (int k = 0; k < 3; ++k) { Vw[k] += aw[k] * qd; Vv[k] += sv[k] * qd; }
            } else {
#pragma unroll
                for (int k = 0; k < 9; ++k) R[k] = Rj[k];
            }
        }
        float c[3];
        matvec(R, mc.com[lane], c);
        float r[3] = {p[0] + c[0] - O[0], p[1] + c[1] - O[1], p[2] + c[2] - O[2]}, wr[3];
        cross3(Vw, r, wr);
        float* o = rbs_out + 13 * lane;
        o[0] = p[0]; o[1] = p[1]; o[2] = p[2];
        float qq[4];
        mat_to_quat(R, qq);
        o[3] = qq[0]; o[4] = qq[1]; o[5] = qq[2]; o[6] = qq[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) { o[7 + k] = Vv[k] + wr[k]; o[10 + k] = Vw[k]; }
    }
}

// PAD: the model may be padded to the kernel's shape (the generic instantiations); else its
// sizes are the template's and every bound below is a compile-time constant
template <int D, int B, int ROWS, int EPW, bool PAD = false>
__device__ __forceinline__ void load_state(Smem<D, B, ROWS>& s, const DevState& st, const DevModel& md, int e) {
    const int Dr = PAD ? md.Dr : D;
    const int lane = hl<EPW>();
    if (lane < 13) s.root[lane] = st.root[13 * e + lane];
    if (lane < 2 * D) {  // (a padded model's inert DOFs rest at 0)
        const float v = lane < 2 * Dr ? st.dofs[(size_t)2 * Dr * e + lane] : 0.f;
        if (lane & 1) s.qd[lane >> 1] = v; else s.q[lane >> 1] = v;
    }
}
template <int D, int B, int ROWS, int EPW, bool PAD = false>
__device__ __forceinline__ void store_state(Smem<D, B, ROWS>& s, const DevState& st, const DevModel& md, int e) {
    int lane = hl<EPW>();
    asm volatile("" : "+v"(lane));  // recompute the lane indices here (no value kept live from load_state)
    if (lane < 13) st.root[13 * e + lane] = s.root[lane];
    const int Dr = PAD ? md.Dr : D, Br = PAD ? md.Br : B;
    if (lane < 2 * Dr) st.dofs[(size_t)2 * Dr * e + lane] = (lane & 1) ? s.qd[lane >> 1] : s.q[lane >> 1];
    for (int i = lane; i < 3 * Br; i += WAVE / EPW) st.cforce[(size_t)3 * Br * e + i] = (&s.cf[0][0])[i];
}

// ---------------------------------------------------------- kernels --------
template <int D, int B, int ROWS, int CH, bool PAD = false>
__global__ __launch_bounds__(WAVE) void k_simulate(DevModel md, DevSim sp, DevState st, int N) {
    __shared__ Smem<D, B, ROWS> s;
    __shared__ ModelCache<D, B> mc;
    const int e = xcd_env(blockIdx.x, gridDim.x);
    if (e >= N) return;
    load_model(mc, md);
    const int Dr = PAD ? md.Dr : D, Br = PAD ? md.Br : B;
    load_state<D, B, ROWS, 1, PAD>(s, st, md, e);
    if (threadIdx.x < D)
        s.tau[threadIdx.x] = threadIdx.x < Dr ? st.torques_in[(size_t)Dr * e + threadIdx.x] : 0.f;
    __syncthreads();
    substep<D, B, ROWS, CH, 1, PAD>(&s, mc, md, sp, st.added_mass ? st.added_mass[e] : 0.f, st.friction ? st.friction[e] : 1.f);
    store_state<D, B, ROWS, 1, PAD>(s, st, md, e);
    if (st.rbs) body_states<D, B, ROWS, 1>(s, mc, st.rbs + (size_t)13 * Br * e, Br);
}

template <int D, int B, int ROWS, int CH, bool PAD = false>
__global__ __launch_bounds__(WAVE) void k_fk(DevModel md, DevState st, int N) {
    __shared__ Smem<D, B, ROWS> s;
    __shared__ ModelCache<D, B> mc;
    const int e = xcd_env(blockIdx.x, gridDim.x);
    if (e >= N) return;
    load_model(mc, md);
    const int Br = PAD ? md.Br : B;
    load_state<D, B, ROWS, 1, PAD>(s, st, md, e);
    __syncthreads();
    body_states<D, B, ROWS, 1>(s, mc, st.rbs + (size_t)13 * Br * e, Br);
}

struct DevEnv {
    lgs_env_buffers b;
};

// torch.remainder-style modulo for positive divisor
__device__ __forceinline__ float fmod_pos(float a, float b) {
    float m = fmodf(a, b);
    if (m != 0.f && m < 0.f) m += b;
    return m;
}

__device__ __forceinline__ void quat_rotate_inverse(const float* q, const float* v, float* o) {
    float w = q[3];
    float s = 2.0f * w * w - 1.0f;
    float c[3];
    cross3(q, v, c);
    float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) o[k] = v[k] * s - c[k] * w * 2.0f + q[k] * d * 2.0f;
}

__device__ __forceinline__ void resample_commands(const lgs_task_params& T, float* cmd, uint64_t seed, uint32_t env,
                                                  uint32_t step, uint32_t stream) {
    cmd[0] = rand_range(T.cmd_lin_vel_x[0], T.cmd_lin_vel_x[1], philox_uniform(seed, env, step, stream, 0));
    cmd[1] = rand_range(T.cmd_lin_vel_y[0], T.cmd_lin_vel_y[1], philox_uniform(seed, env, step, stream, 1));
    if (T.heading_command)
        cmd[3] = rand_range(T.cmd_heading[0], T.cmd_heading[1], philox_uniform(seed, env, step, stream, 2));
    else
        cmd[2] = rand_range(T.cmd_ang_vel_yaw[0], T.cmd_ang_vel_yaw[1], philox_uniform(seed, env, step, stream, 2));
    float nrm = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]);
    float keep = nrm > 0.2f ? 1.f : 0.f;
    cmd[0] *= keep; cmd[1] *= keep;
}

// ------------------------------------------------ post-physics (scalar) ----
// legged_robot.py:673-709 with _post_physics_step_callback, check_termination,
// compute_reward; humanoid variants h1_env.py / g1_env.py.  Everything up to
// the reset decision; returns the reset flag in s.flags[0].  Called by all lanes:
// lane 0 derives the base-frame state, commands and termination; then lane k
// evaluates reward term k (all terms at once); lane 0 sums them in the reference's
// (alphabetical) order, the same arithmetic as one lane summing term by term.
template <int D, int B, int ROWS, bool PAD = false>
__device__ __forceinline__ float reward_term(Smem<D, B, ROWS>& s, const lgs_task_params& T, const lgs_env_buffers& E,
                                             const float* rbs, int e, int id) {
    const int A = T.num_actions;
    const float* root = s.root;
    const float* bl = s.u.post.misc;
    const float* ba = s.u.post.misc + 3;
    const float* pg = s.u.post.misc + 6;
    const float* leg_phase = s.u.post.misc + 10;
    const float* cmd = s.u.post.misc + 12;
    const float* act = s.act;
    const float* last_act = E.last_actions + A * e;
    const float* last_qd = E.last_dof_vel + (PAD ? A : D) * e;
    float* air = E.feet_air_time + T.num_feet * e;
    uint8_t* lastc = E.last_contacts + T.num_feet * e;
    const float* tau = s.tau;
    float sum = 0.f, r;
    switch (id) {
    case LGS_REW_LIN_VEL_Z: r = bl[2] * bl[2]; break;
    case LGS_REW_ANG_VEL_XY: r = ba[0] * ba[0] + ba[1] * ba[1]; break;
    case LGS_REW_ORIENTATION: r = pg[0] * pg[0] + pg[1] * pg[1]; break;
    case LGS_REW_BASE_HEIGHT: { float d = root[2] - T.base_height_target; r = d * d; } break;
    case LGS_REW_TORQUES: for (int j = 0; j < A; ++j) sum += tau[j] * tau[j]; r = sum; break;
    case LGS_REW_DOF_VEL: for (int j = 0; j < A; ++j) sum += s.qd[j] * s.qd[j]; r = sum; break;
    case LGS_REW_DOF_ACC:
        for (int j = 0; j < A; ++j) { float d = (last_qd[j] - s.qd[j]) / T.control_dt; sum += d * d; }
        r = sum; break;
    case LGS_REW_ACTION_RATE:
        for (int j = 0; j < A; ++j) { float d = last_act[j] - act[j]; sum += d * d; }
        r = sum; break;
    case LGS_REW_COLLISION:
        for (int i = 0; i < T.num_penalised; ++i) {
            const float* F = s.cf[T.penalised_idx[i]];
            sum += (sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) > 0.1f) ? 1.f : 0.f;
        }
        r = sum; break;
    case LGS_REW_DOF_POS_LIMITS:
        for (int j = 0; j < A; ++j) {
            float o = -fminf(s.q[j] - T.soft_dof_pos_lower[j], 0.f);
            o += fmaxf(s.q[j] - T.soft_dof_pos_upper[j], 0.f);
            sum += o;
        }
        r = sum; break;
    case LGS_REW_DOF_VEL_LIMITS:
        for (int j = 0; j < A; ++j) sum += clipf(fabsf(s.qd[j]) - T.dof_vel_limits[j] * T.soft_dof_vel_limit, 0.f, 1.f);
        r = sum; break;
    case LGS_REW_TORQUE_LIMITS:
        for (int j = 0; j < A; ++j) sum += fmaxf(fabsf(tau[j]) - T.torque_limits[j] * T.soft_torque_limit, 0.f);
        r = sum; break;
    case LGS_REW_TRACKING_LIN_VEL: {
        float e0 = cmd[0] - bl[0], e1 = cmd[1] - bl[1];
        r = lgs_expf(-(e0 * e0 + e1 * e1) / T.tracking_sigma);
    } break;
    case LGS_REW_TRACKING_ANG_VEL: {
        float d = cmd[2] - ba[2];
        r = lgs_expf(-(d * d) / T.tracking_sigma);
    } break;
    case LGS_REW_FEET_AIR_TIME: {
        int filt[LGS_MAX_FEET];
        for (int f = 0; f < T.num_feet; ++f) {
            int contact = s.cf[T.feet_idx[f]][2] > 1.f;
            filt[f] = contact || lastc[f];
            lastc[f] = (uint8_t)contact;
            float first = (air[f] > 0.f && filt[f]) ? 1.f : 0.f;
            air[f] += T.control_dt;
            sum += (air[f] - 0.5f) * first;
        }
        float cn = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]);
        sum *= (cn > 0.1f) ? 1.f : 0.f;
        for (int f = 0; f < T.num_feet; ++f)
            if (filt[f]) air[f] = 0.f;
        r = sum;
    } break;
    case LGS_REW_FEET_STUMBLE: {
        r = 0.f;
        for (int f = 0; f < T.num_feet; ++f) {
            const float* F = s.cf[T.feet_idx[f]];
            if (sqrtf(F[0] * F[0] + F[1] * F[1]) > 5.f * fabsf(F[2])) r = 1.f;
        }
    } break;
    case LGS_REW_STAND_STILL: {
        for (int j = 0; j < A; ++j) sum += fabsf(s.q[j] - T.default_dof_pos[j]);
        float cn = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]);
        r = sum * ((cn < 0.1f) ? 1.f : 0.f);
    } break;
    case LGS_REW_FEET_CONTACT_FORCES:
        for (int f = 0; f < T.num_feet; ++f) {
            const float* F = s.cf[T.feet_idx[f]];
            sum += fmaxf(sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) - T.max_contact_force, 0.f);
        }
        r = sum; break;
    case LGS_REW_ALIVE: r = 1.0f; break;
    case LGS_REW_CONTACT:
        for (int f = 0; f < T.num_feet; ++f) {
            int stance = leg_phase[f] < T.stance_threshold;
            int contact = s.cf[T.feet_idx[f]][2] > 1.f;
            sum += (contact == stance) ? 1.f : 0.f;
        }
        r = sum; break;
    case LGS_REW_FEET_SWING_HEIGHT:
        for (int f = 0; f < T.num_feet; ++f) {
            const float* F = s.cf[T.feet_idx[f]];
            int contact = sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) > 1.f;
            float d = rbs[13 * T.feet_idx[f] + 2] - T.swing_height_target;
            sum += d * d * (contact ? 0.f : 1.f);
        }
        r = sum; break;
    case LGS_REW_CONTACT_NO_VEL:
        for (int f = 0; f < T.num_feet; ++f) {
            const float* F = s.cf[T.feet_idx[f]];
            float c = sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) > 1.f ? 1.f : 0.f;
            const float* vv = rbs + 13 * T.feet_idx[f] + 7;
            for (int k2 = 0; k2 < 3; ++k2) { float xx = vv[k2] * c; sum += xx * xx; }
        }
        r = sum; break;
    case LGS_REW_HIP_POS:
        for (int i = 0; i < T.num_hip; ++i) sum += s.q[T.hip_dofs[i]] * s.q[T.hip_dofs[i]];
        r = sum; break;
    default: r = 0.f;
    }
    return r;
}

// post_physics parts: everything, only up to the rewards (lgs_post_physics_rewards), or
// the rest from the state the first part left in the env buffers (lgs_post_physics_finish);
// the rewards part itself in two: the base-frame state and _post_physics_step_callback's
// commands / gait phase (lgs_post_physics_prepare), then termination and the rewards on
// what the env buffers hold after a task's Python callback (lgs_post_physics_term_rewards)
enum { PART_ALL = 0, PART_REWARDS = 1, PART_FINISH = 2, PART_PREPARE = 3, PART_TERM_REWARDS = 4 };

template <int D, int B, int ROWS, int EPW, bool PAD = false>
__device__ void post_physics_scalar(Smem<D, B, ROWS>& s, const lgs_task_params& T, const lgs_env_buffers& E,
                                    const float* rbs, int N, int e, uint32_t step, int part) {
    const int lane = hl<EPW>();
    if (lane == 0 && part == PART_TERM_REWARDS) {
        // the prepare part's results, as a Python callback may have left them
        const int64_t ep = E.episode_length[e];
        int reset = 0;
        for (int i = 0; i < T.num_termination; ++i) {
            const float* F = s.cf[T.termination_idx[i]];
            if (sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) > 1.f) reset = 1;
        }
        if (fabsf(E.rpy[3 * e + 1]) > 1.0f || fabsf(E.rpy[3 * e]) > 0.8f) reset = 1;
        const int timeout = (float)ep > T.max_episode_length;
        reset |= timeout;
        for (int i = 0; i < 3; ++i) {
            s.u.post.misc[i] = E.base_lin_vel[3 * e + i];
            s.u.post.misc[3 + i] = E.base_ang_vel[3 * e + i];
            s.u.post.misc[6 + i] = E.projected_gravity[3 * e + i];
        }
        s.u.post.misc[9] = E.phase ? E.phase[e] : 0.f;
        s.u.post.misc[10] = E.leg_phase ? E.leg_phase[2 * e] : 0.f;
        s.u.post.misc[11] = E.leg_phase ? E.leg_phase[2 * e + 1] : 0.f;
        for (int i = 0; i < 4; ++i) s.u.post.misc[12 + i] = E.commands[4 * e + i];
        s.flags[0] = reset;
        s.flags[1] = timeout;
    } else if (lane == 0) {
        float* root = s.root;
        float* cmd = E.commands + 4 * e;
        int64_t* ep = E.episode_length + e;
        *ep += 1;
        float bl[3], ba[3], pg[3], rpy[3];
        const float g[3] = {0.f, 0.f, -1.f};
        quat_rotate_inverse(root + 3, root + 7, bl);
        quat_rotate_inverse(root + 3, root + 10, ba);
        quat_rotate_inverse(root + 3, g, pg);
        {
            const float* q = root + 3;
            float qx = q[0], qy = q[1], qz = q[2], qw = q[3];
            float sinr = 2.0f * (qw * qx + qy * qz);
            float cosr = qw * qw - qx * qx - qy * qy + qz * qz;
            rpy[0] = lgs_atan2f(sinr, cosr);
            float sinp = 2.0f * (qw * qy - qz * qx);
            rpy[1] = fabsf(sinp) >= 1.f ? copysignf(3.14159265358979323846f / 2.0f, sinp) : lgs_asinf(sinp);
            float siny = 2.0f * (qw * qz + qx * qy);
            float cosy = qw * qw + qx * qx - qy * qy - qz * qz;
            rpy[2] = lgs_atan2f(siny, cosy);
        }
        float phase = 0.f, leg_phase[2] = {0.f, 0.f};
        if (T.obs_layout == LGS_OBS_HUMANOID) {
            float t = (float)(*ep) * T.control_dt;
            phase = fmod_pos(t, T.phase_period) / T.phase_period;
            leg_phase[0] = phase;
            leg_phase[1] = fmod_pos(phase + T.phase_offset, 1.0f);
        }
        const uint64_t seed = T.seed;
        if ((*ep) % T.resample_interval == 0) resample_commands(T, cmd, seed, (uint32_t)e, step, LGS_STREAM_CMD);
        if (T.heading_command) {
            const float* q = root + 3;
            const float fx[3] = {1.f, 0.f, 0.f};
            float t[3], u[3];
            cross3(q, fx, t);
            t[0] *= 2.f; t[1] *= 2.f; t[2] *= 2.f;
            cross3(q, t, u);
            float fwd0 = fx[0] + q[3] * t[0] + u[0];
            float fwd1 = fx[1] + q[3] * t[1] + u[1];
            float heading = lgs_atan2f(fwd1, fwd0);
            const float tp = 2.0f * 3.14159265358979323846f;
            float wv = fmod_pos(cmd[3] - heading, tp);
            if (wv > 3.14159265358979323846f) wv -= tp;
            cmd[2] = clipf(0.5f * wv, -1.f, 1.f);
        }
        int reset = 0;
        for (int i = 0; i < T.num_termination; ++i) {
            const float* F = s.cf[T.termination_idx[i]];
            if (sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) > 1.f) reset = 1;
        }
        if (fabsf(rpy[1]) > 1.0f || fabsf(rpy[0]) > 0.8f) reset = 1;
        const int timeout = (float)(*ep) > T.max_episode_length;
        reset |= timeout;
        for (int i = 0; i < 3; ++i) {
            E.base_lin_vel[3 * e + i] = bl[i];
            E.base_ang_vel[3 * e + i] = ba[i];
            E.projected_gravity[3 * e + i] = pg[i];
            E.rpy[3 * e + i] = rpy[i];
            s.u.post.misc[i] = bl[i]; s.u.post.misc[3 + i] = ba[i]; s.u.post.misc[6 + i] = pg[i];
        }
        s.u.post.misc[9] = phase;
        s.u.post.misc[10] = leg_phase[0]; s.u.post.misc[11] = leg_phase[1];
        for (int i = 0; i < 4; ++i) s.u.post.misc[12 + i] = cmd[i];
        if (E.phase) E.phase[e] = phase;
        if (E.leg_phase) { E.leg_phase[2 * e] = leg_phase[0]; E.leg_phase[2 * e + 1] = leg_phase[1]; }
        s.flags[0] = reset;
        s.flags[1] = timeout;
    }
    if (part == PART_PREPARE) return;  // (the base-frame state and commands are in E)
    __syncthreads();
    // rewards: lane k evaluates active term k (alphabetical order, legged_robot.py:770-787)
    if (lane < T.num_rewards) {
        const float r = reward_term<D, B, ROWS, PAD>(s, T, E, rbs, e, T.reward_ids[lane]) * T.reward_scales[lane];
        s.u.post.terms[lane] = r;
        E.episode_sums[(size_t)lane * N + e] += r;
        if (E.rew_terms) E.rew_terms[(size_t)lane * N + e] = r;
    }
    __syncthreads();
    if (lane == 0) {
        const int reset = s.flags[0], timeout = s.flags[1];
        float rew = 0.f;
        for (int k = 0; k < T.num_rewards; ++k) rew += s.u.post.terms[k];
        if (T.only_positive_rewards && !T.defer_reward_total) rew = fmaxf(rew, 0.f);
        if (T.has_termination_reward && !T.defer_reward_total) {
            float r = ((reset && !timeout) ? 1.f : 0.f) * T.termination_scale;
            rew += r;
            E.episode_sums[(size_t)T.num_rewards * N + e] += r;
        }
        E.rew[e] = rew;
        E.reset[e] = (uint8_t)reset;
        E.time_out[e] = (uint8_t)timeout;
    }
}

// episode-sum rows: native terms, termination, then the caller's (Python) terms
__device__ __forceinline__ int num_sums(const lgs_task_params& T) {
    return T.num_rewards + (T.has_termination_reward ? 1 : 0) + T.num_extra_sums;
}

// reset modes of post_physics: the control step (reset decided by check_termination),
// BaseTask.reset (every env, no episode extras), reset_idx(env_ids) (the masked envs:
// episode sums into the extras accumulator, reset_buf set, legged_robot.py:723-768)
enum { RESET_STEP = 0, RESET_ALL = 1, RESET_IDS = 2 };

template <int D, int B, int ROWS, int EPW, bool PAD = false>
__device__ void post_physics(Smem<D, B, ROWS>& s, const lgs_task_params& T, const lgs_env_buffers& E,
                             const float* rbs, int N, int e, uint32_t step, int reset_mode, int part = PART_ALL,
                             float* vsim = nullptr, unsigned* pushed = nullptr) {
    const int lane = hl<EPW>();
    const int A = T.num_actions;
    const int Ad = PAD ? A : D;  // (unpadded: num_actions == D, a compile-time bound)
    const uint64_t seed = T.seed;
    const bool force_reset = reset_mode != RESET_STEP;
    if (force_reset) {
        if (lane == 0) s.flags[0] = 1;
    } else if (part != PART_FINISH) {
        post_physics_scalar<D, B, ROWS, EPW, PAD>(s, T, E, rbs, N, e, step, part);
        if (part != PART_ALL) return;
    } else if (lane == 0) {  // the first part's results: reset decision, base-frame state, commands
        s.flags[0] = E.reset[e];
        s.flags[1] = E.time_out[e];
        for (int i = 0; i < 3; ++i) {
            s.u.post.misc[i] = E.base_lin_vel[3 * e + i];
            s.u.post.misc[3 + i] = E.base_ang_vel[3 * e + i];
            s.u.post.misc[6 + i] = E.projected_gravity[3 * e + i];
        }
        s.u.post.misc[9] = E.phase ? E.phase[e] : 0.f;
        s.u.post.misc[10] = E.leg_phase ? E.leg_phase[2 * e] : 0.f;
        s.u.post.misc[11] = E.leg_phase ? E.leg_phase[2 * e + 1] : 0.f;
        for (int i = 0; i < 4; ++i) s.u.post.misc[12 + i] = E.commands[4 * e + i];
    }
    __syncthreads();
    const int reset = s.flags[0];
    float* act = s.act;
    if (reset) {  // reset_idx (legged_robot.py:723-768)
        if (lane < D) {  // (a padded model's inert DOFs: default 0)
            s.q[lane] = T.default_dof_pos[lane] *
                        rand_range(0.5f, 1.5f, philox_uniform(seed, e, step, LGS_STREAM_RESET_DOF, lane));
            s.qd[lane] = 0.f;
            if (lane < Ad) E.last_dof_vel[Ad * e + lane] = 0.f;
        }
        if (lane < A) { act[lane] = 0.f; E.actions[A * e + lane] = 0.f; E.last_actions[A * e + lane] = 0.f; }
        if (lane < T.num_feet) E.feet_air_time[T.num_feet * e + lane] = 0.f;
        float rv = (lane < 6) ? rand_range(-0.5f, 0.5f, philox_uniform(seed, e, step, LGS_STREAM_RESET_ROOT, lane)) : 0.f;
        __syncthreads();
        if (lane < 13) {
            float x = T.base_init_state[lane];
            if (lane < 3) x += E.env_origins[3 * e + lane];
            // terrain origins: xy within 1 m of the tile centre (legged_robot.py:582-585)
            if (lane < 2 && T.custom_origins)
                x += rand_range(-1.f, 1.f, philox_uniform(seed, e, step, LGS_STREAM_RESET_ROOT, 6 + lane));
            s.root[lane] = x;
        }
        __syncthreads();
        if (lane < 6) s.root[7 + lane] = rv;
        if (reset_mode == RESET_IDS && lane == 0) E.reset[e] = 1;  // reset_buf[env_ids] = 1 (:758)
        if (reset_mode != RESET_ALL) {
            // (strided: two envs per wave leave 32 lanes per env, and a task may have more sums)
            const int nsum = num_sums(T);
            for (int k = lane; k < nsum; k += WAVE / EPW) {
                atomicAdd(E.episode_acc + k, E.episode_sums[(size_t)k * N + e]);
                E.episode_sums[(size_t)k * N + e] = 0.f;
            }
            if (lane == 0) atomicAdd(E.episode_acc + nsum, 1.f);
        } else {
            const int nsum = num_sums(T);
            for (int k = lane; k < nsum; k += WAVE / EPW) E.episode_sums[(size_t)k * N + e] = 0.f;
        }
        if (lane == 0) {
            resample_commands(T, E.commands + 4 * e, seed, (uint32_t)e, step, LGS_STREAM_RESET_CMD);
            E.episode_length[e] = 0;
        }
        __syncthreads();
    }
    if (force_reset) return;  // BaseTask.reset: the following step() builds obs
    // _push_robots (legged_robot.py:540-555)
    if (lane == 0 && T.push_robots && E.episode_length[e] % T.push_interval == 0) {
        s.root[7] = rand_range(-T.max_push_vel_xy, T.max_push_vel_xy, philox_uniform(seed, e, step, LGS_STREAM_PUSH, 0));
        s.root[8] = rand_range(-T.max_push_vel_xy, T.max_push_vel_xy, philox_uniform(seed, e, step, LGS_STREAM_PUSH, 1));
        if (pushed) atomicOr(pushed + (step & 1u), 1u);  // (few envs per step: the pushed and the reset ones)
    }
    // compute_observations
    if (lane == 0) {
        const float* cmd = E.commands + 4 * e;
        // quadruped obs = tmp[0:O]; humanoid priv = tmp[0:P], obs = tmp[3:3+O]
        float* tmp = s.u.post.obs_tmp;
        tmp[0] = s.u.post.misc[0] * T.obs_scale_lin_vel;
        tmp[1] = s.u.post.misc[1] * T.obs_scale_lin_vel;
        tmp[2] = s.u.post.misc[2] * T.obs_scale_lin_vel;
        int k = 3;
        for (int i = 0; i < 3; ++i) tmp[k++] = s.u.post.misc[3 + i] * T.obs_scale_ang_vel;
        for (int i = 0; i < 3; ++i) tmp[k++] = s.u.post.misc[6 + i];
        for (int i = 0; i < 3; ++i) tmp[k++] = cmd[i] * T.commands_scale[i];
        for (int j = 0; j < Ad; ++j) tmp[k++] = (s.q[j] - T.default_dof_pos[j]) * T.obs_scale_dof_pos;
        for (int j = 0; j < Ad; ++j) tmp[k++] = s.qd[j] * T.obs_scale_dof_vel;
        for (int j = 0; j < Ad; ++j) tmp[k++] = act[j];
        if (T.obs_layout == LGS_OBS_HUMANOID) {
            float ph = 2.0f * 3.14159265358979323846f * s.u.post.misc[9];
            float sp_, cp_;
            lgs_sincosf(ph, &sp_, &cp_);
            tmp[k++] = sp_;
            tmp[k++] = cp_;
        }
    }
    __syncthreads();
    const int O = T.num_obs, P = T.num_privileged_obs;
    const int off = (T.obs_layout == LGS_OBS_HUMANOID) ? 3 : 0;
    for (int i = lane; i < O; i += WAVE / EPW) {
        float x = s.u.post.obs_tmp[off + i];
        if (T.add_noise) x += (2.f * philox_uniform(seed, e, step, LGS_STREAM_NOISE, i) - 1.f) * T.noise_vec[i];
        E.obs[(size_t)O * e + i] = clipf(x, -T.clip_observations, T.clip_observations);
    }
    if (P > 0 && E.priv_obs && T.obs_layout == LGS_OBS_HUMANOID)
        for (int i = lane; i < P; i += WAVE / EPW)
            E.priv_obs[(size_t)P * e + i] = clipf(s.u.post.obs_tmp[i], -T.clip_observations, T.clip_observations);
    // bookkeeping (:707-709)
    if (lane < A) E.last_actions[A * e + lane] = act[lane];
    if (lane < Ad) E.last_dof_vel[Ad * e + lane] = s.qd[lane];
    if (vsim && T.push_robots && lane < 2) {
        // last_root_vel[:, 0:2]: the all-env push draw whenever any env is pushed this step
        // (legged_robot.py:549-550, 709), which is nearly every step; the simulated values
        // go to vsim, and k_step_extras puts them back on the steps where no env is pushed
        vsim[2 * e + lane] = s.root[7 + lane];
        E.last_root_vel[6 * e + lane] =
            rand_range(-T.max_push_vel_xy, T.max_push_vel_xy, philox_uniform(seed, e, step, LGS_STREAM_PUSH, lane));
    } else if (lane < 6) {
        E.last_root_vel[6 * e + lane] = s.root[7 + lane];
    }
    if (vsim && lane >= 2 && lane < 6) E.last_root_vel[6 * e + lane] = s.root[7 + lane];
}

// k_step modes: the fused control step (lgs_step), or its two halves -- the physics
// (clip, decimation x (PD + substep), torques, body states: lgs_step_physics) and the
// post-physics stack on the bound state (lgs_post_physics).  STEP == PHYSICS then POST,
// bit for bit: the post half reads back exactly what the physics half stored.
enum { MODE_STEP = 0, MODE_PHYSICS = 1, MODE_POST = 2, MODE_POST_REWARDS = 3, MODE_POST_FINISH = 4,
       MODE_POST_PREPARE = 5, MODE_POST_TERM_REWARDS = 6 };
__host__ __device__ constexpr int mode_part(int mode) {
    return mode == MODE_POST_REWARDS ? PART_REWARDS
         : mode == MODE_POST_FINISH ? PART_FINISH
         : mode == MODE_POST_PREPARE ? PART_PREPARE
         : mode == MODE_POST_TERM_REWARDS ? PART_TERM_REWARDS : PART_ALL;
}

// EPW envs per workgroup (one wave): env EPW * xcd_env(block) + hh; with EPW = 2 the grid
// has N / 2 workgroups (N even) and every wave carries two envs.
// WPE > 0: the waves/SIMD the build targets (the 48-row variant at <= 4096 envs takes 4:
// one round of waves, worth its spills; 8192 envs run 3, fewer spills)
template <int D, int B, int ROWS, int CH, int EPW, int WPE = 0, bool PAD = false>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : (EPW == 2 ? 2 : (ROWS <= 32 ? LGS_WAVES_PER_EU : LGS_WAVES_PER_EU_48))))) void k_step(DevModel md, DevSim sp, DevState st, const lgs_task_params* __restrict__ Tp,
                                               lgs_env_buffers E, int N, uint32_t step, int mode) {
    STAMP_BEGIN();
    __shared__ Smem<D, B, ROWS> sm[EPW];
    __shared__ ModelCache<D, B> mc;
    if (E.step_counter) step = (uint32_t)*E.step_counter;
    // the step key whose parity indexes this step's push flag, for a deferred step's consumer
    // (lgs_step_deferred: the consumer advances the counter, so it cannot read the key there)
    if (blockIdx.x == 0 && threadIdx.x == 0 && st.pushed && mode != MODE_PHYSICS) st.pushed[2] = step;
    const int e = EPW * xcd_env(blockIdx.x, gridDim.x) + hh<EPW>();
    if (EPW * xcd_env(blockIdx.x, gridDim.x) >= N) return;  // (EPW = 2: N is even, both envs exist)
    Smem<D, B, ROWS>& s = sm[hh<EPW>()];
    const lgs_task_params& T = *Tp;
    const int lane = hl<EPW>();
    load_model(mc, md);
#ifdef LGS_DIAG_MULTISTEP
    // diagnostic build (never the shipped library): LGS_DIAG_MULTISTEP control steps per launch
    // on the same actions, no kernel boundary between them -- what a multi-step rollout kernel
    // would save of the per-launch barrier (the launch ends with its slowest wave)
    const uint32_t step0 = step;
    for (int tt = 0; tt < LGS_DIAG_MULTISTEP; ++tt) {
    step = step0 + (uint32_t)tt;
    __syncthreads();
#endif
    load_state<D, B, ROWS, EPW, PAD>(s, st, md, e);
    const int A = T.num_actions;
    const int Ad = PAD ? A : D, Br = PAD ? md.Br : B;  // (unpadded: compile-time bounds)
    float* rbs = (T.write_body_states && st.rbs) ? st.rbs + (size_t)13 * Br * e : nullptr;
    STAMP_INIT();
    if (mode == MODE_STEP || mode == MODE_PHYSICS) {
        float a = 0.f;
        if (lane < A) {
            const float* ain = E.actions_in ? E.actions_in : E.actions;
            a = clipf(ain[A * e + lane], -T.clip_actions, T.clip_actions);  // :623-624
            E.actions[A * e + lane] = a;
            s.act[lane] = a;
        }
        const float lqd = (lane < Ad) ? E.last_dof_vel[Ad * e + lane] : 0.f;
        const float am = st.added_mass ? st.added_mass[e] : 0.f;
        const float mu = st.friction ? st.friction[e] : 1.f;
        __syncthreads();
        for (int it = 0; it < T.decimation; ++it) {  // :627-639
            if (lane < D) {  // _compute_torques :649-671
                const float as = a * T.action_scale;
                const float q = s.q[lane], qd = s.qd[lane];
                float t;
                if (T.control_type == 0) t = T.p_gains[lane] * (as + T.default_dof_pos[lane] - q) - T.d_gains[lane] * qd;
                else if (T.control_type == 1) t = T.p_gains[lane] * (as - qd) - T.d_gains[lane] * (qd - lqd) / sp.dt;
                else t = as;
                s.tau[lane] = clipf(t, -T.torque_limits[lane], T.torque_limits[lane]);
            }
            __syncthreads();
#ifndef LGS_DIAG_IO_ONLY
            substep<D, B, ROWS, CH, EPW, PAD>(sm, mc, md, sp, am, mu);
#else
            // diagnostic build (never the shipped library): no physics, the step's global loads
            // and stores unchanged -- a known-byte calibration of the traffic counters
            if (lane < 3 * B) (&s.cf[0][0])[lane] = 0.f;
#endif
        }
        STAMP(0);
        if (lane < Ad) E.torques[Ad * e + lane] = s.tau[lane];
        // refresh_rigid_body_state (h1_env.py:49), humanoid tasks only: the rows they read
        if (rbs) body_states<D, B, ROWS, EPW>(s, mc, rbs, Br, T.body_state_mask);
    } else {  // the physics half's outputs, as it stored them
        if (lane < A) s.act[lane] = E.actions[A * e + lane];
        if (lane < D) s.tau[lane] = lane < Ad ? E.torques[Ad * e + lane] : 0.f;
        for (int i = lane; i < 3 * B; i += WAVE / EPW)
            (&s.cf[0][0])[i] = i < 3 * Br ? st.cforce[(size_t)3 * Br * e + i] : 0.f;
    }
    __syncthreads();
    STAMP(15);
    if (mode != MODE_PHYSICS)
        post_physics<D, B, ROWS, EPW, PAD>(s, T, E, rbs, N, e, step, RESET_STEP, mode_part(mode), st.vsim, st.pushed);
    __syncthreads();
    STAMP(16);
    store_state<D, B, ROWS, EPW, PAD>(s, st, md, e);
    STAMP(17);
    STAMP_END();
    STAMP_FLUSH(e);
#ifdef LGS_DIAG_MULTISTEP
    }
#endif
}

// reset_idx: every env (mask == NULL, BaseTask.reset) or the envs whose mask byte is set
template <int D, int B, int ROWS, int CH, bool PAD = false>
__global__ __launch_bounds__(WAVE) void k_reset_all(DevModel md, DevState st, const lgs_task_params* __restrict__ Tp,
                                                    lgs_env_buffers E, int N, uint32_t step, const uint8_t* mask) {
    __shared__ Smem<D, B, ROWS> s;
    __shared__ ModelCache<D, B> mc;
    const int e = xcd_env(blockIdx.x, gridDim.x);
    if (e >= N) return;
    if (mask && !mask[e]) return;
    if (E.step_counter) step = (uint32_t)*E.step_counter;
    load_model(mc, md);
    const int Br = PAD ? md.Br : B;
    load_state<D, B, ROWS, 1, PAD>(s, st, md, e);
    if (threadIdx.x < 3 * B)
        (&s.cf[0][0])[threadIdx.x] = threadIdx.x < 3 * Br ? st.cforce[(size_t)3 * Br * e + threadIdx.x] : 0.f;
    __syncthreads();
    post_physics<D, B, ROWS, 1, PAD>(s, *Tp, E, nullptr, N, e, step, mask ? RESET_IDS : RESET_ALL);
    __syncthreads();
    store_state<D, B, ROWS, 1, PAD>(s, st, md, e);
    if (st.rbs) body_states<D, B, ROWS, 1>(s, mc, st.rbs + (size_t)13 * Br * e, Br);
}

// After k_step (one block): the extras of reset_idx (legged_robot.py:742-768) —
// episode means over the envs reset this step, carried when none reset, and the
// carried time-out flags — then episode_acc zeroed for the next step and the
// device step counter advanced (the Philox key of graph-replayed steps).
// advance = 1 (after a control step) also finishes _push_robots (:540-555): when ANY env
// was pushed, the reference writes root_states[:, 7:9] of EVERY env with one draw per env
// and only the pushed envs reach the simulation; bookkeeping (:709) then copies that
// tensor into last_root_vel.  root_states here IS the simulation state, so it keeps the
// simulated velocities of the envs not pushed; last_root_vel[:, 0:2] takes
// the draws for every env, as in the reference (the pushed envs' draws are the ones
// k_step applied: same Philox key).  k_step itself writes every env's draw there (and its
// simulated xy velocity to vsim): this one-workgroup kernel only restores vsim on the
// rare steps where no env was pushed (it drew 2 Philox per env itself before: 4.6 -> 9.5 us).
__global__ __launch_bounds__(1024) void k_step_extras(lgs_env_buffers E, const lgs_task_params* __restrict__ Tp,
                                                      int N, int advance, uint32_t step, const float* vsim,
                                                      unsigned* pushed_flag) {
    const lgs_task_params& T = *Tp;
    const int nsum = num_sums(T);
    const float cnt = E.episode_acc[nsum];
    const bool any = cnt > 0.f;
    const int t = threadIdx.x;
    if (E.step_counter) step = (uint32_t)*E.step_counter;  // the key k_step used (read before the advance)
    if (advance && T.push_robots && E.last_root_vel && vsim) {
        // k_step wrote every env's draw; no env pushed (episode_length % push_interval == 0
        // after this step, reset ones at 0): the simulated velocities go back
        // (k_step raised this step's flag for every env it pushed: no scan over the envs)
        if (!pushed_flag[step & 1u])
            for (int e = t; e < N; e += blockDim.x) {
                E.last_root_vel[6 * e] = vsim[2 * e];
                E.last_root_vel[6 * e + 1] = vsim[2 * e + 1];
            }
    }
    if (E.ep_means && t < nsum) {
        float m = E.ep_means[t];
        if (any) m = E.episode_acc[t] / fmaxf(cnt, 1.f) / T.max_episode_length_s;
        E.ep_means[t] = m;
        if (E.ep_snapshot) E.ep_snapshot[t] = m;
    }
    if (E.time_outs_carry && any)
        for (int e = t; e < N; e += blockDim.x) E.time_outs_carry[e] = E.time_out[e];
    __syncthreads();
    if (t <= nsum) E.episode_acc[t] = 0.f;
    if (E.episode_acc_next && t <= nsum) E.episode_acc_next[t] = 0.f;  // (a deferred consumer's)
    if (t == 0 && advance) pushed_flag[(step + 1u) & 1u] = 0u;  // the next step's flag
    if (t == 0 && E.step_counter && advance) *E.step_counter += 1;
}

__global__ void k_copy_rows(float* dst, const float* src, const int32_t* ids, int n, int width) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int row = i / width, col = i % width;
    if (row >= n) return;
    const size_t r = (size_t)ids[row];
    dst[r * width + col] = src[r * width + col];
}

// ------------------------------------------------------------ host side ----
struct lgs_sim {
    int N, B, D, P;
    int Dt, Bt;  // the instantiation shape the model is padded to (>= D, B; see LGS_GENERIC_SHAPES)
    int device;
    hipStream_t stream = nullptr;
    DevModel md{};
    DevSim sp{};
    void* model_mem = nullptr;
    float* friction = nullptr;
    float* added_mass = nullptr;
    float* vsim = nullptr;  // [N,2] scratch of the all-env push bookkeeping (DevState::vsim)
    unsigned* pushed = nullptr;  // [3] the push flags and the last step key (DevState::pushed)
    unsigned long long* stats = nullptr;  // [8][LGS_NUM_CONTACT_STATS] capacity-drop counters (DevState::stats)
    float* root = nullptr;
    float* dofs = nullptr;
    float* cforce = nullptr;
    float* rbs = nullptr;
    const float* torques = nullptr;
    lgs_task_params* task_dev = nullptr;
    int16_t* hf_mem = nullptr;
    float4* self_mem = nullptr;
    int has_task = 0;
    int rows = 32;
    int chain = 0;  // dof_chain_length of the model
    int epw = 1;    // envs per wave of k_step (2 for the 32-row variant at even N)
    std::vector<std::string> body_names, dof_names;  // name queries (empty when not given)
};

// Compiled (dofs, max bodies, constraint-row capacity, chain length) variants.  The
// row capacity sets the LDS footprint (Y, A): the 32-row variant is the Go2 one.  The
// chain length CH is the sparsity the Cholesky exploits (l_nz); a tree that is not
// D/CH equal chains hanging from the base takes the dense (CH = 0) variant.
enum Variant { V_12_19, V_12_13_32, V_10_11_32, V_12_13, V_10_11, V_12_19_48, V_EXTRA, V_NONE };

// Build-time instantiation hook for other robots: every X(D, B) listed here compiles the
// 48-row, one-env-per-wave kernels (dense Cholesky) for models with exactly D DOFs and at
// most B bodies (D <= LGS_MAX_DOFS, B <= LGS_MAX_BODIES).  Add a shape here, or pass
//   make LGS_EXTRA_SHAPES='X(23,24) X(18,19)'
// and rebuild; lgs_create_sim then accepts the robot.  The default adds the G1 23-DOF
// description the reference ships (resources/robots/g1_description/g1_23dof.urdf: 23 DOFs,
// 24 bodies after fixed-joint collapse).
#ifndef LGS_EXTRA_SHAPES
#define LGS_EXTRA_SHAPES X(23, 24)
#endif
// Runtime generality: any other robot (D <= LGS_MAX_DOFS, B <= LGS_MAX_BODIES) runs on the
// smallest of these padded instantiations it fits, X(Dt, Bt) with D <= Dt and
// B + (Dt - D) <= Bt, with no rebuild: lgs_create_sim appends Dt - D inert DOFs (each on
// a massless body hinged to the base, M_jj = 1, no gains, no limits, no candidates) and
// then inert fixed bodies up to Bt.  An inert DOF's rows and columns of every matrix the
// step factorises are zero off the diagonal, so the real DOFs' arithmetic -- and the
// results, bit for bit -- are those of the unpadded model (tests/test_gpu_padded.py).
#ifndef LGS_GENERIC_SHAPES
#define LGS_GENERIC_SHAPES X(16, 24) X(26, 32)
#endif
#define LGS_ALL_48_SHAPES LGS_EXTRA_SHAPES LGS_GENERIC_SHAPES

// the instantiation shape (Dt, Bt) a model of D DOFs and B bodies is padded to among the
// extra (exact D) and generic (padded D) shapes; false if none fits
static bool extra_shape(int D, int B, int* Dt, int* Bt) {
#define X(D_, B_) if (D == D_ && B <= B_) { *Dt = D_; *Bt = B_; return true; }
    LGS_EXTRA_SHAPES
#undef X
#define X(D_, B_) if (D <= D_ && B + (D_ - D) <= B_) { *Dt = D_; *Bt = B_; return true; }
    LGS_GENERIC_SHAPES
#undef X
    return false;
}
static bool extra_shape(const lgs_sim* s) {
    int dt, bt;
    return extra_shape(s->D, s->B, &dt, &bt);
}

static Variant pick(const lgs_sim* s) {
    // 32-row humanoid variants (8 contacts): two envs per wave, as Go2
    // (exact shapes only: these kernels take the model's sizes as compile-time bounds)
    if (s->D == 12 && s->B == 13 && s->rows <= 32) return V_12_13_32;
    if (s->D == 10 && s->B == 11 && s->rows <= 32) return V_10_11_32;
    if (s->D == 12 && s->B == 19 && s->rows <= 32) return V_12_19;
    if (s->D == 12 && s->B == 13) return V_12_13;
    if (s->D == 12 && s->B == 19) return V_12_19_48;
    if (s->D == 10 && s->B == 11) return V_10_11;
    if (extra_shape(s)) return V_EXTRA;
    return V_NONE;
}
static void variant_shape(const lgs_sim* s, Variant v, int* Dt, int* Bt) {
    switch (v) {
    case V_12_19: case V_12_19_48: *Dt = 12; *Bt = 19; break;
    case V_12_13_32: case V_12_13: *Dt = 12; *Bt = 13; break;
    case V_10_11_32: case V_10_11: *Dt = 10; *Bt = 11; break;
    default: if (!extra_shape(s->D, s->B, Dt, Bt)) { *Dt = s->D; *Bt = s->B; }
    }
}
static int variant_rows(Variant v) { return (v == V_12_19 || v == V_12_13_32 || v == V_10_11_32) ? 32 : 48; }  // (V_EXTRA: 48)
static int variant_chain(Variant v) {
    return (v == V_12_13 || v == V_12_13_32) ? 6 : ((v == V_10_11 || v == V_10_11_32) ? 5 : 3);
}

#define LGS_LAUNCH(sim, KERNEL, D_, B_, R_, ...)                                                         \
    do {                                                                                                 \
        if ((sim)->chain == variant_chain(pick(sim)))                                                    \
            hipLaunchKernelGGL((KERNEL<D_, B_, R_, (D_ == 10 ? 5 : (B_ == 13 ? 6 : 3))>), dim3((sim)->N), \
                               dim3(WAVE), 0, (sim)->stream, __VA_ARGS__);                               \
        else                                                                                             \
            hipLaunchKernelGGL((KERNEL<D_, B_, R_, 0>), dim3((sim)->N), dim3(WAVE), 0, (sim)->stream,    \
                               __VA_ARGS__);                                                             \
    } while (0)
// k_step with EPW envs per wave (grid N / EPW)
#define LGS_LAUNCH_EPW(sim, KERNEL, D_, B_, R_, EPW_, ...)                                                 \
    do {                                                                                                  \
        if ((sim)->chain == variant_chain(pick(sim)))                                                     \
            hipLaunchKernelGGL((KERNEL<D_, B_, R_, (D_ == 10 ? 5 : (B_ == 13 ? 6 : 3)), EPW_>),            \
                               dim3((sim)->N / EPW_), dim3(WAVE), 0, (sim)->stream, __VA_ARGS__);         \
        else                                                                                              \
            hipLaunchKernelGGL((KERNEL<D_, B_, R_, 0, EPW_>), dim3((sim)->N / EPW_), dim3(WAVE), 0,        \
                               (sim)->stream, __VA_ARGS__);                                               \
    } while (0)
// the 48-row variants: 4 waves/SIMD when all envs fit one round of them, else the default
#define LGS_LAUNCH_48W(sim, KERNEL, D_, B_, WPE_, ...)                                                    \
    do {                                                                                                  \
        if ((sim)->chain == variant_chain(pick(sim)))                                                     \
            hipLaunchKernelGGL((KERNEL<D_, B_, 48, (D_ == 10 ? 5 : (B_ == 13 ? 6 : 3)), 1, WPE_>),        \
                               dim3((sim)->N), dim3(WAVE), 0, (sim)->stream, __VA_ARGS__);                \
        else                                                                                              \
            hipLaunchKernelGGL((KERNEL<D_, B_, 48, 0, 1, WPE_>), dim3((sim)->N), dim3(WAVE), 0,           \
                               (sim)->stream, __VA_ARGS__);                                               \
    } while (0)
#define LGS_LAUNCH_48(sim, KERNEL, D_, B_, ...)                                                           \
    do {                                                                                                  \
        if ((sim)->N <= 4 * 1024) LGS_LAUNCH_48W(sim, KERNEL, D_, B_, 4, __VA_ARGS__);                    \
        else LGS_LAUNCH_48W(sim, KERNEL, D_, B_, 0, __VA_ARGS__);                                         \
    } while (0)
// the extra shapes' launches (one env per wave, 48 rows, CH = 0)
template <int D, int B>
static void ex_step(const lgs_sim* s, DevModel md, DevSim sp, DevState st, const lgs_task_params* tp,
                    lgs_env_buffers E, int N, uint32_t step, int mode) {
    // (2 waves/SIMD: the 29-row dense factorisation does not fit the 48-row default's 168 VGPRs)
    hipLaunchKernelGGL((k_step<D, B, 48, 0, 1, 2, true>), dim3(N), dim3(WAVE), 0, s->stream, md, sp, st, tp, E, N, step, mode);
}
template <int D, int B>
static void ex_simulate(const lgs_sim* s, DevModel md, DevSim sp, DevState st, int N) {
    hipLaunchKernelGGL((k_simulate<D, B, 48, 0, true>), dim3(N), dim3(WAVE), 0, s->stream, md, sp, st, N);
}
template <int D, int B>
static void ex_fk(const lgs_sim* s, DevModel md, DevState st, int N) {
    hipLaunchKernelGGL((k_fk<D, B, 48, 0, true>), dim3(N), dim3(WAVE), 0, s->stream, md, st, N);
}
template <int D, int B>
static void ex_reset(const lgs_sim* s, DevModel md, DevState st, const lgs_task_params* tp, lgs_env_buffers E, int N,
                     uint32_t step, const uint8_t* mask) {
    hipLaunchKernelGGL((k_reset_all<D, B, 48, 0, true>), dim3(N), dim3(WAVE), 0, s->stream, md, st, tp, E, N, step, mask);
}
static int extra_step(const lgs_sim* s, DevModel md, DevSim sp, DevState st, const lgs_task_params* tp,
                      lgs_env_buffers E, int N, uint32_t step, int mode) {
#define X(D_, B_) if (s->Dt == D_ && s->Bt == B_) { ex_step<D_, B_>(s, md, sp, st, tp, E, N, step, mode); return LGS_OK; }
    LGS_ALL_48_SHAPES
#undef X
    return set_err(LGS_ERR_ARG, "unsupported model size (D,B)");
}
static int extra_simulate(const lgs_sim* s, DevModel md, DevSim sp, DevState st, int N) {
#define X(D_, B_) if (s->Dt == D_ && s->Bt == B_) { ex_simulate<D_, B_>(s, md, sp, st, N); return LGS_OK; }
    LGS_ALL_48_SHAPES
#undef X
    return set_err(LGS_ERR_ARG, "unsupported model size (D,B)");
}
static int extra_fk(const lgs_sim* s, DevModel md, DevState st, int N) {
#define X(D_, B_) if (s->Dt == D_ && s->Bt == B_) { ex_fk<D_, B_>(s, md, st, N); return LGS_OK; }
    LGS_ALL_48_SHAPES
#undef X
    return set_err(LGS_ERR_ARG, "unsupported model size (D,B)");
}
static int extra_reset(const lgs_sim* s, DevModel md, DevState st, const lgs_task_params* tp, lgs_env_buffers E,
                       int N, uint32_t step, const uint8_t* mask) {
#define X(D_, B_) if (s->Dt == D_ && s->Bt == B_) { ex_reset<D_, B_>(s, md, st, tp, E, N, step, mask); return LGS_OK; }
    LGS_ALL_48_SHAPES
#undef X
    return set_err(LGS_ERR_ARG, "unsupported model size (D,B)");
}

#define LGS_DISPATCH_STEP(sim, KERNEL, ...)                                                               \
    switch (pick(sim)) {                                                                                  \
    case V_12_19:                                                                                         \
        if ((sim)->epw == 2) LGS_LAUNCH_EPW(sim, KERNEL, 12, 19, 32, 2, __VA_ARGS__);                     \
        else LGS_LAUNCH_EPW(sim, KERNEL, 12, 19, 32, 1, __VA_ARGS__);                                     \
        break;                                                                                            \
    case V_12_13_32:                                                                                      \
        if ((sim)->epw == 2) LGS_LAUNCH_EPW(sim, KERNEL, 12, 13, 32, 2, __VA_ARGS__);                     \
        else LGS_LAUNCH_EPW(sim, KERNEL, 12, 13, 32, 1, __VA_ARGS__);                                     \
        break;                                                                                            \
    case V_10_11_32:                                                                                      \
        if ((sim)->epw == 2) LGS_LAUNCH_EPW(sim, KERNEL, 10, 11, 32, 2, __VA_ARGS__);                     \
        else LGS_LAUNCH_EPW(sim, KERNEL, 10, 11, 32, 1, __VA_ARGS__);                                     \
        break;                                                                                            \
    case V_12_13: LGS_LAUNCH_48(sim, KERNEL, 12, 13, __VA_ARGS__); break;                                 \
    case V_10_11: LGS_LAUNCH_48(sim, KERNEL, 10, 11, __VA_ARGS__); break;                                 \
    case V_12_19_48: LGS_LAUNCH_48(sim, KERNEL, 12, 19, __VA_ARGS__); break;                              \
    default: return set_err(LGS_ERR_ARG, "unsupported model size (D,B)");                                 \
    }
#define LGS_DISPATCH(sim, KERNEL, ...)                                                                    \
    switch (pick(sim)) {                                                                                  \
    case V_12_19: LGS_LAUNCH(sim, KERNEL, 12, 19, 32, __VA_ARGS__); break;                                \
    case V_12_13_32: LGS_LAUNCH(sim, KERNEL, 12, 13, 32, __VA_ARGS__); break;                             \
    case V_10_11_32: LGS_LAUNCH(sim, KERNEL, 10, 11, 32, __VA_ARGS__); break;                             \
    case V_12_13: LGS_LAUNCH(sim, KERNEL, 12, 13, 48, __VA_ARGS__); break;                                \
    case V_10_11: LGS_LAUNCH(sim, KERNEL, 10, 11, 48, __VA_ARGS__); break;                                \
    case V_12_19_48: LGS_LAUNCH(sim, KERNEL, 12, 19, 48, __VA_ARGS__); break;                             \
    default: return set_err(LGS_ERR_ARG, "unsupported model size (D,B)");                                 \
    }

// Chain length of the DOF tree: CH if the D DOFs are D/CH chains of CH joints, each
// hanging from the base, in DFS order (DOF j's nearest moving ancestor is DOF j-1, or
// the base when j % CH == 0); 0 otherwise.
static int dof_chain_length(const lgs_model_desc* m) {
    const int D = m->num_dofs;
    if (D <= 0) return 0;
    int par[LGS_MAX_DOFS];
    for (int b = 0; b < m->num_bodies; ++b) {
        const int j = m->dof[b];
        if (j < 0) continue;
        int a = m->parent[b];
        while (a > 0 && m->dof[a] < 0) a = m->parent[a];
        par[j] = a > 0 ? m->dof[a] : -1;
    }
    for (int ch = 1; ch <= D; ++ch) {
        if (D % ch) continue;
        bool ok = true;
        for (int j = 0; j < D && ok; ++j) ok = par[j] == (j % ch == 0 ? -1 : j - 1);
        if (ok) return ch;
    }
    return 0;
}

static DevState state_of(lgs_sim* s) {
    DevState st;
    st.root = s->root; st.dofs = s->dofs; st.cforce = s->cforce; st.rbs = s->rbs;
    st.friction = s->friction; st.added_mass = s->added_mass; st.torques_in = s->torques; st.vsim = s->vsim;
    st.pushed = s->pushed;
    return st;
}

extern "C" {

LGS_API const char* lgs_last_error(void) { return g_err.c_str(); }
LGS_API int lgs_version(void) { return 1; }

LGS_API float lgs_uniform(uint64_t seed, uint32_t env, uint32_t step, uint32_t stream, uint32_t index) {
    return philox_uniform(seed, env, step, stream, index);
}

LGS_API int lgs_create_sim(const lgs_model_desc* m, const lgs_sim_params* p, int32_t num_envs, int32_t device_id,
                           lgs_sim** out) {
    if (!m || !p || !out || num_envs <= 0) return set_err(LGS_ERR_ARG, "lgs_create_sim: null argument or num_envs <= 0");
    if (m->num_bodies < 1 || m->num_bodies > LGS_MAX_BODIES || m->num_dofs < 0 || m->num_dofs > LGS_MAX_DOFS)
        return set_err(LGS_ERR_ARG, "lgs_create_sim: model exceeds LGS_MAX_BODIES/LGS_MAX_DOFS");
    for (int b = 0; b < m->num_bodies; ++b)
        if (m->depth[b] >= LGS_MAX_DEPTH) return set_err(LGS_ERR_ARG, "lgs_create_sim: tree deeper than LGS_MAX_DEPTH");
    if (m->num_points < 0 || m->num_points > 32 * LGS_MAX_CHUNKS)
        return set_err(LGS_ERR_ARG, "lgs_create_sim: more than " + std::to_string(32 * LGS_MAX_CHUNKS) +
                                        " contact candidates");
    for (int k = 0; k < m->num_points; ++k)
        if (m->pt_body[k] < 0 || m->pt_body[k] >= m->num_bodies)
            return set_err(LGS_ERR_ARG, "lgs_create_sim: contact candidate body out of range");
    HIP_TRY(hipSetDevice(device_id));
    lgs_sim* s = new lgs_sim();
    s->N = num_envs; s->B = m->num_bodies; s->D = m->num_dofs; s->P = m->num_points; s->device = device_id;
    s->rows = p->max_rows;
    s->chain = dof_chain_length(m);
    // two envs per wave for the 32-row variant at an even env count (LGS_ENVS_PER_WAVE=1: one)
    {
        const char* ev = getenv("LGS_ENVS_PER_WAVE");
        const bool one = ev && atoi(ev) == 1;
        const Variant v = pick(s);
        s->epw = (!one && num_envs % 2 == 0 && (v == V_12_19 || v == V_12_13_32 || v == V_10_11_32)) ? 2 : 1;
    }
    if (pick(s) == V_NONE) {
        delete s;
        return set_err(LGS_ERR_ARG, "lgs_create_sim: no kernel instantiation for this (dofs, bodies)");
    }
    {
        const int cap = variant_rows(pick(s));
        // contact c occupies rows 3c..3c+2 (c < cap/4), limit rows the tail block
        const int cm = cap / 4, lm = cap - 3 * cm;
        if (p->max_rows > cap || p->max_rows < 3 * p->max_contacts || p->max_contacts < 0 || p->max_contacts > cm ||
            p->max_rows - 3 * p->max_contacts > lm) {
            delete s;
            return set_err(LGS_ERR_ARG, "lgs_create_sim: need max_contacts <= " + std::to_string(cm) +
                                            ", 3*max_contacts <= max_rows <= " + std::to_string(cap) +
                                            ", max_rows - 3*max_contacts <= " + std::to_string(lm));
        }
    }
    const int B = s->B, D = s->D, P = s->P;
    variant_shape(s, pick(s), &s->Dt, &s->Bt);
    if (m->body_names)
        for (int b = 0; b < B; ++b) s->body_names.emplace_back(m->body_names[b] ? m->body_names[b] : "");
    if (m->dof_names)
        for (int j = 0; j < D; ++j) s->dof_names.emplace_back(m->dof_names[j] ? m->dof_names[j] : "");
    // pack the model into one device allocation
    // contact pre-filter data: per body the bounding sphere of its candidates (centre = the
    // middle of their box, rho = the largest distance to it, rmax = the largest radius, all
    // rounded up), per chunk of 32 candidates the bit mask of their bodies
    std::vector<float> bsph((size_t)5 * B, 0.f);
    const int nch32 = (P + 31) / 32;
    std::vector<unsigned> chunk32((size_t)(nch32 > 0 ? nch32 : 1), 0u);
    for (int b = 0; b < B; ++b) {
        double lo[3] = {1e30, 1e30, 1e30}, hi[3] = {-1e30, -1e30, -1e30}, rmax = 0.0;
        int cnt = 0;
        for (int k = 0; k < P; ++k) {
            if (m->pt_body[k] != b) continue;
            ++cnt;
            for (int t = 0; t < 3; ++t) {
                lo[t] = std::min(lo[t], (double)m->pt_pos[3 * k + t]);
                hi[t] = std::max(hi[t], (double)m->pt_pos[3 * k + t]);
            }
            rmax = std::max(rmax, (double)m->pt_radius[k]);
        }
        float* o = &bsph[(size_t)5 * b];
        if (!cnt) { o[3] = -1.f; continue; }
        double c[3], rho = 0.0;
        for (int t = 0; t < 3; ++t) c[t] = 0.5 * (lo[t] + hi[t]);
        for (int k = 0; k < P; ++k) {
            if (m->pt_body[k] != b) continue;
            double d2 = 0.0;
            for (int t = 0; t < 3; ++t) d2 += (m->pt_pos[3 * k + t] - c[t]) * (m->pt_pos[3 * k + t] - c[t]);
            rho = std::max(rho, std::sqrt(d2));
        }
        for (int t = 0; t < 3; ++t) o[t] = (float)c[t];
        o[3] = (float)(rho * (1.0 + 1e-6) + 1e-6);
        o[4] = (float)(rmax * (1.0 + 1e-6) + 1e-6);
    }
    for (int k = 0; k < P; ++k) chunk32[k / 32] |= 1u << m->pt_body[k];
    // the model padded to the instantiation shape (Dt, Bt): DOF D + k on body B + k, a
    // massless body hinged to the base about z (M_jj = 1 in the kernel, no limits); then
    // fixed massless bodies on the base; the base's subtree covers them all
    const int Dt = s->Dt, Bt = s->Bt;
    std::vector<int> parent(m->parent, m->parent + B), dofv(m->dof, m->dof + B), se(m->subtree_end, m->subtree_end + B);
    std::vector<int> depth(m->depth, m->depth + B), chain(m->chain, m->chain + (size_t)B * LGS_MAX_DEPTH);
    std::vector<float> jr(m->joint_rot, m->joint_rot + 9 * B), jp(m->joint_pos, m->joint_pos + 3 * B);
    std::vector<float> ax(m->axis, m->axis + 3 * B), mass(m->mass, m->mass + B), com(m->com, m->com + 3 * B);
    std::vector<float> inertia(m->inertia, m->inertia + 6 * B);
    std::vector<float> dlo(m->dof_lower, m->dof_lower + D), dhi(m->dof_upper, m->dof_upper + D);
    std::vector<float> dvel(m->dof_velocity, m->dof_velocity + D);
    for (int b = B; b < Bt; ++b) {
        const int j = D + (b - B) < Dt ? D + (b - B) : -1;
        parent.push_back(0); dofv.push_back(j); se.push_back(b + 1); depth.push_back(1);
        for (int k = 0; k < LGS_MAX_DEPTH; ++k) chain.push_back(k == 0 ? 0 : (k == 1 ? b : -1));
        const float rot[9] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f};
        jr.insert(jr.end(), rot, rot + 9);
        for (int k = 0; k < 3; ++k) { jp.push_back(0.f); ax.push_back(k == 2 ? 1.f : 0.f); com.push_back(0.f); }
        mass.push_back(0.f);
        for (int k = 0; k < 6; ++k) inertia.push_back(0.f);
        if (j >= 0) { dlo.push_back(-1e30f); dhi.push_back(1e30f); dvel.push_back(0.f); }
    }
    se[0] = Bt;
    bsph.resize((size_t)5 * Bt, 0.f);
    for (int b = B; b < Bt; ++b) bsph[(size_t)5 * b + 3] = -1.f;
    size_t ints = (size_t)Bt * (4 + LGS_MAX_DEPTH) + (size_t)P + chunk32.size();
    size_t floats = (size_t)Bt * (9 + 3 + 3 + 1 + 3 + 6 + 5) + (size_t)Dt * 3 + (size_t)P * 4;
    size_t bytes = ints * 4 + floats * 4 + 512;
    HIP_TRY(hipMalloc(&s->model_mem, bytes));
    char* host = (char*)calloc(1, bytes);
    size_t off = 0;
    auto put = [&](const void* src, size_t n) -> size_t {
        size_t o = off;
        if (n) memcpy(host + off, src, n);
        off += (n + 15) & ~size_t(15);
        return o;
    };
    size_t o_parent = put(parent.data(), 4 * Bt), o_dof = put(dofv.data(), 4 * Bt), o_se = put(se.data(), 4 * Bt);
    size_t o_depth = put(depth.data(), 4 * Bt), o_chain = put(chain.data(), 4 * Bt * LGS_MAX_DEPTH);
    size_t o_jr = put(jr.data(), 36 * Bt), o_jp = put(jp.data(), 12 * Bt), o_ax = put(ax.data(), 12 * Bt);
    size_t o_mass = put(mass.data(), 4 * Bt), o_com = put(com.data(), 12 * Bt), o_in = put(inertia.data(), 24 * Bt);
    size_t o_lo = put(dlo.data(), 4 * Dt), o_hi = put(dhi.data(), 4 * Dt), o_vel = put(dvel.data(), 4 * Dt);
    size_t o_pb = put(m->pt_body, 4 * P), o_pp = put(m->pt_pos, 12 * P), o_pr = put(m->pt_radius, 4 * P);
    size_t o_bs = put(bsph.data(), 20 * Bt), o_ch = put(chunk32.data(), 4 * chunk32.size());
    if (off > bytes) { free(host); return set_err(LGS_ERR_STATE, "model packing overflow"); }
    HIP_TRY(hipMemcpy(s->model_mem, host, off, hipMemcpyHostToDevice));
    free(host);
    char* d = (char*)s->model_mem;
    DevModel& md = s->md;
    md.B = Bt; md.D = Dt; md.P = P; md.Br = B; md.Dr = D;
    md.parent = (const int*)(d + o_parent); md.dof = (const int*)(d + o_dof); md.subtree_end = (const int*)(d + o_se);
    md.depth = (const int*)(d + o_depth); md.chain = (const int*)(d + o_chain);
    md.joint_rot = (const float*)(d + o_jr); md.joint_pos = (const float*)(d + o_jp); md.axis = (const float*)(d + o_ax);
    md.mass = (const float*)(d + o_mass); md.com = (const float*)(d + o_com); md.inertia = (const float*)(d + o_in);
    md.dof_lower = (const float*)(d + o_lo); md.dof_upper = (const float*)(d + o_hi); md.dof_velocity = (const float*)(d + o_vel);
    md.pt_body = (const int*)(d + o_pb); md.pt_pos = (const float*)(d + o_pp); md.pt_radius = (const float*)(d + o_pr);
    md.bsph = (const float*)(d + o_bs); md.chunk32 = (const unsigned*)(d + o_ch); md.nch32 = nch32;
    DevSim& sp = s->sp;
    sp.dt = p->dt; sp.gx = p->gravity[0]; sp.gy = p->gravity[1]; sp.gz = p->gravity[2];
    sp.iters = p->solver_iterations; sp.contact_offset = p->contact_offset; sp.rest_offset = p->rest_offset;
    sp.max_depen = p->max_depenetration_velocity; sp.beta = p->baumgarte; sp.ground_friction = p->ground_friction;
    sp.armature = p->armature; sp.clamp_qd = p->clamp_joint_velocity; sp.max_contacts = p->max_contacts;
    sp.max_rows = p->max_rows;
    sp.hf = nullptr; sp.hf_rows = sp.hf_cols = 0; sp.hf_inv_hs = sp.hf_vs = sp.hf_border = 0.f;
    sp.hf_slope1 = 1.f; sp.hf_nmin = 1.f;
    sp.selfp = nullptr; sp.n_selfp = 0; sp.max_self = 0;
    HIP_TRY(hipMalloc(&s->friction, sizeof(float) * num_envs));
    HIP_TRY(hipMalloc(&s->added_mass, sizeof(float) * num_envs));
    HIP_TRY(hipMalloc(&s->vsim, sizeof(float) * 2 * num_envs));
    HIP_TRY(hipMalloc(&s->pushed, sizeof(unsigned) * 3));
    HIP_TRY(hipMemset(s->pushed, 0, sizeof(unsigned) * 3));
    HIP_TRY(hipMalloc(&s->stats, sizeof(unsigned long long) * 8 * LGS_NUM_CONTACT_STATS));
    HIP_TRY(hipMemset(s->stats, 0, sizeof(unsigned long long) * 8 * LGS_NUM_CONTACT_STATS));
    s->sp.stats = s->stats;
    HIP_TRY(hipMemset(s->added_mass, 0, sizeof(float) * num_envs));
    {
        float* ones = (float*)malloc(sizeof(float) * num_envs);
        for (int i = 0; i < num_envs; ++i) ones[i] = p->ground_friction;
        HIP_TRY(hipMemcpy(s->friction, ones, sizeof(float) * num_envs, hipMemcpyHostToDevice));
        free(ones);
    }
    HIP_TRY(hipMalloc(&s->task_dev, sizeof(lgs_task_params)));
    *out = s;
    return LGS_OK;
}

LGS_API int lgs_destroy_sim(lgs_sim* s) {
    if (!s) return LGS_OK;
    (void)hipFree(s->model_mem);
    (void)hipFree(s->friction);
    (void)hipFree(s->added_mass);
    (void)hipFree(s->vsim);
    (void)hipFree(s->pushed);
    (void)hipFree(s->stats);
    (void)hipFree(s->task_dev);
    (void)hipFree(s->hf_mem);
    (void)hipFree(s->self_mem);
    delete s;
    return LGS_OK;
}

LGS_API int lgs_set_heightfield(lgs_sim* s, const int16_t* heights, int32_t rows, int32_t cols,
                                float horizontal_scale, float vertical_scale, float border_size) {
    if (!s) return set_err(LGS_ERR_ARG, "null sim");
    if (heights && rows > 0 && (rows < 2 || cols < 2 || !(horizontal_scale > 0.f) || !(vertical_scale > 0.f)))
        return set_err(LGS_ERR_ARG, "lgs_set_heightfield: need rows, cols >= 2 and positive scales");
    HIP_TRY(hipStreamSynchronize(s->stream));  // no step may still read the previous map
    (void)hipFree(s->hf_mem);
    s->hf_mem = nullptr;
    s->sp.hf = nullptr;
    s->sp.hf_rows = s->sp.hf_cols = 0;
    if (!heights || rows <= 0) return LGS_OK;
    const size_t bytes = sizeof(int16_t) * (size_t)rows * (size_t)cols;
    HIP_TRY(hipMalloc(&s->hf_mem, bytes));
    HIP_TRY(hipMemcpy(s->hf_mem, heights, bytes, hipMemcpyHostToDevice));
    s->sp.hf = s->hf_mem;
    s->sp.hf_rows = rows; s->sp.hf_cols = cols;
    s->sp.hf_inv_hs = 1.0f / horizontal_scale;
    s->sp.hf_vs = vertical_scale;
    s->sp.hf_border = border_size;
    // slope bound of the map for the contact pre-filter: the largest gradient norm over the
    // triangles terrain_sample() builds (both halves of every cell), rounded up
    double g2 = 0.0;
    const double is = 1.0 / horizontal_scale;
    for (int i = 0; i + 1 < rows; ++i)
        for (int j = 0; j + 1 < cols; ++j) {
            const double h00 = heights[(size_t)i * cols + j] * (double)vertical_scale;
            const double h01 = heights[(size_t)i * cols + j + 1] * (double)vertical_scale;
            const double h10 = heights[(size_t)(i + 1) * cols + j] * (double)vertical_scale;
            const double h11 = heights[(size_t)(i + 1) * cols + j + 1] * (double)vertical_scale;
            const double a0 = (h10 - h00) * is, a1 = (h11 - h10) * is, b0 = (h11 - h01) * is, b1 = (h01 - h00) * is;
            g2 = std::max(g2, std::max(a0 * a0 + a1 * a1, b0 * b0 + b1 * b1));
        }
    const double G = std::sqrt(g2) * (1.0 + 1e-6) + 1e-6;
    s->sp.hf_slope1 = (float)(1.0 + G);
    s->sp.hf_nmin = (float)(1.0 / std::sqrt(1.0 + G * G) * (1.0 - 1e-6));
    return LGS_OK;
}

LGS_API int lgs_set_self_collision(lgs_sim* s, const lgs_self_collision_desc* d) {
    if (!s) return set_err(LGS_ERR_ARG, "null sim");
    if (d && d->num_pairs > 0) {
        if (d->num_pairs > LGS_MAX_SELF_PAIRS || d->num_proxies <= 0 || d->num_proxies > LGS_MAX_SELF_PROXIES ||
            !d->proxy_body || !d->capsule || !d->pair || d->max_self_contacts < 0 ||
            d->max_self_contacts > s->sp.max_contacts)
            return set_err(LGS_ERR_ARG, "lgs_set_self_collision: need 0 < num_pairs <= LGS_MAX_SELF_PAIRS, 0 < num_proxies <= "
                                        "LGS_MAX_SELF_PROXIES, 0 <= max_self_contacts <= max_contacts");
        for (int i = 0; i < d->num_proxies; ++i)
            if (d->proxy_body[i] < 0 || d->proxy_body[i] >= s->B)
                return set_err(LGS_ERR_ARG, "lgs_set_self_collision: proxy body out of range");
        for (int q = 0; q < 2 * d->num_pairs; ++q)
            if (d->pair[q] < 0 || d->pair[q] >= d->num_proxies)
                return set_err(LGS_ERR_ARG, "lgs_set_self_collision: pair proxy index out of range");
    }
    HIP_TRY(hipStreamSynchronize(s->stream));  // no step may still read the previous pairs
    (void)hipFree(s->self_mem);
    s->self_mem = nullptr;
    s->sp.selfp = nullptr;
    s->sp.n_selfp = 0;
    s->sp.max_self = 0;
    if (!d || d->num_pairs <= 0) return LGS_OK;
    // one 64-byte record per pair: [p0 p1 r body] of each proxy (the lane's four float4 loads)
    const int Q = d->num_pairs;
    float* host = (float*)malloc(sizeof(float) * 16 * Q);
    for (int q = 0; q < Q; ++q)
        for (int h = 0; h < 2; ++h) {
            const int px = d->pair[2 * q + h];
            float* o = host + 16 * q + 8 * h;
            for (int k = 0; k < 7; ++k) o[k] = d->capsule[7 * px + k];
            int32_t b = d->proxy_body[px];
            memcpy(o + 7, &b, 4);
        }
    hipError_t e = hipMalloc(&s->self_mem, sizeof(float) * 16 * Q);
    if (e == hipSuccess) e = hipMemcpy(s->self_mem, host, sizeof(float) * 16 * Q, hipMemcpyHostToDevice);
    free(host);
    if (e != hipSuccess) return set_err(LGS_ERR_HIP, std::string("lgs_set_self_collision: ") + hipGetErrorString(e));
    s->sp.selfp = s->self_mem;
    s->sp.n_selfp = Q;
    s->sp.max_self = d->max_self_contacts;
    return LGS_OK;
}

LGS_API int lgs_set_stream(lgs_sim* s, void* stream) {
    if (!s) return set_err(LGS_ERR_ARG, "null sim");
    s->stream = (hipStream_t)stream;
    return LGS_OK;
}

LGS_API int lgs_synchronize(lgs_sim* s) {
    if (!s) return set_err(LGS_ERR_ARG, "null sim");
    HIP_TRY(hipStreamSynchronize(s->stream));
    return LGS_OK;
}

LGS_API int lgs_set_env_properties(lgs_sim* s, const float* friction, const float* added_mass) {
    if (!s) return set_err(LGS_ERR_ARG, "null sim");
    if (friction) HIP_TRY(hipMemcpy(s->friction, friction, sizeof(float) * s->N, hipMemcpyHostToDevice));
    if (added_mass) HIP_TRY(hipMemcpy(s->added_mass, added_mass, sizeof(float) * s->N, hipMemcpyHostToDevice));
    return LGS_OK;
}

LGS_API int lgs_bind_state(lgs_sim* s, float* root, float* dofs, float* cforce, float* rbs) {
    if (!s || !root || !dofs || !cforce || !rbs) return set_err(LGS_ERR_ARG, "lgs_bind_state: null pointer");
    s->root = root; s->dofs = dofs; s->cforce = cforce; s->rbs = rbs;
    return LGS_OK;
}

LGS_API int lgs_refresh(lgs_sim* s) { return s ? LGS_OK : set_err(LGS_ERR_ARG, "null sim"); }

LGS_API int lgs_set_dof_actuation_force(lgs_sim* s, const float* tau) {
    if (!s || !tau) return set_err(LGS_ERR_ARG, "null argument");
    s->torques = tau;
    return LGS_OK;
}

LGS_API int lgs_simulate(lgs_sim* s) {
    if (!s || !s->root) return set_err(LGS_ERR_STATE, "lgs_simulate: state not bound");
    if (!s->torques) return set_err(LGS_ERR_STATE, "lgs_simulate: no actuation force set");
    DevState st = state_of(s);
    if (pick(s) == V_EXTRA) {
        const int rc = extra_simulate(s, s->md, s->sp, st, s->N);
        if (rc != LGS_OK) return rc;
    } else {
        LGS_DISPATCH(s, k_simulate, s->md, s->sp, st, s->N);
    }
    HIP_TRY(hipGetLastError());
    return LGS_OK;
}

LGS_API int lgs_forward_kinematics(lgs_sim* s) {
    if (!s || !s->root) return set_err(LGS_ERR_STATE, "state not bound");
    DevState st = state_of(s);
    if (pick(s) == V_EXTRA) {
        const int rc = extra_fk(s, s->md, st, s->N);
        if (rc != LGS_OK) return rc;
    } else {
        LGS_DISPATCH(s, k_fk, s->md, st, s->N);
    }
    HIP_TRY(hipGetLastError());
    return LGS_OK;
}

LGS_API int lgs_set_actor_root_state_indexed(lgs_sim* s, const float* src, const int32_t* ids, int32_t n) {
    if (!s || !src || (!ids && n > 0)) return set_err(LGS_ERR_ARG, "null argument");
    if (src == s->root || n == 0) return LGS_OK;
    const int total = n * 13;
    hipLaunchKernelGGL(k_copy_rows, dim3((total + 255) / 256), dim3(256), 0, s->stream, s->root, src, ids, n, 13);
    HIP_TRY(hipGetLastError());
    return LGS_OK;
}

LGS_API int lgs_set_dof_state_indexed(lgs_sim* s, const float* src, const int32_t* ids, int32_t n) {
    if (!s || !src || (!ids && n > 0)) return set_err(LGS_ERR_ARG, "null argument");
    if (src == s->dofs || n == 0) return LGS_OK;
    const int w = 2 * s->D, total = n * w;
    hipLaunchKernelGGL(k_copy_rows, dim3((total + 255) / 256), dim3(256), 0, s->stream, s->dofs, src, ids, n, w);
    HIP_TRY(hipGetLastError());
    return LGS_OK;
}

LGS_API int lgs_set_task(lgs_sim* s, const lgs_task_params* t) {
    if (!s || !t) return set_err(LGS_ERR_ARG, "null argument");
    if (t->num_actions != s->D) return set_err(LGS_ERR_ARG, "lgs_set_task: num_actions must equal num_dofs");
    if (t->num_obs > LGS_MAX_OBS || t->num_privileged_obs > LGS_MAX_OBS || t->num_rewards > LGS_MAX_REWARDS ||
        t->num_extra_sums < 0 || t->num_rewards + 1 + t->num_extra_sums > WAVE - 1)
        return set_err(LGS_ERR_ARG, "lgs_set_task: obs/reward counts exceed limits");
    if (t->num_feet > LGS_MAX_FEET || t->resample_interval <= 0 || t->push_interval <= 0 || t->decimation <= 0)
        return set_err(LGS_ERR_ARG, "lgs_set_task: invalid feet count / intervals / decimation");
    for (int i = 0; i < t->num_feet; ++i)
        if (t->feet_idx[i] < 0 || t->feet_idx[i] >= s->B) return set_err(LGS_ERR_ARG, "feet index out of range");
    for (int i = 0; i < t->num_penalised; ++i)
        if (t->penalised_idx[i] < 0 || t->penalised_idx[i] >= s->B) return set_err(LGS_ERR_ARG, "penalised index out of range");
    for (int i = 0; i < t->num_termination; ++i)
        if (t->termination_idx[i] < 0 || t->termination_idx[i] >= s->B) return set_err(LGS_ERR_ARG, "termination index out of range");
    for (int i = 0; i < t->num_hip; ++i)
        if (t->hip_dofs[i] < 0 || t->hip_dofs[i] >= s->D) return set_err(LGS_ERR_ARG, "hip dof out of range");
    lgs_task_params tt = *t;  // a padded model's inert DOFs: no gains, no torque, no limits
    for (int j = t->num_actions; j < LGS_MAX_DOFS; ++j) {
        tt.p_gains[j] = tt.d_gains[j] = tt.default_dof_pos[j] = tt.torque_limits[j] = 0.f;
        tt.soft_dof_pos_lower[j] = tt.soft_dof_pos_upper[j] = tt.dof_vel_limits[j] = 0.f;
    }
    HIP_TRY(hipMemcpy(s->task_dev, &tt, sizeof(lgs_task_params), hipMemcpyHostToDevice));
    s->has_task = 1;
    return LGS_OK;
}

static int launch_step(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter, int mode, const char* what,
                       bool extras = true) {
    if (!s || !env) return set_err(LGS_ERR_ARG, std::string(what) + ": null argument");
    if (!s->root || !s->has_task) return set_err(LGS_ERR_STATE, std::string(what) + ": state not bound or task not set");
    DevState st = state_of(s);
    if (pick(s) == V_EXTRA) {
        const int rc = extra_step(s, s->md, s->sp, st, s->task_dev, *env, s->N, (uint32_t)step_counter, mode);
        if (rc != LGS_OK) return rc;
    } else {
        LGS_DISPATCH_STEP(s, k_step, s->md, s->sp, st, s->task_dev, *env, s->N, (uint32_t)step_counter, mode);
    }
    HIP_TRY(hipGetLastError());
    if (extras && (mode == MODE_STEP || mode == MODE_POST || mode == MODE_POST_FINISH)) {  // extras, episode_acc zeroed, counter advanced
        hipLaunchKernelGGL(k_step_extras, dim3(1), dim3(1024), 0, s->stream, *env, s->task_dev, s->N, 1,
                           (uint32_t)step_counter, (const float*)s->vsim, s->pushed);
        HIP_TRY(hipGetLastError());
    }
    return LGS_OK;
}

LGS_API int lgs_step(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    return launch_step(s, env, step_counter, MODE_STEP, "lgs_step");
}

LGS_API int lgs_step_deferred(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    return launch_step(s, env, step_counter, MODE_STEP, "lgs_step_deferred", false);
}

LGS_API int lgs_step_extras(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    if (!s || !env) return set_err(LGS_ERR_ARG, "lgs_step_extras: null argument");
    if (!s->root || !s->has_task) return set_err(LGS_ERR_STATE, "lgs_step_extras: state not bound or task not set");
    hipLaunchKernelGGL(k_step_extras, dim3(1), dim3(1024), 0, s->stream, *env, s->task_dev, s->N, 1,
                       (uint32_t)step_counter, (const float*)s->vsim, s->pushed);
    HIP_TRY(hipGetLastError());
    return LGS_OK;
}

LGS_API int lgs_get_push_state(lgs_sim* s, float** vsim, uint32_t** pushed) {
    if (!s || !vsim || !pushed) return set_err(LGS_ERR_ARG, "lgs_get_push_state: null argument");
    *vsim = s->vsim;
    *pushed = s->pushed;
    return LGS_OK;
}

LGS_API int lgs_step_physics(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    return launch_step(s, env, step_counter, MODE_PHYSICS, "lgs_step_physics");
}

LGS_API int lgs_post_physics(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    return launch_step(s, env, step_counter, MODE_POST, "lgs_post_physics");
}

LGS_API int lgs_post_physics_rewards(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    return launch_step(s, env, step_counter, MODE_POST_REWARDS, "lgs_post_physics_rewards");
}

LGS_API int lgs_post_physics_finish(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    return launch_step(s, env, step_counter, MODE_POST_FINISH, "lgs_post_physics_finish");
}

LGS_API int lgs_post_physics_prepare(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    return launch_step(s, env, step_counter, MODE_POST_PREPARE, "lgs_post_physics_prepare");
}

LGS_API int lgs_post_physics_term_rewards(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    return launch_step(s, env, step_counter, MODE_POST_TERM_REWARDS, "lgs_post_physics_term_rewards");
}

LGS_API int lgs_reset_all(lgs_sim* s, const lgs_env_buffers* env, int64_t step_counter) {
    if (!s || !env) return set_err(LGS_ERR_ARG, "null argument");
    if (!s->root || !s->has_task) return set_err(LGS_ERR_STATE, "lgs_reset_all: state not bound or task not set");
    DevState st = state_of(s);
    if (pick(s) == V_EXTRA) {
        const int rc = extra_reset(s, s->md, st, s->task_dev, *env, s->N, (uint32_t)step_counter, nullptr);
        if (rc != LGS_OK) return rc;
    } else {
        LGS_DISPATCH(s, k_reset_all, s->md, st, s->task_dev, *env, s->N, (uint32_t)step_counter, (const uint8_t*)nullptr);
    }
    HIP_TRY(hipGetLastError());
    return LGS_OK;
}

LGS_API int lgs_reset_idx(lgs_sim* s, const lgs_env_buffers* env, const uint8_t* env_mask, int64_t step_counter) {
    if (!s || !env || !env_mask) return set_err(LGS_ERR_ARG, "lgs_reset_idx: null argument");
    if (!s->root || !s->has_task) return set_err(LGS_ERR_STATE, "lgs_reset_idx: state not bound or task not set");
    DevState st = state_of(s);
    if (pick(s) == V_EXTRA) {
        const int rc = extra_reset(s, s->md, st, s->task_dev, *env, s->N, (uint32_t)step_counter, env_mask);
        if (rc != LGS_OK) return rc;
    } else {
        LGS_DISPATCH(s, k_reset_all, s->md, st, s->task_dev, *env, s->N, (uint32_t)step_counter, env_mask);
    }
    HIP_TRY(hipGetLastError());
    // extras["episode"] over the reset envs and extras["time_outs"]; no step-counter advance
    hipLaunchKernelGGL(k_step_extras, dim3(1), dim3(1024), 0, s->stream, *env, s->task_dev, s->N, 0,
                       (uint32_t)step_counter, (const float*)s->vsim, s->pushed);
    HIP_TRY(hipGetLastError());
    return LGS_OK;
}

LGS_API int lgs_get_contact_stats(lgs_sim* s, uint64_t* out, int32_t reset) {
    if (!s || !out) return set_err(LGS_ERR_ARG, "lgs_get_contact_stats: null argument");
    unsigned long long h[8 * LGS_NUM_CONTACT_STATS];
    HIP_TRY(hipMemcpyAsync(h, s->stats, sizeof(h), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    for (int k = 0; k < LGS_NUM_CONTACT_STATS; ++k) {
        uint64_t t = 0;
        for (int x = 0; x < 8; ++x) t += h[LGS_NUM_CONTACT_STATS * x + k];
        out[k] = t;
    }
    if (reset) {
        HIP_TRY(hipMemsetAsync(s->stats, 0, sizeof(h), s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
    }
    return LGS_OK;
}

LGS_API int lgs_debug_set_phase_buffer(void* dev_ptr) {
#ifdef LGS_PHASE_STAMPS
    unsigned long long* p = (unsigned long long*)dev_ptr;
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_phase_buf), &p, sizeof(p)));
    return LGS_OK;
#else
    (void)dev_ptr;
    return set_err(LGS_ERR_STATE, "library built without -DLGS_PHASE_STAMPS");
#endif
}

LGS_API const char* lgs_get_body_name(lgs_sim* s, int32_t i) {
    if (!s || i < 0 || i >= (int32_t)s->body_names.size()) { set_err(LGS_ERR_ARG, "lgs_get_body_name: no such body"); return nullptr; }
    return s->body_names[i].c_str();
}

LGS_API const char* lgs_get_dof_name(lgs_sim* s, int32_t i) {
    if (!s || i < 0 || i >= (int32_t)s->dof_names.size()) { set_err(LGS_ERR_ARG, "lgs_get_dof_name: no such dof"); return nullptr; }
    return s->dof_names[i].c_str();
}

static int32_t find_name(const std::vector<std::string>& names, const char* name) {
    if (!name) return -1;
    for (size_t i = 0; i < names.size(); ++i)
        if (names[i] == name) return (int32_t)i;
    return -1;
}

LGS_API int32_t lgs_find_body(lgs_sim* s, const char* name) { return s ? find_name(s->body_names, name) : -1; }
LGS_API int32_t lgs_find_dof(lgs_sim* s, const char* name) { return s ? find_name(s->dof_names, name) : -1; }

LGS_API int lgs_get_instantiation(lgs_sim* s, int32_t* dofs, int32_t* bodies, int32_t* rows) {
    if (!s) return set_err(LGS_ERR_ARG, "null argument");
    if (dofs) *dofs = s->Dt;
    if (bodies) *bodies = s->Bt;
    if (rows) *rows = variant_rows(pick(s));
    return LGS_OK;
}

LGS_API int lgs_get_factor_chain(lgs_sim* s, int32_t* chain) {
    if (!s || !chain) return set_err(LGS_ERR_ARG, "null argument");
    const Variant v = pick(s);
    *chain = (v != V_EXTRA && v != V_NONE && s->chain == variant_chain(v)) ? variant_chain(v) : 0;
    return LGS_OK;
}

LGS_API int lgs_get_counts(lgs_sim* s, int32_t* n, int32_t* b, int32_t* d) {
    if (!s) return set_err(LGS_ERR_ARG, "null sim");
    if (n) *n = s->N;
    if (b) *b = s->B;
    if (d) *d = s->D;
    return LGS_OK;
}

}  // extern "C"
