/*
 * lgs_oracle.c — CPU ORACLE (test infrastructure only; never shipped or measured
 * as the product).  Plain serial C restatement of the hot path so that the HIP
 * implementation in unitree-rl-gym_amd/csrc can be checked against it.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 * Two halves, with different parity status:
 *
 *  A. post-physics stack (PD torque, base-frame quantities, commands, termination,
 *     rewards, reset, push, observations) — a restatement of the reference:
 *       legged_gym/envs/base/legged_robot.py  (cited per function below)
 *       legged_gym/envs/h1/h1_env.py, g1/g1_env.py, h1_2/h1_2_env.py
 *       legged_gym/utils/isaacgym_utils.py, utils/math.py
 *     PINNED against golden vectors produced by running the reference's own
 *     Python code (tests/golden/, generator oracle/gen_golden.py).
 *
 *  B. rigid-body dynamics + contact (what IsaacGym/PhysX's gym.simulate does,
 *     legged_robot.py:630).  PhysX is closed source and absent, so this half is
 *     the build's own algorithm, stated once here and once (wave-parallel) in HIP:
 *       floating-base reduced coordinates, world-aligned Plücker frame at the root
 *       origin; composite-rigid-body mass matrix, recursive Newton-Euler bias,
 *       dense Cholesky; joint limits + point contacts vs the z=0 plane as
 *       unilateral rows solved by projected Gauss-Seidel with a circular friction
 *       cone; capsule-proxy self-collision between links of one actor
 *       (create_actor's self_collisions filter, legged_robot.py:373-374);
 *       semi-implicit Euler.  PARITY UNPINNED vs PhysX; pinned only by
 *       analytic tests (free fall, resting height, momentum) and HIP==oracle.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/leggedsim.h"
#include "../unitree-rl-gym_amd/csrc/lgs_detmath.h"

#define NMAX (6 + LGS_MAX_DOFS)
#define ROWMAX 64
#define LGS_PI_F 3.14159265358979323846f

/* ----------------------------------------------------------------- RNG -- */
/* Philox4x32-10, counter = (env, step, stream, index), key = seed.         */
static void philox_round(uint32_t c[4], uint32_t k[2]) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k[0];
    uint32_t n2 = hi0 ^ c[3] ^ k[1];
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k[0] += 0x9E3779B9u; k[1] += 0xBB67AE85u;
}

float orc_uniform(uint64_t seed, uint32_t env, uint32_t step, uint32_t stream, uint32_t index) {
    uint32_t c[4] = {env, step, stream, index};
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int r = 0; r < 10; ++r) philox_round(c, k);
    return (float)(c[0] >> 8) * (1.0f / 16777216.0f);
}

/* torch_rand_float(lo, hi) = (hi - lo) * rand + lo  (isaacgym.torch_utils) */
static float rand_range(float lo, float hi, float u) { return (hi - lo) * u + lo; }

/* ------------------------------------------------------------ 3-vectors -- */
static void cross3(const float a[3], const float b[3], float o[3]) {
    float x = a[1] * b[2] - a[2] * b[1];
    float y = a[2] * b[0] - a[0] * b[2];
    float z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}

/* ---- ground: the z = 0 plane, or a heightfield (lgs_set_heightfield semantics).
 * Cell (i, j) is split along its (i,j)-(i+1,j+1) diagonal (isaacgym
 * terrain_utils.convert_heightfield_to_trimesh); outside the map the edge samples
 * continue.  Set once per process by orc_set_heightfield (test infrastructure). */
static struct {
    const int16_t* h;
    int rows, cols;
    float inv_hs, vs, border;
} g_hf;

void orc_set_heightfield(const int16_t* heights, int rows, int cols, float horizontal_scale, float vertical_scale,
                         float border_size) {
    g_hf.h = (heights && rows > 0) ? heights : NULL;
    g_hf.rows = rows; g_hf.cols = cols;
    g_hf.inv_hs = horizontal_scale > 0.f ? 1.0f / horizontal_scale : 0.f;
    g_hf.vs = vertical_scale;
    g_hf.border = border_size;
}

/* ground height under (x, y) and the unit normal of the triangle there */
float orc_terrain_sample(float x, float y, float* nrm) {
    if (!g_hf.h) {
        nrm[0] = 0.f; nrm[1] = 0.f; nrm[2] = 1.f;
        return 0.f;
    }
    float u = (x + g_hf.border) * g_hf.inv_hs, v = (y + g_hf.border) * g_hf.inv_hs;
    u = fminf(fmaxf(u, 0.f), (float)(g_hf.rows - 1));
    v = fminf(fmaxf(v, 0.f), (float)(g_hf.cols - 1));
    int i = (int)u, j = (int)v;
    if (i > g_hf.rows - 2) i = g_hf.rows - 2;
    if (j > g_hf.cols - 2) j = g_hf.cols - 2;
    const float fu = u - (float)i, fv = v - (float)j;
    const int16_t* h0 = g_hf.h + (size_t)i * g_hf.cols + j;
    const float h00 = (float)h0[0] * g_hf.vs, h01 = (float)h0[1] * g_hf.vs;
    const float h10 = (float)h0[g_hf.cols] * g_hf.vs, h11 = (float)h0[g_hf.cols + 1] * g_hf.vs;
    float du, dv;
    if (fu >= fv) { du = h10 - h00; dv = h11 - h10; }
    else { du = h11 - h01; dv = h01 - h00; }
    const float h = h00 + fu * du + fv * dv;
    const float gx = du * g_hf.inv_hs, gy = dv * g_hf.inv_hs;
    const float inv = 1.f / sqrtf(gx * gx + gy * gy + 1.f);
    nrm[0] = 0.f - gx * inv; nrm[1] = 0.f - gy * inv; nrm[2] = inv;
    return h;
}

/* contact frame: t1 = normalise(e_x - n_x n), t2 = n x t1 (flat ground: +x, +y exactly) */
static void contact_tangents(const float* n, float* t1, float* t2) {
    const float a0 = 1.f - n[0] * n[0], a1 = 0.f - n[0] * n[1], a2 = 0.f - n[0] * n[2];
    const float inv = 1.f / sqrtf(a0 * a0 + a1 * a1 + a2 * a2);
    t1[0] = a0 * inv; t1[1] = a1 * inv; t1[2] = a2 * inv;
    cross3(n, t1, t2);
}
static float dot3(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void matvec(const float R[9], const float v[3], float o[3]) {
    float x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    float y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    float z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}
static float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

/* ---- self-collision (lgs_set_self_collision semantics, include/leggedsim.h): capsule
 * proxies in body frames and the proxy pairs tested every substep.  Set once per process
 * by orc_set_self_collision (test infrastructure). */
static struct {
    int npairs, max_self;
    int body[LGS_MAX_SELF_PAIRS][2];
    float cap[LGS_MAX_SELF_PAIRS][2][7];
} g_self;

void orc_set_self_collision(const lgs_self_collision_desc* d) {
    g_self.npairs = 0;
    g_self.max_self = 0;
    if (!d || d->num_pairs <= 0) return;
    int Q = d->num_pairs < LGS_MAX_SELF_PAIRS ? d->num_pairs : LGS_MAX_SELF_PAIRS;
    for (int q = 0; q < Q; ++q)
        for (int h = 0; h < 2; ++h) {
            int px = d->pair[2 * q + h];
            g_self.body[q][h] = d->proxy_body[px];
            memcpy(g_self.cap[q][h], d->capsule + 7 * px, sizeof(float) * 7);
        }
    g_self.npairs = Q;
    g_self.max_self = d->max_self_contacts;
}

/* closest points of segments p1-q1 and p2-q2 (Ericson, Real-Time Collision Detection,
 * 5.1.9: parameters s, t of the two segments clamped to [0, 1]) */
static void seg_closest(const float p1[3], const float q1[3], const float p2[3], const float q2[3], float c1[3],
                        float c2[3]) {
    float d1[3], d2[3], r[3];
    for (int k = 0; k < 3; ++k) { d1[k] = q1[k] - p1[k]; d2[k] = q2[k] - p2[k]; r[k] = p1[k] - p2[k]; }
    float a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    float s = 0.f, t = 0.f;
    const float eps = 1e-12f;
    if (a <= eps && e <= eps) {
        /* both degenerate: the two points */
    } else if (a <= eps) {
        t = clampf(f / e, 0.f, 1.f);
    } else {
        float c = dot3(d1, r);
        if (e <= eps) {
            s = clampf(-c / a, 0.f, 1.f);
        } else {
            float b = dot3(d1, d2);
            float den = a * e - b * b;
            s = (den != 0.f) ? clampf((b * f - c * e) / den, 0.f, 1.f) : 0.f;
            t = (b * s + f) / e;
            if (t < 0.f) {
                t = 0.f;
                s = clampf(-c / a, 0.f, 1.f);
            } else if (t > 1.f) {
                t = 1.f;
                s = clampf((b - c) / a, 0.f, 1.f);
            }
        }
    }
    for (int k = 0; k < 3; ++k) { c1[k] = p1[k] + d1[k] * s; c2[k] = p2[k] + d2[k] * t; }
}

/* friction frame of a self contact: e = x unless n is within 55 degrees of x (then y),
 * t1 = normalise(e - (e.n) n), t2 = n x t1 */
static void self_tangents(const float n[3], float t1[3], float t2[3]) {
    float a[3];
    if (fabsf(n[0]) < 0.57735f) { a[0] = 1.f - n[0] * n[0]; a[1] = 0.f - n[0] * n[1]; a[2] = 0.f - n[0] * n[2]; }
    else { a[0] = 0.f - n[1] * n[0]; a[1] = 1.f - n[1] * n[1]; a[2] = 0.f - n[1] * n[2]; }
    float inv = 1.f / sqrtf(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    for (int k = 0; k < 3; ++k) t1[k] = a[k] * inv;
    cross3(n, t1, t2);
}
static void matmul(const float A[9], const float B[9], float C[9]) {
    float T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    memcpy(C, T, sizeof(T));
}
static void quat_to_mat(const float q[4], float R[9]) {
    float x = q[0], y = q[1], z = q[2], w = q[3];
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w);     R[2] = 2 * (x * z + y * w);
    R[3] = 2 * (x * y + z * w);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
    R[6] = 2 * (x * z - y * w);     R[7] = 2 * (y * z + x * w);     R[8] = 1 - 2 * (x * x + y * y);
}
static void mat_to_quat(const float R[9], float q[4]) {
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
/* rotation by angle about unit axis a (Rodrigues) */
static void axis_angle(const float a[3], float ang, float R[9]) {
    float s, c;
    lgs_sincosf(ang, &s, &c);
    float t = 1.f - c;
    float x = a[0], y = a[1], z = a[2];
    R[0] = t * x * x + c;     R[1] = t * x * y - s * z; R[2] = t * x * z + s * y;
    R[3] = t * x * y + s * z; R[4] = t * y * y + c;     R[5] = t * y * z - s * x;
    R[6] = t * x * z - s * y; R[7] = t * y * z + s * x; R[8] = t * z * z + c;
}

/* --------------------------------------------------- spatial algebra ---- */
/* motion vector (w, v) at O; force vector (n, f) at O.
 * spatial inertia at O kept as (m, h = m*(c - O), Ib = Icom + m[(r.r)1 - r r^T]) */
typedef struct { float m, h[3], I[6]; } sinertia; /* I: xx yy zz xy xz yz */

static void sin_apply(const sinertia* S, const float w[3], const float v[3], float n[3], float f[3]) {
    float Iw0 = S->I[0] * w[0] + S->I[3] * w[1] + S->I[4] * w[2];
    float Iw1 = S->I[3] * w[0] + S->I[1] * w[1] + S->I[5] * w[2];
    float Iw2 = S->I[4] * w[0] + S->I[5] * w[1] + S->I[2] * w[2];
    float hv[3], hw[3];
    cross3(S->h, v, hv);
    cross3(S->h, w, hw);
    n[0] = Iw0 + hv[0]; n[1] = Iw1 + hv[1]; n[2] = Iw2 + hv[2];
    f[0] = S->m * v[0] - hw[0]; f[1] = S->m * v[1] - hw[1]; f[2] = S->m * v[2] - hw[2];
}

/* ------------------------------------------------------------- model --- */
typedef struct {
    const lgs_model_desc* md;
    int B, D, P, n;
} omodel;

typedef struct {
    float R[LGS_MAX_BODIES][9], p[LGS_MAX_BODIES][3];
    float aw[LGS_MAX_BODIES][3];   /* joint axis, world */
    float cw[LGS_MAX_BODIES][3];   /* com, world */
} okin;

/* forward kinematics (URDF: child = parent * origin * Rot(axis, q)) */
static void fk(const lgs_model_desc* md, const float* root13, const float* dofq, okin* K) {
    int B = md->num_bodies;
    quat_to_mat(root13 + 3, K->R[0]);
    K->p[0][0] = root13[0]; K->p[0][1] = root13[1]; K->p[0][2] = root13[2];
    K->aw[0][0] = K->aw[0][1] = K->aw[0][2] = 0.f;
    for (int b = 1; b < B; ++b) {
        int P = md->parent[b];
        float Rj[9], t[3];
        matmul(K->R[P], md->joint_rot + 9 * b, Rj);
        matvec(K->R[P], md->joint_pos + 3 * b, t);
        K->p[b][0] = K->p[P][0] + t[0]; K->p[b][1] = K->p[P][1] + t[1]; K->p[b][2] = K->p[P][2] + t[2];
        int j = md->dof[b];
        if (j >= 0) {
            float Ra[9];
            matvec(Rj, md->axis + 3 * b, K->aw[b]);
            axis_angle(md->axis + 3 * b, dofq[2 * j], Ra);
            matmul(Rj, Ra, K->R[b]);
        } else {
            memcpy(K->R[b], Rj, sizeof(Rj));
            K->aw[b][0] = K->aw[b][1] = K->aw[b][2] = 0.f;
        }
    }
    for (int b = 0; b < B; ++b) {
        float c[3];
        matvec(K->R[b], md->com + 3 * b, c);
        K->cw[b][0] = K->p[b][0] + c[0]; K->cw[b][1] = K->p[b][1] + c[1]; K->cw[b][2] = K->p[b][2] + c[2];
    }
}

static int g_factor_chain;  /* 0: ascending reduction order; CH > 0: level order (below) */

/* The factorisation order of the HIP instantiation that runs this model
 * (lgs_get_factor_chain): its chain-structured variants eliminate the joint pivots level
 * by level (k = t, CH+t, 2CH+t, .. for t = 0..CH-1, then the base), so every sum below
 * runs over the earlier columns in that order.  Set per model by test infrastructure. */
void orc_set_factor_chain(int ch) { g_factor_chain = ch; }

/* dense Cholesky in place (lower), n <= NMAX.  The reciprocal of each pivot is taken
 * once (IEEE 1/d) and every division by L_kk -- here and in the triangular solves --
 * is a multiplication by it: the HIP kernel's arithmetic, operation for operation
 * (one division per pivot instead of five on its serial chain).  Every update is one
 * fused multiply-add (fmaf), as in the kernel (both build with -ffp-contract=off). */
static void cholesky(float* M, float* invd, int n) {
    /* reduction order: joint columns by level, then the base columns ascending (with the
     * default 0: plain ascending).  Columns of other chains contribute exact zeros, so
     * only the order of the base rows' sums differs between the two. */
    int ord[NMAX];
    const int D = n - 6, ch = g_factor_chain;
    int q = 0;
    if (ch > 0 && D % ch == 0) {
        for (int t = 0; t < ch; ++t)
            for (int c = 0; c < D / ch; ++c) ord[q++] = c * ch + t;
        for (int s = D; s < n; ++s) ord[q++] = s;
    } else {
        for (int s = 0; s < n; ++s) ord[q++] = s;
    }
    for (int k = 0; k < n; ++k) {
        float d = M[k * NMAX + k];
        for (int o = 0; o < n; ++o) {
            const int s = ord[o];
            if (s < k) d = fmaf(-M[k * NMAX + s], M[k * NMAX + s], d);
        }
        d = sqrtf(fmaxf(d, 1e-12f));
        const float inv = 1.0f / d;
        M[k * NMAX + k] = d;
        invd[k] = inv;
        for (int i = k + 1; i < n; ++i) {
            float v = M[i * NMAX + k];
            for (int o = 0; o < n; ++o) {
                const int s = ord[o];
                if (s < k) v = fmaf(-M[i * NMAX + s], M[k * NMAX + s], v);
            }
            M[i * NMAX + k] = v * inv;
        }
    }
}
static void fwd_sub(const float* L, const float* invd, int n, float* x) {
    for (int i = 0; i < n; ++i) {
        float v = x[i];
        for (int s = 0; s < i; ++s) v = fmaf(-L[i * NMAX + s], x[s], v);
        x[i] = v * invd[i];
    }
}
static void bwd_sub(const float* L, const float* invd, int n, float* x) {
    /* subtraction order s = n-1 .. i+1 (the order a column sweep produces) */
    for (int i = n - 1; i >= 0; --i) {
        float v = x[i];
        for (int s = n - 1; s > i; --s) v = fmaf(-L[s * NMAX + i], x[s], v);
        x[i] = v * invd[i];
    }
}

/* capacity-drop counters (lgs_get_contact_stats semantics): bodies touching the ground
 * without a slot, self contacts without a slot, violated joint limits without a row */
static uint64_t g_stats[LGS_NUM_CONTACT_STATS];
static void stats_add(int k, int v) {
    if (v > 0) {
#pragma omp atomic
        g_stats[k] += (uint64_t)v;
    }
}
void orc_contact_stats(uint64_t* out, int reset) {
    for (int k = 0; k < LGS_NUM_CONTACT_STATS; ++k) {
        out[k] = g_stats[k];
        if (reset) g_stats[k] = 0;
    }
}

/* One physics substep of one env (gym.simulate, legged_robot.py:630).
 * root13/dof (in/out), tau [D], contact forces out [B][3], added base mass, friction. */
void orc_substep_env(const lgs_model_desc* md, const lgs_sim_params* sp, float* root13, float* dofs,
                     const float* tau, float* cforce, float added_mass, float shape_friction) {
    const int B = md->num_bodies, D = md->num_dofs, n = 6 + D;
    const float dt = sp->dt;
    const float idt = 1.0f / dt; /* divisions by dt are multiplications by 1/dt (the HIP kernel's) */
    okin K;
    fk(md, root13, dofs, &K);
    const float* O = K.p[0];
    /* root origin velocity from COM velocity */
    float w0[3] = {root13[10], root13[11], root13[12]};
    float rc[3] = {K.cw[0][0] - O[0], K.cw[0][1] - O[1], K.cw[0][2] - O[2]};
    float wxr[3];
    cross3(w0, rc, wxr);
    float vO[3] = {root13[7] - wxr[0], root13[8] - wxr[1], root13[9] - wxr[2]};

    /* spatial inertias at O */
    sinertia Sb[LGS_MAX_BODIES], Ic[LGS_MAX_BODIES];
    for (int b = 0; b < B; ++b) {
        float m = md->mass[b];
        float scale = 1.f;
        if (b == 0 && added_mass != 0.f && m > 0.f) { scale = (m + added_mass) / m; m = m + added_mass; }
        const float* Il = md->inertia + 6 * b;
        float IL[9] = {Il[0] * scale, Il[3] * scale, Il[4] * scale, Il[3] * scale, Il[1] * scale,
                       Il[5] * scale, Il[4] * scale, Il[5] * scale, Il[2] * scale};
        float T[9], Iw[9], Rt[9];
        const float* R = K.R[b];
        for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) Rt[3 * i + j] = R[3 * j + i];
        matmul(R, IL, T);
        matmul(T, Rt, Iw);
        float r[3] = {K.cw[b][0] - O[0], K.cw[b][1] - O[1], K.cw[b][2] - O[2]};
        float rr = dot3(r, r);
        Sb[b].m = m;
        Sb[b].h[0] = m * r[0]; Sb[b].h[1] = m * r[1]; Sb[b].h[2] = m * r[2];
        Sb[b].I[0] = Iw[0] + m * (rr - r[0] * r[0]);
        Sb[b].I[1] = Iw[4] + m * (rr - r[1] * r[1]);
        Sb[b].I[2] = Iw[8] + m * (rr - r[2] * r[2]);
        Sb[b].I[3] = Iw[1] - m * r[0] * r[1];
        Sb[b].I[4] = Iw[2] - m * r[0] * r[2];
        Sb[b].I[5] = Iw[5] - m * r[1] * r[2];
    }
    /* motion subspaces S_j = (a, (p_j - O) x a) */
    float Sw[LGS_MAX_BODIES][3], Sv[LGS_MAX_BODIES][3];
    for (int b = 1; b < B; ++b) {
        float r[3] = {K.p[b][0] - O[0], K.p[b][1] - O[1], K.p[b][2] - O[2]};
        memcpy(Sw[b], K.aw[b], sizeof(float) * 3);
        cross3(r, K.aw[b], Sv[b]);
    }
    /* velocities and bias accelerations (RNEA, qdd = 0, gravity as base accel) */
    float Vw[LGS_MAX_BODIES][3], Vv[LGS_MAX_BODIES][3], Aw[LGS_MAX_BODIES][3], Av[LGS_MAX_BODIES][3];
    float Fn[LGS_MAX_BODIES][3], Ff[LGS_MAX_BODIES][3];
    for (int b = 0; b < B; ++b) {
        if (b == 0) {
            memcpy(Vw[0], w0, 12); memcpy(Vv[0], vO, 12);
            Aw[0][0] = Aw[0][1] = Aw[0][2] = 0.f;
            Av[0][0] = -sp->gravity[0]; Av[0][1] = -sp->gravity[1]; Av[0][2] = -sp->gravity[2];
        } else {
            int P = md->parent[b], j = md->dof[b];
            memcpy(Vw[b], Vw[P], 12); memcpy(Vv[b], Vv[P], 12);
            memcpy(Aw[b], Aw[P], 12); memcpy(Av[b], Av[P], 12);
            if (j >= 0) {
                float qd = dofs[2 * j + 1];
                float sw[3] = {Sw[b][0] * qd, Sw[b][1] * qd, Sw[b][2] * qd};
                float sv[3] = {Sv[b][0] * qd, Sv[b][1] * qd, Sv[b][2] * qd};
                /* A += V_parent x (S qd):  (w x sw, w x sv + v x sw) */
                float t1[3], t2[3], t3[3];
                cross3(Vw[P], sw, t1);
                cross3(Vw[P], sv, t2);
                cross3(Vv[P], sw, t3);
                for (int k = 0; k < 3; ++k) {
                    Aw[b][k] += t1[k];
                    Av[b][k] += t2[k] + t3[k];
                    Vw[b][k] += sw[k];
                    Vv[b][k] += sv[k];
                }
            }
        }
        /* f = I A + V x* (I V) ; (w,v) x* (n,f) = (w x n + v x f, w x f) */
        float IAn[3], IAf[3], IVn[3], IVf[3], a1[3], a2[3], a3[3];
        sin_apply(&Sb[b], Aw[b], Av[b], IAn, IAf);
        sin_apply(&Sb[b], Vw[b], Vv[b], IVn, IVf);
        cross3(Vw[b], IVn, a1);
        cross3(Vv[b], IVf, a2);
        cross3(Vw[b], IVf, a3);
        for (int k = 0; k < 3; ++k) {
            Fn[b][k] = IAn[k] + a1[k] + a2[k];
            Ff[b][k] = IAf[k] + a3[k];
        }
    }
    /* composites: subtree(b) is the DFS range [b, subtree_end[b]); summed last to first */
    float CFn[LGS_MAX_BODIES][3], CFf[LGS_MAX_BODIES][3];
    for (int b = 0; b < B; ++b) {
        memset(&Ic[b], 0, sizeof(sinertia));
        for (int k = 0; k < 3; ++k) CFn[b][k] = CFf[b][k] = 0.f;
        for (int x = md->subtree_end[b] - 1; x >= b; --x) {
            Ic[b].m += Sb[x].m;
            for (int k = 0; k < 3; ++k) { Ic[b].h[k] += Sb[x].h[k]; CFn[b][k] += Fn[x][k]; CFf[b][k] += Ff[x][k]; }
            for (int k = 0; k < 6; ++k) Ic[b].I[k] += Sb[x].I[k];
        }
    }
    /* mass matrix + bias */
    static __thread float M[NMAX * NMAX];
    float C[NMAX];
    memset(M, 0, sizeof(M));
    {
        const sinertia* S = &Ic[0];
        float I3[9] = {S->I[0], S->I[3], S->I[4], S->I[3], S->I[1], S->I[5], S->I[4], S->I[5], S->I[2]};
        const float* h = S->h;
        float H[9] = {0, -h[2], h[1], h[2], 0, -h[0], -h[1], h[0], 0}; /* [h]x */
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                M[i * NMAX + j] = I3[3 * i + j];
                M[i * NMAX + 3 + j] = H[3 * i + j];
                M[(3 + i) * NMAX + j] = H[3 * j + i];
                M[(3 + i) * NMAX + 3 + j] = (i == j) ? S->m : 0.f;
            }
        for (int k = 0; k < 3; ++k) { C[k] = CFn[0][k]; C[3 + k] = CFf[0][k]; }
    }
    for (int b = 1; b < B; ++b) {
        int j = md->dof[b];
        if (j < 0) continue;
        float cn[3], cf[3];
        sin_apply(&Ic[b], Sw[b], Sv[b], cn, cf);
        for (int k = 0; k < 3; ++k) {
            M[k * NMAX + 6 + j] = M[(6 + j) * NMAX + k] = cn[k];
            M[(3 + k) * NMAX + 6 + j] = M[(6 + j) * NMAX + 3 + k] = cf[k];
        }
        C[6 + j] = dot3(Sw[b], CFn[b]) + dot3(Sv[b], CFf[b]);
        /* ancestors (and self) along the chain */
        for (int d = 1; d <= md->depth[b]; ++d) {
            int a = md->chain[b * LGS_MAX_DEPTH + d];
            int i = md->dof[a];
            if (i < 0) continue;
            float v = dot3(Sw[a], cn) + dot3(Sv[a], cf);
            M[(6 + i) * NMAX + 6 + j] = v;
            M[(6 + j) * NMAX + 6 + i] = v;
        }
        M[(6 + j) * NMAX + 6 + j] += sp->armature;
    }
    float rhs0[NMAX];
    for (int k = 0; k < 6; ++k) rhs0[k] = -C[k];
    for (int j = 0; j < D; ++j) rhs0[6 + j] = tau[j] - C[6 + j];
    /* The factorisation and every solve run in the LEAVES-FIRST order p = n-1-i of the
     * natural [base, joints in DFS order] index (each DOF after all of its descendants):
     * L then has no fill-in, its structural zeros are exact, and the HIP kernel skips
     * them (leggedsim.hip l_nz) without changing a result bit. */
    static __thread float Mp[NMAX * NMAX];
    float rhs[NMAX], qdd[NMAX];
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) Mp[i * NMAX + j] = M[(n - 1 - i) * NMAX + (n - 1 - j)];
        rhs[i] = rhs0[n - 1 - i];
    }
    float invd[NMAX];
    cholesky(Mp, invd, n);
    fwd_sub(Mp, invd, n, rhs);
    bwd_sub(Mp, invd, n, rhs);
    for (int i = 0; i < n; ++i) qdd[i] = rhs[n - 1 - i];

    /* free velocity (classical velocity of the root origin after dt) */
    float qf[NMAX];
    float wxv[3];
    cross3(w0, vO, wxv);
    for (int k = 0; k < 3; ++k) {
        qf[k] = w0[k] + dt * qdd[k];
        qf[3 + k] = vO[k] + dt * (qdd[3 + k] + wxv[k]);
    }
    for (int j = 0; j < D; ++j) qf[6 + j] = dofs[2 * j + 1] + dt * qdd[6 + j];

    /* ---- constraint rows: contacts (n, t1, t2) first, then joint limits.
     * Gauss-Seidel visits them in this order (the HIP kernel keeps contact c at
     * rows 3c..3c+2 so its row registers are compile-time indexed).
     * Contact slots (include/leggedsim.h, above lgs_self_collision_desc): one per body
     * touching the ground, for its first touching candidate (candidate order); then up to
     * max_self self contacts (pair order); then the other touching ground candidates
     * (candidate order), while the max_contacts slots last.  Joint limits (DOF order) take
     * max_rows - 3*max_contacts rows plus those of the unused contact slots.  What does not
     * fit is counted (orc_contact_stats). ---- */
    static __thread float J[ROWMAX][NMAX];
    float tgt[ROWMAX], lam[ROWMAX], v[ROWMAX];
    int kind[ROWMAX]; /* 0 unilateral, 1 friction pair head, 2 friction pair tail */
    int cb[ROWMAX / 3 + 1], cb2[ROWMAX / 3 + 1];
    float cmu[ROWMAX / 3 + 1];                           /* friction coefficient per contact */
    const float mu = 0.5f * (sp->ground_friction + shape_friction); /* ground: average with the plane */
    int nr = 0;
    const float beta = sp->baumgarte;
    const int max_rows = sp->max_rows < ROWMAX ? sp->max_rows : ROWMAX;
    const int maxc = sp->max_contacts;
    const int max_limit = max_rows - 3 * maxc;
    int nc = 0;
    float cpt[ROWMAX / 3 + 1][3];
    float cfr[ROWMAX / 3 + 1][3][3]; /* contact frame: normal, tangent 1, tangent 2 */
    /* self contacts: every pair tested, the first maxc (pair order) kept */
    int nsf = 0, sc_body[ROWMAX / 3 + 1][2];
    float sc_pt[ROWMAX / 3 + 1][3], sc_sep[ROWMAX / 3 + 1], sc_n[ROWMAX / 3 + 1][3];
    for (int q = 0; q < g_self.npairs; ++q) {
        float seg[2][2][3];
        for (int h = 0; h < 2; ++h) {
            int b = g_self.body[q][h];
            for (int e = 0; e < 2; ++e) {
                matvec(K.R[b], g_self.cap[q][h] + 3 * e, seg[h][e]);
                for (int k = 0; k < 3; ++k) seg[h][e][k] += K.p[b][k];
            }
        }
        float c1[3], c2[3];
        seg_closest(seg[0][0], seg[0][1], seg[1][0], seg[1][1], c1, c2);
        float dx[3] = {c1[0] - c2[0], c1[1] - c2[1], c1[2] - c2[2]};
        float dist = sqrtf(dot3(dx, dx));
        float nrm[3] = {0.f, 0.f, 1.f};
        if (dist > 1e-9f) {
            float inv = 1.f / dist;
            for (int k = 0; k < 3; ++k) nrm[k] = dx[k] * inv;
        }
        float ra = g_self.cap[q][0][6], rb = g_self.cap[q][1][6];
        float sep = dist - ra - rb - sp->rest_offset;
        if (!(sep < sp->contact_offset)) continue;
        if (nsf < maxc) {
            sc_body[nsf][0] = g_self.body[q][0];
            sc_body[nsf][1] = g_self.body[q][1];
            for (int k = 0; k < 3; ++k) {
                sc_pt[nsf][k] = 0.5f * ((c1[k] - ra * nrm[k]) + (c2[k] + rb * nrm[k]));
                sc_n[nsf][k] = nrm[k];
            }
            sc_sep[nsf] = sep;
        }
        ++nsf;
    }
    /* ground candidates: primaries (a body's first touching candidate) and the others */
    struct gcand { int b; float pc[3], sep, nrm[3]; } prim[ROWMAX / 3 + 1], sec[ROWMAX / 3 + 1];
    int np = 0, nsec = 0;
    int seen[LGS_MAX_BODIES];
    memset(seen, 0, sizeof(seen));
    for (int k = 0; k < md->num_points; ++k) {
        int b = md->pt_body[k];
        float c[3];
        matvec(K.R[b], md->pt_pos + 3 * k, c);
        c[0] += K.p[b][0]; c[1] += K.p[b][1]; c[2] += K.p[b][2];
        float nrm[3];
        const float rad = md->pt_radius[k];
        const float hg = orc_terrain_sample(c[0], c[1], nrm);
        /* signed distance of the sphere centre to the ground triangle's plane */
        float sep = (c[2] - hg) * nrm[2] - rad - sp->rest_offset;
        if (!(sep < sp->contact_offset)) continue;
        struct gcand* g = NULL;
        if (!seen[b]) {
            seen[b] = 1;
            if (np < maxc) g = &prim[np];
            ++np;
        } else {
            if (nsec < maxc) g = &sec[nsec];
            ++nsec;
        }
        if (!g) continue;
        g->b = b;
        g->sep = sep;
        for (int t = 0; t < 3; ++t) { g->pc[t] = c[t] - rad * nrm[t]; g->nrm[t] = nrm[t]; }
    }
    const int npg = np < maxc ? np : maxc;
    int nsc = nsf < g_self.max_self ? nsf : g_self.max_self;
    if (nsc > maxc - npg) nsc = maxc - npg;
    const int nsu = nsec < maxc - npg - nsc ? nsec : maxc - npg - nsc;
    stats_add(0, np - npg);
    stats_add(1, nsf - nsc);
    for (int i = 0; i < npg + nsu; ++i) {
        const struct gcand* g = i < npg ? &prim[i] : &sec[i - npg];
        const int b = g->b;
        const float* pc = g->pc;
        const float sep = g->sep;
        float r[3] = {pc[0] - O[0], pc[1] - O[1], pc[2] - O[2]};
        float dirs[3][3];
        memcpy(dirs[0], g->nrm, 12);
        contact_tangents(g->nrm, dirs[1], dirs[2]);
        memcpy(cfr[nc], dirs, 36);
        for (int dd = 0; dd < 3; ++dd) {
            const float* d = dirs[dd];
            float* row = J[nr + dd];
            memset(row, 0, sizeof(float) * n);
            cross3(r, d, row);
            row[3] = d[0]; row[4] = d[1]; row[5] = d[2];
            for (int l = 1; l <= md->depth[b]; ++l) {
                int a = md->chain[b * LGS_MAX_DEPTH + l];
                int j = md->dof[a];
                if (j < 0) continue;
                float rp[3] = {pc[0] - K.p[a][0], pc[1] - K.p[a][1], pc[2] - K.p[a][2]}, t[3];
                cross3(K.aw[a], rp, t);
                row[6 + j] = dot3(d, t);
            }
        }
        tgt[nr] = sep >= 0.f ? -sep * idt : fminf(-beta * sep * idt, sp->max_depenetration_velocity);
        tgt[nr + 1] = tgt[nr + 2] = 0.f;
        kind[nr] = 0; kind[nr + 1] = 1; kind[nr + 2] = 2;
        cb[nc] = b;
        cb2[nc] = -1;
        cmu[nc] = mu;
        memcpy(cpt[nc], pc, 12);
        nr += 3;
        ++nc;
    }
    /* the self contacts: rows J_a(pc) d - J_b(pc) d (the floating-base columns cancel) */
    for (int i = 0; i < nsc; ++i) {
        const int a = sc_body[i][0], b = sc_body[i][1];
        const float* pc = sc_pt[i];
        float dirs[3][3];
        memcpy(dirs[0], sc_n[i], 12);
        self_tangents(sc_n[i], dirs[1], dirs[2]);
        memcpy(cfr[nc], dirs, 36);
        for (int dd = 0; dd < 3; ++dd) {
            const float* d = dirs[dd];
            float* row = J[nr + dd];
            memset(row, 0, sizeof(float) * n);
            for (int l = 1; l <= md->depth[a]; ++l) {
                int x = md->chain[a * LGS_MAX_DEPTH + l];
                int j = md->dof[x];
                if (j < 0) continue;
                float rp[3] = {pc[0] - K.p[x][0], pc[1] - K.p[x][1], pc[2] - K.p[x][2]}, t[3];
                cross3(K.aw[x], rp, t);
                row[6 + j] = dot3(d, t);
            }
            for (int l = 1; l <= md->depth[b]; ++l) {
                int x = md->chain[b * LGS_MAX_DEPTH + l];
                int j = md->dof[x];
                if (j < 0) continue;
                float rp[3] = {pc[0] - K.p[x][0], pc[1] - K.p[x][1], pc[2] - K.p[x][2]}, t[3];
                cross3(K.aw[x], rp, t);
                row[6 + j] = row[6 + j] - dot3(d, t);
            }
        }
        const float sep = sc_sep[i];
        tgt[nr] = sep >= 0.f ? -sep * idt : fminf(-beta * sep * idt, sp->max_depenetration_velocity);
        tgt[nr + 1] = tgt[nr + 2] = 0.f;
        kind[nr] = 0; kind[nr + 1] = 1; kind[nr + 2] = 2;
        cb[nc] = a;
        cb2[nc] = b;
        cmu[nc] = shape_friction; /* both shapes carry the env's friction: their average */
        memcpy(cpt[nc], pc, 12);
        nr += 3;
        ++nc;
    }
    /* joint limits in DOF order: max_limit rows, then the rows of the unused contact slots */
    const int max_lim_all = max_limit + 3 * (maxc - nc);
    int nl = 0;
    for (int j = 0; j < D; ++j) {
        float q = dofs[2 * j], lo = md->dof_lower[j], hi = md->dof_upper[j];
        float qn = q + dt * qf[6 + j];
        if (!(qn < lo) && !(qn > hi)) continue;
        if (nl++ >= max_lim_all) continue;
        memset(J[nr], 0, sizeof(float) * n);
        float gap;
        if (qn < lo) {
            J[nr][6 + j] = 1.f;
            gap = q - lo;
        } else {
            J[nr][6 + j] = -1.f;
            gap = hi - q;
        }
        tgt[nr] = gap >= 0.f ? -gap * idt : -beta * gap * idt;
        kind[nr++] = 0;
    }
    stats_add(2, nl > max_lim_all ? nl - max_lim_all : 0);
    /* Y = L^-1 J^T (leaves-first columns) ; A = Y^T Y ; v = J qf (natural order) */
    static __thread float Y[ROWMAX][NMAX];
    static __thread float A[ROWMAX][ROWMAX];
    for (int r = 0; r < nr; ++r) {
        for (int i = 0; i < n; ++i) Y[r][i] = J[r][n - 1 - i];
        fwd_sub(Mp, invd, n, Y[r]);
        float s = 0.f;
        for (int i = 0; i < n; ++i) s = fmaf(J[r][i], qf[i], s);
        v[r] = s;
        lam[r] = 0.f;
    }
    for (int r = 0; r < nr; ++r)
        for (int s = 0; s <= r; ++s) {
            float a = 0.f;
            for (int i = 0; i < n; ++i) a = fmaf(Y[r][i], Y[s][i], a); /* the MFMA's fp32 fma chain */
            A[r][s] = A[s][r] = a;
        }
    float inv[ROWMAX];
    for (int r = 0; r < nr; ++r) inv[r] = 1.f / (A[r][r] + 1e-9f);
    for (int it = 0; it < sp->solver_iterations; ++it) {
        for (int r = 0; r < nr; ++r) {
            if (kind[r] == 0) {
                float ln = fmaxf(0.f, lam[r] + (tgt[r] - v[r]) * inv[r]);
                float d = ln - lam[r];
                lam[r] = ln;
                for (int s = 0; s < nr; ++s) v[s] = fmaf(A[s][r], d, v[s]); /* the kernel's fused update */
            } else if (kind[r] == 1) {
                float lim = cmu[r / 3] * lam[r - 1];
                float l1 = lam[r] - v[r] * inv[r];
                float l2 = lam[r + 1] - v[r + 1] * inv[r + 1];
                /* the cone test on squared norms: the square root (and the division) only when
                   the friction impulse is projected back onto the cone (sliding) */
                const float n2 = l1 * l1 + l2 * l2;
                if (n2 > lim * lim) {
                    const float nrm = sqrtf(n2);
                    float s = nrm > 0.f ? lim / nrm : 0.f;
                    l1 *= s; l2 *= s;
                }
                float d1 = l1 - lam[r], d2 = l2 - lam[r + 1];
                lam[r] = l1; lam[r + 1] = l2;
                for (int s = 0; s < nr; ++s) v[s] = fmaf(A[s][r + 1], d2, fmaf(A[s][r], d1, v[s]));
            }
        }
    }
    /* qd' = qf + L^-T (Y lambda) */
    float z[NMAX];
    for (int i = 0; i < n; ++i) {
        float s = 0.f;
        for (int r = 0; r < nr; ++r) s = fmaf(Y[r][i], lam[r], s);
        z[i] = s;
    }
    bwd_sub(Mp, invd, n, z);
    float qn[NMAX];
    for (int i = 0; i < n; ++i) qn[i] = qf[i] + z[n - 1 - i];
    if (sp->clamp_joint_velocity)
        for (int j = 0; j < D; ++j) {
            float lim = md->dof_velocity[j];
            if (lim > 0.f) qn[6 + j] = fminf(fmaxf(qn[6 + j], -lim), lim);
        }
    /* contact forces (last substep), world frame */
    for (int b = 0; b < B; ++b) cforce[3 * b] = cforce[3 * b + 1] = cforce[3 * b + 2] = 0.f;
    for (int c = 0; c < nc; ++c) {
        int r = 3 * c;
        float* F = cforce + 3 * cb[c];
        for (int t = 0; t < 3; ++t) /* ln n + l1 t1 + l2 t2 */
            F[t] += (lam[r] * cfr[c][0][t] + lam[r + 1] * cfr[c][1][t] + lam[r + 2] * cfr[c][2][t]) * idt;
        if (cb2[c] >= 0) { /* a self contact pushes its second body the other way */
            float* G = cforce + 3 * cb2[c];
            for (int t = 0; t < 3; ++t)
                G[t] -= (lam[r] * cfr[c][0][t] + lam[r + 1] * cfr[c][1][t] + lam[r + 2] * cfr[c][2][t]) * idt;
        }
    }
    (void)cpt;
    /* integrate (semi-implicit Euler) */
    for (int k = 0; k < 3; ++k) root13[k] += dt * qn[3 + k];
    {
        float* q = root13 + 3;
        const float* w = qn;
        float dq[4];
        dq[0] = 0.5f * dt * (q[3] * w[0] + (w[1] * q[2] - w[2] * q[1]));
        dq[1] = 0.5f * dt * (q[3] * w[1] + (w[2] * q[0] - w[0] * q[2]));
        dq[2] = 0.5f * dt * (q[3] * w[2] + (w[0] * q[1] - w[1] * q[0]));
        dq[3] = 0.5f * dt * (-(w[0] * q[0] + w[1] * q[1] + w[2] * q[2]));
        float nn = 0.f;
        for (int k = 0; k < 4; ++k) { q[k] += dq[k]; nn += q[k] * q[k]; }
        nn = 1.f / sqrtf(nn);
        for (int k = 0; k < 4; ++k) q[k] *= nn;
    }
    for (int j = 0; j < D; ++j) {
        dofs[2 * j + 1] = qn[6 + j];
        dofs[2 * j] += dt * qn[6 + j];
    }
    {
        float R[9], c[3], wc[3];
        quat_to_mat(root13 + 3, R);
        matvec(R, md->com, c);
        cross3(qn, c, wc);
        for (int k = 0; k < 3; ++k) { root13[10 + k] = qn[k]; root13[7 + k] = qn[3 + k] + wc[k]; }
    }
}

/* rigid_body_states [B][13] of one env from its state */
void orc_body_states_env(const lgs_model_desc* md, const float* root13, const float* dofs, float* rbs) {
    okin K;
    fk(md, root13, dofs, &K);
    const int B = md->num_bodies;
    const float* O = K.p[0];
    float w0[3] = {root13[10], root13[11], root13[12]};
    float rc[3] = {K.cw[0][0] - O[0], K.cw[0][1] - O[1], K.cw[0][2] - O[2]}, t[3];
    cross3(w0, rc, t);
    float Vw[LGS_MAX_BODIES][3], Vv[LGS_MAX_BODIES][3];
    Vw[0][0] = w0[0]; Vw[0][1] = w0[1]; Vw[0][2] = w0[2];
    for (int k = 0; k < 3; ++k) Vv[0][k] = root13[7 + k] - t[k];
    for (int b = 1; b < B; ++b) {
        int P = md->parent[b], j = md->dof[b];
        memcpy(Vw[b], Vw[P], 12); memcpy(Vv[b], Vv[P], 12);
        if (j >= 0) {
            float qd = dofs[2 * j + 1], r[3] = {K.p[b][0] - O[0], K.p[b][1] - O[1], K.p[b][2] - O[2]}, sv[3];
            cross3(r, K.aw[b], sv);
            for (int k = 0; k < 3; ++k) { Vw[b][k] += K.aw[b][k] * qd; Vv[b][k] += sv[k] * qd; }
        }
    }
    for (int b = 0; b < B; ++b) {
        float* o = rbs + 13 * b;
        o[0] = K.p[b][0]; o[1] = K.p[b][1]; o[2] = K.p[b][2];
        mat_to_quat(K.R[b], o + 3);
        float r[3] = {K.cw[b][0] - O[0], K.cw[b][1] - O[1], K.cw[b][2] - O[2]}, wr[3];
        cross3(Vw[b], r, wr);
        for (int k = 0; k < 3; ++k) { o[7 + k] = Vv[b][k] + wr[k]; o[10 + k] = Vw[b][k]; }
    }
}

/* ===================================================== post-physics ==== */

/* isaacgym.torch_utils.quat_rotate_inverse, op order of the torch code */
static void quat_rotate_inverse(const float q[4], const float v[3], float o[3]) {
    float w = q[3];
    float s = 2.0f * w * w - 1.0f;
    float c[3];
    cross3(q, v, c);
    float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
    for (int k = 0; k < 3; ++k) o[k] = v[k] * s - c[k] * w * 2.0f + q[k] * d * 2.0f;
}
/* isaacgym.torch_utils.quat_apply */
static void quat_apply(const float q[4], const float v[3], float o[3]) {
    float t[3], u[3];
    cross3(q, v, t);
    t[0] *= 2.f; t[1] *= 2.f; t[2] *= 2.f;
    cross3(q, t, u);
    for (int k = 0; k < 3; ++k) o[k] = v[k] + q[3] * t[k] + u[k];
}
/* legged_gym/utils/isaacgym_utils.py:11-29 */
static void get_euler_xyz(const float q[4], float rpy[3]) {
    float qx = q[0], qy = q[1], qz = q[2], qw = q[3];
    float sinr = 2.0f * (qw * qx + qy * qz);
    float cosr = qw * qw - qx * qx - qy * qy + qz * qz;
    rpy[0] = lgs_atan2f(sinr, cosr);
    float sinp = 2.0f * (qw * qy - qz * qx);
    rpy[1] = fabsf(sinp) >= 1.f ? copysignf(LGS_PI_F / 2.0f, sinp) : lgs_asinf(sinp);
    float siny = 2.0f * (qw * qz + qx * qy);
    float cosy = qw * qw + qx * qx - qy * qy - qz * qz;
    rpy[2] = lgs_atan2f(siny, cosy);
}
/* legged_gym/utils/math.py:15-19 (torch remainder semantics) */
static float wrap_to_pi(float a) {
    const float tp = 2.0f * LGS_PI_F;
    float m = fmodf(a, tp);
    if (m != 0.f && m < 0.f) m += tp;
    if (m > LGS_PI_F) m -= tp;
    return m;
}
static float clipf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

typedef struct {
    float* root; float* dofs; float* cforce; float* rbs;
} ostate;

/* _resample_commands (legged_robot.py:519-538) */
static void resample_commands(const lgs_task_params* T, float* cmd, uint64_t seed, uint32_t env, uint32_t step,
                              uint32_t stream) {
    cmd[0] = rand_range(T->cmd_lin_vel_x[0], T->cmd_lin_vel_x[1], orc_uniform(seed, env, step, stream, 0));
    cmd[1] = rand_range(T->cmd_lin_vel_y[0], T->cmd_lin_vel_y[1], orc_uniform(seed, env, step, stream, 1));
    if (T->heading_command)
        cmd[3] = rand_range(T->cmd_heading[0], T->cmd_heading[1], orc_uniform(seed, env, step, stream, 2));
    else
        cmd[2] = rand_range(T->cmd_ang_vel_yaw[0], T->cmd_ang_vel_yaw[1], orc_uniform(seed, env, step, stream, 2));
    float nrm = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]);
    float keep = nrm > 0.2f ? 1.f : 0.f;
    cmd[0] *= keep; cmd[1] *= keep;
}

/* reward terms (legged_robot.py:843-939, h1_env.py:98-123) */
static float reward_term(int id, const lgs_task_params* T, int A, const float* bl, const float* ba, const float* pg,
                         const float* root, const float* q, const float* qd, const float* last_qd, const float* act,
                         const float* last_act, const float* tau, const float* cf, const float* cmd,
                         float* air, uint8_t* last_c, const float* rbs, const float* leg_phase, int reset, int timeout) {
    float s = 0.f;
    switch (id) {
    case LGS_REW_LIN_VEL_Z: return bl[2] * bl[2];
    case LGS_REW_ANG_VEL_XY: return ba[0] * ba[0] + ba[1] * ba[1];
    case LGS_REW_ORIENTATION: return pg[0] * pg[0] + pg[1] * pg[1];
    case LGS_REW_BASE_HEIGHT: { float d = root[2] - T->base_height_target; return d * d; }
    case LGS_REW_TORQUES: for (int j = 0; j < A; ++j) s += tau[j] * tau[j]; return s;
    case LGS_REW_DOF_VEL: for (int j = 0; j < A; ++j) s += qd[j] * qd[j]; return s;
    case LGS_REW_DOF_ACC:
        for (int j = 0; j < A; ++j) { float d = (last_qd[j] - qd[j]) / T->control_dt; s += d * d; }
        return s;
    case LGS_REW_ACTION_RATE:
        for (int j = 0; j < A; ++j) { float d = last_act[j] - act[j]; s += d * d; }
        return s;
    case LGS_REW_COLLISION:
        for (int i = 0; i < T->num_penalised; ++i) {
            const float* F = cf + 3 * T->penalised_idx[i];
            s += (sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) > 0.1f) ? 1.f : 0.f;
        }
        return s;
    case LGS_REW_DOF_POS_LIMITS:
        for (int j = 0; j < A; ++j) {
            float o = -fminf(q[j] - T->soft_dof_pos_lower[j], 0.f);
            o += fmaxf(q[j] - T->soft_dof_pos_upper[j], 0.f);
            s += o;
        }
        return s;
    case LGS_REW_DOF_VEL_LIMITS:
        for (int j = 0; j < A; ++j)
            s += clipf(fabsf(qd[j]) - T->dof_vel_limits[j] * T->soft_dof_vel_limit, 0.f, 1.f);
        return s;
    case LGS_REW_TORQUE_LIMITS:
        for (int j = 0; j < A; ++j) s += fmaxf(fabsf(tau[j]) - T->torque_limits[j] * T->soft_torque_limit, 0.f);
        return s;
    case LGS_REW_TRACKING_LIN_VEL: {
        float e0 = cmd[0] - bl[0], e1 = cmd[1] - bl[1];
        float e = e0 * e0 + e1 * e1;
        return lgs_expf(-e / T->tracking_sigma);
    }
    case LGS_REW_TRACKING_ANG_VEL: {
        float e = cmd[2] - ba[2];
        e = e * e;
        return lgs_expf(-e / T->tracking_sigma);
    }
    case LGS_REW_FEET_AIR_TIME: { /* legged_robot.py:912-923, mutates air/last_c */
        float r = 0.f;
        int filt[LGS_MAX_FEET];
        for (int f = 0; f < T->num_feet; ++f) {
            int contact = cf[3 * T->feet_idx[f] + 2] > 1.f;
            filt[f] = contact || last_c[f];
            last_c[f] = (uint8_t)contact;
            float first = (air[f] > 0.f && filt[f]) ? 1.f : 0.f;
            air[f] += T->control_dt;
            r += (air[f] - 0.5f) * first;
        }
        float cn = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]);
        r *= (cn > 0.1f) ? 1.f : 0.f;
        for (int f = 0; f < T->num_feet; ++f)
            if (filt[f]) air[f] = 0.f; /* feet_air_time *= ~contact_filt */
        return r;
    }
    case LGS_REW_FEET_STUMBLE: {
        for (int f = 0; f < T->num_feet; ++f) {
            const float* F = cf + 3 * T->feet_idx[f];
            if (sqrtf(F[0] * F[0] + F[1] * F[1]) > 5.f * fabsf(F[2])) return 1.f;
        }
        return 0.f;
    }
    case LGS_REW_STAND_STILL: {
        for (int j = 0; j < A; ++j) s += fabsf(q[j] - T->default_dof_pos[j]);
        float cn = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]);
        return s * ((cn < 0.1f) ? 1.f : 0.f);
    }
    case LGS_REW_FEET_CONTACT_FORCES:
        for (int f = 0; f < T->num_feet; ++f) {
            const float* F = cf + 3 * T->feet_idx[f];
            s += fmaxf(sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) - T->max_contact_force, 0.f);
        }
        return s;
    case LGS_REW_ALIVE: return 1.0f;
    case LGS_REW_CONTACT: /* h1_env.py:98-105 */
        for (int f = 0; f < T->num_feet; ++f) {
            int stance = leg_phase[f] < T->stance_threshold;
            int contact = cf[3 * T->feet_idx[f] + 2] > 1.f;
            s += (contact == stance) ? 1.f : 0.f;
        }
        return s;
    case LGS_REW_FEET_SWING_HEIGHT: /* h1_env.py:107-110 */
        for (int f = 0; f < T->num_feet; ++f) {
            const float* F = cf + 3 * T->feet_idx[f];
            int contact = sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) > 1.f;
            float d = rbs[13 * T->feet_idx[f] + 2] - T->swing_height_target;
            s += d * d * (contact ? 0.f : 1.f);
        }
        return s;
    case LGS_REW_CONTACT_NO_VEL: /* h1_env.py:115-119 */
        for (int f = 0; f < T->num_feet; ++f) {
            const float* F = cf + 3 * T->feet_idx[f];
            float c = sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) > 1.f ? 1.f : 0.f;
            const float* v = rbs + 13 * T->feet_idx[f] + 7;
            for (int k = 0; k < 3; ++k) { float x = v[k] * c; s += x * x; }
        }
        return s;
    case LGS_REW_HIP_POS: /* h1_env.py:121-123 */
        for (int i = 0; i < T->num_hip; ++i) s += q[T->hip_dofs[i]] * q[T->hip_dofs[i]];
        return s;
    default: return 0.f;
    }
    (void)reset; (void)timeout;
}

/* _compute_torques (legged_robot.py:649-671), P/V/T control */
static void compute_torques(const lgs_task_params* T, int D, const float* act, const float* dofs,
                            const float* last_qd, float sim_dt, float* tau) {
    for (int j = 0; j < D; ++j) {
        float as = act[j] * T->action_scale;
        float q = dofs[2 * j], qd = dofs[2 * j + 1], t;
        if (T->control_type == 0)
            t = T->p_gains[j] * (as + T->default_dof_pos[j] - q) - T->d_gains[j] * qd;
        else if (T->control_type == 1)
            t = T->p_gains[j] * (as - qd) - T->d_gains[j] * (qd - last_qd[j]) / sim_dt;
        else
            t = as;
        tau[j] = clipf(t, -T->torque_limits[j], T->torque_limits[j]);
    }
}

/* reset_idx (legged_robot.py:723-768) of env e: dofs, root, commands, buffers, episode sums
 * into the extras accumulator */
static void reset_env(const lgs_model_desc* md, const lgs_task_params* T, int N, int e, float* root, float* dofs,
                      const lgs_env_buffers* E, int64_t step_counter) {
    const int D = md->num_dofs, A = T->num_actions;
    const uint64_t seed = T->seed;
    const uint32_t step = (uint32_t)step_counter;
    float* act = E->actions + A * e;
    float* last_act = E->last_actions + A * e;
    float* last_qd = E->last_dof_vel + D * e;
    float* air = E->feet_air_time + T->num_feet * e;
    for (int j = 0; j < D; ++j) {                              /* _reset_dofs :566-567 */
        dofs[2 * j] = T->default_dof_pos[j] * rand_range(0.5f, 1.5f, orc_uniform(seed, e, step, LGS_STREAM_RESET_DOF, j));
        dofs[2 * j + 1] = 0.f;
    }
    for (int k = 0; k < 13; ++k) root[k] = T->base_init_state[k];  /* _reset_root_states :587-590 */
    for (int k = 0; k < 3; ++k) root[k] += E->env_origins[3 * e + k];
    if (T->custom_origins) /* terrain tiles: xy within 1 m of the centre (:582-585) */
        for (int k = 0; k < 2; ++k) root[k] += rand_range(-1.f, 1.f, orc_uniform(seed, e, step, LGS_STREAM_RESET_ROOT, 6 + k));
    for (int k = 0; k < 6; ++k) root[7 + k] = rand_range(-0.5f, 0.5f, orc_uniform(seed, e, step, LGS_STREAM_RESET_ROOT, k));
    resample_commands(T, E->commands + 4 * e, seed, (uint32_t)e, step, LGS_STREAM_RESET_CMD);
    for (int j = 0; j < A; ++j) { act[j] = 0.f; last_act[j] = 0.f; }
    for (int j = 0; j < D; ++j) last_qd[j] = 0.f;
    for (int f = 0; f < T->num_feet; ++f) air[f] = 0.f;
    E->episode_length[e] = 0;
    int nsum = T->num_rewards + (T->has_termination_reward ? 1 : 0);
    for (int k = 0; k < nsum; ++k) {  /* shared across the OpenMP env loop */
#pragma omp atomic
        E->episode_acc[k] += E->episode_sums[(size_t)k * N + e];
        E->episode_sums[(size_t)k * N + e] = 0.f;
    }
#pragma omp atomic
    E->episode_acc[nsum] += 1.f;
}

/* post_physics_step (legged_robot.py:673-709) for env e, state already simulated.
 * `full` = 1 runs the whole stack incl. reset/push; feet rigid states must be
 * current in st->rbs for humanoid layouts. */
void orc_post_physics_env(const lgs_model_desc* md, const lgs_task_params* T, int N, int e, ostate* st,
                          const lgs_env_buffers* E, int64_t step_counter) {
    const int D = md->num_dofs, B = md->num_bodies, A = T->num_actions;
    const int O = T->num_obs, P = T->num_privileged_obs;
    const uint64_t seed = T->seed;
    const uint32_t step = (uint32_t)step_counter;
    float* root = st->root + 13 * e;
    float* dofs = st->dofs + 2 * D * e;
    const float* cf = st->cforce + 3 * B * e;
    const float* rbs = st->rbs ? st->rbs + 13 * B * e : NULL;
    float* cmd = E->commands + 4 * e;
    float* act = E->actions + A * e;
    float* last_act = E->last_actions + A * e;
    float* last_qd = E->last_dof_vel + D * e;
    float* air = E->feet_air_time + T->num_feet * e;
    uint8_t* lastc = E->last_contacts + T->num_feet * e;
    int64_t* ep = E->episode_length + e;
    float* tau = E->torques + D * e;

    *ep += 1;                                                       /* :681 */
    float bl[3], ba[3], pg[3], rpy[3];
    const float g[3] = {0.f, 0.f, -1.f};
    quat_rotate_inverse(root + 3, root + 7, bl);                    /* :688 */
    quat_rotate_inverse(root + 3, root + 10, ba);                   /* :689 */
    quat_rotate_inverse(root + 3, g, pg);                           /* :690 */
    get_euler_xyz(root + 3, rpy);                                   /* :687 */
    float phase = 0.f, leg_phase[2] = {0.f, 0.f};
    if (T->obs_layout == LGS_OBS_HUMANOID) {                        /* h1_env.py:58-63 */
        float t = (float)(*ep) * T->control_dt;
        phase = fmodf(t, T->phase_period);
        if (phase != 0.f && phase < 0.f) phase += T->phase_period;
        phase = phase / T->phase_period;
        leg_phase[0] = phase;
        float pr = fmodf(phase + T->phase_offset, 1.0f);
        if (pr != 0.f && pr < 0.f) pr += 1.0f;
        leg_phase[1] = pr;
    }
    /* _post_physics_step_callback (:511-516) */
    if ((*ep) % T->resample_interval == 0) resample_commands(T, cmd, seed, (uint32_t)e, step, LGS_STREAM_CMD);
    if (T->heading_command) {
        const float fx[3] = {1.f, 0.f, 0.f};
        float fwd[3];
        quat_apply(root + 3, fx, fwd);
        float heading = lgs_atan2f(fwd[1], fwd[0]);
        cmd[2] = clipf(0.5f * wrap_to_pi(cmd[3] - heading), -1.f, 1.f);
    }
    /* check_termination (:711-721) */
    int reset = 0;
    for (int i = 0; i < T->num_termination; ++i) {
        const float* F = cf + 3 * T->termination_idx[i];
        if (sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) > 1.f) reset = 1;
    }
    if (fabsf(rpy[1]) > 1.0f || fabsf(rpy[0]) > 0.8f) reset = 1;
    int timeout = (float)(*ep) > T->max_episode_length;
    reset |= timeout;
    /* compute_reward (:770-787) */
    float q[LGS_MAX_DOFS], qd[LGS_MAX_DOFS];
    for (int j = 0; j < D; ++j) { q[j] = dofs[2 * j]; qd[j] = dofs[2 * j + 1]; }
    float rew = 0.f;
    for (int k = 0; k < T->num_rewards; ++k) {
        float r = reward_term(T->reward_ids[k], T, A, bl, ba, pg, root, q, qd, last_qd, act, last_act, tau, cf, cmd,
                              air, lastc, rbs, leg_phase, reset, timeout) * T->reward_scales[k];
        rew += r;
        E->episode_sums[(size_t)k * N + e] += r;
        if (E->rew_terms) E->rew_terms[(size_t)k * N + e] = r;
    }
    if (T->only_positive_rewards) rew = fmaxf(rew, 0.f);
    if (T->has_termination_reward) {
        float r = ((reset && !timeout) ? 1.f : 0.f) * T->termination_scale;
        rew += r;
        E->episode_sums[(size_t)T->num_rewards * N + e] += r;
    }
    E->rew[e] = rew;
    E->reset[e] = (uint8_t)reset;
    E->time_out[e] = (uint8_t)timeout;
    /* reset_idx (:723-768) */
    if (reset) reset_env(md, T, N, e, root, dofs, E, step_counter);
    /* _push_robots (:540-555): envs with ep_len % interval == 0, incl. just-reset ones */
    if (T->push_robots && (*ep) % T->push_interval == 0) {
        root[7] = rand_range(-T->max_push_vel_xy, T->max_push_vel_xy, orc_uniform(seed, e, step, LGS_STREAM_PUSH, 0));
        root[8] = rand_range(-T->max_push_vel_xy, T->max_push_vel_xy, orc_uniform(seed, e, step, LGS_STREAM_PUSH, 1));
    }
    /* compute_observations (:800-811 / h1_env.py:70-95); q/qd/actions/commands post-reset */
    float* ob = E->obs + (size_t)O * e;
    float* pr = P > 0 && E->priv_obs ? E->priv_obs + (size_t)P * e : NULL;
    float tmp[LGS_MAX_OBS];
    int k = 0;
    if (T->obs_layout == LGS_OBS_QUADRUPED) {
        for (int i = 0; i < 3; ++i) tmp[k++] = bl[i] * T->obs_scale_lin_vel;
    }
    for (int i = 0; i < 3; ++i) tmp[k++] = ba[i] * T->obs_scale_ang_vel;
    for (int i = 0; i < 3; ++i) tmp[k++] = pg[i];
    for (int i = 0; i < 3; ++i) tmp[k++] = cmd[i] * T->commands_scale[i];
    for (int j = 0; j < D; ++j) tmp[k++] = (dofs[2 * j] - T->default_dof_pos[j]) * T->obs_scale_dof_pos;
    for (int j = 0; j < D; ++j) tmp[k++] = dofs[2 * j + 1] * T->obs_scale_dof_vel;
    for (int j = 0; j < A; ++j) tmp[k++] = act[j];
    if (T->obs_layout == LGS_OBS_HUMANOID) {
        float ph = 2.0f * LGS_PI_F * phase;
        float sph, cph;
        lgs_sincosf(ph, &sph, &cph);
        tmp[k++] = sph;
        tmp[k++] = cph;
        if (pr) {
            for (int i = 0; i < 3; ++i) pr[i] = clipf(bl[i] * T->obs_scale_lin_vel, -T->clip_observations, T->clip_observations);
            for (int i = 0; i < k; ++i) pr[3 + i] = clipf(tmp[i], -T->clip_observations, T->clip_observations);
        }
    }
    for (int i = 0; i < O; ++i) {
        float x = tmp[i];
        if (T->add_noise) x += (2.f * orc_uniform(seed, e, step, LGS_STREAM_NOISE, i) - 1.f) * T->noise_vec[i];
        ob[i] = clipf(x, -T->clip_observations, T->clip_observations);
    }
    /* diagnostics buffers mirrored for the python attributes */
    for (int i = 0; i < 3; ++i) {
        E->base_lin_vel[3 * e + i] = bl[i];
        E->base_ang_vel[3 * e + i] = ba[i];
        E->projected_gravity[3 * e + i] = pg[i];
        E->rpy[3 * e + i] = rpy[i];
    }
    if (E->phase) E->phase[e] = phase;
    if (E->leg_phase) { E->leg_phase[2 * e] = leg_phase[0]; E->leg_phase[2 * e + 1] = leg_phase[1]; }
    /* bookkeeping (:707-709) */
    for (int j = 0; j < A; ++j) last_act[j] = act[j];
    for (int j = 0; j < D; ++j) last_qd[j] = dofs[2 * j + 1];
    for (int i = 0; i < 6; ++i) E->last_root_vel[6 * e + i] = root[7 + i];
}

/* _push_robots (:549-550) + bookkeeping (:709) across envs: when ANY env was pushed this
 * step, the reference writes root_states[:, 7:9] of every env (one draw per env; only the
 * pushed envs are sent to the simulation, :553-555) and last_root_vel then copies that
 * tensor.  The simulated state keeps the velocities of the envs not pushed; last_root_vel
 * takes the draws of all envs.  Pushed envs are those with ep_len % interval == 0 after the
 * step (the ones reset this step included). */
static void push_last_root_vel(const lgs_task_params* T, int N, const lgs_env_buffers* E, int64_t step_counter) {
    if (!T->push_robots) return;
    int any = 0;
    for (int e = 0; e < N && !any; ++e) any = (E->episode_length[e] % T->push_interval) == 0;
    if (!any) return;
    for (int e = 0; e < N; ++e)
        for (int j = 0; j < 2; ++j)
            E->last_root_vel[6 * e + j] = rand_range(-T->max_push_vel_xy, T->max_push_vel_xy,
                                                     orc_uniform(T->seed, e, (uint32_t)step_counter, LGS_STREAM_PUSH, j));
}

/* ====================================================== entry points === */

/* one substep for all envs (lgs_simulate) */
void orc_simulate(const lgs_model_desc* md, const lgs_sim_params* sp, int N, float* root, float* dofs,
                  const float* tau, float* cforce, float* rbs, const float* added_mass, const float* friction) {
    const int B = md->num_bodies, D = md->num_dofs;
#pragma omp parallel for schedule(static)
    for (int e = 0; e < N; ++e) {
        orc_substep_env(md, sp, root + 13 * e, dofs + 2 * D * e, tau + D * e, cforce + 3 * B * e,
                        added_mass ? added_mass[e] : 0.f, friction ? friction[e] : 1.f);
        if (rbs) orc_body_states_env(md, root + 13 * e, dofs + 2 * D * e, rbs + 13 * B * e);
    }
}

/* the step's rigid_body_states refresh: the bodies of T->body_state_mask (0: every body) */
static void step_body_states(const lgs_model_desc* md, const lgs_task_params* T, const float* root13,
                             const float* dofs, float* rbs) {
    float tmp[LGS_MAX_BODIES * 13];
    orc_body_states_env(md, root13, dofs, tmp);
    for (int b = 0; b < md->num_bodies; ++b)
        if (!T->body_state_mask || ((T->body_state_mask >> b) & 1u)) memcpy(rbs + 13 * b, tmp + 13 * b, 13 * sizeof(float));
}

/* the fused control step (LeggedRobot.step, legged_robot.py:615-647) for all envs */
void orc_step(const lgs_model_desc* md, const lgs_sim_params* sp, const lgs_task_params* T, int N, float* root,
              float* dofs, float* cforce, float* rbs, const float* added_mass, const float* friction,
              const lgs_env_buffers* E, int64_t step_counter) {
    const int B = md->num_bodies, D = md->num_dofs, A = T->num_actions;
#pragma omp parallel for schedule(static)
    for (int e = 0; e < N; ++e) {
        float* act = E->actions + A * e;
        for (int j = 0; j < A; ++j) act[j] = clipf(act[j], -T->clip_actions, T->clip_actions); /* :623-624 */
        for (int s = 0; s < T->decimation; ++s) {                      /* :627-639 */
            compute_torques(T, D, act, dofs + 2 * D * e, E->last_dof_vel + D * e, sp->dt, E->torques + D * e);
            orc_substep_env(md, sp, root + 13 * e, dofs + 2 * D * e, E->torques + D * e, cforce + 3 * B * e,
                            added_mass ? added_mass[e] : 0.f, friction ? friction[e] : 1.f);
        }
        if (rbs && T->write_body_states) step_body_states(md, T, root + 13 * e, dofs + 2 * D * e, rbs + 13 * B * e);
        ostate st = {root, dofs, cforce, T->write_body_states ? rbs : NULL};
        orc_post_physics_env(md, T, N, e, &st, E, step_counter);
    }
    push_last_root_vel(T, N, E, step_counter);
}

/* lgs_step_physics: clip + decimation x (PD + substep) + body states, no post-physics */
void orc_step_physics(const lgs_model_desc* md, const lgs_sim_params* sp, const lgs_task_params* T, int N,
                      float* root, float* dofs, float* cforce, float* rbs, const float* added_mass,
                      const float* friction, const lgs_env_buffers* E) {
    const int B = md->num_bodies, D = md->num_dofs, A = T->num_actions;
#pragma omp parallel for schedule(static)
    for (int e = 0; e < N; ++e) {
        float* act = E->actions + A * e;
        for (int j = 0; j < A; ++j) act[j] = clipf(act[j], -T->clip_actions, T->clip_actions);
        for (int s = 0; s < T->decimation; ++s) {
            compute_torques(T, D, act, dofs + 2 * D * e, E->last_dof_vel + D * e, sp->dt, E->torques + D * e);
            orc_substep_env(md, sp, root + 13 * e, dofs + 2 * D * e, E->torques + D * e, cforce + 3 * B * e,
                            added_mass ? added_mass[e] : 0.f, friction ? friction[e] : 1.f);
        }
        if (rbs && T->write_body_states) step_body_states(md, T, root + 13 * e, dofs + 2 * D * e, rbs + 13 * B * e);
    }
}

/* reset_idx(env_ids) for the envs with mask[e] != 0 (lgs_reset_idx, legged_robot.py:723-768) */
void orc_reset_idx(const lgs_model_desc* md, const lgs_task_params* T, int N, float* root, float* dofs,
                   const lgs_env_buffers* E, const uint8_t* mask, int64_t step_counter) {
    for (int e = 0; e < N; ++e)
        if (mask[e]) {
            reset_env(md, T, N, e, root + 13 * e, dofs + 2 * md->num_dofs * e, E, step_counter);
            E->reset[e] = 1;
        }
}

/* post-physics only (golden-vector tests): torques already in E->torques */
void orc_post_physics(const lgs_model_desc* md, const lgs_task_params* T, int N, float* root, float* dofs,
                      float* cforce, float* rbs, const lgs_env_buffers* E, int64_t step_counter) {
    for (int e = 0; e < N; ++e) {
        ostate st = {root, dofs, cforce, rbs};
        orc_post_physics_env(md, T, N, e, &st, E, step_counter);
    }
    push_last_root_vel(T, N, E, step_counter);
}

void orc_compute_torques(const lgs_task_params* T, int N, int D, const float* act, const float* dofs,
                         const float* last_qd, float sim_dt, float* tau) {
    for (int e = 0; e < N; ++e) compute_torques(T, D, act + D * e, dofs + 2 * D * e, last_qd + D * e, sim_dt, tau + D * e);
}

/* ABI self-description for the ctypes mirror test */
long orc_sizeof(int which) {
    switch (which) {
    case 0: return (long)sizeof(lgs_model_desc);
    case 1: return (long)sizeof(lgs_sim_params);
    case 2: return (long)sizeof(lgs_task_params);
    case 3: return (long)sizeof(lgs_env_buffers);
    case 4: return (long)sizeof(lgs_self_collision_desc);
    default: return -1;
    }
}

/* the shared deterministic transcendentals (lgs_detmath.h), for tests/test_detmath.py */
float orc_detmath(int which, float a, float b) {
    switch (which) {
    case 0: return lgs_sinf(a);
    case 1: return lgs_cosf(a);
    case 2: return lgs_expf(a);
    case 3: return lgs_atan2f(a, b);
    case 4: return lgs_asinf(a);
    default: return 0.f;
    }
}
