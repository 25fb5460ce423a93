"""PGS sweep-count study, measurement only: writes exp_sweeps.c, a copy of
oracle/lgs_oracle.c whose contact solve also
  * solves every substep's constraint problem with REF_SWEEPS (200) plain sweeps from zero (the
    converged reference), and records, after each sweep k = 1..KMAX of the solver under study,
    the error of its iterate against that reference (per-thread accumulators, exp_stats);
  * can run solver variants (exp_set): the shipped PGS (each contact's normal row, then its
    friction pair projected onto the cone), the same with the sweep direction alternating
    (symmetric Gauss-Seidel), and a per-contact 3x3 block step (the contact's three rows solved
    jointly with the inverse of their A block, then projected: normal clamped at 0, friction
    scaled back into the cone);
  * integrates with the iterate after `sp->solver_iterations` sweeps, so the trajectory is that
    of the chosen count (or, exp_set int_ref = 1, with the reference solution: every variant's
    error curve is then measured on the same states).
Build: python make_exp.py && gcc -O3 -march=native -ffp-contract=off -fPIC -fopenmp -std=gnu11
-shared -o libexp_sweeps.so exp_sweeps.c -lm   (study.py does both)."""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
s = open(os.path.join(ROOT, "oracle", "lgs_oracle.c")).read()
s = s.replace('"../include/leggedsim.h"', '"' + ROOT + '/include/leggedsim.h"')
s = s.replace('"../unitree-rl-gym_amd/csrc/lgs_detmath.h"', '"' + ROOT + '/unitree-rl-gym_amd/csrc/lgs_detmath.h"')

hdr = r'''
/* ---------------- sweep-count study hooks (tools/pgs_sweeps) ---------------- */
#include <omp.h>
#define EXP_KMAX 24
#define EXP_NM 12
#define EXP_THREADS 256
int g_variant = 0;      /* 8 / 9 group sweeps (g_group); 0 PGS, 1 symmetric PGS, 2 block 3x3, 3 block 3x3 symmetric, 4 PGS stopped at a
                           residual, 5 PGS over-relaxed (exp_omega), 7 normals pass then friction pass */
float g_tol = 1e-3f;    /* variant 4: stop after the sweep whose largest row residual |dlam_r| A_rr is <= g_tol (m/s) */
void exp_tol(float t) { g_tol = t; }
float g_omega = 1.0f;   /* variant 5: PGS with the normal (and limit) rows over-relaxed by omega */
void exp_omega(float w) { g_omega = w; }
static float g_maxres[EXP_THREADS];
int g_kmax = 16;        /* sweeps recorded (>= solver_iterations) */
int g_ref = 200;        /* reference sweeps (0: no reference, no statistics) */
int g_int_ref = 0;      /* 1: integrate with the reference solution (every variant sees the same states) */
static double g_acc[EXP_THREADS][EXP_KMAX + 1][EXP_NM];
void exp_set(int variant, int kmax, int ref, int int_ref) { g_variant = variant; g_kmax = kmax > EXP_KMAX ? EXP_KMAX : kmax; g_ref = ref; g_int_ref = int_ref; }
void exp_reset(void) { memset(g_acc, 0, sizeof(g_acc)); }
/* out[k][m] summed over threads; m: 0 solves, 1 rel impulse err normal, 2 rel impulse err friction,
   3 max |v - v*| (m/s), 4 P(max |v - v*| > 1 cm/s), 5 rel energy-norm err sqrt(dl^T A dl / l*^T A l*),
   6 rel total normal impulse err, 7 P(rel energy err > 5%), 8 max normal-velocity residual of the
   rows the reference loads (m/s), 9 solves with load, 10 sweeps used (k = 0: variant 4's stopped
   iterate), 11 solves that used every sweep allowed */
void exp_stats(double* out) {
    memset(out, 0, sizeof(double) * (EXP_KMAX + 1) * EXP_NM);
    for (int t = 0; t < EXP_THREADS; ++t)
        for (int k = 0; k <= EXP_KMAX; ++k)
            for (int m = 0; m < EXP_NM; ++m) out[k * EXP_NM + m] += g_acc[t][k][m];
}
static int g_group = 0;        /* variants 8 / 9: a body's ground contacts as one group per sweep: their normal
                                  rows (g_group inner passes: 8 solves the group's normal LCP, 9 is one pass,
                                  i.e. only the order changes), then their friction pairs */
static const int* g_cbp = NULL; static const int* g_cb2p = NULL; static int g_nc = 0;
#pragma omp threadprivate(g_group, g_cbp, g_cb2p, g_nc)
static void exp_sweep_group(int nr, const int* kind, const float* tgt, const float* inv, const float* cmu,
                            float A[][ROWMAX], float* lam, float* v) {
    int done[ROWMAX / 3 + 1];
    for (int c = 0; c < g_nc; ++c) done[c] = 0;
    for (int r = 0; r < nr; ++r) {
        if (kind[r] != 0) continue;
        if (r >= 3 * g_nc) {  /* a limit row */
            float ln = fmaxf(0.f, lam[r] + (tgt[r] - v[r]) * inv[r]);
            float d = ln - lam[r]; lam[r] = ln;
            for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][r], d, v[s2]);
            continue;
        }
        const int c = r / 3;
        if (done[c]) continue;
        int g[ROWMAX / 3 + 1], k = 0;
        if (g_cb2p[c] < 0) {
            for (int c2 = c; c2 < g_nc; ++c2) if (g_cb2p[c2] < 0 && g_cbp[c2] == g_cbp[c]) g[k++] = c2;
        } else g[k++] = c;
        for (int it = 0; it < (k > 1 ? g_group : 1); ++it)
            for (int i = 0; i < k; ++i) {
                const int rr = 3 * g[i];
                float ln = fmaxf(0.f, lam[rr] + (tgt[rr] - v[rr]) * inv[rr]);
                float d = ln - lam[rr]; lam[rr] = ln;
                for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][rr], d, v[s2]);
            }
        for (int i = 0; i < k; ++i) {
            const int rr = 3 * g[i] + 1;
            float lim = cmu[g[i]] * lam[rr - 1];
            float l1 = lam[rr] - v[rr] * inv[rr], l2 = lam[rr + 1] - v[rr + 1] * inv[rr + 1];
            float n2 = l1 * l1 + l2 * l2;
            if (n2 > lim * lim) { float nrm = sqrtf(n2); float sc = nrm > 0.f ? lim / nrm : 0.f; l1 *= sc; l2 *= sc; }
            float d1 = l1 - lam[rr], d2 = l2 - lam[rr + 1]; lam[rr] = l1; lam[rr + 1] = l2;
            for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][rr + 1], d2, fmaf(A[s2][rr], d1, v[s2]));
            done[g[i]] = 1;
        }
    }
}
static int g_split_pass = 0;  /* variant 7: a sweep visits every normal / limit row, then every friction pair */
#pragma omp threadprivate(g_split_pass)
static void exp_sweep(int nr, const int* kind, const float* tgt, const float* inv, const float* cmu,
                      float A[][ROWMAX], float* lam, float* v, int backward, int block, const float (*binv)[9]) {
    float mres = 0.f;
    if (g_group) { exp_sweep_group(nr, kind, tgt, inv, cmu, A, lam, v); return; }
    if (g_split_pass) {  /* every normal / limit row first, then every friction pair */
        for (int r = 0; r < nr; ++r) if (kind[r] == 0) {
            float ln = fmaxf(0.f, lam[r] + (tgt[r] - v[r]) * inv[r]);
            float d = ln - lam[r]; lam[r] = ln;
            for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][r], d, v[s2]);
        }
        for (int r = 0; r < nr; ++r) if (kind[r] == 1) {
            float lim = cmu[r / 3] * lam[r - 1];
            float l1 = lam[r] - v[r] * inv[r], l2 = lam[r + 1] - v[r + 1] * inv[r + 1];
            float n2 = l1 * l1 + l2 * l2;
            if (n2 > lim * lim) { float nrm = sqrtf(n2); float sc = nrm > 0.f ? lim / nrm : 0.f; l1 *= sc; l2 *= sc; }
            float d1 = l1 - lam[r], d2 = l2 - lam[r + 1]; lam[r] = l1; lam[r + 1] = l2;
            for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][r + 1], d2, fmaf(A[s2][r], d1, v[s2]));
        }
        return;
    }
    const int nc3 = nr; /* rows in order; contacts are row triples starting at kind 0 followed by 1, 2 */
    int r0 = backward ? nr - 1 : 0, dr = backward ? -1 : 1;
    for (int q = 0; q < nc3; ++q) {
        int r = r0 + dr * q;
        /* visit a contact at its head row (kind 0 followed by kind 1) */
        if (kind[r] == 2 || kind[r] == 1) continue;
        const int is_contact = (r + 2 < nr && kind[r + 1] == 1);
        if (!is_contact) { /* a limit row */
            float ln = fmaxf(0.f, lam[r] + (tgt[r] - v[r]) * inv[r]);
            float d = ln - lam[r]; lam[r] = ln;
            mres = fmaxf(mres, fabsf(d) * A[r][r]);
            for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][r], d, v[s2]);
            continue;
        }
        if (!block) {
            float ln = fmaxf(0.f, lam[r] + g_omega * (tgt[r] - v[r]) * inv[r]);
            float d = ln - lam[r]; lam[r] = ln;
            mres = fmaxf(mres, fabsf(d) * A[r][r]);
            for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][r], d, v[s2]);
            float lim = cmu[r / 3] * lam[r];
            float l1 = lam[r + 1] - v[r + 1] * inv[r + 1], l2 = lam[r + 2] - v[r + 2] * inv[r + 2];
            float n2 = l1 * l1 + l2 * l2;
            if (n2 > lim * lim) { float nrm = sqrtf(n2); float sc = nrm > 0.f ? lim / nrm : 0.f; l1 *= sc; l2 *= sc; }
            float d1 = l1 - lam[r + 1], d2 = l2 - lam[r + 2]; lam[r + 1] = l1; lam[r + 2] = l2;
            mres = fmaxf(mres, fmaxf(fabsf(d1) * A[r + 1][r + 1], fabsf(d2) * A[r + 2][r + 2]));
            for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][r + 2], d2, fmaf(A[s2][r + 1], d1, v[s2]));
        } else {
            const float* Bi = binv[r / 3];
            float e0 = tgt[r] - v[r], e1 = -v[r + 1], e2 = -v[r + 2];
            float ln = lam[r] + Bi[0] * e0 + Bi[1] * e1 + Bi[2] * e2;
            float l1 = lam[r + 1] + Bi[3] * e0 + Bi[4] * e1 + Bi[5] * e2;
            float l2 = lam[r + 2] + Bi[6] * e0 + Bi[7] * e1 + Bi[8] * e2;
            if (ln <= 0.f) {  /* separating: the contact carries nothing */
                ln = 0.f; l1 = 0.f; l2 = 0.f;
            } else {
                float lim = cmu[r / 3] * ln, n2 = l1 * l1 + l2 * l2;
                if (n2 > lim * lim) {  /* sliding: normal from its own row given the friction, then the cone */
                    float nrm = sqrtf(n2); float sc = nrm > 0.f ? lim / nrm : 0.f; l1 *= sc; l2 *= sc;
                }
            }
            float d0 = ln - lam[r], d1 = l1 - lam[r + 1], d2 = l2 - lam[r + 2];
            lam[r] = ln; lam[r + 1] = l1; lam[r + 2] = l2;
            for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][r + 2], d2, fmaf(A[s2][r + 1], d1, fmaf(A[s2][r], d0, v[s2])));
        }
    }
    g_maxres[omp_get_thread_num() % EXP_THREADS] = mres;
}
static void exp_inv3(const float* a, float* o) {
    double m[9]; for (int i = 0; i < 9; ++i) m[i] = a[i];
    double c0 = m[4] * m[8] - m[5] * m[7], c1 = m[5] * m[6] - m[3] * m[8], c2 = m[3] * m[7] - m[4] * m[6];
    double det = m[0] * c0 + m[1] * c1 + m[2] * c2; double id = 1.0 / (det + 1e-18);
    o[0] = c0 * id; o[1] = (m[2] * m[7] - m[1] * m[8]) * id; o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    o[3] = c1 * id; o[4] = (m[0] * m[8] - m[2] * m[6]) * id; o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    o[6] = c2 * id; o[7] = (m[1] * m[6] - m[0] * m[7]) * id; o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}
static void exp_record(int k, int nr, const int* kind, float A[][ROWMAX], const float* lam, const float* v,
                       const float* lr, const float* vr) {
    double* acc = g_acc[omp_get_thread_num() % EXP_THREADS][k];
    double en = 0, ln2 = 0, ef = 0, lf2 = 0, vmax = 0, tn = 0, tnr = 0, res = 0;
    float dl[ROWMAX];
    for (int r = 0; r < nr; ++r) {
        dl[r] = lam[r] - lr[r];
        double d = fabs((double)v[r] - vr[r]); if (d > vmax) vmax = d;
        if (kind[r] == 0) { en += (double)dl[r] * dl[r]; ln2 += (double)lr[r] * lr[r]; tn += lam[r]; tnr += lr[r];
                            if (lr[r] > 0.f) { double rr = fabs((double)v[r] - vr[r]); if (rr > res) res = rr; } }
        else { ef += (double)dl[r] * dl[r]; lf2 += (double)lr[r] * lr[r]; }
    }
    double ea = 0, la = 0;
    for (int r = 0; r < nr; ++r) for (int c = 0; c < nr; ++c) { ea += (double)dl[r] * A[r][c] * dl[c]; la += (double)lr[r] * A[r][c] * lr[c]; }
    acc[0] += 1;
    acc[3] += vmax; acc[4] += vmax > 0.01; acc[8] += res;
    if (ln2 > 1e-16) {
        acc[9] += 1;
        acc[1] += sqrt(en / ln2);
        acc[2] += lf2 > 1e-16 ? sqrt(ef / lf2) : 0.0;
        double rel = sqrt(fmax(ea, 0.0) / fmax(la, 1e-30));
        acc[5] += rel; acc[7] += rel > 0.05;
        acc[6] += tnr > 0 ? fabs(tn - tnr) / tnr : 0.0;
    }
}
'''
s = s.replace("void orc_substep_env(", hdr + "\nvoid orc_substep_env(", 1)

old_loop_head = '''    for (int it = 0; it < sp->solver_iterations; ++it) {
        for (int r = 0; r < nr; ++r) {'''
assert s.count(old_loop_head) == 1
i0 = s.index(old_loop_head)
i1 = s.index("    /* qd' = qf + L^-T (Y lambda) */", i0)
new_loop = '''    {
        float v0[ROWMAX], lr[ROWMAX], vr[ROWMAX], lkeep[ROWMAX];
        for (int r = 0; r < nr; ++r) { v0[r] = v[r]; lr[r] = 0.f; vr[r] = v[r]; }
        g_split_pass = 0; g_group = 0;
        g_cbp = cb; g_cb2p = cb2; g_nc = nc;
        if (g_ref > 0 && nr > 0)  /* the converged reference: plain PGS from zero */
            for (int it = 0; it < g_ref; ++it) exp_sweep(nr, kind, tgt, inv, cmu, A, lr, vr, 0, 0, NULL);
        float binv[ROWMAX / 3 + 1][9];
        const int block = g_variant == 2 || g_variant == 3, sym = g_variant == 1 || g_variant == 3;
        const int adaptive = g_variant == 4;
        g_split_pass = g_variant == 7;
        g_group = g_variant == 8 ? 30 : g_variant == 9 ? 1 : 0;
        int stopped = 0, used = 0;
        float lstop[ROWMAX], vstop[ROWMAX];
        if (block)
            for (int r = 0; r + 2 < nr; ++r)
                if (kind[r] == 0 && kind[r + 1] == 1) {
                    float a[9];
                    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) a[3 * i + j] = A[r + i][r + j];
                    a[0] += 1e-9f; a[4] += 1e-9f; a[8] += 1e-9f;
                    exp_inv3(a, binv[r / 3]);
                }
        const int K = g_kmax > sp->solver_iterations ? g_kmax : sp->solver_iterations;
        for (int r = 0; r < nr; ++r) lkeep[r] = 0.f;
        const float om_keep = g_omega;
        if (g_variant != 5) g_omega = 1.0f;
        for (int it = 0; it < K; ++it) {
            exp_sweep(nr, kind, tgt, inv, cmu, A, lam, v, sym && (it & 1), block, binv);
            if (g_ref > 0 && nr > 0 && it + 1 <= EXP_KMAX) exp_record(it + 1, nr, kind, A, lam, v, lr, vr);
            if (it + 1 == sp->solver_iterations) for (int r = 0; r < nr; ++r) lkeep[r] = lam[r];
            if (adaptive && !stopped && it < sp->solver_iterations) {
                used = it + 1;
                if (g_maxres[omp_get_thread_num() % EXP_THREADS] <= g_tol || used == sp->solver_iterations) {
                    stopped = 1;
                    for (int r = 0; r < nr; ++r) { lstop[r] = lam[r]; vstop[r] = v[r]; }
                }
            }
        }
        g_omega = om_keep;
        if (adaptive && nr > 0) {
            for (int r = 0; r < nr; ++r) lkeep[r] = lstop[r];
            if (g_ref > 0) {
                exp_record(0, nr, kind, A, lstop, vstop, lr, vr);
                double* acc = g_acc[omp_get_thread_num() % EXP_THREADS][0];
                acc[10] += used; acc[11] += used == sp->solver_iterations;
            }
        }
        for (int r = 0; r < nr; ++r) lam[r] = (g_int_ref && g_ref > 0) ? lr[r] : lkeep[r];
        (void)v0;
    }
'''
s = s[:i0] + new_loop + s[i1:]
open(os.path.join(HERE, "exp_sweeps.c"), "w").write(s)
