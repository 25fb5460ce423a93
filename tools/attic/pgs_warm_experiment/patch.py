"""PGS warm-start experiment (round 5, measured and dropped: DESIGN 3.1).  Writes exp.c: a copy
of oracle/lgs_oracle.c with per-env warm-start state keyed by contact point / self pair / limit
side, switchable sweep counts, SOR, a warm-start scale and a 200-sweep reference solve per
substep for the convergence error.  Build: gcc -O3 -march=native -ffp-contract=off -fPIC -fopenmp
-std=gnu11 -shared -o libexp.so exp.c -lm; then drive.py / ws2.py / kneel2.py."""
import os
import re
ROOT = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
HERE = os.path.dirname(os.path.abspath(__file__))
s = open(os.path.join(ROOT, "oracle", "lgs_oracle.c")).read().replace("\"../include/leggedsim.h\"", "\"" + ROOT + "/include/leggedsim.h\"").replace("\"../unitree-rl-gym_amd/csrc/lgs_detmath.h\"", "\"" + ROOT + "/unitree-rl-gym_amd/csrc/lgs_detmath.h\"")
s = s.replace('#include "leggedsim.h"', '#include "/root/repo/include/leggedsim.h"') if '#include "leggedsim.h"' in s else s
hdr = r'''
/* ---- PGS experiment hooks ---- */
float g_imp = 0.0f; void exp_imp(float f) { g_imp = f; }
float g_wfac = 1.0f; void exp_wfac(float f) { g_wfac = f; }
float g_omega = 1.0f; void exp_omega(float w) { g_omega = w; }
int g_sweeps_cold = 8, g_sweeps_warm = 8, g_warm = 0, g_ref_sweeps = 0;
#define WS_MAX 64
typedef struct { int n; int key[WS_MAX]; float lam[WS_MAX]; } wstate;
static wstate* g_ws = 0; static int g_ws_n = 0;
static __thread int g_cur_env = 0;
double g_err[8]; long g_err_n = 0; long g_sweep_total = 0; long g_solves = 0;
void exp_set(int cold, int warm_sweeps, int warm, int ref) { g_sweeps_cold = cold; g_sweeps_warm = warm_sweeps; g_warm = warm; g_ref_sweeps = ref; }
void exp_alloc(int n) { free(g_ws); g_ws = calloc(n, sizeof(wstate)); g_ws_n = n; }
void exp_clear_one(int e) { if (g_ws && e < g_ws_n) g_ws[e].n = 0; }
void exp_clear_ws(void) { for (int i = 0; i < g_ws_n; ++i) g_ws[i].n = 0; }
void exp_stats(double* out) { for (int i = 0; i < 8; ++i) out[i] = g_err[i]; out[6] = (double)g_err_n; out[7] = g_solves ? (double)g_sweep_total / g_solves : 0; }
void exp_reset_stats(void) { for (int i = 0; i < 8; ++i) g_err[i] = 0; g_err_n = 0; g_sweep_total = 0; g_solves = 0; }
'''
s = s.replace('void orc_substep_env(', hdr + '\nvoid orc_substep_env(', 1)
# keys per row
s = s.replace('int kind[ROWMAX]; /* 0 unilateral', 'int rkey[ROWMAX]; int kind[ROWMAX]; /* 0 unilateral')
s = s.replace('struct gcand { int b; float pc[3], sep, nrm[3]; }', 'struct gcand { int b, k; float pc[3], sep, nrm[3]; }')
s = s.replace('        g->b = b;\n        g->sep = sep;', '        g->b = b; g->k = k;\n        g->sep = sep;')
s = s.replace('        kind[nr] = 0; kind[nr + 1] = 1; kind[nr + 2] = 2;\n        cb[nc] = b;\n        cb2[nc] = -1;',
              '        kind[nr] = 0; kind[nr + 1] = 1; kind[nr + 2] = 2;\n        rkey[nr] = 3 * g->k; rkey[nr + 1] = 3 * g->k + 1; rkey[nr + 2] = 3 * g->k + 2;\n        cb[nc] = b;\n        cb2[nc] = -1;')
# self contacts: need pair index; store in sc arrays
s = s.replace('            sc_body[nsf][0] = g_self.body[q][0];', '            sc_q[nsf] = q;\n            sc_body[nsf][0] = g_self.body[q][0];')
s = s.replace('int nsf = 0, sc_body[ROWMAX / 3 + 1][2];', 'int nsf = 0, sc_body[ROWMAX / 3 + 1][2], sc_q[ROWMAX / 3 + 1];')
s = s.replace('        kind[nr] = 0; kind[nr + 1] = 1; kind[nr + 2] = 2;\n        cb[nc] = a;',
              '        kind[nr] = 0; kind[nr + 1] = 1; kind[nr + 2] = 2;\n        rkey[nr] = 100000 + 3 * sc_q[i]; rkey[nr + 1] = rkey[nr] + 1; rkey[nr + 2] = rkey[nr] + 2;\n        cb[nc] = a;')
s = s.replace('        tgt[nr] = gap >= 0.f ? -gap * idt : -beta * gap * idt;\n        kind[nr++] = 0;',
              '        tgt[nr] = gap >= 0.f ? -gap * idt : -beta * gap * idt;\n        rkey[nr] = 200000 + 2 * j + (qn < lo ? 0 : 1);\n        kind[nr++] = 0;')
# warm start + reference + sweeps
old = '''    for (int it = 0; it < sp->solver_iterations; ++it) {
        for (int r = 0; r < nr; ++r) {'''
new = '''    float v0[ROWMAX];
    for (int r = 0; r < nr; ++r) v0[r] = v[r];
    wstate* W = g_ws ? &g_ws[g_cur_env] : 0;
    int warmed = 0;
    if (g_warm && W && W->n > 0) {
        for (int r = 0; r < nr; ++r) {
            for (int t = 0; t < W->n; ++t) if (W->key[t] == rkey[r]) { lam[r] = g_wfac * W->lam[t]; warmed = 1; break; }
        }
        for (int r = 0; r < nr; ++r) if (lam[r] != 0.f) for (int s2 = 0; s2 < nr; ++s2) v[s2] = fmaf(A[s2][r], lam[r], v[s2]);
    }
    const int nsweeps = (g_warm && warmed) ? g_sweeps_warm : g_sweeps_cold;
    g_sweep_total += nsweeps; g_solves += 1;
    for (int it = 0; it < nsweeps; ++it) {
        for (int r = 0; r < nr; ++r) {'''
assert old in s
s = s.replace(old, new)
# after solving, store ws and compute reference
old = '''    /* qd' = qf + L^-T (Y lambda) */
    float z[NMAX];'''
new = '''    if (W) { W->n = nr < WS_MAX ? nr : WS_MAX; for (int r = 0; r < W->n; ++r) { W->key[r] = rkey[r]; W->lam[r] = lam[r]; }
      if (g_imp > 0.f) { const float thr = -g_imp * 9.81f * dt;
        for (int r = 0; r < W->n; ++r) { int h = r; if (kind[r] == 1) h = r - 1; else if (kind[r] == 2) h = r - 2; if (v0[h] < thr) W->lam[r] = 0.f; } } }
    if (g_ref_sweeps > 0 && nr > 0) {
        float lr[ROWMAX], vr[ROWMAX];
        for (int r = 0; r < nr; ++r) { lr[r] = 0.f; vr[r] = v0[r]; }
        for (int it = 0; it < g_ref_sweeps; ++it)
            for (int r = 0; r < nr; ++r) {
                if (kind[r] == 0) {
                    float ln = fmaxf(0.f, lr[r] + (tgt[r] - vr[r]) * inv[r]); float d = ln - lr[r]; lr[r] = ln;
                    for (int s2 = 0; s2 < nr; ++s2) vr[s2] = fmaf(A[s2][r], d, vr[s2]);
                } else if (kind[r] == 1) {
                    float lim = cmu[r / 3] * lr[r - 1];
                    float l1 = lr[r] - vr[r] * inv[r], l2 = lr[r + 1] - vr[r + 1] * inv[r + 1];
                    float n2 = l1 * l1 + l2 * l2;
                    if (n2 > lim * lim) { float nrm = sqrtf(n2); float sc = nrm > 0.f ? lim / nrm : 0.f; l1 *= sc; l2 *= sc; }
                    float d1 = l1 - lr[r], d2 = l2 - lr[r + 1]; lr[r] = l1; lr[r + 1] = l2;
                    for (int s2 = 0; s2 < nr; ++s2) vr[s2] = fmaf(A[s2][r + 1], d2, fmaf(A[s2][r], d1, vr[s2]));
                }
            }
        /* errors: constraint-space velocity (v - vr) and impulses */
        double ev = 0, el = 0, lmag = 0, vmax = 0;
        for (int r = 0; r < nr; ++r) { double d = v[r] - vr[r]; ev += d * d; if (fabs(d) > vmax) vmax = fabs(d); double e2 = lam[r] - lr[r]; el += e2 * e2; lmag += (double)lr[r] * lr[r]; }
        /* generalized velocity error: z difference through L^-T */
        float zd[NMAX];
        for (int i = 0; i < n; ++i) { float s3 = 0.f; for (int r = 0; r < nr; ++r) s3 = fmaf(Y[r][i], lam[r] - lr[r], s3); zd[i] = s3; }
        double ek = 0; for (int i = 0; i < n; ++i) ek += (double)zd[i] * zd[i];   /* = dq^T M dq (energy norm) */
        #pragma omp critical
        { g_err[0] += sqrt(ev / nr); g_err[1] += vmax; g_err[2] += sqrt(el); g_err[3] += sqrt(lmag); g_err[4] += sqrt(ek); g_err[5] += (vmax > 0.01); g_err_n += 1; }
    }
    /* qd' = qf + L^-T (Y lambda) */
    float z[NMAX];'''
assert old in s
s = s.replace(old, new)
# env id in orc_simulate
s = s.replace('''    for (int e = 0; e < N; ++e) {
        orc_substep_env(md, sp, root + 13 * e, dofs + 2 * D * e, tau + D * e, cforce + 3 * B * e,''', '''    for (int e = 0; e < N; ++e) {
        g_cur_env = e;
        orc_substep_env(md, sp, root + 13 * e, dofs + 2 * D * e, tau + D * e, cforce + 3 * B * e,''')
old_n = '''                float ln = fmaxf(0.f, lam[r] + (tgt[r] - v[r]) * inv[r]);
                float d = ln - lam[r];
                lam[r] = ln;'''
assert old_n in s
s = s.replace(old_n, '''                float ln = fmaxf(0.f, lam[r] + g_omega * (tgt[r] - v[r]) * inv[r]);
                float d = ln - lam[r];
                lam[r] = ln;''')
old_f = '''                float l1 = lam[r] - v[r] * inv[r];
                float l2 = lam[r + 1] - v[r + 1] * inv[r + 1];'''
assert old_f in s
s = s.replace(old_f, '''                float l1 = lam[r] - g_omega * v[r] * inv[r];
                float l2 = lam[r + 1] - g_omega * v[r + 1] * inv[r + 1];''')
open(os.path.join(HERE, "exp.c"), "w").write(s)
