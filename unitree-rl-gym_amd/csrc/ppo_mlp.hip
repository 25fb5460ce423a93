// ppo_mlp.hip — bf16 MFMA kernels for the actor-critic MLPs (include/ppo_mlp.h).
//
// Every GEMM of an MLP layer's forward and backward is written as
//     C[M,N] = A[M,K] . B[N,K]^T          (A, B bf16, k contiguous)
// by keeping each activation in BOTH layouts (row-major for the next layer's
// forward A operand, transposed for the weight gradient's B operand):
//     forward        y_l   = ELU(x_l W_l^T + b_l)       A = x_l,     B = W_l
//     input grad     dz_l-1 = (dz_l W_l) * ELU'(x_l)    A = dz_l,    B = W_l^T
//     weight grad    dW_l  = dz_l^T x_l                 A = dz_l^T,  B = x_l^T
// The weight gradient reduces over the 24,576-row mini-batch, so it is split
// over k into fp32 slabs (grid.z) and combined by pmlp_reduce_slabs: every
// output tile gets ~32-96 workgroups instead of one, and the sum order is fixed
// (deterministic; no atomics).
//
// Tiles: BMxBN per 64*WM*WN-thread block, BK = 64 staged through LDS (row
// stride 72 bf16 = 144 B keeps the 16-B fragment reads aligned), register
// prefetch of the next k-tile while the MFMAs of this one run.  Each wave owns
// a (BM/WM)x(BN/WN) sub-tile of 32x32 v_mfma_f32_32x32x16_bf16 accumulators
// (operand map: lane l holds row l&31, k = 8(l>>5)..+7; result: column l&31,
// rows (t&3)+8(t>>2)+4(l>>5), guide §3).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include <string>

#include "../../include/ppo_mlp.h"
#include "pmlp_noise.h"

typedef __bf16 bf16;
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) shortx4 lds_shortx4;
typedef float floatx16 __attribute__((ext_vector_type(16)));

static thread_local std::string g_err;
static int fail(int code, const std::string& m) {
    g_err = m;
    return code;
}
#define PMLP_CHECK_LAUNCH(what)                                                                       \
    do {                                                                                              \
        hipError_t _e = hipGetLastError();                                                            \
        if (_e != hipSuccess) return fail(-2, std::string(what) + ": " + hipGetErrorString(_e));      \
    } while (0)

// LDS stages of the GEMM main loop (2: one barrier per k-tile)
// diagnostic builds (never shipped): PMLP_DIAG_NOSTORE skips the GEMM's global result
// stores behind a condition the compiler cannot fold (the work is still done)
#ifdef PMLP_DIAG_NOSTORE
#define PMLP_STORE_OK (g.K < 0)
#else
#define PMLP_STORE_OK true
#endif

#ifndef PMLP_NBUF
#define PMLP_NBUF 1
#endif

struct GemmArgs {
    const bf16* A;
    const bf16* B;
    const float* bias;
    const bf16* yp;
    float* cf;
    bf16* cb;
    bf16* ct;
    int lda, ldb, ldyp, ldcf, ldcb, ldct;
    int M, N, K, ksplit;
    // MODE & 1: A = fp32 af[rows[m]][k] (k < kaf, else 0) converted on load; the blocks of
    // the first column tile also store the bf16 rows to xa (ld ldxa)
    const float* af;
    const int64_t* rows;
    bf16* xa;
    int ldaf, kaf, ldxa;
    int sumc;  // PARTIAL_TN: slab column of sum_k A (the bias gradient), 0 = none
};

#ifdef PMLP_EXACT_ELU
__device__ __forceinline__ float elu(float v) { return v > 0.f ? v : expm1f(v); }
#else
// exp(v) - 1 on v_exp_f32 (a few instructions instead of expm1f's ~20): the absolute
// error stays within a few ulp of 1.0, far below the bf16 rounding every ELU output gets
__device__ __forceinline__ float elu(float v) { return v > 0.f ? v : __expf(v) - 1.f; }
#endif

struct GemmBatch {
    GemmArgs j[PMLP_MAX_GEMM_JOBS];
    int slabs;  // PARTIAL: slabs per job (grid.z = njobs * slabs)
};

// ds_read_b64_tr_b16 (guide T10): per 16-lane group, lane 4q+p addresses row q,
// columns 4p..4p+3 of a 4 x 16 block; lane i receives column i, rows 0..3
__device__ __forceinline__ shortx4 lds_read_tr(const bf16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_shortx4*)p);
}

// MODE bit 0: A is fp32 rows gathered and converted on load (the first forward GEMM reads
// the observations itself: no conversion launch); bit 1: B is given [K][N] (n contiguous)
// and staged k-major like PARTIAL_TN's operands (the input gradient reads W[out][in]
// itself: no transposed weight copy).
//
// LDS-DMA (global_load_lds_dwordx4): one wave-instruction writes 64 x 16 B contiguously from
// a wave-uniform LDS base; the source address is per lane (guide §5 'Async global->LDS copy').
__device__ __forceinline__ void glds16(const void* src, bf16* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// ds_read_b64_tr_b16 in inline asm (the GL ring): hipcc waits vmcnt(0) before any LDS read
// it may alias with an LDS-DMA still in flight, which drains the ring every k-step; the
// ring orders its reads itself (counted vmcnt + barrier) and waits lgkmcnt by hand (gl_wait)
__device__ __forceinline__ shortx4 lds_read_tr_asm(const bf16* p) {
    shortx4 v;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a) : "memory");
    return v;
}

// k-major GL image: the 64-B chunk permutation of k-row r for R-wide rows
template <int R>
__device__ __forceinline__ int gl_swz(int r) { return R == 128 ? (r & 3) : ((r >> 1) & 1); }

// GL = 1: the k-loop stages both operands by LDS-DMA into two LDS buffers (no VGPR staging, no
// ds_write), one barrier per k-tile: the DMA of k-tile t+1 is issued right after the barrier
// that retires k-tile t and lands while tile t's MFMAs run.  The images are unpadded and
// XOR-swizzled on the SOURCE address (the DMA destination is lane-linear; guide rule 21):
//   rows form  [R][64] (k contiguous, 128-B rows): 16-B chunk c of row r at c ^ ((r >> 1) & 7)
//              -> conflict-free ds_read_b128 fragment reads;
//   k-major    [64][R] (R contiguous, 2R-B rows): 64-B chunk c of k-row r at c ^ swz(r)
//              (R = 128: r & 3; R = 64: (r >> 1) & 1) -> conflict-free ds_read_b64_tr_b16 reads.
// Needs whole 64-deep k-tiles (K, and the split-K slab, multiples of 64) and, for a k-major
// operand, R a multiple of the tile (rows-form tiles past M / N read a clamped row instead;
// those outputs are never stored).  Same MFMA order as GL = 0: bitwise the same results.
// LDS elements (bf16) of one k_gemm_nt tile: the staging buffers, or the epilogue tiles
template <int BM, int BN, int WM, int WN, int EPI, int NKS, int MODE, int GL>
__host__ __device__ constexpr int gemm_smem() {
    constexpr bool TNL = EPI == PMLP_EPI_PARTIAL_TN, PART = EPI == PMLP_EPI_PARTIAL || TNL;
    constexpr bool BKN = TNL || (MODE & 2) != 0;
    constexpr int BK = 64, LS = BK + 8;
    constexpr int SA = TNL ? BM + 32 : LS, SB = BKN ? BN + 32 : LS;
    constexpr int ATILE = TNL ? BK * SA : BM * LS, BTILE = BKN ? BK * SB : BN * LS;
    constexpr int GSTAGE = (BM + BN) * BK, GNS = GL == 2 ? 4 : 2;
    constexpr int STAGE = GL ? GNS * GSTAGE : (ATILE + BTILE) * PMLP_NBUF, CTILE = BM * (BN + 8), TTILE = BN * (BM + 8);
    return PART ? STAGE : (STAGE > CTILE ? (STAGE > TTILE ? STAGE : TTILE) : (CTILE > TTILE ? CTILE : TTILE));
}

// One output tile of the batched GEMM: block b of a gx x gy x gz grid (b linear), smem the
// gemm_smem<...>() bf16 elements of LDS.  k_gemm_nt runs it as a kernel of its own;
// k_gemm_pair runs two of them (a weight gradient beside an input gradient) in one grid.
template <int BM, int BN, int WM, int WN, int EPI, int NKS = 4, int MODE = 0, int GL = 0>
__device__ __forceinline__ void gemm_tile(const GemmBatch& gb, bf16* smem, int b, int gx, int gy, int gz) {
    // XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs (b % 8), each
    // with its own L2; give every XCD a contiguous range of logical tiles, ordered so that
    // the tiles sharing an operand panel are neighbours -- the n-tiles of one row block
    // (forward / input gradient: they share the A rows), the tiles of one split-K slab
    // (weight gradient: they share its rows of both operands) -- and read it from one L2.
    // (In a paired grid b is the block's index within its half: the halves' XCDs are
    // rotated by the offset, each XCD still owns one contiguous range.)
    int bx, by, bz;
    {
        const int nwg = gx * gy * gz;
        const int xcd = b % 8, q = nwg / 8, r = nwg % 8;
        const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
        if (EPI == PMLP_EPI_PARTIAL || EPI == PMLP_EPI_PARTIAL_TN) {
            bx = L % gx; by = (L / gx) % gy;
        } else {
            by = L % gy; bx = (L / gy) % gx;
        }
        bz = L / (gx * gy);
    }
    const int job = bz / gb.slabs, slice = bz % gb.slabs;
    const GemmArgs& g = gb.j[job];
    if (bx * BM >= g.M || by * BN >= g.N) return;  // grid covers the largest job
    // PARTIAL_TN: A[K,M] and B[K,N] (m / n contiguous: the row-major activations and
    // gradients), staged k-major in LDS and fed to the MFMAs by transposed reads
    constexpr bool TNL = EPI == PMLP_EPI_PARTIAL_TN;
    constexpr bool PART = EPI == PMLP_EPI_PARTIAL || TNL;
    // SW: the MFMAs take (B, A), so the accumulators hold C^T in the MFMA layout: a lane owns
    // ONE row m of C and 4 consecutive columns n per register quad -- 16-byte slab stores and
    // 8-byte LDS accesses in the epilogue instead of one per element (the same products, the
    // same k order)
    constexpr bool SW = PART || EPI == PMLP_EPI_BWD_DX;
    constexpr bool AF32 = (MODE & 1) != 0;
    constexpr bool BKN = TNL || (MODE & 2) != 0;  // B staged from [K][N]
    static_assert(!BKN || PMLP_NBUF == 1, "k-major B stages one k-tile");
    constexpr int BK = 64, LS = BK + 8;  // LDS row stride (bf16 elements, 144 B)
    constexpr int CPR = BK / 8;          // 16-byte chunks per staged row
    // TN images [BK][BM + 32]: a row stride of 16 (mod 64) dwords puts the four rows of
    // one transposed read on disjoint banks (conflict-free for BM, BN multiples of 64)
    constexpr int SA = TNL ? BM + 32 : LS, SB = BKN ? BN + 32 : LS;
    constexpr int ATILE = TNL ? BK * SA : BM * LS, BTILE = BKN ? BK * SB : BN * LS;
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 32, FN = TN / 32;
    constexpr int ACH = BM * BK / 8, BCH = BN * BK / 8;  // 16-byte chunks per tile
    constexpr int AL = (ACH + NT - 1) / NT, BL = (BCH + NT - 1) / NT;
    static_assert(FM >= 1 && FN >= 1, "wave tile must be a multiple of 32x32");
    constexpr int CS = BN + 8;  // row-major epilogue tile [BM][CS] (bf16)
    constexpr int TS = BM + 8;  // transposed epilogue tile [BN][TS]: 16-B aligned rows, 2-way b64 writes
    constexpr int GSTAGE = (BM + BN) * BK;  // GL: one unpadded k-tile of both operands (bf16)
    constexpr int GNS = GL == 2 ? 4 : 2;     // GL: LDS buffers (GL = 2: a ring, 2 k-tiles in flight)
    static_assert(GL != 2 || GNS == 4, "the ring's vmcnt counts assume 4 buffers");
    constexpr int STAGE = GL ? GNS * GSTAGE : (ATILE + BTILE) * PMLP_NBUF, CTILE = BM * CS, TTILE = BN * TS;
    static_assert(!GL || (!AF32 && PMLP_NBUF == 1 && NKS == 4), "GL: bf16 operands, whole k-tiles");
    static_assert(!GL || ((TNL ? BM : 64) % 64 == 0 && (BKN ? BN : 64) % 64 == 0), "GL k-major tiles: 64 or 128");
    constexpr int SMEM = PART ? STAGE
                              : (STAGE > CTILE ? (STAGE > TTILE ? STAGE : TTILE) : (CTILE > TTILE ? CTILE : TTILE));
    static_assert(SMEM == gemm_smem<BM, BN, WM, WN, EPI, NKS, MODE, GL>(), "gemm_smem out of step");
    bf16* As = smem;
    bf16* Bs = smem + ATILE;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int m0 = bx * BM, n0 = by * BN;
    int kb = 0, ke = g.K;
    if (PART) {
        kb = slice * g.ksplit;
        ke = min(g.K, kb + g.ksplit);
    }
    floatx16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int t = 0; t < 16; ++t) acc[i][j][t] = 0.f;
    // PARTIAL_TN bias gradient: the first column tile's wn == 0 waves also multiply their A
    // fragments by a column of ones (every output column = sum_k A[k][m])
    const bool dosum = TNL && g.sumc > 0 && by == 0 && wn == 0;  // wave-uniform
    floatx16 accs[TNL ? FM : 1];
#pragma unroll
    for (int i = 0; i < (TNL ? FM : 1); ++i)
#pragma unroll
        for (int t = 0; t < 16; ++t) accs[i][t] = 0.f;

    uint4 ra[1][AL], rb[1][BL];
    auto gload = [&](int p, int k0) {
#ifdef PMLP_DIAG_NOLOAD
        if (k0 != kb) return;  // diagnostic build: operands of the first k-tile only
#endif
        if constexpr (TNL) {
#pragma unroll
            for (int i = 0; i < AL; ++i) {
                const int c = tid + i * NT;
                const int r = c / (BM / 8), mc = (c % (BM / 8)) * 8;  // k row, m chunk
                const int gk = k0 + r, gm = m0 + mc;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (c < ACH && gk < ke && gm < g.M) v = *(const uint4*)(g.A + (size_t)gk * g.lda + gm);
                ra[p][i] = v;
            }
        } else if constexpr (AF32) {
#pragma unroll
            for (int i = 0; i < AL; ++i) {
                const int c = tid + i * NT;
                const int r = c / CPR, kc = (c % CPR) * 8;
                const int gr = m0 + r, gk = k0 + kc;
                bf16x8 t;
#pragma unroll
                for (int u = 0; u < 8; ++u) t[u] = (bf16)0.f;
                if (c < ACH && gr < g.M && gk < ke) {
                    const float* src = g.af + (size_t)(g.rows ? g.rows[gr] : (int64_t)gr) * g.ldaf + gk;
                    if (gk + 8 <= g.kaf) {
                        const float4 x0 = *(const float4*)src, x1 = *(const float4*)(src + 4);
                        t[0] = (bf16)x0.x; t[1] = (bf16)x0.y; t[2] = (bf16)x0.z; t[3] = (bf16)x0.w;
                        t[4] = (bf16)x1.x; t[5] = (bf16)x1.y; t[6] = (bf16)x1.z; t[7] = (bf16)x1.w;
                    } else {
#pragma unroll
                        for (int u = 0; u < 8; ++u) t[u] = gk + u < g.kaf ? (bf16)src[u] : (bf16)0.f;
                    }
                    if (g.xa && by == 0) *(bf16x8*)(g.xa + (size_t)gr * g.ldxa + gk) = t;
                }
                ra[p][i] = *(const uint4*)&t;
            }
        } else {
#pragma unroll
            for (int i = 0; i < AL; ++i) {
                const int c = tid + i * NT;
                const int r = c / CPR, kc = (c % CPR) * 8;
                const int gr = m0 + r, gk = k0 + kc;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (c < ACH && gr < g.M && gk < ke) v = *(const uint4*)(g.A + (size_t)gr * g.lda + gk);
                ra[p][i] = v;
            }
        }
        if constexpr (BKN) {
#pragma unroll
            for (int i = 0; i < BL; ++i) {
                const int c = tid + i * NT;
                const int r = c / (BN / 8), nc = (c % (BN / 8)) * 8;
                const int gk = k0 + r, gn = n0 + nc;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (c < BCH && gk < ke && gn < g.N) v = *(const uint4*)(g.B + (size_t)gk * g.ldb + gn);
                rb[p][i] = v;
            }
        } else {
#pragma unroll
            for (int i = 0; i < BL; ++i) {
                const int c = tid + i * NT;
                const int r = c / CPR, kc = (c % CPR) * 8;
                const int gr = n0 + r, gk = k0 + kc;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (c < BCH && gr < g.N && gk < ke) v = *(const uint4*)(g.B + (size_t)gr * g.ldb + gk);
                rb[p][i] = v;
            }
        }
    };
    auto lstore = [&](int p) {
        if constexpr (TNL) {
#pragma unroll
            for (int i = 0; i < AL; ++i) {
                const int c = tid + i * NT;
                if (c < ACH) *(uint4*)(As + (c / (BM / 8)) * SA + (c % (BM / 8)) * 8) = ra[p][i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < AL; ++i) {
                const int c = tid + i * NT;
                if (c < ACH) *(uint4*)(As + (c / CPR) * LS + (c % CPR) * 8) = ra[p][i];
            }
        }
        if constexpr (BKN) {
#pragma unroll
            for (int i = 0; i < BL; ++i) {
                const int c = tid + i * NT;
                if (c < BCH) *(uint4*)(Bs + (c / (BN / 8)) * SB + (c % (BN / 8)) * 8) = rb[p][i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < BL; ++i) {
                const int c = tid + i * NT;
                if (c < BCH) *(uint4*)(Bs + (c / CPR) * LS + (c % CPR) * 8) = rb[p][i];
            }
        }
    };

    // TN operand fragments: lane l (row/col 16*((l>>4)&1) + (l&15) of its 32-block,
    // k = 8(l>>5)..+7) = two transposed reads of k rows 8(l>>5) + {0..3, 4..7}
    const int tr_off = 8 * (lane >> 5) + ((lane >> 2) & 3);  // k row within a 16-step
    const int tr_col = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
    int gstage = 0;  // GL: the LDS buffer of the k-tile being computed
    auto kstep = [&](int s) {
        bf16x8 af[FM], bfr[FN];
        const int ko = s * 16 + (lane >> 5) * 8;
        if constexpr (GL) {
            const bf16* Ag = smem + gstage * GSTAGE;
            const bf16* Bg = Ag + BM * BK;
            const int kr = s * 16 + tr_off;  // k-major: this lane's first k row (the second is +4)
            auto trd = [](const bf16* p) { return GL == 2 ? lds_read_tr_asm(p) : lds_read_tr(p); };
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                if constexpr (TNL) {
                    const int ch = (wm * TM + i * 32) >> 5;
                    const bf16* p0 = Ag + kr * BM + ((ch ^ gl_swz<BM>(kr)) << 5) + tr_col;
                    const bf16* p1 = Ag + (kr + 4) * BM + ((ch ^ gl_swz<BM>(kr + 4)) << 5) + tr_col;
                    const shortx4 lo = trd(p0), hi = trd(p1);
                    af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
                } else {
                    const int r = wm * TM + i * 32 + (lane & 31), c = ko >> 3;
                    af[i] = *(const bf16x8*)(Ag + r * BK + ((c ^ ((r >> 1) & 7)) << 3));
                }
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                if constexpr (BKN) {
                    const int ch = (wn * TN + j * 32) >> 5;
                    const bf16* p0 = Bg + kr * BN + ((ch ^ gl_swz<BN>(kr)) << 5) + tr_col;
                    const bf16* p1 = Bg + (kr + 4) * BN + ((ch ^ gl_swz<BN>(kr + 4)) << 5) + tr_col;
                    const shortx4 lo = trd(p0), hi = trd(p1);
                    bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
                } else {
                    const int r = wn * TN + j * 32 + (lane & 31), c = ko >> 3;
                    bfr[j] = *(const bf16x8*)(Bg + r * BK + ((c ^ ((r >> 1) & 7)) << 3));
                }
            }
            if constexpr (GL == 2) {  // the asm reads' results: wait here, tied to the fragments
                static_assert(TNL && BKN && FM <= 2 && FN <= 2, "GL ring: k-major operands, <= 2x2 fragments");
                if constexpr (FM == 1 && FN == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[0]), "+v"(bfr[0]));
                else if constexpr (FM == 2 && FN == 1)
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[0]), "+v"(af[1]), "+v"(bfr[0]));
                else if constexpr (FM == 1 && FN == 2)
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[0]), "+v"(bfr[0]), "+v"(bfr[1]));
                else
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[0]), "+v"(af[1]), "+v"(bfr[0]), "+v"(bfr[1]));
            }
        } else if constexpr (TNL) {
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const bf16* p = As + (s * 16 + tr_off) * SA + wm * TM + i * 32 + tr_col;
                const shortx4 lo = lds_read_tr(p), hi = lds_read_tr(p + 4 * SA);
                af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
        } else {
#pragma unroll
            for (int i = 0; i < FM; ++i) af[i] = *(const bf16x8*)(As + (wm * TM + i * 32 + (lane & 31)) * LS + ko);
        }
        if constexpr (GL) {
            // (read above)
        } else if constexpr (BKN) {
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const bf16* p = Bs + (s * 16 + tr_off) * SB + wn * TN + j * 32 + tr_col;
                const shortx4 lo = lds_read_tr(p), hi = lds_read_tr(p + 4 * SB);
                bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
        } else {
#pragma unroll
            for (int j = 0; j < FN; ++j) bfr[j] = *(const bf16x8*)(Bs + (wn * TN + j * 32 + (lane & 31)) * LS + ko);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
                acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0)
                               : __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if constexpr (TNL) {
            if (dosum) {
                bf16x8 ones;
#pragma unroll
                for (int u = 0; u < 8; ++u) ones[u] = (bf16)1.f;
#pragma unroll
                for (int i = 0; i < FM; ++i) accs[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, af[i], accs[i], 0, 0, 0);
            }
        }
    };
    // NKS < 4: a single short k-tile (K <= 16 NKS: 48 for the first layer's forward, 16
    // for the last layer's input gradient), so the k-steps of zero operands are not issued
    auto compute = [&](int) {
#pragma unroll
        for (int s = 0; s < NKS; ++s) kstep(s);
    };

#if PMLP_NBUF == 2
    // two LDS stages: the next k-tile is stored into the other stage while this one
    // is consumed -> one barrier per k-tile
    gload(0, kb);
    lstore(0);
    __syncthreads();
    for (int k0 = kb; k0 < ke; k0 += BK) {
        const bool more = k0 + BK < ke;
        if (more) gload(0, k0 + BK);
        compute(k0);
        if (more) {
            As = (As == smem) ? smem + (BM + BN) * LS : smem;
            Bs = As + BM * LS;
            lstore(0);
        }
        __syncthreads();
    }
#else
    if constexpr (GL) {
        // DMA issue of one k-tile into LDS buffer st: operand X (rows R0.., ld) in the rows
        // form [R][64] or the k-major form [64][R]; NW waves share its wave-instructions
        auto gl_issue = [&](int st, int k0) {
            bf16* base = smem + st * GSTAGE;
            auto op = [&](const bf16* X, int ld, int r0, int nrows, auto kmaj_c, auto R_c, bf16* img) {
                constexpr bool kmaj = decltype(kmaj_c)::value;
                constexpr int R = decltype(R_c)::value;
                constexpr int ninst = R * BK * 2 / 1024, NW = WM * WN;  // 1 KiB per wave-instruction
#pragma unroll
                for (int qq = 0; qq < (ninst + NW - 1) / NW; ++qq) {  // (compile-time trip count)
                    const int q = wid + qq * NW;
                    if (ninst % NW != 0 && q >= ninst) break;
                    const int o = q * 1024 + 16 * lane;  // byte offset of this lane in the image
                    const bf16* src;
                    if constexpr (kmaj) {
                        const int rb = 2 * R, kr = o / rb, w = o % rb, c = (w >> 6) ^ (R == 128 ? (kr & 3) : ((kr >> 1) & 1));
                        src = X + (size_t)(k0 + kr) * ld + r0 + c * 32 + ((w & 63) >> 1);
                    } else {
                        const int r = o >> 7, c = ((o >> 4) & 7) ^ ((r >> 1) & 7);
                        src = X + (size_t)min(r0 + r, nrows - 1) * ld + k0 + c * 8;
                    }
                    glds16(src, img + __builtin_amdgcn_readfirstlane(q) * 512);
                }
            };
            op(g.A, g.lda, m0, g.M, std::integral_constant<bool, TNL>(), std::integral_constant<int, BM>(), base);
            op(g.B, g.ldb, n0, g.N, std::integral_constant<bool, BKN>(), std::integral_constant<int, BN>(),
               base + BM * BK);
        };
        if constexpr (GL == 1) {
            gl_issue(0, kb);
            int st = 0;
            for (int k0 = kb; k0 < ke; k0 += BK) {
                __syncthreads();  // (vmcnt(0)) this k-tile landed for every wave; the other buffer's reads are done
                if (k0 + BK < ke) gl_issue(st ^ 1, k0 + BK);
                gstage = st;
                compute(k0);
                st ^= 1;
            }
        } else {
            // GL = 2: a ring of GNS buffers, GNS - 2 k-tiles in flight behind the one computed.
            // Each wave counts its own DMAs (GW per k-tile): vmcnt(GW * newer tiles) retires this
            // k-tile's, the raw barrier (no vmcnt(0)) publishes it to every wave, and the
            // lgkmcnt(0) before it retires this wave's reads of the buffer refilled next.
            constexpr int GW = (BM + BN) * BK * 2 / 1024 / (WM * WN);
            static_assert((BM + BN) * BK * 2 / 1024 % (WM * WN) == 0, "GL ring: whole DMAs per wave");
            const int nt = (ke - kb) / BK;
            for (int p = 0; p < GNS - 1 && p < nt; ++p) gl_issue(p, kb + p * BK);
            for (int t = 0; t < nt; ++t) {
                const int newer = min(GNS - 2, nt - 1 - t);
                if (newer >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GW) : "memory");
                else if (newer == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GW) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (t + GNS - 1 < nt) gl_issue((t + GNS - 1) % GNS, kb + (t + GNS - 1) * BK);
                gstage = t % GNS;
                compute(0);
            }
        }
    } else {
        gload(0, kb);
        for (int k0 = kb; k0 < ke; k0 += BK) {
            __syncthreads();
            lstore(0);
            __syncthreads();
            if (k0 + BK < ke) gload(0, k0 + BK);
            compute(k0);
        }
    }
#endif

    // ---- epilogue: lane owns column (lane&31), rows (t&3)+8(t>>2)+4(lane>>5)
    if constexpr (TNL) {
        if (dosum && lane < 32) {  // (C^T layout: every register of a lane holds its row's sum)
            float* slab = g.cf + (size_t)slice * g.M * g.ldcf;
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int row = m0 + wm * TM + i * 32 + lane;
                if (row < g.M) slab[(size_t)row * g.ldcf + g.sumc] = accs[i][0];
            }
        }
    }
    constexpr int RCH = BM * BN / 8;  // 16-byte chunks of a bf16 output tile
    if (EPI == PMLP_EPI_BWD_DX) {
        // ELU' operand: the y tile [BM][BN] read coalesced (16-byte chunks along n),
        // issued before the LDS-reuse barrier, then staged in LDS for the accumulator
        // layout (per-element global loads in that layout cost 2x the kernel's time)
        constexpr int YL = (RCH + NT - 1) / NT;
        uint4 yr[YL];
        const bool yvec = (g.N % 8) == 0 && (g.ldyp % 8) == 0;  // (block-uniform: whole 16-B chunks)
#pragma unroll
        for (int u = 0; u < YL; ++u) {
            const int c = tid + u * NT;
            const int lr = c / (BN / 8), lc = (c % (BN / 8)) * 8;
            const int row = m0 + lr, col = n0 + lc;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (c < RCH && row < g.M && col < g.N) {
                if (yvec) {
                    v = *(const uint4*)(g.yp + (size_t)row * g.ldyp + col);
                } else {
                    bf16x8 t;
                    for (int e = 0; e < 8; ++e) t[e] = col + e < g.N ? g.yp[(size_t)row * g.ldyp + col + e] : (bf16)0.f;
                    v = *(const uint4*)&t;
                }
            }
            yr[u] = v;
        }
        __syncthreads();  // LDS reuse
#pragma unroll
        for (int u = 0; u < YL; ++u) {
            const int c = tid + u * NT;
            if (c < RCH) *(uint4*)(smem + (c / (BN / 8)) * CS + (c % (BN / 8)) * 8) = yr[u];
        }
        __syncthreads();
    }
    // the tile's 16-byte output chunks: row-major C (cb) and transposed C^T (ct), from the
    // bf16 tiles [BM][CS] / [BN][TS] in LDS
    auto cb_out = [&]() {
        for (int c = tid; c < RCH; c += NT) {
            const int lr = c / (BN / 8), lc = (c % (BN / 8)) * 8;
            const int row = m0 + lr, col = n0 + lc;
            if (row >= g.M || col >= g.N || !PMLP_STORE_OK) continue;
            const bf16* src = smem + lr * CS + lc;
            if (col + 8 <= g.N && (g.ldcb % 8) == 0) {
                *(uint4*)(g.cb + (size_t)row * g.ldcb + col) = *(const uint4*)src;
            } else {
                for (int u = 0; u < 8 && col + u < g.N; ++u) g.cb[(size_t)row * g.ldcb + col + u] = src[u];
            }
        }
    };
    auto ct_out = [&]() {
        for (int c = tid; c < RCH; c += NT) {
            const int lc = c / (BM / 8), lr = (c % (BM / 8)) * 8;
            const int col = n0 + lc, row = m0 + lr;
            if (col >= g.N || row >= g.M || !PMLP_STORE_OK) continue;
            const bf16* src = smem + lc * TS + lr;
            if (row + 8 <= g.M && (g.ldct % 8) == 0) {
                *(uint4*)(g.ct + (size_t)col * g.ldct + row) = *(const uint4*)src;
            } else {
                for (int u = 0; u < 8 && row + u < g.M; ++u) g.ct[(size_t)col * g.ldct + row + u] = src[u];
            }
        }
    };
    if constexpr (SW) {
        // C^T accumulators: lane -> tile row lr0 + 32 i, columns lc0 + 32 j + 8 q + (0..3) in
        // registers 4q..4q+3
        const int lr0 = wm * TM + (lane & 31), lc0 = wn * TN + 4 * (lane >> 5);
        if constexpr (PART) {
            float* slab = g.cf + (size_t)slice * g.M * g.ldcf;
            const bool vec = (g.ldcf & 3) == 0;
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int row = m0 + lr0 + i * 32;
                if (row >= g.M || !PMLP_STORE_OK) continue;
                float* dst = slab + (size_t)row * g.ldcf;
#pragma unroll
                for (int j = 0; j < FN; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int col = n0 + lc0 + j * 32 + 8 * q;
                        const float a[4] = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2],
                                            acc[i][j][4 * q + 3]};
                        if (vec && col + 4 <= g.N) {
                            *(float4*)(dst + col) = make_float4(a[0], a[1], a[2], a[3]);
                        } else {
                            for (int u = 0; u < 4; ++u)
                                if (col + u < g.N) dst[col + u] = a[u];
                        }
                    }
            }
        } else {  // BWD_DX: ELU' from the staged y tile, 4 columns per LDS read
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int lr = lr0 + i * 32, lc = lc0 + j * 32 + 8 * q;
                        const bf16x4 yv = *(const bf16x4*)(smem + lr * CS + lc);
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const float y = (float)yv[u], v = acc[i][j][4 * q + u];
                            acc[i][j][4 * q + u] = y > 0.f ? v : v * (y + 1.f);
                        }
                    }
            __syncthreads();  // y tile consumed before the LDS is rewritten
            if (g.cb) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int lr = lr0 + i * 32, lc = lc0 + j * 32 + 8 * q;
                            bf16x4 o;
#pragma unroll
                            for (int u = 0; u < 4; ++u) o[u] = (bf16)acc[i][j][4 * q + u];
                            *(bf16x4*)(smem + lr * CS + lc) = o;
                        }
                __syncthreads();
                cb_out();
                if (g.ct) __syncthreads();
            }
            if (g.ct) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
#pragma unroll
                        for (int q = 0; q < 4; ++q)
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                smem[(lc0 + j * 32 + 8 * q + u) * TS + lr0 + i * 32] = (bf16)acc[i][j][4 * q + u];
                __syncthreads();
                ct_out();
            }
        }
        return;
    }
    if (EPI == PMLP_EPI_FWD_HIDDEN) __syncthreads();  // LDS reuse
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 32 + (lane & 31);
            const int rbase = m0 + wm * TM + i * 32 + 4 * (lane >> 5);
            if (col >= g.N && EPI == PMLP_EPI_FWD_OUT) continue;
            if (EPI == PMLP_EPI_FWD_OUT) {
                const float b = g.bias ? g.bias[col] : 0.f;
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const int row = rbase + (t & 3) + 8 * (t >> 2);
                    if (row < g.M) g.cf[(size_t)row * g.ldcf + col] = acc[i][j][t] + b;
                }
            } else {
                // bias + ELU in place; stored below
                const float b = (g.bias && col < g.N) ? g.bias[col] : 0.f;
#pragma unroll
                for (int t = 0; t < 16; ++t) acc[i][j][t] = elu(acc[i][j][t] + b);
            }
        }
    }
    if (EPI == PMLP_EPI_FWD_HIDDEN) {
        if (g.cb) {
            // row-major: bf16 tile [BM][CS] in LDS, then 16-byte chunks along n
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int lc = wn * TN + j * 32 + (lane & 31);
#pragma unroll
                    for (int t = 0; t < 16; ++t) {
                        const int lr = wm * TM + i * 32 + 4 * (lane >> 5) + (t & 3) + 8 * (t >> 2);
                        smem[lr * CS + lc] = (bf16)acc[i][j][t];
                    }
                }
            __syncthreads();
            cb_out();
            if (g.ct) __syncthreads();  // the transposed tile reuses the LDS
        }
        if (g.ct) {
            // transposed: a lane's 4 consecutive accumulator rows are 4 consecutive m of
            // one column -> one 8-byte write into the [BN][TS] tile; then 16-byte chunks
            // along m (coalesced rows of C^T)
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int lc = wn * TN + j * 32 + (lane & 31);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int lr = wm * TM + i * 32 + 4 * (lane >> 5) + 8 * q;
                        bf16x4 v;
#pragma unroll
                        for (int u = 0; u < 4; ++u) v[u] = (bf16)acc[i][j][4 * q + u];
                        *(bf16x4*)(smem + lc * TS + lr) = v;
                    }
                }
            __syncthreads();
            ct_out();
        }
    }
}

template <int BM, int BN, int WM, int WN, int EPI, int NKS = 4, int MODE = 0, int GL = 0>
__global__ __launch_bounds__(64 * WM* WN) void k_gemm_nt(GemmBatch gb) {
    __shared__ __attribute__((aligned(16))) bf16 smem[gemm_smem<BM, BN, WM, WN, EPI, NKS, MODE, GL>()];
    gemm_tile<BM, BN, WM, WN, EPI, NKS, MODE, GL>(gb, smem, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                                                  gridDim.x, gridDim.y, gridDim.z);
}

// A k_gemm_nt instantiation as a type (k_gemm_pair's halves)
template <int BM_, int BN_, int WM_, int WN_, int EPI_, int NKS_ = 4, int MODE_ = 0, int GL_ = 0>
struct GemmCfg {
    static constexpr int BM = BM_, BN = BN_, NT = 64 * WM_ * WN_;
    static constexpr int SMEM = gemm_smem<BM_, BN_, WM_, WN_, EPI_, NKS_, MODE_, GL_>();
    __device__ static void run(const GemmBatch& gb, bf16* smem, int b, int gx, int gy, int gz) {
        gemm_tile<BM_, BN_, WM_, WN_, EPI_, NKS_, MODE_, GL_>(gb, smem, b, gx, gy, gz);
    }
};

// Two independent GEMM batches in ONE grid (1-D, block-uniform split): blocks [0, nA) run
// batch A's tiles on a dA grid, the rest batch B's on a dB grid.  The backward's weight
// gradient and input gradient of a layer both read only that layer's output gradient, so they
// share a launch: one kernel boundary fewer per layer, and the small weight-gradient grid runs
// beside the input gradient's instead of alone.  Each tile computes exactly what it computes
// in its own launch (bitwise the same results).
template <class CA, class CB>
__global__ __launch_bounds__(CA::NT) void k_gemm_pair(GemmBatch ga, GemmBatch gbb, int nA, int3 dA, int3 dB) {
    static_assert(CA::NT == CB::NT, "paired halves need one block size");
    __shared__ __attribute__((aligned(16))) bf16 smem[CA::SMEM > CB::SMEM ? CA::SMEM : CB::SMEM];
    const int b = blockIdx.x;
    if (b < nA) CA::run(ga, smem, b, dA.x, dA.y, dA.z);
    else CB::run(gbb, smem, b - nA, dB.x, dB.y, dB.z);
}

// Batched fp32 -> bf16 conversion, 64x64 tiles through LDS (blockIdx.z = job):
// x[M,K] (ld ldx) -> y[M,Kp] (ld Kp, columns K.. zero) and/or y^T[Kp,ldyt]
// (rows K.. and columns M.. zero).
struct CvtJob {
    const float* x;
    bf16* y;
    bf16* yt;
    const int64_t* rows;  // optional gather: row m of the output is row rows[m] of x
    int M, K, ldx, Kp, ldyt, one_col;
};
struct CvtJobs {
    CvtJob j[PMLP_MAX_JOBS];
    int start[PMLP_MAX_JOBS + 1];  // first block of each job (1-D grid, no idle blocks)
    int gm[PMLP_MAX_JOBS];         // 64-row tiles of each job
    int njobs;
};
__global__ __launch_bounds__(256) void k_convert_jobs(CvtJobs jobs) {
    int jb = 0;
    while (jb + 1 < jobs.njobs && (int)blockIdx.x >= jobs.start[jb + 1]) ++jb;
    const CvtJob J = jobs.j[jb];
    const int b = blockIdx.x - jobs.start[jb];
    const int m0 = (b % jobs.gm[jb]) * 64, k0 = (b / jobs.gm[jb]) * 64;
    __shared__ float tile[64][65];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    // every load of the tile is issued before any store (a store could alias the next
    // row's source as far as the compiler knows, which serialised 16 gather round trips)
    int64_t src[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int m = m0 + ty + 4 * u;
        src[u] = (m < J.M) ? (J.rows ? J.rows[m] : (int64_t)m) : -1;
    }
    float v[16];
    const int k = k0 + tx;
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = (src[u] >= 0 && k < J.K) ? J.x[(size_t)src[u] * J.ldx + k] : 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int r = ty + 4 * u, m = m0 + r;
        tile[r][tx] = v[u];
        if (J.y && m < J.M && k < J.Kp) J.y[(size_t)m * J.Kp + k] = (bf16)(k == J.one_col ? 1.f : v[u]);
    }
    if (!J.yt) return;
    __syncthreads();
    for (int c = ty; c < 64; c += 4) {
        const int k = k0 + c, m = m0 + tx;
        if (k < J.Kp && m < J.ldyt) J.yt[(size_t)k * J.ldyt + m] = (bf16)tile[tx][c];
    }
}

struct RedJob {
    const float* slab;
    float* out;
    float* bias_out;
    int64_t stride, n;
    int nslabs, cols_in, cols_out;
    int groups;  // slab groups per element quad (threads summing disjoint slab subsets)
};
struct RedJobs {
    RedJob j[PMLP_MAX_JOBS];
    int start[PMLP_MAX_JOBS + 1];  // first block of each job (1-D grid)
    int njobs;
};
// out = sum over slabs (fixed order per element: deterministic).  With bias_out: the slab
// is [rows, cols_in]; columns < cols_out go to out[rows, cols_out] and column cols_out
// (the ones-row product) to bias_out[rows].  Four consecutive elements per thread (16-byte
// loads), the slab loop unrolled so the loads of several slabs are in flight together.
// A job with many slabs (the small layers' weight gradients: 64-96 slabs) splits them over
// G = J.groups threads per element quad (slabs g, g+G, ...), summed through LDS in group
// order: its serial chain of dependent adds is G times shorter.
// RedStep (pmlp_reduce_slabs_step): one more workgroup finishes the PPO loss (the
// per-block partials of k_ppo_loss_step*: stats and the std gradient, what
// k_ppo_loss_step_final computed, same summation order), and with norm set every
// workgroup writes the sum of squares of the gradient elements it produced (the last one:
// of the std gradient) and the loss one does k_opt_prepare's step / loss / LR bookkeeping
// -- one launch instead of three (world size 1: nothing is all-reduced in between).
struct RedStep {
    const float* lpartial;  // null: no loss finish (plain pmlp_reduce_slabs)
    int lblocks, A, M;
    float ecoef;
    const float* stdv;
    float* stats;
    float* dstd;
    float* norm;  // null: no norm partials / bookkeeping
    float* step;
    float* lr;
    float* acc;
    float desired_kl;
    int adaptive;
};

__device__ __forceinline__ float red_block_sum(float v, float* sh) {  // 256 threads
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

__device__ void reduce_step_finish(const RedStep& r) {
    __shared__ float q_out[64];
    __shared__ float sh[4];
    const int W = 3 + r.A, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // one wave per quantity q (q = w, w + 4, ...): k_ppo_loss_step_final's order exactly
    for (int q = w; q < W; q += 4) {
        float x = 0.f;
#pragma unroll 8
        for (int b = lane; b < r.lblocks; b += 64) x += r.lpartial[(size_t)b * W + q];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        if (lane == 0) q_out[q] = x;
    }
    __syncthreads();
    float sq = 0.f;
    if (threadIdx.x < W) {
        const int q = threadIdx.x;
        const float x = q_out[q];
        if (q < 3) {
            r.stats[q] = x * (1.f / (float)r.M);
        } else {
            const float d = x - r.ecoef / r.stdv[q - 3];
            r.dstd[q - 3] = d;
            sq = d * d;
        }
    }
    if (threadIdx.x == 0) {
        float ent = 0.f;
        for (int k = 0; k < r.A; ++k) ent += 0.5f + 0.91893853320467274f + logf(r.stdv[k]);  // log(sqrt(2 pi))
        r.stats[3] = ent;
    }
    if (!r.norm) return;  // (block-uniform)
    sq = red_block_sum(sq, sh);
    if (threadIdx.x == 0) {
        r.norm[blockIdx.x] = sq;
        // k_opt_prepare's block-0 bookkeeping at scale 1 (the stats of this launch)
        r.step[0] += 1.f;
        const float s0 = q_out[0] * (1.f / (float)r.M), s1 = q_out[1] * (1.f / (float)r.M);
        if (r.acc) {
            r.acc[0] += s1;
            r.acc[1] += s0;
        }
        if (r.adaptive) {
            const float kl = q_out[2] * (1.f / (float)r.M);
            float l = r.lr[0];
            if (kl > r.desired_kl * 2.f) l = fmaxf(l / 1.5f, 1e-5f);
            else if (kl < r.desired_kl / 2.f && kl > 0.f) l = fminf(l * 1.5f, 1e-2f);
            r.lr[0] = l;
        }
    }
}

__global__ __launch_bounds__(256) void k_reduce_jobs(RedJobs jobs, RedStep rs) {
    __shared__ float4 red[256];
    __shared__ float sh[4];
    // the loss workgroup is the first one (dispatched first: its serial sums overlap the rest)
    if (rs.lpartial && blockIdx.x == 0) {
        reduce_step_finish(rs);
        return;
    }
    const int bx = (int)blockIdx.x - (rs.lpartial ? 1 : 0);
    int jb = 0;
    while (jb + 1 < jobs.njobs && bx >= jobs.start[jb + 1]) ++jb;
    const RedJob J = jobs.j[jb];
    const int G = J.groups, EQ = 256 / G;  // block-uniform
    const int sg = threadIdx.x / EQ, eq = threadIdx.x % EQ;
    const int64_t i0 = 4 * ((int64_t)(bx - jobs.start[jb]) * EQ + eq);
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    if (i0 < J.n) {
        if (i0 + 4 <= J.n && (J.stride % 4) == 0 && ((uintptr_t)J.slab & 15) == 0) {
            const float4* p = (const float4*)(J.slab + i0);
            const int64_t st = J.stride / 4;
#pragma unroll 8
            for (int k = sg; k < J.nslabs; k += G) {
                const float4 v = p[(size_t)k * st];
                s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
            }
        } else {
            for (int k = sg; k < J.nslabs; k += G)
                for (int e = 0; e < 4 && i0 + e < J.n; ++e) s[e] += J.slab[(size_t)k * J.stride + i0 + e];
        }
    }
    if (G > 1) {
        red[threadIdx.x] = make_float4(s[0], s[1], s[2], s[3]);
        __syncthreads();
        if (sg != 0 && !rs.norm) return;
        if (sg == 0)
            for (int g = 1; g < G; ++g) {
                const float4 v = red[g * EQ + eq];
                s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
            }
    }
    float sq = 0.f;
    if (i0 < J.n && sg == 0) {
        for (int e = 0; e < 4 && i0 + e < J.n; ++e) {
            const int64_t i = i0 + e;
            int64_t o = i;
            float* dst = J.out;
            if (J.bias_out) {
                const int64_t row = i / J.cols_in, col = i % J.cols_in;
                if (col < J.cols_out) {
                    o = row * J.cols_out + col;
                } else if (col == J.cols_out) {
                    dst = J.bias_out;
                    o = row;
                } else {
                    continue;
                }
            }
            dst[o] = s[e];
            sq = fmaf(s[e], s[e], sq);
        }
    }
    if (!rs.norm) return;  // (block-uniform)
    sq = red_block_sum(sq, sh);
    if (threadIdx.x == 0) rs.norm[blockIdx.x] = sq;
}

struct SumJob {
    const bf16* x;
    float* out;
    int rows, cols, ld;
};
struct SumJobs {
    SumJob j[PMLP_MAX_JOBS];
};
__global__ __launch_bounds__(256) void k_rowsum_jobs(SumJobs jobs) {
    __shared__ float part[4];
    const SumJob J = jobs.j[blockIdx.y];
    const int r = blockIdx.x, tid = threadIdx.x;
    if (r >= J.rows) return;
    const bf16* row = J.x + (size_t)r * J.ld;
    float s = 0.f;
    const int full = J.cols / 8;
    for (int c = tid; c < full; c += 256) {
        bf16x8 v = *(const bf16x8*)(row + 8 * c);
#pragma unroll
        for (int u = 0; u < 8; ++u) s += (float)v[u];
    }
    for (int u = 8 * full + tid; u < J.cols; u += 256) s += (float)row[u];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if ((tid & 63) == 0) part[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) J.out[r] = (part[0] + part[1]) + (part[2] + part[3]);
}


// ---------------------------------------------------------------- PPO loss --
// rsl_rl v1.0.2 PPO.update loss for a diagonal Gaussian policy, one row per
// thread, forward and backward fused (see ppo.py _minibatch_step for the torch
// statement it replaces).  Reductions: per-block partials, then one block sums
// them in a fixed order (deterministic).
#define PMLP_LOSS_THREADS 256
struct LossArgs {
    const float *mu, *stdv, *value, *actions, *old_logp, *old_mu, *old_sigma, *adv, *ret, *target;
    const int64_t* rows;  // optional: rollout inputs (actions .. target) are read at row rows[i]
    int M, A, clipped_value;
    float clip, vcoef, ecoef;
    __device__ size_t src(int i) const { return rows ? (size_t)rows[i] : (size_t)i; }
};

__device__ __forceinline__ float block_sum(float v, float* sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

__global__ __launch_bounds__(PMLP_LOSS_THREADS) void k_ppo_loss_fwd(LossArgs a, float* __restrict__ partial) {
    __shared__ float sh[4];
    const int i = blockIdx.x * PMLP_LOSS_THREADS + threadIdx.x;
    float surr = 0.f, vl = 0.f, kl = 0.f;
    if (i < a.M) {
        const size_t si = a.src(i);
        float logp = 0.f;
        for (int k = 0; k < a.A; ++k) {
            const float sg = a.stdv[k], mu = a.mu[(size_t)i * a.A + k];
            const float d = a.actions[si * a.A + k] - mu;
            logp += -(d * d) / (2.f * sg * sg) - logf(sg) - kHalfLog2Pi;
            const float os = a.old_sigma[si * a.A + k], om = a.old_mu[si * a.A + k] - mu;
            kl += logf(sg / os + 1.0e-5f) + (os * os + om * om) / (2.f * sg * sg) - 0.5f;
        }
        const float ratio = expf(logp - a.old_logp[si]);
        const float adv = a.adv[si];
        const float s1 = -adv * ratio, s2 = -adv * fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip);
        surr = fmaxf(s1, s2);
        const float v = a.value[i], r = a.ret[si];
        if (a.clipped_value) {
            const float t = a.target[si];
            const float vc = t + fminf(fmaxf(v - t, -a.clip), a.clip);
            vl = fmaxf((v - r) * (v - r), (vc - r) * (vc - r));
        } else {
            vl = (r - v) * (r - v);
        }
    }
    surr = block_sum(surr, sh);
    vl = block_sum(vl, sh);
    kl = block_sum(kl, sh);
    if (threadIdx.x == 0) {
        partial[blockIdx.x * 4 + 0] = surr;
        partial[blockIdx.x * 4 + 1] = vl;
        partial[blockIdx.x * 4 + 2] = kl;
    }
}

// loss[0]; stats = [surrogate_loss, value_loss, kl_mean, entropy_mean]
__global__ __launch_bounds__(PMLP_LOSS_THREADS) void k_ppo_loss_final(LossArgs a, const float* __restrict__ partial,
                                                                      int nblocks, float* __restrict__ loss,
                                                                      float* __restrict__ stats) {
    __shared__ float sh[4];
    float s[3] = {0.f, 0.f, 0.f};
    for (int b = threadIdx.x; b < nblocks; b += PMLP_LOSS_THREADS)
        for (int k = 0; k < 3; ++k) s[k] += partial[b * 4 + k];
    for (int k = 0; k < 3; ++k) s[k] = block_sum(s[k], sh);
    if (threadIdx.x == 0) {
        float ent = 0.f;
        for (int k = 0; k < a.A; ++k) ent += 0.5f + kHalfLog2Pi + logf(a.stdv[k]);
        const float inv = 1.f / (float)a.M;
        const float surr = s[0] * inv, vl = s[1] * inv;
        loss[0] = surr + a.vcoef * vl - a.ecoef * ent;
        stats[0] = surr;
        stats[1] = vl;
        stats[2] = s[2] * inv;
        stats[3] = ent;
    }
}

// torch.maximum backward: the larger input takes the gradient, ties split it
__device__ __forceinline__ void max_weights(float x, float y, float& wx, float& wy) {
    wx = x > y ? 1.f : (x == y ? 0.5f : 0.f);
    wy = y > x ? 1.f : (x == y ? 0.5f : 0.f);
}

__global__ __launch_bounds__(PMLP_LOSS_THREADS) void k_ppo_loss_bwd(LossArgs a, const float* __restrict__ gout,
                                                                    float* __restrict__ dmu, float* __restrict__ dvalue,
                                                                    float* __restrict__ partial_std) {
    __shared__ float sh[4];
    const int i = blockIdx.x * PMLP_LOSS_THREADS + threadIdx.x;
    const float g = gout[0];
    const float gs = g / (float)a.M, gv = g * a.vcoef / (float)a.M;
    float dlogp = 0.f;
    const size_t si = i < a.M ? a.src(i) : 0;
    if (i < a.M) {
        float logp = 0.f;
        for (int k = 0; k < a.A; ++k) {
            const float sg = a.stdv[k];
            const float d = a.actions[si * a.A + k] - a.mu[(size_t)i * a.A + k];
            logp += -(d * d) / (2.f * sg * sg) - logf(sg) - kHalfLog2Pi;
        }
        const float ratio = expf(logp - a.old_logp[si]);
        const float adv = a.adv[si];
        const float lo = 1.f - a.clip, hi = 1.f + a.clip;
        const float s1 = -adv * ratio, s2 = -adv * fminf(fmaxf(ratio, lo), hi);
        float w1, w2;
        max_weights(s1, s2, w1, w2);
        const float dclamp = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
        dlogp = gs * (-adv) * (w1 + w2 * dclamp) * ratio;
        for (int k = 0; k < a.A; ++k) {
            const float sg = a.stdv[k];
            const float d = a.actions[si * a.A + k] - a.mu[(size_t)i * a.A + k];
            dmu[(size_t)i * a.A + k] = dlogp * d / (sg * sg);
        }
        const float v = a.value[i], r = a.ret[si];
        float dv;
        if (a.clipped_value) {
            const float t = a.target[si];
            const float vc = t + fminf(fmaxf(v - t, -a.clip), a.clip);
            float u1, u2;
            max_weights((v - r) * (v - r), (vc - r) * (vc - r), u1, u2);
            const float dcv = (v - t >= -a.clip && v - t <= a.clip) ? 1.f : 0.f;
            dv = gv * (u1 * 2.f * (v - r) + u2 * 2.f * (vc - r) * dcv);
        } else {
            dv = gv * 2.f * (v - r);
        }
        dvalue[i] = dv;
    }
    // d logp / d sigma_k summed over the block's rows
    for (int k = 0; k < a.A; ++k) {
        float c = 0.f;
        if (i < a.M) {
            const float sg = a.stdv[k];
            const float d = a.actions[si * a.A + k] - a.mu[(size_t)i * a.A + k];
            c = dlogp * (d * d / (sg * sg * sg) - 1.f / sg);
        }
        c = block_sum(c, sh);
        if (threadIdx.x == 0) partial_std[(size_t)blockIdx.x * a.A + k] = c;
    }
}

__global__ __launch_bounds__(PMLP_LOSS_THREADS) void k_ppo_loss_std(LossArgs a, const float* __restrict__ gout,
                                                                    const float* __restrict__ partial_std, int nblocks,
                                                                    float* __restrict__ dstd) {
    __shared__ float sh[4];
    for (int k = 0; k < a.A; ++k) {
        float c = 0.f;
        for (int b = threadIdx.x; b < nblocks; b += PMLP_LOSS_THREADS) c += partial_std[(size_t)b * a.A + k];
        c = block_sum(c, sh);
        if (threadIdx.x == 0) dstd[k] = c - a.ecoef * gout[0] / a.stdv[k];  // + entropy term
    }
}

// Fused PPO loss forward + backward for the optimizer step (the gradient of the
// loss itself, gout = 1): one wave per 64 rows, writing the output gradients straight
// into the MLP backward's bf16 operands (row-major and transposed, padded columns
// zero) and per-wave partials of [surrogate, value loss, kl, d/dstd_k (k < A)].
struct LossStepOut {
    float* partial;
    bf16 *dmu_b, *dmu_t, *dv_b, *dv_t;
    int Ap, Vp;  // padded widths of the actor / critic output gradients (0: no bf16 output)
    float *dmu_f, *dv_f;  // optional fp32 output gradients [M, A] and [M] (the recurrent heads)
};
__global__ __launch_bounds__(64) void k_ppo_loss_step(LossArgs a, LossStepOut o) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    const int W = 3 + a.A;
    float surr = 0.f, vl = 0.f, kl = 0.f, dlogp = 0.f;
    const bool valid = i < a.M;
    const size_t si = valid ? a.src(i) : 0;
    if (valid) {
        float logp = 0.f;
        for (int k = 0; k < a.A; ++k) {
            const float sg = a.stdv[k], mu = a.mu[(size_t)i * a.A + k];
            const float d = a.actions[si * a.A + k] - mu;
            logp += -(d * d) / (2.f * sg * sg) - logf(sg) - kHalfLog2Pi;
            const float os = a.old_sigma[si * a.A + k], om = a.old_mu[si * a.A + k] - mu;
            kl += logf(sg / os + 1.0e-5f) + (os * os + om * om) / (2.f * sg * sg) - 0.5f;
        }
        const float ratio = expf(logp - a.old_logp[si]);
        const float adv = a.adv[si];
        const float lo = 1.f - a.clip, hi = 1.f + a.clip;
        const float s1 = -adv * ratio, s2 = -adv * fminf(fmaxf(ratio, lo), hi);
        surr = fmaxf(s1, s2);
        float w1, w2;
        max_weights(s1, s2, w1, w2);
        const float dclamp = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
        const float gs = 1.f / (float)a.M, gv = a.vcoef / (float)a.M;
        dlogp = gs * (-adv) * (w1 + w2 * dclamp) * ratio;
        for (int k = 0; k < o.Ap; ++k) {
            float g = 0.f;
            if (k < a.A) {
                const float sg = a.stdv[k];
                const float d = a.actions[si * a.A + k] - a.mu[(size_t)i * a.A + k];
                g = dlogp * d / (sg * sg);
            }
            o.dmu_b[(size_t)i * o.Ap + k] = (bf16)g;
            if (o.dmu_t) o.dmu_t[(size_t)k * a.M + i] = (bf16)g;
        }
        if (o.dmu_f)
            for (int k = 0; k < a.A; ++k) {
                const float sg = a.stdv[k];
                const float d = a.actions[si * a.A + k] - a.mu[(size_t)i * a.A + k];
                o.dmu_f[(size_t)i * a.A + k] = dlogp * d / (sg * sg);
            }
        const float v = a.value[i], r = a.ret[si];
        float dv;
        if (a.clipped_value) {
            const float t = a.target[si];
            const float vc = t + fminf(fmaxf(v - t, -a.clip), a.clip);
            vl = fmaxf((v - r) * (v - r), (vc - r) * (vc - r));
            float u1, u2;
            max_weights((v - r) * (v - r), (vc - r) * (vc - r), u1, u2);
            const float dcv = (v - t >= -a.clip && v - t <= a.clip) ? 1.f : 0.f;
            dv = gv * (u1 * 2.f * (v - r) + u2 * 2.f * (vc - r) * dcv);
        } else {
            vl = (r - v) * (r - v);
            dv = gv * 2.f * (v - r);
        }
        for (int k = 0; k < o.Vp; ++k) {
            o.dv_b[(size_t)i * o.Vp + k] = (bf16)(k == 0 ? dv : 0.f);
            if (o.dv_t) o.dv_t[(size_t)k * a.M + i] = (bf16)(k == 0 ? dv : 0.f);
        }
        if (o.dv_f) o.dv_f[i] = dv;
    }
    auto wsum = [](float x) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        return x;
    };
    surr = wsum(surr);
    vl = wsum(vl);
    kl = wsum(kl);
    if (threadIdx.x == 0) {
        o.partial[(size_t)blockIdx.x * W + 0] = surr;
        o.partial[(size_t)blockIdx.x * W + 1] = vl;
        o.partial[(size_t)blockIdx.x * W + 2] = kl;
    }
    for (int k = 0; k < a.A; ++k) {
        float c = 0.f;
        if (valid) {
            const float sg = a.stdv[k];
            const float d = a.actions[si * a.A + k] - a.mu[(size_t)i * a.A + k];
            c = dlogp * (d * d / (sg * sg * sg) - 1.f / sg);
        }
        c = wsum(c);
        if (threadIdx.x == 0) o.partial[(size_t)blockIdx.x * W + 3 + k] = c;
    }
}

// The same step with the row's A <= AM action entries held in registers (loaded once,
// gathered rows read as one contiguous record) and the per-action constants of sigma
// (1/(2s^2), 1/s^2, 1/s^3, 1/s, log s) computed once per block: the generic kernel above
// re-reads actions/mu in each of its three loops and takes 12 logf(sigma) per row.
template <int AM>
__global__ __launch_bounds__(64) void k_ppo_loss_step_reg(LossArgs a, LossStepOut o) {
    __shared__ float c_h[AM], c_i2[AM], c_i3[AM], c_i1[AM], c_lg[AM], c_sg[AM];
    const int A = a.A, W = 3 + A;
    if (threadIdx.x < A) {
        const float sg = a.stdv[threadIdx.x];
        c_sg[threadIdx.x] = sg;
        c_h[threadIdx.x] = 1.f / (2.f * sg * sg);
        c_i2[threadIdx.x] = 1.f / (sg * sg);
        c_i3[threadIdx.x] = 1.f / (sg * sg * sg);
        c_i1[threadIdx.x] = 1.f / sg;
        c_lg[threadIdx.x] = logf(sg);
    }
    __syncthreads();
    const int i = blockIdx.x * 64 + threadIdx.x;
    const bool valid = i < a.M;
    const size_t si = valid ? a.src(i) : 0;
    float d[AM];
    float surr = 0.f, vl = 0.f, kl = 0.f, dlogp = 0.f;
    if (valid) {
        // the row's records: 16-byte loads when A is a multiple of 4 (every record then
        // starts on 16 bytes), else one float per entry
        float rmu[AM], ract[AM], ros[AM], rom[AM];
        if ((A & 3) == 0) {
#pragma unroll
            for (int k = 0; k < AM; k += 4) {
                if (k < A) {
                    const float4 m4 = *(const float4*)(a.mu + (size_t)i * A + k);
                    const float4 a4 = *(const float4*)(a.actions + si * A + k);
                    const float4 s4 = *(const float4*)(a.old_sigma + si * A + k);
                    const float4 o4 = *(const float4*)(a.old_mu + si * A + k);
                    rmu[k] = m4.x; rmu[k + 1] = m4.y; rmu[k + 2] = m4.z; rmu[k + 3] = m4.w;
                    ract[k] = a4.x; ract[k + 1] = a4.y; ract[k + 2] = a4.z; ract[k + 3] = a4.w;
                    ros[k] = s4.x; ros[k + 1] = s4.y; ros[k + 2] = s4.z; ros[k + 3] = s4.w;
                    rom[k] = o4.x; rom[k + 1] = o4.y; rom[k + 2] = o4.z; rom[k + 3] = o4.w;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < AM; ++k)
                if (k < A) {
                    rmu[k] = a.mu[(size_t)i * A + k];
                    ract[k] = a.actions[si * A + k];
                    ros[k] = a.old_sigma[si * A + k];
                    rom[k] = a.old_mu[si * A + k];
                }
        }
        float logp = 0.f;
#pragma unroll
        for (int k = 0; k < AM; ++k) {
            if (k < A) {
                const float mu = rmu[k];
                d[k] = ract[k] - mu;
                logp += -(d[k] * d[k]) * c_h[k] - c_lg[k] - kHalfLog2Pi;
                const float os = ros[k], om = rom[k] - mu;
                kl += logf(c_sg[k] / os + 1.0e-5f) + (os * os + om * om) * c_h[k] - 0.5f;
            } else {
                d[k] = 0.f;
            }
        }
        const float ratio = expf(logp - a.old_logp[si]);
        const float adv = a.adv[si];
        const float lo = 1.f - a.clip, hi = 1.f + a.clip;
        const float s1 = -adv * ratio, s2 = -adv * fminf(fmaxf(ratio, lo), hi);
        surr = fmaxf(s1, s2);
        float w1, w2;
        max_weights(s1, s2, w1, w2);
        const float dclamp = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
        dlogp = (1.f / (float)a.M) * (-adv) * (w1 + w2 * dclamp) * ratio;
        for (int k = 0; k < o.Ap; k += 8) {  // 16-byte chunks of the padded dmu row
            bf16x8 g;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                float gv = 0.f;
#pragma unroll
                for (int kk = 0; kk < AM; ++kk)
                    if (kk == k + u && kk < A) gv = dlogp * d[kk] * c_i2[kk];
                g[u] = (bf16)gv;
                if (o.dmu_t) o.dmu_t[(size_t)(k + u) * a.M + i] = (bf16)gv;
            }
            *(bf16x8*)(o.dmu_b + (size_t)i * o.Ap + k) = g;
        }
        if (o.dmu_f) {
#pragma unroll
            for (int kk = 0; kk < AM; ++kk)
                if (kk < A) o.dmu_f[(size_t)i * A + kk] = dlogp * d[kk] * c_i2[kk];
        }
        const float v = a.value[i], r = a.ret[si];
        float dv;
        const float gvc = a.vcoef / (float)a.M;
        if (a.clipped_value) {
            const float t = a.target[si];
            const float vc = t + fminf(fmaxf(v - t, -a.clip), a.clip);
            vl = fmaxf((v - r) * (v - r), (vc - r) * (vc - r));
            float u1, u2;
            max_weights((v - r) * (v - r), (vc - r) * (vc - r), u1, u2);
            const float dcv = (v - t >= -a.clip && v - t <= a.clip) ? 1.f : 0.f;
            dv = gvc * (u1 * 2.f * (v - r) + u2 * 2.f * (vc - r) * dcv);
        } else {
            vl = (r - v) * (r - v);
            dv = gvc * 2.f * (v - r);
        }
        for (int k = 0; k < o.Vp; ++k) {
            o.dv_b[(size_t)i * o.Vp + k] = (bf16)(k == 0 ? dv : 0.f);
            if (o.dv_t) o.dv_t[(size_t)k * a.M + i] = (bf16)(k == 0 ? dv : 0.f);
        }
        if (o.dv_f) o.dv_f[i] = dv;
    } else {
#pragma unroll
        for (int k = 0; k < AM; ++k) d[k] = 0.f;
    }
    auto wsum = [](float x) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        return x;
    };
    surr = wsum(surr);
    vl = wsum(vl);
    kl = wsum(kl);
    if (threadIdx.x == 0) {
        o.partial[(size_t)blockIdx.x * W + 0] = surr;
        o.partial[(size_t)blockIdx.x * W + 1] = vl;
        o.partial[(size_t)blockIdx.x * W + 2] = kl;
    }
#pragma unroll
    for (int k = 0; k < AM; ++k) {
        if (k < A) {
            float c = valid ? dlogp * (d[k] * d[k] * c_i3[k] - c_i1[k]) : 0.f;
            c = wsum(c);
            if (threadIdx.x == 0) o.partial[(size_t)blockIdx.x * W + 3 + k] = c;
        }
    }
}

// The same step with four lanes per row (lane q of a quad owns action entries 4q..4q+3: one
// 16-byte load per record instead of A/4 serial ones) in 256-thread blocks of 64 rows, so
// the 24,576-row mini-batch is 1,536 waves instead of 384 and each lane has a quarter of
// the gathers in flight.  Quad sums combine a row's logp / KL; the block's partials are
// summed per wave (rows in xor order), then over the 4 waves in order (deterministic; the
// same partials layout as k_ppo_loss_step_reg: one record of 3 + A per 64 rows).
// Needs A % 4 == 0, A <= 16, Ap <= 16 and Ap % 4 == 0.
// The quad-lane loss on rows i0 .. i0 + 16 NWV - 1: four lanes per row (each owning 4 actions),
// 16 rows per wave, NWV waves (threads past 64 NWV join the barriers only); the per-wave sums
// are added in a fixed order into partial row `part`.  sh: LDS scratch of >= 96 + 19 NWV floats.
// k_ppo_loss_step_q (NWV = 4, 64 rows per workgroup) and the update forward's epilogue
// (k_mlp_fwd<96, .., LOSS>: NWV = 6, the workgroup's 96 rows) run it.
template <int NWV>
__device__ __forceinline__ void loss_quad_rows(const LossArgs& a, const LossStepOut& o, int i0, int part, float* sh) {
    float* const c_h = sh;
    float* const c_i2 = sh + 16;
    float* const c_i3 = sh + 32;
    float* const c_i1 = sh + 48;
    float* const c_lg = sh + 64;
    float* const c_sg = sh + 80;
    float(*const wpart)[3 + 16] = (float(*)[3 + 16])(sh + 96);
    const int A = a.A, W = 3 + A, tid = threadIdx.x, q = tid & 3, k0 = 4 * q;
    if (tid < A) {
        const float sg = a.stdv[tid];
        c_sg[tid] = sg;
        c_h[tid] = 1.f / (2.f * sg * sg);
        c_i2[tid] = 1.f / (sg * sg);
        c_i3[tid] = 1.f / (sg * sg * sg);
        c_i1[tid] = 1.f / sg;
        c_lg[tid] = logf(sg);
    }
    __syncthreads();
    const int i = i0 + (tid >> 2);
    const bool valid = tid < 64 * NWV && i < a.M;
    const bool own = k0 < A;  // quad-uniform per lane, same for every row
    const size_t si = valid ? a.src(i) : 0;
    float d[4] = {0.f, 0.f, 0.f, 0.f};
    float surr = 0.f, vl = 0.f, kl = 0.f, dlogp = 0.f;
    if (valid) {
        float lp = 0.f, kp = 0.f;
        if (own) {
            const float4 m4 = *(const float4*)(a.mu + (size_t)i * A + k0);
            const float4 a4 = *(const float4*)(a.actions + si * A + k0);
            const float4 s4 = *(const float4*)(a.old_sigma + si * A + k0);
            const float4 o4 = *(const float4*)(a.old_mu + si * A + k0);
            const float rmu[4] = {m4.x, m4.y, m4.z, m4.w}, ract[4] = {a4.x, a4.y, a4.z, a4.w};
            const float ros[4] = {s4.x, s4.y, s4.z, s4.w}, rom[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + u;
                d[u] = ract[u] - rmu[u];
                lp += -(d[u] * d[u]) * c_h[k] - c_lg[k] - kHalfLog2Pi;
                const float os = ros[u], om = rom[u] - rmu[u];
                kp += logf(c_sg[k] / os + 1.0e-5f) + (os * os + om * om) * c_h[k] - 0.5f;
            }
        }
        lp += __shfl_xor(lp, 1);
        lp += __shfl_xor(lp, 2);
        kp += __shfl_xor(kp, 1);
        kp += __shfl_xor(kp, 2);
        const float ratio = expf(lp - a.old_logp[si]);
        const float adv = a.adv[si];
        const float lo = 1.f - a.clip, hi = 1.f + a.clip;
        const float s1 = -adv * ratio, s2 = -adv * fminf(fmaxf(ratio, lo), hi);
        float w1, w2;
        max_weights(s1, s2, w1, w2);
        const float dclamp = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
        dlogp = (1.f / (float)a.M) * (-adv) * (w1 + w2 * dclamp) * ratio;
        if (k0 < o.Ap) {
            bf16x4 g;
#pragma unroll
            for (int u = 0; u < 4; ++u) g[u] = (bf16)(own ? dlogp * d[u] * c_i2[k0 + u] : 0.f);
            *(bf16x4*)(o.dmu_b + (size_t)i * o.Ap + k0) = g;
            if (o.dmu_t) {
#pragma unroll
                for (int u = 0; u < 4; ++u) o.dmu_t[(size_t)(k0 + u) * a.M + i] = g[u];
            }
        }
        const float v = a.value[i], r = a.ret[si];
        float dv;
        const float gvc = a.vcoef / (float)a.M;
        float vq;
        if (a.clipped_value) {
            const float t = a.target[si];
            const float vc = t + fminf(fmaxf(v - t, -a.clip), a.clip);
            vq = fmaxf((v - r) * (v - r), (vc - r) * (vc - r));
            float u1, u2;
            max_weights((v - r) * (v - r), (vc - r) * (vc - r), u1, u2);
            const float dcv = (v - t >= -a.clip && v - t <= a.clip) ? 1.f : 0.f;
            dv = gvc * (u1 * 2.f * (v - r) + u2 * 2.f * (vc - r) * dcv);
        } else {
            vq = (r - v) * (r - v);
            dv = gvc * 2.f * (v - r);
        }
        for (int k = q; k < o.Vp; k += 4) {
            o.dv_b[(size_t)i * o.Vp + k] = (bf16)(k == 0 ? dv : 0.f);
            if (o.dv_t) o.dv_t[(size_t)k * a.M + i] = (bf16)(k == 0 ? dv : 0.f);
        }
        if (o.dv_f && q == 0) o.dv_f[i] = dv;
        if (o.dmu_f && own) {
#pragma unroll
            for (int u = 0; u < 4; ++u) o.dmu_f[(size_t)i * A + k0 + u] = dlogp * d[u] * c_i2[k0 + u];
        }
        if (q == 0) {  // the row's scalars counted once
            surr = fmaxf(s1, s2);
            vl = vq;
            kl = kp;
        }
    }
    // per wave: sums over its 16 rows (xor 4..32 keeps the quad position), then the
    // scalars (nonzero on q == 0 only) over the quad
    auto rsum = [](float x) {
#pragma unroll
        for (int off = 4; off < 64; off <<= 1) x += __shfl_xor(x, off);
        return x;
    };
    surr = rsum(surr);
    vl = rsum(vl);
    kl = rsum(kl);
    float c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int k = k0 + u;
        c[u] = rsum(valid && own ? dlogp * (d[u] * d[u] * c_i3[k] - c_i1[k]) : 0.f);
    }
    const int w = tid >> 6, lane = tid & 63;
    if (lane == 0 && w < NWV) {
        wpart[w][0] = surr;
        wpart[w][1] = vl;
        wpart[w][2] = kl;
    }
    if (lane < 4 && own && w < NWV) {
#pragma unroll
        for (int u = 0; u < 4; ++u) wpart[w][3 + k0 + u] = c[u];
    }
    __syncthreads();
    if (tid < W) {
        float x = (wpart[0][tid] + wpart[1][tid]) + (wpart[2][tid] + wpart[3][tid]);
#pragma unroll
        for (int v = 4; v < NWV; v += 2) x += wpart[v][tid] + wpart[v + 1][tid];
        o.partial[(size_t)part * W + tid] = x;
    }
}

__global__ __launch_bounds__(256) void k_ppo_loss_step_q(LossArgs a, LossStepOut o) {
    __shared__ float sh[96 + 4 * 19];
    loss_quad_rows<4>(a, o, blockIdx.x * 64, blockIdx.x, sh);
}

// stats = [surrogate_loss, value_loss, kl_mean, entropy_mean]; dstd[k] incl. the entropy term.
// One wave per reduced quantity q (block q): the per-wave partials of k_ppo_loss_step summed
// in a fixed order (deterministic), all quantities at once.
__global__ __launch_bounds__(64) void k_ppo_loss_step_final(LossArgs a, const float* __restrict__ partial,
                                                            int nblocks, float* __restrict__ stats,
                                                            float* __restrict__ dstd) {
    const int W = 3 + a.A, q = blockIdx.x;
    float x = 0.f;
#pragma unroll 8
    for (int b = threadIdx.x; b < nblocks; b += 64) x += partial[(size_t)b * W + q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    if (threadIdx.x == 0) {
        if (q < 3) stats[q] = x * (1.f / (float)a.M);
        else dstd[q - 3] = x - a.ecoef / a.stdv[q - 3];
        if (q == 0) {
            float ent = 0.f;
            for (int k = 0; k < a.A; ++k) ent += 0.5f + kHalfLog2Pi + logf(a.stdv[k]);
            stats[3] = ent;
        }
    }
}

// ------------------------------------------------------------ optimizer --
// One PPO optimizer step over the FLAT parameter/gradient buffers (every
// actor/critic parameter is a view of one fp32 buffer): clip_grad_norm_ +
// torch.optim.Adam (amsgrad off, no weight decay) in two launches.
#define PMLP_OPT_THREADS 256
#define PMLP_OPT_PARTS 256

// The per-step bookkeeping of a torch-optimizer PPO step in one thread: the logged
// losses and the KL-adaptive learning rate (rsl_rl v1.0.2 PPO.update), from the fused
// loss's stats = [surrogate, value, kl, entropy] (the ~10 small torch ops it replaces
// are each a launch).
__global__ void k_loss_bookkeeping(const float* __restrict__ stats, float* lr, float* acc, float desired_kl,
                                   int adaptive) {
    if (threadIdx.x != 0) return;
    if (acc) {
        acc[0] += stats[1];
        acc[1] += stats[0];
    }
    if (adaptive) {
        const float kl = stats[2];
        float l = lr[0];
        if (kl > desired_kl * 2.f) l = fmaxf(l / 1.5f, 1e-5f);
        else if (kl < desired_kl / 2.f && kl > 0.f) l = fminf(l * 1.5f, 1e-2f);
        lr[0] = l;
    }
}

// partial[b] = sum of (scale*g)^2 over block b's grid-stride share; block 0 also
// advances Adam's step and, from stats = [surrogate, value, kl, entropy] (sums over
// ranks when scale = 1/world), accumulates the logged losses and adapts the LR.
__global__ __launch_bounds__(PMLP_OPT_THREADS) void k_opt_prepare(const float* __restrict__ g, int64_t n, float scale,
                                                                  float* __restrict__ partial, float* step,
                                                                  const float* stats, float* lr, float* acc,
                                                                  float desired_kl, int adaptive) {
    __shared__ float sh[4];
    float s = 0.f;
    // unrolled so that several of a thread's loads are in flight (a rolled loop is a chain
    // of dependent round trips)
#pragma unroll 8
    for (int64_t i = (int64_t)blockIdx.x * PMLP_OPT_THREADS + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * PMLP_OPT_THREADS) {
        const float v = g[i] * scale;
        s += v * v;
    }
    s = block_sum(s, sh);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        step[0] += 1.f;
        if (stats) {
            if (acc) {
                acc[0] += stats[1] * scale;
                acc[1] += stats[0] * scale;
            }
            if (adaptive) {  // rsl_rl v1.0.2 PPO.update: KL-adaptive learning rate
                const float kl = stats[2] * scale;
                float l = lr[0];
                if (kl > desired_kl * 2.f) l = fmaxf(l / 1.5f, 1e-5f);
                else if (kl < desired_kl / 2.f && kl > 0.f) l = fminf(l * 1.5f, 1e-2f);
                lr[0] = l;
            }
        }
    }
}

struct MirrorJobs {
    int64_t off[PMLP_MAX_MIRROR];
    int rows[PMLP_MAX_MIRROR], cols[PMLP_MAX_MIRROR], ld[PMLP_MAX_MIRROR];
    bf16* dst[PMLP_MAX_MIRROR];
    bf16* frag[PMLP_MAX_MIRROR];
    int n;
};
// One element of torch.optim.Adam after clip_grad_norm_ (coef = clip factor x grad scale):
// updates m, v and returns the new parameter.  The fused multiply-adds are explicit: left to
// contraction, the scalar and the packed (vectorised) forms fused different pairs and the
// kernels disagreed in the last bit.  Shared by k_adam and k_adam_vec.
__device__ __forceinline__ float adam_elem(float g, float& m, float& v, float p, float coef, float b1, float b2,
                                           float eps, float step_size, float bc2s) {
    const float gi = g * coef;
    m = __builtin_fmaf(1.f - b1, gi - m, m);
    v = __builtin_fmaf(v, b2, ((1.f - b2) * gi) * gi);
    return __builtin_fmaf(-step_size, m / (sqrtf(v) / bc2s + eps), p);
}
// the grad-norm partials' sum, in the order of k_adam's first form (thread t adds t, t + 256, ...
// in turn, then block_sum); unrolled so that a thread's loads are in flight together
__device__ __forceinline__ float norm_partials_sum(const float* __restrict__ partial, int nparts, float* sh) {
    float s = 0.f;
#pragma unroll 8
    for (int i = threadIdx.x; i < nparts; i += PMLP_OPT_THREADS) s += partial[i];
    return block_sum(s, sh);
}
// index of the fragment-packed copy's element (r, c) of a weight with row stride ld
// (include/ppo_mlp.h pmlp_mirror_job.frag)
__device__ __forceinline__ size_t frag_index(int r, int c, int ld) {
    return ((((size_t)(r >> 5) * (ld >> 4) + (c >> 4)) * 64 + (r & 31) + 32 * ((c >> 3) & 1)) << 3) + (c & 7);
}
__global__ __launch_bounds__(PMLP_OPT_THREADS) void k_adam(float* __restrict__ p, const float* __restrict__ g,
                                                           float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                           float scale, const float* __restrict__ partial, int nparts,
                                                           const float* step, const float* lr, float max_norm,
                                                           float b1, float b2, float eps, MirrorJobs mj) {
    __shared__ float sh[4];
    const float s = norm_partials_sum(partial, nparts, sh);
    float coef = scale;
    if (max_norm > 0.f) coef = scale * fminf(max_norm / (sqrtf(s) + 1e-6f), 1.f);  // clip_grad_norm_
    const float t = step[0];
    const float bc1 = 1.f - powf(b1, t), bc2s = sqrtf(1.f - powf(b2, t));
    const float step_size = lr[0] / bc1;
    for (int64_t i = (int64_t)blockIdx.x * PMLP_OPT_THREADS + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * PMLP_OPT_THREADS) {
        float mi = m[i], vi = v[i];
        const float pi = adam_elem(g[i], mi, vi, p[i], coef, b1, b2, eps, step_size, bc2s);
        m[i] = mi;
        v[i] = vi;
        p[i] = pi;
        for (int j = 0; j < mj.n; ++j) {  // the bf16 GEMM operand copy of a weight
            const int64_t o = i - mj.off[j];
            if (o >= 0 && o < (int64_t)mj.rows[j] * mj.cols[j]) {
                // a weight has < 2^31 entries: 32-bit division (the 64-bit one is a long
                // VALU sequence per element)
                const int oi = (int)o, r = oi / mj.cols[j], c = oi - r * mj.cols[j];
                mj.dst[j][(size_t)r * mj.ld[j] + c] = (bf16)pi;
                if (mj.frag[j]) mj.frag[j][frag_index(r, c, mj.ld[j])] = (bf16)pi;  // the fragment-packed copy
            }
        }
    }
}

// k_adam over VEC consecutive elements per thread (VEC = 2 or 4), one group per thread at the
// host's grid: the thread's loads are issued before the norm partials are summed (one round
// trip, not two in a row), one mirror-job lookup per group, and the bf16 copies stored VEC at
// a time.  The host checks the layout it relies on: 4 VEC-byte aligned flat buffers, every
// mirrored weight's offset, width and row stride multiples of VEC.  Per element the arithmetic
// of k_adam (adam_elem, same partial-sum order): the same bits.
template <int VEC>
__global__ __launch_bounds__(PMLP_OPT_THREADS) void k_adam_vec(float* __restrict__ p, const float* __restrict__ g,
                                                               float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                               float scale, const float* __restrict__ partial, int nparts,
                                                               const float* step, const float* lr, float max_norm,
                                                               float b1, float b2, float eps, MirrorJobs mj) {
    typedef float vf __attribute__((ext_vector_type(VEC)));
    typedef bf16 vb __attribute__((ext_vector_type(VEC)));
    __shared__ float sh[4];
    const int64_t ng = n / VEC, i0 = (int64_t)blockIdx.x * PMLP_OPT_THREADS + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * PMLP_OPT_THREADS;
    vf G, M, V, P;
    if (i0 < ng) {
        G = ((const vf*)g)[i0];
        M = ((const vf*)m)[i0];
        V = ((const vf*)v)[i0];
        P = ((const vf*)p)[i0];
    }
    const float s = norm_partials_sum(partial, nparts, sh);
    float coef = scale;
    if (max_norm > 0.f) coef = scale * fminf(max_norm / (sqrtf(s) + 1e-6f), 1.f);  // clip_grad_norm_
    const float t = step[0];
    const float bc1 = 1.f - powf(b1, t), bc2s = sqrtf(1.f - powf(b2, t));
    const float step_size = lr[0] / bc1;
    for (int64_t i = i0; i < ng; i += stride) {
        if (i != i0) {
            G = ((const vf*)g)[i];
            M = ((const vf*)m)[i];
            V = ((const vf*)v)[i];
            P = ((const vf*)p)[i];
        }
        vb B;
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
            float me = M[e], ve = V[e];
            P[e] = adam_elem(G[e], me, ve, P[e], coef, b1, b2, eps, step_size, bc2s);
            M[e] = me;
            V[e] = ve;
            B[e] = (bf16)P[e];
        }
        ((vf*)m)[i] = M;
        ((vf*)v)[i] = V;
        ((vf*)p)[i] = P;
        const int64_t e0 = i * VEC;
        for (int j = 0; j < mj.n; ++j) {
            const int64_t o = e0 - mj.off[j];
            if (o >= 0 && o < (int64_t)mj.rows[j] * mj.cols[j]) {  // the whole group: one row of weight j
                const int oi = (int)o, r = oi / mj.cols[j], c = oi - r * mj.cols[j];
                *(vb*)(mj.dst[j] + (size_t)r * mj.ld[j] + c) = B;
                if (mj.frag[j]) *(vb*)(mj.frag[j] + frag_index(r, c, mj.ld[j])) = B;  // c % 8 + VEC <= 8
            }
        }
    }
    // the last n % VEC elements (no weight: a mirrored weight ends on a multiple of VEC)
    if (blockIdx.x == 0 && threadIdx.x < n - ng * VEC) {
        const int64_t i = ng * VEC + threadIdx.x;
        float mi = m[i], vi = v[i];
        p[i] = adam_elem(g[i], mi, vi, p[i], coef, b1, b2, eps, step_size, bc2s);
        m[i] = mi;
        v[i] = vi;
    }
}

// (Philox4x32-10, the rollout's policy noise of k_act, k_act4 and the rollout forward: pmlp_noise.h)

// ------------------------------------------------------------ fused MLP forward --
// The whole forward of a 4-layer Linear/ELU MLP (rsl_rl's actor or critic: K0 -> H0 ->
// H1 -> H2 -> N3) in ONE launch: a workgroup of 8 waves owns R mini-batch rows and keeps
// their activations in LDS from layer to layer; only the weights stream (bf16 W[out,in],
// L2-resident), straight into registers as MFMA B fragments.  The hidden outputs are still
// stored (bf16, row-major) when the backward needs them, by 16-byte copies out of LDS.
// Per output element the MFMA chain (v_mfma_f32_32x32x16_bf16, k ascending in steps of
// 16), the bias + ELU epilogue and the bf16 roundings are those of the per-layer GEMMs
// (k_gemm_nt): the result is bitwise the same.
#define FMLP_MAX_H0 512
#define FMLP_MAX_H1 256
#define FMLP_THREADS 512

struct FmlpJob {
    const float* x;         // fp32 input rows: row m of the batch is x[rows ? rows[m] : m]
    const int64_t* rows;
    int ldx, kx;            // x row stride; real input width (columns >= kx read as 0)
    bf16* xa;               // optional: the converted bf16 input rows [M, K0] (ldxa)
    int ldxa;
    const bf16* W[4];       // W[l] = [N[l], K_l] bf16, ld K_l (K_0 = K0, K_l = N[l-1])
    const float* b[4];
    int N[4];
    int K0;                 // padded input width, a multiple of 16, <= 64
    bf16* y[3];             // optional hidden outputs [M, N[l]] (ld ldy[l])
    int ldy[3];
    float* out;             // fp32 [M, N[3]] (ld ldo)
    int ldo;
    const bf16* Wf[4];      // optional fragment-packed W[l] (include/ppo_mlp.h)
};
struct FmlpJobs {
    FmlpJob j[2];
    int njobs;
};

// One layer: D[R, N] = act(A[R, K] . W[N, K]^T + b), A in LDS (ld lda); wave w takes the
// 32-column tiles w, w + 8, ...; every row tile of the workgroup per column tile, so a
// B fragment (one 16-byte load per lane per k-step) feeds RT MFMAs.
template <int R, bool LAST>
__device__ __forceinline__ void fmlp_layer(const bf16* A, int lda, int K, const bf16* __restrict__ W,
                                           const bf16* __restrict__ Wf,
                                           const float* __restrict__ bias, int N, bf16* D, int ldd,
                                           float* __restrict__ out, int ldo, int r0, int M) {
    constexpr int RT = R / 32, NW = FMLP_THREADS / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nct = (N + 31) >> 5, ks = K >> 4;
    for (int ct = wid; ct < nct; ct += NW) {
        floatx16 acc[RT];
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int t = 0; t < 16; ++t) acc[i][t] = 0.f;
        const int n = ct * 32 + (lane & 31);
        const bool nv = n < N;
        // this lane's B fragment of k-step s at wrow + s * wstep: W[n][16 s + 8 (lane >> 5) ..]
        // (32 row pieces per load), or the fragment-packed copy (1 KB contiguous per load)
        const bf16* wrow = Wf ? Wf + ((size_t)ct * ks * 64 + lane) * 8 : W + (size_t)(nv ? n : 0) * K + 8 * (lane >> 5);
        const int wstep = Wf ? 512 : 16;
        const bf16* arow = A + (lane & 31) * lda + 8 * (lane >> 5);
        // B fragments in groups of FG k-steps, the next group's loads in flight while this
        // group's MFMAs run (k ascending, as the per-layer GEMM).  The loads are unconditional,
        // at clamped addresses (a column past N reads row 0 and is never stored; a k-step past
        // the end re-reads the last one and feeds no MFMA): a load under a branch would make
        // the compiler drain every load in flight at the branch's end.
        constexpr int FG = 4;
        bf16x8 bq[FG], bn[FG];
        auto loadg = [&](int s0, bf16x8(&b)[FG]) {
#if defined(PMLP_FMLP_STAMPS) && PMLP_FMLP_STAMPS == 2  // diagnostic: no weight loads
#pragma unroll
            for (int u = 0; u < FG; ++u)
#pragma unroll
                for (int e = 0; e < 8; ++e) b[u][e] = (bf16)(float)(s0 + u + e + lane);
#else
#pragma unroll
            for (int u = 0; u < FG; ++u) b[u] = *(const bf16x8*)(wrow + min(s0 + u, ks - 1) * wstep);
#endif
        };
        // one k-step's RT MFMAs; the whole-group form has no branch between its MFMAs (a
        // uniform branch per k-step splits the loop into blocks the scheduler cannot overlap)
        auto step = [&](int s, const bf16x8& b) {
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                const bf16x8 af = *(const bf16x8*)(arow + i * 32 * lda + s * 16);
#if defined(PMLP_FMLP_STAMPS) && PMLP_FMLP_STAMPS == 3  // diagnostic: no MFMAs
                acc[i][s & 15] += (float)af[0] * (float)b[0];
#else
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, af, acc[i], 0, 0, 0);
#endif
            }
        };
        auto group = [&](int s0, const bf16x8(&b)[FG]) {
#pragma unroll
            for (int u = 0; u < FG; ++u) step(s0 + u, b[u]);
        };
        auto tail = [&](int s0, const bf16x8(&b)[FG]) {
#pragma unroll
            for (int u = 0; u < FG; ++u)
                if (s0 + u < ks) step(s0 + u, b[u]);
        };
        // the epilogue's 16 bias values (this lane's columns), loaded ahead of the k-loop
        float bq4[4][4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                bq4[q][c] = bias ? bias[min(ct * 32 + 8 * q + 4 * (lane >> 5) + c, N - 1)] : 0.f;
        // two fragment sets used in turn (a register copy from one to the other would wait
        // for the loads it is meant to overlap)
        loadg(0, bq);
        int s0 = 0;
        for (; s0 + 2 * FG <= ks; s0 += 2 * FG) {
            loadg(s0 + FG, bn);
            group(s0, bq);
            loadg(s0 + 2 * FG, bq);
            group(s0 + FG, bn);
        }
        if (s0 < ks) {  // (ks not a multiple of 2 FG: the 48-wide input layer)
            loadg(s0 + FG, bn);
            tail(s0, bq);
            tail(s0 + FG, bn);
        }
        // the tile was formed transposed (W . A^T: the weight fragment is the MFMA's first
        // operand), so a lane holds row (lane & 31) of its row tile and, per quad q, the 4
        // consecutive columns 8q + 4 (lane >> 5) + 0..3: one 8-byte LDS store per quad (the
        // same products and k order per element as A . W^T: bitwise the same values)
        const int rl = lane & 31;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int n0 = ct * 32 + 8 * q + 4 * (lane >> 5);
            if (LAST && n0 >= N) continue;
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                const int r = i * 32 + rl;
                if constexpr (LAST) {
                    if (r0 + r < M) {
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            if (n0 + c < N) out[(size_t)(r0 + r) * ldo + n0 + c] = acc[i][4 * q + c] + bq4[q][c];
                    }
                } else {
                    bf16x4 v;
#pragma unroll
                    for (int c = 0; c < 4; ++c) v[c] = (bf16)elu(acc[i][4 * q + c] + bq4[q][c]);
                    *(bf16x4*)(D + r * ldd + n0) = v;
                }
            }
        }
    }
}

// copy an LDS activation tile [R, N] (ld lds_ld) to the global rows r0.. of y (ld ldy)
template <int R>
__device__ __forceinline__ void fmlp_store(const bf16* D, int lds_ld, int N, bf16* y, int ldy, int r0, int M) {
    if (!y) return;
    const int cpr = N >> 3;
    for (int i = threadIdx.x; i < R * cpr; i += FMLP_THREADS) {
        const int r = i / cpr, c = (i - r * cpr) * 8;
        if (r0 + r < M) *(uint4*)(y + (size_t)(r0 + r) * ldy + c) = *(const uint4*)(D + r * lds_ld + c);
    }
}

#ifdef PMLP_FMLP_STAMPS
// diagnostic build only (never the shipped library): per-block phase clocks of k_mlp_fwd
#define FMLP_NSTAMP 20
__device__ unsigned long long g_fmlp_stamps[4096 * FMLP_NSTAMP];
#define FMLP_STAMP(k)                                                                          \
    do {                                                                                       \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                             \
        if (threadIdx.x == 0 && blockIdx.x < 4096) g_fmlp_stamps[blockIdx.x * FMLP_NSTAMP + (k)] = t_; \
    } while (0)
extern "C" int pmlp_diag_fmlp_stamps(unsigned long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fmlp_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#else
#define FMLP_STAMP(k) ((void)(k))
#endif

// pmlp_rollout_step (include/ppo_mlp.h)
struct RollStep {
    const float* stdv;
    const float* obs;
    const float* cobs;
    int O, CO, A;
    float *actions_out, *st_actions, *st_logp, *st_mu, *st_sigma, *st_value, *st_obs, *st_cobs;
    int64_t* draw;
    int parity;
    uint64_t seed;
    const float* rew;
    const uint8_t* dones;
    const uint8_t* time_outs;
    const float* prev_value;
    float* st_rew;
    uint8_t* st_dones;
    float gamma;
    pmlp_env_extras ex;  // the previous step's deferred env extras (ex.acc == NULL: none)
};

// A deferred env step's extras (include/ppo_mlp.h pmlp_env_extras; leggedsim's k_step_extras,
// whose arithmetic this repeats): per env row, and once in the launch's first workgroup.
__device__ __forceinline__ bool ex_any(const pmlp_env_extras& x) { return x.acc[x.nsum] > 0.f; }
// row i: the carried time-out byte the bootstrap reads (this step's when any env reset: the
// carry is updated first), and the push bookkeeping of the step's all-env draw
__device__ __forceinline__ bool ex_row(const pmlp_env_extras& x, bool any, int i, const uint8_t* time_outs) {
    bool to = false;
    if (x.carry && any) {
        const uint8_t b = x.time_out[i];
        x.carry[i] = b;
        to = b != 0;
    } else if (time_outs) {
        to = time_outs[i] != 0;
    }
    if (x.push && x.last_root_vel && !x.pushed[x.pushed[2] & 1u]) {  // no env pushed: the simulated velocities
        x.last_root_vel[6 * (size_t)i] = x.vsim[2 * (size_t)i];
        x.last_root_vel[6 * (size_t)i + 1] = x.vsim[2 * (size_t)i + 1];
    }
    return to;
}
// once (threads t of one workgroup, t <= nsum < 64 covered): the episode means, the next step's
// accumulator, the next parity's push flag, the step counter
__device__ __forceinline__ void ex_once(const pmlp_env_extras& x, bool any, int t) {
#pragma clang fp contract(off)
    if (x.ep_means && t < x.nsum) {
        float m = x.ep_means[t];
        if (any) m = x.acc[t] / fmaxf(x.acc[x.nsum], 1.f) / x.ep_len_s;
        x.ep_means[t] = m;
        if (x.ep_snapshot) x.ep_snapshot[t] = m;
    }
    if (t <= x.nsum) x.acc_next[t] = 0.f;
    if (t == 0) {
        x.pushed[(x.pushed[2] + 1u) & 1u] = 0u;
        if (x.step_counter) *x.step_counter += 1;
    }
}

// The rollout's work on the workgroup's R rows after job jj's forward (its outputs are in
// J.out, written by this workgroup before the barrier that precedes this call).  Job 0 (the
// actor): sampling and the storage rows, k_act4's Philox counters and arithmetic; the
// deferred store of the previous step.  Job 1 (the critic): the value and privileged rows.
template <int R>
__device__ void roll_epilogue(const FmlpJob& J, int jj, const RollStep& rs, int r0, int M, float* terms) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x;
    if (jj == 0) {
        const uint32_t draw = (uint32_t)rs.draw[rs.parity];
        const uint2 key = make_uint2((uint32_t)rs.seed, (uint32_t)(rs.seed >> 32));
        for (int q = tid; q < R * 4; q += FMLP_THREADS) {  // (row, action quad)
            const int rl = q >> 2, c = q & 3, k0 = 4 * c, i = r0 + rl;
            if (i >= M || k0 >= rs.A) continue;
            const uint4 r = philox4x32(make_uint4(draw, (uint32_t)i, (uint32_t)c, 0x5050u), key);
            const float rad0 = sqrtf(-2.f * logf(u01(r.x))), rad1 = sqrtf(-2.f * logf(u01(r.z)));
            float z[4];
            sincospif(2.f * u01(r.y), &z[1], &z[0]);
            sincospif(2.f * u01(r.w), &z[3], &z[2]);
            z[0] *= rad0; z[1] *= rad0; z[2] *= rad1; z[3] *= rad1;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + u;
                if (k >= rs.A) break;
                const size_t o = (size_t)i * rs.A + k;
                const float sg = rs.stdv[k], mu = J.out[(size_t)i * J.ldo + k];
                const float act = mu + sg * z[u];
                const float d = act - mu;
                terms[rl * 16 + k] = -(d * d) / (2.f * sg * sg) - logf(sg) - kHalfLog2Pi;
                rs.actions_out[o] = act;
                rs.st_actions[o] = act;
                rs.st_mu[o] = mu;
                rs.st_sigma[o] = sg;
            }
        }
        __syncthreads();
        const bool ex = rs.rew && rs.ex.acc;
        const bool any = ex && ex_any(rs.ex);
        if (tid < R && r0 + tid < M) {
            const int i = r0 + tid;
            float logp = 0.f;
            for (int k = 0; k < rs.A; ++k) logp += terms[tid * 16 + k];
            rs.st_logp[i] = logp;
            if (rs.rew) {  // the previous step's process_env_step (k_store_step's arithmetic)
                const bool to = ex ? ex_row(rs.ex, any, i, rs.time_outs) : (rs.time_outs && rs.time_outs[i]);
                float rw = rs.rew[i];
                if (rs.time_outs) rw = rw + rs.gamma * (rs.prev_value[i] * (to ? 1.f : 0.f));
                rs.st_rew[i] = rw;
                rs.st_dones[i] = rs.dones[i] ? 1 : 0;
            }
        }
        if (ex && blockIdx.x == 0) ex_once(rs.ex, any, tid);
        const int nrow = min(R, M - r0);
        for (int q = tid; q < nrow * rs.O; q += FMLP_THREADS)
            rs.st_obs[(size_t)r0 * rs.O + q] = rs.obs[(size_t)r0 * rs.O + q];
        if (blockIdx.x == 0 && tid == 0) rs.draw[rs.parity ^ 1] = (int64_t)draw + 1;
    } else {
        if (tid < R && r0 + tid < M) rs.st_value[r0 + tid] = J.out[(size_t)(r0 + tid) * J.ldo];
        if (rs.st_cobs) {
            const int nrow = min(R, M - r0);
            for (int q = tid; q < nrow * rs.CO; q += FMLP_THREADS)
                rs.st_cobs[(size_t)r0 * rs.CO + q] = rs.cobs[(size_t)r0 * rs.CO + q];
        }
    }
}

// LOSS: the update's PPO loss on the workgroup's rows after both nets (loss_quad_rows; the
// workgroup runs every job, gridDim.y == 1), its partial sums in row blockIdx.x
template <int R, bool ROLL = false, bool LOSS = false>
__global__ __launch_bounds__(FMLP_THREADS) void k_mlp_fwd(FmlpJobs jobs, int M, RollStep rs, LossArgs la = {},
                                                         LossStepOut lo = {}) {
    // y0 (then y2) and x (then y1); row strides 8 elements past the width: ds_read_b128
    // fragment reads of 32 consecutive rows hit 4-bank groups 4 apart (conflict-free)
    constexpr int LD0 = FMLP_MAX_H0 + 8, LD1 = FMLP_MAX_H1 + 8;
    // the 96-row form keeps the input rows in a region of their own (LDX = 64 + 4: the 160 KB
    // hold it), so a second job on the same rows (the critic on the actor's observations)
    // does not gather them again; the 32-row form stages them in Y1 (3 workgroups per CU)
    constexpr bool XR = R >= 96;
    constexpr int LDX = 68;
    __shared__ __attribute__((aligned(16))) bf16 Y0[R * LD0];
    __shared__ __attribute__((aligned(16))) bf16 Y1[R * LD1];
    __shared__ __attribute__((aligned(16))) bf16 X[XR ? R * LDX : 8];
    bf16* const xs = XR ? X : Y1;
    const int ldxs = XR ? LDX : LD1;
    const int r0 = blockIdx.x * R;
    const int jb = gridDim.y > 1 ? blockIdx.y : 0, je = gridDim.y > 1 ? blockIdx.y + 1 : jobs.njobs;
    for (int jj = jb; jj < je; ++jj) {
        const FmlpJob& J = jobs.j[jj];
        const int sb = 9 * (jj - jb);
        FMLP_STAMP(sb + 0);
        const FmlpJob& P = jobs.j[jj > 0 ? jj - 1 : 0];
        const bool same_rows = XR && jj > jb && !J.xa && J.x == P.x && J.rows == P.rows && J.ldx == P.ldx &&
                               J.kx == P.kx && J.K0 == P.K0;
        // input rows: gathered, fp32 -> bf16 (columns >= kx are 0), into LDS (+ the bf16 copy)
        const int cpr = J.K0 >> 3;
        for (int i = threadIdx.x; i < (same_rows ? 0 : R * cpr); i += FMLP_THREADS) {
            const int r = i / cpr, k = (i - r * cpr) * 8, m = r0 + r;
            bf16x8 t;
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] = (bf16)0.f;
            if (m < M) {
                const float* src = J.x + (size_t)(J.rows ? J.rows[m] : (int64_t)m) * J.ldx + k;
                if (k + 8 <= J.kx) {
                    const float4 x0 = *(const float4*)src, x1 = *(const float4*)(src + 4);
                    t[0] = (bf16)x0.x; t[1] = (bf16)x0.y; t[2] = (bf16)x0.z; t[3] = (bf16)x0.w;
                    t[4] = (bf16)x1.x; t[5] = (bf16)x1.y; t[6] = (bf16)x1.z; t[7] = (bf16)x1.w;
                } else {
#pragma unroll
                    for (int u = 0; u < 8; ++u) t[u] = k + u < J.kx ? (bf16)src[u] : (bf16)0.f;
                }
                if (J.xa) *(bf16x8*)(J.xa + (size_t)m * J.ldxa + k) = t;
            }
            *(bf16x8*)(xs + r * ldxs + k) = t;
        }
        __syncthreads();
        FMLP_STAMP(sb + 1);
        fmlp_layer<R, false>(xs, ldxs, J.K0, J.W[0], J.Wf[0], J.b[0], J.N[0], Y0, LD0, nullptr, 0, r0, M);
        FMLP_STAMP(sb + 2);
        __syncthreads();
        fmlp_store<R>(Y0, LD0, J.N[0], J.y[0], J.ldy[0], r0, M);
        FMLP_STAMP(sb + 3);
        fmlp_layer<R, false>(Y0, LD0, J.N[0], J.W[1], J.Wf[1], J.b[1], J.N[1], Y1, LD1, nullptr, 0, r0, M);
        FMLP_STAMP(sb + 4);
        __syncthreads();
        fmlp_store<R>(Y1, LD1, J.N[1], J.y[1], J.ldy[1], r0, M);
        FMLP_STAMP(sb + 5);
        fmlp_layer<R, false>(Y1, LD1, J.N[1], J.W[2], J.Wf[2], J.b[2], J.N[2], Y0, LD0, nullptr, 0, r0, M);
        FMLP_STAMP(sb + 6);
        __syncthreads();
        fmlp_store<R>(Y0, LD0, J.N[2], J.y[2], J.ldy[2], r0, M);
        FMLP_STAMP(sb + 7);
        fmlp_layer<R, true>(Y0, LD0, J.N[2], J.W[3], J.Wf[3], J.b[3], J.N[3], nullptr, 0, J.out, J.ldo, r0, M);
        __syncthreads();  // (the next job restages x over y1)
        FMLP_STAMP(sb + 8);
        if constexpr (ROLL) roll_epilogue<R>(J, jj, rs, r0, M, (float*)Y1);  // (one job per workgroup)
    }
    // both nets' outputs of these rows are in global memory (written by this workgroup before
    // the barrier that ended the last job); Y1 is dead
    if constexpr (LOSS) loss_quad_rows<R / 16>(la, lo, r0, blockIdx.x, (float*)Y1);
}

// ----------------------------------------------------------------- GAE --
// RolloutStorage.compute_returns: one thread per env walks t backwards; the
// advantage sums for the normalisation go to per-block fp64 partials.
__global__ __launch_bounds__(PMLP_OPT_THREADS) void k_gae(const float* __restrict__ rew,
                                                          const uint8_t* __restrict__ dones,
                                                          const float* __restrict__ values,
                                                          const float* __restrict__ last_values,
                                                          float* __restrict__ ret, float* __restrict__ adv, int T,
                                                          int N, float gamma, float lam, double* __restrict__ partial) {
#pragma clang fp contract(off)
    __shared__ double shd[2][4];
    const int e = blockIdx.x * PMLP_OPT_THREADS + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
    if (e < N) {
        float a = 0.f;
        for (int t = T - 1; t >= 0; --t) {
            const size_t i = (size_t)t * N + e;
            const float next = t == T - 1 ? last_values[e] : values[i + N];
            const float nt = 1.f - (dones[i] ? 1.f : 0.f);
            const float delta = (rew[i] + (nt * gamma) * next) - values[i];
            a = delta + ((nt * gamma) * lam) * a;
            const float r = a + values[i];
            ret[i] = r;
            const float ad = r - values[i];
            adv[i] = ad;
            s1 += ad;
            s2 += (double)ad * ad;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        s1 += __shfl_xor(s1, off);
        s2 += __shfl_xor(s2, off);
    }
    if ((threadIdx.x & 63) == 0) {
        shd[0][threadIdx.x >> 6] = s1;
        shd[1][threadIdx.x >> 6] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = (shd[0][0] + shd[0][1]) + (shd[0][2] + shd[0][3]);
        partial[2 * blockIdx.x + 1] = (shd[1][0] + shd[1][1]) + (shd[1][2] + shd[1][3]);
    }
}

// adv = (adv - mean) / (std + 1e-8), unbiased std over all T*N advantages.  gstats
// (data-parallel): the all-reduced {sum, sum of squares, count} of every rank's
// advantages replace this rank's partials, so each rank normalises by the global moments.
__global__ __launch_bounds__(PMLP_OPT_THREADS) void k_adv_norm(float* __restrict__ adv, int64_t n,
                                                               const double* __restrict__ partial, int nparts,
                                                               const double* __restrict__ gstats) {
    __shared__ double sh[3];
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0, c = (double)n;
        if (gstats) {
            a = gstats[0]; b = gstats[1]; c = gstats[2];
        } else {
            for (int i = 0; i < nparts; ++i) {
                a += partial[2 * i];
                b += partial[2 * i + 1];
            }
        }
        sh[0] = a;
        sh[1] = b;
        sh[2] = c;
    }
    __syncthreads();
    const double cnt = sh[2];
    const double mean = sh[0] / cnt;
    const double var = (sh[1] - cnt * mean * mean) / (cnt - 1.0);
    const float meanf = (float)mean, den = (float)sqrt(var > 0.0 ? var : 0.0) + 1e-8f;
    for (int64_t i = (int64_t)blockIdx.x * PMLP_OPT_THREADS + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * PMLP_OPT_THREADS)
        adv[i] = (adv[i] - meanf) / den;
}

// ------------------------------------------------------------- rollout --
// PPO.act tail + RolloutStorage.add_transitions (rsl_rl v1.0.2) for the
// Gaussian MLP policy, and PPO.process_env_step's reward bootstrap + store.
// Policy noise: Philox4x32-10 keyed (seed; draw, row, pair) -> Box-Muller.

struct ActArgs {
    const float *mu, *stdv, *value, *obs, *cobs;
    float *actions_out, *st_actions, *st_logp, *st_mu, *st_sigma, *st_value, *st_obs, *st_cobs;
    const int64_t* draw;
    uint64_t seed;
    int N, A, O, CO;
};

__global__ __launch_bounds__(256) void k_act(ActArgs a) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
    const uint32_t draw = (uint32_t)*a.draw;
    const uint2 key = make_uint2((uint32_t)a.seed, (uint32_t)(a.seed >> 32));
    for (int64_t i = tid; i < a.N; i += nth) {
        float logp = 0.f;
        for (int k0 = 0; k0 < a.A; k0 += 4) {
            const uint4 r = philox4x32(make_uint4(draw, (uint32_t)i, (uint32_t)(k0 >> 2), 0x5050u), key);
            const float rad0 = sqrtf(-2.f * logf(u01(r.x))), rad1 = sqrtf(-2.f * logf(u01(r.z)));
            float z[4];
            sincospif(2.f * u01(r.y), &z[1], &z[0]);
            sincospif(2.f * u01(r.w), &z[3], &z[2]);
            z[0] *= rad0; z[1] *= rad0; z[2] *= rad1; z[3] *= rad1;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + u;
                if (k >= a.A) break;
                const size_t o = (size_t)i * a.A + k;
                const float sg = a.stdv[k], mu = a.mu[o];
                const float act = mu + sg * z[u];
                const float d = act - mu;
                logp += -(d * d) / (2.f * sg * sg) - logf(sg) - kHalfLog2Pi;
                a.actions_out[o] = act;
                a.st_actions[o] = act;
                a.st_mu[o] = mu;
                a.st_sigma[o] = sg;
            }
        }
        a.st_logp[i] = logp;
        a.st_value[i] = a.value[i];
    }
    // observations into the storage row (float4 when aligned)
    const int64_t no = (int64_t)a.N * a.O;
    if ((no & 3) == 0 && (((uintptr_t)a.obs | (uintptr_t)a.st_obs) & 15) == 0) {
        for (int64_t j = tid; j < no / 4; j += nth) ((float4*)a.st_obs)[j] = ((const float4*)a.obs)[j];
    } else {
        for (int64_t j = tid; j < no; j += nth) a.st_obs[j] = a.obs[j];
    }
    if (a.st_cobs) {
        const int64_t nc = (int64_t)a.N * a.CO;
        for (int64_t j = tid; j < nc; j += nth) a.st_cobs[j] = a.cobs[j];
    }
}

// A <= 16: four lanes per env, lane c drawing and storing actions 4c..4c+3 (the Philox
// counters of k_act, so the same samples); the env's log-prob terms go through LDS and
// its first lane sums them in k order (k_act's arithmetic).  4x the sampling lanes of
// k_act, whose one-lane-per-env loop kept the draw on a handful of CUs.
__global__ __launch_bounds__(256) void k_act4(ActArgs a) {
    __shared__ float terms[64][16];
    const int64_t nth = (int64_t)gridDim.x * blockDim.x;
    const uint32_t draw = (uint32_t)*a.draw;
    const uint2 key = make_uint2((uint32_t)a.seed, (uint32_t)(a.seed >> 32));
    const int le = threadIdx.x >> 2, c = threadIdx.x & 3, k0 = 4 * c;
    const bool vec = (a.A & 3) == 0 &&
                     ((((uintptr_t)a.mu | (uintptr_t)a.actions_out | (uintptr_t)a.st_actions | (uintptr_t)a.st_mu |
                        (uintptr_t)a.st_sigma) & 15) == 0);
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < (int64_t)a.N * 4; base += nth) {
        const int64_t i = (base + threadIdx.x) >> 2;
        if (i < a.N && k0 < a.A) {
            const size_t o = (size_t)i * a.A + k0;
            float act[4], mu[4], sg[4], tm[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) mu[u] = k0 + u < a.A ? a.mu[o + u] : 0.f;
            act_quad(draw, key, (uint32_t)i, c, a.A, a.stdv, mu, act, sg, tm);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (k0 + u < a.A) terms[le][k0 + u] = tm[u];
            if (vec) {
                const float4 av = make_float4(act[0], act[1], act[2], act[3]);
                *(float4*)(a.actions_out + o) = av;
                *(float4*)(a.st_actions + o) = av;
                *(float4*)(a.st_mu + o) = make_float4(mu[0], mu[1], mu[2], mu[3]);
                *(float4*)(a.st_sigma + o) = make_float4(sg[0], sg[1], sg[2], sg[3]);
            } else {
                for (int u = 0; u < 4 && k0 + u < a.A; ++u) {
                    a.actions_out[o + u] = act[u];
                    a.st_actions[o + u] = act[u];
                    a.st_mu[o + u] = mu[u];
                    a.st_sigma[o + u] = sg[u];
                }
            }
        }
        __syncthreads();
        if (c == 0 && i < a.N) {
            float logp = 0.f;
            for (int k = 0; k < a.A; ++k) logp += terms[le][k];
            a.st_logp[i] = logp;
            a.st_value[i] = a.value[i];
        }
        __syncthreads();
    }
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t no = (int64_t)a.N * a.O;
    if ((no & 3) == 0 && (((uintptr_t)a.obs | (uintptr_t)a.st_obs) & 15) == 0) {
        for (int64_t j = tid; j < no / 4; j += nth) ((float4*)a.st_obs)[j] = ((const float4*)a.obs)[j];
    } else {
        for (int64_t j = tid; j < no; j += nth) a.st_obs[j] = a.obs[j];
    }
    if (a.st_cobs) {
        const int64_t nc = (int64_t)a.N * a.CO;
        for (int64_t j = tid; j < nc; j += nth) a.st_cobs[j] = a.cobs[j];
    }
}

// rewards[i] + gamma * (value[i] * time_out[i]) and dones into the storage row;
// then the policy-noise draw counter advances (one thread, after k_act)
// the recurrent memories' states [N, H] zeroed on the done envs (Memory.reset's masked_fill_)
struct MemReset {
    float* s[PMLP_MAX_MEM_STATES];
    int n, H;
};

// a deferred env step's extras (ex.acc != NULL) on the same rows, and once in block 0
__global__ __launch_bounds__(256) void k_store_step(const float* __restrict__ rew, const uint8_t* __restrict__ dones,
                                                    const uint8_t* time_outs,
                                                    const float* __restrict__ st_value, float* __restrict__ st_rew,
                                                    uint8_t* __restrict__ st_dones, int N, float gamma,
                                                    int64_t* draw, MemReset mr, pmlp_env_extras ex) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool any = ex.acc && ex_any(ex);
    if (ex.acc && blockIdx.x == 0) ex_once(ex, any, threadIdx.x);
    if (i < N) {
        const bool to = ex.acc ? ex_row(ex, any, i, time_outs) : (time_outs && time_outs[i]);
        float r = rew[i];
        if (time_outs) r = r + gamma * (st_value[i] * (to ? 1.f : 0.f));
        st_rew[i] = r;
        const bool d = dones[i] != 0;
        st_dones[i] = d ? 1 : 0;
        if (d)
            for (int k = 0; k < mr.n; ++k) {
                float4* h = (float4*)(mr.s[k] + (size_t)i * mr.H);
                for (int j = 0; j < mr.H / 4; ++j) h[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
    }
    if (i == 0 && draw) *draw += 1;
}

// GEMM operand staging: 1 = LDS-DMA (GL) where the shapes allow it, 0 = register staging only
// (pmlp_set_gemm_staging selects the others for in-process A/B)
static int g_glds = 1;
static int glds_on() {
    return g_glds;
}

// every job of the batch fits the GL k-loop at this tile (whole 64-deep k-tiles; k-major
// operands whole tiles wide)
template <int BM, int BN>
static bool gl_fits(int epi, int mode, const GemmBatch& gb, int njobs) {
    if (!glds_on() || (mode & 1)) return false;
    const bool tnl = epi == PMLP_EPI_PARTIAL_TN, bkn = tnl || (mode & 2);
    if (glds_on() == 2 && !tnl) return false;  // 2: the LDS-DMA ring, split-K weight gradients only
    if (glds_on() == 3 && !tnl && epi != PMLP_EPI_BWD_DX) return false;  // 3: + two buffers for BWD_DX
    if (epi == PMLP_EPI_PARTIAL) return false;
    if (tnl && (BM % 64 || BM > 128)) return false;
    if (bkn && (BN % 64 || BN > 128)) return false;
    for (int i = 0; i < njobs; ++i) {
        const GemmArgs& g = gb.j[i];
        if (g.K % 64 || (tnl && g.ksplit % 64)) return false;
        if (tnl && (g.M % BM || g.lda < g.M)) return false;
        if (bkn && (g.N % BN || g.ldb < g.N)) return false;
    }
    return true;
}

template <int BM, int BN, int WM, int WN>
static void launch(int epi, int mode, const GemmBatch& gb, int njobs, int maxm, int maxn, int maxk, hipStream_t st) {
    dim3 grid((maxm + BM - 1) / BM, (maxn + BN - 1) / BN, njobs * gb.slabs), block(64 * WM * WN);
    const bool af = (mode & 1) != 0, bkn = (mode & 2) != 0;
    constexpr bool km_a = BM % 64 == 0 && BM <= 128, km_b = BN % 64 == 0 && BN <= 128;  // k-major GL images
    if (gl_fits<BM, BN>(epi, mode, gb, njobs)) {
        switch (epi) {
        case PMLP_EPI_FWD_HIDDEN: hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 0, 4, 0, 1>), grid, block, 0, st, gb); return;
        case PMLP_EPI_FWD_OUT: hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 1, 4, 0, 1>), grid, block, 0, st, gb); return;
        case PMLP_EPI_BWD_DX:
            if (!bkn) {
                hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 2, 4, 0, 1>), grid, block, 0, st, gb);
                return;
            }
            if constexpr (km_b) {
                hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 2, 4, 2, 1>), grid, block, 0, st, gb);
                return;
            }
            break;
        case PMLP_EPI_PARTIAL_TN:
            if constexpr (km_a && km_b) {
                if (glds_on() >= 2) hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 4, 4, 0, 2>), grid, block, 0, st, gb);
                else hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 4, 4, 0, 1>), grid, block, 0, st, gb);
                return;
            }
            break;
        default: break;
        }
    }
    // one short k-tile: only the k-steps that carry data (K = 48 forward, K = 16 input gradient)
    if (epi == PMLP_EPI_FWD_HIDDEN && maxk <= 48 && maxk > 32) {
        if (af) hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 0, 3, 1>), grid, block, 0, st, gb);
        else hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 0, 3>), grid, block, 0, st, gb);
        return;
    }
    if (epi == PMLP_EPI_BWD_DX && maxk <= 16) {
        if (bkn) hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 2, 1, 2>), grid, block, 0, st, gb);
        else hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 2, 1>), grid, block, 0, st, gb);
        return;
    }
    switch (epi) {
    case PMLP_EPI_FWD_HIDDEN:
        if (af) hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 0, 4, 1>), grid, block, 0, st, gb);
        else hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 0>), grid, block, 0, st, gb);
        break;
    case PMLP_EPI_FWD_OUT:
        if (af) hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 1, 4, 1>), grid, block, 0, st, gb);
        else hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 1>), grid, block, 0, st, gb);
        break;
    case PMLP_EPI_BWD_DX:
        if (bkn) hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 2, 4, 2>), grid, block, 0, st, gb);
        else hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 2>), grid, block, 0, st, gb);
        break;
    case PMLP_EPI_PARTIAL: hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 3>), grid, block, 0, st, gb); break;
    default: hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, 4>), grid, block, 0, st, gb); break;
    }
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" {

PMLP_API const char* pmlp_last_error(void) { return g_err.c_str(); }

PMLP_API int pmlp_set_gemm_staging(int32_t glds) {
    const int prev = glds_on();
    g_glds = glds < 0 ? 0 : (glds > 3 ? 3 : glds);
    return prev;
}

PMLP_API int pmlp_convert(int32_t njobs, const pmlp_convert_job* jobs, void* stream) {
    if (njobs <= 0 || njobs > PMLP_MAX_JOBS || !jobs) return fail(-1, "pmlp_convert: 1..PMLP_MAX_JOBS jobs");
    CvtJobs cj{};
    cj.njobs = njobs;
    int nb = 0;
    for (int i = 0; i < njobs; ++i) {
        const pmlp_convert_job& J = jobs[i];
        if (!J.x || J.M <= 0 || J.K <= 0 || J.Kp < J.K || J.ldx < J.K || (!J.y && !J.yt) || (J.yt && J.ldyt < J.M) ||
            J.one_col < 0 || J.one_col >= J.Kp || (J.one_col > 0 && (J.one_col < J.K || J.yt)))
            return fail(-1, "pmlp_convert: bad job " + std::to_string(i));
        cj.j[i] = CvtJob{J.x, (bf16*)J.y, (bf16*)J.yt, J.rows, J.M, J.K, J.ldx, J.Kp, J.yt ? J.ldyt : 0,
                         J.one_col > 0 ? J.one_col : -1};
        const int mext = std::max(J.M, J.yt ? J.ldyt : 0);
        cj.gm[i] = (mext + 63) / 64;
        cj.start[i] = nb;
        nb += cj.gm[i] * ((J.Kp + 63) / 64);
    }
    cj.start[njobs] = nb;
    hipLaunchKernelGGL(k_convert_jobs, dim3(nb), dim3(256), 0, (hipStream_t)stream, cj);
    PMLP_CHECK_LAUNCH("pmlp_convert");
    return 0;
}

}  // extern "C"

// pmlp_gemm's argument checks and packing: one batch of jobs -> GemmBatch (+ its extents)
static int gemm_pack(int32_t epi, int32_t njobs, const pmlp_gemm_job* jobs, int32_t ksplit, GemmBatch& gb, int& maxm,
                     int& maxn, int& maxk, int& mode) {
    if (epi < 0 || epi > 4) return fail(-1, "pmlp_gemm: unknown epilogue");
    const bool part = epi == PMLP_EPI_PARTIAL || epi == PMLP_EPI_PARTIAL_TN;
    if (njobs <= 0 || njobs > PMLP_MAX_GEMM_JOBS || !jobs) return fail(-1, "pmlp_gemm: 1..PMLP_MAX_GEMM_JOBS jobs");
    gb = GemmBatch{};
    gb.slabs = 1;
    maxm = maxn = maxk = 0;
    mode = (jobs[0].af ? 1 : 0) | (jobs[0].b_kn ? 2 : 0);
    for (int i = 0; i < njobs; ++i) {
        const pmlp_gemm_job& J = jobs[i];
        const std::string w = "pmlp_gemm job " + std::to_string(i) + ": ";
        if (((J.af ? 1 : 0) | (J.b_kn ? 2 : 0)) != mode) return fail(-1, w + "every job must use the same operand forms");
        if ((!J.A && !J.af) || !J.B || J.M <= 0 || J.N <= 0 || J.K <= 0) return fail(-1, w + "null operand or empty shape");
        if (J.af) {
            if ((epi != PMLP_EPI_FWD_HIDDEN && epi != PMLP_EPI_FWD_OUT) || J.kaf <= 0 || J.kaf > J.K ||
                J.ldaf < J.kaf || J.ldaf % 4 || ((uintptr_t)J.af & 15) ||
                (J.xa && (J.ldxa < J.K || J.ldxa % 8 || !al16(J.xa))))
                return fail(-1, w + "fp32 A: forward epilogues, 0 < kaf <= K, ldaf >= kaf a multiple of 4, "
                                    "16-byte aligned; xa: ldxa >= K, a multiple of 8");
        }
        if (J.b_kn && (epi != PMLP_EPI_BWD_DX || J.ldb < J.N || J.ldb % 8 || !al16(J.B) || J.K % 8 || J.lda % 8 ||
                       J.lda < J.K || !al16(J.A)))
            return fail(-1, w + "B given [K,N]: BWD_DX only, ldb >= N, K/lda/ldb multiples of 8, 16-byte aligned");
        if (J.af || J.b_kn) {
            // checked above
        } else if (epi == PMLP_EPI_PARTIAL_TN) {
            // A[K,M], B[K,N]: whole 16-byte chunks along m and n are read
            if (J.lda % 8 || J.ldb % 8 || J.lda < (J.M + 7) / 8 * 8 || J.ldb < (J.N + 7) / 8 * 8 || !al16(J.A) ||
                !al16(J.B))
                return fail(-1, w + "PARTIAL_TN: lda >= ceil8(M), ldb >= ceil8(N), multiples of 8, 16-byte aligned");
        } else if (J.K % 8 || J.lda % 8 || J.ldb % 8 || J.lda < J.K || J.ldb < J.K || !al16(J.A) || !al16(J.B)) {
            return fail(-1, w + "K, lda, ldb must be multiples of 8 with 16-byte aligned operands");
        }
        if (J.sum_col && (epi != PMLP_EPI_PARTIAL_TN || J.sum_col < J.N || J.sum_col >= J.ldcf))
            return fail(-1, w + "sum_col: PARTIAL_TN only, N <= sum_col < ldcf");
        if ((epi == PMLP_EPI_FWD_OUT || part) && (!J.cf || J.ldcf < J.N))
            return fail(-1, w + "fp32 output missing or ldcf < N");
        if ((epi == PMLP_EPI_FWD_HIDDEN || epi == PMLP_EPI_BWD_DX) &&
            ((!J.cb && !J.ct) || (J.cb && J.ldcb < J.N) || (J.ct && (J.ldct < J.M || J.ldct % 4))))
            return fail(-1, w + "bf16 output missing or bad leading dimension");
        if (epi == PMLP_EPI_BWD_DX && (!J.yprev || J.ldyp < J.N)) return fail(-1, w + "BWD_DX needs yprev");
        GemmArgs& g = gb.j[i];
        g.A = (const bf16*)J.A; g.B = (const bf16*)J.B; g.bias = J.bias; g.yp = (const bf16*)J.yprev;
        g.cf = J.cf; g.cb = (bf16*)J.cb; g.ct = (bf16*)J.ct;
        g.lda = J.lda; g.ldb = J.ldb; g.ldyp = J.ldyp; g.ldcf = J.ldcf; g.ldcb = J.ldcb; g.ldct = J.ldct;
        g.M = J.M; g.N = J.N; g.K = J.K; g.ksplit = ksplit;
        g.af = J.af; g.rows = J.rows; g.xa = (bf16*)J.xa; g.ldaf = J.ldaf; g.kaf = J.kaf; g.ldxa = J.ldxa;
        g.sumc = J.sum_col;
        maxm = std::max(maxm, J.M); maxn = std::max(maxn, J.N); maxk = std::max(maxk, J.K);
    }
    if (part) {
        if (ksplit <= 0 || ksplit % 32) return fail(-1, "pmlp_gemm: ksplit must be a positive multiple of 32");
        for (int i = 0; i < njobs; ++i)
            if ((jobs[i].K + ksplit - 1) / ksplit != (maxk + ksplit - 1) / ksplit)
                return fail(-1, "pmlp_gemm: PARTIAL jobs must have the same number of slabs");
        gb.slabs = (maxk + ksplit - 1) / ksplit;
    }
    return 0;
}

// The k_gemm_nt instantiations of the backward that k_gemm_pair pairs: the plan code of the
// kernel pmlp_gemm's selection below would launch for this batch, or 0 for any other.
//   1: PARTIAL_TN on 32 x 128 tiles, register staging (a narrow layer's weight gradient)
//   2: BWD_DX, B [K,N], one 16-deep k-tile, 64 x 64 tiles (the output layer's input gradient)
//   3: PARTIAL_TN on 128 x 128 tiles, LDS-DMA staging
//   4: BWD_DX, B [K,N], 128 x 128 tiles, LDS-DMA staging
// Pairs (1, 2) and (3, 4) share a block size (256 / 512 threads).
static int gemm_plan(int epi, int mode, const GemmBatch& gb, int njobs, int maxm, int maxn, int maxk) {
    if (epi == PMLP_EPI_PARTIAL_TN && mode == 0) {
        if (maxm <= 32) return gl_fits<32, 128>(epi, mode, gb, njobs) ? 0 : 1;
        if (maxn > 64) return gl_fits<128, 128>(epi, mode, gb, njobs) && glds_on() == 1 ? 3 : 0;
        return 0;
    }
    if (epi == PMLP_EPI_BWD_DX && mode == 2 && maxm > 32 && maxn > 64) {
        const bool small = (long)((maxm + 127) / 128) * ((maxn + 127) / 128) * njobs < 512;
        if (small) return !gl_fits<64, 64>(epi, mode, gb, njobs) && maxk <= 16 ? 2 : 0;
        return gl_fits<128, 128>(epi, mode, gb, njobs) ? 4 : 0;
    }
    return 0;
}

static dim3 gemm_grid(int BM, int BN, const GemmBatch& gb, int njobs, int maxm, int maxn) {
    return dim3((maxm + BM - 1) / BM, (maxn + BN - 1) / BN, njobs * gb.slabs);
}

template <class CA, class CB>
static void launch_pair(const GemmBatch& ga, int nja, int mma, int mna, const GemmBatch& gb2, int njb, int mmb, int mnb,
                        hipStream_t st) {
    const dim3 da = gemm_grid(CA::BM, CA::BN, ga, nja, mma, mna), db = gemm_grid(CB::BM, CB::BN, gb2, njb, mmb, mnb);
    const int na = (int)(da.x * da.y * da.z), nb = (int)(db.x * db.y * db.z);
    hipLaunchKernelGGL((k_gemm_pair<CA, CB>), dim3(na + nb), dim3(CA::NT), 0, st, ga, gb2, na,
                       make_int3((int)da.x, (int)da.y, (int)da.z), make_int3((int)db.x, (int)db.y, (int)db.z));
}

extern "C" {

PMLP_API int pmlp_gemm(int32_t epi, int32_t njobs, const pmlp_gemm_job* jobs, int32_t ksplit, void* stream) {
    GemmBatch gb;
    int maxm, maxn, maxk, mode;
    if (const int rc = gemm_pack(epi, njobs, jobs, ksplit, gb, maxm, maxn, maxk, mode)) return rc;
    const bool part = epi == PMLP_EPI_PARTIAL || epi == PMLP_EPI_PARTIAL_TN;
    hipStream_t st = (hipStream_t)stream;
    if (maxm <= 32) launch<32, 128, 1, 4>(epi, mode, gb, njobs, maxm, maxn, maxk, st);
    else if (maxn <= 32) launch<128, 32, 4, 1>(epi, mode, gb, njobs, maxm, maxn, maxk, st);
    else if (maxn <= 64) launch<128, 64, 4, 1>(epi, mode, gb, njobs, maxm, maxn, maxk, st);
    else if (!part && (long)((maxm + 127) / 128) * ((maxn + 127) / 128) * njobs < 512)
        launch<64, 64, 2, 2>(epi, mode, gb, njobs, maxm, maxn, maxk, st);  // small grids: 4x the blocks hide the k-loop latency
    else {
        // 128x128 output tiles: 8 waves of 64x32 (accumulators in 32 VGPRs, no AGPRs:
        // 4 waves/SIMD resident instead of 3) for the epilogue-heavy short-K GEMMs; 4 waves
        // of 64x64 for the forward GEMMs with a long k-loop (K >= 256), where the 64x64
        // wave tile's operand reuse wins (-18 us per optimizer step).  (Measured and dropped,
        // 128 x 256 tiles, other 128 x 128 wave splits, register load rings.)
        if (epi == PMLP_EPI_FWD_HIDDEN && maxk >= 256) launch<128, 128, 2, 2>(epi, mode, gb, njobs, maxm, maxn, maxk, st);
        else launch<128, 128, 2, 4>(epi, mode, gb, njobs, maxm, maxn, maxk, st);
    }
    PMLP_CHECK_LAUNCH("pmlp_gemm");
    return 0;
}

PMLP_API int pmlp_gemm_pair(int32_t njobs_w, const pmlp_gemm_job* jobs_w, int32_t ksplit, int32_t njobs_x,
                            const pmlp_gemm_job* jobs_x, void* stream) {
    GemmBatch gw, gx;
    int mmw, mnw, mkw, modew, mmx, mnx, mkx, modex;
    if (const int rc = gemm_pack(PMLP_EPI_PARTIAL_TN, njobs_w, jobs_w, ksplit, gw, mmw, mnw, mkw, modew)) return rc;
    if (const int rc = gemm_pack(PMLP_EPI_BWD_DX, njobs_x, jobs_x, 0, gx, mmx, mnx, mkx, modex)) return rc;
    const int pw = gemm_plan(PMLP_EPI_PARTIAL_TN, modew, gw, njobs_w, mmw, mnw, mkw);
    const int px = gemm_plan(PMLP_EPI_BWD_DX, modex, gx, njobs_x, mmx, mnx, mkx);
    hipStream_t st = (hipStream_t)stream;
    if (pw == 1 && px == 2) {
        launch_pair<GemmCfg<32, 128, 1, 4, PMLP_EPI_PARTIAL_TN>, GemmCfg<64, 64, 2, 2, PMLP_EPI_BWD_DX, 1, 2>>(
            gw, njobs_w, mmw, mnw, gx, njobs_x, mmx, mnx, st);
    } else if (pw == 3 && px == 4) {
        launch_pair<GemmCfg<128, 128, 2, 4, PMLP_EPI_PARTIAL_TN, 4, 0, 1>, GemmCfg<128, 128, 2, 4, PMLP_EPI_BWD_DX, 4, 2, 1>>(
            gw, njobs_w, mmw, mnw, gx, njobs_x, mmx, mnx, st);
    } else {  // no paired instantiation for these shapes: the two launches
        if (const int rc = pmlp_gemm(PMLP_EPI_PARTIAL_TN, njobs_w, jobs_w, ksplit, stream)) return rc;
        return pmlp_gemm(PMLP_EPI_BWD_DX, njobs_x, jobs_x, 0, stream);
    }
    PMLP_CHECK_LAUNCH("pmlp_gemm_pair");
    return 0;
}

static int reduce_pack(int32_t njobs, const pmlp_reduce_job* jobs, RedJobs& rj, int64_t& nb) {
    if (njobs <= 0 || njobs > PMLP_MAX_JOBS || !jobs) return fail(-1, "pmlp_reduce_slabs: 1..PMLP_MAX_JOBS jobs");
    rj = RedJobs{};
    nb = 0;
    for (int i = 0; i < njobs; ++i) {
        const pmlp_reduce_job& J = jobs[i];
        if (!J.slab || !J.out || J.nslabs <= 0 || J.n <= 0 || J.stride < J.n ||
            (J.bias_out && (J.cols_in <= J.cols_out || J.cols_out <= 0 || J.n % J.cols_in)))
            return fail(-1, "pmlp_reduce_slabs: bad job " + std::to_string(i));
        constexpr int spt = 8;  // target slabs per thread (4 / 2 measured slower)
        int G = 1;  // <= spt slabs per thread, at most 32 groups
        while (G < 32 && J.nslabs > spt * G) G *= 2;
        rj.j[i] = RedJob{J.slab, J.out, J.bias_out, J.stride, J.n, J.nslabs, J.cols_in, J.cols_out, G};
        rj.start[i] = (int)nb;
        const int64_t eqb = 256 / G;  // element quads per block
        nb += ((J.n + 3) / 4 + eqb - 1) / eqb;
    }
    rj.start[njobs] = (int)nb;
    rj.njobs = njobs;
    return 0;
}

PMLP_API int pmlp_reduce_slabs(int32_t njobs, const pmlp_reduce_job* jobs, void* stream) {
    RedJobs rj;
    int64_t nb;
    if (int e = reduce_pack(njobs, jobs, rj, nb)) return e;
    const RedStep none{};
    hipLaunchKernelGGL(k_reduce_jobs, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, rj, none);
    PMLP_CHECK_LAUNCH("pmlp_reduce_slabs");
    return 0;
}

PMLP_API int64_t pmlp_reduce_slabs_parts(int32_t njobs, const pmlp_reduce_job* jobs) {
    RedJobs rj;
    int64_t nb;
    if (reduce_pack(njobs, jobs, rj, nb)) return -1;
    return nb + 1;  // every workgroup + the loss-finishing one
}

PMLP_API int pmlp_reduce_slabs_step(int32_t njobs, const pmlp_reduce_job* jobs, pmlp_reduce_step* r, void* stream) {
    RedJobs rj;
    int64_t nb;
    if (int e = reduce_pack(njobs, jobs, rj, nb)) return e;
    if (!r || !r->loss_partial || r->loss_blocks <= 0 || r->A <= 0 || r->A > 61 || r->M <= 0 || !r->stdv ||
        !r->stats || !r->dstd)
        return fail(-1, "pmlp_reduce_slabs_step: loss partials / stats / dstd / 0 < A <= 61");
    if (r->norm_partial && (!r->step || !r->lr))
        return fail(-1, "pmlp_reduce_slabs_step: norm_partial needs step and lr");
    // every workgroup (+ the loss-finishing one) writes one norm partial: check the capacity
    // before anything is launched
    if (r->norm_partial && nb + 1 > (int64_t)r->nparts)
        return fail(-1, "pmlp_reduce_slabs_step: " + std::to_string(nb + 1) + " norm partials > capacity " +
                            std::to_string(r->nparts));
    const RedStep rs{r->loss_partial, r->loss_blocks, r->A, r->M, r->ecoef, r->stdv, r->stats, r->dstd,
                     r->norm_partial, r->step, r->lr, r->acc, r->desired_kl, r->adaptive};
    r->nparts = (int32_t)(nb + 1);  // + the loss-finishing workgroup
    hipLaunchKernelGGL(k_reduce_jobs, dim3((unsigned)(nb + 1)), dim3(256), 0, (hipStream_t)stream, rj, rs);
    PMLP_CHECK_LAUNCH("pmlp_reduce_slabs_step");
    return 0;
}

PMLP_API int pmlp_rowsum(int32_t njobs, const pmlp_rowsum_job* jobs, void* stream) {
    if (njobs <= 0 || njobs > PMLP_MAX_JOBS || !jobs) return fail(-1, "pmlp_rowsum: 1..PMLP_MAX_JOBS jobs");
    SumJobs sj{};
    int maxr = 0;
    for (int i = 0; i < njobs; ++i) {
        const pmlp_rowsum_job& J = jobs[i];
        if (!J.x || !J.out || J.rows <= 0 || J.cols <= 0 || J.ld < J.cols || J.ld % 8 || !al16(J.x))
            return fail(-1, "pmlp_rowsum: bad job " + std::to_string(i));
        sj.j[i] = SumJob{(const bf16*)J.x, J.out, J.rows, J.cols, J.ld};
        maxr = std::max(maxr, J.rows);
    }
    hipLaunchKernelGGL(k_rowsum_jobs, dim3(maxr, njobs), dim3(256), 0, (hipStream_t)stream, sj);
    PMLP_CHECK_LAUNCH("pmlp_rowsum");
    return 0;
}


static int loss_args(LossArgs& a, const float* mu, const float* stdv, const float* value, const float* actions,
                     const float* old_logp, const float* old_mu, const float* old_sigma, const float* adv,
                     const float* ret, const float* target, const int64_t* rows, int32_t M, int32_t A, float clip,
                     int32_t clipped_value, float vcoef, float ecoef) {
    if (!mu || !stdv || !value || !actions || !old_logp || !old_mu || !old_sigma || !adv || !ret ||
        (clipped_value && !target) || M <= 0 || A <= 0)
        return fail(-1, "pmlp_ppo_loss: null input or empty batch");
    a = LossArgs{mu, stdv, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, rows, M, A, clipped_value,
                 clip, vcoef, ecoef};
    return 0;
}

PMLP_API int32_t pmlp_ppo_loss_blocks(int32_t M) { return (M + PMLP_LOSS_THREADS - 1) / PMLP_LOSS_THREADS; }

PMLP_API int pmlp_ppo_loss_fwd(const float* mu, const float* stdv, const float* value, const float* actions,
                               const float* old_logp, const float* old_mu, const float* old_sigma, const float* adv,
                               const float* ret, const float* target, const int64_t* rows, int32_t M, int32_t A,
                               float clip, int32_t clipped_value, float vcoef, float ecoef, float* partial, float* loss,
                               float* stats, void* stream) {
    LossArgs a;
    if (int e = loss_args(a, mu, stdv, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, rows, M, A, clip,
                          clipped_value, vcoef, ecoef))
        return e;
    if (!partial || !loss || !stats) return fail(-1, "pmlp_ppo_loss_fwd: null output");
    const int nb = pmlp_ppo_loss_blocks(M);
    hipLaunchKernelGGL(k_ppo_loss_fwd, dim3(nb), dim3(PMLP_LOSS_THREADS), 0, (hipStream_t)stream, a, partial);
    hipLaunchKernelGGL(k_ppo_loss_final, dim3(1), dim3(PMLP_LOSS_THREADS), 0, (hipStream_t)stream, a, partial, nb,
                       loss, stats);
    PMLP_CHECK_LAUNCH("pmlp_ppo_loss_fwd");
    return 0;
}

PMLP_API int pmlp_ppo_loss_bwd(const float* mu, const float* stdv, const float* value, const float* actions,
                               const float* old_logp, const float* old_mu, const float* old_sigma, const float* adv,
                               const float* ret, const float* target, const int64_t* rows, int32_t M, int32_t A,
                               float clip, int32_t clipped_value, float vcoef, float ecoef, const float* gout,
                               float* dmu, float* dvalue, float* partial_std, float* dstd, void* stream) {
    LossArgs a;
    if (int e = loss_args(a, mu, stdv, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, rows, M, A, clip,
                          clipped_value, vcoef, ecoef))
        return e;
    if (!gout || !dmu || !dvalue || !partial_std || !dstd) return fail(-1, "pmlp_ppo_loss_bwd: null output");
    const int nb = pmlp_ppo_loss_blocks(M);
    hipLaunchKernelGGL(k_ppo_loss_bwd, dim3(nb), dim3(PMLP_LOSS_THREADS), 0, (hipStream_t)stream, a, gout, dmu, dvalue,
                       partial_std);
    hipLaunchKernelGGL(k_ppo_loss_std, dim3(1), dim3(PMLP_LOSS_THREADS), 0, (hipStream_t)stream, a, gout,
                       partial_std, nb, dstd);
    PMLP_CHECK_LAUNCH("pmlp_ppo_loss_bwd");
    return 0;
}

PMLP_API int32_t pmlp_opt_parts(void) { return PMLP_OPT_PARTS; }

PMLP_API int pmlp_opt_prepare(const float* grad, int64_t n, float grad_scale, float* partial, float* step,
                              const float* stats, float* lr, float* acc, float desired_kl, int32_t adaptive,
                              void* stream) {
    if (!grad || n <= 0 || !partial || !step || (adaptive && (!stats || !lr)))
        return fail(-1, "pmlp_opt_prepare: null buffer or empty parameter set");
    hipLaunchKernelGGL(k_opt_prepare, dim3(PMLP_OPT_PARTS), dim3(PMLP_OPT_THREADS), 0, (hipStream_t)stream, grad, n,
                       grad_scale, partial, step, stats, lr, acc, desired_kl, adaptive);
    PMLP_CHECK_LAUNCH("pmlp_opt_prepare");
    return 0;
}

PMLP_API int pmlp_loss_bookkeeping(const float* stats, float* lr, float* acc, float desired_kl, int32_t adaptive,
                                   void* stream) {
    if (!stats || (adaptive && !lr)) return fail(-1, "pmlp_loss_bookkeeping: null stats (or lr with adaptive)");
    hipLaunchKernelGGL(k_loss_bookkeeping, dim3(1), dim3(64), 0, (hipStream_t)stream, stats, lr, acc, desired_kl,
                       adaptive);
    PMLP_CHECK_LAUNCH("pmlp_loss_bookkeeping");
    return 0;
}

PMLP_API int pmlp_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                       float grad_scale, const float* partial, const float* step, const float* lr, float max_norm,
                       float beta1, float beta2, float eps, void* stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || n <= 0 || !partial || !step || !lr)
        return fail(-1, "pmlp_adam: null buffer or empty parameter set");
    const int blocks = (int)std::min<int64_t>(1024, (n + PMLP_OPT_THREADS - 1) / PMLP_OPT_THREADS);
    MirrorJobs mj{};
    hipLaunchKernelGGL(k_adam, dim3(blocks), dim3(PMLP_OPT_THREADS), 0, (hipStream_t)stream, param, grad, exp_avg,
                       exp_avg_sq, n, grad_scale, partial, PMLP_OPT_PARTS, step, lr, max_norm, beta1, beta2, eps, mj);
    PMLP_CHECK_LAUNCH("pmlp_adam");
    return 0;
}

PMLP_API int pmlp_adam_mirror_n(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                float grad_scale, const float* partial, int32_t nparts, const float* step,
                                const float* lr, float max_norm, float beta1, float beta2, float eps, int32_t nmirror,
                                const pmlp_mirror_job* mirror, void* stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || n <= 0 || !partial || nparts <= 0 || !step || !lr)
        return fail(-1, "pmlp_adam_mirror: null buffer, empty parameter set or no norm partials");
    if (nmirror < 0 || nmirror > PMLP_MAX_MIRROR || (nmirror && !mirror))
        return fail(-1, "pmlp_adam_mirror: 0..PMLP_MAX_MIRROR mirror jobs");
    MirrorJobs mj{};
    mj.n = nmirror;
    for (int j = 0; j < nmirror; ++j) {
        const pmlp_mirror_job& J = mirror[j];
        if (!J.dst || J.offset < 0 || J.rows <= 0 || J.cols <= 0 || J.ld < J.cols ||
            J.offset + (int64_t)J.rows * J.cols > n || (J.frag && J.ld % 16))
            return fail(-1, "pmlp_adam_mirror: bad mirror job " + std::to_string(j));
        mj.off[j] = J.offset; mj.rows[j] = J.rows; mj.cols[j] = J.cols; mj.ld[j] = J.ld; mj.dst[j] = (bf16*)J.dst;
        mj.frag[j] = (bf16*)J.frag;
    }
    // VEC consecutive elements per thread where the layout allows (k_adam_vec; PMLP_ADAM_VEC =
    // 1, 2 or 4, default 4)
    static const int vec_env = [] {
        const char* e = getenv("PMLP_ADAM_VEC");
        const int v = e ? atoi(e) : 4;
        return v == 1 || v == 2 ? v : 4;
    }();
    int vec = vec_env;
    auto aligned = [](const void* q, int bytes) { return ((uintptr_t)q % bytes) == 0; };
    for (; vec > 1; vec /= 2) {
        bool ok = aligned(param, 4 * vec) && aligned(grad, 4 * vec) && aligned(exp_avg, 4 * vec) &&
                  aligned(exp_avg_sq, 4 * vec);
        for (int j = 0; j < nmirror && ok; ++j)
            ok = mj.off[j] % vec == 0 && mj.cols[j] % vec == 0 && mj.ld[j] % vec == 0 && aligned(mj.dst[j], 2 * vec) &&
                 (!mj.frag[j] || aligned(mj.frag[j], 2 * vec));
        if (ok) break;
    }
    if (vec > 1) {
        const int64_t groups = n / vec;
        const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(4096, (groups + PMLP_OPT_THREADS - 1) / PMLP_OPT_THREADS));
        if (vec == 4)
            hipLaunchKernelGGL(k_adam_vec<4>, dim3(blocks), dim3(PMLP_OPT_THREADS), 0, (hipStream_t)stream, param, grad,
                               exp_avg, exp_avg_sq, n, grad_scale, partial, nparts, step, lr, max_norm, beta1, beta2,
                               eps, mj);
        else
            hipLaunchKernelGGL(k_adam_vec<2>, dim3(blocks), dim3(PMLP_OPT_THREADS), 0, (hipStream_t)stream, param, grad,
                               exp_avg, exp_avg_sq, n, grad_scale, partial, nparts, step, lr, max_norm, beta1, beta2,
                               eps, mj);
        PMLP_CHECK_LAUNCH("pmlp_adam_mirror");
        return 0;
    }
    // grid cap 1024 blocks: for the Go2 parameters (1,486 blocks at one element per thread)
    // uncapped / 1024 / 512 / 256 measured 9.2-9.5 / 7.5-8.1 / 8.5-10.0 / 12.1-12.7 us
    // (profiles/round2/update/adam_grid_ab.txt)
    constexpr int cap = 1024;
    const int blocks = (int)std::min<int64_t>(cap, (n + PMLP_OPT_THREADS - 1) / PMLP_OPT_THREADS);
    hipLaunchKernelGGL(k_adam, dim3(blocks), dim3(PMLP_OPT_THREADS), 0, (hipStream_t)stream, param, grad, exp_avg,
                       exp_avg_sq, n, grad_scale, partial, nparts, step, lr, max_norm, beta1, beta2, eps, mj);
    PMLP_CHECK_LAUNCH("pmlp_adam_mirror");
    return 0;
}

PMLP_API int pmlp_adam_mirror(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                              float grad_scale, const float* partial, const float* step, const float* lr,
                              float max_norm, float beta1, float beta2, float eps, int32_t nmirror,
                              const pmlp_mirror_job* mirror, void* stream) {
    return pmlp_adam_mirror_n(param, grad, exp_avg, exp_avg_sq, n, grad_scale, partial, PMLP_OPT_PARTS, step, lr,
                              max_norm, beta1, beta2, eps, nmirror, mirror, stream);
}

PMLP_API int32_t pmlp_gae_parts(int32_t num_envs) { return (num_envs + PMLP_OPT_THREADS - 1) / PMLP_OPT_THREADS; }

PMLP_API int pmlp_gae(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
                      float* returns, float* advantages, int32_t T, int32_t N, float gamma, float lam,
                      double* partial, void* stream) {
    if (!rewards || !dones || !values || !last_values || !returns || !advantages || !partial || T <= 0 || N <= 0 ||
        (int64_t)T * N < 2)
        return fail(-1, "pmlp_gae: null buffer or empty rollout");
    const int nb = pmlp_gae_parts(N);
    hipLaunchKernelGGL(k_gae, dim3(nb), dim3(PMLP_OPT_THREADS), 0, (hipStream_t)stream, rewards, dones, values,
                       last_values, returns, advantages, T, N, gamma, lam, partial);
    const int64_t n = (int64_t)T * N;
    const int blocks = (int)std::min<int64_t>(1024, (n + PMLP_OPT_THREADS - 1) / PMLP_OPT_THREADS);
    hipLaunchKernelGGL(k_adv_norm, dim3(blocks), dim3(PMLP_OPT_THREADS), 0, (hipStream_t)stream, advantages, n,
                       partial, nb, (const double*)nullptr);
    PMLP_CHECK_LAUNCH("pmlp_gae");
    return 0;
}

// this rank's {sum, sum of squares, count} of the advantages from the GAE partials
__global__ void k_gae_moments(const double* __restrict__ partial, int nparts, int64_t n, double* __restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double a = 0.0, b = 0.0;
        for (int i = 0; i < nparts; ++i) {
            a += partial[2 * i];
            b += partial[2 * i + 1];
        }
        out[0] = a;
        out[1] = b;
        out[2] = (double)n;
    }
}

PMLP_API int pmlp_gae_local(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
                            float* returns, float* advantages, int32_t T, int32_t N, float gamma, float lam,
                            double* partial, double* moments, void* stream) {
    if (!rewards || !dones || !values || !last_values || !returns || !advantages || !partial || !moments || T <= 0 ||
        N <= 0)
        return fail(-1, "pmlp_gae_local: null buffer or empty rollout");
    const int nb = pmlp_gae_parts(N);
    hipLaunchKernelGGL(k_gae, dim3(nb), dim3(PMLP_OPT_THREADS), 0, (hipStream_t)stream, rewards, dones, values,
                       last_values, returns, advantages, T, N, gamma, lam, partial);
    hipLaunchKernelGGL(k_gae_moments, dim3(1), dim3(64), 0, (hipStream_t)stream, partial, nb, (int64_t)T * N, moments);
    PMLP_CHECK_LAUNCH("pmlp_gae_local");
    return 0;
}

PMLP_API int pmlp_adv_normalize(float* advantages, int64_t n, const double* moments, void* stream) {
    if (!advantages || !moments || n <= 0) return fail(-1, "pmlp_adv_normalize: null buffer or empty");
    const int blocks = (int)std::min<int64_t>(1024, (n + PMLP_OPT_THREADS - 1) / PMLP_OPT_THREADS);
    hipLaunchKernelGGL(k_adv_norm, dim3(blocks), dim3(PMLP_OPT_THREADS), 0, (hipStream_t)stream, advantages, n,
                       (const double*)nullptr, 0, moments);
    PMLP_CHECK_LAUNCH("pmlp_adv_normalize");
    return 0;
}

// the jobs' shape checks, then their kernel form
static int fmlp_pack(int32_t njobs, const pmlp_mlp_fwd_job* jobs, int32_t M, FmlpJobs& fj) {
    if (njobs <= 0 || njobs > 2 || !jobs || M <= 0) return fail(-1, "pmlp_mlp_forward: 1..2 jobs, M > 0");
    fj = FmlpJobs{};
    fj.njobs = njobs;
    for (int i = 0; i < njobs; ++i) {
        const pmlp_mlp_fwd_job& J = jobs[i];
        const std::string w = "pmlp_mlp_forward job " + std::to_string(i) + ": ";
        if (!J.x || J.kx <= 0 || J.ldx < J.kx || J.ldx % 4 || ((uintptr_t)J.x & 15))
            return fail(-1, w + "x: 0 < kx <= ldx, ldx a multiple of 4, 16-byte aligned");
        if (J.K0 <= 0 || J.K0 % 16 || J.K0 > 64 || J.kx > J.K0)
            return fail(-1, w + "K0 must be a multiple of 16, kx <= K0 <= 64");
        if (J.xa && (J.ldxa < J.K0 || J.ldxa % 8 || !al16(J.xa))) return fail(-1, w + "xa: ldxa >= K0, a multiple of 8");
        const int lim[3] = {FMLP_MAX_H0, FMLP_MAX_H1, FMLP_MAX_H0};
        for (int l = 0; l < 4; ++l) {
            if (!J.W[l] || !al16(J.W[l])) return fail(-1, w + "null or unaligned weight");
            if (l < 3 && (J.N[l] <= 0 || J.N[l] % 32 || J.N[l] > lim[l]))
                return fail(-1, w + "hidden widths: multiples of 32, <= 512 / 256 / 512");
            if (l < 3 && J.y[l] && (J.ldy[l] < J.N[l] || J.ldy[l] % 8 || !al16(J.y[l])))
                return fail(-1, w + "y: ld >= N, a multiple of 8, 16-byte aligned");
        }
        if (J.N[3] <= 0 || J.N[3] > 32 || !J.out || J.ldo < J.N[3]) return fail(-1, w + "output: 0 < N3 <= 32, ldo >= N3");
        FmlpJob& f = fj.j[i];
        f.x = J.x; f.rows = J.rows; f.ldx = J.ldx; f.kx = J.kx; f.xa = (bf16*)J.xa; f.ldxa = J.ldxa;
        for (int l = 0; l < 4; ++l) {
            f.W[l] = (const bf16*)J.W[l]; f.Wf[l] = (const bf16*)J.Wf[l]; f.b[l] = J.b[l]; f.N[l] = J.N[l];
        }
        f.K0 = J.K0;
        for (int l = 0; l < 3; ++l) { f.y[l] = (bf16*)J.y[l]; f.ldy[l] = J.ldy[l]; }
        f.out = J.out; f.ldo = J.ldo;
    }
    return 0;
}

PMLP_API int pmlp_mlp_forward(int32_t njobs, const pmlp_mlp_fwd_job* jobs, int32_t M, void* stream) {
    FmlpJobs fj;
    if (int e = fmlp_pack(njobs, jobs, M, fj)) return e;
    // rows per workgroup: 96 (one 150 KB workgroup per CU, every job in turn) for the update's
    // mini-batches; 32 with one job per workgroup for the rollout's num_envs rows
    hipStream_t st = (hipStream_t)stream;
    const RollStep none{};
    if (M >= 96 * 192)
        hipLaunchKernelGGL((k_mlp_fwd<96>), dim3((M + 95) / 96, 1), dim3(FMLP_THREADS), 0, st, fj, M, none);
    else
        hipLaunchKernelGGL((k_mlp_fwd<32>), dim3((M + 31) / 32, njobs), dim3(FMLP_THREADS), 0, st, fj, M, none);
    PMLP_CHECK_LAUNCH("pmlp_mlp_forward");
    return 0;
}

// a deferred env step's extras are complete (acc == NULL: none)
static bool env_extras_ok(const pmlp_env_extras& x) {
    return !x.acc || (x.acc_next && x.nsum >= 0 && x.nsum < 64 && x.ep_len_s > 0.f && x.time_out && x.pushed &&
                      (!x.push || !x.last_root_vel || x.vsim));
}

PMLP_API int pmlp_rollout_forward(const pmlp_mlp_fwd_job* jobs, int32_t N, const pmlp_rollout_step* r, void* stream) {
    if (!r || !r->stdv || !r->obs || r->O <= 0 || r->A <= 0 || r->A > 16 || (r->cobs && r->CO <= 0) || !r->draw ||
        (r->parity & ~1) || !r->actions_out || !r->st_actions || !r->st_logp || !r->st_mu || !r->st_sigma ||
        !r->st_value || !r->st_obs || (r->cobs && !r->st_cobs) ||
        (r->rewards && (!r->dones || !r->prev_value || !r->st_rewards || !r->st_dones)) ||
        (r->extras.acc && (!r->rewards || !env_extras_ok(r->extras))))
        return fail(-1, "pmlp_rollout_forward: bad rollout step arguments");
    if (!jobs || N <= 0 || jobs[0].N[3] != r->A || jobs[1].N[3] != 1)
        return fail(-1, "pmlp_rollout_forward: job 0 = actor [N, A], job 1 = critic [N, 1]");
    // the forward's own checks; then the 32-row form, one job per workgroup (the epilogue's layout)
    FmlpJobs fj;
    if (int e = fmlp_pack(2, jobs, N, fj)) return e;
    const RollStep rs{r->stdv, r->obs, r->cobs, r->O, r->CO, r->A, r->actions_out, r->st_actions, r->st_logp,
                      r->st_mu, r->st_sigma, r->st_value, r->st_obs, r->st_cobs, r->draw, r->parity, r->seed,
                      r->rewards, r->dones, r->time_outs, r->prev_value, r->st_rewards, r->st_dones, r->gamma,
                      r->extras};
    hipLaunchKernelGGL((k_mlp_fwd<32, true>), dim3((N + 31) / 32, 2), dim3(FMLP_THREADS), 0, (hipStream_t)stream,
                       fj, N, rs);
    PMLP_CHECK_LAUNCH("pmlp_rollout_forward");
    return 0;
}

PMLP_API int pmlp_act(const float* mu, const float* stdv, const float* value, const float* obs, const float* cobs,
                      int32_t N, int32_t A, int32_t O, int32_t CO, const int64_t* draw, uint64_t seed,
                      float* actions_out, float* st_actions, float* st_logp, float* st_mu, float* st_sigma,
                      float* st_value, float* st_obs, float* st_cobs, void* stream) {
    if (!mu || !stdv || !value || !obs || !draw || !actions_out || !st_actions || !st_logp || !st_mu || !st_sigma ||
        !st_value || !st_obs || N <= 0 || A <= 0 || O <= 0 || (st_cobs && (!cobs || CO <= 0)))
        return fail(-1, "pmlp_act: null buffer or empty shape");
    ActArgs a{mu, stdv, value, obs, cobs, actions_out, st_actions, st_logp, st_mu, st_sigma, st_value, st_obs,
              st_cobs, draw, seed, N, A, O, CO};
    if (A <= 16) {
        const int64_t work = std::max<int64_t>(4 * (int64_t)N, (int64_t)N * O / 4);
        const int blocks = (int)std::min<int64_t>(1024, (work + 255) / 256);
        hipLaunchKernelGGL(k_act4, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
    } else {
        const int64_t work = std::max<int64_t>(N, (int64_t)N * O / 4);
        const int blocks = (int)std::min<int64_t>(1024, (work + 255) / 256);
        hipLaunchKernelGGL(k_act, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
    }
    PMLP_CHECK_LAUNCH("pmlp_act");
    return 0;
}

// A keyed pseudo-random permutation of [0, n) (the mini-batch permutation of
// RolloutStorage.mini_batch_generator, torch.randperm there): a 4-round alternating Feistel
// network on the b-bit domain, b = ceil(log2 n) split into an a-bit and a c-bit half (rounds
// 0, 2 mix the high half with a keyed function of the low one, rounds 1, 3 the low half with
// one of the high: each round is invertible whatever a and c are; Philox4x32-10 round
// function), restricted to [0, n) by cycle walking (the cycle through i < n returns below n).
// The domain is below 2n, so a walk leaves [0, n) with probability < 1/2 per step: the
// longest walk of 98,304 indices is ~8 steps where a balanced network's 2^(2 ceil(b/2))
// domain (up to 4n) took ~25.  One thread per index, no sort.
__global__ __launch_bounds__(256) void k_permutation(int64_t* __restrict__ out, int64_t n, int a, int c, uint2 key) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t ma = (1u << a) - 1u, mc = (1u << c) - 1u;
    const uint64_t dom = 1ull << (a + c);
    uint64_t x = (uint64_t)i;
    for (uint64_t walk = 0; walk < dom; ++walk) {
        uint32_t H = (uint32_t)(x >> c) & ma, L = (uint32_t)x & mc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (r % 2 == 0) H ^= philox4x32(make_uint4(L, (uint32_t)r, 0x9e11u, 0x7e37u), key).x & ma;
            else L ^= philox4x32(make_uint4(H, (uint32_t)r, 0x9e11u, 0x7e37u), key).x & mc;
        }
        x = ((uint64_t)H << c) | L;
        if (x < (uint64_t)n) break;
    }
    out[i] = (int64_t)x;
}

PMLP_API int pmlp_permutation(int64_t* out, int64_t n, uint64_t seed, void* stream) {
    if (!out || n <= 0 || n > (1ll << 40)) return fail(-1, "pmlp_permutation: null output or n outside 1..2^40");
    int b = 2;  // (two bits at least: both halves nonempty)
    while ((1ll << b) < n) ++b;
    const int a = b / 2, c = b - a;
    const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    hipLaunchKernelGGL(k_permutation, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, out, n, a, c,
                       key);
    PMLP_CHECK_LAUNCH("pmlp_permutation");
    return 0;
}

PMLP_API int pmlp_store_step_env(const float* rewards, const uint8_t* dones, const uint8_t* time_outs,
                                 const float* st_value, float* st_rewards, uint8_t* st_dones, int32_t N, float gamma,
                                 int64_t* draw, int32_t nstates, float* const* states, int32_t H,
                                 const pmlp_env_extras* ex, void* stream) {
    if (!rewards || !dones || !st_value || !st_rewards || !st_dones || N <= 0)
        return fail(-1, "pmlp_store_step: null buffer or empty batch");
    const pmlp_env_extras none{};
    if (ex && !env_extras_ok(*ex)) return fail(-1, "pmlp_store_step_env: bad env extras");
    MemReset mr{};
    if (nstates < 0 || nstates > PMLP_MAX_MEM_STATES || (nstates && (!states || H <= 0 || H % 4)))
        return fail(-1, "pmlp_store_step_reset: 0..PMLP_MAX_MEM_STATES states of H (a multiple of 4) floats per env");
    for (int k = 0; k < nstates; ++k) {
        if (!states[k] || ((uintptr_t)states[k] & 15)) return fail(-1, "pmlp_store_step_reset: null or unaligned state");
        mr.s[k] = states[k];
    }
    mr.n = nstates;
    mr.H = H;
    hipLaunchKernelGGL(k_store_step, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, rewards, dones,
                       time_outs, st_value, st_rewards, st_dones, N, gamma, draw, mr, ex ? *ex : none);
    PMLP_CHECK_LAUNCH("pmlp_store_step");
    return 0;
}

PMLP_API int pmlp_store_step_reset(const float* rewards, const uint8_t* dones, const uint8_t* time_outs,
                                   const float* st_value, float* st_rewards, uint8_t* st_dones, int32_t N, float gamma,
                                   int64_t* draw, int32_t nstates, float* const* states, int32_t H, void* stream) {
    return pmlp_store_step_env(rewards, dones, time_outs, st_value, st_rewards, st_dones, N, gamma, draw, nstates,
                               states, H, nullptr, stream);
}

PMLP_API int pmlp_store_step(const float* rewards, const uint8_t* dones, const uint8_t* time_outs,
                             const float* st_value, float* st_rewards, uint8_t* st_dones, int32_t N, float gamma,
                             int64_t* draw, void* stream) {
    return pmlp_store_step_reset(rewards, dones, time_outs, st_value, st_rewards, st_dones, N, gamma, draw, 0, nullptr,
                                 0, stream);
}


PMLP_API int32_t pmlp_ppo_loss_step_parts(int32_t M, int32_t A) { return ((M + 63) / 64) * (3 + A); }

static int loss_step_launch(const LossArgs& a, const LossStepOut& o, int M, int A, int Ap, float* partial,
                            float* stats, float* dstd, void* stream) {
    const int nb = (M + 63) / 64;
    if (A % 4 == 0 && A <= 16 && Ap <= 16 && Ap % 4 == 0)
        hipLaunchKernelGGL(k_ppo_loss_step_q, dim3(nb), dim3(256), 0, (hipStream_t)stream, a, o);
    else if (A <= 16 && Ap % 8 == 0)
        hipLaunchKernelGGL(k_ppo_loss_step_reg<16>, dim3(nb), dim3(64), 0, (hipStream_t)stream, a, o);
    else
        hipLaunchKernelGGL(k_ppo_loss_step, dim3(nb), dim3(64), 0, (hipStream_t)stream, a, o);
    if (stats)  // (stats = dstd = NULL: pmlp_reduce_slabs_step finishes the loss)
        hipLaunchKernelGGL(k_ppo_loss_step_final, dim3(3 + A), dim3(64), 0, (hipStream_t)stream, a, partial, nb,
                           stats, dstd);
    PMLP_CHECK_LAUNCH("pmlp_ppo_loss_step");
    return 0;
}

PMLP_API int pmlp_ppo_loss_step(const float* mu, const float* stdv, const float* value, const float* actions,
                                const float* old_logp, const float* old_mu, const float* old_sigma, const float* adv,
                                const float* ret, const float* target, const int64_t* rows, int32_t M, int32_t A,
                                float clip, int32_t clipped_value, float vcoef, float ecoef, float* partial,
                                float* stats, float* dstd, pmlp_bf16* dmu, pmlp_bf16* dmu_t, int32_t Ap,
                                pmlp_bf16* dvalue, pmlp_bf16* dvalue_t, int32_t Vp, void* stream) {
    LossArgs a;
    if (int e = loss_args(a, mu, stdv, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, rows, M, A, clip,
                          clipped_value, vcoef, ecoef))
        return e;
    if (!partial || (!stats != !dstd) || !dmu || !dvalue || Ap < A || Vp < 1)
        return fail(-1, "pmlp_ppo_loss_step: null output or padded width too small");
    LossStepOut o{partial, (bf16*)dmu, (bf16*)dmu_t, (bf16*)dvalue, (bf16*)dvalue_t, Ap, Vp, nullptr, nullptr};
    return loss_step_launch(a, o, M, A, Ap, partial, stats, dstd, stream);
}

PMLP_API int32_t pmlp_mlp_forward_ppo_loss_parts(int32_t M, int32_t A) {
    return (M >= 96 * 192 && A > 0 && A % 4 == 0 && A <= 16) ? ((M + 95) / 96) * (3 + A) : 0;
}

PMLP_API int pmlp_mlp_forward_ppo_loss(const pmlp_mlp_fwd_job* jobs, int32_t M, const float* stdv,
                                       const float* actions, const float* old_logp, const float* old_mu,
                                       const float* old_sigma, const float* adv, const float* ret,
                                       const float* target, const int64_t* rows, int32_t A, float clip,
                                       int32_t clipped_value, float vcoef, float ecoef, float* partial,
                                       pmlp_bf16* dmu, pmlp_bf16* dmu_t, int32_t Ap, pmlp_bf16* dvalue,
                                       pmlp_bf16* dvalue_t, int32_t Vp, void* stream) {
    FmlpJobs fj;
    if (int e = fmlp_pack(2, jobs, M, fj)) return e;
    if (pmlp_mlp_forward_ppo_loss_parts(M, A) <= 0 || Ap > 16 || Ap % 4)
        return fail(-1, "pmlp_mlp_forward_ppo_loss: M >= 18432 rows, A a multiple of 4 <= 16, Ap <= 16");
    if (jobs[0].N[3] != A || jobs[0].ldo != A || jobs[1].N[3] != 1 || jobs[1].ldo != 1)
        return fail(-1, "pmlp_mlp_forward_ppo_loss: job 0 is the actor (A outputs), job 1 the critic (1), dense");
    LossArgs a;
    if (int e = loss_args(a, jobs[0].out, stdv, jobs[1].out, actions, old_logp, old_mu, old_sigma, adv, ret, target,
                          rows, M, A, clip, clipped_value, vcoef, ecoef))
        return e;
    if (!partial || !dmu || !dvalue || Ap < A || Vp < 1)
        return fail(-1, "pmlp_mlp_forward_ppo_loss: null output or padded width too small");
    LossStepOut o{partial, (bf16*)dmu, (bf16*)dmu_t, (bf16*)dvalue, (bf16*)dvalue_t, Ap, Vp, nullptr, nullptr};
    const RollStep none{};
    hipLaunchKernelGGL((k_mlp_fwd<96, false, true>), dim3((M + 95) / 96, 1), dim3(FMLP_THREADS), 0,
                       (hipStream_t)stream, fj, M, none, a, o);
    PMLP_CHECK_LAUNCH("pmlp_mlp_forward_ppo_loss");
    return 0;
}

PMLP_API int pmlp_ppo_loss_step_f32(const float* mu, const float* stdv, const float* value, const float* actions,
                                    const float* old_logp, const float* old_mu, const float* old_sigma,
                                    const float* adv, const float* ret, const float* target, const int64_t* rows,
                                    int32_t M, int32_t A, float clip, int32_t clipped_value, float vcoef, float ecoef,
                                    float* partial, float* stats, float* dstd, float* dmu, float* dvalue,
                                    void* stream) {
    LossArgs a;
    if (int e = loss_args(a, mu, stdv, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, rows, M, A, clip,
                          clipped_value, vcoef, ecoef))
        return e;
    if (!partial || !dmu || !dvalue || (!stats) != (!dstd))
        return fail(-1, "pmlp_ppo_loss_step_f32: null output (stats and dstd both set, or both NULL)");
    if (A % 4 == 0 && ((uintptr_t)dmu & 15)) return fail(-1, "pmlp_ppo_loss_step_f32: dmu 16-byte aligned");
    LossStepOut o{partial, nullptr, nullptr, nullptr, nullptr, 0, 0, dmu, dvalue};
    return loss_step_launch(a, o, M, A, 0, partial, stats, dstd, stream);
}



}  // extern "C"
