/*
 * ppo_mlp.h — C ABI of the hand-written bf16-MFMA kernels behind the rsl_rl
 * actor-critic MLPs and the PPO loss (ActorCritic.act/
 * evaluate in the rollout and the PPO mini-batch forward/backward).
 *
 * The reference runs these as torch nn.Linear/nn.ELU modules and torch loss
 * ops (rsl_rl v1.0.2 ActorCritic, PPO.update; called from OnPolicyRunner.learn,
 * call sites train.py:14, task_registry.py:119).  Here torch.autograd.Functions
 * (rsl_rl/modules/mfma_mlp.py) drive these entry points; parameters and the
 * optimizer stay fp32 torch tensors.
 *
 * Conventions: every pointer is a DEVICE pointer; matrices are row-major with
 * the given leading dimension (in elements; a multiple of 8 for bf16 operands,
 * 16-byte aligned rows); "bf16" is the 16-bit bfloat16 storage type.  Work is
 * enqueued on `stream` (a hipStream_t; NULL = default stream); nothing
 * synchronises the host; nothing allocates, so every call is graph-capturable.
 * Return value: 0, or a negative status with pmlp_last_error() describing it.
 */
#ifndef PPO_MLP_H
#define PPO_MLP_H
#include <stdint.h>

#ifdef __cplusplus
#define PMLP_EXTERN extern "C"
#else
#define PMLP_EXTERN
#endif
#define PMLP_API PMLP_EXTERN __attribute__((visibility("default")))

typedef uint16_t pmlp_bf16;

/* Every entry point takes a batch of independent jobs (the actor and the
 * critic of a step run as one launch each).                                 */
#define PMLP_MAX_JOBS 16
#define PMLP_MAX_GEMM_JOBS 4

/* GEMM epilogues.  All GEMMs are C[M,N] = A[M,K] . B[N,K]^T with A and B bf16
 * and k contiguous (the MFMA operand order).                                 */
enum {
    PMLP_EPI_FWD_HIDDEN = 0, /* y = ELU(acc + bias[n]) -> bf16 y[M,N] and y^T[N,M]           */
    PMLP_EPI_FWD_OUT = 1,    /* out = acc + bias[n]    -> fp32 out[M,N]                      */
    PMLP_EPI_BWD_DX = 2,     /* dz = acc * ELU'(yprev) -> bf16 dz[M,N] and dz^T[N,M]          */
    PMLP_EPI_PARTIAL = 3,    /* split-K slab s: fp32 slab[s][M,N] over k in [s*ks, (s+1)*ks)  */
    PMLP_EPI_PARTIAL_TN = 4  /* PARTIAL with A[K,M] (lda) and B[K,N] (ldb), m / n contiguous:
                                the weight gradient dz^T y read from the row-major activations */
};

PMLP_API const char* pmlp_last_error(void);

/* fp32 x[M,K] (ld ldx) -> bf16 y[M,Kp] (ld Kp; columns K..Kp-1 zero) and/or
 * y^T[Kp,ldyt] (rows K..Kp-1 and columns M..ldyt-1 zero); y or yt may be NULL.
 * one_col > 0: column one_col of y (< Kp) is 1.0 instead (the ones column that
 * makes a weight-gradient GEMM's extra output column the bias gradient).
 * rows (optional, int64[M]): output row m is input row rows[m] (the PPO
 * mini-batch gather of RolloutStorage.mini_batch_generator fused in).
 * Used for observations, output gradients and weights (W and W^T).          */
typedef struct {
    const float* x;
    pmlp_bf16* y;
    pmlp_bf16* yt;
    const int64_t* rows;
    int32_t M, K, ldx, Kp, ldyt, one_col;
} pmlp_convert_job;
PMLP_API int pmlp_convert(int32_t njobs, const pmlp_convert_job* jobs, void* stream);

/* C = A . B^T with epilogue `epi` (see enum).  A: [M,K] (lda), B: [N,K] (ldb).
 *   FWD_HIDDEN: bias[N]; cb[M,N] (ldcb) and/or ct[N,M] (ldct): either may be NULL
 *   FWD_OUT:    bias[N]; cf[M,N] (ldcf)
 *   BWD_DX:     yprev[M,N] bf16 (ldyp) = the ELU output the gradient flows through;
 *               cb/ct as FWD_HIDDEN
 *   PARTIAL:    cf = slab base, slab s at cf + s*M*ldcf; ksplit = k per slab
 *               (multiple of 32); every job must give the same ceil(K/ksplit)
 *   PARTIAL_TN: as PARTIAL with A[K,M], B[K,N] (lda >= ceil8(M), ldb >= ceil8(N)) */
typedef struct {
    const pmlp_bf16* A;
    const pmlp_bf16* B;
    const float* bias;
    const pmlp_bf16* yprev;
    float* cf;
    pmlp_bf16* cb;
    pmlp_bf16* ct;
    int32_t lda, ldb, ldyp, ldcf, ldcb, ldct;
    int32_t M, N, K;
    /* Optional operand forms (NULL / 0: the defaults above; every job of a call alike):
     *  af (FWD_HIDDEN, FWD_OUT): A is fp32 af[rows[m]][k] (ld ldaf, a multiple of 4; rows
     *      NULL = row m; columns >= kaf read as 0) converted to bf16 on load -- the mini-batch
     *      gather and conversion of the observations inside the first layer's GEMM; A is
     *      unused.  xa (optional): the converted bf16 rows are also stored to xa[M, ldxa]
     *      (the weight gradient's operand).
     *  b_kn (BWD_DX): B is given as [K,N] (ldb >= N, n contiguous): the layer's weight
     *      W[out,in] itself, read through transposed LDS reads (no W^T copy).
     *  sum_col (PARTIAL_TN, > 0): slab column sum_col (N <= sum_col < ldcf) also receives
     *      sum_k A[k,m], the product with a column of ones: the bias gradient, without
     *      the extra (mostly empty) column tile a ones column in B would cost.          */
    const float* af;
    const int64_t* rows;
    pmlp_bf16* xa;
    int32_t ldaf, kaf, ldxa, b_kn, sum_col;
} pmlp_gemm_job;
PMLP_API int pmlp_gemm(int32_t epi, int32_t njobs, const pmlp_gemm_job* jobs, int32_t ksplit, void* stream);
/* A layer's backward in one launch: the PARTIAL_TN weight-gradient batch jobs_w (ksplit as
 * pmlp_gemm) and the BWD_DX input-gradient batch jobs_x (B given [K,N]) read the same output
 * gradient and nothing the other writes, so both run in one grid where their tile
 * configurations share a block size (else as two pmlp_gemm launches).  Results are bitwise
 * those of the two launches. */
PMLP_API int pmlp_gemm_pair(int32_t njobs_w, const pmlp_gemm_job* jobs_w, int32_t ksplit, int32_t njobs_x,
                            const pmlp_gemm_job* jobs_x, void* stream);
/* operand staging of pmlp_gemm's k-loop: 1 (default; env PMLP_GLDS) = LDS-DMA into two LDS buffers,
 * one barrier per k-tile, wherever the shapes allow (whole 64-deep k-tiles); 0 = register staging.
 * Both compute the same MFMA chain (bitwise equal).  Returns the previous setting. */
PMLP_API int pmlp_set_gemm_staging(int32_t glds);

/* out[i] = sum_s slab[s*stride + i], i < n (fp32): the split-K combine.
 * bias_out (optional): the slab is [n/cols_in, cols_in]; columns < cols_out go to
 * out[n/cols_in, cols_out] and column cols_out to bias_out (the weight gradient's
 * extra ones-row column = the bias gradient); later columns are dropped.     */
typedef struct {
    const float* slab;
    float* out;
    float* bias_out;
    int64_t stride, n;
    int32_t nslabs, cols_in, cols_out;
} pmlp_reduce_job;
PMLP_API int pmlp_reduce_slabs(int32_t njobs, const pmlp_reduce_job* jobs, void* stream);
/* pmlp_reduce_slabs plus the end of the PPO loss and, at world size 1, pmlp_opt_prepare, in
 * ONE launch (FusedPPOStep): the loss step ran with stats = dstd = NULL (partials only); one
 * more workgroup sums its partials into stats [surrogate, value, kl, entropy] and the std
 * gradient dstd (bitwise what pmlp_ppo_loss_step writes).  norm_partial (optional): every
 * workgroup writes the sum of squares of the gradient elements it produced, the std
 * gradient's included, and the loss workgroup advances step, accumulates acc and adapts lr
 * as pmlp_opt_prepare at scale 1; nparts (out) is the count for pmlp_adam_mirror_n.  The
 * jobs' outputs and dstd must be the whole gradient for the norm to be clip_grad_norm_'s. */
typedef struct pmlp_reduce_step {
    const float* loss_partial;  /* pmlp_ppo_loss_step's partial buffer             */
    int32_t loss_blocks;        /* pmlp_ppo_loss_step_parts(M, A) / (3 + A)         */
    int32_t A, M;
    float ecoef;
    const float* stdv;
    float *stats, *dstd;
    float* norm_partial;        /* optional: nparts (in) floats                      */
    float *step, *lr, *acc;
    float desired_kl;
    int32_t adaptive;
    int32_t nparts;             /* in: norm_partial's capacity (floats; checked before the launch,
                                   -1 when short); out: the partials written           */
} pmlp_reduce_step;
PMLP_API int pmlp_reduce_slabs_step(int32_t njobs, const pmlp_reduce_job* jobs, pmlp_reduce_step* r, void* stream);
/* The norm partials pmlp_reduce_slabs_step writes for these jobs (its nparts after the call;
 * the capacity its norm_partial buffer needs), or -1 for malformed jobs. */
PMLP_API int64_t pmlp_reduce_slabs_parts(int32_t njobs, const pmlp_reduce_job* jobs);

/* out[r] = sum_c x[r*ld + c], c < cols (bf16 in, fp32 sum): bias gradients. */
typedef struct {
    const pmlp_bf16* x;
    float* out;
    int32_t rows, cols, ld;
} pmlp_rowsum_job;
PMLP_API int pmlp_rowsum(int32_t njobs, const pmlp_rowsum_job* jobs, void* stream);

/* Fused PPO loss of rsl_rl v1.0.2 PPO.update for a diagonal Gaussian policy
 * (ratio, clipped surrogate, optionally clipped value loss, entropy bonus,
 * and the KL the adaptive learning rate reads).  Inputs fp32, row-major:
 * mu/actions/old_mu/old_sigma [M,A], stdv [A], value/old_logp/adv/ret/target [M].
 * rows (optional, int64[M]): the rollout inputs actions, old_logp, old_mu,
 * old_sigma, adv, ret and target are read at row rows[i] (flat T*N storage);
 * mu and value are the mini-batch's own rows.
 * fwd: loss[1]; stats[4] = {surrogate_loss, value_loss, kl_mean, entropy_mean};
 *      partial = scratch of 4*pmlp_ppo_loss_blocks(M) floats.
 * bwd: gout = device scalar d(total)/d(loss); dmu [M,A], dvalue [M], dstd [A];
 *      partial_std = scratch of A*pmlp_ppo_loss_blocks(M) floats.          */
PMLP_API int32_t pmlp_ppo_loss_blocks(int32_t M);
PMLP_API int pmlp_ppo_loss_fwd(const float* mu, const float* stdv, const float* value, const float* actions,
                               const float* old_logp, const float* old_mu, const float* old_sigma, const float* adv,
                               const float* ret, const float* target, const int64_t* rows, int32_t M, int32_t A,
                               float clip, int32_t clipped_value, float vcoef, float ecoef, float* partial, float* loss,
                               float* stats, void* stream);
PMLP_API int pmlp_ppo_loss_bwd(const float* mu, const float* stdv, const float* value, const float* actions,
                               const float* old_logp, const float* old_mu, const float* old_sigma, const float* adv,
                               const float* ret, const float* target, const int64_t* rows, int32_t M, int32_t A,
                               float clip, int32_t clipped_value, float vcoef, float ecoef, const float* gout,
                               float* dmu, float* dvalue, float* partial_std, float* dstd, void* stream);

/* One optimizer step over FLAT fp32 parameter / gradient / moment buffers of n
 * entries (nn.utils.clip_grad_norm_ then torch.optim.Adam, amsgrad off, no
 * weight decay; rsl_rl v1.0.2 PPO.update).  grad_scale multiplies the gradient
 * first (1/world_size after an all-reduce sum).
 * pmlp_opt_prepare: partial[pmlp_opt_parts()] = squared-norm partials; step[0] += 1;
 *   with stats = [surrogate, value, kl, entropy] (scaled by grad_scale too):
 *   acc[0] += value loss, acc[1] += surrogate loss (acc may be NULL), and when
 *   adaptive != 0 the KL rule of rsl_rl's adaptive schedule updates lr[0].
 * pmlp_adam: clip coefficient min(1, max_norm/(|g|+1e-6)) (max_norm <= 0: no
 *   clipping), then Adam with bias corrections from step[0] and lr[0].        */
PMLP_API int32_t pmlp_opt_parts(void);
PMLP_API int pmlp_opt_prepare(const float* grad, int64_t n, float grad_scale, float* partial, float* step,
                              const float* stats, float* lr, float* acc, float desired_kl, int32_t adaptive,
                              void* stream);
PMLP_API int pmlp_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                       float grad_scale, const float* partial, const float* step, const float* lr, float max_norm,
                       float beta1, float beta2, float eps, void* stream);
/* For a torch-optimizer step on the fused loss (the recurrent policy): from stats = [surrogate,
 * value, kl, entropy], acc[0] += value loss, acc[1] += surrogate loss (acc may be NULL) and, when
 * adaptive != 0, the KL rule of rsl_rl's adaptive schedule updates lr[0]; one launch.          */
PMLP_API int pmlp_loss_bookkeeping(const float* stats, float* lr, float* acc, float desired_kl, int32_t adaptive,
                                   void* stream);
/* pmlp_adam that also refreshes bf16 copies of the updated weights (the GEMM operands):
 * param[offset + r*cols + c] -> dst[r*ld + c] for every mirror job, so no conversion launch
 * precedes the next forward.  At most PMLP_MAX_MIRROR jobs, disjoint parameter ranges.
 * frag (optional, ld a multiple of 16): the same weight also into the fragment-packed
 * layout pmlp_mlp_forward reads (pmlp_mlp_fwd_job.Wf): element (r, c) at
 *   ((((r / 32) * (ld / 16) + c / 16) * 64 + r % 32 + 32 * ((c / 8) % 2)) * 8 + c % 8
 * (ceil(rows / 32) * 32 * ld elements; the padding entries are the caller's zeros).      */
#define PMLP_MAX_MIRROR 8
typedef struct {
    int64_t offset;
    int32_t rows, cols, ld;
    pmlp_bf16* dst;
    pmlp_bf16* frag;
} pmlp_mirror_job;
PMLP_API int pmlp_adam_mirror(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                              float grad_scale, const float* partial, const float* step, const float* lr,
                              float max_norm, float beta1, float beta2, float eps, int32_t nmirror,
                              const pmlp_mirror_job* mirror, void* stream);
/* pmlp_adam_mirror with the norm partials' count given (pmlp_reduce_slabs_step's nparts). */
PMLP_API int pmlp_adam_mirror_n(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                float grad_scale, const float* partial, int32_t nparts, const float* step,
                                const float* lr, float max_norm, float beta1, float beta2, float eps, int32_t nmirror,
                                const pmlp_mirror_job* mirror, void* stream);

/* RolloutStorage.compute_returns (rsl_rl v1.0.2): GAE(gamma, lam) over [T,N]
 * rewards/dones(bool bytes)/values with last_values[N], writing returns and
 * advantages, then advantages normalised by their mean and unbiased std.
 * partial: 2 * pmlp_gae_parts(N) doubles of scratch.                        */
PMLP_API int32_t pmlp_gae_parts(int32_t num_envs);
PMLP_API int pmlp_gae(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
                      float* returns, float* advantages, int32_t T, int32_t N, float gamma, float lam,
                      double* partial, void* stream);
/* The same in two halves for data-parallel training (rsl_rl v1.0.2 normalises with the
 * statistics of the whole batch; across ranks that is the all-reduced moments):
 * pmlp_gae_local writes returns/advantages and this rank's moments[3] = {sum, sum of
 * squares, count} (doubles); the caller all-reduces moments (sum) and pmlp_adv_normalize
 * normalises the n local advantages with the global mean and unbiased std. */
PMLP_API int pmlp_gae_local(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
                            float* returns, float* advantages, int32_t T, int32_t N, float gamma, float lam,
                            double* partial, double* moments, void* stream);
PMLP_API int pmlp_adv_normalize(float* advantages, int64_t n, const double* moments, void* stream);

/* Rollout step of PPO (rsl_rl v1.0.2 PPO.act + RolloutStorage.add_transitions):
 * from the policy mean mu[N,A], std[A] and value[N] (the MLP outputs) draw
 * actions = mu + std * n, n ~ N(0,1) from Philox4x32-10 keyed (seed; draw[0],
 * row, pair) with Box-Muller; write actions_out[N,A] and storage row t:
 * actions, log_prob[N] (sum over A of the Gaussian log-density), mu, sigma
 * (std broadcast), value, observations obs[N,O] (and critic observations
 * cobs[N,CO] when st_cobs != NULL).
 * pmlp_store_step (PPO.process_env_step): st_rewards = rewards + gamma *
 * (st_value * time_outs) (time_outs may be NULL: no bootstrap), st_dones =
 * dones (bool bytes), then draw[0] += 1.                                     */
PMLP_API int pmlp_act(const float* mu, const float* stdv, const float* value, const float* obs, const float* cobs,
                      int32_t N, int32_t A, int32_t O, int32_t CO, const int64_t* draw, uint64_t seed,
                      float* actions_out, float* st_actions, float* st_logp, float* st_mu, float* st_sigma,
                      float* st_value, float* st_obs, float* st_cobs, void* stream);
PMLP_API int pmlp_store_step(const float* rewards, const uint8_t* dones, const uint8_t* time_outs,
                             const float* st_value, float* st_rewards, uint8_t* st_dones, int32_t N, float gamma,
                             int64_t* draw, void* stream);
/* The extras of a control step the env left to the rollout (leggedsim lgs_step_deferred,
 * include/leggedsim.h; the reference's reset_idx extras and push bookkeeping,
 * legged_robot.py:540-555, 742-768): the work of lgs_step's k_step_extras, done by the launch
 * that consumes the step (pmlp_rollout_forward's deferred store, pmlp_store_step_env) on its own
 * env rows and, in its first workgroup, once.  any = acc[nsum] > 0 (some env reset this step);
 * slot = pushed[2] & 1 (the parity of the step's key):
 *   per env i: carry[i] = time_out[i] when any, and the store's bootstrap reads that value;
 *              last_root_vel[i][0:2] = vsim[i] when push and no env was pushed (!pushed[slot]);
 *   once:      ep_means[k] = ep_snapshot[k] = acc[k] / max(acc[nsum], 1) / ep_len_s when any;
 *              acc_next[0..nsum] = 0; pushed[slot ^ 1] = 0; *step_counter += 1.
 * acc is read by every workgroup, so the launch zeroes acc_next (the next step's slot), never acc.
 * acc == NULL: no extras.                                                                     */
typedef struct {
    const float* acc;            /* [nsum + 1] this step's episode sums, then the reset count */
    float* acc_next;             /* [nsum + 1] the next step's slot                           */
    int32_t nsum;
    float ep_len_s;              /* max_episode_length_s                                       */
    float* ep_means;             /* [nsum] or NULL                                             */
    float* ep_snapshot;          /* [nsum] or NULL                                             */
    const uint8_t* time_out;     /* [N] this step's time-outs                                  */
    uint8_t* carry;              /* [N] extras["time_outs"], or NULL                           */
    float* last_root_vel;        /* [N, 6] or NULL                                             */
    const float* vsim;           /* [N, 2]                                                     */
    uint32_t* pushed;            /* [3] (lgs_get_push_state)                                   */
    int32_t push;                /* push_robots                                                */
    int64_t* step_counter;       /* or NULL                                                    */
} pmlp_env_extras;
/* pmlp_store_step_reset with a deferred step's extras (ex may be NULL) in the same launch; the
 * bootstrap reads the carried time-outs after the launch's own update of them (time_outs is
 * then ex->carry). */
PMLP_API int pmlp_store_step_env(const float* rewards, const uint8_t* dones, const uint8_t* time_outs,
                                 const float* st_value, float* st_rewards, uint8_t* st_dones, int32_t N, float gamma,
                                 int64_t* draw, int32_t nstates, float* const* states, int32_t H,
                                 const pmlp_env_extras* ex, void* stream);
/* pmlp_store_step plus ActorCriticRecurrent.reset(dones) (each memory's Memory.reset:
 * hidden_state.masked_fill_(dones, 0)) in the same launch: the nstates (<= PMLP_MAX_MEM_STATES)
 * state buffers [N, H] (H a multiple of 4, 16-byte aligned) get zero rows for the done envs. */
#define PMLP_MAX_MEM_STATES 4
PMLP_API int pmlp_store_step_reset(const float* rewards, const uint8_t* dones, const uint8_t* time_outs,
                                   const float* st_value, float* st_rewards, uint8_t* st_dones, int32_t N, float gamma,
                                   int64_t* draw, int32_t nstates, float* const* states, int32_t H, void* stream);
/* The update's mini-batch permutation (RolloutStorage.mini_batch_generator's
 * torch.randperm(num_mini_batches * mini_batch_size)): out[i], i < n, a keyed pseudo-random
 * permutation of [0, n) (4-round alternating Feistel on the ceil(log2 n)-bit domain, Philox
 * round function, cycle walking), no sort. */
PMLP_API int pmlp_permutation(int64_t* out, int64_t n, uint64_t seed, void* stream);

/* The whole forward of 4-layer Linear/ELU MLPs (rsl_rl's actor and critic) in ONE launch
 * (PPO.act's policy inference, the update's forward): per job
 *   y0 = ELU(x W0^T + b0), y1 = ELU(y0 W1^T + b1), y2 = ELU(y1 W2^T + b2), out = y2 W3^T + b3
 * with x fp32 (row m = x[rows ? rows[m] : m], columns >= kx read as 0, converted to bf16),
 * bf16 W[l] = [N[l], K_l] (K_0 = K0, K_l = N[l-1]), fp32 b and out; the activations stay on
 * chip (LDS) between layers.  Optional stores: xa = the bf16 input rows [M, K0] and y[l] = the
 * bf16 hidden outputs (the backward's operands).  Bitwise equal to the per-layer pmlp_gemm
 * forward (FWD_HIDDEN x3 with the af operand form, FWD_OUT).  Limits: K0 a multiple of 16,
 * <= 64; N0, N2 <= 512 and N1 <= 256, multiples of 32; N3 <= 32; 1..2 jobs.              */
typedef struct {
    const float* x;
    const int64_t* rows;
    int32_t ldx, kx;
    pmlp_bf16* xa;
    int32_t ldxa;
    const pmlp_bf16* W[4];
    const float* b[4];
    int32_t N[4];
    int32_t K0;
    pmlp_bf16* y[3];
    int32_t ldy[3];
    float* out;
    int32_t ldo;
    /* optional: W[l] fragment-packed (the pmlp_mirror_job.frag layout with ld = K_l): each
     * wave's weight-fragment load is then 1 KB contiguous instead of 32 row pieces */
    const pmlp_bf16* Wf[4];
} pmlp_mlp_fwd_job;
PMLP_API int pmlp_mlp_forward(int32_t njobs, const pmlp_mlp_fwd_job* jobs, int32_t M, void* stream);

/* One env step's policy work of the fused rollout in the forward launch (pmlp_mlp_forward
 * of job 0 = the actor [N, A] means and job 1 = the critic [N, 1] values, N = M envs):
 *  - PPO.act + RolloutStorage.add_transitions (pmlp_act's arithmetic): a ~ N(mu, std) with
 *    Philox draw counter draw[parity], log-prob, and the storage rows (actions, log-prob, mu,
 *    sigma, value, observations); then draw[parity ^ 1] = draw[parity] + 1 (the next step
 *    reads that one: the counters alternate with the step parity, so no launch reads and
 *    advances the same counter);
 *  - optionally the PREVIOUS env step's PPO.process_env_step (pmlp_store_step without the
 *    draw advance), deferred into this launch: st_rewards = rewards + gamma * (prev_value *
 *    time_outs), st_dones = dones (rewards == NULL: none), with that step's deferred env extras
 *    (pmlp_env_extras) when the env left them.  The caller issues the last step's with
 *    pmlp_store_step_env (draw = NULL) before anything reads the storage.
 * One launch per env step instead of three (forward, pmlp_act, pmlp_store_step).          */
typedef struct {
    const float* stdv;                  /* [A]                                              */
    const float* obs;                   /* [N, O] (storage observations)                    */
    const float* cobs;                  /* [N, CO] or NULL (no privileged storage)          */
    int32_t O, CO, A;                   /* A <= 16                                          */
    float *actions_out, *st_actions, *st_logp, *st_mu, *st_sigma, *st_value, *st_obs, *st_cobs;
    int64_t* draw;                      /* [2]                                              */
    int32_t parity;
    uint64_t seed;
    const float* rewards;               /* deferred store of the previous step, or NULL     */
    const uint8_t* dones;
    const uint8_t* time_outs;           /* or NULL: no bootstrap                            */
    const float* prev_value;
    float* st_rewards;
    uint8_t* st_dones;
    float gamma;
    pmlp_env_extras extras;             /* the previous step's deferred extras (acc NULL: none);
                                           they ride with its deferred store (rewards != NULL) */
} pmlp_rollout_step;
PMLP_API int pmlp_rollout_forward(const pmlp_mlp_fwd_job* jobs, int32_t N, const pmlp_rollout_step* rs,
                                  void* stream);

/* ---- recurrent heads (the fused recurrent optimizer step, rsl_rl/algorithms/fused_recurrent.py):
 * the MLP heads of ActorCriticRecurrent on the LSTM output h [M, H] (rsl_rl
 * actor_critic_recurrent.py: the actor / critic Sequential(Linear(H, N0), ELU, Linear(N0, N1))),
 * fp32, up to two nets per launch.  H in {32, 64, 128}; N0 <= 32 a multiple of 8; N1 <= 16.
 * pmlp_heads_forward:  y0 = elu(W0 h + b0) [M, N0], out = W1 y0 + b1 [M, N1]
 * pmlp_heads_backward: from dout [M, N1] (the loss gradient): dh = W0^T ((W1^T dout) * elu'(y0))
 *   [M, H] (the LSTM's output gradient, elu' from the output as torch), and the partial
 *   weight gradients of every block of 128 rows, slab[b] = [dW0 | db0 | dW1 | db1]
 *   (N0 H + N0 + N1 N0 + N1 floats per row of the slab, pmlp_heads_blocks(M) rows): summed
 *   by pmlp_reduce_slabs into the flat gradient (the Sequential's parameter order).
 * Weights row-major as nn.Linear ([out, in]); h, W0, dh and slab 16-byte aligned.        */
typedef struct {
    const float *h, *W0, *b0, *W1, *b1;
    float *y0, *out;
    const float* dout;
    float *dh, *slab;
    int32_t N0, N1;
} pmlp_head_job;
PMLP_API int32_t pmlp_heads_blocks(int32_t M);
PMLP_API int pmlp_heads_forward(int32_t njobs, const pmlp_head_job* jobs, int32_t M, int32_t H, void* stream);
PMLP_API int pmlp_heads_backward(int32_t njobs, const pmlp_head_job* jobs, int32_t M, int32_t H, void* stream);
/* pmlp_heads_forward of the actor (jobs[0], N1 = A <= 16) and the critic (jobs[1], N1 = 1)
 * with pmlp_act in the same launch (the recurrent rollout's policy step): each workgroup
 * samples its rows' actions from the mu it just computed (pmlp_act's Philox counters and
 * arithmetic: the same bits) and writes the storage rows; the critic's workgroups write the
 * values and privileged rows.  The draw counter is read, not advanced (the store advances it). */
typedef struct {
    const float *stdv, *obs, *cobs;
    int32_t O, CO, A;
    const int64_t* draw;
    uint64_t seed;
    float *actions_out, *st_actions, *st_logp, *st_mu, *st_sigma, *st_value, *st_obs, *st_cobs;
} pmlp_head_act;
PMLP_API int pmlp_heads_forward_act(const pmlp_head_job* jobs, int32_t M, int32_t H, const pmlp_head_act* act,
                                    void* stream);

/* The same loss for the fused optimizer step (gradient of the loss itself):
 * one pass writes the output gradients straight into the MLP backward's bf16
 * operands, dmu[M,Ap] + dmu_t[Ap,M] and dvalue[M,Vp] + dvalue_t[Vp,M]
 * (padding columns/rows written as zero; dmu_t / dvalue_t may be NULL), dstd[A] (incl. the entropy term) and
 * stats[4] = {surrogate_loss, value_loss, kl_mean, entropy_mean}.
 * partial: pmlp_ppo_loss_step_parts(M, A) floats of scratch.  stats = dstd = NULL: only the
 * per-block partials are written, and pmlp_reduce_slabs_step finishes the loss.        */
PMLP_API int32_t pmlp_ppo_loss_step_parts(int32_t M, int32_t A);
PMLP_API int pmlp_ppo_loss_step(const float* mu, const float* stdv, const float* value, const float* actions,
                                const float* old_logp, const float* old_mu, const float* old_sigma, const float* adv,
                                const float* ret, const float* target, const int64_t* rows, int32_t M, int32_t A,
                                float clip, int32_t clipped_value, float vcoef, float ecoef, float* partial,
                                float* stats, float* dstd, pmlp_bf16* dmu, pmlp_bf16* dmu_t, int32_t Ap,
                                pmlp_bf16* dvalue, pmlp_bf16* dvalue_t, int32_t Vp, void* stream);
/* The update's forward and this loss step in ONE launch (rsl_rl PPO.update: evaluate + the
 * loss + its backward to the output layer): pmlp_mlp_forward of job 0 = the actor (A outputs,
 * ldo = A) and job 1 = the critic (1 output, ldo = 1), then, in the same workgroup on its 96
 * rows, pmlp_ppo_loss_step's per-row arithmetic and outputs on mu = jobs[0].out, value =
 * jobs[1].out, with the per-workgroup partials only (the folded form: pmlp_reduce_slabs_step
 * finishes the loss over pmlp_mlp_forward_ppo_loss_parts(M, A) / (3 + A) partial rows; the
 * partials sum 96-row groups, so the logged losses and the std gradient round differently
 * from the 64-row groups of pmlp_ppo_loss_step).  Applies when
 * pmlp_mlp_forward_ppo_loss_parts(M, A) > 0 (M >= 18432, A a multiple of 4 <= 16) and
 * Ap <= 16, a multiple of 4; replaces PPO.update's separate forward and loss launches.   */
PMLP_API int32_t pmlp_mlp_forward_ppo_loss_parts(int32_t M, int32_t A);
PMLP_API int pmlp_mlp_forward_ppo_loss(const pmlp_mlp_fwd_job* jobs, int32_t M, const float* stdv,
                                       const float* actions, const float* old_logp, const float* old_mu,
                                       const float* old_sigma, const float* adv, const float* ret,
                                       const float* target, const int64_t* rows, int32_t A, float clip,
                                       int32_t clipped_value, float vcoef, float ecoef, float* partial,
                                       pmlp_bf16* dmu, pmlp_bf16* dmu_t, int32_t Ap, pmlp_bf16* dvalue,
                                       pmlp_bf16* dvalue_t, int32_t Vp, void* stream);
/* The same step with fp32 output gradients dmu [M, A] (16-byte aligned when A % 4 == 0) and
 * dvalue [M] (the recurrent heads' fp32 backward, pmlp_heads_backward).  stats = dstd = NULL:
 * partials only, pmlp_reduce_slabs_step finishes the loss.                             */
PMLP_API int pmlp_ppo_loss_step_f32(const float* mu, const float* stdv, const float* value, const float* actions,
                                    const float* old_logp, const float* old_mu, const float* old_sigma,
                                    const float* adv, const float* ret, const float* target, const int64_t* rows,
                                    int32_t M, int32_t A, float clip, int32_t clipped_value, float vcoef, float ecoef,
                                    float* partial, float* stats, float* dstd, float* dmu, float* dvalue,
                                    void* stream);

/* ---- recurrent memory: rsl_rl v1.0.2 Memory (one-layer LSTM, gate order i, f, g, o)
 * for ActorCriticRecurrent (the G1 / H1 / H1_2 policies: g1_config.py:92-108,
 * h1_config.py:103-118, h1_2_config.py:115-130).  Dense form of the padded-trajectory
 * update: the [T, B] reset mask zeroes (h, c) before step t when the env was done at t-1.
 *  gx      [T,B,4H]  x W_ih^T + b_ih + b_hh (one GEMM over T*B rows, by the caller)
 *  whh     [4H,H]    weight_hh_l0 (16-byte aligned)
 *  h0, c0  [B,H]     state before step 0 (NULL: zeros); reset [T,B] bytes or NULL
 *  h_out, c_out [T,B,H], gact [T,B,4H] (activated gates): outputs, each may be NULL
 *  h_last, c_last [B,H]: state after step T-1 (may alias h0/c0: rollout mode, T = 1)
 * pmlp_lstm_bwd: dh_out [T,B,H] -> dgx [T,B,4H] (gradient of the gate pre-activations);
 * the caller forms dW_ih = dgx^T x, dW_hh = dgx^T h_prev, db = sum(dgx).
 * H = 32, 64 or 128 (pmlp_lstm_supported). */
PMLP_API const char* pmlp_lstm_last_error(void);
PMLP_API int pmlp_lstm_supported(int32_t hidden);
PMLP_API int pmlp_lstm_fwd(int32_t T, int32_t B, int32_t H, const float* gx, const float* whh, const float* h0,
                           const float* c0, const uint8_t* reset, float* h_out, float* c_out, float* gact,
                           float* h_last, float* c_last, void* stream);
/* pmlp_lstm_fwd with the input projection fused in: x [T,B,I] (I <= 64), wih [4H,I], bih / bhh [4H]
 * (either may be NULL) instead of gx; xh (optional) [T,B,I+H+1] receives [x | h_prev | 1] per row
 * (h_prev = the state the step starts from, after a reset): the operand of the weight gradients
 * dW_ih, dW_hh and the bias (dgx^T xh). */
PMLP_API int pmlp_lstm_fwd_x(int32_t T, int32_t B, int32_t H, int32_t I, const float* x, const float* wih,
                             const float* bih, const float* bhh, const float* whh, const float* h0, const float* c0,
                             const uint8_t* reset, float* h_out, float* c_out, float* gact, float* h_last,
                             float* c_last, float* xh, void* stream);
/* One rollout step in place (T = 1): h, c [B,H] are read and overwritten; h_save / c_save
 * (optional) receive the state the step started from (the rollout storage's saved hidden
 * state, RolloutStorage._save_hidden_states). */
PMLP_API int pmlp_lstm_step(int32_t B, int32_t H, const float* gx, const float* whh, float* h, float* c,
                            float* h_save, float* c_save, void* stream);
PMLP_API int pmlp_lstm_bwd(int32_t T, int32_t B, int32_t H, const float* whh, const float* c0, const uint8_t* reset,
                           const float* c_out, const float* gact, const float* dh_out, float* dgx, void* stream);
/* The update's dense sequences on the matrix cores (hidden 64, input <= 64): the forward of
 * pmlp_lstm_fwd_x and the backward of pmlp_lstm_bwd with the per-step products
 * [x_t | h_{t-1}] . [W_ih | W_hh]^T and dG . W_hh as bf16 MFMAs (fp32 accumulation, the cell
 * state and every output fp32).  Same outputs and layouts as the fp32 kernels, to bf16 operand
 * rounding; the rollout's step (pmlp_lstm_step) stays fp32. */
PMLP_API int pmlp_lstm_fwd_mfma(int32_t T, int32_t B, int32_t H, int32_t I, const float* x, const float* wih,
                                const float* bih, const float* bhh, const float* whh, const float* h0, const float* c0,
                                const uint8_t* reset, float* h_out, float* c_out, float* gact, float* xh, void* stream);
PMLP_API int pmlp_lstm_bwd_mfma(int32_t T, int32_t B, int32_t H, const float* whh, const float* c0,
                                const uint8_t* reset, const float* c_out, const float* gact, const float* dh_out,
                                float* dgx, void* stream);
/* pmlp_lstm_bwd_mfma plus the three weight gradients (the fused recurrent step): per
 * workgroup of 16 envs (pmlp_lstm_bwd_dw_blocks(B) of them) the partial sums over its envs
 * and the T steps of dG^T [x | h_prev | 1] (xh: the rows pmlp_lstm_fwd_mfma wrote), as one
 * slab row [dW_ih (4H x I) | dW_hh (4H x H) | db (4H)] of 4H (I + H + 1) floats in torch's
 * row order (summed over the rows by pmlp_reduce_slabs; db is the gradient of b_ih and b_hh).
 * The gate gradients themselves are not written.  H = 64, I + H + 1 <= 128.            */
/* One rollout step of a hidden-64 memory on the matrix cores: the arithmetic of
 * pmlp_lstm_fwd_mfma at T = 1 (so the rollout's log-probabilities come from the same
 * numbers the update recomputes), input projection inside, h / c [B, 64] updated in place;
 * h_save / c_save (both or neither) receive the state the step starts from.   I <= 64.  */
PMLP_API int pmlp_lstm_step_mfma(int32_t B, int32_t H, int32_t I, const float* x, const float* wih, const float* bih,
                                 const float* bhh, const float* whh, float* h, float* c, float* h_save, float* c_save,
                                 void* stream);
PMLP_API int32_t pmlp_lstm_bwd_dw_blocks(int32_t B);
PMLP_API int pmlp_lstm_bwd_dw_mfma(int32_t T, int32_t B, int32_t H, int32_t I, const float* whh, const float* c0,
                                   const uint8_t* reset, const float* c_out, const float* gact, const float* dh_out,
                                   const float* xh, float* slab, void* stream);
/* The actor's and the critic's memory in ONE launch each way (rsl_rl ActorCriticRecurrent's
 * memory_a / memory_c: independent sequences over the same [T, B] mini-batch and reset mask;
 * one 2,048-env mini-batch is 128 workgroups, half of the 256 CUs).  Per job exactly
 * pmlp_lstm_fwd_mfma (x, w_ih, b_ih, b_hh, w_hh, h0, c0 -> h_out, c_out, gact, xh) and
 * pmlp_lstm_bwd_dw_mfma (w_hh, c0, c_out, gact, dh_out, xh -> slab).  1 <= njobs <= 2. */
typedef struct pmlp_lstm_job {
    int32_t I;                                   /* input width, 1..63                   */
    const float *x, *w_ih, *b_ih, *b_hh, *w_hh;  /* [T,B,I], torch nn.LSTM parameters   */
    const float *h0, *c0;                        /* [B,64] state the sequence starts from */
    float *h_out, *c_out, *gact, *xh;            /* forward outputs (backward inputs)     */
    const float* dh_out;                         /* backward: gradient of h_out [T,B,64]  */
    float* slab;                                 /* backward: weight-gradient partials    */
    float *h_save, *c_save;                      /* step: the state the step starts from  */
} pmlp_lstm_job;
PMLP_API int pmlp_lstm_fwd_mfma_jobs(int32_t njobs, const pmlp_lstm_job* jobs, int32_t T, int32_t B, int32_t H,
                                     const uint8_t* reset, void* stream);
PMLP_API int pmlp_lstm_bwd_dw_mfma_jobs(int32_t njobs, const pmlp_lstm_job* jobs, int32_t T, int32_t B, int32_t H,
                                        const uint8_t* reset, void* stream);
/* The rollout's memory step of both memories in one launch: per job pmlp_lstm_step_mfma with
 * h = h_out, c = c_out (the state [B,64], updated in place), h_save / c_save optional (both
 * or neither); x, w_ih, b_ih, b_hh, w_hh as above; the other fields are ignored.          */
PMLP_API int pmlp_lstm_step_mfma_jobs(int32_t njobs, const pmlp_lstm_job* jobs, int32_t B, int32_t H, void* stream);

#endif
