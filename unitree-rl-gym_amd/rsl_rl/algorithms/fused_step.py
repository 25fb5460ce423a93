"""One PPO mini-batch optimizer step of the Gaussian MLP actor-critic as ~20
kernel launches, with no autograd and no torch glue (rsl_rl v1.0.2
PPO.update body).

What the reference does per mini-batch:
    gather the rollout rows -> actor/critic forward -> loss -> backward ->
    clip_grad_norm_ -> Adam
What runs here (csrc/ppo_mlp.hip through include/ppo_mlp.h):
    1 convert   observations gathered by the mini-batch index (fused gather)
                + every weight and weight^T to bf16
    L GEMMs     forward, actor and critic sharing every launch
    2 + 2       loss forward (+ final) / backward (+ std gradient); the loss
                reads actions, old log-probs, advantages, ... through the index
    1 convert   output gradients to bf16
    2L-1 GEMMs  weight-gradient slabs and input gradients
    2           slab combine + bias sums, written into the flat gradient
    2           grad-norm partials (+ step/LR/loss bookkeeping) and Adam

Every parameter is a view of ONE flat fp32 buffer (`flat`), every gradient a view
of another (`grad`, whose 4-float tail holds the loss statistics), and Adam's
moments are flat too.  The module's parameters, state_dict and the optimizer's
state_dict keep their reference structure: the Parameters are the same objects
(`.data` re-pointed) and the torch Adam's per-parameter state entries are views
of the flat moments.  With torch.distributed the gradient (and the statistics
tail) is all-reduced as one bucket and averaged inside the kernels.
"""

import ctypes as C
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from rsl_rl.modules import lstm_seq
from rsl_rl.modules import mfma_mlp as mm


def noise_seed():
    """The rollout's policy-noise Philox key: from torch's seeded generator, mixed with
    the data-parallel rank so the ranks (which start from the same torch seed) explore
    with independent noise, as their envs do (seed + rank)."""
    s = int(torch.randint(0, 2 ** 62, (1,)).item())
    if dist.is_available() and dist.is_initialized():
        s ^= (dist.get_rank() * 0x9E3779B97F4A7C15) & (2 ** 62 - 1)
    return s


def _ceil8(n):
    return (n + 7) // 8 * 8


class FusedPPOStep:
    def __init__(self, alg, mini_batch_size):
        ac = alg.actor_critic
        seqs = [ac.actor, ac.critic]
        if not all(mm.supported(s) for s in seqs):
            raise ValueError("fused PPO step: actor/critic must be Linear/ELU MLPs")
        self.lins = [[m for m in s if isinstance(m, nn.Linear)] for s in seqs]
        if len(self.lins[0]) != len(self.lins[1]):
            raise ValueError("fused PPO step: actor and critic must have the same depth")
        if 2 * len(self.lins[0]) > mm.PMLP_MAX_MIRROR:
            # every weight's bf16 copy is one Adam mirror job (include/ppo_mlp.h); a deeper
            # net keeps the autograd update (PPO.init_storage catches this)
            raise ValueError(f"fused PPO step: at most {mm.PMLP_MAX_MIRROR // 2} Linear layers per net")
        params = [p for ls in self.lins for lin in ls for p in (lin.weight, lin.bias)] + [ac.std]
        if sorted(map(id, params)) != sorted(map(id, ac.parameters())):
            raise ValueError("fused PPO step: unexpected parameter set")
        self.alg, self.ac, self.M = alg, ac, int(mini_batch_size)
        if self.M % 8:
            raise ValueError("fused PPO step: mini-batch size must be a multiple of 8")
        dev = ac.std.device
        self.dev = dev
        n = sum(p.numel() for p in params)
        self.n = n
        self.flat = torch.empty(n, device=dev)
        self.grad = torch.zeros(n + 4, device=dev)  # tail: [surrogate, value, kl, entropy]
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        self.step_t = torch.zeros((), device=dev)
        self.params = params
        self._gview, self._mview, self._vview = {}, {}, {}
        off = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                v = self.flat[off:off + k].view_as(p)
                v.copy_(p.data)
                p.data = v
                p.grad = self.grad[off:off + k].view_as(p)
                self._gview[id(p)] = p.grad
                self._mview[id(p)] = self.exp_avg[off:off + k].view_as(p)
                self._vview[id(p)] = self.exp_avg_sq[off:off + k].view_as(p)
                off += k
        self.stats = self.grad[n:n + 4]
        self._offset = {}  # flat offset of every parameter
        off = 0
        for p in params:
            self._offset[id(p)] = off
            off += p.numel()
        # the bf16 weight copies (wb) are the GEMM operands of the rollout and the update;
        # every fused Adam step rewrites them (pmlp_adam_mirror).  weights_changed: they lag
        # the fp32 weights (construction, a checkpoint load, any update outside this path)
        # and are reconverted before their next use (ensure_weights)
        self.weights_changed = True
        self.sync_optimizer_state(alg.optimizer)
        self._alloc()

    # ------------------------------------------------------------ buffers --
    def _alloc(self):
        M, dev, bf = self.M, self.dev, torch.bfloat16
        L = len(self.lins[0])
        self.L = L
        self.k0p = [_ceil8(ls[0].in_features) for ls in self.lins]
        # row-major activations of exactly the layer's width (rows of 512 / 256 / 128 features
        # start on 128-byte lines); the weight gradients read them through LDS-transposed MFMA
        # operands (PARTIAL_TN: no transposed copy is ever written) and form the bias gradient
        # as their A operand times ones (sum_col)
        self.xb = [torch.empty(M, k, dtype=bf, device=dev) for k in self.k0p]
        # W[out, in] in bf16: the forward's B[N, K] and, unchanged, the input gradient's B[K, N]
        # (b_kn); the last layer's rows are padded to a multiple of 8 with zero rows (the input
        # gradient's K) -- no transposed copy
        self.wb = [[torch.zeros(_ceil8(lin.out_features) if l == len(ls) - 1 else lin.out_features,
                                self.k0p[n] if l == 0 else lin.in_features, dtype=bf, device=dev)
                    for l, lin in enumerate(ls)] for n, ls in enumerate(self.lins)]
        # the whole forward of both nets in ONE launch (pmlp_mlp_forward: activations kept on
        # chip between layers, bitwise the per-layer GEMMs) where its shapes allow; else per-layer GEMMs
        self.fused_fwd = all(mm.mlp_forward_supported(self.lins[n], self.k0p[n]) for n in range(2))
        # its weight operands fragment-packed (include/ppo_mlp.h, pmlp_mirror_job.frag): one
        # contiguous 1 KB per wave and k-step
        self.wf = [[torch.zeros(-(-w.shape[0] // 32) * 32 * w.shape[1], dtype=bf, device=dev) for w in ws]
                   for ws in self.wb] if self.fused_fwd else None
        self.mirror = (mm.MirrorJob * (2 * len(self.lins[0])))(*[
            mm.MirrorJob(self._offset[id(lin.weight)], lin.out_features, lin.in_features, self.wb[n][l].shape[1],
                         self.wb[n][l].data_ptr(), self.wf[n][l].data_ptr() if self.wf else None)
            for n, ls in enumerate(self.lins) for l, lin in enumerate(ls)])
        self.y = [[torch.empty(M, lin.out_features, dtype=bf, device=dev) for lin in ls[:-1]] for ls in self.lins]
        self.out = [torch.empty(M, ls[-1].out_features, device=dev) for ls in self.lins]
        A = self.lins[0][-1].out_features
        if self.lins[1][-1].out_features != 1:
            raise ValueError("fused PPO step: the critic must output one value")
        self.loss_partial = torch.empty(mm.load().pmlp_ppo_loss_step_parts(M, A), device=dev)
        # output gradients (bf16) and the hidden-layer input gradients
        self.dz_out = [torch.empty(M, _ceil8(ls[-1].out_features), dtype=bf, device=dev) for ls in self.lins]
        self.dz = [[torch.empty(M, lin.in_features, dtype=bf, device=dev) if l > 0 else None
                    for l, lin in enumerate(ls)] for ls in self.lins]
        # split-K weight-gradient slabs; layers whose padded width differs from the
        # parameter's get a staging buffer (copied into the flat gradient)
        self.ks, self.slab, self.dw_stage = [], [], []
        for l in range(L):
            kps = [self.k0p[n] if l == 0 else self.lins[n][l].in_features for n in range(2)]
            # (the bias column is the TN kernel's ones product, not an extra column tile)
            ks = mm._ksplit(M, max(mm._tiles(self.lins[n][l].out_features, kps[n]) for n in range(2)),
                            slab_bytes=max(4 * self.lins[n][l].out_features * (kps[n] + 8) for n in range(2)))
            nsl = (M + ks - 1) // ks
            self.ks.append(ks)
            self.slab.append([torch.empty(nsl, self.lins[n][l].out_features, kps[n] + 8, device=dev)
                              for n in range(2)])
            self.dw_stage.append([None if kps[n] == self.lins[n][l].in_features else
                                  torch.empty(self.lins[n][l].out_features, kps[n], device=dev) for n in range(2)])
        self.opt_partial = torch.empty(mm.load().pmlp_opt_parts(), device=dev)
        # the loss end (and, at world size 1, the optimizer's norm partials and bookkeeping)
        # inside the slab-reduce launch (pmlp_reduce_slabs_step): two launches fewer per step.
        # The reduce jobs plus the std gradient must then be the whole gradient.
        covered = sum(lin.out_features * (lin.in_features + 1) for ls in self.lins for lin in ls) + A
        self.fold_loss = 2 * L <= mm.MAX_JOBS
        self.fold_opt = self.fold_loss and covered == self.n and all(d is None for ds in self.dw_stage for d in ds)
        # the slab-combine jobs (layer L-1 .. 0, actor then critic: run()'s order) and the
        # staged weight gradients' copies
        self.red, self.copies = [], []
        for l in range(L - 1, -1, -1):
            for n in range(2):
                lin = self.lins[n][l]
                kp = self.k0p[n] if l == 0 else lin.in_features
                slab = self.slab[l][n]
                dw = self._gview[id(lin.weight)] if self.dw_stage[l][n] is None else self.dw_stage[l][n]
                self.red.append((slab, dw, lin.out_features * (kp + 8), slab.shape[0], self._gview[id(lin.bias)],
                                 kp + 8, kp))
                if self.dw_stage[l][n] is not None:
                    self.copies.append((self._gview[id(lin.weight)], self.dw_stage[l][n][:, :lin.in_features]))
        # one grad-norm partial per workgroup of the combine launch (sized from its jobs)
        self.norm_partial = None
        if self.fold_opt:
            arr = (mm.ReduceJob * len(self.red))(*[mm._reduce_job(j) for j in self.red])
            nparts = mm.load().pmlp_reduce_slabs_parts(len(self.red), arr)
            if nparts <= 0:
                raise ValueError("fused PPO step: malformed slab-combine jobs")
            self.norm_partial = torch.empty(int(nparts), device=dev)
        self.nparts = 0
        # the loss in the forward's launch (pmlp_mlp_forward_ppo_loss: 96-row partials, fewer
        # than pmlp_ppo_loss_step's 64-row ones, so loss_partial holds them) where it applies
        lib = mm.load()
        fl_parts = lib.pmlp_mlp_forward_ppo_loss_parts(M, A) if hasattr(lib, "pmlp_mlp_forward_ppo_loss") else 0
        Ap = self.dz_out[0].shape[1]
        self.fused_loss = bool(self.fused_fwd and self.fold_loss and 0 < fl_parts <= self.loss_partial.numel()
                               and Ap <= 16 and Ap % 4 == 0 and os.environ.get("PMLP_FUSED_LOSS", "1") != "0")
        self.loss_nb = (fl_parts if self.fused_loss else self.loss_partial.numel()) // (3 + A)
        # a layer's weight and input gradients in one launch (PMLP_GEMM_PAIR=0: two launches)
        self.pair_backward = os.environ.get("PMLP_GEMM_PAIR", "1") != "0"

    # -------------------------------------------------------- optimizer state --
    def sync_optimizer_state(self, opt):
        """Point the torch Adam's per-parameter state at the flat moments (after
        construction or an optimizer.load_state_dict, copying loaded values in)."""
        with torch.no_grad():
            for p in self.params:
                st = opt.state.get(p)
                m, v = self._mview[id(p)], self._vview[id(p)]
                if st and st.get("exp_avg") is not None and st["exp_avg"].data_ptr() == m.data_ptr():
                    continue
                if st and "exp_avg" in st:
                    m.copy_(st["exp_avg"])
                    v.copy_(st["exp_avg_sq"])
                    self.step_t.fill_(float(st["step"]))
                opt.state[p] = {"step": self.step_t, "exp_avg": m, "exp_avg_sq": v}
            for p in self.params:  # gradients must alias the flat buffer
                if p.grad is None or p.grad.data_ptr() != self._gview[id(p)].data_ptr():
                    p.grad = self._gview[id(p)]

    def ensure_weights(self):
        """Refresh the bf16 weight copies when they lag the fp32 weights (outside any
        captured graph: the captured steps keep them current through the Adam mirror)."""
        if not self.weights_changed:
            return
        jobs = []
        for n in range(2):
            for l, lin in enumerate(self.lins[n]):
                jobs.append((lin.weight.detach(), self.wb[n][l].shape[1], self.wb[n][l][:lin.out_features], None))
        mm._convert(jobs)
        if self.wf:
            for n in range(2):
                for wb, wf in zip(self.wb[n], self.wf[n]):
                    wf.copy_(mm.frag_pack(wb, wf.numel() // wb.shape[1]))
        self.weights_changed = False

    # -------------------------------------------------------------- step ----
    def run(self, rows, src, acc):
        """One optimizer step on mini-batch rows `rows` (int64 [M]) of the flat rollout
        `src` = (obs, critic_obs, actions, values, advantages, returns, log_prob, mu, sigma),
        each [T*N, ...] fp32.  acc[0] += value loss, acc[1] += surrogate loss."""
        alg, ac, M, L = self.alg, self.ac, self.M, self.L
        obs, cobs, actions, values, adv, ret, logp, mu_old, sigma_old = src
        shared = cobs is obs and self.k0p[0] == self.k0p[1]
        lib = mm.load()
        self.ensure_weights()  # (a no-op once the Adam mirror keeps them current)
        # 1. no conversion launch: the first forward GEMM gathers the mini-batch's fp32
        #    observations through `rows` and converts them on load, storing the bf16 rows
        #    (the first weight gradient's operand) on the way; the bf16 weights are current
        #    (the previous Adam step wrote them)
        xb = [self.xb[0], self.xb[0] if shared else self.xb[1]]
        fobs = [obs, cobs]
        # 2. forward (and, where it applies, 3. in the same launch)
        A = self.out[0].shape[1]
        std = ac.std.detach()
        st = mm._stream()
        P = mm._p
        if self.fused_fwd:
            loss = (P(std), P(actions), P(logp), P(mu_old), P(sigma_old), P(adv), P(ret), P(values), P(rows), A,
                    float(alg.clip_param), int(bool(alg.use_clipped_value_loss)), float(alg.value_loss_coef),
                    float(alg.entropy_coef), P(self.loss_partial), P(self.dz_out[0]), None, self.dz_out[0].shape[1],
                    P(self.dz_out[1]), None, self.dz_out[1].shape[1], st) if self.fused_loss else None
            mm.mlp_forward([dict(x=fobs[n], kx=self.lins[n][0].in_features, rows=rows,
                                 xa=self.xb[n] if (n == 0 or not shared) else None, K0=self.k0p[n],
                                 W=self.wb[n], Wf=self.wf[n] if self.wf else None,
                                 b=[lin.bias.detach() for lin in self.lins[n]],
                                 N=[lin.out_features for lin in self.lins[n]], y=self.y[n], out=self.out[n])
                            for n in range(2)], M, loss=loss)
        for l in range(L if not self.fused_fwd else 0):
            last = l == L - 1
            gj = []
            for n in range(2):
                lin = self.lins[n][l]
                K = self.k0p[n] if l == 0 else lin.in_features
                if l == 0:
                    a = dict(af=fobs[n], rows=rows, xa=self.xb[n] if (n == 0 or not shared) else None)
                else:
                    a = dict(A=self.y[n][l - 1])
                if last:
                    gj.append(dict(B=self.wb[n][l], M=M, N=lin.out_features, K=K, bias=lin.bias.detach(),
                                   cf=self.out[n], **a))
                else:
                    gj.append(dict(B=self.wb[n][l], M=M, N=lin.out_features, K=K, bias=lin.bias.detach(),
                                   cb=self.y[n][l], **a))
            mm._gemm(mm.EPI_FWD_OUT if last else mm.EPI_FWD_HIDDEN, gj)
        # 3. loss forward + backward in one pass (rollout inputs read through `rows`); the
        #    output gradients land directly in the backward's bf16 operands
        if not self.fused_loss:
            mm._ok(lib.pmlp_ppo_loss_step(P(self.out[0]), P(std), P(self.out[1]), P(actions), P(logp), P(mu_old),
                                          P(sigma_old), P(adv), P(ret), P(values), P(rows), M, A, float(alg.clip_param),
                                          int(bool(alg.use_clipped_value_loss)), float(alg.value_loss_coef),
                                          float(alg.entropy_coef), P(self.loss_partial),
                                          None if self.fold_loss else P(self.stats),
                                          None if self.fold_loss else P(self._gview[id(ac.std)]),
                                          P(self.dz_out[0]), None, self.dz_out[0].shape[1], P(self.dz_out[1]), None,
                                          self.dz_out[1].shape[1], st), "pmlp_ppo_loss_step")
        # 4. backward through both MLPs; the weight-gradient slabs carry the bias column.
        #    A layer's weight gradient and input gradient read only its output gradient: one
        #    launch for both (pmlp_gemm_pair) where their tiles pair.  (dW_l beside dX_l on a
        #    second stream measured slower)
        dz = list(self.dz_out)
        red, copies = self.red, self.copies
        for l in range(L - 1, -1, -1):
            gj = []
            for n in range(2):
                lin = self.lins[n][l]
                kp = self.k0p[n] if l == 0 else lin.in_features
                # A = dz [M, out], B = activations [M, kp] (row-major)
                B = xb[n] if l == 0 else self.y[n][l - 1]
                gj.append(dict(A=dz[n], B=B, M=lin.out_features, N=kp, K=M, cf=self.slab[l][n], sum_col=kp))
            if l == 0:
                mm._gemm(mm.EPI_PARTIAL_TN, gj, ksplit=self.ks[l])
            else:
                gx = []
                for n in range(2):
                    lin = self.lins[n][l]
                    # the input layer's gradient is only consumed transposed (its weight gradient)
                    gx.append(dict(A=dz[n], B=self.wb[n][l], b_kn=1, M=M, N=lin.in_features, K=dz[n].shape[1],
                                   yprev=self.y[n][l - 1], cb=self.dz[n][l]))
                if self.pair_backward:
                    mm._gemm_pair(gj, self.ks[l], gx)
                else:
                    mm._gemm(mm.EPI_PARTIAL_TN, gj, ksplit=self.ks[l])
                    mm._gemm(mm.EPI_BWD_DX, gx)
                dz = [self.dz[n][l] for n in range(2)]
        adaptive = int(alg.desired_kl is not None and alg.schedule == "adaptive")
        dkl = float(alg.desired_kl if alg.desired_kl is not None else 0.0)
        fold_opt = self.fold_opt and alg.world_size == 1
        if self.fold_loss:
            rs = mm.ReduceStep(P(self.loss_partial), self.loss_nb, A, M,
                               float(alg.entropy_coef), P(std), P(self.stats), P(self._gview[id(ac.std)]),
                               P(self.norm_partial) if fold_opt else None, P(self.step_t), P(alg._lr), P(acc), dkl,
                               adaptive, self.norm_partial.numel() if fold_opt else 0)
            self.nparts = mm._reduce_step(red, rs)  # (raises before launching if the partials do not fit)
        else:
            mm._reduce(red)
        for dst, srcv in copies:
            dst.copy_(srcv)
        # 5. data-parallel: one bucket (gradient + loss statistics)
        scale = 1.0
        if alg.world_size > 1:
            dist.all_reduce(self.grad)
            scale = 1.0 / alg.world_size
        # 6. clip_grad_norm_ + Adam
        grp = alg.optimizer.param_groups[0]
        b1, b2 = grp.get("betas", (0.9, 0.999))
        eps = grp.get("eps", 1e-8)
        if not fold_opt:
            mm._ok(lib.pmlp_opt_prepare(mm._p(self.grad), self.n, scale, mm._p(self.opt_partial), mm._p(self.step_t),
                                        mm._p(self.stats), mm._p(alg._lr), mm._p(acc), dkl, adaptive, st),
                   "pmlp_opt_prepare")
        max_norm = float(alg.max_grad_norm) if alg.max_grad_norm is not None else 0.0
        # Adam, and the bf16 weight copies of the next forward written on the way
        part, nparts = (self.norm_partial, self.nparts) if fold_opt else (self.opt_partial, self.opt_partial.numel())
        mm._ok(lib.pmlp_adam_mirror_n(mm._p(self.flat), mm._p(self.grad), mm._p(self.exp_avg),
                                      mm._p(self.exp_avg_sq), self.n, scale, mm._p(part), nparts, mm._p(self.step_t),
                                      mm._p(alg._lr), max_norm, float(b1), float(b2), float(eps), len(self.mirror),
                                      self.mirror, st), "pmlp_adam_mirror_n")


class FusedRollout:
    """PPO.act + RolloutStorage.add_transitions and PPO.process_env_step for the
    Gaussian MLP policy in ONE launch per env step (pmlp_rollout_forward): the bf16
    forward of both nets, the sampling / log-prob / storage rows (incl. the
    observations) in the actor job's epilogue, and the previous step's deferred
    process_env_step (bootstrapped reward, dones).  The policy noise is Philox keyed on
    a device draw counter, so a captured rollout draws fresh noise on every replay; the
    seed comes from torch's (seeded) generator."""

    def __init__(self, step: FusedPPOStep, num_envs):
        self.f = step
        N, dev, bf = int(num_envs), step.dev, torch.bfloat16
        self.N = N
        lins = step.lins
        self.y = [[torch.empty(N, lin.out_features, dtype=bf, device=dev) for lin in ls[:-1]] for ls in lins]
        self.out = [torch.empty(N, ls[-1].out_features, device=dev) for ls in lins]
        self.actions = torch.empty(N, lins[0][-1].out_features, device=dev)
        # policy-noise draw counters: the k-th act samples with draw[k % 2] and sets
        # draw[(k + 1) % 2] (pmlp_rollout_forward), so the forward launch both draws and
        # advances without racing itself.  k counts acts across iterations (not the storage
        # index t): with an odd num_steps_per_env, keying on t would make the next
        # iteration's first step reread the counter the last step read.  A captured rollout
        # has an even T (_RolloutGraph), so its replays keep k's parity.
        self.draw = torch.zeros(2, dtype=torch.int64, device=dev)
        self.k = 0
        self.seed = noise_seed()
        # the last process_env_step's store, deferred into the next act's launch (or flush())
        self.pending = None

    def usable(self, obs, cobs, storage):
        ok = lambda t, w: (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and  # noqa: E731
                           t.shape == (self.N, w) and t.is_contiguous())
        f = self.f
        if not ok(obs, f.lins[0][0].in_features) or not ok(cobs, f.lins[1][0].in_features):
            return False
        if storage.privileged_observations is None and cobs is not obs:
            return False
        return storage.num_envs == self.N

    def forward(self, obs, cobs, t=None):
        """(mu, value) of the actor and critic on N rows into static buffers: L GEMM launches,
        the first reading the fp32 observations itself.  The bf16 weight copies are current
        (the fused Adam step writes them); they are reconverted only when they lag."""
        f, N = self.f, self.N
        f.ensure_weights()
        xs = [obs, cobs]
        if f.fused_fwd:  # one launch for both nets (pmlp_mlp_forward)
            mm.mlp_forward([dict(x=xs[n], kx=f.lins[n][0].in_features, K0=f.k0p[n], W=f.wb[n],
                                 Wf=f.wf[n] if f.wf else None, b=[lin.bias.detach() for lin in f.lins[n]],
                                 N=[lin.out_features for lin in f.lins[n]], out=self.out[n]) for n in range(2)], N)
            return self.out
        for l in range(f.L):
            last = l == f.L - 1
            gj = []
            for n in range(2):
                lin = f.lins[n][l]
                a = dict(af=xs[n]) if l == 0 else dict(A=self.y[n][l - 1])
                K = f.k0p[n] if l == 0 else lin.in_features
                if last:
                    gj.append(dict(B=f.wb[n][l], M=N, N=lin.out_features, K=K, bias=lin.bias.detach(),
                                   cf=self.out[n], **a))
                else:
                    gj.append(dict(B=f.wb[n][l], M=N, N=lin.out_features, K=K, bias=lin.bias.detach(),
                                   cb=self.y[n][l], **a))
            mm._gemm(mm.EPI_FWD_OUT if last else mm.EPI_FWD_HIDDEN, gj)
        return self.out

    def values(self, cobs):
        """ActorCritic.evaluate on N rows (compute_returns' last values) as ONE launch of the
        critic's fused forward (bitwise the per-layer GEMMs evaluate runs: 4-5 launches), or
        None when the rows do not fit the fused path."""
        f = self.f
        if not (f.fused_fwd and cobs.is_cuda and cobs.dtype == torch.float32 and cobs.dim() == 2 and
                cobs.shape == (self.N, f.lins[1][0].in_features) and cobs.is_contiguous()):
            return None
        f.ensure_weights()
        mm.mlp_forward([dict(x=cobs, kx=f.lins[1][0].in_features, K0=f.k0p[1], W=f.wb[1],
                             Wf=f.wf[1] if f.wf else None, b=[lin.bias.detach() for lin in f.lins[1]],
                             N=[lin.out_features for lin in f.lins[1]], out=self.out[1])], self.N)
        return self.out[1]

    def act(self, obs, cobs, storage, t):
        """PPO.act + add_transitions for storage step t, and the previous step's deferred
        process_env_step, in the forward's launch (pmlp_rollout_forward): one launch per env
        step where the forward, pmlp_act and pmlp_store_step were three."""
        f, N = self.f, self.N
        A = self.actions.shape[1]
        priv = storage.privileged_observations
        P = mm._p
        par = self.k % 2
        self.k += 1
        if not f.fused_fwd:  # per-layer GEMMs, then the separate sampling launch
            self.flush(storage)
            self.forward(obs, cobs, t)
            mm._ok(mm.load().pmlp_act(P(self.out[0]), P(f.ac.std.detach()), P(self.out[1]), P(obs),
                                      P(cobs) if priv is not None else None, N, A, obs.shape[1],
                                      cobs.shape[1] if priv is not None else 0, P(self.draw[par:]), self.seed,
                                      P(self.actions), P(storage.actions[t]), P(storage.actions_log_prob[t]),
                                      P(storage.mu[t]), P(storage.sigma[t]), P(storage.values[t]),
                                      P(storage.observations[t]), P(priv[t]) if priv is not None else None,
                                      mm._stream()), "pmlp_act")
            self.draw[par ^ 1].copy_(self.draw[par] + 1)
            return self.actions
        f.ensure_weights()
        pend = self.pending
        self.pending = None
        rs = mm.RolloutStep(P(f.ac.std.detach()), P(obs), P(cobs) if priv is not None else None, obs.shape[1],
                            cobs.shape[1] if priv is not None else 0, A, P(self.actions), P(storage.actions[t]),
                            P(storage.actions_log_prob[t]), P(storage.mu[t]), P(storage.sigma[t]),
                            P(storage.values[t]), P(storage.observations[t]), P(priv[t]) if priv is not None else None,
                            P(self.draw), par, self.seed)
        if pend is not None:
            rew, dones, tout, tp, gamma, job = pend
            rs.rewards, rs.dones, rs.time_outs = P(rew), P(dones), P(tout)
            rs.prev_value, rs.st_rewards, rs.st_dones = P(storage.values[tp]), P(storage.rewards[tp]), P(storage.dones[tp])
            rs.gamma = float(gamma)
            if job is not None:  # that step's env extras, in this launch (pmlp_env_extras)
                rs.extras = mm.EnvExtras(**job.fields)
                job.consumed = True
        xs = [obs, cobs]
        mm.mlp_forward([dict(x=xs[n], kx=f.lins[n][0].in_features, K0=f.k0p[n], W=f.wb[n],
                             Wf=f.wf[n] if f.wf else None, b=[lin.bias.detach() for lin in f.lins[n]],
                             N=[lin.out_features for lin in f.lins[n]], out=self.out[n]) for n in range(2)], N,
                       rollout=rs)
        return self.actions

    def store(self, rewards, dones, time_outs, storage, t, gamma, extras=None):
        """PPO.process_env_step: deferred into the next act's launch; flush() issues it alone
        (the buffers are the env's: rewards is overwritten by the next env.step, which runs
        after that launch).  `extras`: the env step's own deferred extras (the env's
        _DeferredExtras), done in the same launch before the bootstrap reads the time-outs."""
        self.pending = (rewards, dones, time_outs, t, gamma, extras)

    def flush(self, storage):
        """Issue a deferred process_env_step (and its env extras) on its own (before the
        storage is read)."""
        if self.pending is None:
            return
        rewards, dones, time_outs, t, gamma, job = self.pending
        self.pending = None
        P = mm._p
        ex = None
        if job is not None:
            ex = mm.EnvExtras(**job.fields)
            job.consumed = True
        mm._ok(mm.load().pmlp_store_step_env(P(rewards), P(dones), P(time_outs), P(storage.values[t]),
                                             P(storage.rewards[t]), P(storage.dones[t]), self.N, float(gamma),
                                             None, 0, None, 0, C.byref(ex) if ex is not None else None,
                                             mm._stream()), "pmlp_store_step_env")

    @staticmethod
    def storable(rewards, dones, time_outs, N):
        ok = lambda t, dt: t.is_cuda and t.dtype == dt and t.numel() == N and t.is_contiguous()  # noqa: E731
        return ok(rewards, torch.float32) and ok(dones, torch.bool) and (time_outs is None or
                                                                         ok(time_outs, torch.bool))


class RecurrentRollout:
    """PPO.act + RolloutStorage.add_transitions and PPO.process_env_step for
    ActorCriticRecurrent on the GPU: the state before the step is saved, both memories
    step in place on the LSTM kernel, the fp32 MLP heads run as torch ops, and pmlp_act /
    pmlp_store_step sample the actions, compute the log-probability and write the storage
    rows and the bootstrapped reward in one launch each (the distribution object and the
    per-field copies of the generic path are never built).  Capturable: the noise is
    Philox keyed on a device draw counter, as in FusedRollout."""

    def __init__(self, alg, num_envs):
        self.alg = alg
        self.N = int(num_envs)
        ac = alg.actor_critic
        self.actions = torch.empty(self.N, ac.std.shape[0], device=ac.std.device)
        self.draw = torch.zeros((), dtype=torch.int64, device=ac.std.device)
        self.seed = noise_seed()
        # both Linear/ELU/Linear heads in one launch (pmlp_heads_forward, fp32) where the
        # fused recurrent step covers the policy; else the torch modules
        from rsl_rl.algorithms import fused_recurrent
        # the memories' rollout step on the update's matrix-core kernel (pmlp_lstm_step_mfma)
        # when the update runs the fused recurrent step with it: the stored log-probabilities
        # then come from the numbers the update recomputes.  Gated on the update's own choice
        # (FusedRecurrentStep.mfma, I + H + 1 <= 128), so both always use the same arithmetic.
        rf = alg._rfused
        self.mfma_step = rf is not None and all(rf.mfma)
        self.heads = None
        # pmlp_act inside the heads' launch where the shapes allow (PMLP_HEADS_ACT=0: two launches)
        self.fuse_act = os.environ.get("PMLP_HEADS_ACT", "1") != "0"
        if fused_recurrent.supported(ac, self.N, 1) and ac.memory_a.rnn.hidden_size == ac.memory_c.rnn.hidden_size:
            dev = ac.std.device
            self.heads = [ac.actor, ac.critic]
            self.y0 = [torch.empty(self.N, s[0].out_features, device=dev) for s in self.heads]
            self.out = [torch.empty(self.N, s[2].out_features, device=dev) for s in self.heads]

    def _mstate(self, mem, x):
        """The memory's static state buffers (created as Memory.step_ creates them)."""
        B, H = x.shape[0], mem.rnn.hidden_size
        hs = mem.hidden_states
        if hs is None or not isinstance(hs, tuple) or hs[0].shape != (1, B, H) or hs[0].device != x.device:
            with torch.inference_mode(False):
                mem.hidden_states = (torch.zeros(1, B, H, device=x.device), torch.zeros(1, B, H, device=x.device))
        return mem.hidden_states

    def _mstep_pair(self, ma, obs, sa, mc, cobs, sc):
        """Both memories' Memory.step_ on ONE pmlp_lstm_step_mfma_jobs launch."""
        (ha, ca), (hc, cc) = self._mstate(ma, obs), self._mstate(mc, cobs)
        return lstm_seq.lstm_step_mfma_pair_([(ma.rnn, obs, ha, ca, sa), (mc.rnn, cobs, hc, cc, sc)])

    def usable(self, obs, cobs, storage):
        ok = lambda t: (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and  # noqa: E731
                        t.shape[0] == self.N and t.is_contiguous())
        if not ok(obs) or not ok(cobs) or storage.num_envs != self.N:
            return False
        if storage.privileged_observations is None and cobs is not obs:
            return False
        return self.alg.actor_critic.rollout_capturable()

    def act(self, obs, cobs, storage, t):
        ac = self.alg.actor_critic
        ma, mc = ac.memory_a, ac.memory_c
        H = ma.rnn.hidden_size
        if isinstance(ma.rnn, torch.nn.LSTM) and isinstance(mc.rnn, torch.nn.LSTM):
            # the state BEFORE this step goes to the storage slot from inside the step kernel
            shape = (1, self.N, H)
            sa, sc = storage.hidden_state_slots(t, [shape, shape], [(1, self.N, mc.rnn.hidden_size)] * 2)
            if self.mfma_step:  # the update's matrix-core arithmetic, both memories in one launch
                ha, hc = self._mstep_pair(ma, obs, (sa[0], sa[1]), mc, cobs, (sc[0], sc[1]))
            else:
                ha = ma.step_(obs, save=(sa[0], sa[1]))
                hc = mc.step_(cobs, save=(sc[0], sc[1]))
        else:
            storage._save_hidden_states(ac.get_hidden_states())
            ha, hc = ma(obs), mc(cobs)
        A = self.actions.shape[1]
        priv = storage.privileged_observations
        P = mm._p
        if self.heads is not None and ha.is_contiguous() and hc.is_contiguous():
            jobs = (mm.HeadJob * 2)(*[mm.HeadJob(P(h), P(s[0].weight), P(s[0].bias), P(s[2].weight), P(s[2].bias),
                                                 P(self.y0[n]), P(self.out[n]), None, None, None, s[0].out_features,
                                                 s[2].out_features)
                                      for n, (h, s) in enumerate(zip((ha, hc), self.heads))])
            if self.fuse_act and A <= 16 and self.heads[1][2].out_features == 1:
                # the sampling and the storage rows in the heads' launch (pmlp_heads_forward_act)
                act = mm.HeadAct(P(ac.std.detach()), P(obs), P(cobs) if priv is not None else None, obs.shape[1],
                                 cobs.shape[1] if priv is not None else 0, A, P(self.draw), self.seed,
                                 P(self.actions), P(storage.actions[t]), P(storage.actions_log_prob[t]),
                                 P(storage.mu[t]), P(storage.sigma[t]), P(storage.values[t]),
                                 P(storage.observations[t]), P(priv[t]) if priv is not None else None)
                mm._ok(mm.load().pmlp_heads_forward_act(jobs, self.N, H, C.byref(act), mm._stream()),
                       "pmlp_heads_forward_act")
                return self.actions
            mm._ok(mm.load().pmlp_heads_forward(2, jobs, self.N, H, mm._stream()), "pmlp_heads_forward")
            mu, value = self.out
        else:
            mu = ac.actor(ha.squeeze(0)).contiguous()
            value = ac.critic(hc.squeeze(0)).contiguous()
        mm._ok(mm.load().pmlp_act(P(mu), P(ac.std.detach()), P(value), P(obs), P(cobs) if priv is not None else None,
                                  self.N, A, obs.shape[1], cobs.shape[1] if priv is not None else 0, P(self.draw),
                                  self.seed, P(self.actions), P(storage.actions[t]), P(storage.actions_log_prob[t]),
                                  P(storage.mu[t]), P(storage.sigma[t]), P(storage.values[t]),
                                  P(storage.observations[t]), P(priv[t]) if priv is not None else None,
                                  mm._stream()), "pmlp_act")
        return self.actions

    pending = None

    def flush(self, storage):
        pass  # nothing is deferred: store() issues its launch at once

    def _reset_states(self):
        """The memories' (h, c) buffers [1, N, H] that ActorCriticRecurrent.reset(dones) masks,
        when the store launch can zero them itself (static contiguous fp32 LSTM states of one
        width), else None."""
        ac = self.alg.actor_critic
        out, H = [], None
        for mem in (ac.memory_a, ac.memory_c):
            hs = mem.hidden_states
            if not isinstance(mem.rnn, torch.nn.LSTM) or not isinstance(hs, tuple):
                return None
            for h in hs:
                if not (h.is_cuda and h.dtype == torch.float32 and h.is_contiguous() and h.dim() == 3 and
                        h.shape[1] == self.N and h.shape[2] % 4 == 0 and (H is None or h.shape[2] == H)):
                    return None
                H = h.shape[2]
                out.append(h)
        return out, H

    def store(self, rewards, dones, time_outs, storage, t, gamma, extras=None):
        """PPO.process_env_step: pmlp_store_step at once (no forward launch to ride in).
        The launch also advances the policy-noise draw counter pmlp_act read (one thread,
        after the store), so every step and every iteration samples fresh noise, and zeroes
        the done envs' memory states (ActorCriticRecurrent.reset(dones), four masked_fill_
        launches in the reference statement), and does the env step's deferred extras
        (`extras`, the env's _DeferredExtras) before the bootstrap reads the time-outs.
        Returns True when it did that reset."""
        P = mm._p
        rs = self._reset_states()
        ex = None
        if extras is not None:
            ex = mm.EnvExtras(**extras.fields)
            extras.consumed = True
        states, H = rs if rs is not None else ([], 0)
        ptrs = (C.c_void_p * len(states))(*[h.data_ptr() for h in states]) if states else None
        mm._ok(mm.load().pmlp_store_step_env(P(rewards), P(dones), P(time_outs), P(storage.values[t]),
                                             P(storage.rewards[t]), P(storage.dones[t]), self.N, float(gamma),
                                             P(self.draw), len(states), ptrs, H,
                                             C.byref(ex) if ex is not None else None, mm._stream()),
               "pmlp_store_step_env")
        return rs is not None


def gae(storage, last_values, gamma, lam, world_size=1):
    """RolloutStorage.compute_returns on the GPU in two launches (pmlp_gae): GAE
    backwards over T per env, then advantage normalisation.  world_size > 1: the
    normalisation uses the moments of every rank's advantages (one fp64 all-reduce of
    {sum, sum of squares, count} between the two halves), i.e. the whole batch's, as a
    single-GPU run over all ranks' envs would."""
    lib = mm.load()
    T, N = storage.num_transitions_per_env, storage.num_envs
    key = (T, N)
    if getattr(storage, "_gae_partial_key", None) != key:
        storage._gae_partial = torch.empty(2 * lib.pmlp_gae_parts(N), dtype=torch.float64, device=storage.device)
        storage._gae_moments = torch.empty(3, dtype=torch.float64, device=storage.device)
        storage._gae_partial_key = key
    lv = last_values.reshape(N).contiguous()
    if world_size == 1:
        mm._ok(lib.pmlp_gae(mm._p(storage.rewards), mm._p(storage.dones), mm._p(storage.values), mm._p(lv),
                            mm._p(storage.returns), mm._p(storage.advantages), T, N, float(gamma), float(lam),
                            mm._p(storage._gae_partial), mm._stream()), "pmlp_gae")
        return
    mom = storage._gae_moments
    mm._ok(lib.pmlp_gae_local(mm._p(storage.rewards), mm._p(storage.dones), mm._p(storage.values), mm._p(lv),
                              mm._p(storage.returns), mm._p(storage.advantages), T, N, float(gamma), float(lam),
                              mm._p(storage._gae_partial), mm._p(mom), mm._stream()), "pmlp_gae_local")
    dist.all_reduce(mom)
    mm._ok(lib.pmlp_adv_normalize(mm._p(storage.advantages), T * N, mm._p(mom), mm._stream()), "pmlp_adv_normalize")