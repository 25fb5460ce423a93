"""One PPO mini-batch optimizer step of the recurrent actor-critic (ActorCriticRecurrent:
one-layer LSTM memories + Linear/ELU/Linear heads, the G1 / H1 / H1_2 policies) as ~12
kernel launches, with no autograd (rsl_rl v1.0.2 PPO.update body on the dense recurrent
mini-batches; the dense form is storage.recurrent_dense_mini_batch_generator).

What the autograd update ran per mini-batch: the two LSTM kernels, ~10 library GEMMs for the
heads' forward and backward, ELU / ELU' / bias-sum / copy launches, the loss kernels, the
LSTM weight-gradient product, clip_grad_norm_'s per-tensor norms and torch's Adam.  Here
(csrc/lstm_seq.hip, csrc/ppo_mlp.hip through include/ppo_mlp.h):
    1   LSTM forward, actor and critic memories side by side (matrix-core kernels, fp32
        state, pmlp_lstm_fwd_mfma_jobs: one 2,048-env memory alone fills half the CUs)
    1   both heads forward, fp32 (pmlp_heads_forward)
    2   the PPO loss and its fp32 output gradients (pmlp_ppo_loss_step_f32)
    1   both heads backward: the LSTM output gradients and per-block weight-gradient partials
    1   LSTM backward of both memories, each accumulating its weight gradients
        dG^T [x | h_prev | 1] on the matrix cores into per-workgroup partials
        (pmlp_lstm_bwd_dw_mfma_jobs)
    1   every partial (heads, memories) summed into the flat gradient (pmlp_reduce_slabs)
    2   grad-norm partials (+ step / adaptive LR / loss bookkeeping) and Adam
Every parameter is a view of ONE flat fp32 buffer (each tensor starting on 16 bytes), the
gradient a view of another (its 4-float tail: the loss statistics, all-reduced with it at
world > 1), Adam's moments flat too -- as FusedPPOStep (fused_step.py).
"""

import ctypes as C

import torch
import torch.distributed as dist
import torch.nn as nn

from rsl_rl.modules import lstm_seq
from rsl_rl.modules import mfma_mlp as mm


def _pad4(n):
    return (n + 3) // 4 * 4


def supported(ac, num_envs, num_mini_batches):
    """The policy shapes the fused recurrent step covers (else the autograd update runs)."""
    if not getattr(ac, "is_recurrent", False) or not hasattr(ac, "memory_a") or num_envs % num_mini_batches:
        return False
    for seq in (ac.actor, ac.critic):
        if not isinstance(seq, nn.Sequential) or len(seq) != 3 or not isinstance(seq[0], nn.Linear) or \
                not isinstance(seq[1], nn.ELU) or seq[1].alpha != 1.0 or not isinstance(seq[2], nn.Linear):
            return False
        # (pmlp_heads_forward / _backward take hidden widths N0 <= 32, a multiple of 8, and N1 <= 16)
        if seq[0].bias is None or seq[2].bias is None or seq[0].out_features > 32 or seq[0].out_features % 8 or \
                seq[2].out_features > 16:
            return False
    if ac.memory_a.rnn.hidden_size != ac.memory_c.rnn.hidden_size:  # (one H per launch)
        return False
    if ac.critic[2].out_features != 1:
        return False
    for m in (ac.memory_a, ac.memory_c):
        rnn = m.rnn
        if not isinstance(rnn, nn.LSTM) or rnn.num_layers != 1 or not rnn.bias or rnn.batch_first or \
                rnn.hidden_size not in (32, 64, 128) or rnn.input_size > 64:
            return False
        if rnn.hidden_size != (ac.actor if m is ac.memory_a else ac.critic)[0].in_features:
            return False
    return True


class FusedRecurrentStep:
    def __init__(self, alg, num_envs, num_steps):
        ac = alg.actor_critic
        self.alg, self.ac = alg, ac
        self.heads = [ac.actor, ac.critic]
        self.rnns = [ac.memory_a.rnn, ac.memory_c.rnn]
        self.H = self.rnns[0].hidden_size
        if self.rnns[1].hidden_size != self.H:
            raise ValueError("fused recurrent step: both memories must have the same hidden size")
        self.T, self.mb = int(num_steps), num_envs // alg.num_mini_batches
        self.M = self.T * self.mb
        dev = ac.std.device
        self.dev = dev
        # flat parameter layout: each head's [W0 | b0 | W1 | b1] contiguous (the slab order of
        # pmlp_heads_backward), every block / LSTM tensor starting on 16 bytes
        # and each memory's [w_ih | w_hh | b_ih | b_hh] contiguous (the slab order of
        # pmlp_lstm_bwd_dw_mfma, b_ih first)
        groups = [[s[0].weight, s[0].bias, s[2].weight, s[2].bias] for s in self.heads] + [[ac.std]] + \
            [[r.weight_ih_l0, r.weight_hh_l0, r.bias_ih_l0, r.bias_hh_l0] for r in self.rnns]
        params = [p for g in groups for p in g]
        if sorted(map(id, params)) != sorted(map(id, ac.parameters())):
            raise ValueError("fused recurrent step: unexpected parameter set")
        self.params = params
        self._offset, off = {}, 0
        for g in groups:
            for p in g:
                self._offset[id(p)] = off
                off += p.numel()
            off = _pad4(off)
        n = off
        self.n = n
        self.flat = torch.zeros(n, device=dev)
        self.grad = torch.zeros(n + 4, device=dev)  # tail: [surrogate, value, kl, entropy]
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        self.step_t = torch.zeros((), device=dev)
        self.stats = self.grad[n:n + 4]
        self._gview, self._mview, self._vview = {}, {}, {}
        with torch.no_grad():
            for p in params:
                o, k = self._offset[id(p)], p.numel()
                v = self.flat[o:o + k].view_as(p)
                v.copy_(p.data)
                p.data = v
                p.grad = self.grad[o:o + k].view_as(p)
                self._gview[id(p)] = p.grad
                self._mview[id(p)] = self.exp_avg[o:o + k].view_as(p)
                self._vview[id(p)] = self.exp_avg_sq[o:o + k].view_as(p)
        self.sync_optimizer_state(alg.optimizer)
        # buffers (fixed addresses: the captured update reads them)
        T, mb, M, H = self.T, self.mb, self.M, self.H
        self.I = [r.input_size for r in self.rnns]
        self.N0 = [s[0].out_features for s in self.heads]
        self.N1 = [s[2].out_features for s in self.heads]
        f = lambda *shape: torch.empty(*shape, device=dev)  # noqa: E731
        self.h_out = [f(T, mb, H) for _ in range(2)]
        self.c_out = [f(T, mb, H) for _ in range(2)]
        self.gact = [f(T, mb, 4 * H) for _ in range(2)]
        self.xh = [f(T, mb, self.I[n] + H + 1) for n in range(2)]
        self.dgx = [None if self.mfma_of(n) else f(T, mb, 4 * H) for n in range(2)]
        self.dh = [f(T, mb, H) for _ in range(2)]
        self.y0 = [f(M, self.N0[n]) for n in range(2)]
        self.out = [f(M, self.N1[n]) for n in range(2)]
        self.dout = [f(M, self.N1[n]) for n in range(2)]
        lib = mm.load()
        self.nblk = lib.pmlp_heads_blocks(M)
        self.nh = [self.N0[n] * H + self.N0[n] + self.N1[n] * self.N0[n] + self.N1[n] for n in range(2)]
        self.slab = [f(self.nblk, self.nh[n]) for n in range(2)]
        self.loss_partial = f(lib.pmlp_ppo_loss_step_parts(M, self.N1[0]))
        self.opt_partial = f(lib.pmlp_opt_parts())
        self.mfma = [self.mfma_of(n) for n in range(2)]
        self._head_jobs = (mm.HeadJob * 2)(*[self._head_job(n) for n in range(2)])
        # the memories' weight gradients: accumulated inside the matrix-core backward (one slab
        # row per 16 envs); else the gate gradients and a row-chunked product (lstm_seq._rows_tn)
        L = lstm_seq._lib()
        self.lblk = L.pmlp_lstm_bwd_dw_blocks(mb)
        self.lrow = [4 * H * (self.I[n] + H + 1) for n in range(2)]
        self.lslab = [f(self.lblk, self.lrow[n]) if self.mfma[n] else None for n in range(2)]
        red = [mm.ReduceJob(mm._p(self.slab[n]), mm._p(self.grad) + 4 * self._offset[id(self.heads[n][0].weight)],
                            None, self.nh[n], self.nh[n], self.nblk, 0, 0) for n in range(2)]
        for n in range(2):
            if self.mfma[n]:
                r = self.rnns[n]
                red.append(mm.ReduceJob(mm._p(self.lslab[n]), mm._p(self.grad) + 4 * self._offset[id(r.weight_ih_l0)],
                                        None, self.lrow[n], self.lrow[n], self.lblk, 0, 0))
                red.append(mm.ReduceJob(mm._p(self.lslab[n]) + 4 * 4 * H * (self.I[n] + H),
                                        mm._p(self.grad) + 4 * self._offset[id(r.bias_hh_l0)], None, self.lrow[n],
                                        4 * H, self.lblk, 0, 0))
        self._red_jobs = (mm.ReduceJob * len(red))(*red)
        # the loss end (and at world size 1 the grad-norm partials and the step / LR / loss
        # bookkeeping) ride in the slab-reduce launch (pmlp_reduce_slabs_step), as in the MLP
        # step: two launches fewer per optimizer step.  One norm partial per workgroup of that
        # launch: sized from its jobs, so any memory / head width fits
        nparts = lib.pmlp_reduce_slabs_parts(len(red), self._red_jobs)
        if nparts <= 0:
            raise ValueError("fused recurrent step: malformed slab-reduce jobs")
        self.norm_partial = f(int(nparts))

    def mfma_of(self, n):
        return lstm_seq.mfma_usable(self.rnns[n], torch.empty(1, self.rnns[n].input_size)) and \
            self.rnns[n].input_size + self.H + 1 <= 128

    def _head_job(self, n):
        s, p = self.heads[n], mm._p
        return mm.HeadJob(p(self.h_out[n]), p(s[0].weight), p(s[0].bias), p(s[2].weight), p(s[2].bias), p(self.y0[n]),
                          p(self.out[n]), p(self.dout[n]), p(self.dh[n]), p(self.slab[n]), self.N0[n], self.N1[n])

    def sync_optimizer_state(self, opt):
        """Point the torch Adam's per-parameter state at the flat moments (after construction
        or an optimizer.load_state_dict, copying loaded values in); gradients alias the flat
        gradient (as FusedPPOStep.sync_optimizer_state)."""
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
            for p in self.params:
                if p.grad is None or p.grad.data_ptr() != self._gview[id(p)].data_ptr():
                    p.grad = self._gview[id(p)]

    # -------------------------------------------------------------- step ----
    def run(self, batch, acc):
        """One optimizer step on one dense recurrent mini-batch (the tuple
        recurrent_dense_mini_batch_generator yields).  acc[0] += value loss, acc[1] += surrogate."""
        obs, cobs, actions, values, adv, ret, logp, mu_old, sigma_old, (hid_a, hid_c), reset = batch
        alg, ac, T, mb, M, H = self.alg, self.ac, self.T, self.mb, self.M, self.H
        if obs.shape[:2] != (T, mb):
            raise ValueError(f"fused recurrent step: mini-batch {tuple(obs.shape[:2])}, built for {(T, mb)}")
        lib, L, P, st = mm.load(), lstm_seq._lib(), mm._p, mm._stream()
        reset = reset.contiguous()
        # 1. the memories over the T steps (zeroing the state where reset[t])
        xs, hids = (obs, cobs), (hid_a, hid_c)
        both = self.mfma[0] and self.mfma[1]  # both memories in one launch each way
        if both:
            jobs = (lstm_seq.LstmJob * 2)()
            for n in range(2):
                r, (h0, c0) = self.rnns[n], (t.reshape(mb, H) for t in hids[n])
                jobs[n] = lstm_seq.LstmJob(self.I[n], P(xs[n]), P(r.weight_ih_l0), P(r.bias_ih_l0), P(r.bias_hh_l0),
                                           P(r.weight_hh_l0), P(h0), P(c0), P(self.h_out[n]), P(self.c_out[n]),
                                           P(self.gact[n]), P(self.xh[n]), P(self.dh[n]), P(self.lslab[n]))
            lstm_seq._ok(L.pmlp_lstm_fwd_mfma_jobs(2, jobs, T, mb, H, P(reset), st), "pmlp_lstm_fwd_mfma_jobs")
        for n in range(0 if both else 2):
            r = self.rnns[n]
            h0, c0 = (t.reshape(mb, H) for t in hids[n])
            args = (T, mb, H, self.I[n], P(xs[n]), P(r.weight_ih_l0), P(r.bias_ih_l0), P(r.bias_hh_l0),
                    P(r.weight_hh_l0), P(h0), P(c0), P(reset), P(self.h_out[n]), P(self.c_out[n]), P(self.gact[n]))
            if self.mfma[n]:
                lstm_seq._ok(L.pmlp_lstm_fwd_mfma(*args, P(self.xh[n]), st), "pmlp_lstm_fwd_mfma")
            else:
                lstm_seq._ok(L.pmlp_lstm_fwd_x(*args, None, None, P(self.xh[n]), st), "pmlp_lstm_fwd_x")
        # 2. both heads: y0 and (mu, value)
        mm._ok(lib.pmlp_heads_forward(2, self._head_jobs, M, H, st), "pmlp_heads_forward")
        # 3. the loss; fp32 gradients of mu and value, the std gradient, the statistics tail
        A = self.N1[0]
        fl = lambda t: t.reshape(M, -1)  # noqa: E731
        mm._ok(lib.pmlp_ppo_loss_step_f32(P(self.out[0]), P(ac.std), P(self.out[1]), P(fl(actions)), P(fl(logp)),
                                          P(fl(mu_old)), P(fl(sigma_old)), P(fl(adv)), P(fl(ret)), P(fl(values)), None,
                                          M, A, float(alg.clip_param), int(bool(alg.use_clipped_value_loss)),
                                          float(alg.value_loss_coef), float(alg.entropy_coef), P(self.loss_partial),
                                          None, None, P(self.dout[0]), P(self.dout[1]), st), "pmlp_ppo_loss_step_f32")
        # 4. both heads backward: the memories' output gradients + weight-gradient partials
        mm._ok(lib.pmlp_heads_backward(2, self._head_jobs, M, H, st), "pmlp_heads_backward")
        # 5. the memories backward, with their weight gradients (slab partials) on the matrix cores
        if both:
            lstm_seq._ok(L.pmlp_lstm_bwd_dw_mfma_jobs(2, jobs, T, mb, H, P(reset), st), "pmlp_lstm_bwd_dw_mfma_jobs")
        for n in range(0 if both else 2):
            r, I = self.rnns[n], self.I[n]
            c0 = hids[n][1].reshape(mb, H)
            if self.mfma[n]:
                lstm_seq._ok(L.pmlp_lstm_bwd_dw_mfma(T, mb, H, I, P(r.weight_hh_l0), P(c0), P(reset),
                                                     P(self.c_out[n]), P(self.gact[n]), P(self.dh[n]), P(self.xh[n]),
                                                     P(self.lslab[n]), st), "pmlp_lstm_bwd_dw_mfma")
                continue
            lstm_seq._ok(L.pmlp_lstm_bwd(T, mb, H, P(r.weight_hh_l0), P(c0), P(reset), P(self.c_out[n]),
                                         P(self.gact[n]), P(self.dh[n]), P(self.dgx[n]), st), "pmlp_lstm_bwd")
            dw = lstm_seq._rows_tn(self.dgx[n].view(M, 4 * H), self.xh[n].view(M, I + H + 1))
            self._gview[id(r.weight_ih_l0)].copy_(dw[:, :I])
            self._gview[id(r.weight_hh_l0)].copy_(dw[:, I:I + H])
            self._gview[id(r.bias_ih_l0)].copy_(dw[:, I + H])
            self._gview[id(r.bias_hh_l0)].copy_(dw[:, I + H])
        # every slab (heads, memories) summed into the flat gradient in one launch, with the
        # loss end (the statistics tail, the std gradient) and at world size 1 the grad-norm
        # partials and the step / LR / loss bookkeeping (k_opt_prepare's work)
        adaptive = int(alg.desired_kl is not None and alg.schedule == "adaptive")
        dkl = float(alg.desired_kl if alg.desired_kl is not None else 0.0)
        # (the memories' gradients go through the reduce only on the matrix-core path: their
        # squares must be in the partials the clip reads)
        fold_opt = alg.world_size == 1 and all(self.mfma)
        rs = mm.ReduceStep(P(self.loss_partial), self.loss_partial.numel() // (3 + A), A, M, float(alg.entropy_coef),
                           P(ac.std), P(self.stats), P(self._gview[id(ac.std)]),
                           P(self.norm_partial) if fold_opt else None, P(self.step_t), P(alg._lr), P(acc), dkl,
                           adaptive, self.norm_partial.numel() if fold_opt else 0)
        mm._ok(lib.pmlp_reduce_slabs_step(len(self._red_jobs), self._red_jobs, C.byref(rs), st),
               "pmlp_reduce_slabs_step")
        # 6. data-parallel: one bucket (gradient + loss statistics)
        scale = 1.0
        if alg.world_size > 1:
            dist.all_reduce(self.grad)
            scale = 1.0 / alg.world_size
        # 7. clip_grad_norm_ + Adam (+ the adaptive LR from this step's KL, before Adam)
        grp = alg.optimizer.param_groups[0]
        b1, b2 = grp.get("betas", (0.9, 0.999))
        eps = grp.get("eps", 1e-8)
        if not fold_opt:  # the norm of the SUMMED gradient, the step count, the LR from the global KL
            mm._ok(lib.pmlp_opt_prepare(P(self.grad), self.n, scale, P(self.opt_partial), P(self.step_t),
                                        P(self.stats), P(alg._lr), P(acc), dkl, adaptive, st), "pmlp_opt_prepare")
        part, nparts = (self.norm_partial, rs.nparts) if fold_opt else (self.opt_partial, self.opt_partial.numel())
        max_norm = float(alg.max_grad_norm) if alg.max_grad_norm is not None else 0.0
        mm._ok(lib.pmlp_adam_mirror_n(P(self.flat), P(self.grad), P(self.exp_avg), P(self.exp_avg_sq), self.n, scale,
                                      P(part), nparts, P(self.step_t), P(alg._lr), max_norm, float(b1), float(b2),
                                      float(eps), 0, None, st), "pmlp_adam_mirror_n")
