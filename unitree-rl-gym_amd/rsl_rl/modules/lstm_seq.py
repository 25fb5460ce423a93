"""The recurrent memory of ActorCriticRecurrent on hand-written HIP sequence kernels
(csrc/lstm_seq.hip through include/ppo_mlp.h, "recurrent memory").

rsl_rl v1.0.2 trains the LSTM on trajectories split at dones and zero-padded
(``split_and_pad_trajectories``): the trajectory count depends on the data, so every
mini-batch costs a device->host sync and nothing can be captured in a graph.  The
dense form computes the same outputs with fixed shapes: every env's T steps run in
order and (h, c) is zeroed before step t when the env was done at t-1, which is the
zero state a padded trajectory that starts there begins from.  (The trajectory that
starts at t = 0 begins from the hidden state saved at t = 0, in both forms.)

``lstm_dense`` is differentiable w.r.t. the four LSTM parameters (autograd Function
around pmlp_lstm_fwd / pmlp_lstm_bwd plus three GEMMs for the weight gradients);
``lstm_dense_reference`` is the same recurrence in plain torch ops (CPU, tests).
"""
import ctypes as C

import torch

from . import mfma_mlp as mm

_bound = False


class LstmJob(C.Structure):
    """include/ppo_mlp.h pmlp_lstm_job: one memory's sequence in a two-memory launch."""
    _fields_ = [("I", C.c_int32), ("x", C.c_void_p), ("w_ih", C.c_void_p), ("b_ih", C.c_void_p),
                ("b_hh", C.c_void_p), ("w_hh", C.c_void_p), ("h0", C.c_void_p), ("c0", C.c_void_p),
                ("h_out", C.c_void_p), ("c_out", C.c_void_p), ("gact", C.c_void_p), ("xh", C.c_void_p),
                ("dh_out", C.c_void_p), ("slab", C.c_void_p), ("h_save", C.c_void_p), ("c_save", C.c_void_p)]


def _lib():
    global _bound
    L = mm.load()
    if not _bound:
        vp, i32 = C.c_void_p, C.c_int32
        L.pmlp_lstm_last_error.restype = C.c_char_p
        L.pmlp_lstm_supported.argtypes = [i32]
        L.pmlp_lstm_fwd.argtypes = [i32, i32, i32] + [vp] * 10 + [vp]
        L.pmlp_lstm_bwd.argtypes = [i32, i32, i32] + [vp] * 7 + [vp]
        L.pmlp_lstm_fwd_x.argtypes = [i32, i32, i32, i32] + [vp] * 14 + [vp]
        L.pmlp_lstm_step.argtypes = [i32, i32] + [vp] * 6 + [vp]
        L.pmlp_lstm_fwd_mfma.argtypes = [i32, i32, i32, i32] + [vp] * 12 + [vp]
        L.pmlp_lstm_bwd_mfma.argtypes = [i32, i32, i32] + [vp] * 7 + [vp]
        L.pmlp_lstm_bwd_dw_blocks.argtypes = [i32]
        L.pmlp_lstm_bwd_dw_blocks.restype = i32
        L.pmlp_lstm_bwd_dw_mfma.argtypes = [i32, i32, i32, i32] + [vp] * 8 + [vp]
        L.pmlp_lstm_step_mfma.argtypes = [i32, i32, i32] + [vp] * 9 + [vp]
        L.pmlp_lstm_fwd_mfma_jobs.argtypes = [i32, C.POINTER(LstmJob), i32, i32, i32, vp, vp]
        L.pmlp_lstm_bwd_dw_mfma_jobs.argtypes = [i32, C.POINTER(LstmJob), i32, i32, i32, vp, vp]
        L.pmlp_lstm_step_mfma_jobs.argtypes = [i32, C.POINTER(LstmJob), i32, i32, vp]
        _bound = True
    return L


def _ok(status, what):
    if status != 0:
        raise RuntimeError(f"{what} failed: {_lib().pmlp_lstm_last_error().decode(errors='replace')}")


# The update's dense sequences on the matrix cores (pmlp_lstm_fwd_mfma / _bwd_mfma: bf16
# products, fp32 state) for hidden 64 and inputs <= 64; other shapes take the fp32 kernels.
def mfma_usable(rnn, x):
    return rnn.hidden_size == 64 and x.shape[-1] <= 64


def usable(rnn, x):
    """The kernels cover a one-layer LSTM with hidden 32/64/128 on a GPU, fp32."""
    return (x.is_cuda and isinstance(rnn, torch.nn.LSTM) and rnn.num_layers == 1 and rnn.bias
            and x.dtype == torch.float32 and rnn.hidden_size in (32, 64, 128) and not rnn.batch_first)


def _gx(x, w_ih, b_ih, b_hh):
    T, B, I = x.shape
    return torch.addmm(b_ih + b_hh, x.reshape(T * B, I), w_ih.t()).view(T, B, w_ih.shape[0])


_ROWS_CHUNK = 1024


def _rows_tn(g, x, chunk=None):
    """g^T x for tall g [m, p], x [m, q]: a batched product over row chunks, then the sum
    over chunks (fp32 throughout)."""
    chunk = chunk or _ROWS_CHUNK
    m = g.shape[0]
    c = m // chunk
    if c < 2:
        return g.t().mm(x)
    main = torch.bmm(g[:c * chunk].view(c, chunk, -1).transpose(1, 2), x[:c * chunk].view(c, chunk, -1)).sum(0)
    if c * chunk < m:
        main += g[c * chunk:].t().mm(x[c * chunk:])
    return main


class _LSTMDense(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h0, c0, reset, w_ih, w_hh, b_ih, b_hh, mfma=False):
        T, B, I = x.shape
        H = w_hh.shape[1]
        whh = w_hh.detach().contiguous()
        h_out = torch.empty(T, B, H, device=x.device)
        c_out = torch.empty(T, B, H, device=x.device)
        gact = torch.empty(T, B, 4 * H, device=x.device)
        # [x | h_prev | 1] per row: the operand of all three weight gradients
        xh = torch.empty(T, B, I + H + 1, device=x.device)
        p = mm._p
        ctx.mfma = mfma
        if mfma:  # the per-step products on the matrix cores (bf16 operands, fp32 state)
            _ok(_lib().pmlp_lstm_fwd_mfma(T, B, H, I, p(x), p(w_ih.detach().contiguous()), p(b_ih.detach()),
                                          p(b_hh.detach()), p(whh), p(h0), p(c0), p(reset), p(h_out), p(c_out),
                                          p(gact), p(xh), mm._stream()), "pmlp_lstm_fwd_mfma")
        elif I <= 64:  # the input projection inside the sequence kernel, which also writes xh
            _ok(_lib().pmlp_lstm_fwd_x(T, B, H, I, p(x), p(w_ih.detach().contiguous()), p(b_ih.detach()),
                                       p(b_hh.detach()), p(whh), p(h0), p(c0), p(reset), p(h_out), p(c_out), p(gact),
                                       None, None, p(xh), mm._stream()), "pmlp_lstm_fwd_x")
        else:
            gx = _gx(x.detach(), w_ih.detach(), b_ih.detach(), b_hh.detach())
            _ok(_lib().pmlp_lstm_fwd(T, B, H, p(gx), p(whh), p(h0), p(c0), p(reset), p(h_out), p(c_out), p(gact),
                                     None, None, mm._stream()), "pmlp_lstm_fwd")
            xh[..., :I].copy_(x)
            if h0 is None:
                xh[0, :, I:I + H].zero_()
            else:
                xh[0, :, I:I + H].copy_(h0)
            xh[1:, :, I:I + H].copy_(h_out[:-1])
            if reset is not None:
                xh[..., I:I + H].masked_fill_(reset.bool().unsqueeze(-1), 0.0)
            xh[..., I + H].fill_(1.0)
        ctx.save_for_backward(xh, c0, reset, whh, c_out, gact)
        ctx.I = I
        return h_out

    @staticmethod
    def backward(ctx, dh_out):
        xh, c0, reset, whh, c_out, gact = ctx.saved_tensors
        I = ctx.I
        T, B, _ = xh.shape
        H = whh.shape[1]
        dgx = torch.empty(T, B, 4 * H, device=xh.device)
        p = mm._p
        bwd = _lib().pmlp_lstm_bwd_mfma if ctx.mfma else _lib().pmlp_lstm_bwd
        _ok(bwd(T, B, H, p(whh), p(c0), p(reset), p(c_out), p(gact), p(dh_out.contiguous()), p(dgx), mm._stream()),
            "pmlp_lstm_bwd_mfma" if ctx.mfma else "pmlp_lstm_bwd")
        # all three weight gradients from ONE product dgx^T [x | h_prev | 1] over the T*B
        # rows, split over the rows (a library GEMM puts a 49k-long reduction on a few
        # output tiles: 170 us per call at H1 scale)
        dw = _rows_tn(dgx.view(T * B, 4 * H), xh.view(T * B, I + H + 1))
        dw_ih, dw_hh, db = dw[:, :I].contiguous(), dw[:, I:I + H].contiguous(), dw[:, I + H].contiguous()
        return None, None, None, None, dw_ih, dw_hh, db, db, None


def lstm_dense(rnn, x, h0, c0, reset, mfma=None):
    """[T,B,I] -> [T,B,H] through rnn (nn.LSTM, one layer) with resets before step t where
    reset[t] != 0; h0/c0 [B,H] (detached: the saved rollout state) or None.  mfma: the
    matrix-core kernels (default: where mfma_usable)."""
    def state(s):
        if s is None:
            return None
        s = s.detach().reshape(x.shape[1], -1)
        return s.clone() if s.is_inference() else s.contiguous()

    h0, c0 = state(h0), state(c0)
    reset = None if reset is None else reset.to(torch.uint8).contiguous()
    mfma = mfma_usable(rnn, x) if mfma is None else bool(mfma)
    return _LSTMDense.apply(x.contiguous(), h0, c0, reset, rnn.weight_ih_l0, rnn.weight_hh_l0, rnn.bias_ih_l0,
                            rnn.bias_hh_l0, mfma)


def lstm_dense_reference(rnn, x, h0, c0, reset):
    """The same recurrence in torch ops (any device): the statement the kernels are checked against."""
    T, B, _ = x.shape
    H = rnn.hidden_size
    h = x.new_zeros(B, H) if h0 is None else h0.reshape(B, H)
    c = x.new_zeros(B, H) if c0 is None else c0.reshape(B, H)
    gx = _gx(x, rnn.weight_ih_l0, rnn.bias_ih_l0, rnn.bias_hh_l0)
    out = []
    for t in range(T):
        if reset is not None:
            keep = (reset[t] == 0).to(x.dtype).unsqueeze(-1)
            h, c = h * keep, c * keep
        g = gx[t] + h.mm(rnn.weight_hh_l0.t())
        i, f, gg, o = g.chunk(4, dim=-1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        out.append(h)
    return torch.stack(out)


def lstm_step_(rnn, x, h, c, save=None):
    """One rollout step in place: h, c [1,B,H] static buffers (the policy's memory) are read
    and overwritten by the kernel (capturable); returns h (the step's output, [1,B,H]).
    save = (h_dst, c_dst): the state the step starts from is also written there (the rollout
    storage's saved hidden state) by the same kernel."""
    B = x.shape[0]
    H = rnn.hidden_size
    p = mm._p
    with torch.no_grad():
        # (one step: the GEMM + sequence kernel beats the fused input projection, whose
        # per-workgroup W_ih row loads dominate at T = 1: 28 vs 43 us at 8192 envs)
        gx = torch.addmm(rnn.bias_ih_l0 + rnn.bias_hh_l0, x, rnn.weight_ih_l0.t())
        hs, cs = (None, None) if save is None else save
        _ok(_lib().pmlp_lstm_step(B, H, p(gx), p(rnn.weight_hh_l0.detach().contiguous()), p(h), p(c), p(hs), p(cs),
                                  mm._stream()), "pmlp_lstm_step")
    return h


def lstm_step_mfma_pair_(steps):
    """Both memories' rollout step in ONE launch (pmlp_lstm_step_mfma_jobs: the kernel of
    lstm_step_mfma_ per job, side by side in the grid).  steps: [(rnn, x, h, c, save)] x 2,
    same batch size.  Returns the h buffers."""
    p = mm._p
    B = steps[0][1].shape[0]
    jobs = (LstmJob * len(steps))()
    for n, (rnn, x, h, c, save) in enumerate(steps):
        hs, cs = (None, None) if save is None else save
        jobs[n] = LstmJob(x.shape[1], p(x), p(rnn.weight_ih_l0), p(rnn.bias_ih_l0), p(rnn.bias_hh_l0),
                          p(rnn.weight_hh_l0), None, None, p(h), p(c), None, None, None, None, p(hs), p(cs))
    with torch.no_grad():
        _ok(_lib().pmlp_lstm_step_mfma_jobs(len(steps), jobs, B, steps[0][0].hidden_size, mm._stream()),
            "pmlp_lstm_step_mfma_jobs")
    return [st[2] for st in steps]


def lstm_step_mfma_(rnn, x, h, c, save=None):
    """One rollout step in place on the matrix-core kernel (pmlp_lstm_step_mfma: the update's
    arithmetic at T = 1, hidden 64): h, c [1,B,H] static buffers; save = (h_dst, c_dst)
    receives the state the step starts from.  Returns h."""
    B, I = x.shape
    H = rnn.hidden_size
    p = mm._p
    hs, cs = (None, None) if save is None else save
    with torch.no_grad():
        _ok(_lib().pmlp_lstm_step_mfma(B, H, I, p(x), p(rnn.weight_ih_l0), p(rnn.bias_ih_l0), p(rnn.bias_hh_l0),
                                       p(rnn.weight_hh_l0), p(h), p(c), p(hs), p(cs), mm._stream()),
            "pmlp_lstm_step_mfma")
    return h
