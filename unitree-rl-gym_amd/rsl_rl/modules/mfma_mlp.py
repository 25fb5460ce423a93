"""Actor/critic MLP forward + backward on hand-written bf16 MFMA kernels.

`mlp_apply(seq, x)` runs an `nn.Sequential(Linear, ELU, ..., Linear)` (the
rsl_rl v1.0.2 actor / critic shape) through `libppomlp.so` (include/ppo_mlp.h):
bf16 operands, fp32 accumulation, fp32 parameters/gradients (the torch
optimizer and loss are unchanged).  Every GEMM is one of the library's
C = A . B^T forms; activations are kept row-major (next layer's input) and
transposed (weight-gradient operand), see csrc/ppo_mlp.hip.

Kernels are launched on torch's current stream, allocate nothing (buffers are
torch tensors) and are deterministic, so the PPO update graph can capture them.
There is no fallback: a missing library raises.
"""
import ctypes as C
import os

import torch
import torch.nn as nn

EPI_FWD_HIDDEN, EPI_FWD_OUT, EPI_BWD_DX, EPI_PARTIAL = 0, 1, 2, 3
_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib_path():
    env = os.environ.get("PPOMLP_LIB")
    if env:
        return env
    return os.path.normpath(os.path.join(_HERE, "..", "..", "csrc", "build", "libppomlp.so"))


def load():
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(f"libppomlp.so not found at {path}: build it (make -C unitree-rl-gym_amd/csrc)")
        L = C.CDLL(path)
        vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
        L.pmlp_last_error.restype = C.c_char_p
        L.pmlp_convert.argtypes = [vp, i32, i32, i32, i32, vp, i32, vp, i32, vp]
        L.pmlp_gemm.argtypes = [i32, vp, i32, vp, i32, i32, i32, i32, vp, vp, i32, vp, i32, vp, i32, vp, i32, i32, vp]
        L.pmlp_reduce_slabs.argtypes = [vp, i32, i64, i64, vp, vp]
        L.pmlp_rowsum.argtypes = [vp, i32, i32, i32, vp, vp]
        L.pmlp_convert_weights.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp, vp]
        f32 = C.c_float
        L.pmlp_ppo_loss_blocks.argtypes = [i32]
        L.pmlp_ppo_loss_blocks.restype = i32
        L.pmlp_ppo_loss_fwd.argtypes = [vp] * 10 + [i32, i32, f32, i32, f32, f32, vp, vp, vp, vp]
        L.pmlp_ppo_loss_bwd.argtypes = [vp] * 10 + [i32, i32, f32, i32, f32, f32, vp, vp, vp, vp, vp, vp]
        _lib = L
    return _lib


def _ok(status, what):
    if status != 0:
        raise RuntimeError(f"{what} failed ({status}): {load().pmlp_last_error().decode(errors='replace')}")


def _p(t):
    return None if t is None else t.data_ptr()


def _ceil8(n):
    return (n + 7) // 8 * 8


def supported(seq):
    """Linear (ELU(alpha=1) Linear)* with hidden widths that are multiples of 8."""
    if not isinstance(seq, nn.Sequential) or len(seq) % 2 != 1:
        return False
    for i, m in enumerate(seq):
        if i % 2 == 0:
            if not isinstance(m, nn.Linear) or m.bias is None:
                return False
            if i > 0 and m.in_features % 8:
                return False
        elif not (isinstance(m, nn.ELU) and m.alpha == 1.0):
            return False
    return True


def _convert(x, Kp, y=None, yt=None):
    M, K = x.shape
    _ok(load().pmlp_convert(_p(x), M, K, x.stride(0), Kp, _p(y), 0 if y is None else y.stride(0), _p(yt),
                            0 if yt is None else yt.stride(0), _stream()), "pmlp_convert")


def _convert_weights(ws, ys, yts):
    n = len(ws)
    arr = lambda T, v: (T * n)(*v)  # noqa: E731
    vp = C.c_void_p
    _ok(load().pmlp_convert_weights(
        n, arr(vp, [w.data_ptr() for w in ws]), arr(C.c_int32, [w.shape[0] for w in ws]),
        arr(C.c_int32, [w.shape[1] for w in ws]), arr(C.c_int32, [y.shape[1] for y in ys]),
        arr(vp, [y.data_ptr() for y in ys]), arr(vp, [None if t is None else t.data_ptr() for t in yts]),
        arr(C.c_int32, [0 if t is None else t.shape[1] for t in yts]), _stream()), "pmlp_convert_weights")


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _gemm(epi, A, B, M, N, K, bias=None, yprev=None, cf=None, cb=None, ct=None, ksplit=0):
    _ok(load().pmlp_gemm(epi, _p(A), A.stride(0), _p(B), B.stride(0), M, N, K, _p(bias), _p(yprev),
                         0 if yprev is None else yprev.stride(0), _p(cf), 0 if cf is None else cf.shape[-1], _p(cb),
                         0 if cb is None else cb.stride(0), _p(ct), 0 if ct is None else ct.stride(0), ksplit,
                         _stream()), "pmlp_gemm")


def _tiles(M, N):
    """Output tiles of the configuration pmlp_gemm picks for an M x N product."""
    if M <= 32:
        bm, bn = 32, 128
    elif N <= 32:
        bm, bn = 128, 32
    elif N <= 64:
        bm, bn = 128, 64
    else:
        bm, bn = 128, 128
    return ((M + bm - 1) // bm) * ((N + bn - 1) // bn)


def _ksplit(batch, tiles, target_blocks=256):
    # >= ~1024 rows per slab: the slab combine (pmlp_reduce_slabs) reads every slab once
    slabs = max(1, min(batch // 1024, round(target_blocks / tiles)))
    ks = (batch + slabs - 1) // slabs
    return (ks + 63) // 64 * 64


class _MfmaMLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, train, *params):
        Ws, bs = params[0::2], params[1::2]
        L = len(Ws)
        x = x.contiguous()
        M = x.shape[0]
        dev = x.device
        bf = torch.bfloat16
        k0p = _ceil8(x.shape[1])
        xb = torch.empty(M, k0p, dtype=bf, device=dev)
        xt = torch.empty(k0p, M, dtype=bf, device=dev) if train else None
        _convert(x, k0p, xb, xt)
        acts, acts_t = [xb], [xt]
        # every layer's bf16 W [N, kp] and (training) W^T [K, N8] in one launch
        wbs = [torch.empty(W.shape[0], k0p if l == 0 else W.shape[1], dtype=bf, device=dev) for l, W in enumerate(Ws)]
        wts = [torch.empty(W.shape[1], _ceil8(W.shape[0]), dtype=bf, device=dev) if (train and l > 0) else None
               for l, W in enumerate(Ws)]
        _convert_weights([W.detach() for W in Ws], wbs, wts)
        h = xb
        for l in range(L):
            W, b = Ws[l], bs[l]
            N, K = W.shape
            kp = k0p if l == 0 else K
            wb = wbs[l]
            if l < L - 1:
                y = torch.empty(M, N, dtype=bf, device=dev)
                yt = torch.empty(N, M, dtype=bf, device=dev) if train else None
                _gemm(EPI_FWD_HIDDEN, h, wb, M, N, kp, bias=b.detach(), cb=y, ct=yt)
                acts.append(y)
                acts_t.append(yt)
                h = y
            else:
                out = torch.empty(M, N, dtype=torch.float32, device=dev)
                _gemm(EPI_FWD_OUT, h, wb, M, N, kp, bias=b.detach(), cf=out)
        if train:
            ctx.acts, ctx.acts_t, ctx.wts = acts, acts_t, wts
            ctx.shapes = [tuple(W.shape) for W in Ws]
            ctx.k0p = k0p
        return out

    @staticmethod
    def backward(ctx, dout):
        shapes, acts, acts_t, wts = ctx.shapes, ctx.acts, ctx.acts_t, ctx.wts
        L = len(shapes)
        dout = dout.contiguous().float()
        M = dout.shape[0]
        dev = dout.device
        bf = torch.bfloat16
        n_last = shapes[-1][0]
        np_ = _ceil8(n_last)
        dz = torch.empty(M, np_, dtype=bf, device=dev)
        dzt = torch.empty(np_, M, dtype=bf, device=dev)
        _convert(dout, np_, dz, dzt)
        grads = [None] * (2 * L)
        for l in range(L - 1, -1, -1):
            N, K = shapes[l]
            kp = ctx.k0p if l == 0 else K
            # weight gradient: dW = dz^T x  (A = dz^T [N, M], B = x^T [kp, M]), split over the batch
            ks = _ksplit(M, _tiles(N, kp))
            slabs = (M + ks - 1) // ks
            slab = torch.empty(slabs, N, kp, dtype=torch.float32, device=dev)
            _gemm(EPI_PARTIAL, dzt, acts_t[l], N, kp, M, cf=slab, ksplit=ks)
            dw = torch.empty(N, kp, dtype=torch.float32, device=dev)
            _ok(load().pmlp_reduce_slabs(_p(slab), slabs, N * kp, N * kp, _p(dw), _stream()), "pmlp_reduce_slabs")
            db = torch.empty(N, dtype=torch.float32, device=dev)
            _ok(load().pmlp_rowsum(_p(dzt), N, M, dzt.stride(0), _p(db), _stream()), "pmlp_rowsum")
            grads[2 * l] = dw if kp == K else dw[:, :K].contiguous()
            grads[2 * l + 1] = db
            if l > 0:  # input gradient through the ELU below: dz_prev = (dz W) * ELU'(y_prev)
                dzp = torch.empty(M, K, dtype=bf, device=dev)
                dztp = torch.empty(K, M, dtype=bf, device=dev)
                _gemm(EPI_BWD_DX, dz, wts[l], M, K, dz.shape[1], yprev=acts[l], cb=dzp, ct=dztp)
                dz, dzt = dzp, dztp
        ctx.acts = ctx.acts_t = ctx.wts = None
        return (None, None, *grads)


def usable(seq, x):
    """The kernel path needs a CUDA batch whose row count is a multiple of 8 (16-byte rows
    of the transposed activations) and the supported layer pattern."""
    return x.is_cuda and x.dim() == 2 and x.shape[0] % 8 == 0 and supported(seq)


def mlp_apply(seq, x):
    """Run nn.Sequential `seq` on x [M, in] through the MFMA kernels (autograd-aware)."""
    params = []
    for m in seq:
        if isinstance(m, nn.Linear):
            params += [m.weight, m.bias]
    train = torch.is_grad_enabled() and any(p.requires_grad for p in params)
    return _MfmaMLPFn.apply(x, train, *params)


class _PPOLossFn(torch.autograd.Function):
    """rsl_rl v1.0.2 PPO loss (Gaussian policy), forward + backward in two fused
    kernels each (csrc/ppo_mlp.hip k_ppo_loss_*).  Returns (loss, stats) with
    stats = [surrogate_loss, value_loss, kl_mean, entropy_mean] (no gradient)."""

    @staticmethod
    def forward(ctx, mu, std, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, clip, clipped, vcoef,
                ecoef):
        M, A = mu.shape
        ins = [t.contiguous().float() for t in (mu, std, value.reshape(M), actions, old_logp.reshape(M), old_mu,
                                                  old_sigma, adv.reshape(M), ret.reshape(M), target.reshape(M))]
        nb = load().pmlp_ppo_loss_blocks(M)
        partial = torch.empty(4 * nb, device=mu.device)
        loss = torch.empty((), device=mu.device)
        stats = torch.empty(4, device=mu.device)
        _ok(load().pmlp_ppo_loss_fwd(*[_p(t) for t in ins], M, A, float(clip), int(bool(clipped)), float(vcoef),
                                     float(ecoef), _p(partial), _p(loss), _p(stats), _stream()), "pmlp_ppo_loss_fwd")
        ctx.save_for_backward(*ins)
        ctx.cfg = (M, A, float(clip), int(bool(clipped)), float(vcoef), float(ecoef), tuple(value.shape))
        ctx.mark_non_differentiable(stats)
        return loss, stats

    @staticmethod
    def backward(ctx, gloss, gstats):
        ins = ctx.saved_tensors
        M, A, clip, clipped, vcoef, ecoef, vshape = ctx.cfg
        dev = ins[0].device
        g = gloss.contiguous().float().reshape(1)
        nb = load().pmlp_ppo_loss_blocks(M)
        dmu = torch.empty(M, A, device=dev)
        dvalue = torch.empty(M, device=dev)
        dstd = torch.empty(A, device=dev)
        partial = torch.empty(A * nb, device=dev)
        _ok(load().pmlp_ppo_loss_bwd(*[_p(t) for t in ins], M, A, clip, clipped, vcoef, ecoef, _p(g), _p(dmu),
                                     _p(dvalue), _p(partial), _p(dstd), _stream()), "pmlp_ppo_loss_bwd")
        return (dmu, dstd, dvalue.view(vshape)) + (None,) * 11


def ppo_loss(mu, std, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, clip, clipped, vcoef, ecoef):
    return _PPOLossFn.apply(mu, std, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, clip, clipped,
                            vcoef, ecoef)
