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

EPI_FWD_HIDDEN, EPI_FWD_OUT, EPI_BWD_DX, EPI_PARTIAL, EPI_PARTIAL_TN = 0, 1, 2, 3, 4
_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib_path():
    env = os.environ.get("PPOMLP_LIB")
    if env:
        return env
    return os.path.normpath(os.path.join(_HERE, "..", "..", "csrc", "build", "libppomlp.so"))


class ConvertJob(C.Structure):
    _fields_ = [("x", C.c_void_p), ("y", C.c_void_p), ("yt", C.c_void_p), ("rows", C.c_void_p), ("M", C.c_int32),
                ("K", C.c_int32), ("ldx", C.c_int32), ("Kp", C.c_int32), ("ldyt", C.c_int32),
                ("one_col", C.c_int32)]


class GemmJob(C.Structure):
    _fields_ = [("A", C.c_void_p), ("B", C.c_void_p), ("bias", C.c_void_p), ("yprev", C.c_void_p),
                ("cf", C.c_void_p), ("cb", C.c_void_p), ("ct", C.c_void_p), ("lda", C.c_int32), ("ldb", C.c_int32),
                ("ldyp", C.c_int32), ("ldcf", C.c_int32), ("ldcb", C.c_int32), ("ldct", C.c_int32),
                ("M", C.c_int32), ("N", C.c_int32), ("K", C.c_int32),
                ("af", C.c_void_p), ("rows", C.c_void_p), ("xa", C.c_void_p), ("ldaf", C.c_int32),
                ("kaf", C.c_int32), ("ldxa", C.c_int32), ("b_kn", C.c_int32),
                ("sum_col", C.c_int32)]


class MirrorJob(C.Structure):
    _fields_ = [("offset", C.c_int64), ("rows", C.c_int32), ("cols", C.c_int32), ("ld", C.c_int32),
                ("dst", C.c_void_p), ("frag", C.c_void_p)]


class ReduceJob(C.Structure):
    _fields_ = [("slab", C.c_void_p), ("out", C.c_void_p), ("bias_out", C.c_void_p), ("stride", C.c_int64),
                ("n", C.c_int64), ("nslabs", C.c_int32), ("cols_in", C.c_int32), ("cols_out", C.c_int32)]


class ReduceStep(C.Structure):
    """include/ppo_mlp.h pmlp_reduce_step (pmlp_reduce_slabs_step)."""
    _fields_ = [("loss_partial", C.c_void_p), ("loss_blocks", C.c_int32), ("A", C.c_int32), ("M", C.c_int32),
                ("ecoef", C.c_float), ("stdv", C.c_void_p), ("stats", C.c_void_p), ("dstd", C.c_void_p),
                ("norm_partial", C.c_void_p), ("step", C.c_void_p), ("lr", C.c_void_p), ("acc", C.c_void_p),
                ("desired_kl", C.c_float), ("adaptive", C.c_int32), ("nparts", C.c_int32)]


class RowsumJob(C.Structure):
    _fields_ = [("x", C.c_void_p), ("out", C.c_void_p), ("rows", C.c_int32), ("cols", C.c_int32),
                ("ld", C.c_int32)]


class MlpFwdJob(C.Structure):
    _fields_ = [("x", C.c_void_p), ("rows", C.c_void_p), ("ldx", C.c_int32), ("kx", C.c_int32), ("xa", C.c_void_p),
                ("ldxa", C.c_int32), ("W", C.c_void_p * 4), ("b", C.c_void_p * 4), ("N", C.c_int32 * 4),
                ("K0", C.c_int32), ("y", C.c_void_p * 3), ("ldy", C.c_int32 * 3), ("out", C.c_void_p),
                ("ldo", C.c_int32), ("Wf", C.c_void_p * 4)]


class EnvExtras(C.Structure):
    """include/ppo_mlp.h pmlp_env_extras: a deferred env step's extras (leggedsim
    lgs_step_deferred), done by the launch that consumes the step."""
    _fields_ = [("acc", C.c_void_p), ("acc_next", C.c_void_p), ("nsum", C.c_int32), ("ep_len_s", C.c_float)] + \
        [(n, C.c_void_p) for n in ("ep_means", "ep_snapshot", "time_out", "carry", "last_root_vel", "vsim",
                                   "pushed")] + \
        [("push", C.c_int32), ("step_counter", C.c_void_p)]


class RolloutStep(C.Structure):
    """include/ppo_mlp.h pmlp_rollout_step (pmlp_rollout_forward)."""
    _fields_ = [("stdv", C.c_void_p), ("obs", C.c_void_p), ("cobs", C.c_void_p), ("O", C.c_int32),
                ("CO", C.c_int32), ("A", C.c_int32)] + \
        [(n, C.c_void_p) for n in ("actions_out", "st_actions", "st_logp", "st_mu", "st_sigma", "st_value",
                                   "st_obs", "st_cobs", "draw")] + \
        [("parity", C.c_int32), ("seed", C.c_uint64)] + \
        [(n, C.c_void_p) for n in ("rewards", "dones", "time_outs", "prev_value", "st_rewards", "st_dones")] + \
        [("gamma", C.c_float), ("extras", EnvExtras)]


class HeadJob(C.Structure):
    _fields_ = [("h", C.c_void_p), ("W0", C.c_void_p), ("b0", C.c_void_p), ("W1", C.c_void_p), ("b1", C.c_void_p),
                ("y0", C.c_void_p), ("out", C.c_void_p), ("dout", C.c_void_p), ("dh", C.c_void_p),
                ("slab", C.c_void_p), ("N0", C.c_int32), ("N1", C.c_int32)]


class HeadAct(C.Structure):
    """include/ppo_mlp.h pmlp_head_act (pmlp_heads_forward_act)."""
    _fields_ = [("stdv", C.c_void_p), ("obs", C.c_void_p), ("cobs", C.c_void_p), ("O", C.c_int32),
                ("CO", C.c_int32), ("A", C.c_int32), ("draw", C.c_void_p), ("seed", C.c_uint64),
                ("actions_out", C.c_void_p), ("st_actions", C.c_void_p), ("st_logp", C.c_void_p),
                ("st_mu", C.c_void_p), ("st_sigma", C.c_void_p), ("st_value", C.c_void_p), ("st_obs", C.c_void_p),
                ("st_cobs", C.c_void_p)]


MAX_JOBS, MAX_GEMM_JOBS = 16, 4
PMLP_MAX_MIRROR = 8  # include/ppo_mlp.h: bf16 weight copies one Adam launch writes


def load():
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(f"libppomlp.so not found at {path}: build it (make -C unitree-rl-gym_amd/csrc)")
        L = C.CDLL(path)
        vp, i32 = C.c_void_p, C.c_int32
        L.pmlp_last_error.restype = C.c_char_p
        L.pmlp_convert.argtypes = [i32, C.POINTER(ConvertJob), vp]
        L.pmlp_gemm.argtypes = [i32, i32, C.POINTER(GemmJob), i32, vp]
        L.pmlp_gemm_pair.argtypes = [i32, C.POINTER(GemmJob), i32, i32, C.POINTER(GemmJob), vp]
        L.pmlp_reduce_slabs.argtypes = [i32, C.POINTER(ReduceJob), vp]
        L.pmlp_reduce_slabs_step.argtypes = [i32, C.POINTER(ReduceJob), C.POINTER(ReduceStep), vp]
        L.pmlp_reduce_slabs_parts.argtypes = [i32, C.POINTER(ReduceJob)]
        L.pmlp_reduce_slabs_parts.restype = C.c_int64
        L.pmlp_permutation.argtypes = [vp, C.c_int64, C.c_uint64, vp]
        L.pmlp_rowsum.argtypes = [i32, C.POINTER(RowsumJob), vp]
        f32 = C.c_float
        L.pmlp_ppo_loss_blocks.argtypes = [i32]
        L.pmlp_ppo_loss_blocks.restype = i32
        L.pmlp_ppo_loss_fwd.argtypes = [vp] * 11 + [i32, i32, f32, i32, f32, f32, vp, vp, vp, vp]
        L.pmlp_ppo_loss_bwd.argtypes = [vp] * 11 + [i32, i32, f32, i32, f32, f32, vp, vp, vp, vp, vp, vp]
        i64 = C.c_int64
        L.pmlp_opt_parts.restype = i32
        L.pmlp_opt_prepare.argtypes = [vp, i64, f32, vp, vp, vp, vp, vp, f32, i32, vp]
        L.pmlp_loss_bookkeeping.argtypes = [vp, vp, vp, C.c_float, i32, vp]
        L.pmlp_adam.argtypes = [vp, vp, vp, vp, i64, f32, vp, vp, vp, f32, f32, f32, f32, vp]
        L.pmlp_adam_mirror.argtypes = [vp, vp, vp, vp, i64, f32, vp, vp, vp, f32, f32, f32, f32, i32,
                                       C.POINTER(MirrorJob), vp]
        L.pmlp_adam_mirror_n.argtypes = [vp, vp, vp, vp, i64, f32, vp, i32, vp, vp, f32, f32, f32, f32, i32,
                                         C.POINTER(MirrorJob), vp]
        L.pmlp_gae_parts.argtypes = [i32]
        L.pmlp_gae_parts.restype = i32
        L.pmlp_gae.argtypes = [vp] * 6 + [i32, i32, f32, f32, vp, vp]
        L.pmlp_gae_local.argtypes = [vp] * 6 + [i32, i32, f32, f32, vp, vp, vp]
        L.pmlp_adv_normalize.argtypes = [vp, i64, vp, vp]
        L.pmlp_ppo_loss_step_parts.argtypes = [i32, i32]
        L.pmlp_ppo_loss_step_parts.restype = i32
        L.pmlp_ppo_loss_step.argtypes = [vp] * 11 + [i32, i32, f32, i32, f32, f32, vp, vp, vp, vp, vp, i32, vp, vp,
                                                     i32, vp]
        L.pmlp_act.argtypes = [vp] * 5 + [i32, i32, i32, i32, vp, C.c_uint64] + [vp] * 9
        L.pmlp_store_step.argtypes = [vp] * 6 + [i32, f32, vp, vp]
        L.pmlp_store_step_reset.argtypes = [vp] * 6 + [i32, f32, vp, i32, vp, i32, vp]
        L.pmlp_store_step_env.argtypes = [vp] * 6 + [i32, f32, vp, i32, vp, i32, C.POINTER(EnvExtras), vp]
        L.pmlp_mlp_forward.argtypes = [i32, C.POINTER(MlpFwdJob), i32, vp]
        if hasattr(L, "pmlp_mlp_forward_ppo_loss"):  # (absent from builds before round 4's end)
            L.pmlp_mlp_forward_ppo_loss_parts.argtypes = [i32, i32]
            L.pmlp_mlp_forward_ppo_loss_parts.restype = i32
            L.pmlp_mlp_forward_ppo_loss.argtypes = [C.POINTER(MlpFwdJob), i32] + [vp] * 9 + \
                [i32, f32, i32, f32, f32, vp, vp, vp, i32, vp, vp, i32, vp]
        L.pmlp_rollout_forward.argtypes = [C.POINTER(MlpFwdJob), i32, C.POINTER(RolloutStep), vp]
        L.pmlp_ppo_loss_step_f32.argtypes = [vp] * 11 + [i32, i32, f32, i32, f32, f32, vp, vp, vp, vp, vp, vp]
        L.pmlp_heads_blocks.argtypes = [i32]
        L.pmlp_heads_blocks.restype = i32
        L.pmlp_heads_forward.argtypes = [i32, C.POINTER(HeadJob), i32, i32, vp]
        L.pmlp_heads_backward.argtypes = [i32, C.POINTER(HeadJob), i32, i32, vp]
        L.pmlp_heads_forward_act.argtypes = [C.POINTER(HeadJob), i32, i32, C.POINTER(HeadAct), vp]
        _lib = L
    return _lib


def _ok(status, what):
    if status != 0:
        raise RuntimeError(f"{what} failed ({status}): {load().pmlp_last_error().decode(errors='replace')}")


def _p(t):
    return None if t is None else t.data_ptr()


def _ceil8(n):
    return (n + 7) // 8 * 8


def _stream():
    return torch.cuda.current_stream().cuda_stream


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


def mlp_forward_supported(lins, k0p):
    """pmlp_mlp_forward's shape limits (include/ppo_mlp.h): 4 Linear layers, K0 a multiple
    of 16 (<= 64), hidden widths multiples of 32 (<= 512 / 256 / 512), output <= 32."""
    if len(lins) != 4 or k0p % 16 or k0p > 64:
        return False
    lim = (512, 256, 512)
    return all(lins[l].out_features % 32 == 0 and lins[l].out_features <= lim[l] for l in range(3)) and \
        lins[3].out_features <= 32


def frag_pack(w, rows32):
    """The fragment-packed copy of a bf16 weight w [R, K] (K a multiple of 16) that
    pmlp_mlp_forward's Wf reads and pmlp_mirror_job.frag writes (include/ppo_mlp.h): rows
    zero-padded to rows32 (a multiple of 32), element (r, c) at
    ((((r / 32) * (K / 16) + c / 16) * 64 + r % 32 + 32 * ((c / 8) % 2)) * 8 + c % 8."""
    R, K = w.shape
    p = torch.zeros(rows32, K, dtype=w.dtype, device=w.device)
    p[:R] = w
    return p.view(rows32 // 32, 32, K // 16, 2, 8).permute(0, 2, 3, 1, 4).reshape(-1)


def mlp_forward(nets, M, rollout=None, loss=None):
    """One launch of the whole forward of up to two 4-layer MLPs (pmlp_mlp_forward).  nets:
    dicts x (fp32 [*, ldx]), kx, rows (int64 [M] | None), xa (bf16 [M, K0] | None), K0,
    W (4 bf16 [N, K] tensors), Wf (None or 4 frag_pack copies of W), b (4 fp32 tensors),
    N (4 ints), y (3 bf16 [M, N] tensors or None), out (fp32 [M, N3]).  rollout: a
    RolloutStep (actor and critic over the M envs: pmlp_rollout_forward).  loss: the
    arguments of pmlp_mlp_forward_ppo_loss after M (the update's loss in the same launch)."""
    def mk(n):
        y = n.get("y") or (None, None, None)
        return MlpFwdJob(_p(n["x"]), _p(n.get("rows")), n["x"].stride(0), n["kx"], _p(n.get("xa")),
                         0 if n.get("xa") is None else n["xa"].stride(0),
                         (C.c_void_p * 4)(*[_p(w) for w in n["W"]]), (C.c_void_p * 4)(*[_p(b) for b in n["b"]]),
                         (C.c_int32 * 4)(*n["N"]), n["K0"], (C.c_void_p * 3)(*[_p(t) for t in y]),
                         (C.c_int32 * 3)(*[0 if t is None else t.stride(0) for t in y]), _p(n["out"]),
                         n["out"].stride(0), (C.c_void_p * 4)(*[_p(w) for w in (n.get("Wf") or (None,) * 4)]))
    arr = (MlpFwdJob * len(nets))(*[mk(n) for n in nets])
    if rollout is not None:  # the rollout step's sampling, storage rows and deferred store ride along
        _ok(load().pmlp_rollout_forward(arr, int(M), C.byref(rollout), _stream()), "pmlp_rollout_forward")
    elif loss is not None:  # the update's PPO loss on the workgroups' rows
        _ok(load().pmlp_mlp_forward_ppo_loss(arr, int(M), *loss), "pmlp_mlp_forward_ppo_loss")
    else:
        _ok(load().pmlp_mlp_forward(len(nets), arr, int(M), _stream()), "pmlp_mlp_forward")


def _convert(jobs):
    """jobs: (x fp32 [*,K], Kp, y bf16 [M,Kp] | None, yt bf16 [Kp,ld] | None[, rows int64 [M]
    | None[, one_col]]); without rows M = x.shape[0], with rows output row m is x[rows[m]];
    one_col > 0: that column of y is 1.0 (the bias column of a weight-gradient operand)."""
    def mk(j):
        x, kp, y, yt = j[:4]
        rows = j[4] if len(j) > 4 else None
        one = j[5] if len(j) > 5 else 0
        M = x.shape[0] if rows is None else rows.shape[0]
        return ConvertJob(_p(x), _p(y), _p(yt), _p(rows), M, x.shape[1], x.stride(0), kp,
                          0 if yt is None else yt.shape[1], one)
    for i in range(0, len(jobs), MAX_JOBS):
        chunk = jobs[i:i + MAX_JOBS]
        arr = (ConvertJob * len(chunk))(*[mk(j) for j in chunk])
        _ok(load().pmlp_convert(len(chunk), arr, _stream()), "pmlp_convert")


def _gemm_job(j):
    g = lambda k: j.get(k)  # noqa: E731
    ld = lambda t: 0 if t is None else t.stride(0)  # noqa: E731
    af = g("af")
    return GemmJob(_p(g("A")), _p(j["B"]), _p(g("bias")), _p(g("yprev")), _p(g("cf")), _p(g("cb")), _p(g("ct")),
                   ld(g("A")), j["B"].stride(0), ld(g("yprev")),
                   0 if g("cf") is None else g("cf").shape[-1], ld(g("cb")), ld(g("ct")), j["M"], j["N"], j["K"],
                   _p(af), _p(g("rows")), _p(g("xa")), ld(af), 0 if af is None else af.shape[1], ld(g("xa")),
                   int(bool(g("b_kn"))), int(g("sum_col") or 0))


def _gemm_pair(jobs_w, ksplit, jobs_x):
    """A layer's weight gradient (PARTIAL_TN jobs_w) and input gradient (BWD_DX jobs_x, B
    given [K,N]) in one launch where their tile configurations pair (pmlp_gemm_pair; else the
    two launches): bitwise the results of two _gemm calls."""
    aw = (GemmJob * len(jobs_w))(*[_gemm_job(j) for j in jobs_w])
    ax = (GemmJob * len(jobs_x))(*[_gemm_job(j) for j in jobs_x])
    _ok(load().pmlp_gemm_pair(len(jobs_w), aw, ksplit, len(jobs_x), ax, _stream()), "pmlp_gemm_pair")


def _gemm(epi, jobs, ksplit=0):
    """jobs: dicts with A, B, M, N, K and optional bias, yprev, cf, cb, ct (tensors); the
    first forward may give af (fp32 rows, A unused) with rows (int64 gather) and xa (bf16
    copy of the converted rows); the input gradient may give b_kn=1 (B = W[out, in]); a
    PARTIAL_TN weight gradient may give sum_col (slab column receiving sum_k A = the bias
    gradient)."""
    arr = (GemmJob * len(jobs))(*[_gemm_job(j) for j in jobs])
    _ok(load().pmlp_gemm(epi, len(jobs), arr, ksplit, _stream()), "pmlp_gemm")


def permutation_(out):
    """out (int64 [n], device) = a random permutation of [0, n) (pmlp_permutation: the
    mini-batch permutation without torch.randperm's device sort); the key comes from
    torch's seeded CPU generator."""
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    _ok(load().pmlp_permutation(_p(out), out.numel(), seed, _stream()), "pmlp_permutation")
    return out


def _reduce_job(j):
    sl, out, n, ns = j[:4]
    bias, ci, co = j[4:7] if len(j) > 4 else (None, 0, 0)
    return ReduceJob(_p(sl), _p(out), _p(bias), n, n, ns, ci, co)


def _reduce_step(jobs, rs):
    """pmlp_reduce_slabs_step: the slab jobs (as _reduce, at most MAX_JOBS) + the loss end
    (+ the optimizer preparation when rs.norm_partial is set); returns rs.nparts."""
    arr = (ReduceJob * len(jobs))(*[_reduce_job(j) for j in jobs])
    _ok(load().pmlp_reduce_slabs_step(len(jobs), arr, C.byref(rs), _stream()), "pmlp_reduce_slabs_step")
    return rs.nparts


def _reduce(jobs):
    """jobs: (slab, out, n, nslabs[, bias_out, cols_in, cols_out])"""
    mk = _reduce_job
    for i in range(0, len(jobs), MAX_JOBS):
        chunk = jobs[i:i + MAX_JOBS]
        arr = (ReduceJob * len(chunk))(*[mk(j) for j in chunk])
        _ok(load().pmlp_reduce_slabs(len(chunk), arr, _stream()), "pmlp_reduce_slabs")


def _rowsum(jobs):
    for i in range(0, len(jobs), MAX_JOBS):
        chunk = jobs[i:i + MAX_JOBS]
        arr = (RowsumJob * len(chunk))(*[RowsumJob(_p(x), _p(out), rows, x.shape[1], x.stride(0))
                                         for x, out, rows in chunk])
        _ok(load().pmlp_rowsum(len(chunk), arr, _stream()), "pmlp_rowsum")


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


# ~128 workgroups per weight-gradient job: fewer slabs than 256 cut the slab combine
# 16.8 -> 11.6 us per optimizer step at equal GEMM time
_KS_TARGET = 128
_KS_BUDGET = 12 << 20  # slab bytes per job


def _ksplit(batch, tiles, slab_bytes=0, target_blocks=None, min_rows=256, budget=None):
    """Rows per slab of a split-K weight gradient: ~target_blocks workgroups per job (the
    short-K GEMM is latency-bound, so more slabs = more blocks in flight), >= min_rows rows
    per slab, and at most `budget` bytes of fp32 slabs per job (written once by the GEMM,
    read once by the slab combine)."""
    target_blocks = _KS_TARGET if target_blocks is None else target_blocks
    budget = _KS_BUDGET if budget is None else budget
    # (floor: a job count of blocks just above a multiple of the 256 CUs leaves a
    # second round of blocks on a few CUs)
    slabs = max(1, min(batch // min_rows, target_blocks // tiles))
    if slab_bytes:
        slabs = max(1, min(slabs, budget // slab_bytes))
    ks = (batch + slabs - 1) // slabs
    return (ks + 63) // 64 * 64


class _MfmaMLPsFn(torch.autograd.Function):
    """Several same-depth Linear/ELU MLPs on the same batch size, every stage of all of
    them in one launch (the actor and the critic of PPO)."""

    @staticmethod
    def forward(ctx, nnets, train, *args):
        xs = [x.contiguous() for x in args[:nnets]]
        params = args[nnets:]
        L = len(params) // (2 * nnets)
        Ws = [params[2 * L * n:2 * L * (n + 1)][0::2] for n in range(nnets)]
        bs = [params[2 * L * n:2 * L * (n + 1)][1::2] for n in range(nnets)]
        M = xs[0].shape[0]
        assert all(x.shape[0] == M for x in xs)
        dev, bf = xs[0].device, torch.bfloat16
        k0p = [_ceil8(x.shape[1]) for x in xs]
        xb = [torch.empty(M, k0p[n], dtype=bf, device=dev) for n in range(nnets)]
        xt = [torch.empty(k0p[n], M, dtype=bf, device=dev) if train else None for n in range(nnets)]
        wb = [[torch.empty(W.shape[0], k0p[n] if l == 0 else W.shape[1], dtype=bf, device=dev)
               for l, W in enumerate(Ws[n])] for n in range(nnets)]
        wt = [[torch.empty(W.shape[1], _ceil8(W.shape[0]), dtype=bf, device=dev) if (train and l > 0) else None
               for l, W in enumerate(Ws[n])] for n in range(nnets)]
        jobs = []
        for n in range(nnets):
            jobs.append((xs[n], k0p[n], xb[n], xt[n]))
            for l, W in enumerate(Ws[n]):
                Wd = W.detach()
                jobs.append((Wd, wb[n][l].shape[1], wb[n][l], None))
                if wt[n][l] is not None:  # W^T [K, N8] for the input-gradient GEMM
                    jobs.append((Wd, W.shape[1], None, wt[n][l]))
        _convert(jobs)
        acts = [[xb[n]] for n in range(nnets)]
        acts_t = [[xt[n]] for n in range(nnets)]
        outs = [None] * nnets
        for l in range(L):
            last = l == L - 1
            gj = []
            for n in range(nnets):
                N, K = Ws[n][l].shape
                kp = k0p[n] if l == 0 else K
                if last:
                    outs[n] = torch.empty(M, N, dtype=torch.float32, device=dev)
                    gj.append(dict(A=acts[n][-1], B=wb[n][l], M=M, N=N, K=kp, bias=bs[n][l].detach(), cf=outs[n]))
                else:
                    y = torch.empty(M, N, dtype=bf, device=dev)
                    yt = torch.empty(N, M, dtype=bf, device=dev) if train else None
                    gj.append(dict(A=acts[n][-1], B=wb[n][l], M=M, N=N, K=kp, bias=bs[n][l].detach(), cb=y, ct=yt))
                    acts[n].append(y)
                    acts_t[n].append(yt)
            _gemm(EPI_FWD_OUT if last else EPI_FWD_HIDDEN, gj)
        if train:
            ctx.acts, ctx.acts_t, ctx.wt = acts, acts_t, wt
            ctx.shapes = [[tuple(W.shape) for W in Ws[n]] for n in range(nnets)]
            ctx.k0p, ctx.nnets = k0p, nnets
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        nnets, shapes, acts, acts_t, wt, k0p = ctx.nnets, ctx.shapes, ctx.acts, ctx.acts_t, ctx.wt, ctx.k0p
        L = len(shapes[0])
        M = acts[0][0].shape[0]
        dev, bf = acts[0][0].device, torch.bfloat16
        dz, dzt, jobs = [], [], []
        for n in range(nnets):
            n_out = shapes[n][-1][0]
            d = douts[n]
            d = torch.zeros(M, n_out, device=dev) if d is None else d.contiguous().float()
            npad = _ceil8(n_out)
            dz.append(torch.empty(M, npad, dtype=bf, device=dev))
            dzt.append(torch.empty(npad, M, dtype=bf, device=dev))
            jobs.append((d, npad, dz[n], dzt[n]))
        _convert(jobs)
        grads = [[None] * (2 * L) for _ in range(nnets)]
        red, rsum = [], []
        for l in range(L - 1, -1, -1):
            # weight gradients dW = dz^T x (split over the batch) for every net in one launch
            kps = [k0p[n] if l == 0 else shapes[n][l][1] for n in range(nnets)]
            ks = _ksplit(M, max(_tiles(shapes[n][l][0], kps[n]) for n in range(nnets)),
                         slab_bytes=max(4 * shapes[n][l][0] * kps[n] for n in range(nnets)))
            slabs = (M + ks - 1) // ks
            gj = []
            for n in range(nnets):
                N = shapes[n][l][0]
                slab = torch.empty(slabs, N, kps[n], dtype=torch.float32, device=dev)
                dw = torch.empty(N, kps[n], dtype=torch.float32, device=dev)
                db = torch.empty(N, dtype=torch.float32, device=dev)
                gj.append(dict(A=dzt[n], B=acts_t[n][l], M=N, N=kps[n], K=M, cf=slab))
                red.append((slab, dw, N * kps[n], slabs))
                rsum.append((dzt[n], db, N))
                K = shapes[n][l][1]
                grads[n][2 * l] = dw if kps[n] == K else dw[:, :K]
                grads[n][2 * l + 1] = db
            _gemm(EPI_PARTIAL, gj, ksplit=ks)
            if l > 0:  # input gradients through the ELU below, every net in one launch
                gj, nxt = [], []
                for n in range(nnets):
                    K = shapes[n][l][1]
                    dzp = torch.empty(M, K, dtype=bf, device=dev)
                    dztp = torch.empty(K, M, dtype=bf, device=dev)
                    gj.append(dict(A=dz[n], B=wt[n][l], M=M, N=K, K=dz[n].shape[1], yprev=acts[n][l], cb=dzp,
                                   ct=dztp))
                    nxt.append((dzp, dztp))
                _gemm(EPI_BWD_DX, gj)
                dz, dzt = [a for a, _ in nxt], [b for _, b in nxt]
        _reduce(red)
        _rowsum(rsum)
        for n in range(nnets):
            for l in range(L):
                K = shapes[n][l][1]
                if grads[n][2 * l].shape[1] != K or not grads[n][2 * l].is_contiguous():
                    grads[n][2 * l] = grads[n][2 * l].contiguous()
        ctx.acts = ctx.acts_t = ctx.wt = None
        flat = [g for n in range(nnets) for g in grads[n]]
        return (None, None) + (None,) * nnets + tuple(flat)


def usable(seq, x):
    """The kernel path needs a CUDA batch whose row count is a multiple of 8 (16-byte rows
    of the transposed activations) and the supported layer pattern."""
    return x.is_cuda and x.dim() == 2 and x.shape[0] % 8 == 0 and supported(seq)


def _params(seq):
    ps = []
    for m in seq:
        if isinstance(m, nn.Linear):
            ps += [m.weight, m.bias]
    return ps


def mlps_apply(seqs, xs):
    """Run nn.Sequentials `seqs` on inputs `xs` (same batch size) through the MFMA kernels,
    every stage of all nets in one launch.  Returns a tuple of outputs (autograd-aware)."""
    params = [p for s in seqs for p in _params(s)]
    train = torch.is_grad_enabled() and any(p.requires_grad for p in params)
    return _MfmaMLPsFn.apply(len(seqs), train, *xs, *params)


def mlp_apply(seq, x):
    """Run nn.Sequential `seq` on x [M, in] through the MFMA kernels (autograd-aware)."""
    return mlps_apply([seq], [x])[0]


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
        _ok(load().pmlp_ppo_loss_fwd(*[_p(t) for t in ins], None, M, A, float(clip), int(bool(clipped)), float(vcoef),
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
        _ok(load().pmlp_ppo_loss_bwd(*[_p(t) for t in ins], None, M, A, clip, clipped, vcoef, ecoef, _p(g), _p(dmu),
                                     _p(dvalue), _p(partial), _p(dstd), _stream()), "pmlp_ppo_loss_bwd")
        return (dmu, dstd, dvalue.view(vshape)) + (None,) * 11


def ppo_loss(mu, std, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, clip, clipped, vcoef, ecoef):
    return _PPOLossFn.apply(mu, std, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, clip, clipped,
                            vcoef, ecoef)
