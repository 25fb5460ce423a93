"""libppomlp.so (include/ppo_mlp.h) on the CPU: the library loads and exports every
function the header declares, the ctypes job structs have the C layout (checked against a
helper compiled from the header with gcc), and malformed jobs come back as a status with a
message -- the argument checks run before any HIP call, so no GPU is needed."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ppo_mlp.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"PMLP_API\s+[\w\s\*]+?\b(pmlp_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import torch  # noqa: F401  (the HIP runtime first)
    from rsl_rl.modules import mfma_mlp
    return mfma_mlp.load()


def test_library_exports_every_declared_symbol(lib):
    names = declared_functions()
    for must in ("pmlp_gemm", "pmlp_adam", "pmlp_adam_mirror", "pmlp_ppo_loss_step", "pmlp_gae", "pmlp_lstm_fwd"):
        assert must in names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_job_structs_match_c_layout(tmp_path):
    from rsl_rl.modules import mfma_mlp as mm
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "ppo_mlp.h"\nint main(void){printf("%zu %zu %zu %zu\\n",'
                   ' sizeof(pmlp_gemm_job), sizeof(pmlp_mirror_job), sizeof(pmlp_convert_job),'
                   ' sizeof(pmlp_reduce_job)); printf("%zu %zu %zu\\n", sizeof(pmlp_head_job), sizeof(pmlp_lstm_job), sizeof(pmlp_reduce_step));'
                   ' printf("%zu %zu %zu\\n", sizeof(pmlp_env_extras), sizeof(pmlp_rollout_step), sizeof(pmlp_head_act));'
                   ' return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    from rsl_rl.modules import lstm_seq
    assert got == [C.sizeof(mm.GemmJob), C.sizeof(mm.MirrorJob), C.sizeof(mm.ConvertJob), C.sizeof(mm.ReduceJob),
                   C.sizeof(mm.HeadJob), C.sizeof(lstm_seq.LstmJob), C.sizeof(mm.ReduceStep),
                   C.sizeof(mm.EnvExtras), C.sizeof(mm.RolloutStep), C.sizeof(mm.HeadAct)]


def _job(**kw):
    from rsl_rl.modules import mfma_mlp as mm
    j = mm.GemmJob()
    j.A, j.B = 16, 16  # non-null, 16-byte aligned (never dereferenced: the checks fail first)
    j.lda = j.ldb = 64
    j.M, j.N, j.K = 128, 64, 64
    j.cb, j.ldcb, j.yprev, j.ldyp = 16, 64, 16, 64
    for k, v in kw.items():
        setattr(j, k, v)
    return j


@pytest.mark.parametrize("epi,kw,msg", [
    (0, dict(b_kn=1), b"B given [K,N]"),          # W[out,in] operand only for the input gradient
    (2, dict(af=16, kaf=64, ldaf=64), b"fp32 A"),  # fp32-gathered A only for the forward
    (0, dict(af=16, kaf=96, ldaf=96), b"fp32 A"),  # kaf > K
    (0, dict(af=16, kaf=64, ldaf=66), b"fp32 A"),  # ldaf not a multiple of 4
    (0, dict(sum_col=64), b"sum_col"),             # the ones product only for PARTIAL_TN
    (4, dict(sum_col=32, cf=16, ldcf=72, M=64), b"sum_col"),  # sum_col inside the N columns
])
def test_malformed_gemm_jobs_are_refused(lib, epi, kw, msg):
    from rsl_rl.modules import mfma_mlp as mm
    arr = (mm.GemmJob * 1)(_job(**kw))
    assert lib.pmlp_gemm(epi, 1, arr, 0, None) != 0
    assert msg in lib.pmlp_last_error()


def test_mixed_operand_forms_in_one_call_are_refused(lib):
    from rsl_rl.modules import mfma_mlp as mm
    arr = (mm.GemmJob * 2)(_job(), _job(b_kn=1))
    assert lib.pmlp_gemm(2, 2, arr, 0, None) != 0
    assert b"same operand forms" in lib.pmlp_last_error()


def test_adam_mirror_checks_its_jobs(lib):
    from rsl_rl.modules import mfma_mlp as mm
    ok = mm.MirrorJob(0, 4, 4, 4, 16)
    over = mm.MirrorJob(8, 4, 4, 4, 16)  # runs past n = 16
    for jobs, n_jobs in (((mm.MirrorJob * 1)(over), 1), ((mm.MirrorJob * 9)(*([ok] * 9)), 9)):
        rc = lib.pmlp_adam_mirror(16, 16, 16, 16, 16, 1.0, 16, 16, 16, 1.0, 0.9, 0.999, 1e-8, n_jobs, jobs, None)
        assert rc != 0 and b"pmlp_adam_mirror" in lib.pmlp_last_error()


def test_recurrent_and_bookkeeping_entries_refuse_bad_arguments(lib):
    """The LSTM entries, the folded reduce step and the loss bookkeeping check their
    arguments before any launch."""
    from rsl_rl.modules import lstm_seq
    from rsl_rl.modules import mfma_mlp as mm
    L = lstm_seq._lib()
    assert L.pmlp_lstm_step(0, 64, 16, 16, 16, 16, None, None, None) != 0  # empty batch
    assert L.pmlp_lstm_step(8, 64, 16, 8, 16, 16, None, None, None) != 0  # whh not 16-byte aligned
    assert b"pmlp_lstm_step" in L.pmlp_lstm_last_error()
    assert L.pmlp_lstm_fwd_x(4, 8, 64, 65, 16, 16, None, None, 16, None, None, None, None, None, None, None, None,
                             None, None) != 0  # input wider than 64
    assert b"input size" in L.pmlp_lstm_last_error()
    jobs = (lstm_seq.LstmJob * 3)()
    assert L.pmlp_lstm_fwd_mfma_jobs(3, jobs, 24, 64, 64, None, None) != 0  # at most two memories
    assert b"1..2 jobs" in L.pmlp_lstm_last_error()
    jobs[0].I = 44
    assert L.pmlp_lstm_bwd_dw_mfma_jobs(1, jobs, 24, 64, 64, None, None) != 0  # null buffers
    assert b"pmlp_lstm_bwd_dw_mfma_jobs" in L.pmlp_lstm_last_error()
    job = (mm.ReduceJob * 1)(mm.ReduceJob(16, 16, None, 64, 64, 2, 0, 0))
    rs = mm.ReduceStep()
    assert lib.pmlp_reduce_slabs_step(1, job, C.byref(rs), None) != 0  # no loss partials
    assert b"pmlp_reduce_slabs_step" in lib.pmlp_last_error()
    rs.loss_partial, rs.loss_blocks, rs.A, rs.M, rs.stdv, rs.stats, rs.dstd, rs.norm_partial = 16, 4, 12, 256, 16, 16, 16, 16
    assert lib.pmlp_reduce_slabs_step(1, job, C.byref(rs), None) != 0  # norm partials without step / lr
    assert b"step and lr" in lib.pmlp_last_error()
    assert lib.pmlp_adam_mirror_n(16, 16, 16, 16, 16, 1.0, 16, 0, 16, 16, 1.0, 0.9, 0.999, 1e-8, 0, None, None) != 0
    lib.pmlp_loss_bookkeeping.restype = C.c_int
    assert lib.pmlp_loss_bookkeeping(None, None, None, C.c_float(0.01), 1, None) != 0
    assert b"pmlp_loss_bookkeeping" in lib.pmlp_last_error()


def test_reduce_slabs_parts_sizes_the_norm_partials(lib):
    """the grad-norm partial buffer of the folded reduce step is sized from its jobs
    (pmlp_reduce_slabs_parts = the launch's workgroups + the loss-finishing one), and a step
    whose buffer is smaller is refused before launch."""
    from rsl_rl.modules import mfma_mlp as mm
    # one job of 64 floats, 2 slabs: 16 element quads, G = 1 -> 256 quads per block: 1 block
    job = (mm.ReduceJob * 1)(mm.ReduceJob(16, 16, None, 64, 64, 2, 0, 0))
    assert lib.pmlp_reduce_slabs_parts(1, job) == 2
    # 2M floats over 96 slabs (G = 16: 16 quads per block): 500k / 16 blocks, + 1 + 1
    big = (mm.ReduceJob * 2)(mm.ReduceJob(16, 16, None, 2_000_000, 2_000_000, 96, 0, 0),
                             mm.ReduceJob(16, 16, None, 64, 64, 2, 0, 0))
    n = lib.pmlp_reduce_slabs_parts(2, big)
    assert n == 500_000 // 16 + 1 + 1 and n > 16384  # (the fixed buffer held 16384)
    assert lib.pmlp_reduce_slabs_parts(0, big) == -1
    rs = mm.ReduceStep()
    rs.loss_partial, rs.loss_blocks, rs.A, rs.M, rs.stdv, rs.stats, rs.dstd = 16, 4, 12, 256, 16, 16, 16
    rs.norm_partial, rs.step, rs.lr, rs.nparts = 16, 16, 16, n - 1
    assert lib.pmlp_reduce_slabs_step(2, big, C.byref(rs), None) != 0
    assert b"capacity" in lib.pmlp_last_error()


def test_store_step_refuses_incomplete_env_extras(lib):
    """pmlp_store_step_env with a deferred env step's extras missing a buffer (include/ppo_mlp.h
    pmlp_env_extras): refused before launch."""
    from rsl_rl.modules import mfma_mlp as mm
    ex = mm.EnvExtras(acc=16, acc_next=None, nsum=10, ep_len_s=20.0, time_out=16, pushed=16)
    rc = lib.pmlp_store_step_env(16, 16, 16, 16, 16, 16, 64, 0.99, None, 0, None, 0, C.byref(ex), None)
    assert rc != 0 and b"env extras" in lib.pmlp_last_error()
    ex.acc_next, ex.ep_len_s = 16, 0.0  # no episode length
    assert lib.pmlp_store_step_env(16, 16, 16, 16, 16, 16, 64, 0.99, None, 0, None, 0, C.byref(ex), None) != 0
