"""GPU: the fused Viterbi decode (HMM355_VIT_PLAN_BANDED; csrc/recur.h rec_band vtail) -- the
chunk maps composed by a wave of the chain kernel while the chain runs, and the backtrace
after it in the same launch -- against the C oracle (bit-exact states and trellis, reference
hmm.py:154-184) and against the three-kernel path (HMM355_VIT_TAIL=0) it replaces.

Covers chunk edges (T = 1, 63, 64, 65, 127, 128, 129), a long sequence, both fused-chain widths
(NP = 128 and NP = 256), tie-heavy trellises (the first-index rule of torch.max, hmm.py:167),
and a caller error (the flag with a dense plan: states -1, score NaN)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _plan(P):
    from pytorch_hmm_amd import ops
    lP, lp0 = O.hmm_params(P)
    lPd = lP.to(DEV)
    plan = ops.make_plan(lPd)
    return lP, lp0, lPd, plan


def _run(lo, lPd, lp0, plan, tail, monkeypatch):
    from pytorch_hmm_amd import ops
    monkeypatch.setenv("HMM355_VIT_TAIL", "1" if tail else "0")
    s, d, f = ops.viterbi(torch.from_numpy(lo).to(DEV), lPd, lp0.to(DEV), ops.OBS_LOG, plan)
    torch.cuda.synchronize()
    return s.cpu().numpy(), d.cpu().numpy(), f.cpu().numpy()


@pytest.mark.parametrize("mat,N", [("l2r", 128), ("ergodic", 128), ("skip", 200), ("l2r", 100)])
@pytest.mark.parametrize("T", [1, 2, 63, 64, 65, 127, 128, 129, 700])
def test_fused_decode_vs_c_oracle(mat, N, T, monkeypatch):
    P = {"l2r": lambda: O.left_to_right_matrix(N, 0.7),
         "ergodic": lambda: O.transition_matrix(N, "ergodic"),
         "skip": lambda: O.transition_matrix(N, "left_to_right_skip", 0.5, 0.4, 0.1)}[mat]()
    lP, lp0, lPd, plan = _plan(P)
    assert plan._hmm355_banded
    rng = np.random.default_rng(T * 7 + N)
    B = 3
    lo = np.log(rng.random((B, T, N), dtype=np.float32) + np.float32(1e-3)).astype(np.float32)
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    s1, d1, f1 = _run(lo, lPd, lp0, plan, True, monkeypatch)
    assert np.array_equal(d1, cd)
    assert np.array_equal(s1, cs)
    assert np.array_equal(f1, cd[:, -1].max(-1))
    s0, d0, f0 = _run(lo, lPd, lp0, plan, False, monkeypatch)
    assert np.array_equal(s0, s1) and np.array_equal(f0, f1)


@pytest.mark.parametrize("N", [128, 256])
def test_fused_decode_ties_long(N, monkeypatch):
    """Coarse log-emissions (many equal trellis values, so psi takes the first index on ties)
    over T = 3000 (47 chunk maps, several expansion rounds per wave)."""
    P = O.left_to_right_matrix(N, 0.5)
    lP, lp0, lPd, plan = _plan(P)
    rng = np.random.default_rng(N)
    B, T = 4, 3000
    lo = np.round(-(rng.random((B, T, N)) * 6), 0).astype(np.float32)
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    s1, d1, f1 = _run(lo, lPd, lp0, plan, True, monkeypatch)
    assert np.array_equal(d1, cd) and np.array_equal(s1, cs)


def test_fused_decode_obs_prob_matches_three_kernel_path(monkeypatch):
    """OBS_PROB (the staging takes log(x + 1e-8), logcr.h): same states and trellis either way."""
    from pytorch_hmm_amd import ops
    P = O.left_to_right_matrix(128, 0.7)
    lP, lp0, lPd, plan = _plan(P)
    g = torch.Generator(device=DEV).manual_seed(5)
    obs = torch.softmax(torch.randn(8, 1000, 128, device=DEV, generator=g), -1)
    out = []
    for tail in ("1", "0"):
        monkeypatch.setenv("HMM355_VIT_TAIL", tail)
        out.append([x.cpu() for x in ops.viterbi(obs, lPd, lp0.to(DEV), ops.OBS_PROB, plan)])
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_fused_decode_flag_with_dense_plan_marks_invalid():
    """The flag is the caller's word that the plan is banded; with a dense plan the chain kernel
    cannot finish the decode, and says so (states -1, final score NaN) instead of leaving stale
    buffers."""
    import pytorch_hmm_amd._native as nat
    from pytorch_hmm_amd import ops
    N, B, T = 128, 2, 200
    rng = np.random.default_rng(3)
    P = torch.from_numpy(rng.random((N, N), dtype=np.float32))
    lP, lp0 = O.hmm_params(P)
    lPd = lP.to(DEV)
    plan = ops.make_plan(lPd)
    assert not plan._hmm355_banded
    L = nat.lib()
    obs = torch.from_numpy(np.log(rng.random((B, T, N), dtype=np.float32) + np.float32(1e-3))).to(DEV)
    states = torch.zeros(B, T, dtype=torch.int64, device=DEV)
    delta = torch.empty(B, T, N, device=DEV)
    final = torch.zeros(B, device=DEV)
    ws = torch.empty(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=DEV)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = L.hmm355_viterbi_plan_ex_f32(p(obs), ops.OBS_LOG, p(lPd), p(lp0.to(DEV)), p(plan), nat.VIT_PLAN_BANDED,
                                      B, T, N, p(states), p(delta), p(final), p(ws), ws.numel(),
                                      nat.stream_of(torch.device(DEV, 0)))
    assert rc == 0
    torch.cuda.synchronize()
    assert bool((states == -1).all()) and bool(torch.isnan(final).all())
    _, cd, _ = O.c_viterbi(obs.cpu().numpy(), lP.numpy(), lp0.numpy())
    assert np.array_equal(delta.cpu().numpy(), cd)   # the trellis itself is still complete
