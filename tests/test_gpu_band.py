"""GPU: the banded chains (csrc/band.h — one wave per chain, O(N W) per step) against the
oracle and against the dense chains on the same inputs.

Contracts: Viterbi states and trellis bit-identical to the C oracle (the decomposition is an
exact reorganisation of the max); forward-backward within the dense path's tolerances.
A plan made with HMM355_PLAN_DENSE (ops.make_plan(..., dense=True)) forces the dense chains."""
import os

import numpy as np
import pytest
import torch

from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def t(a):
    return torch.as_tensor(np.asarray(a)).to(DEV)


def ops():
    from pytorch_hmm_amd import ops as o
    return o


def dense_plan(lP, flag):
    """None (the chains detect the structure per call) or a plan that forces the dense chains"""
    return ops().make_plan(lP, dense=True) if flag else None


def banded_matrix(N, kind, rng):
    if kind == "l2r":
        return O.left_to_right_matrix(N, 0.7).numpy()
    if kind in ("left_to_right_skip", "circular", "ergodic"):
        return O.transition_matrix(N, kind).numpy()
    # random band of half-width 2 around the diagonal, zeros elsewhere
    P = np.zeros((N, N), np.float32)
    for i in range(N):
        for o in range(max(0, i - 2), min(N, i + 3)):
            P[i, o] = rng.random() + 0.05
    return P


@pytest.mark.parametrize("kind", ["l2r", "left_to_right_skip", "circular", "ergodic", "band5"])
@pytest.mark.parametrize("B,T,N", [(2, 300, 128), (3, 77, 40), (1, 50, 256), (2, 129, 64)])
def test_banded_viterbi_bitexact(kind, B, T, N):
    rng = np.random.default_rng(N * 7 + T)
    P = banded_matrix(N, kind, rng)
    lP, lp0 = O.hmm_params(torch.from_numpy(P))
    lo = np.log(rng.random((B, T, N), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    o = ops()
    for d in (False, True):
        states, delta, final = o.viterbi(t(lo), t(lP), t(lp0), o.OBS_LOG, dense_plan(t(lP), d))
        assert np.array_equal(states.cpu().numpy(), cs), f"dense={d}"
        assert np.array_equal(delta.cpu().numpy(), cd), f"dense={d}"


@pytest.mark.parametrize("kind", ["l2r", "band5"])
def test_banded_viterbi_ties(kind):
    """Coarse emissions force many equal candidates: first-index argmax must survive the
    banded reorganisation (psi from the row maximum + window)."""
    rng = np.random.default_rng(5)
    N, B, T = 32, 3, 200
    P = banded_matrix(N, kind, rng)
    P = np.round(P * 4) / 4 + (P > 0) * 0.25
    lP, lp0 = O.hmm_params(torch.from_numpy(P.astype(np.float32)))
    lo = np.log(np.round(rng.random((B, T, N)) * 2) / 2 + 0.25).astype(np.float32)
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    o = ops()
    states, delta, _ = o.viterbi(t(lo), t(lP), t(lp0), o.OBS_LOG)
    assert np.array_equal(delta.cpu().numpy(), cd)
    assert np.array_equal(states.cpu().numpy(), cs)


@pytest.mark.parametrize("kind", ["l2r", "band5"])
@pytest.mark.parametrize("N", [128, 97, 256])
def test_fused_psi_block_and_chunk_edges(kind, N):
    """NP >= 128: the banded chain forms psi and the 64-step chunk maps in its helper waves
    (recur.h kVitFused) instead of vit_psi_kernel.  Every T around the 16-step block and
    64-step chunk boundaries, tie-heavy emissions; states and trellis exact."""
    rng = np.random.default_rng(N + 11)
    P = banded_matrix(N, kind, rng)
    P = np.round(P * 4) / 4 + (P > 0) * 0.25
    lP, lp0 = O.hmm_params(torch.from_numpy(P.astype(np.float32)))
    o = ops()
    for T in (1, 2, 15, 16, 17, 33, 47, 48, 63, 64, 65, 127, 128, 129, 191, 257):
        lo = np.log(np.round(rng.random((2, T, N)) * 2) / 2 + 0.25).astype(np.float32)
        cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
        states, delta, _ = o.viterbi(t(lo), t(lP), t(lp0), o.OBS_LOG)
        assert np.array_equal(delta.cpu().numpy(), cd), f"T={T}"
        assert np.array_equal(states.cpu().numpy(), cs), f"T={T}"


@pytest.mark.parametrize("kind", ["l2r", "left_to_right_skip", "circular", "ergodic", "band5"])
@pytest.mark.parametrize("B,T,N", [(2, 300, 128), (3, 77, 40), (1, 50, 256)])
def test_banded_fb_vs_fp64(kind, B, T, N):
    rng = np.random.default_rng(N + T)
    P = banded_matrix(N, kind, rng)
    lP, lp0 = O.hmm_params(torch.from_numpy(P))
    obs = rng.random((B, T, N), dtype=np.float32)
    la, lb, post64, ll64 = O.c_fb64(np.log(obs + np.float32(1e-8)), lP.numpy(), lp0.numpy())
    o = ops()
    outs = {}
    for d in (False, True):
        post, fwd, bwd, loglik, lik_ref = o.forward_backward(t(obs), t(lP), t(lp0), o.OBS_PROB,
                                                             o.FB_POSTERIOR | o.FB_FORWARD | o.FB_BACKWARD,
                                                             dense_plan(t(lP), d))
        np.testing.assert_allclose(post.cpu().numpy(), post64, atol=2e-5)
        np.testing.assert_allclose(loglik.cpu().numpy(), ll64, rtol=2e-6)
        outs[d] = (fwd.cpu().numpy(), bwd.cpu().numpy(), lik_ref.cpu().numpy())
    for a, b in zip(outs[False], outs[True]):
        big = np.abs(b) > 1e-30
        np.testing.assert_allclose(a[big], b[big], rtol=1e-4)


def test_dense_matrix_stays_dense_and_exact():
    """A random dense matrix has no band: the decomposition must not engage (results
    identical with and without a dense plan).  (The factory's 'ergodic' matrix IS banded in
    this sense — a constant off-diagonal floor plus the diagonal, W = 1.)"""
    rng = np.random.default_rng(3)
    N, B, T = 128, 2, 100
    lP, lp0 = O.hmm_params(torch.from_numpy(rng.random((N, N), dtype=np.float32)))
    lo = np.log(rng.random((B, T, N), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    o = ops()
    r = {}
    for d in (False, True):
        r[d] = o.viterbi(t(lo), t(lP), t(lp0), o.OBS_LOG, dense_plan(t(lP), d))[1].cpu().numpy()
    assert np.array_equal(r[False], r[True])
