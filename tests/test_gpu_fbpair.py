"""GPU: forward-backward with both chains of a sequence in one workgroup (csrc/fbpair.h,
HMM355_FB_PAIR, forced with pair=True) against the two-kernel path (fb_recur + fb_posterior) on the same inputs.

Both paths run the same chain code, so the scaled rows and log-scales are the same bits; the
pair kernel forms forward / backward / loglik / lik_ref from them with the same formulas
(identical bits) and the posterior as x*y / sum(x*y) (the two-kernel path max-normalises
first: ~1 ulp apart), in the helper waves, while the rows are still in LDS (or after one HBM
round trip for the chain that reaches a time step second).  Contract: rtol 2e-6 (posterior
atol 1e-12), over block-edge lengths,
padded state counts, every banded factory matrix, OBS_LOG, partial output masks, and the
wrong-hint fallback (a dense matrix whose plan claims to be banded).  Reference semantics:
hmm.py:66-130 (forward_backward), :186-211 (compute_likelihood)."""
import numpy as np
import pytest
import torch

from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def ops():
    from pytorch_hmm_amd import ops as o
    return o


def matrix(N, kind, rng):
    if kind == "l2r":
        return O.left_to_right_matrix(N, 0.7).numpy()
    if kind in ("left_to_right_skip", "circular", "ergodic"):
        return O.transition_matrix(N, kind).numpy()
    if kind == "band5":
        P = np.zeros((N, N), np.float32)
        for i in range(N):
            for o in range(max(0, i - 2), min(N, i + 3)):
                P[i, o] = rng.random() + 0.05
        return P
    return rng.random((N, N)).astype(np.float32) + 0.01  # dense


def run_both(obs, lP, lp0, mode, mask):
    o = ops()
    plan = o.make_plan(lP)
    plain = plan.clone()  # no banded attribute: the two-kernel path
    a = o.forward_backward(obs, lP, lp0, mode, mask, plan, pair=True)
    b = o.forward_backward(obs, lP, lp0, mode, mask, plain)
    return plan, a, b


def check(a, b, mask):
    o = ops()
    names = ["posterior", "forward", "backward", "loglik", "lik_ref"]
    bits = [o.FB_POSTERIOR, o.FB_FORWARD, o.FB_BACKWARD, 0, 0]
    for name, x, y, bit in zip(names, a, b, bits):
        if bit and not (mask & bit):
            continue
        # the posterior is normalised once (x*y / sum) instead of max-then-sum: ~1 ulp apart
        atol = 1e-12 if name == "posterior" else 1e-30
        np.testing.assert_allclose(x.cpu().numpy(), y.cpu().numpy(), rtol=2e-6, atol=atol, err_msg=name)


@pytest.mark.parametrize("kind", ["l2r", "left_to_right_skip", "circular", "ergodic", "band5"])
@pytest.mark.parametrize("B,T,N", [(2, 300, 128), (3, 77, 40), (2, 129, 64), (1, 2000, 128), (2, 33, 100)])
def test_pair_matches_two_kernel_path(kind, B, T, N):
    rng = np.random.default_rng(N * 31 + T)
    P = torch.from_numpy(matrix(N, kind, rng))
    lP, lp0 = O.hmm_params(P)
    obs = torch.softmax(torch.from_numpy(rng.standard_normal((B, T, N)).astype(np.float32)), -1)
    plan, a, b = run_both(obs.to(DEV), lP.to(DEV), lp0.to(DEV), ops().OBS_PROB, 7)
    assert plan._hmm355_banded == (kind != "circular")  # the wrap-around band is as wide as N
    check(a, b, 7)


@pytest.mark.parametrize("T", [1, 2, 15, 16, 17, 31, 32, 33, 47, 48, 49, 64, 65, 80, 95, 96, 97])
def test_pair_short_and_block_edge_lengths(T):
    rng = np.random.default_rng(T)
    N = 128
    lP, lp0 = O.hmm_params(O.left_to_right_matrix(N, 0.7))
    obs = torch.from_numpy(rng.random((3, T, N), dtype=np.float32))
    _, a, b = run_both(obs.to(DEV), lP.to(DEV), lp0.to(DEV), ops().OBS_PROB, 7)
    check(a, b, 7)
    # and against the oracle (reference op sequence), posterior within the FB tolerance
    p_ref = O.forward_backward(obs, lP, lp0)[0].numpy()
    np.testing.assert_allclose(a[0].cpu().numpy(), p_ref, atol=2e-4)


@pytest.mark.parametrize("mask", [1, 2, 4, 3, 6, 0])
def test_pair_output_masks(mask):
    rng = np.random.default_rng(mask)
    lP, lp0 = O.hmm_params(O.transition_matrix(64, "ergodic"))
    obs = torch.from_numpy(rng.random((2, 250, 64), dtype=np.float32))
    _, a, b = run_both(obs.to(DEV), lP.to(DEV), lp0.to(DEV), ops().OBS_PROB, mask)
    check(a, b, mask)


def test_pair_obs_log_peaked_emissions():
    # Gaussian-like log-emissions far below -87 (the row-max shift of OBS_LOG)
    rng = np.random.default_rng(5)
    B, T, N = 3, 500, 128
    lo = (-250.0 + 40.0 * rng.standard_normal((B, T, N))).astype(np.float32)
    lP, lp0 = O.hmm_params(O.left_to_right_matrix(N, 0.7))
    _, a, b = run_both(torch.from_numpy(lo).to(DEV), lP.to(DEV), lp0.to(DEV), ops().OBS_LOG, 7)
    check(a, b, 7)
    _, _, post64, ll64 = O.c_fb64(lo, lP.numpy(), lp0.numpy())
    np.testing.assert_allclose(a[0].cpu().numpy(), post64, atol=2e-5)
    np.testing.assert_allclose(a[3].cpu().numpy(), ll64, rtol=2e-6)


def test_pair_wrong_hint_falls_back_to_dense():
    rng = np.random.default_rng(9)
    B, T, N = 2, 200, 128
    lP, lp0 = O.hmm_params(torch.from_numpy(matrix(N, "dense", rng)))
    obs = torch.from_numpy(rng.random((B, T, N), dtype=np.float32)).to(DEV)
    o = ops()
    plan = o.make_plan(lP.to(DEV))
    assert not plan._hmm355_banded
    wrong = plan.clone()
    wrong._hmm355_banded = True  # the C ABI then runs the pair kernel, which finds dense chains
    a = o.forward_backward(obs, lP.to(DEV), lp0.to(DEV), o.OBS_PROB, 7, wrong, pair=True)
    b = o.forward_backward(obs, lP.to(DEV), lp0.to(DEV), o.OBS_PROB, 7, plan)
    check(a, b, 7)
