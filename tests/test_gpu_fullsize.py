"""GPU parity at the BASELINE shapes, against the reference's own outputs.

tests/golden/fullsize_ns.npz holds the reference's results for the north-star workload
(HMMPyTorch, left_to_right(0.7), B=32, T=2000, N=128; /root/reference/pytorch_hmm/hmm.py:95-117
forward-backward, :162-178 Viterbi) on machine-independent PCG64 inputs that are regenerated
here bit-for-bit (input_sha256 checked).  tests/golden/fullsize_mixture.npz does the same for
BASELINE config 3 (MixtureGaussianHMMLayer(128, 80, num_components=4), mixture_gaussian.py:157-214,
290-338).  Both ops run through the bench's path (HMMPyTorch -> transition plan -> ops), once on
the banded chains and once with dense plans (HMM355_PLAN_DENSE: the dense chains).

Tolerances (north_star: "within 1e-4 on log-likelihoods, bit-exact on Viterbi state paths"):
  * Viterbi states and the final trellis row: bit-exact vs the reference.
  * loglik = LSE(log alpha_{T-1}): rtol 1e-4 vs the reference (whose own fp32 drift from fp64 is
    1.44e-5 relative here) and rtol 2e-6 vs the fp64 C oracle.
  * posterior rows: atol 5e-4 vs the reference (its fp32 drift from fp64 reaches 3.1e-4 at this
    T), atol 2e-5 vs the fp64 oracle on every row.
  * compute_likelihood (the reference's saturating value): rtol 1e-6.
"""
import hashlib
import os

import numpy as np
import pytest
import torch

from conftest import force_dense_plans, golden
from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ns():
    g = golden("fullsize_ns")
    B, T, N = (int(v) for v in g["shape"])
    obs = O.uniform_obs(int(g["seed"]), (B, T, N))
    assert hashlib.sha256(obs.tobytes()).hexdigest() == str(g["input_sha256"]), "PCG64 input drift"
    # the fp64 oracle on the same fp32 log-emissions the GPU forms (correctly rounded log)
    lo_cr = np.log((obs + np.float32(1e-8)).astype(np.float64)).astype(np.float32)
    _, _, post64, ll64 = O.c_fb64(lo_cr, g["log_P"], g["log_p0"])
    cs, cd, _ = O.c_viterbi(lo_cr, g["log_P"], g["log_p0"])
    return g, obs, lo_cr, post64, ll64, cs, cd


@pytest.mark.parametrize("dense", [False, True], ids=["banded", "dense"])
@torch.no_grad()
def test_north_star_shape_vs_reference(ns, dense, monkeypatch):
    import pytorch_hmm_amd as ph
    g, obs, lo_cr, post64, ll64, cs, cd = ns
    if dense:
        force_dense_plans(monkeypatch)
    N = obs.shape[-1]
    hmm = ph.HMMPyTorch(ph.create_left_to_right_matrix(N, 0.7))
    # parameter bits are the reference's (hmm.py:39-55)
    assert np.array_equal(hmm.log_P.numpy(), g["log_P"]) and np.array_equal(hmm.log_p0.numpy(), g["log_p0"])
    x = torch.from_numpy(obs).to(DEV)

    states, delta = hmm.viterbi_decode(x)
    states, delta = states.cpu().numpy(), delta.cpu().numpy()
    assert np.array_equal(states.astype(np.uint8), g["states"]), "Viterbi path != reference"
    assert np.array_equal(delta[:, -1].view(np.int32), g["delta_last"].view(np.int32))
    assert np.array_equal(states, cs) and np.array_equal(delta.view(np.int32), cd.view(np.int32))

    post, fwd, bwd = hmm.forward_backward(x)
    post = post.cpu().numpy()
    rows = g["post_rows"]
    np.testing.assert_allclose(post[:, rows], g["posterior_rows"], atol=5e-4, rtol=0)
    np.testing.assert_allclose(post, post64, atol=2e-5, rtol=0)
    ll = hmm.log_likelihood(x).cpu().numpy()
    np.testing.assert_allclose(ll, g["loglik"], rtol=1e-4)
    np.testing.assert_allclose(ll, ll64, rtol=2e-6)
    lik = hmm.compute_likelihood(x).cpu().numpy()
    np.testing.assert_allclose(lik, g["compute_likelihood"], rtol=1e-6)
    # forward = exp(log alpha), backward = exp(log beta): relative 1e-4 where representable
    # (the last forward row has underflowed to 0 at this T, as the reference's has)
    for ours, ref in ((fwd[:, -1], g["log_alpha_last"]), (bwd[:, 0], g["log_beta_first"])):
        ref = np.exp(ref.astype(np.float32))
        ours = ours.cpu().numpy()
        big = ref > 1e-30
        np.testing.assert_allclose(ours[big], ref[big], rtol=1e-4)
        assert np.all(np.abs(ours[~big]) < 1e-29)


@pytest.mark.parametrize("dense", [False, True], ids=["banded", "dense"])
@torch.no_grad()
def test_north_star_ops_with_plan(ns, dense, monkeypatch):
    """The exact calls bench.py times: ops.forward_backward / ops.viterbi with the cached plan
    (OBS_PROB, all three FB outputs)."""
    import pytorch_hmm_amd as ph
    from pytorch_hmm_amd import ops
    g, obs, lo_cr, post64, ll64, cs, cd = ns
    if dense:
        force_dense_plans(monkeypatch)
    hmm = ph.HMMPyTorch(ph.create_left_to_right_matrix(obs.shape[-1], 0.7))
    lP, lp0, plan = hmm._device_params(torch.device(DEV, 0))
    x = torch.from_numpy(obs).to(DEV)
    for _ in range(2):   # a second call reuses the plan (graph-replay equivalence)
        states, delta, final = ops.viterbi(x, lP, lp0, ops.OBS_PROB, plan)
        post, fwd, bwd, loglik, lik_ref = ops.forward_backward(x, lP, lp0, ops.OBS_PROB, 7, plan)
        assert np.array_equal(states.cpu().numpy().astype(np.uint8), g["states"])
        assert np.array_equal(final.cpu().numpy(), g["delta_last"].max(-1))
        np.testing.assert_allclose(post.cpu().numpy(), post64, atol=2e-5, rtol=0)
        np.testing.assert_allclose(loglik.cpu().numpy(), ll64, rtol=2e-6)
        np.testing.assert_allclose(lik_ref.cpu().numpy(), g["compute_likelihood"], rtol=1e-6)


@pytest.fixture(scope="module")
def mix():
    g = golden("fullsize_mixture")
    B, T, D, S, C = (int(v) for v in g["shape"])
    x = O.uniform_obs(int(g["x_seed"]), (B, T, D), -2.0, 2.0)
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["input_sha256"]), "PCG64 input drift"
    return g, x


@pytest.mark.parametrize("dense", [False, True], ids=["auto", "dense"])
def test_config3_mixture_vs_reference(mix, dense, monkeypatch):
    """BASELINE config 3 at full size: GMM emission (rtol 2e-6 of the reference's rows), then the
    Viterbi states and final scores; the random learned matrix takes the dense chain either way."""
    import pytorch_hmm_amd as ph
    g, x = mix
    if dense:
        force_dense_plans(monkeypatch)
    B, T, D, S, C = (int(v) for v in g["shape"])
    m = ph.MixtureGaussianHMMLayer(S, D, num_components=C)
    with torch.no_grad():
        for k in ("transition_logits", "mixture_weights_logits", "means", "log_vars"):
            getattr(m, k).copy_(torch.from_numpy(g[k]))
    m = m.to(DEV)
    xd = torch.from_numpy(x).to(DEV)
    with torch.no_grad():
        lp = m.get_observation_log_probs(xd)
        states, scores = m(xd, return_log_probs=True)
    lp = lp.cpu().numpy()
    np.testing.assert_allclose(lp[:, :4], g["lp_rows"], rtol=2e-6, atol=2e-5)
    assert np.array_equal(states.cpu().numpy().astype(np.uint8), g["states"]), "mixture Viterbi path != reference"
    np.testing.assert_allclose(scores.cpu().numpy(), g["scores"], rtol=2e-6)
    # given the GPU's own emissions the recursion is bit-exact vs the C oracle
    lT = O.mixture_log_transitions(torch.from_numpy(g["transition_logits"])).numpy()
    cs, cd, _ = O.c_viterbi(lp, lT, O.mixture_init_vector(S).numpy())
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(scores.cpu().numpy(), cd[:, -1].max(-1))
