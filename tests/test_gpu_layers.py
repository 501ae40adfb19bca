"""GPU: the reference's layer call sequences (tests/golden/make_golden.py, the same calls the
reference's tests and BASELINE configs make) through the drop-in layers, against the
reference's own outputs.

Tolerances: the layers derive log_P / emissions on the GPU (softmax, sigmoid, Gaussian
scores), which may differ from the reference's torch-CPU bits by an ulp; the recursions
then carry the FB tolerances of test_gpu_kernels.py.  Viterbi states are compared exactly.
"""
import numpy as np
import pytest
import torch

import pytorch_hmm_amd as ph
from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


def t(a):
    return torch.as_tensor(np.asarray(a)).to(DEV)


@torch.no_grad()
def test_hmmlayer_c1_call_sequence():
    g = golden("hmmlayer_c1")
    torch.manual_seed(0)
    layer = ph.HMMLayer(5).to(DEV)
    x = t(g["x"])
    layer.train()
    post1 = layer(x)                                   # call 1: FB posteriors
    np.testing.assert_allclose(post1.cpu().numpy(), g["posterior1"], atol=2e-4)
    layer.eval()
    onehot2, align2 = layer(x, return_alignment=True)  # call 2: Viterbi one-hot
    assert np.array_equal(align2.cpu().numpy(), g["align2"])
    assert np.array_equal(onehot2.cpu().numpy(), g["onehot2"])
    states3, delta3 = layer.align(x)                   # call 3
    assert np.array_equal(states3.cpu().numpy(), g["states3"])
    np.testing.assert_allclose(delta3.cpu().numpy(), g["log_delta3"], rtol=2e-6, atol=2e-5)
    layer.train()
    loss4 = layer.compute_loss(x)                      # call 4: -mean compute_likelihood
    np.testing.assert_allclose(loss4.cpu().numpy(), g["loss4"], rtol=1e-5)


@torch.no_grad()
@pytest.mark.parametrize("name,K,D,seed", [("gaussian_c2", 64, 80, 0), ("gaussian_small", 3, 5, 1)])
def test_gaussian_layer(name, K, D, seed):
    g = golden(name)
    torch.manual_seed(seed)
    layer = ph.GaussianHMMLayer(K, D).to(DEV)
    x = t(g["x"])
    lp = layer._compute_gaussian_log_probs(x).detach().cpu().numpy()
    np.testing.assert_allclose(lp, g["log_probs"], rtol=2e-6, atol=2e-5)
    layer.train()
    post = layer(x)
    np.testing.assert_allclose(post.cpu().numpy(), g["posterior"], atol=2e-4)
    layer.eval()
    onehot, states = layer.hmm_layer(torch.exp(layer._compute_gaussian_log_probs(x)), return_alignment=True)
    assert np.array_equal(states.cpu().numpy(), g["states"])
    np.testing.assert_allclose(layer.compute_loss(x).cpu().numpy(), g["loss"], rtol=1e-5)


@pytest.mark.parametrize("name,S,D,C,seed", [("mixture_s16", 16, 80, 4, 0), ("mixture_s128", 128, 80, 4, 0),
                                             ("mixture_single", 1, 10, 1, 3)])
def test_mixture_layer(name, S, D, C, seed):
    g = golden(name)
    torch.manual_seed(seed)
    m = ph.MixtureGaussianHMMLayer(S, D, num_components=C).to(DEV)
    x = t(g["x"])
    with torch.no_grad():
        lp = m.get_observation_log_probs(x)
    np.testing.assert_allclose(lp.cpu().numpy(), g["log_probs"], rtol=2e-6, atol=2e-5)
    states, scores = m(x, return_log_probs=True)   # grad-enabled path (ViterbiScore)
    scores = scores.detach()
    assert np.array_equal(states.cpu().numpy(), g["states"])
    np.testing.assert_allclose(scores.cpu().numpy(), g["scores"], rtol=2e-6)
    s2, none = m(x)
    assert none is None and torch.equal(s2, states)


def test_mixture_full_covariance():
    """covariance_type='full' (mixture_gaussian.py:216-240): whitening GEMMs vs the
    reference's triangular solve (fixture made by the reference; fp32 rounding differs, so the
    log-probs match to 1e-4 and the Viterbi path is compared on the reference's own log-probs
    bit-exactly, and end to end)."""
    g = golden("mixture_full")
    m = ph.MixtureGaussianHMMLayer(6, 7, num_components=3, covariance_type="full").to(DEV)
    with torch.no_grad():
        for k in ("transition_logits", "mixture_weights_logits", "means", "cholesky_params"):
            getattr(m, k).copy_(t(g[k]))
    x = t(g["x"])
    with torch.no_grad():
        lp = m.get_observation_log_probs(x)
    np.testing.assert_allclose(lp.cpu().numpy(), g["log_probs"], rtol=1e-4, atol=1e-4)
    with torch.no_grad():
        states, scores = m._viterbi_decode(t(g["log_probs"]), t(g["log_T"]))
    assert np.array_equal(states.cpu().numpy(), g["states"])
    np.testing.assert_allclose(scores.cpu().numpy(), g["scores"], rtol=2e-6)
    s2, sc2 = m(x, return_log_probs=True)
    assert np.array_equal(s2.cpu().numpy(), g["states"])
    np.testing.assert_allclose(sc2.detach().cpu().numpy(), g["scores"], rtol=1e-4)
    # trainable: gradients reach the Cholesky parameters through the whitening GEMMs
    sc2.sum().backward()
    assert m.cholesky_params.grad is not None and torch.isfinite(m.cholesky_params.grad).all()


@pytest.mark.parametrize("name", ["mixture_tied", "mixture_spherical"])
def test_mixture_layer_covariance(name):
    """covariance_type='tied' / 'spherical' (mixture_gaussian.py:242-269) against the reference's
    fixtures (tests/golden/make_golden.py fx_mixture_cov): the scorer takes per-dimension
    log-variances (the tied vector or the spherical scalar repeated over D) in fp64, so the
    emissions are within the diag scorer's rtol 2e-6 of the reference's fp32 expression, and the
    decoded states are bit-exact end to end."""
    g = golden(name)
    cov = str(g["covariance_type"])
    S, C, D = g["means"].shape
    m = ph.MixtureGaussianHMMLayer(S, D, num_components=C, covariance_type=cov).to(DEV)
    with torch.no_grad():
        for k in ("transition_logits", "mixture_weights_logits", "means", "log_vars"):
            getattr(m, k).copy_(t(g[k]))
    x = t(g["x"])
    with torch.no_grad():
        lp = m.get_observation_log_probs(x)
    np.testing.assert_allclose(lp.cpu().numpy(), g["log_probs"], rtol=2e-6, atol=2e-5)
    with torch.no_grad():
        states, scores = m(x, return_log_probs=True)
    assert np.array_equal(states.cpu().numpy(), g["states"])
    np.testing.assert_allclose(scores.cpu().numpy(), g["scores"], rtol=2e-6)
    # given the reference's own log-probs the decode is bit-exact, score included
    with torch.no_grad():
        s2, sc2 = m._viterbi_decode(t(g["log_probs"]), t(g["log_T"]))
    assert np.array_equal(s2.cpu().numpy(), g["states"]) and np.array_equal(sc2.cpu().numpy(), g["scores"])
    # trainable through the emission's analytic backward
    s3, sc3 = m(x, return_log_probs=True)
    sc3.sum().backward()
    assert m.log_vars.grad is not None and torch.isfinite(m.log_vars.grad).all()


@pytest.mark.parametrize("name", ["gaussian_spherical", "gaussian_full"])
def test_gaussian_layer_covariance(name):
    """GaussianHMMLayer 'spherical' (hmm_layer.py:289-298) and 'full' (its diagonal, :311-319)
    with D = 6 (real, non-underflowing emissions) against the reference's call sequence."""
    g = golden(name)
    cov = str(g["covariance_type"])
    K, D = g["means"].shape
    layer = ph.GaussianHMMLayer(K, D, covariance_type=cov).to(DEV)
    with torch.no_grad():
        layer.means.copy_(t(g["means"]))
        layer.log_scales.copy_(t(g["log_scales"]))
        layer.hmm_layer.log_transition_logits.copy_(t(g["logits"]))
        layer.hmm_layer.log_initial_logits.copy_(t(g["init_logits"]))
    x = t(g["x"])
    with torch.no_grad():
        lp = layer._compute_gaussian_log_probs(x).cpu().numpy()
        np.testing.assert_allclose(lp, g["log_probs"], rtol=2e-6, atol=2e-5)
        layer.train()
        post = layer(x)
        np.testing.assert_allclose(post.cpu().numpy(), g["posterior"], atol=2e-4)
        layer.eval()
        onehot, states = layer.hmm_layer(torch.exp(layer._compute_gaussian_log_probs(x)), return_alignment=True)
        assert np.array_equal(states.cpu().numpy(), g["states"])
        assert np.array_equal(onehot.cpu().numpy(), g["onehot"])
        np.testing.assert_allclose(layer.compute_loss(x).cpu().numpy(), g["loss"], rtol=1e-5)


@pytest.mark.parametrize("name,S,D,Dm,seed", [("hsmm_s5", 5, 30, 20, 0), ("hsmm_s2", 2, 3, 2, 1),
                                              ("hsmm_s8", 8, 20, 10, 2)])
def test_hsmm_layer(name, S, D, Dm, seed):
    g = golden(name)
    torch.manual_seed(seed)
    h = ph.HSMMLayer(S, D, max_duration=Dm).to(DEV)
    x = t(g["x"])
    np.testing.assert_allclose(h.get_observation_log_probs(x).detach().cpu().numpy(), g["log_probs"],
                               rtol=2e-6, atol=2e-5)
    states, scores = h(x)
    assert np.array_equal(states.cpu().numpy(), g["states"])
    np.testing.assert_allclose(scores.cpu().numpy(), g["scores"], rtol=2e-6)


def test_mixture_inference_tables_follow_data_writes():
    """The no-grad forward caches log T / log w per parameter version: writes through
    .data are invisible to the version counter, refresh_tables() drops the cache, and a parameter
    replaced by vector_to_parameters (a new .data pointer) is seen without it.  After each, the
    decode equals a fresh layer holding the same parameters."""
    torch.manual_seed(0)
    S, D, C, B, T = 16, 8, 3, 2, 60
    m = ph.MixtureGaussianHMMLayer(S, D, num_components=C).to(DEV).eval()
    x = torch.randn(B, T, D, device=DEV)

    def fresh():
        f = ph.MixtureGaussianHMMLayer(S, D, num_components=C).to(DEV).eval()
        f.load_state_dict(m.state_dict())
        return f(x)[0]

    s0 = m(x)[0]
    with torch.no_grad():
        m.transition_logits.data.copy_(torch.randn_like(m.transition_logits) * 4)
        m.mixture_weights_logits.data -= 3 * torch.randn_like(m.mixture_weights_logits)
    m.refresh_tables()
    s1 = m(x)[0]
    assert torch.equal(s1, fresh())
    assert not torch.equal(s0, s1)
    vec = torch.nn.utils.parameters_to_vector(m.parameters())
    torch.nn.utils.vector_to_parameters(vec + 0.5 * torch.randn_like(vec), m.parameters())
    assert torch.equal(m(x)[0], fresh())
