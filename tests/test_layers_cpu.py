"""CPU: the layer wrappers keep the reference's parameter names, shapes and initial values
(state_dict drop-in), the same validation errors, and fail loudly (no CPU fallback) when
asked to run on host tensors."""
import numpy as np
import pytest
import torch

import pytorch_hmm_amd as ph
from conftest import golden


def eq(a, b):
    return np.array_equal(np.asarray(a), np.asarray(b))


def test_hmmlayer_init_matches_reference():
    g = golden("hmmlayer_c1")
    torch.manual_seed(0)
    layer = ph.HMMLayer(5)
    sd = layer.state_dict()
    assert set(sd) == {"log_transition_logits", "log_initial_logits"}
    assert eq(sd["log_transition_logits"], g["logits"]) and eq(sd["log_initial_logits"], g["init_logits"])
    assert eq(torch.randn(2, 100, 5), g["x"])  # same RNG stream consumption as the reference
    fixed = ph.HMMLayer(5, learnable_transitions=False)
    assert set(fixed.state_dict()) == {"transition_matrix", "log_initial_logits"}


@pytest.mark.parametrize("name,K,D,seed", [("gaussian_c2", 64, 80, 0), ("gaussian_small", 3, 5, 1)])
def test_gaussian_layer_init_matches_reference(name, K, D, seed):
    g = golden(name)
    torch.manual_seed(seed)
    layer = ph.GaussianHMMLayer(K, D)
    sd = layer.state_dict()
    assert set(sd) == {"hmm_layer.log_transition_logits", "hmm_layer.log_initial_logits", "means", "log_scales"}
    assert eq(sd["means"], g["means"]) and eq(sd["log_scales"], g["log_scales"])
    assert eq(sd["hmm_layer.log_transition_logits"], g["logits"])
    for cov, shape in (("full", (K, D, D)), ("spherical", (K, 1))):
        assert tuple(ph.GaussianHMMLayer(K, D, covariance_type=cov).log_scales.shape) == shape
    with pytest.raises(ValueError):
        ph.GaussianHMMLayer(K, D, covariance_type="bogus")


@pytest.mark.parametrize("name,S,D,C,seed", [("mixture_s16", 16, 80, 4, 0), ("mixture_single", 1, 10, 1, 3)])
def test_mixture_layer_init_matches_reference(name, S, D, C, seed):
    g = golden(name)
    torch.manual_seed(seed)
    m = ph.MixtureGaussianHMMLayer(S, D, num_components=C)
    for k in ("transition_logits", "mixture_weights_logits", "means", "log_vars"):
        assert eq(m.state_dict()[k], g[k]), k
    fixed = ph.MixtureGaussianHMMLayer(4, 3, learnable_transitions=False)
    P = fixed.get_transition_matrix()
    assert torch.allclose(P.sum(1), torch.ones(4)) and P[0, 0] == 0.8 and P[3, 3] == 1.0
    for cov, shape in (("tied", (D,)), ("spherical", (S, C))):
        assert tuple(ph.MixtureGaussianHMMLayer(S, D, C, covariance_type=cov).log_vars.shape) == shape
    with pytest.raises(ValueError):
        ph.MixtureGaussianHMMLayer(S, D, C, covariance_type="bogus")


@pytest.mark.parametrize("name,S,D,Dm,seed", [("hsmm_s5", 5, 30, 20, 0), ("hsmm_s8", 8, 20, 10, 2)])
def test_hsmm_layer_tables_match_reference(name, S, D, Dm, seed):
    g = golden(name)
    torch.manual_seed(seed)
    h = ph.HSMMLayer(S, D, max_duration=Dm)
    for k in ("transition_logits", "observation_means", "observation_log_vars", "duration_shape", "duration_rate"):
        assert eq(h.state_dict()[k], g[k]), k
    with torch.no_grad():
        assert eq(torch.log(h.get_duration_probabilities() + h.eps), g["dur_log_probs"])
        assert eq(torch.log(h.get_transition_matrix() + h.eps), g["log_T"])
    for dist, names in (("poisson", {"duration_lambda"}), ("weibull", {"duration_scale", "duration_concentration"})):
        assert names <= set(ph.HSMMLayer(S, D, duration_distribution=dist).state_dict())
    with pytest.raises(ValueError):
        ph.HSMMLayer(S, D, duration_distribution="bogus")


def test_hmm_validation_errors_match_reference():
    with pytest.raises(ValueError):
        ph.HMMPyTorch(torch.rand(3, 4))
    with pytest.raises(ValueError):
        ph.HMMPyTorch(torch.rand(3, 3, 3))
    with pytest.raises(ValueError):
        ph.HMMPyTorch(torch.rand(3, 3), torch.rand(4))
    h = ph.HMMPyTorch(ph.create_left_to_right_matrix(4, 0.7))
    assert torch.allclose(h.P.sum(1), torch.ones(4))
    with pytest.raises(AssertionError):
        h.forward_backward(torch.rand(1, 10, 5))
    with pytest.raises(AssertionError):
        h.viterbi_decode(torch.rand(10, 3))
    layer = ph.HMMLayer(4)
    with pytest.raises(ValueError):
        layer(torch.randn(2, 10, 5))


def test_no_cpu_fallback():
    """The product path has no host implementation: CPU tensors raise instead of silently
    computing somewhere else."""
    h = ph.HMMPyTorch(ph.create_left_to_right_matrix(4, 0.7))
    obs = torch.rand(1, 10, 4)
    for fn in (h.forward_backward, h.viterbi_decode, h.compute_likelihood):
        with pytest.raises(RuntimeError):
            with torch.no_grad():
                fn(obs)


def test_mixture_full_init_and_cholesky_match_reference():
    """covariance_type='full': the reference's draws (mixture_gaussian.py:59-105) and its
    Cholesky reconstruction (:271-289); the whitening form's math (L^-1 x - L^-1 mu) equals the
    reference's triangular solve on the fixture's parameters (torch-CPU, fp64)."""
    g = golden("mixture_full")
    torch.manual_seed(11)
    m = ph.MixtureGaussianHMMLayer(6, 7, num_components=3, covariance_type="full")
    base = m.state_dict()
    diff = g["cholesky_params"] - base["cholesky_params"].numpy()   # the fixture's perturbation only
    assert eq(base["means"], g["means"]) and eq(base["transition_logits"], g["transition_logits"])
    assert np.abs(diff).max() < 1.0
    with torch.no_grad():
        m.cholesky_params.copy_(torch.from_numpy(g["cholesky_params"]))
    L = m._get_cholesky_factors().double()
    x = torch.from_numpy(g["x"]).double()
    mu = m.means.detach().double()
    W = torch.linalg.inv(L)
    z1 = torch.einsum("scij,btj->btsci", W, x) - torch.einsum("scij,scj->sci", W, mu)
    z2 = torch.linalg.solve_triangular(L[None, None], (x[:, :, None, None, :] - mu[None, None]).unsqueeze(-1),
                                       upper=False).squeeze(-1)
    assert torch.allclose(z1, z2, rtol=1e-9, atol=1e-9)


def test_hsmm_layer_rejects_sizes_beyond_the_kernel():
    with pytest.raises(ValueError):
        ph.HSMMLayer(1025, 4)
    with pytest.raises(ValueError):
        ph.HSMMLayer(8, 4, max_duration=1025)
    ph.HSMMLayer(64, 4, max_duration=63)    # BASELINE config 5 is S = 64, Dmax = 40
    ph.HSMMLayer(64, 4, max_duration=127)   # the geometries of csrc/hsmm.hip
    ph.HSMMLayer(128, 4, max_duration=63)
    ph.HSMMLayer(100, 4)                    # the reference's default max_duration = 50
    ph.HSMMLayer(65, 4, max_duration=64)    # the general form of csrc/hsmm_wide.hip
    ph.HSMMLayer(300, 4)
