"""CPU: the NeuralHMM drop-in's networks (pytorch_hmm_amd/neural.py) against the reference's
golden vectors — state_dict compatibility, the observation / transition networks' outputs
(the recursion inputs), and the no-CPU-fallback / error behaviour.  The recursions
themselves are GPU-only (tests/test_gpu_neural.py)."""
import numpy as np
import pytest
import torch

from conftest import golden
from pytorch_hmm_amd.neural import NeuralHMM, ContextualNeuralHMM

CASES = [("neural_mlp_small", "mlp", "gaussian"), ("neural_static", "mlp", "gaussian"),
         ("neural_rnn", "rnn", "gaussian"), ("neural_mixture", "mlp", "mixture"), ("neural_k32", "mlp", "gaussian")]


def _sd(g):
    return {k[4:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd__")}


def _module(g, ttype, otype):
    K, D, C, H = (int(v) for v in g["config"])
    m = NeuralHMM(num_states=K, observation_dim=D, context_dim=C, hidden_dim=H, transition_type=ttype,
                  observation_type=otype)
    return m


@pytest.mark.parametrize("name,ttype,otype", CASES)
def test_state_dict_compatible(name, ttype, otype):
    g = golden(name)
    m = _module(g, ttype, otype)
    ours = m.state_dict()
    ref = _sd(g)
    assert set(ours) == set(ref)
    for k in ref:
        assert tuple(ours[k].shape) == tuple(ref[k].shape), k
    m.load_state_dict(ref)


@pytest.mark.parametrize("name,ttype,otype", CASES)
def test_networks_reproduce_recursion_inputs(name, ttype, otype):
    """neural.py:182-209 (observation model, eval) and :64-120 (transition model) on CPU."""
    g = golden(name)
    m = _module(g, ttype, otype)
    m.load_state_dict(_sd(g))
    m.eval()
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        lo = m.observation_model(x)
        np.testing.assert_allclose(lo.numpy(), g["log_obs"], rtol=1e-5, atol=1e-5)
        B, T, _ = x.shape
        ctx = torch.from_numpy(g["ctx"]) if g["ctx"].size else None
        lt = m._log_transitions(B, T, ctx)
        np.testing.assert_allclose(lt.numpy(), g["log_trans"], rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(m._log_initial().numpy(), g["log_init"])


def test_contextual_encode_context():
    g = golden("contextual_small")
    K, D, V, LD, PD = (int(v) for v in g["config"])
    m = ContextualNeuralHMM(K, D, phoneme_vocab_size=V, linguistic_context_dim=LD, prosody_dim=PD)
    m.load_state_dict(_sd(g))
    m.eval()
    with torch.no_grad():
        ctx = m.encode_context(torch.from_numpy(g["phonemes"]), torch.from_numpy(g["prosody"]))
    np.testing.assert_allclose(ctx.numpy(), g["ctx"], rtol=1e-6, atol=1e-6)


def test_train_mode_observation_model_draws_per_state_masks():
    """neural.py:195-200 calls feature_net once per state: in train mode every state gets its
    own dropout masks, so state columns differ even with identical embeddings."""
    torch.manual_seed(0)
    m = NeuralHMM(num_states=4, observation_dim=6, context_dim=3, hidden_dim=32)
    with torch.no_grad():
        m.observation_model.state_embedding.weight.zero_()
    m.train()
    with torch.no_grad():
        lp = m.observation_model(torch.randn(1, 10, 6))
    assert lp.shape == (1, 10, 4)
    assert not torch.allclose(lp[..., 0], lp[..., 1])
    m.eval()
    with torch.no_grad():
        lp = m.observation_model(torch.randn(1, 10, 6))
    assert torch.allclose(lp[..., 0], lp[..., 1])


def test_cpu_tensors_have_no_fallback():
    m = NeuralHMM(num_states=4, observation_dim=6, context_dim=3, hidden_dim=16)
    with pytest.raises(RuntimeError, match="ROCm"):
        m(torch.randn(1, 5, 6), torch.randn(1, 5, 3))
    with pytest.raises(RuntimeError, match="ROCm"):
        m.viterbi_decode(torch.randn(1, 5, 6), torch.randn(1, 5, 3))


def test_context_network_without_context_raises_like_reference():
    """With a transition network and no context the reference falls through to the missing
    static matrix (neural.py:382-385) and raises AttributeError; so does the drop-in."""
    m = NeuralHMM(num_states=4, observation_dim=6, context_dim=3, hidden_dim=16)
    with pytest.raises(AttributeError):
        m(torch.randn(1, 5, 6))


def test_unknown_model_types_raise():
    with pytest.raises(ValueError):
        NeuralHMM(num_states=4, observation_dim=6, context_dim=3, transition_type="gru")
