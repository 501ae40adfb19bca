"""GPU parity for the time-varying recursions (csrc/tv.hip; NeuralHMM, reference
neural.py:391-519) against the reference's golden vectors (tests/golden/neural_*.npz,
contextual_small.npz — produced by the reference itself) and the C oracle
(oracle/hmm_oracle.c tv_viterbi_f32 / tv_fb_f64).

Contracts: Viterbi states and log_delta bit-exact given identical fp32 log-emissions and
log-transition tensors; forward-backward posteriors within 2e-4 absolute, forward/backward
within 1e-4 relative where representable, log-likelihoods within 1e-5 relative (fp32
kernels vs the reference's fp32 / the oracle's fp64)."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
NEURAL = ["neural_mlp_small", "neural_static", "neural_rnn", "neural_mixture", "neural_k32", "neural_k128",
          "contextual_small"]
ALL = ("posterior", "forward", "backward")


def t(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a)).to(DEV, dtype)


def ops():
    from pytorch_hmm_amd import ops as o
    return o


def check_fb(post, fwd, bwd, g):
    post, fwd, bwd = post.cpu().numpy(), fwd.cpu().numpy(), bwd.cpu().numpy()
    np.testing.assert_allclose(post, g["posterior"], atol=2e-4, rtol=0)
    for ours, ref in ((fwd, g["forward"]), (bwd, g["backward"])):
        big = ref > 1e-30
        np.testing.assert_allclose(ours[big], ref[big], rtol=1e-4)
        assert np.all(np.abs(ours[~big]) < 1e-29)


@pytest.mark.parametrize("name", NEURAL)
def test_tv_forward_backward_vs_reference(name):
    g = golden(name)
    o = ops()
    mask = o.FB_POSTERIOR | o.FB_FORWARD | o.FB_BACKWARD
    post, fwd, bwd, loglik, lik_ref = o.tv_forward_backward(t(g["log_obs"]), t(g["log_trans"]), t(g["log_init"]),
                                                            mask)
    check_fb(post, fwd, bwd, g)
    ll = np.logaddexp.reduce(g["log_forward"][:, -1].astype(np.float64), axis=-1)
    np.testing.assert_allclose(loglik.cpu().numpy(), ll, rtol=1e-5)
    np.testing.assert_allclose(lik_ref.cpu().numpy(), g["compute_likelihood"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", NEURAL)
def test_tv_viterbi_bitexact_vs_reference(name):
    g = golden(name)
    o = ops()
    states, delta = o.tv_viterbi(t(g["log_obs"]), t(g["log_trans"]), t(g["log_init"]))
    assert np.array_equal(states.cpu().numpy(), g["states"])
    assert np.array_equal(delta.cpu().numpy().view(np.int32), g["log_delta"].view(np.int32))


def _random_case(B, T, N, seed, static=False, spread=4.0):
    rng = np.random.default_rng(seed)
    lo = (rng.standard_normal((B, T, N)).astype(np.float32) * np.float32(spread) - np.float32(40.0))
    shape = (N, N) if static else (B, T, N, N)
    logits = rng.standard_normal(shape).astype(np.float32) * np.float32(2.0)
    p = np.exp(logits - logits.max(-1, keepdims=True))
    lA = np.log(p / p.sum(-1, keepdims=True) + np.float32(1e-8)).astype(np.float32)
    init = np.log(np.full(N, 1.0 / N, np.float32) + np.float32(1e-8)).astype(np.float32)
    return lo, lA, init


# shapes: ragged T around the prefetch ring (PD = 8/4/1), N padded to 64 / 128 / 256, N % 4 != 0
# (scalar matrix loads) and == 0 (float4 loads), one matrix for all steps (zero strides)
SHAPES = [(2, 1, 5, False), (3, 2, 7, False), (2, 9, 64, False), (2, 37, 100, False), (1, 19, 128, False),
          (2, 70, 33, True), (1, 11, 256, False), (2, 45, 128, True), (1, 6, 130, False)]


@pytest.mark.parametrize("B,T,N,static", SHAPES)
def test_tv_viterbi_vs_c_oracle(B, T, N, static):
    lo, lA, init = _random_case(B, T, N, B * 100 + T * 10 + N, static)
    cs, cd = O.c_tv_viterbi(lo, lA, init)
    o = ops()
    states, delta = o.tv_viterbi(t(lo), t(lA), t(init))
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(delta.cpu().numpy(), cd)


@pytest.mark.parametrize("B,T,N,static", SHAPES)
def test_tv_forward_backward_vs_fp64_oracle(B, T, N, static):
    lo, lA, init = _random_case(B, T, N, B * 100 + T * 10 + N + 1, static)
    la, lb, post64, ll64 = O.c_tv_fb64(lo, lA, init)
    o = ops()
    post, fwd, bwd, loglik, _ = o.tv_forward_backward(t(lo), t(lA), t(init), o.FB_POSTERIOR | o.FB_FORWARD
                                                      | o.FB_BACKWARD)
    np.testing.assert_allclose(post.cpu().numpy(), post64, atol=2e-5)
    np.testing.assert_allclose(loglik.cpu().numpy(), ll64, rtol=2e-6)
    # log alpha / log beta through the returned exp() values where they are representable
    f, b_ = fwd.cpu().numpy().astype(np.float64), bwd.cpu().numpy().astype(np.float64)
    ok = f > 1e-30
    np.testing.assert_allclose(np.log(f[ok]), la[ok], atol=2e-4 * max(1.0, np.abs(la[ok]).max() / 100))
    ok = b_ > 1e-30
    np.testing.assert_allclose(np.log(b_[ok]), lb[ok], atol=2e-4 * max(1.0, np.abs(lb[ok]).max() / 100))


def test_tv_expanded_view_is_not_materialised():
    """A static matrix expand()ed over (B,T) is read through zero strides (neural.py:385)."""
    lo, lA, init = _random_case(3, 40, 64, 5, static=True)
    o = ops()
    A = t(lA)
    big = A.unsqueeze(0).unsqueeze(0).expand(3, 40, 64, 64)
    s1, d1 = o.tv_viterbi(t(lo), big, t(init))
    s2, d2 = o.tv_viterbi(t(lo), A, t(init))
    assert torch.equal(s1, s2) and torch.equal(d1, d2)
    # and the time-invariant Viterbi kernel agrees (same max-plus sums)
    s3, d3, _ = o.viterbi(t(lo), A, t(init), o.OBS_LOG)
    assert torch.equal(s1, s3) and torch.equal(d1, d3)


def test_tv_full_size_properties():
    """North-star shape with per-step matrices (B=32, T=2000, N=128: 4.2 GB of log-matrices):
    posterior rows sum to 1, Viterbi states equal the C oracle on two sequences, loglik equals
    the fp64 oracle on one sequence."""
    B, T, N = 32, 2000, 128
    g = torch.Generator(device=DEV).manual_seed(0)
    lo = torch.randn(B, T, N, device=DEV, generator=g) * 3 - 50
    lA = torch.log_softmax(torch.randn(B, T, N, N, device=DEV, generator=g) * 2, dim=-1)
    init = torch.full((N,), -float(np.log(N)), device=DEV)
    o = ops()
    post, _, _, loglik, _ = o.tv_forward_backward(lo, lA, init, o.FB_POSTERIOR)
    states, delta = o.tv_viterbi(lo, lA, init)
    torch.cuda.synchronize()
    assert torch.allclose(post.sum(-1), torch.ones(B, T, device=DEV), atol=1e-5)
    sub = [0, 31]
    lo_c, lA_c = lo[sub].cpu().numpy(), lA[sub].cpu().numpy()
    cs, cd = O.c_tv_viterbi(lo_c, lA_c, init.cpu().numpy())
    assert np.array_equal(states[sub].cpu().numpy(), cs)
    assert np.array_equal(delta[sub].cpu().numpy(), cd)
    _, _, _, ll64 = O.c_tv_fb64(lo_c[:1, :200], lA_c[:1, :200], init.cpu().numpy())
    _, _, _, ll200, _ = o.tv_forward_backward(lo[:1, :200], lA[:1, :200], init, 0)
    np.testing.assert_allclose(ll200.cpu().numpy(), ll64, rtol=2e-6)


def test_tv_errors():
    o = ops()
    lo = torch.zeros(2, 5, 4, device=DEV)
    with pytest.raises(ValueError):
        o.tv_viterbi(lo, torch.zeros(2, 5, 3, 3, device=DEV), torch.zeros(4, device=DEV))
    with pytest.raises(IndexError):
        o.tv_forward_backward(lo, torch.zeros(2, 3, 4, 4, device=DEV), torch.zeros(4, device=DEV), 1)
    # T-1 matrices suffice (matrix T-1 is never read), as in the reference's loops
    o.tv_forward_backward(lo, torch.zeros(2, 4, 4, 4, device=DEV), torch.zeros(4, device=DEV), 1)
    with pytest.raises(RuntimeError):
        o.tv_viterbi(lo.cpu(), torch.zeros(4, 4), torch.zeros(4))


# ------------------------------------------------------------------- the module drop-ins
def _load_module(g, cls, **kw):
    import pytorch_hmm_amd.neural as NM
    m = getattr(NM, cls)(**kw)
    sd = {k[4:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd__")}
    m.load_state_dict(sd)
    return m.to(DEV).eval()


@pytest.mark.parametrize("name,ttype,otype", [("neural_mlp_small", "mlp", "gaussian"),
                                              ("neural_static", "mlp", "gaussian"),
                                              ("neural_rnn", "rnn", "gaussian"),
                                              ("neural_mixture", "mlp", "mixture"),
                                              ("neural_k32", "mlp", "gaussian")])
def test_neural_hmm_module_matches_reference(name, ttype, otype):
    g = golden(name)
    K, D, C, H = (int(v) for v in g["config"])
    m = _load_module(g, "NeuralHMM", num_states=K, observation_dim=D, context_dim=C, hidden_dim=H,
                     transition_type=ttype, observation_type=otype)
    x = t(g["x"])
    ctx = t(g["ctx"]) if C > 0 else None
    with torch.no_grad():
        lo = m.observation_model(x)
        np.testing.assert_allclose(lo.cpu().numpy(), g["log_obs"], rtol=1e-5, atol=1e-4)
        post, fwd, bwd = m(x, ctx)
        np.testing.assert_allclose(post.cpu().numpy(), g["posterior"], atol=1e-3)
        states, delta = m.viterbi_decode(x, ctx)
        np.testing.assert_allclose(delta.cpu().numpy(), g["log_delta"], rtol=1e-5, atol=1e-3)
        agree = (states.cpu().numpy() == g["states"]).mean()
        assert agree > 0.95, agree   # emissions are recomputed on the GPU (ulp-level differences)
        lik = m.compute_likelihood(x, ctx)
        np.testing.assert_allclose(lik.cpu().numpy(), g["compute_likelihood"], rtol=1e-4, atol=1e-3)


def test_contextual_module_matches_reference():
    g = golden("contextual_small")
    K, D, V, LD, PD = (int(v) for v in g["config"])
    m = _load_module(g, "ContextualNeuralHMM", num_states=K, observation_dim=D, phoneme_vocab_size=V,
                     linguistic_context_dim=LD, prosody_dim=PD)
    with torch.no_grad():
        post, _, _ = m.forward_with_context(t(g["x"]), t(g["phonemes"], torch.int64), t(g["prosody"]))
    np.testing.assert_allclose(post.cpu().numpy(), g["posterior"], atol=1e-3)
    assert torch.allclose(post.sum(-1), torch.ones_like(post[..., 0]), atol=1e-5)


def test_neural_hmm_reference_integration_checks():
    """tests/test_integration.py:82-116 and :309-373 of the reference on the MI355X path."""
    from pytorch_hmm_amd.neural import NeuralHMM
    for (K, D, C, H, B, T) in [(5, 8, 12, 64, 2, 20), (6, 10, 5, 32, 4, 25), (4, 6, 4, 16, 2, 15)]:
        m = NeuralHMM(num_states=K, observation_dim=D, context_dim=C, hidden_dim=H).to(DEV)
        x = torch.randn(B, T, D, device=DEV)
        ctx = torch.randn(B, T, C, device=DEV)
        post, fwd, bwd = m(x, ctx)
        states, _ = m.viterbi_decode(x, ctx)
        assert post.shape == (B, T, K) and states.shape == (B, T)
        assert torch.allclose(post.sum(-1), torch.ones(B, T, device=DEV), atol=1e-5)
        assert torch.all(states >= 0) and torch.all(states < K)
        assert post.device.type == "cuda" and states.device.type == "cuda"


# -------------------------------------------------------------------------- gradients
def _oracle_tv_grads(lo, lA, l0, kind):
    lo = torch.from_numpy(lo).double().requires_grad_(True)
    lA = torch.from_numpy(lA).double().requires_grad_(True)
    l0 = torch.from_numpy(l0).double().requires_grad_(True)
    B, T, N = lo.shape
    A = lA if lA.dim() == 4 else lA.expand(B, T, N, N)
    la = lo[:, 0] + l0
    for s in range(1, T):
        la = torch.logsumexp(la.unsqueeze(-1) + A[:, s - 1], dim=1) + lo[:, s]
    ll = torch.logsumexp(torch.log(torch.exp(la) + 1e-8), -1) if kind == "ref" else torch.logsumexp(la, -1)
    w = torch.linspace(0.5, 1.5, B, dtype=torch.float64)
    (ll * w).sum().backward()
    return ll.detach(), lo.grad, lA.grad, l0.grad, w


@pytest.mark.parametrize("kind", ["exact", "ref"])
@pytest.mark.parametrize("B,T,N,static", [(2, 12, 5, False), (2, 30, 64, False), (1, 20, 100, True),
                                          (2, 8, 128, False)])
def test_tv_loglik_gradients(kind, B, T, N, static):
    lo, lA, l0 = _random_case(B, T, N, 11 * T + N, static, spread=1.0)
    lo = lo + np.float32(40.0)   # O(1) emissions: the reference-style loss is not saturated
    ll_ref, g_lo, g_lA, g_l0, w = _oracle_tv_grads(lo, lA, l0, kind)
    from pytorch_hmm_amd.autograd import TvSequenceLogLik
    a, b_, c = (t(v).requires_grad_(True) for v in (lo, lA, l0))
    ll = TvSequenceLogLik.apply(a, b_, c, kind)
    (ll * w.float().to(DEV)).sum().backward()
    np.testing.assert_allclose(ll.detach().cpu().numpy(), ll_ref.numpy(), rtol=2e-5, atol=2e-5)
    for got, ref in ((a.grad, g_lo), (b_.grad, g_lA), (c.grad, g_l0)):
        got, ref = got.cpu().numpy().astype(np.float64), ref.numpy()
        assert np.abs(got - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-30), (np.abs(got - ref).max(),
                                                                                 np.abs(ref).max())


def test_neural_hmm_training_step():
    """compute_likelihood back-propagates into both networks and the initial logits."""
    from pytorch_hmm_amd.neural import NeuralHMM
    torch.manual_seed(0)
    m = NeuralHMM(num_states=6, observation_dim=8, context_dim=5, hidden_dim=32).to(DEV).train()
    x, ctx = torch.randn(2, 20, 8, device=DEV), torch.randn(2, 20, 5, device=DEV)
    loss = -m.compute_likelihood(x, ctx).mean()
    loss.backward()
    for name, p in m.named_parameters():
        if "observation_model.logvar_net" in name or "mean_net" in name or "network" in name or "initial" in name:
            assert p.grad is not None and torch.isfinite(p.grad).all(), name


# ------------------------------------------- gradients through the forward-backward outputs
def _fp64_tv_outputs(lo, lA, l0):
    """neural.py:391-401 in float64 with autograd (list-based, no in-place writes): posterior,
    forward = exp(log_forward), backward = exp(log_backward)."""
    B, T, N = lo.shape
    A = lA if lA.dim() == 4 else lA.expand(B, T, N, N)
    la = [l0 + lo[:, 0]]
    for s in range(1, T):
        la.append(torch.logsumexp(la[-1].unsqueeze(-1) + A[:, s - 1], dim=1) + lo[:, s])
    lb = [torch.zeros(B, N, dtype=lo.dtype)]
    for s in range(T - 2, -1, -1):
        lb.insert(0, torch.logsumexp(A[:, s] + lo[:, s + 1].unsqueeze(1) + lb[0].unsqueeze(1), dim=-1))
    la, lb = torch.stack(la, 1), torch.stack(lb, 1)
    lp = la + lb
    lp = lp - torch.logsumexp(lp, dim=-1, keepdim=True)
    return torch.exp(lp), torch.exp(la), torch.exp(lb)


@pytest.mark.parametrize("which", ["post", "all"])
@pytest.mark.parametrize("B,T,N,static", [(2, 12, 5, False), (2, 30, 64, False), (1, 20, 100, True),
                                          (2, 8, 128, False), (1, 9, 200, False), (2, 1, 7, False),
                                          (2, 17, 33, True)])
def test_tv_output_gradients_vs_fp64_autograd(which, B, T, N, static):
    """NeuralHMM trains through its posteriors (and forward / backward) in the reference
    (neural.py:355-461, plain autograd over the loops).  The analytic adjoint on
    hmm355_tv_fb_adjoint_f32 against fp64 autograd through those loops, for a random linear loss
    on the outputs: every gradient within 1e-4 of its tensor's largest entry."""
    lo, lA, l0 = _random_case(B, T, N, 7 * T + N + B, static, spread=1.0)
    lo = lo + np.float32(40.0)   # O(1) log-emissions: forward / backward stay representable
    rng = np.random.default_rng(N + T)
    gw = [rng.standard_normal((B, T, N)) for _ in range(3)]
    ref_in = [torch.from_numpy(v).double().requires_grad_(True) for v in (lo, lA, l0)]
    outs = _fp64_tv_outputs(*ref_in)
    use = (0,) if which == "post" else (0, 1, 2)
    sum(((outs[k] * torch.from_numpy(gw[k])).sum() for k in use)).backward()
    from pytorch_hmm_amd import ops as o
    from pytorch_hmm_amd.autograd import TvForwardBackwardFn
    mask = o.FB_POSTERIOR if which == "post" else o.FB_POSTERIOR | o.FB_FORWARD | o.FB_BACKWARD
    a, b_, c = (t(v).requires_grad_(True) for v in (lo, lA, l0))
    got = TvForwardBackwardFn.apply(a, b_, c, mask)
    np.testing.assert_allclose(got[0].detach().cpu().numpy(), outs[0].detach().numpy(), atol=2e-5)
    sum(((got[i] * t(gw[k])).sum() for i, k in enumerate(use))).backward()
    for name, g_, r_ in (("log_obs", a.grad, ref_in[0].grad), ("log_A", b_.grad, ref_in[1].grad),
                         ("log_p0", c.grad, ref_in[2].grad)):
        g_ = g_.cpu().numpy().astype(np.float64)
        r_ = r_.numpy() if r_ is not None else np.zeros_like(g_)   # T = 1: no matrix is used
        assert g_.shape == r_.shape, name
        err, scale = np.abs(g_ - r_).max(), max(np.abs(r_).max(), 1e-30)
        assert err <= 1e-4 * scale, (name, err, scale)


def test_neural_hmm_trains_through_posteriors():
    """NeuralHMM.forward's posteriors are differentiable into both networks and the initial
    logits (the reference's natural training use); the gradient w.r.t. the networks' outputs
    equals fp64 autograd through the reference loops on the same outputs."""
    from pytorch_hmm_amd.neural import NeuralHMM
    torch.manual_seed(0)
    m = NeuralHMM(num_states=6, observation_dim=8, context_dim=5, hidden_dim=32).to(DEV).train()
    x, ctx = torch.randn(2, 20, 8, device=DEV), torch.randn(2, 20, 5, device=DEV)
    target = torch.randint(0, 6, (2, 20), device=DEV)
    post, fwd, bwd = m(x, ctx)
    loss = torch.nn.functional.cross_entropy(post.reshape(-1, 6), target.reshape(-1))
    loss.backward()
    for name, p in m.named_parameters():
        if "observation_model" in name or "transition_model" in name or "initial" in name:
            if p.requires_grad and ("net" in name or "network" in name or "initial" in name):
                assert p.grad is not None and torch.isfinite(p.grad).all(), name
    assert float(m.initial_logits.grad.abs().sum()) > 0
