"""GPU: the analytic adjoint of the forward recursion (pytorch_hmm_amd/autograd.py over
hmm355_forward_backward_ex_f32) against autograd through the oracle's restatement of the
reference loops (oracle/hmm_oracle.py -> hmm.py:89-101), float64 on CPU.

Tolerance: relative 1e-4 of the largest gradient entry (fp32 kernels vs fp64 autograd)."""
import numpy as np
import pytest
import torch

import pytorch_hmm_amd as ph
from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def oracle_grads(obs, lP, lp0, kind):
    obs = obs.double().requires_grad_(True)
    lP = lP.double().requires_grad_(True)
    lp0 = lp0.double().requires_grad_(True)
    B, T, K = obs.shape
    log_obs = torch.log(obs + 1e-8)
    la = [lp0 + log_obs[:, 0]]
    for t in range(1, T):
        la.append(torch.logsumexp(la[-1][:, :, None] + lP[None], dim=1) + log_obs[:, t])
    a = la[-1]
    if kind == "ref":
        ll = torch.logsumexp(torch.log(torch.exp(a) + 1e-8), dim=-1)
    else:
        ll = torch.logsumexp(a, dim=-1)
    w = torch.linspace(0.5, 1.5, B, dtype=torch.float64)
    (ll * w).sum().backward()
    return ll.detach(), obs.grad, lP.grad, lp0.grad, w


def close(a, b, rel=1e-4):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    assert np.abs(a - b).max() <= rel * scale, (np.abs(a - b).max(), scale)


@pytest.mark.parametrize("kind", ["ref", "exact"])
@pytest.mark.parametrize("B,T,N,mat", [(2, 12, 5, "l2r"), (3, 30, 16, "rand"), (2, 25, 70, "ergodic"),
                                       (1, 40, 128, "l2r"), (1, 30, 200, "l2r"), (1, 30, 200, "rand")])
def test_loglik_gradients(kind, B, T, N, mat):
    rng = np.random.default_rng(T * N)
    if mat == "l2r":
        P = O.left_to_right_matrix(N, 0.7)
    elif mat == "ergodic":
        P = O.transition_matrix(N, "ergodic")
    else:
        P = torch.from_numpy(rng.random((N, N), dtype=np.float32))
    lP, lp0 = O.hmm_params(P)
    obs = torch.from_numpy(rng.random((B, T, N), dtype=np.float32) * 0.9 + 0.1)
    ll_ref, g_obs, g_lP, g_lp0, w = oracle_grads(obs, lP, lp0, kind)

    o = obs.to(DEV).requires_grad_(True)
    P_ = lP.to(DEV).requires_grad_(True)
    p0 = lp0.to(DEV).requires_grad_(True)
    from pytorch_hmm_amd.autograd import SequenceLogLik
    from pytorch_hmm_amd import ops
    ll = SequenceLogLik.apply(o, P_, p0, ops.OBS_PROB, kind)
    (ll * w.float().to(DEV)).sum().backward()
    np.testing.assert_allclose(ll.detach().cpu().numpy(), ll_ref.numpy(), rtol=2e-5, atol=2e-5)
    close(o.grad.cpu(), g_obs)
    close(P_.grad.cpu(), g_lP)
    close(p0.grad.cpu(), g_lp0)


@pytest.mark.parametrize("dense", [False, True])
def test_gradients_dense_and_banded_agree(dense):
    rng = np.random.default_rng(3)
    B, T, N = 2, 50, 64
    lP, lp0 = O.hmm_params(O.left_to_right_matrix(N, 0.7))
    obs = torch.from_numpy(rng.random((B, T, N), dtype=np.float32) * 0.9 + 0.1)
    _, g_obs, g_lP, g_lp0, w = oracle_grads(obs, lP, lp0, "exact")
    o = obs.to(DEV).requires_grad_(True)
    P_ = lP.to(DEV).requires_grad_(True)
    p0 = lp0.to(DEV).requires_grad_(True)
    from pytorch_hmm_amd.autograd import SequenceLogLik
    from pytorch_hmm_amd import ops
    plan = ops.make_plan(P_.detach(), dense=dense)   # dense: HMM355_PLAN_DENSE on a banded matrix
    (SequenceLogLik.apply(o, P_, p0, ops.OBS_PROB, "exact", plan) * w.float().to(DEV)).sum().backward()
    close(o.grad.cpu(), g_obs)
    close(P_.grad.cpu(), g_lP)


def test_saturated_reference_loss_has_zero_gradient():
    """At N=128, T=2000 the reference's compute_likelihood saturates (exp underflow) and its
    gradient is exactly 0; the adjoint reproduces that instead of a spurious value."""
    hmm = ph.HMMPyTorch(ph.create_left_to_right_matrix(128, 0.7))
    obs = torch.softmax(torch.randn(2, 2000, 128, device=DEV), -1).requires_grad_(True)
    ll = hmm.compute_likelihood(obs)
    ll.sum().backward()
    assert torch.isfinite(ll).all()
    assert torch.count_nonzero(obs.grad) == 0


def test_hmmlayer_training_step_changes_transitions():
    """The reference's test_parameter_learning (test_hmm.py:189-208) on the MI355X path."""
    torch.manual_seed(0)
    layer = ph.HMMLayer(5).to(DEV)
    obs = torch.rand(2, 10, 5, device=DEV)
    opt = torch.optim.Adam(layer.parameters(), lr=0.01)
    before = layer.get_transition_matrix().detach().clone()
    layer.train()
    loss = layer.compute_loss(obs)
    opt.zero_grad()
    loss.backward()
    assert layer.log_transition_logits.grad is not None and torch.isfinite(layer.log_transition_logits.grad).all()
    assert layer.log_initial_logits.grad is not None
    opt.step()
    assert not torch.allclose(before, layer.get_transition_matrix())


# ------------------------------------------------- gradients THROUGH the FB outputs
def fb_ref64(x, lP, lp0, log_mode):
    """hmm.py:86-130 in float64 autograd (the reference's log-space loops)."""
    lo = x if log_mode else torch.log(x + 1e-8)
    B, T, K = lo.shape
    la = [lp0 + lo[:, 0]]
    for t in range(1, T):
        la.append(torch.logsumexp(la[-1][:, :, None] + lP[None], dim=1) + lo[:, t])
    lb = [torch.zeros(B, K, dtype=lo.dtype)]
    for t in range(T - 2, -1, -1):
        lb.insert(0, torch.logsumexp(lP[None] + lo[:, t + 1, None, :] + lb[0][:, None, :], dim=2))
    la, lb = torch.stack(la, 1), torch.stack(lb, 1)
    lp = la + lb
    lp = lp - torch.logsumexp(lp, dim=-1, keepdim=True)
    return torch.exp(lp), torch.exp(la), torch.exp(lb)


def _matrix(kind, N):
    if kind == "l2r":
        return O.left_to_right_matrix(N, 0.7)
    if kind == "ergodic":
        return O.transition_matrix(N, "ergodic")
    g = torch.Generator().manual_seed(N)
    return torch.softmax(torch.randn(N, N, generator=g), -1)


@pytest.mark.parametrize("N", [5, 70, 128, 200])   # (200: the NP = 256 chains' CA / CB)
@pytest.mark.parametrize("kind", ["l2r", "ergodic", "random"])
@pytest.mark.parametrize("log_mode", [False, True])
@pytest.mark.parametrize("outs", ["post", "all"])
def test_output_vjp_matches_fp64_autograd(N, kind, log_mode, outs):
    """d(sum Gp*posterior + Gf*forward + Gb*backward) / d(obs, log_P, log_p0) through
    ForwardBackwardFn (hmm355_fb_adjoint_f32) vs float64 autograd through the loops."""
    from pytorch_hmm_amd import ops
    from pytorch_hmm_amd.autograd import ForwardBackwardFn
    g = torch.Generator().manual_seed(7 * N + (3 if log_mode else 0))
    B, T = 2, 40
    if log_mode:   # Gaussian-like log-emissions far below -87 (the OBS_LOG row-max shift)
        x = -150.0 + 20.0 * torch.randn(B, T, N, generator=g)
    else:
        x = torch.softmax(torch.randn(B, T, N, generator=g), -1)
    lP, lp0 = O.hmm_params(_matrix(kind, N))
    Gp = torch.randn(B, T, N, generator=g)
    Gf = torch.randn(B, T, N, generator=g) if outs == "all" else None
    Gb = torch.randn(B, T, N, generator=g) if outs == "all" else None
    ref = [t.double().requires_grad_(True) for t in (x, lP, lp0)]
    p, f, b = fb_ref64(ref[0], ref[1], ref[2], log_mode)
    loss = (p * Gp.double()).sum()
    if outs == "all":
        loss = loss + (f * Gf.double()).sum() + (b * Gb.double()).sum()
    loss.backward()
    ours = [t.to(DEV).requires_grad_(True) for t in (x, lP, lp0)]
    mask = ops.FB_POSTERIOR | (ops.FB_FORWARD | ops.FB_BACKWARD if outs == "all" else 0)
    res = ForwardBackwardFn.apply(ours[0], ours[1], ours[2], ops.OBS_LOG if log_mode else ops.OBS_PROB, mask)
    l2 = (res[0] * Gp.to(DEV)).sum()
    if outs == "all":
        l2 = l2 + (res[1] * Gf.to(DEV)).sum() + (res[2] * Gb.to(DEV)).sum()
    l2.backward()
    # per tensor: 1e-4 of its largest entry, plus 1e-5 of the emission-gradient scale (with
    # log-emissions 20 nats apart the log_p0 gradient is a ~1e-4 residue of O(1) adjoints;
    # the reference's own fp32 autograd misses it by ~1e-3 there)
    gscale = float(ref[0].grad.abs().max())
    for a, r in zip(ours, ref):
        err = float((a.grad.cpu().double() - r.grad).abs().max())
        assert err <= 1e-4 * float(r.grad.abs().max()) + 1e-5 * gscale, (err, float(r.grad.abs().max()), gscale)


def test_hmmlayer_supervised_loss_gradients():
    """HMMLayer training mode + compute_loss(target_alignment) (hmm_layer.py:119-121,159-165):
    the cross-entropy on the posteriors back-propagates to the logits and the input as the
    reference's autograd does.  compute_loss calls _get_hmm() and then forward() calls it
    again, so the posteriors use the later-call tables log(softmax + 1e-8) (hmm_layer.py:83-86)."""
    torch.manual_seed(3)
    K, B, T = 6, 3, 30
    layer = ph.HMMLayer(K).to(DEV)
    layer.train()
    x = torch.randn(B, T, K)
    tgt = torch.randint(0, K, (B, T))
    xd = x.to(DEV).requires_grad_(True)
    loss = layer.compute_loss(xd, target_alignment=tgt.to(DEV))
    loss.backward()
    lt = layer.log_transition_logits.detach().cpu().double().requires_grad_(True)
    li = layer.log_initial_logits.detach().cpu().double().requires_grad_(True)
    xr = x.double().requires_grad_(True)
    P = torch.softmax(lt, dim=1)
    p0 = torch.softmax(li, dim=0)
    post = fb_ref64(torch.sigmoid(xr), torch.log(P + 1e-8), torch.log(p0 + 1e-8), False)[0]
    lref = torch.nn.functional.cross_entropy(post.reshape(-1, K), tgt.reshape(-1))
    lref.backward()
    assert abs(float(loss) - float(lref)) < 1e-5
    close(xd.grad.cpu(), xr.grad)
    close(layer.log_transition_logits.grad.cpu(), lt.grad)
    close(layer.log_initial_logits.grad.cpu(), li.grad)


def test_hmmlayer_posterior_training_step():
    """A training step on a loss of the train-mode posteriors changes the transitions."""
    torch.manual_seed(0)
    layer = ph.HMMLayer(4).to(DEV)
    layer.train()
    opt = torch.optim.SGD(layer.parameters(), lr=0.5)
    x = torch.randn(2, 8, 4, device=DEV, requires_grad=True)
    before = layer.get_transition_matrix().detach().clone()
    post = layer(x)
    assert post.requires_grad and torch.allclose(post.sum(-1), torch.ones(2, 8, device=DEV), atol=1e-5)
    (post[..., 0] ** 2).sum().backward()
    assert torch.isfinite(x.grad).all() and x.grad.abs().sum() > 0
    opt.step()
    assert not torch.allclose(before, layer.get_transition_matrix())


# ------------------------------------------------------------------ emission / Viterbi score
def test_gmm_gradients_match_autograd():
    torch.manual_seed(1)
    B, T, S, C, D = 2, 20, 6, 3, 10
    x = torch.randn(B, T, D)
    wl = torch.randn(S, C) * 0.5
    mu = torch.randn(S, C, D) * 0.4
    lv = torch.randn(S, C, D) * 0.2
    W = torch.randn(B, T, S)
    ref = [t.clone().double().requires_grad_(True) for t in (x, wl, mu, lv)]
    lp_ref = O.mixture_log_probs(ref[0], ref[1], ref[2], ref[3])
    (lp_ref * W.double()).sum().backward()
    from pytorch_hmm_amd.autograd import GmmLogProb
    ours = [t.clone().to(DEV).requires_grad_(True) for t in (x, wl, mu, lv)]
    log_w = torch.log(torch.clamp(torch.softmax(ours[1], -1), min=1e-8))
    lp = GmmLogProb.apply(ours[0], ours[2], ours[3], log_w, 1)
    np.testing.assert_allclose(lp.detach().cpu().numpy(), lp_ref.detach().numpy(), rtol=1e-5, atol=1e-4)
    (lp * W.to(DEV)).sum().backward()
    for a, r in zip(ours, ref):
        close(a.grad.cpu(), r.grad)


def test_single_gaussian_gradients_match_autograd():
    torch.manual_seed(2)
    B, T, S, D = 2, 15, 5, 7
    x, mu, lv = torch.randn(B, T, D), torch.randn(S, D) * 0.3, torch.randn(S, D) * 0.2
    W = torch.randn(B, T, S)
    ref = [t.clone().double().requires_grad_(True) for t in (x, mu, lv)]
    (O.hsmm_log_probs(*ref) * W.double()).sum().backward()
    from pytorch_hmm_amd.autograd import GmmLogProb
    ours = [t.clone().to(DEV).requires_grad_(True) for t in (x, mu, lv)]
    lp = GmmLogProb.apply(ours[0], ours[1].unsqueeze(1), ours[2].unsqueeze(1), torch.zeros(S, 1, device=DEV), 0)
    (lp * W.to(DEV)).sum().backward()
    for a, r in zip(ours, ref):
        close(a.grad.cpu(), r.grad)


def test_viterbi_score_gradient_follows_the_path():
    torch.manual_seed(3)
    B, T, S = 3, 40, 8
    lp = torch.randn(B, T, S)
    lT = torch.log_softmax(torch.randn(S, S), -1)
    init = -(torch.zeros(S) + np.log(S))
    w = torch.tensor([1.0, -0.5, 2.0])
    lpr, lTr = lp.clone().requires_grad_(True), lT.clone().requires_grad_(True)
    _, delta = O.viterbi_from_log(lpr, lTr, init)
    (delta[:, -1].max(-1)[0] * w).sum().backward()
    from pytorch_hmm_amd.autograd import ViterbiScore
    lpo, lTo = lp.to(DEV).requires_grad_(True), lT.to(DEV).requires_grad_(True)
    states, final = ViterbiScore.apply(lpo, lTo, init.to(DEV))
    (final * w.to(DEV)).sum().backward()
    assert np.array_equal(lpo.grad.cpu().numpy(), lpr.grad.numpy())
    assert np.array_equal(lTo.grad.cpu().numpy(), lTr.grad.numpy())


def test_mixture_layer_gradient_flow():
    """test_mixture_gaussian.py:164-176 on the MI355X path: every parameter gets a finite grad."""
    torch.manual_seed(0)
    m = ph.MixtureGaussianHMMLayer(6, 10, num_components=3).to(DEV)
    m.train()
    states, log_probs = m(torch.randn(2, 30, 10, device=DEV), return_log_probs=True)
    (-log_probs.mean()).backward()
    for name, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), name


def test_hsmm_observation_gradient_flow():
    """test_hsmm.py:283-296: observation parameters get gradients from get_observation_log_probs."""
    torch.manual_seed(0)
    h = ph.HSMMLayer(5, 30, max_duration=10).to(DEV)
    x = torch.randn(1, 20, 30, device=DEV, requires_grad=True)
    h.get_observation_log_probs(x).sum().backward()
    assert h.observation_means.grad is not None and torch.isfinite(h.observation_means.grad).all()
    assert h.observation_log_vars.grad is not None and torch.isfinite(h.observation_log_vars.grad).all()
    assert x.grad is not None


def test_gaussian_layer_compute_loss_backward():
    torch.manual_seed(0)
    layer = ph.GaussianHMMLayer(4, 3).to(DEV)
    loss = layer.compute_loss(torch.randn(2, 12, 3, device=DEV))
    loss.backward()
    assert torch.isfinite(loss)
    for name, p in layer.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), name


@pytest.mark.parametrize("mat", ["l2r", "rand"])
def test_loglik_gradients_obs_log_low_emissions(mat):
    """OBS_LOG with log-emissions around -200 (the shifted-emission chains): gradients of the
    exact log-likelihood vs fp64 autograd through the reference's log-space loop."""
    rng = np.random.default_rng(17)
    B, T, N = 2, 40, 32
    P = O.left_to_right_matrix(N, 0.7) if mat == "l2r" else torch.from_numpy(rng.random((N, N), dtype=np.float32))
    lP, lp0 = O.hmm_params(P)
    lo = torch.from_numpy((-(rng.random((B, T, N)) * 240 + 80)).astype(np.float32))
    lo64 = lo.double().requires_grad_(True)
    lP64 = lP.double().requires_grad_(True)
    l064 = lp0.double().requires_grad_(True)
    la = l064 + lo64[:, 0]
    for tt in range(1, T):
        la = torch.logsumexp(la[:, :, None] + lP64[None], dim=1) + lo64[:, tt]
    w = torch.linspace(0.5, 1.5, B, dtype=torch.float64)
    (torch.logsumexp(la, -1) * w).sum().backward()

    from pytorch_hmm_amd.autograd import SequenceLogLik
    from pytorch_hmm_amd import ops
    o = lo.to(DEV).requires_grad_(True)
    P_ = lP.to(DEV).requires_grad_(True)
    p0 = lp0.to(DEV).requires_grad_(True)
    ll = SequenceLogLik.apply(o, P_, p0, ops.OBS_LOG, "exact")
    (ll * w.float().to(DEV)).sum().backward()
    np.testing.assert_allclose(ll.detach().cpu().numpy(), torch.logsumexp(la, -1).detach().numpy(), rtol=2e-6)
    close(o.grad.cpu(), lo64.grad)
    close(P_.grad.cpu(), lP64.grad)
    close(p0.grad.cpu(), l064.grad)
