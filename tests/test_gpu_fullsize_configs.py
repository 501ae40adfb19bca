"""GPU parity at the remaining BASELINE workloads, at the sizes bench.py times them.

* Config 2 — GaussianHMMLayer(64, 80), B=32, T=2000 (hmm_layer.py:220-359), against the
  reference's own full-size outputs (tests/golden/fullsize_gaussian.npz, make_golden.py
  fx_fullsize_gaussian).  At D = 80 every Gaussian density underflows in exp, so the HMM sees
  log(0 + 1e-8) in every cell: 2000 steps of first-index ties (hmm.py:167, :174) on the
  64-state chain.  States bit-exact vs the reference; the full trellis bit-exact vs the C
  oracle; posterior rows atol 2e-3 vs the reference (its own fp32 drift from fp64 is 1.37e-3
  here) and 2e-5 vs fp64; the saturating
  compute_loss rtol 1e-6.
* Config 5 — HSMMLayer(64, 80, max_duration=40), T=2000 (hsmm.py:208-354): the GPU segment
  Viterbi against the C restatement (oracle/hmm_oracle.c hsmm_viterbi_fast, itself proven equal
  to the literal 5-deep loop, which is pinned to the reference's hsmm_* fixtures) on the
  layer's own tables and the GPU's own emission scores: states and scores bit-exact.
* The auto-selected pair forward-backward kernel (csrc/fbpair.h, ops._use_pair: B > CUs/2)
  at B=256, T=2000, N=128 through the bench's call (ops.forward_backward with a plan):
  posteriors within atol 2e-5 of fp64 on a subset of sequences, loglik rtol 2e-6, and the
  Viterbi states / trellis of the same batch bit-exact.
"""
import hashlib

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lo_cr(x):
    """fp32 log(x + 1e-8) correctly rounded (the kernels' logcr.h)."""
    return np.log((x + np.float32(1e-8)).astype(np.float64)).astype(np.float32)


# --------------------------------------------------------------------------- config 2
@torch.no_grad()
def test_config2_gaussian_fullsize_vs_reference():
    import pytorch_hmm_amd as ph
    g = golden("fullsize_gaussian")
    B, T, K, D = (int(v) for v in g["shape"])
    x = O.uniform_obs(int(g["x_seed"]), (B, T, D), -2.0, 2.0)
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["input_sha256"]), "PCG64 input drift"
    layer = ph.GaussianHMMLayer(K, D)
    layer.means.copy_(torch.from_numpy(g["means"]))
    layer.log_scales.copy_(torch.from_numpy(g["log_scales"]))
    layer.hmm_layer.log_transition_logits.copy_(torch.from_numpy(g["logits"]))
    layer.hmm_layer.log_initial_logits.copy_(torch.from_numpy(g["init_logits"]))
    layer = layer.to(DEV)
    xd = torch.from_numpy(x).to(DEV)

    lp = layer._compute_gaussian_log_probs(xd)
    np.testing.assert_allclose(lp[:, :4].cpu().numpy(), g["lp_rows"], rtol=2e-6, atol=2e-5)
    probs = torch.exp(lp)
    assert int((probs > 0).sum()) == int(g["probs_nonzero"]) == 0, "config 2 is the all-underflow case"

    # same call order as the reference fixture: train FB (call 1), eval Viterbi (call 2), loss
    layer.train()
    post = layer(xd).cpu().numpy()
    layer.eval()
    onehot, states = layer.hmm_layer(probs, return_alignment=True)
    loss = layer.compute_loss(xd)

    st = states.cpu().numpy()
    assert np.array_equal(st.astype(np.uint8), g["states"]), "config-2 Viterbi path != reference"
    assert np.array_equal(onehot.cpu().numpy().argmax(-1), st)
    rows = g["post_rows"]
    # the reference's own fp32 posteriors drift from fp64 by up to 1.37e-3 on this input (its
    # rows sum to 1 only within 1.6e-3 after 2000 steps of fp32 logsumexp; measured against
    # O.c_fb64 on the fixture's tables), so the bound against the reference is 2e-3 and the
    # strict check is the fp64 one below (atol 2e-5)
    np.testing.assert_allclose(post[:, rows], g["posterior_rows"], atol=2e-3, rtol=0)
    np.testing.assert_allclose(float(loss), float(g["loss"]), rtol=1e-6)

    # full trellis bit-exact vs the C oracle on the layer's call-2 tables (log(P + 1e-8))
    hmm = layer.hmm_layer._get_hmm()
    lP, lp0 = hmm.log_P.detach().cpu().numpy(), hmm.log_p0.detach().cpu().numpy()
    lo = np.broadcast_to(_lo_cr(np.zeros((1, 1, 1), np.float32)), (B, T, K)).copy()
    cs, cd, _ = O.c_viterbi(lo[:2], lP, lp0)
    s2, d2 = hmm.viterbi_decode(probs)
    assert np.array_equal(s2.cpu().numpy(), st)
    assert np.array_equal(s2[:2].cpu().numpy(), cs)
    assert np.array_equal(d2[:2].cpu().numpy().view(np.int32), cd.view(np.int32))
    # every sequence sees the same (constant) emissions: identical outputs across the batch
    assert (post == post[:1]).all() and (st == st[:1]).all()
    # posterior vs fp64 on the call-1 tables (HMMPyTorch renormalises P on the first call)
    p1 = ph.HMMPyTorch(torch.softmax(torch.from_numpy(g["logits"]), 1),
                       torch.softmax(torch.from_numpy(g["init_logits"]), 0))
    _, _, post64, _ = O.c_fb64(lo[:1], p1.log_P.numpy(), p1.log_p0.numpy())
    np.testing.assert_allclose(post[:1], post64, atol=2e-5, rtol=0)


# --------------------------------------------------------------------------- config 5
@torch.no_grad()
def test_config5_hsmm_fullsize_vs_c_oracle():
    """BASELINE config 5 at the bench's own size (B = 16: the chunk-walk and stitch grid of
    the chunked backtrace at its real extent), bit-exact against the C restatement."""
    import pytorch_hmm_amd as ph
    B, T, S, D, Dm = 16, 2000, 64, 80, 40
    torch.manual_seed(0)
    layer = ph.HSMMLayer(S, D, max_duration=Dm).to(DEV)
    x = torch.from_numpy(O.uniform_obs(5, (B, T, D), -2.0, 2.0)).to(DEV)
    states, scores = layer(x)
    lp = layer.get_observation_log_probs(x).cpu().numpy()
    dur = torch.log(layer.get_duration_probabilities() + layer.eps)[:, :Dm].cpu().numpy()
    lT = torch.log(layer.get_transition_matrix() + layer.eps).cpu().numpy()
    cs, csc = O.c_hsmm(lp, dur, lT, workers=8)
    st = states.cpu().numpy()
    assert np.array_equal(st, cs), "HSMM segmentation != C oracle at T=2000"
    assert np.array_equal(scores.cpu().numpy().view(np.int32), csc.view(np.int32))
    # the emission scores themselves: fp64 scorer within summation-order tolerance
    sd = {k: v.cpu() for k, v in layer.state_dict().items()}
    ref = O.hsmm_log_probs(x[:1].cpu(), sd["observation_means"], sd["observation_log_vars"]).numpy()
    np.testing.assert_allclose(lp[:1], ref, rtol=2e-6, atol=2e-5)
    # a non-trivial segmentation: many segments, every duration within [1, Dmax]
    for b in range(B):
        cuts = np.flatnonzero(np.diff(st[b])) + 1
        seg = np.diff(np.concatenate([[0], cuts, [T]]))
        assert len(seg) > 20 and seg.max() <= Dm


@torch.no_grad()
def test_hsmm_layer_beyond_register_kernels_vs_c_oracle():
    """An HSMMLayer the register-slot kernels cannot hold (150 states with the reference's
    default max_duration = 50) runs end to end on the general form (csrc/hsmm_wide.hip)."""
    import pytorch_hmm_amd as ph
    B, T, S, D, Dm = 2, 400, 150, 16, 50
    torch.manual_seed(1)
    layer = ph.HSMMLayer(S, D).to(DEV)
    assert layer.max_duration == Dm
    x = torch.from_numpy(O.uniform_obs(7, (B, T, D), -2.0, 2.0)).to(DEV)
    states, scores = layer(x)
    lp = layer.get_observation_log_probs(x).cpu().numpy()
    dur = torch.log(layer.get_duration_probabilities() + layer.eps)[:, :Dm].cpu().numpy()
    lT = torch.log(layer.get_transition_matrix() + layer.eps).cpu().numpy()
    cs, csc = O.c_hsmm(lp, dur, lT)
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(scores.cpu().numpy().view(np.int32), csc.view(np.int32))


# ------------------------------------------------------------- large-batch pair kernel
@torch.no_grad()
def test_pair_kernel_b256_fullsize(monkeypatch):
    import pytorch_hmm_amd as ph
    from pytorch_hmm_amd import ops
    B, T, N = 256, 2000, 128
    hmm = ph.HMMPyTorch(ph.create_left_to_right_matrix(N, 0.7))
    dev = torch.device(DEV, 0)
    lP, lp0, plan = hmm._device_params(dev)
    assert plan._hmm355_banded and ops._use_pair(B, dev), "B=256 must select the pair kernel"
    g = torch.Generator(device=dev).manual_seed(1234)
    obs = torch.softmax(torch.randn(B, T, N, device=dev, generator=g), dim=-1)
    post, fwd, bwd, loglik, lik_ref = ops.forward_backward(obs, lP, lp0, ops.OBS_PROB, 7, plan)
    states, delta, final = ops.viterbi(obs, lP, lp0, ops.OBS_PROB, plan)
    pick = np.array([0, 1, 77, 128, 200, 255])
    lo = _lo_cr(obs[pick].cpu().numpy())
    lPn, lp0n = lP.cpu().numpy(), lp0.cpu().numpy()
    la, lb, post64, ll64 = O.c_fb64(lo, lPn, lp0n)
    np.testing.assert_allclose(post[pick].cpu().numpy(), post64, atol=2e-5, rtol=0)
    np.testing.assert_allclose(loglik[pick].cpu().numpy(), ll64, rtol=2e-6)
    # forward = exp(log alpha) where representable (rows 0..63 still carry mass)
    f = fwd[pick, :64].cpu().numpy()
    ref = np.exp(la[:, :64])
    big = ref > 1e-30
    np.testing.assert_allclose(f[big], ref[big], rtol=1e-4)
    cs, cd, _ = O.c_viterbi(lo, lPn, lp0n)
    assert np.array_equal(states[pick].cpu().numpy(), cs)
    assert np.array_equal(delta[pick].cpu().numpy().view(np.int32), cd.view(np.int32))
    assert np.array_equal(final[pick].cpu().numpy(), cd[:, -1].max(-1))
    # the whole batch: every posterior row is a distribution, every loglik finite
    rs = post.sum(-1)
    assert float((rs - 1).abs().max()) < 1e-4 and bool(torch.isfinite(loglik).all())
    # and the two-kernel path gives the same posteriors on the whole batch
    p2 = ops.forward_backward(obs, lP, lp0, ops.OBS_PROB, 1, plan, pair=False)[0]
    assert float((p2 - post).abs().max()) < 1e-5
