"""GPU: Viterbi time parts (hmm355_viterbi_part_f32) and the overlapped GMM scorer + decode
(ops.gmm_viterbi, MixtureGaussianHMMLayer.forward in inference).  A decode run as parts, each
resuming from the previous part's last trellis row, is bit-identical (trellis, states, final
score) to the one-launch decode and to the C restatement of hmm.py:154-184 /
mixture_gaussian.py:290-338; the scorer's time slices are bit-identical to the whole-tensor
call (mixture_gaussian.py:157-214)."""
import ctypes

import numpy as np
import pytest
import torch

import pytorch_hmm_amd as ph
import pytorch_hmm_amd._native as nat
from pytorch_hmm_amd import ops
from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _parts_decode(lo, lP, lp0, plan, bounds):
    B, T, N = lo.shape
    L = nat.lib()
    states = torch.zeros(B, T, dtype=torch.int64, device=DEV)
    delta = torch.empty(B, T, N, device=DEV)
    final = torch.empty(B, device=DEV)
    ws = torch.empty(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=DEV)
    st = nat.stream_of(torch.device(DEV, 0))
    for t0, t1 in zip(bounds[:-1], bounds[1:]):
        rc = L.hmm355_viterbi_part_f32(nat.ptr(lo), ops.OBS_LOG, nat.ptr(lP), nat.ptr(lp0), nat.ptr(plan),
                                       nat.VIT_PLAN_DENSE, B, T, N, t0, t1, nat.ptr(states), nat.ptr(delta),
                                       nat.ptr(final), nat.ptr(ws), ws.numel(), st)
        assert rc == 0
    torch.cuda.synchronize()
    return states.cpu().numpy(), delta.cpu().numpy(), final.cpu().numpy()


@pytest.mark.parametrize("N,T,bounds", [
    (128, 1000, [0, 64, 320, 1000]),
    (128, 2000, [0, 192, 576, 1216, 1856, 2000]),
    (100, 700, [0, 128, 640, 700]),
    (64, 300, [0, 256, 300]),
    (37, 130, [0, 64, 128, 130]),
])
def test_parts_equal_whole_and_oracle(N, T, bounds):
    rng = np.random.default_rng(N + T)
    lP, lp0 = O.hmm_params(torch.from_numpy(rng.random((N, N), dtype=np.float32)))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = ops.make_plan(lPd)
    assert plan._hmm355_banded is False
    B = 4
    lo = np.log(rng.random((B, T, N), dtype=np.float32) + np.float32(1e-3)).astype(np.float32)
    lod = torch.from_numpy(lo).to(DEV)
    s, d, f = _parts_decode(lod, lPd, lp0d, plan, bounds)
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    assert np.array_equal(d, cd) and np.array_equal(s, cs)
    assert np.array_equal(f, cd[:, -1].max(-1))
    s1, d1, f1 = ops.viterbi(lod, lPd, lp0d, ops.OBS_LOG, plan)
    assert np.array_equal(s1.cpu().numpy(), s) and np.array_equal(d1.cpu().numpy(), d)


def test_parts_rejected_without_dense_word():
    """A part (not the whole range) needs the host's dense word, OBS_LOG and q_lo % 64 == 0."""
    d = {"E_ARG": -1}
    N, B, T = 64, 2, 256
    L = nat.lib()
    lP, lp0 = O.hmm_params(torch.rand(N, N))
    lPd = lP.to(DEV)
    plan = ops.make_plan(lPd)
    lo = torch.randn(B, T, N, device=DEV)
    out = [torch.empty(B, T, dtype=torch.int64, device=DEV), torch.empty(B, T, N, device=DEV), torch.empty(B, device=DEV)]
    ws = torch.empty(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=DEV)
    st = nat.stream_of(torch.device(DEV, 0))
    call = lambda flags, mode, a, b: L.hmm355_viterbi_part_f32(
        nat.ptr(lo), mode, nat.ptr(lPd), nat.ptr(lp0.to(DEV)), nat.ptr(plan), flags, B, T, N, a, b,
        *(nat.ptr(t) for t in out), nat.ptr(ws), ws.numel(), st)
    assert call(0, ops.OBS_LOG, 0, 128) != 0                       # no dense word
    assert call(nat.VIT_PLAN_DENSE, ops.OBS_PROB, 0, 128) != 0     # probabilities
    assert call(nat.VIT_PLAN_DENSE, ops.OBS_LOG, 32, 128) != 0     # not a chunk boundary
    assert call(nat.VIT_PLAN_DENSE, ops.OBS_LOG, 128, 64) != 0     # empty
    assert call(0, ops.OBS_LOG, 0, T) == 0                          # the whole range: any plan
    torch.cuda.synchronize()


@pytest.mark.parametrize("S,C,T,B", [(128, 4, 2000, 3), (128, 4, 700, 2), (64, 1, 1300, 2), (40, 2, 900, 3)])
def test_gmm_viterbi_equals_sequential(S, C, T, B, monkeypatch):
    """ops.gmm_viterbi (scorer slices on a side stream, chain parts on the current one) against the
    scorer then the decode, bit for bit: log-probabilities, states, trellis and final scores."""
    torch.manual_seed(S + C + T)
    D = 24
    m = ph.MixtureGaussianHMMLayer(S, D, num_components=C).to(DEV)
    x = torch.randn(B, T, D, device=DEV)
    with torch.no_grad():
        log_T = m._safe_log(m.get_transition_matrix())
        log_w = m._safe_log(torch.softmax(m.mixture_weights_logits, -1))
        init = -(torch.zeros(S, device=DEV) + np.log(S))
        plan = m._transition_plan(log_T)
        assert plan._hmm355_banded is False
        monkeypatch.setenv("HMM355_GMM_VIT_PARTS", "1")
        lp, st, de, fi = ops.gmm_viterbi(x, m.means, m.log_vars, log_w, 1, log_T, init, plan)
        monkeypatch.setenv("HMM355_GMM_VIT_PARTS", "0")
        lp2, st2, de2, fi2 = ops.gmm_viterbi(x, m.means, m.log_vars, log_w, 1, log_T, init, plan)
        torch.cuda.synchronize()
    assert torch.equal(lp, lp2) and torch.equal(st, st2) and torch.equal(de, de2) and torch.equal(fi, fi2)
    cs, cd, _ = O.c_viterbi(lp.cpu().numpy(), log_T.cpu().numpy(), init.cpu().numpy())
    assert np.array_equal(st.cpu().numpy(), cs) and np.array_equal(de.cpu().numpy(), cd)


@pytest.mark.parametrize("parts", ["0", "1"])
def test_mixture_forward_inference_matches_training_path(parts, monkeypatch):
    """MixtureGaussianHMMLayer.forward without grad (ops.gmm_viterbi with the cached inference
    tables; parts on and off) and with grad (scorer then decode, ViterbiScore) give the same
    states and scores; a parameter update is seen by the cached tables."""
    monkeypatch.setenv("HMM355_GMM_VIT_PARTS", parts)
    torch.manual_seed(7)
    m = ph.MixtureGaussianHMMLayer(128, 20, num_components=4).to(DEV)
    x = torch.randn(2, 900, 20, device=DEV)
    with torch.no_grad():
        s1, c1 = m(x, return_log_probs=True)
    s2, c2 = m(x, return_log_probs=True)
    assert torch.equal(s1, s2) and torch.equal(c1, c2.detach())
    with torch.no_grad():
        m.transition_logits.mul_(3.0)   # a new version: the cached tables are re-formed
        s3, c3 = m(x, return_log_probs=True)
    s4, c4 = m(x, return_log_probs=True)
    assert torch.equal(s3, s4) and torch.equal(c3, c4.detach()) and not torch.equal(c3, c1)
