"""GPU: a TRAINED HMMLayer — the path every learned model takes.

A few Adam steps move the floor entries of log(softmax(logits) + 1e-8) off the floor, so the
band detector (band.h, kBandMax) finds no band and the dense chains (recur.h rec_run_rb, the
dense psi pass of vit_kern.h) run.  The test records which chain ran (ops.plan_info) and checks
the decode bit-exact against the C restatement of hmm.py:132-184 on the layer's own tables
(hmm_layer.py:61-89, later-call form), and the posteriors against float64 (hmm.py:66-130).
"""
import numpy as np
import pytest
import torch

import pytorch_hmm_amd as ph
from pytorch_hmm_amd import ops
from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def trained_layer(N, steps=3, seed=0):
    """HMMLayer(N) after `steps` Adam steps (lr 1e-3) on compute_loss over random scores, at
    B=4, T=64 (short enough that the reference likelihood does not saturate, so the gradient
    is non-zero; hmm_layer.py:144-173)."""
    torch.manual_seed(seed)
    layer = ph.HMMLayer(N).to(DEV)
    opt = torch.optim.Adam(layer.parameters(), lr=1e-3)
    g = torch.Generator(device=DEV).manual_seed(seed)
    layer.train()
    for _ in range(steps):
        x = torch.randn(4, 64, N, device=DEV, generator=g)
        loss = layer.compute_loss(x)
        opt.zero_grad()
        loss.backward()
        opt.step()
    layer.eval()
    return layer


@pytest.mark.parametrize("N,T", [(128, 700), (64, 300), (100, 257)])
def test_trained_hmmlayer_decode_dense_vs_c_oracle(N, T):
    layer = trained_layer(N)
    lg = layer.log_transition_logits.detach().cpu()
    assert torch.count_nonzero(lg > -18.0) > 8 * N   # the trained rows are no longer banded
    g = torch.Generator(device=DEV).manual_seed(N + T)
    x = torch.randn(3, T, N, device=DEV, generator=g)
    with torch.no_grad():
        onehot, states = layer(x, return_alignment=True)
        st2, delta = layer.align(x)
    hmm = layer._get_hmm()
    _, _, plan = hmm._device_params(x.device)
    info = ops.plan_info(plan)
    print("chains:", info)
    assert info["viterbi"] == "dense" and info["forward"] == "dense"
    # the layer's tables: later calls assign log(P + 1e-8) (hmm_layer.py:83-86)
    lP, lp0 = O.hmmlayer_params(layer.log_transition_logits.detach().cpu(),
                                layer.log_initial_logits.detach().cpu(), False)
    obs = torch.sigmoid(x).cpu()                   # the layer's own sigmoid (hmm_layer.py:105)
    lo = torch.log(obs + 1e-8).numpy()             # hmm.py:152
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(st2.cpu().numpy(), cs)
    assert np.array_equal(delta.cpu().numpy(), cd)
    assert torch.equal(onehot.cpu(), torch.nn.functional.one_hot(torch.from_numpy(cs), N).float())


def test_trained_hmmlayer_posteriors_dense_vs_fp64():
    N, T = 128, 400
    layer = trained_layer(N)
    layer.train()
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(2, T, N, device=DEV, generator=g)
    with torch.no_grad():
        post = layer(x)
    lP, lp0 = O.hmmlayer_params(layer.log_transition_logits.detach().cpu(),
                                layer.log_initial_logits.detach().cpu(), False)
    lo = torch.log(torch.sigmoid(x).cpu() + 1e-8)
    ref = O.c_fb64(lo.numpy(), lP.numpy(), lp0.numpy())[2]
    assert np.allclose(post.cpu().numpy(), ref, atol=2e-5, rtol=0)
