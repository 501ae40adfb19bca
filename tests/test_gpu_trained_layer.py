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
    B=4, T=8: short enough that exp(log alpha) stays far above the 1e-8 the reference adds
    before its log (hmm.py:186-211), so the likelihood does not saturate and every transition
    logit gets a non-zero gradient (hmm_layer.py:144-173)."""
    torch.manual_seed(seed)
    layer = ph.HMMLayer(N).to(DEV)
    opt = torch.optim.Adam(layer.parameters(), lr=1e-3)
    g = torch.Generator(device=DEV).manual_seed(seed)
    layer.train()
    for _ in range(steps):
        x = torch.randn(4, 8, N, device=DEV, generator=g)
        loss = layer.compute_loss(x)
        opt.zero_grad()
        loss.backward()
        opt.step()
    layer.eval()
    return layer


@pytest.mark.parametrize("N,T", [(128, 700), (64, 300), (100, 257)])
def test_trained_hmmlayer_decode_dense_vs_c_oracle(N, T):
    layer = trained_layer(N)
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
    # the tables the decode ran on: later calls assign log(P + 1e-8) of the device softmax
    # (hmm_layer.py:83-86); the CPU restatement of that expression agrees closely (GPU and CPU exp differ in the last bits)
    lP, lp0 = hmm.log_P.detach().cpu(), hmm.log_p0.detach().cpu()
    rP, rp0 = O.hmmlayer_params(layer.log_transition_logits.detach().cpu(),
                                layer.log_initial_logits.detach().cpu(), False)
    assert torch.allclose(lP, rP, rtol=0, atol=1e-4) and torch.allclose(lp0, rp0, rtol=0, atol=1e-4)
    obs = torch.sigmoid(x).cpu().numpy()           # the layer's own sigmoid (hmm_layer.py:105)
    # log(obs + 1e-8) (hmm.py:152): the sum in fp32, the log correctly rounded, as the kernels
    # take it (logcr.h; torch-CPU's logf is one ulp off on ~2.5e-5 of inputs)
    lo = np.log((obs + np.float32(1e-8)).astype(np.float64)).astype(np.float32)
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(st2.cpu().numpy(), cs)
    assert np.array_equal(delta.cpu().numpy().view(np.int32), cd.view(np.int32))
    assert torch.equal(onehot.cpu(), torch.nn.functional.one_hot(torch.from_numpy(cs), N).float())


def test_trained_hmmlayer_posteriors_dense_vs_fp64():
    N, T = 128, 400
    layer = trained_layer(N)
    layer.train()
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(2, T, N, device=DEV, generator=g)
    with torch.no_grad():
        post = layer(x)
    hmm = layer._get_hmm()
    lP, lp0 = hmm.log_P.detach().cpu(), hmm.log_p0.detach().cpu()
    lo = np.log((torch.sigmoid(x).cpu().numpy() + np.float32(1e-8)).astype(np.float64)).astype(np.float32)
    ref = O.c_fb64(lo, lP.numpy(), lp0.numpy())[2]
    assert np.allclose(post.cpu().numpy(), ref, atol=2e-5, rtol=0)


def test_training_step_makes_no_plan_sync():
    """A training step re-forms the transition plan (log_P changes every step) without the
    plan's synchronous device -> host read (ops.make_plan read_banded=False): over 20 Adam steps
    of HMMLayer (train-mode posteriors with a supervised loss, and compute_loss) the read is
    never called, and torch's sync debug mode sees no synchronising torch op in the forward or
    backward.  (hmm_layer.py:73-89,144-173)"""
    import warnings
    import pytorch_hmm_amd._native as nat
    L = nat.lib()
    calls = []
    real = L.hmm355_plan_banded

    def counted(*a):
        calls.append(1)
        return real(*a)
    N, B, T = 32, 4, 50
    torch.manual_seed(0)
    layer = ph.HMMLayer(N).to(DEV)
    opt = torch.optim.Adam(layer.parameters(), lr=1e-3)
    g = torch.Generator(device=DEV).manual_seed(1)
    xs = [torch.randn(B, T, N, device=DEV, generator=g) for _ in range(20)]
    tgt = torch.randint(0, N, (B, T), device=DEV, generator=g)
    layer.train()
    layer(xs[0])  # first call (HMMPyTorch construction, the reference's renormalisation)
    torch.cuda.synchronize()
    L.hmm355_plan_banded = counted
    try:
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            torch.cuda.set_sync_debug_mode("warn")
            try:
                for i, x in enumerate(xs):
                    loss = layer.compute_loss(x, tgt) if i % 2 else layer.compute_loss(x)
                    opt.zero_grad()
                    loss.backward()
                    opt.step()
            finally:
                torch.cuda.set_sync_debug_mode("default")
    finally:
        L.hmm355_plan_banded = real
    torch.cuda.synchronize()
    assert not calls, f"{len(calls)} synchronous plan reads in 20 training steps"
    syncs = [str(w.message) for w in rec if "called a synchronizing" in str(w.message)]
    assert not syncs, syncs[:3]
    assert torch.isfinite(loss.detach())
