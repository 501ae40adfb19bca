"""GPU: the GMM scorer in published time slices beside a Viterbi decode that starts at once
(ops.gmm_viterbi: hmm355_gmm_diag_logprob_ready_f32 on a side stream, hmm355_viterbi_ready_f32 on
the current one) -- the same bits as the scorer and the decode in series (mixture_gaussian.py
:157-214 then :290-338), over dense and banded plans, every scorer form (C = 1, 2, 4 sliced;
C = 3 whole), lengths around the slice and block edges, and a count whose producer slices
arrive late (a long first slice)."""
import numpy as np
import pytest
import torch

from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(S, C, D, seed):
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(S, C, D, generator=g)
    log_vars = 0.3 * torch.randn(S, C, D, generator=g)
    log_w = torch.log_softmax(torch.randn(S, C, generator=g), -1).clamp_min(np.log(1e-8))
    return means.to(DEV), log_vars.to(DEV), log_w.to(DEV)


def _matrix(S, kind, seed):
    if kind == "dense":
        g = torch.Generator().manual_seed(seed)
        P = torch.softmax(torch.randn(S, S, generator=g), -1)
    else:
        P = O.left_to_right_matrix(S, 0.7)
    return torch.log(P + 1e-8).to(DEV)


@pytest.mark.parametrize("kind", ["dense", "banded"])
@pytest.mark.parametrize("S,C,D,T", [(128, 4, 80, 2000), (64, 1, 40, 700), (100, 2, 24, 65), (128, 4, 80, 17),
                                     (40, 3, 16, 300), (128, 4, 80, 1000)])
def test_gmm_viterbi_overlap_equals_series(kind, S, C, D, T):
    from pytorch_hmm_amd import ops
    B = 6
    means, log_vars, log_w = _params(S, C, D, S + C + T)
    lT = _matrix(S, kind, S)
    init = torch.full((S,), -float(np.log(S)), device=DEV)
    plan = ops.make_plan(lT)
    x = torch.randn(B, T, D, generator=torch.Generator().manual_seed(T)).to(DEV)
    a = ops.gmm_viterbi(x, means, log_vars, log_w, lT, init, plan, overlap=True)
    b = ops.gmm_viterbi(x, means, log_vars, log_w, lT, init, plan, overlap=False)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    # slices of other widths (a late first slice: the chains wait for it)
    c = ops.gmm_viterbi(x, means, log_vars, log_w, lT, init, plan, overlap=True, first_frames=512, slice_frames=64)
    for u, v in zip(c, b):
        assert torch.equal(u, v)


def test_gmm_viterbi_repeated_on_busy_stream():
    """Back-to-back calls (the count word and buffers re-used by the caching allocator) beside a
    queue of GEMMs on a third stream: every call's own result."""
    from pytorch_hmm_amd import ops
    B, T, S, C, D = 32, 2000, 128, 4, 80
    means, log_vars, log_w = _params(S, C, D, 1)
    lT = _matrix(S, "dense", 2)
    init = torch.full((S,), -float(np.log(S)), device=DEV)
    plan = ops.make_plan(lT)
    xs = [torch.randn(B, T, D, generator=torch.Generator().manual_seed(k)).to(DEV) for k in range(3)]
    refs = [ops.gmm_viterbi(x, means, log_vars, log_w, lT, init, plan, overlap=False) for x in xs]
    a = torch.randn(4096, 4096, device=DEV)
    busy = torch.cuda.Stream()
    busy.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(busy):
        for _ in range(20):
            a = a @ a * 1e-3
    outs = [ops.gmm_viterbi(x, means, log_vars, log_w, lT, init, plan) for x in xs]
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        for u, v in zip(o, r):
            assert torch.equal(u, v)
