"""GPU: the work beside the banded chains inside their own launch (csrc/follow.h).

  * Viterbi (HMM355_VIT_PLAN_BANDED): per sequence one workgroup forms log(x + 1e-8) ahead of
    the chain (OBS_PROB), composes the 64-step chunk maps from the psi rows the chain publishes,
    and backtraces the path -- checked bit-exact against the C oracle (hmm.py:154-184) and
    against the same call with the passes after the chain (follow=False), over chunk and block
    edges, padded state counts, tie-heavy emissions, both emission encodings, and a second
    stream keeping the chip busy.
  * forward-backward (HMM355_FB_PLAN_BANDED): per sequence one workgroup forms the posterior of
    each row as both chains publish it (hmm.py:119-126) and the alpha chain the reference's
    compute_likelihood value (hmm.py:206) -- against the posterior pass (follow=False) and the
    fp64 oracle.
  * A plan passed as banded that is not: the outputs come back invalid (states -1, NaN), never
    stale.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def ops():
    from pytorch_hmm_amd import ops as o
    return o


def banded(N, kind="l2r"):
    if kind == "l2r":
        return O.left_to_right_matrix(N, 0.7)
    return O.transition_matrix(N, kind)


def lo_cr(x):
    """log(x + 1e-8): fp32 sum, correctly rounded log (the kernels' logcr.h)"""
    return np.log((x + np.float32(1e-8)).astype(np.float64)).astype(np.float32)


@pytest.mark.parametrize("N", [128, 100, 200, 256])
@pytest.mark.parametrize("T", [1, 15, 16, 17, 64, 65, 80, 129, 1000])
def test_viterbi_decode_followers_vs_oracle(N, T):
    o = ops()
    rng = np.random.default_rng(N * 1000 + T)
    B = 3
    lP, lp0 = O.hmm_params(banded(N))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    assert plan._hmm355_banded
    x = rng.random((B, T, N), dtype=np.float32)
    cs, cd, _ = O.c_viterbi(lo_cr(x), lP.numpy(), lp0.numpy())
    xd = torch.from_numpy(x).to(DEV)
    for follow in (True, False):
        s, d, f = o.viterbi(xd, lPd, lp0d, o.OBS_PROB, plan, follow=follow)
        assert np.array_equal(d.cpu().numpy().view(np.int32), cd.view(np.int32)), follow
        assert np.array_equal(s.cpu().numpy(), cs), follow
        assert np.array_equal(f.cpu().numpy(), cd[:, -1].max(-1)), follow


@pytest.mark.parametrize("kind", ["l2r", "left_to_right_skip", "ergodic"])
def test_viterbi_decode_followers_log_and_ties(kind):
    """OBS_LOG input (no leaders: the chain stages the log-emissions as given) with coarse values
    (many exact ties: the first index), and the factory's other banded matrices."""
    o = ops()
    rng = np.random.default_rng(7)
    B, T, N = 6, 700, 128
    lP, lp0 = O.hmm_params(banded(N, kind))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    lo = np.round(-(rng.random((B, T, N)) * 6), 0).astype(np.float32)
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    s, d, f = o.viterbi(torch.from_numpy(lo).to(DEV), lPd, lp0d, o.OBS_LOG, plan)
    assert np.array_equal(s.cpu().numpy(), cs)
    assert np.array_equal(d.cpu().numpy(), cd)


def test_viterbi_followers_fullsize_batch_and_repeat():
    """The north-star shape, twice on the same buffers (the counts are re-zeroed per call), and a
    batch too large for the followers (B = 100: the passes after the chain), same bits."""
    o = ops()
    N, T = 128, 2000
    lP, lp0 = O.hmm_params(banded(N))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    for B in (32, 100):
        g = torch.Generator(device=DEV).manual_seed(B)
        x = torch.softmax(torch.randn(B, T, N, device=DEV, generator=g), -1)
        a = o.viterbi(x, lPd, lp0d, o.OBS_PROB, plan)
        b = o.viterbi(x, lPd, lp0d, o.OBS_PROB, plan)
        c = o.viterbi(x, lPd, lp0d, o.OBS_PROB, plan, follow=False)
        for u, v, w in zip(a, b, c):
            assert torch.equal(u, v) and torch.equal(u, w)
        pick = [0, B // 2, B - 1]
        cs, cd, _ = O.c_viterbi(lo_cr(x[pick].cpu().numpy()), lP.numpy(), lp0.numpy())
        assert np.array_equal(a[0][pick].cpu().numpy(), cs)


@pytest.mark.parametrize("N", [128, 64, 100, 256])
@pytest.mark.parametrize("T", [1, 2, 17, 65, 300, 2000])
def test_fb_posterior_followers_vs_pass(N, T):
    o = ops()
    rng = np.random.default_rng(N + T)
    B = 4
    lP, lp0 = O.hmm_params(banded(N))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    x = torch.from_numpy(rng.random((B, T, N), dtype=np.float32)).to(DEV)
    mask = o.FB_POSTERIOR | o.FB_FORWARD | o.FB_BACKWARD
    a = o.forward_backward(x, lPd, lp0d, o.OBS_PROB, mask, plan)
    b = o.forward_backward(x, lPd, lp0d, o.OBS_PROB, mask, plan, follow=False)
    if N == 128 or N == 64 or N == 256:
        assert torch.equal(a[0], b[0])          # the same arithmetic on the same rows
    else:
        np.testing.assert_allclose(a[0].cpu().numpy(), b[0].cpu().numpy(), atol=1e-6, rtol=0)
    for k in (1, 2, 3, 4):                      # forward, backward, loglik, lik_ref: identical bits
        assert torch.equal(a[k], b[k]), k
    _, _, post64, ll64 = O.c_fb64(lo_cr(x.cpu().numpy()), lP.numpy(), lp0.numpy())
    np.testing.assert_allclose(a[0].cpu().numpy(), post64, atol=2e-5, rtol=0)
    np.testing.assert_allclose(a[3].cpu().numpy(), ll64, rtol=2e-6)


def test_fb_followers_obs_log_and_posterior_only():
    """OBS_LOG emissions far below -87 (the row-max shift) and the posterior-only mask."""
    o = ops()
    rng = np.random.default_rng(3)
    B, T, N = 5, 900, 128
    lo = (-250.0 + 40.0 * rng.standard_normal((B, T, N))).astype(np.float32)
    lP, lp0 = O.hmm_params(banded(N))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    x = torch.from_numpy(lo).to(DEV)
    for mask in (o.FB_POSTERIOR, o.FB_POSTERIOR | o.FB_FORWARD | o.FB_BACKWARD):
        a = o.forward_backward(x, lPd, lp0d, o.OBS_LOG, mask, plan)
        b = o.forward_backward(x, lPd, lp0d, o.OBS_LOG, mask, plan, follow=False)
        assert torch.equal(a[0], b[0]) and torch.equal(a[3], b[3]) and torch.equal(a[4], b[4])
    _, _, post64, ll64 = O.c_fb64(lo, lP.numpy(), lp0.numpy())
    np.testing.assert_allclose(a[0].cpu().numpy(), post64, atol=2e-5)


def test_followers_beside_a_busy_stream():
    """A queue of GEMMs on another stream while both ops run with their followers: same bits as
    the idle-chip run, and the ops finish (the followers wait only for their own chains)."""
    o = ops()
    B, T, N = 32, 2000, 128
    lP, lp0 = O.hmm_params(banded(N))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.softmax(torch.randn(B, T, N, device=DEV, generator=g), -1)
    ref_v = o.viterbi(x, lPd, lp0d, o.OBS_PROB, plan)
    ref_f = o.forward_backward(x, lPd, lp0d, o.OBS_PROB, 7, plan)
    torch.cuda.synchronize()
    a = torch.randn(4096, 4096, device=DEV)
    busy, s1, s2 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    for s_ in (busy, s1, s2):
        s_.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(busy):
        for _ in range(30):
            a = a @ a * 1e-3
    with torch.cuda.stream(s1):
        v = o.viterbi(x, lPd, lp0d, o.OBS_PROB, plan)
    with torch.cuda.stream(s2):
        f = o.forward_backward(x, lPd, lp0d, o.OBS_PROB, 7, plan)
    torch.cuda.synchronize()
    for u, w in zip(v, ref_v):
        assert torch.equal(u, w)
    for u, w in zip(f, ref_f):
        assert torch.equal(u, w)


def test_wrong_banded_hint_marks_outputs_invalid():
    """A dense matrix's plan passed with the banded flags: the chains publish nothing, so the
    followers report invalid outputs (states -1, final score NaN, posterior NaN) -- the
    documented caller error -- instead of stale ones or a hang."""
    from pytorch_hmm_amd import _native as nat
    o = ops()
    rng = np.random.default_rng(1)
    B, T, N = 2, 150, 128
    lP, lp0 = O.hmm_params(torch.from_numpy(rng.random((N, N), dtype=np.float32) + 0.01))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    assert not plan._hmm355_banded
    x = torch.from_numpy(rng.random((B, T, N), dtype=np.float32)).to(DEV)
    L = nat.lib()
    p = nat.ptr
    st = nat.stream_of(torch.device(DEV))
    states = torch.zeros(B, T, dtype=torch.int64, device=DEV)
    delta = torch.empty(B, T, N, device=DEV)
    final = torch.zeros(B, device=DEV)
    ws = torch.empty(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=DEV)
    rc = L.hmm355_viterbi_plan_ex_f32(p(x), o.OBS_PROB, p(lPd), p(lp0d), p(plan), nat.VIT_PLAN_BANDED, B, T, N,
                                      p(states), p(delta), p(final), p(ws), ws.numel(), st)
    assert rc == 0
    torch.cuda.synchronize()
    assert bool((states == -1).all()) and bool(torch.isnan(final).all())
    post = torch.zeros(B, T, N, device=DEV)
    ll, lr = torch.empty(B, device=DEV), torch.zeros(B, device=DEV)
    wsf = torch.empty(L.hmm355_fb_workspace_bytes(B, T, N), dtype=torch.uint8, device=DEV)
    rc = L.hmm355_forward_backward_plan_f32(p(x), o.OBS_PROB, p(lPd), p(lp0d), p(plan), None, B, T, N,
                                            o.FB_POSTERIOR | nat.FB_PLAN_BANDED, p(post), None, None, p(ll), p(lr),
                                            p(wsf), wsf.numel(), st)
    assert rc == 0
    torch.cuda.synchronize()
    assert bool(torch.isnan(post).all()) and bool(torch.isnan(lr).all())


def test_followers_in_graph_replays():
    """Both ops with their followers captured into two HIP graphs each (own workspaces and
    outputs) and replayed alternately on changing inputs: every replay resets the counts (a
    kernel node: a captured hipMemsetAsync did not order against the chain launch in replay and
    the followers read the previous replay's rows), so each replay's outputs are its own."""
    o = ops()
    B, T, N = 8, 600, 128
    lP, lp0 = O.hmm_params(banded(N))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    g = torch.Generator(device=DEV).manual_seed(5)
    base = torch.softmax(torch.randn(B, T, N, device=DEV, generator=g), -1)
    obs = base.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            o.forward_backward(obs, lPd, lp0d, o.OBS_PROB, 7, plan)
            o.viterbi(obs, lPd, lp0d, o.OBS_PROB, plan)
    torch.cuda.synchronize()
    graphs, outs = [], []
    for _ in range(2):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            f = o.forward_backward(obs, lPd, lp0d, o.OBS_PROB, 7, plan)
            v = o.viterbi(obs, lPd, lp0d, o.OBS_PROB, plan)
        graphs.append(gr)
        outs.append((f, v))
    torch.cuda.synchronize()
    for k in range(6):
        x = base.clone()
        x[:, :, (7 * k) % N] += 0.5 + 0.1 * k
        obs.copy_(x)
        torch.cuda.synchronize()
        graphs[k % 2].replay()
        torch.cuda.synchronize()
        f, v = outs[k % 2]
        rf = o.forward_backward(obs, lPd, lp0d, o.OBS_PROB, 7, plan, follow=False)
        rv = o.viterbi(obs, lPd, lp0d, o.OBS_PROB, plan, follow=False)
        for a, b_ in zip(f, rf):
            assert torch.equal(a, b_), k
        for a, b_ in zip(v, rv):
            assert torch.equal(a, b_), k


def _counts(region, n):
    """the published counts of a workspace's count region (common.h: one 8-byte word per 128-B
    line, {call token, count ^ (token * 2654435761)})"""
    out = []
    for v in region.view(torch.int64).view(n, 16)[:, 0].cpu().tolist():
        v &= (1 << 64) - 1
        hi, lo = v >> 32, v & 0xffffffff
        out.append(lo ^ ((hi * 2654435761) & 0xffffffff))
    return out


def test_leaders_and_followers_did_the_work():
    """After a banded call the workspace's published counts (the last 2B x 128 bytes of each
    workspace, tokened words) show the hand-offs ran in the launch: every chain published completion
    (nblocks + 1), and the Viterbi log leaders converted every block they own (count = nblocks)."""
    from pytorch_hmm_amd import _native as nat
    o = ops()
    B, T, N = 4, 2000, 128
    nblocks = (T + 15) // 16
    lP, lp0 = O.hmm_params(banded(N))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.softmax(torch.randn(B, T, N, device=DEV, generator=g), -1)
    L, p, st = nat.lib(), nat.ptr, nat.stream_of(torch.device(DEV))
    states = torch.empty(B, T, dtype=torch.int64, device=DEV)
    delta = torch.empty(B, T, N, device=DEV)
    final = torch.empty(B, device=DEV)
    ws = torch.zeros(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=DEV)
    assert L.hmm355_viterbi_plan_ex_f32(p(x), o.OBS_PROB, p(lPd), p(lp0d), p(plan), nat.VIT_PLAN_BANDED, B, T, N,
                                        p(states), p(delta), p(final), p(ws), ws.numel(), st) == 0
    torch.cuda.synchronize()
    cnt = _counts(ws[ws.numel() - 2 * B * 128:], 2 * B)
    assert cnt[:B] == [nblocks + 1] * B, cnt     # the chains: psi rows and trellis complete
    assert cnt[B:] == [nblocks] * B, cnt         # the leaders: every block's log rows
    cs, _, _ = O.c_viterbi(lo_cr(x.cpu().numpy()), lP.numpy(), lp0.numpy())
    assert np.array_equal(states.cpu().numpy(), cs)
    post = torch.empty(B, T, N, device=DEV)
    ll, lr = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    nbytes = L.hmm355_fb_workspace_bytes(B, T, N)
    wsf = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)
    assert L.hmm355_forward_backward_plan_f32(p(x), o.OBS_PROB, p(lPd), p(lp0d), p(plan), None, B, T, N,
                                              o.FB_POSTERIOR | nat.FB_PLAN_BANDED, p(post), None, None, p(ll),
                                              p(lr), p(wsf), nbytes, st) == 0
    torch.cuda.synchronize()
    span = (2 * B * 128 + 255) // 256 * 256
    cf = _counts(wsf[nbytes - span: nbytes - span + 2 * B * 128], 2 * B)
    assert cf == [nblocks + 1] * (2 * B), cf      # both chains of every sequence published completion
    ref = o.forward_backward(x, lPd, lp0d, o.OBS_PROB, o.FB_POSTERIOR, plan, follow=False)
    assert torch.equal(post, ref[0])


@pytest.mark.parametrize("fill", ["ones_f32", "ff", "random", "stale_final"])
def test_counts_ignore_workspace_garbage(fill):
    """Eager calls reset no counts: each takes a fresh call token, so whatever the workspace
    holds (float ones, 0xff bytes, random bytes, the final counts of an earlier call) reads as
    no progress and the outputs are this call's own."""
    from pytorch_hmm_amd import _native as nat
    o = ops()
    B, T, N = 3, 700, 128
    lP, lp0 = O.hmm_params(banded(N))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = o.make_plan(lPd)
    g = torch.Generator(device=DEV).manual_seed(8)
    x = torch.softmax(torch.randn(B, T, N, device=DEV, generator=g), -1)
    L, p, st = nat.lib(), nat.ptr, nat.stream_of(torch.device(DEV))

    def filled(nbytes):
        if fill == "ones_f32":
            return torch.ones((nbytes + 3) // 4, device=DEV).view(torch.uint8)[:nbytes]
        if fill == "ff":
            return torch.full((nbytes,), 255, dtype=torch.uint8, device=DEV)
        if fill == "random":
            return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=DEV, generator=g)
        return torch.zeros(nbytes, dtype=torch.uint8, device=DEV)

    nv = L.hmm355_viterbi_workspace_bytes(B, T, N)
    ws = filled(nv)
    states = torch.empty(B, T, dtype=torch.int64, device=DEV)
    delta = torch.empty(B, T, N, device=DEV)
    final = torch.empty(B, device=DEV)
    x_other = torch.softmax(torch.randn(B, T, N, device=DEV, generator=g), -1)
    for inp in ([x_other, x] if fill == "stale_final" else [x]):
        assert L.hmm355_viterbi_plan_ex_f32(p(inp), o.OBS_PROB, p(lPd), p(lp0d), p(plan), nat.VIT_PLAN_BANDED, B, T,
                                            N, p(states), p(delta), p(final), p(ws), nv, st) == 0
    ref = o.viterbi(x, lPd, lp0d, o.OBS_PROB, plan, follow=False)
    assert torch.equal(states, ref[0]) and torch.equal(delta, ref[1])
    nf = L.hmm355_fb_workspace_bytes(B, T, N)
    wsf = filled(nf)
    post = torch.empty(B, T, N, device=DEV)
    ll, lr = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    for inp in ([x_other, x] if fill == "stale_final" else [x]):
        assert L.hmm355_forward_backward_plan_f32(p(inp), o.OBS_PROB, p(lPd), p(lp0d), p(plan), None, B, T, N,
                                                  o.FB_POSTERIOR | nat.FB_PLAN_BANDED, p(post), None, None, p(ll),
                                                  p(lr), p(wsf), nf, st) == 0
    reff = o.forward_backward(x, lPd, lp0d, o.OBS_PROB, o.FB_POSTERIOR, plan, follow=False)
    assert torch.equal(post, reff[0]) and torch.equal(lr, reff[4])
