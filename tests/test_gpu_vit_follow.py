"""GPU: psi followers (HMM355_VIT_PLAN_DENSE; csrc/vit_kern.h vit_psi_follow) -- the argmax
pointers of a dense chain computed beside it by extra workgroups of the chain's launch, which
follow the rows the chain's helpers publish.  Checked bit-exact against the C oracle
(hmm.py:154-184) with the followers on and off, at chunk edges, with a batch larger than the
CUs left for followers, and with the flag given for a banded plan (the followers step aside)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _dense(N, seed):
    rng = np.random.default_rng(seed)
    return torch.from_numpy(rng.random((N, N), dtype=np.float32))


def _run(lo, lP, lp0, plan, follow, monkeypatch, mode=None):
    from pytorch_hmm_amd import ops
    x = torch.from_numpy(lo).to(DEV)
    s, d, f = ops.viterbi(x, lP.to(DEV), lp0.to(DEV), ops.OBS_LOG if mode is None else mode, plan, follow=follow)
    torch.cuda.synchronize()
    return s.cpu().numpy(), d.cpu().numpy(), f.cpu().numpy()


@pytest.mark.parametrize("N", [128, 100, 64, 37])
@pytest.mark.parametrize("T", [1, 2, 63, 64, 65, 129, 1000])
def test_followers_vs_c_oracle(N, T, monkeypatch):
    from pytorch_hmm_amd import ops
    lP, lp0 = O.hmm_params(_dense(N, N + T))
    plan = ops.make_plan(lP.to(DEV))
    assert not plan._hmm355_banded
    rng = np.random.default_rng(T)
    B = 5
    lo = np.log(rng.random((B, T, N), dtype=np.float32) + np.float32(1e-3)).astype(np.float32)
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    for follow in (True, False):
        s, d, f = _run(lo, lP, lp0, plan, follow, monkeypatch)
        assert np.array_equal(d, cd), follow
        assert np.array_equal(s, cs), follow
        assert np.array_equal(f, cd[:, -1].max(-1)), follow


def test_followers_tie_heavy_and_large_batch(monkeypatch):
    """Coarse emissions (many equal trellis values: the first index on ties) and B = 300, more
    sequences than CUs: no room for followers, the pass after the chain does every chunk."""
    from pytorch_hmm_amd import ops
    N = 128
    lP, lp0 = O.hmm_params(_dense(N, 3))
    plan = ops.make_plan(lP.to(DEV))
    for B, T in ((8, 2000), (300, 130)):
        rng = np.random.default_rng(B)
        lo = np.round(-(rng.random((B, T, N)) * 4), 0).astype(np.float32)
        cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
        s, d, _ = _run(lo, lP, lp0, plan, True, monkeypatch)
        assert np.array_equal(d, cd) and np.array_equal(s, cs), B


def test_dense_flag_with_banded_plan(monkeypatch):
    """The flag with a banded plan: the followers see a banded chain and leave; the psi pass
    after the chain does its usual work."""
    import pytorch_hmm_amd._native as nat
    from pytorch_hmm_amd import ops
    N, B, T = 128, 3, 300
    lP, lp0 = O.hmm_params(O.left_to_right_matrix(N, 0.7))
    lPd = lP.to(DEV)
    plan = ops.make_plan(lPd)
    assert plan._hmm355_banded
    rng = np.random.default_rng(1)
    lo = np.log(rng.random((B, T, N), dtype=np.float32) + np.float32(1e-3)).astype(np.float32)
    obs = torch.from_numpy(lo).to(DEV)
    L = nat.lib()
    states = torch.zeros(B, T, dtype=torch.int64, device=DEV)
    delta = torch.empty(B, T, N, device=DEV)
    final = torch.zeros(B, device=DEV)
    ws = torch.empty(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=DEV)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = L.hmm355_viterbi_plan_ex_f32(p(obs), ops.OBS_LOG, p(lPd), p(lp0.to(DEV)), p(plan), nat.VIT_PLAN_DENSE,
                                      B, T, N, p(states), p(delta), p(final), p(ws), ws.numel(),
                                      nat.stream_of(torch.device(DEV, 0)))
    assert rc == 0
    torch.cuda.synchronize()
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    assert np.array_equal(delta.cpu().numpy(), cd) and np.array_equal(states.cpu().numpy(), cs)


def test_followers_obs_prob(monkeypatch):
    """OBS_PROB (the chain's helpers take log(x + 1e-8)): followers on and off agree."""
    from pytorch_hmm_amd import ops
    N, B, T = 128, 6, 777
    lP, lp0 = O.hmm_params(_dense(N, 11))
    plan = ops.make_plan(lP.to(DEV))
    g = torch.Generator().manual_seed(2)
    x = torch.softmax(torch.randn(B, T, N, generator=g), -1).numpy()
    a = _run(x, lP, lp0, plan, True, monkeypatch, ops.OBS_PROB)
    b = _run(x, lP, lp0, plan, False, monkeypatch, ops.OBS_PROB)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


def _abi_viterbi(lo_dev, lPd, lp0d, plan, flags, stream=None):
    """hmm355_viterbi_plan_ex_f32 through ctypes; returns (states, delta, workspace)."""
    import pytorch_hmm_amd._native as nat
    from pytorch_hmm_amd import ops
    B, T, N = lo_dev.shape
    L = nat.lib()
    states = torch.zeros(B, T, dtype=torch.int64, device=DEV)
    delta = torch.empty(B, T, N, device=DEV)
    final = torch.zeros(B, device=DEV)
    # (the OBS_LOG size: test_followers_complete_chunks reads the done words from the end)
    ws = torch.empty(L.hmm355_viterbi_workspace_bytes_ex(B, T, N, ops.OBS_LOG), dtype=torch.uint8, device=DEV)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = nat.stream_of(torch.device(DEV, 0)) if stream is None else ctypes.c_void_p(stream.cuda_stream)
    rc = L.hmm355_viterbi_plan_ex_f32(p(lo_dev), ops.OBS_LOG, p(lPd), p(lp0d), p(plan), flags, B, T, N,
                                      p(states), p(delta), p(final), p(ws), ws.numel(), st)
    assert rc == 0
    return states, delta, ws


def test_followers_complete_chunks():
    """The followers really do the work: after a dense decode the workspace's done words
    (viterbi.hip layout: B*nchunks bytes, 256-aligned, before the banded followers' 2B counts of
    128 bytes each at the end) mark the chunks they finished.
    With two followers per sequence keeping pace with the chain nearly every chunk is theirs."""
    import pytorch_hmm_amd._native as nat
    from pytorch_hmm_amd import ops
    N, B, T = 128, 8, 2000
    lP, lp0 = O.hmm_params(_dense(N, 5))
    lPd = lP.to(DEV)
    plan = ops.make_plan(lPd)
    rng = np.random.default_rng(4)
    lo = np.log(rng.random((B, T, N), dtype=np.float32) + np.float32(1e-3)).astype(np.float32)
    s, d, ws = _abi_viterbi(torch.from_numpy(lo).to(DEV), lPd, lp0.to(DEV), plan, nat.VIT_PLAN_DENSE)
    torch.cuda.synchronize()
    nc = (T + 63) // 64
    span = (B * nc + 255) // 256 * 256
    end = ws.numel() - 2 * B * 128
    done = ws[end - span: end - span + B * nc].cpu().numpy()
    frac = float((done == 1).mean())
    print(f"followers finished {int((done == 1).sum())} of {B * nc} chunks")
    assert frac > 0.5, frac
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    assert np.array_equal(d.cpu().numpy(), cd) and np.array_equal(s.cpu().numpy(), cs)


def test_followers_no_cliff_beside_busy_stream(monkeypatch):
    """A second stream keeps the chip busy (a queue of GEMMs) while a dense decode runs: the
    decode with followers stays within 2x of the same decode without them under the same load,
    and far from the old per-task 200 ms wait bound (one 2 ms stall budget per launch now)."""
    from pytorch_hmm_amd import ops
    N, B, T = 128, 32, 2000
    lP, lp0 = O.hmm_params(_dense(N, 9))
    lPd, lp0d = lP.to(DEV), lp0.to(DEV)
    plan = ops.make_plan(lPd)
    g = torch.Generator().manual_seed(3)
    lo = torch.log(torch.rand(B, T, N, generator=g) + 1e-3).to(DEV)
    a = torch.randn(4096, 4096, device=DEV)
    busy = torch.cuda.Stream()
    vs = torch.cuda.Stream()

    def run(follow):
        with torch.cuda.stream(vs):
            ops.viterbi(lo, lPd, lp0d, ops.OBS_LOG, plan, follow=follow)   # warm
        torch.cuda.synchronize()
        times = []
        for _ in range(3):
            with torch.cuda.stream(busy):
                for _ in range(40):
                    a2 = a @ a
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(vs):
                e0.record()
                out = ops.viterbi(lo, lPd, lp0d, ops.OBS_LOG, plan, follow=follow)
                e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        return min(times), out
    t_on, out_on = run(True)
    t_off, out_off = run(False)
    print(f"busy-stream Viterbi op: followers on {t_on:.3f} ms, off {t_off:.3f} ms")
    assert torch.equal(out_on[0], out_off[0]) and torch.equal(out_on[1], out_off[1])
    assert t_on < 2 * t_off + 1.0, (t_on, t_off)
    assert t_on < 50.0
