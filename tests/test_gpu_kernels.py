"""GPU parity: the HIP kernels (through the C ABI / torch ops) against the reference's
golden vectors (tests/golden, produced by the reference itself) and the oracle.

Contracts:
  * Viterbi, mixture Viterbi, HSMM: bit-exact states and scores/trellis given identical
    fp32 log-emissions and log-transition tables.
  * Forward-backward: fp32 tolerances written per test (the reference's own fp32 result
    differs from float64 by up to ~6e-4 on posteriors at T=2000, N=128).
"""
import math

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hmm_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def t(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a)).to(DEV, dtype)


@pytest.fixture(scope="module", autouse=True)
def _native():
    import pytorch_hmm_amd._native as nat
    nat.lib()  # fail loudly if the HIP library is missing
    assert torch.cuda.is_available()


def ops():
    from pytorch_hmm_amd import ops as o
    return o


# ---------------------------------------------------------------------------- Viterbi
@pytest.mark.parametrize("name", ["hmmpytorch_l2r", "hmmpytorch_ergodic", "hmmpytorch_small",
                                  "hmmpytorch_n200"])
def test_viterbi_bitexact_given_log_obs(name):
    g = golden(name)
    o = ops()
    states, delta, final = o.viterbi(t(g["log_obs"]), t(g["log_P"]), t(g["log_p0"]), o.OBS_LOG)
    torch.cuda.synchronize()
    assert np.array_equal(states.cpu().numpy(), g["states"])
    assert np.array_equal(delta.cpu().numpy().view(np.int32), g["log_delta"].view(np.int32))
    assert np.array_equal(final.cpu().numpy(), g["log_delta"][:, -1].max(-1))


@pytest.mark.parametrize("name", ["hmmpytorch_l2r", "hmmpytorch_ergodic", "hmmpytorch_small",
                                  "hmmpytorch_n200"])
def test_viterbi_end_to_end_prob_input(name):
    """In-kernel log(x + 1e-8) (correctly rounded) vs the reference's torch-CPU log."""
    g = golden(name)
    o = ops()
    states, delta, _ = o.viterbi(t(g["obs"]), t(g["log_P"]), t(g["log_p0"]), o.OBS_PROB)
    lo_gpu_path = delta.cpu().numpy()
    assert np.array_equal(states.cpu().numpy(), g["states"])
    # any difference can only come from a 1-ulp log difference on an emission
    np.testing.assert_allclose(lo_gpu_path, g["log_delta"], rtol=2e-6, atol=1e-5)


def test_viterbi_ties_first_index():
    g = golden("ties")
    o = ops()
    s1, d1, _ = o.viterbi(t(g["log_obs"]), t(g["log_P"]), t(g["log_p0"]), o.OBS_LOG)
    s2, d2, _ = o.viterbi(t(g["log_obs"]), t(g["log_Pu"]), t(g["log_p0u"]), o.OBS_LOG)
    assert np.array_equal(s1.cpu().numpy(), g["states"])
    assert np.array_equal(s2.cpu().numpy(), g["states_u"])
    assert np.array_equal(d2.cpu().numpy(), g["log_delta_u"])


def test_viterbi_hmmlayer_c1_params():
    g = golden("hmmlayer_c1")
    o = ops()
    states, delta, _ = o.viterbi(t(g["log_obs"]), t(g["log_P2"]), t(g["log_p02"]), o.OBS_LOG)
    assert np.array_equal(states.cpu().numpy(), g["states3"])
    assert np.array_equal(delta.cpu().numpy(), g["log_delta3"])


@pytest.mark.parametrize("B,T,N", [(3, 1, 7), (2, 65, 64), (5, 129, 100), (1, 300, 256), (4, 64, 128),
                                   (2, 257, 33)])
def test_viterbi_vs_c_oracle_shapes(B, T, N):
    """Ragged T around the 16-step staging blocks and 64-step chunks, N padded to 64/128/256."""
    rng = np.random.default_rng(B * 1000 + T * 7 + N)
    lo = np.log(rng.random((B, T, N), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    P = rng.random((N, N), dtype=np.float32) ** 4
    lP = np.log(P / P.sum(1, keepdims=True) + np.float32(1e-8)).astype(np.float32)
    init = np.log(np.full(N, 1.0 / N, np.float32) + np.float32(1e-8)).astype(np.float32)
    cs, cd, _ = O.c_viterbi(lo, lP, init)
    o = ops()
    states, delta, final = o.viterbi(t(lo), t(lP), t(init), o.OBS_LOG)
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(delta.cpu().numpy(), cd)


# --------------------------------------------------------------------- forward-backward
@pytest.mark.parametrize("name", ["hmmpytorch_l2r", "hmmpytorch_ergodic", "hmmpytorch_small",
                                  "hmmpytorch_n200", "wiki"])
def test_forward_backward_vs_reference(name):
    g = golden(name)
    o = ops()
    obs = g["obs"] if g["obs"].ndim == 3 else g["obs"][None]
    post, fwd, bwd, loglik, lik_ref = o.forward_backward(
        t(obs), t(g["log_P"]), t(g["log_p0"]), o.OBS_PROB, o.FB_POSTERIOR | o.FB_FORWARD | o.FB_BACKWARD)
    post, fwd, bwd = post.cpu().numpy(), fwd.cpu().numpy(), bwd.cpu().numpy()
    # posterior: absolute tolerance 2e-4 (reference fp32 vs fp64 differs by up to 7.7e-5 here)
    np.testing.assert_allclose(post, g["posterior"], atol=2e-4, rtol=0)
    # forward/backward = exp(log alpha)/exp(log beta): relative 1e-4 where representable
    for ours, ref in ((fwd, g["forward"]), (bwd, g["backward"])):
        big = ref > 1e-30
        np.testing.assert_allclose(ours[big], ref[big], rtol=1e-4)
        assert np.all(np.abs(ours[~big]) < 1e-29)
    if "loglik" in g:
        np.testing.assert_allclose(loglik.cpu().numpy(), g["loglik"], rtol=1e-5)
    lik = g["compute_likelihood"].reshape(-1)
    np.testing.assert_allclose(lik_ref.cpu().numpy(), lik, rtol=1e-5, atol=1e-5)


def test_forward_backward_vs_fp64_oracle_shapes():
    for (B, T, N) in [(2, 1, 5), (3, 17, 64), (2, 300, 100), (1, 50, 256), (2, 33, 130)]:
        rng = np.random.default_rng(T * N)
        obs = rng.random((B, T, N), dtype=np.float32)
        P = rng.random((N, N), dtype=np.float32)
        lP, lp0 = O.hmm_params(torch.from_numpy(P))
        la, lb, post64, ll64 = O.c_fb64(np.log(obs + np.float32(1e-8)), lP.numpy(), lp0.numpy())
        o = ops()
        post, _, _, loglik, _ = o.forward_backward(t(obs), t(lP), t(lp0), o.OBS_PROB, o.FB_POSTERIOR)
        np.testing.assert_allclose(post.cpu().numpy(), post64, atol=2e-5)
        np.testing.assert_allclose(loglik.cpu().numpy(), ll64, rtol=2e-6)


# ------------------------------------------------------------------------- mixture
@pytest.mark.parametrize("name", ["mixture_s16", "mixture_s128", "mixture_single"])
def test_gmm_emission_vs_reference(name):
    g = golden(name)
    o = ops()
    lp = o.gmm_diag_logprob(t(g["x"]), t(g["means"]), t(g["log_vars"]), t(g["log_w"]), 1).cpu().numpy()
    ref = g["log_probs"]
    # fp32 summation-order differences only: relative 2e-6 of the magnitude
    np.testing.assert_allclose(lp, ref, rtol=2e-6, atol=2e-5)
    lp64 = O.c_gmm64(g["x"], g["means"], g["log_vars"], g["log_w"])
    np.testing.assert_allclose(lp, lp64, rtol=2e-6, atol=2e-5)


@pytest.mark.parametrize("D,S,C,mix", [(200, 16, 4, 1), (513, 8, 2, 1), (1031, 5, 1, 0)])
def test_gmm_emission_wide_features_vs_fp64_oracle(D, S, C, mix):
    """Feature dimensions beyond 128 (round 4: the scorer's D loop has no per-D state): the
    GMM scores against the fp64 C oracle (mixture_gaussian.py:157-214; C = 1 without the LSE is
    the Gaussian / HSMM emission, hmm_layer.py:270-323)."""
    rng = np.random.default_rng(D)
    B, T = 2, 77
    x = rng.standard_normal((B, T, D)).astype(np.float32)
    means = (rng.standard_normal((S, C, D)) * 0.3).astype(np.float32)
    log_vars = (rng.standard_normal((S, C, D)) * 0.2).astype(np.float32)
    log_w = np.log(np.full((S, C), 1.0 / C, np.float32)).astype(np.float32)
    o = ops()
    lp = o.gmm_diag_logprob(t(x), t(means), t(log_vars), t(log_w), mix).cpu().numpy()
    lp64 = O.c_gmm64(x, means, log_vars, log_w)
    if not mix:   # C = 1 without the LSE: the plain component log-density (log_w = 0)
        lp64 = lp64 - log_w[:, 0][None, None, :]
    np.testing.assert_allclose(lp, lp64, rtol=2e-6, atol=2e-5 * D / 80)


@pytest.mark.parametrize("name", ["mixture_s16", "mixture_s128", "mixture_single"])
def test_mixture_viterbi_bitexact_given_lp(name):
    g = golden(name)
    o = ops()
    S = g["log_T"].shape[0]
    init = O.mixture_init_vector(S).numpy()
    states, _, final = o.viterbi(t(g["log_probs"]), t(g["log_T"]), t(init), o.OBS_LOG)
    assert np.array_equal(states.cpu().numpy(), g["states"])
    assert np.array_equal(final.cpu().numpy(), g["scores"])


# ---------------------------------------------------------------------------- HSMM
@pytest.mark.parametrize("name", ["hsmm_s5", "hsmm_s2", "hsmm_s8", "hsmm_d96"])
def test_hsmm_bitexact_given_lp(name):
    g = golden(name)
    o = ops()
    states, scores = o.hsmm_viterbi(t(g["log_probs"]), t(g["dur_log_probs"]), t(g["log_T"]))
    assert np.array_equal(states.cpu().numpy(), g["states"])
    assert np.array_equal(scores.cpu().numpy(), g["scores"])


@pytest.mark.parametrize("seed,T,S,Dm", [(1, 60, 6, 9), (2, 45, 4, 20), (3, 80, 9, 7), (4, 130, 12, 33),
                                         (5, 150, 90, 50), (6, 100, 30, 110)])
def test_hsmm_ties_vs_c_oracle(seed, T, S, Dm):
    """Coarse values (many equal totals): the first-candidate rule and the backtrace's
    re-resolution of earlier candidates that round to the same total."""
    rng = np.random.default_rng(seed)
    lp = np.round(-(rng.random((2, T, S)) * 8 + 4), 1).astype(np.float32)
    dur = np.round(np.log(rng.random((S, Dm)) + 1e-3), 1).astype(np.float32)
    logT = np.round(np.log(rng.random((S, S)) + 1e-3), 1).astype(np.float32)
    # the literal 5-deep loop where it is cheap; the reorganised C form (proven equal to it in
    # tests/test_oracle.py) for the large geometries
    cs, csc = O.c_hsmm(lp, dur, logT, literal=S * Dm <= 400)
    o = ops()
    states, scores = o.hsmm_viterbi(t(lp), t(dur), t(logT))
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(scores.cpu().numpy(), csc)


# every kernel geometry (csrc/hsmm.hip hsmm_cfg): (4,16,64) S <= 64 / Dmax <= 63, (8,16,64)
# Dmax <= 71, (4,16,128) S <= 128 / Dmax <= 63, and the general form beyond
@pytest.mark.parametrize("B,T,S,Dm", [(2, 150, 16, 12), (1, 300, 64, 40), (3, 70, 7, 63), (2, 260, 40, 100),
                                      (1, 200, 100, 50), (2, 180, 128, 63), (1, 90, 65, 63), (2, 130, 3, 127)])
def test_hsmm_vs_c_oracle(B, T, S, Dm):
    rng = np.random.default_rng(T + S + Dm)
    lp = (-(rng.random((B, T, S), dtype=np.float32) * 40 + 80)).astype(np.float32)
    dur = np.log(rng.random((S, Dm), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    logT = np.log(rng.random((S, S), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    cs, csc = O.c_hsmm(lp, dur, logT)
    o = ops()
    states, scores = o.hsmm_viterbi(t(lp), t(dur), t(logT))
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(scores.cpu().numpy(), csc)


# the general form (csrc/hsmm_wide.hip): sizes beyond the register-slot geometries, and
# (HMM355_FORM_GENERAL) sizes those also cover, against the C oracle; uniform and coarse
# tie-heavy tables
@pytest.mark.parametrize("B,T,S,Dm,force,coarse", [(2, 120, 200, 12, 0, False), (1, 150, 70, 80, 0, False),
                                                   (2, 90, 8, 150, 0, False), (2, 100, 140, 10, 0, True),
                                                   (2, 200, 16, 12, 1, False), (1, 300, 64, 40, 1, False),
                                                   (2, 150, 12, 33, 1, True)])
def test_hsmm_wide_vs_c_oracle(B, T, S, Dm, force, coarse):
    rng = np.random.default_rng(T + S + Dm)
    if coarse:
        lp = np.round(-(rng.random((B, T, S)) * 8 + 4), 1).astype(np.float32)
        dur = np.round(np.log(rng.random((S, Dm)) + 1e-3), 1).astype(np.float32)
        logT = np.round(np.log(rng.random((S, S)) + 1e-3), 1).astype(np.float32)
    else:
        lp = (-(rng.random((B, T, S), dtype=np.float32) * 40 + 80)).astype(np.float32)
        dur = np.log(rng.random((S, Dm), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
        logT = np.log(rng.random((S, S), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    cs, csc = O.c_hsmm(lp, dur, logT)
    o = ops()
    states, scores = o.hsmm_viterbi(t(lp), t(dur), t(logT), o.FORM_GENERAL if force else 0)
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(scores.cpu().numpy(), csc)


@pytest.mark.parametrize("case", ["random", "peaked", "ties", "longdur", "s128"])
def test_hsmm_chunked_backtrace_equals_serial(case):
    """The chunked backtrace (parallel chunk walks from guessed segments, stitched top-down,
    csrc/hsmm.hip) against the serial walk and the C oracle: uniform random tables (short
    segments), peaked emissions (long segments), coarse tie-heavy values, Dmax > the 64-frame
    chunk, and 128 states."""
    rng = np.random.default_rng(11)
    B, T, S, Dm = {"random": (3, 700, 64, 40), "peaked": (2, 900, 32, 60), "ties": (2, 500, 20, 30),
                   "longdur": (2, 600, 16, 127), "s128": (2, 400, 128, 40)}[case]
    lp = (-(rng.random((B, T, S), dtype=np.float32) * 40 + 80)).astype(np.float32)
    if case == "peaked":  # one favoured state per 37-frame run: long segments
        good = (np.arange(T)[:, None] // 37) % S == np.arange(S)[None, :]
        lp = (lp - 30 * ~good[None]).astype(np.float32)
    if case == "ties":
        lp = np.round(lp).astype(np.float32)
    dur = np.log(rng.random((S, Dm), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    logT = np.log(rng.random((S, S), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    if case == "ties":
        dur, logT = np.round(dur).astype(np.float32), np.round(logT).astype(np.float32)
    cs, csc = O.c_hsmm(lp, dur, logT)
    o = ops()
    s1, sc1 = o.hsmm_viterbi(t(lp), t(dur), t(logT), o.FORM_SERIAL_WALK)
    s2, sc2 = o.hsmm_viterbi(t(lp), t(dur), t(logT))
    assert np.array_equal(s1.cpu().numpy(), cs) and np.array_equal(sc1.cpu().numpy(), csc)
    assert np.array_equal(s2.cpu().numpy(), cs) and np.array_equal(sc2.cpu().numpy(), csc)


def test_hsmm_impossible_transitions_and_durations():
    """-inf in the tables (a left-to-right transition matrix, durations below a minimum, a state
    no segment may take): the kernel's folded conditions (M = -inf for slots not started, -inf
    duration rows) against the C oracle."""
    rng = np.random.default_rng(5)
    B, T, S, Dm = 3, 140, 12, 20
    lp = (-(rng.random((B, T, S), dtype=np.float32) * 30 + 10)).astype(np.float32)
    dur = np.log(rng.random((S, Dm), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    dur[:, :2] = -np.inf          # min_duration 3
    dur[5, :] = -np.inf           # state 5 never holds a segment
    logT = np.log(rng.random((S, S), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    logT[np.tril_indices(S, -1)] = -np.inf   # left to right
    cs, csc = O.c_hsmm(lp, dur, logT)
    o = ops()
    states, scores = o.hsmm_viterbi(t(lp), t(dur), t(logT))
    assert np.array_equal(states.cpu().numpy(), cs)
    assert np.array_equal(scores.cpu().numpy(), csc)


@pytest.mark.parametrize("T,Dm", [(1, 1), (7, 7), (50, 64), (300, 400), (1024, 1024), (90, 40)])
def test_hsmm_single_state_contiguous_sum(T, Dm):
    """num_states = 1: obs_log_probs[b] is (T, 1), so the reference's only scoring segment
    sum(lp[0:T, 0]) is a CONTIGUOUS slice and torch.sum takes its vectorised order; pinned to
    torch.sum itself (hsmm.py:266-274).  T > Dmax: no segment scores (-inf; the reference's walk
    would not terminate), the path stays the reference's torch.zeros."""
    rng = np.random.default_rng(T + Dm)
    lp = (-(rng.random((3, T, 1), dtype=np.float32) * 40 + 80)).astype(np.float32)
    dur = np.log(rng.random((1, Dm), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    logT = np.zeros((1, 1), np.float32)
    o = ops()
    states, scores = o.hsmm_viterbi(t(lp), t(dur), t(logT))
    assert np.array_equal(states.cpu().numpy(), np.zeros((3, T), np.int64))
    lpt = torch.from_numpy(lp)
    for b in range(3):
        want = (torch.sum(lpt[b][0:T, 0]) + torch.from_numpy(dur)[0, T - 1]).numpy() if T <= Dm else np.float32(-np.inf)
        assert scores[b].cpu().numpy().tobytes() == np.float32(want).tobytes()


@pytest.mark.parametrize("S,Dm,wide", [(4, 20, 0), (40, 100, 0), (6, 30, 1)])
def test_hsmm_no_path_leaves_reference_zeros(S, Dm, wide):
    """A left-to-right chain of S states with durations <= Dm cannot cover T > S * Dm frames:
    every final score is -inf, the walk has no predecessor after its first segment, and the
    frames it never reaches keep the reference's torch.zeros value (hsmm.py:332; the reference's
    own walk would not terminate here).  Both the register-slot and the general form."""
    rng = np.random.default_rng(S)
    T = S * Dm + 10
    lp = (-(rng.random((2, T, S), dtype=np.float32) * 10 + 5)).astype(np.float32)
    dur = np.log(rng.random((S, Dm), dtype=np.float32) + np.float32(1e-3)).astype(np.float32)
    logT = np.full((S, S), -np.inf, np.float32)
    for i in range(S - 1):
        logT[i, i + 1] = 0.0
    o = ops()
    for _ in range(2):  # the second call reuses a dirty output buffer from the caching allocator
        states, scores = o.hsmm_viterbi(t(lp), t(dur), t(logT), o.FORM_GENERAL if wide else 0)
        assert np.all(np.isneginf(scores.cpu().numpy()))
        assert np.array_equal(states.cpu().numpy(), np.zeros((2, T), np.int64))


def test_hsmm_workspace_check_slices_the_batch(monkeypatch):
    """The general form's (B,T,S,Dmax+1) workspace is checked against free device memory: a
    batch that does not fit is decoded in slices that do (same results), and a single sequence
    that does not fit raises OutOfMemoryError with the sizes, before any allocation."""
    from pytorch_hmm_amd import ops as o
    import pytorch_hmm_amd._native as nat
    rng = np.random.default_rng(9)
    B, T, S, Dm = 5, 120, 70, 80
    lp = (-(rng.random((B, T, S), dtype=np.float32) * 40 + 80)).astype(np.float32)
    dur = np.log(rng.random((S, Dm), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    logT = np.log(rng.random((S, S), dtype=np.float32) + np.float32(1e-8)).astype(np.float32)
    cs, csc = O.c_hsmm(lp, dur, logT)
    per_seq = nat.lib().hmm355_hsmm_workspace_bytes(1, T, S, Dm)
    monkeypatch.setattr(o, "_HSMM_WS_CHECK_BYTES", 0)
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda *a: 0)
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda *a: 0)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a: (int(2.5 * per_seq / 0.9), 1 << 40))
    states, scores = o.hsmm_viterbi(t(lp), t(dur), t(logT))   # slices of 2, 2, 1
    assert np.array_equal(states.cpu().numpy(), cs) and np.array_equal(scores.cpu().numpy(), csc)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a: (per_seq // 2, 1 << 40))
    with pytest.raises(torch.cuda.OutOfMemoryError, match="max_duration"):
        o.hsmm_viterbi(t(lp), t(dur), t(logT))


# ---------------------------------------------- forward-backward on log-emissions (OBS_LOG)
@pytest.mark.parametrize("mat", ["l2r", "ergodic", "rand"])
@pytest.mark.parametrize("B,T,N", [(2, 300, 128), (3, 77, 40), (1, 50, 256), (2, 129, 64)])
def test_forward_backward_obs_log_low_emissions(mat, B, T, N):
    """Log-emissions in [-400, -80] (Gaussian log-densities at D = 80, the producers
    mixture_gaussian.py:354 / hsmm.py:225): exp(lo) alone underflows, the chains stage
    exp(lo - max_j lo) and carry the shift in the log-scales.  Banded (l2r, ergodic) and dense
    (rand) chains, against the fp64 oracle: posterior atol 2e-5, loglik rtol 2e-6."""
    rng = np.random.default_rng(B * T + N)
    if mat == "l2r":
        P = O.left_to_right_matrix(N, 0.7)
    elif mat == "ergodic":
        P = O.transition_matrix(N, "ergodic")
    else:
        P = torch.from_numpy(rng.random((N, N), dtype=np.float32))
    lP, lp0 = O.hmm_params(P)
    lo = (-(rng.random((B, T, N)) * 320 + 80)).astype(np.float32)
    lo[0, T // 2, :] -= 5000.0    # a whole row far below the rest: only the shift keeps it
    la, lb, post64, ll64 = O.c_fb64(lo, lP.numpy(), lp0.numpy())
    o = ops()
    post, fwd, bwd, loglik, lik_ref = o.forward_backward(t(lo), t(lP), t(lp0), o.OBS_LOG,
                                                         o.FB_POSTERIOR | o.FB_FORWARD | o.FB_BACKWARD)
    assert np.all(np.isfinite(post.cpu().numpy())) and np.all(np.isfinite(loglik.cpu().numpy()))
    np.testing.assert_allclose(post.cpu().numpy(), post64, atol=2e-5, rtol=0)
    np.testing.assert_allclose(loglik.cpu().numpy(), ll64, rtol=2e-6)
    # exp(log alpha) / exp(log beta) underflow to 0 wherever the true values do
    assert np.all(fwd.cpu().numpy()[np.exp(la) == 0] == 0)


def test_forward_backward_obs_log_matches_obs_prob():
    """Ordinary probabilities: OBS_LOG on log(x + 1e-8) and OBS_PROB on x give the same
    posteriors (the shift is exact bookkeeping)."""
    rng = np.random.default_rng(9)
    B, T, N = 2, 200, 128
    obs = rng.random((B, T, N), dtype=np.float32)
    lP, lp0 = O.hmm_params(O.left_to_right_matrix(N, 0.7))
    lo = np.log((obs + np.float32(1e-8)).astype(np.float64)).astype(np.float32)
    o = ops()
    p1, _, _, l1, _ = o.forward_backward(t(obs), t(lP), t(lp0), o.OBS_PROB, o.FB_POSTERIOR)
    p2, _, _, l2, _ = o.forward_backward(t(lo), t(lP), t(lp0), o.OBS_LOG, o.FB_POSTERIOR)
    np.testing.assert_allclose(p1.cpu().numpy(), p2.cpu().numpy(), atol=1e-5)
    np.testing.assert_allclose(l1.cpu().numpy(), l2.cpu().numpy(), rtol=2e-6)
