"""GPU: the semi-Markov kernels (csrc/semimarkov.hip) through the C ABI.

- quad table: bit-exact against the C oracle (same k-ascending fp32 order);
- segment Viterbi: bit-exact (segments AND score) against the C restatement of the
  reference's literal loop (oracle/hmm_oracle.c: smk_viterbi_literal) given the same fp32
  quad table, including tie-heavy inputs where the first-candidate rule decides;
- SemiMarkovHMM.viterbi_decode against the reference's own outputs (tests/golden/smk_*):
  segments exact, score within 2e-6 relative (the reference's reduction order over
  features / frames is torch-CPU's, ISA-dependent);
- segment forward against the fp64 oracle (relative 2e-6 on log P, absolute 2e-4 on
  finite log alpha entries).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hmm_oracle as O
from pytorch_hmm_amd import ops
from pytorch_hmm_amd.semi_markov import SemiMarkovHMM
from test_semimarkov_cpu import SMK, load_model

pytestmark = pytest.mark.gpu
DEV = "cuda"


def t(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV)


def random_tables(rng, B, T, S, Dm, gaussian=True, ties=False):
    if ties:  # small integers: many exactly equal candidate totals
        q = rng.integers(0, 3, (B, T, S)).astype(np.float32)
        lT = np.full((S, S), -1.0, np.float32)
        du = -rng.integers(0, 2, (S, Dm)).astype(np.float32)
        li = np.zeros(S, np.float32)
        cs = np.zeros(S, np.float32) if gaussian else None
        return q, cs, li, lT, du
    q = (rng.random((B, T, S), dtype=np.float32) * 30).astype(np.float32)
    cs = rng.standard_normal(S).astype(np.float32) * 3 if gaussian else None
    li = np.log(rng.dirichlet(np.ones(S))).astype(np.float32)
    lT = np.log(rng.dirichlet(np.ones(S), size=S) + 1e-8).astype(np.float32)
    du = np.log(rng.dirichlet(np.ones(Dm), size=S) + 1e-8).astype(np.float32)
    return q, cs, li, lT, du


def gpu_viterbi(q, cs, li, lT, du, flags=0):
    ss, sd, cnt, sc = ops.semimarkov_viterbi(t(q), None if cs is None else t(cs), t(li), t(lT), t(du), flags)
    T = q.shape[1]
    ss, sd, cnt, sc = ss.cpu().numpy(), sd.cpu().numpy(), cnt.cpu().numpy(), sc.cpu().numpy()
    return [(ss[b, T - cnt[b]:], sd[b, T - cnt[b]:], sc[b]) for b in range(q.shape[0])]


def test_quad_bitexact():
    rng = np.random.default_rng(0)
    for (B, T, D, S) in [(2, 37, 80, 64), (1, 5, 3, 7), (3, 130, 13, 33)]:
        x = rng.standard_normal((B, T, D)).astype(np.float32)
        mu = rng.standard_normal((S, D)).astype(np.float32)
        var = np.exp(rng.standard_normal((S, D)).astype(np.float32) * 0.3).astype(np.float32)
        q = ops.semimarkov_quad(t(x), t(mu.T), t(var.T)).cpu().numpy()
        for b in range(B):
            assert np.array_equal(q[b], O.c_smk_quad(x[b], mu, var))


@pytest.mark.parametrize("seed,B,T,S,Dm,gaussian,ties", [
    (0, 3, 50, 4, 10, True, False),
    (1, 2, 200, 16, 20, True, False),
    (2, 2, 120, 7, 63, False, False),
    (3, 1, 80, 64, 40, True, False),
    (4, 4, 70, 5, 8, True, True),
    (5, 2, 90, 12, 16, False, True),
    (6, 2, 1, 3, 5, True, False),       # T = 1
    (7, 2, 3, 2, 10, True, False),      # T < Dmax
    (8, 1, 150, 1, 9, True, False),     # one state: only the initial segment is possible
])
def test_viterbi_bitexact_vs_literal(seed, B, T, S, Dm, gaussian, ties):
    rng = np.random.default_rng(seed)
    q, cs, li, lT, du = random_tables(rng, B, T, S, Dm, gaussian, ties)
    got = gpu_viterbi(q, cs, li, lT, du)
    for b in range(B):
        ss, sd, sc = O.c_smk_viterbi(q[b], cs, li, lT, du)
        gs, gd, gsc = got[b]
        assert np.array_equal(gs, ss) and np.array_equal(gd, sd), (b, gs, ss, gd, sd)
        assert np.float32(gsc) == np.float32(sc) or (np.isinf(gsc) and np.isinf(sc)), (gsc, sc)


def test_viterbi_unreachable_defaults():
    """min duration above T: every delta is -inf and the reference walks its defaults
    (state 0, duration 1) back to t = 0 (semi_markov.py:548-568)."""
    rng = np.random.default_rng(9)
    q, cs, li, lT, du = random_tables(rng, 1, 6, 3, 8)
    du[:, :] = -np.inf
    (gs, gd, gsc), = gpu_viterbi(q, cs, li, lT, du)
    ss, sd, sc = O.c_smk_viterbi(q[0], cs, li, lT, du)
    assert np.array_equal(gs, ss) and np.array_equal(gd, sd) and np.isinf(gsc) and np.isinf(sc)


@pytest.mark.parametrize("name", SMK)
def test_module_viterbi_vs_reference(name):
    g = golden(name)
    m = load_model(g).to(DEV)
    x = t(g["x"])
    res = m.viterbi_decode_batch(x)
    for b in range(x.shape[0]):
        n = int(g["seg_count"][b])
        st, du, sc = res[b]
        assert np.array_equal(st.cpu().numpy(), g["seg_states"][b, :n])
        assert np.array_equal(du.cpu().numpy(), g["seg_durs"][b, :n])
        ref = float(g["scores"][b])
        assert abs(float(sc) - ref) <= 2e-6 * max(1.0, abs(ref)), (float(sc), ref)
    st1, du1, sc1 = m.viterbi_decode(x[0])       # the reference's (T, D) signature
    assert st1.dtype == torch.int64 and sc1.dim() == 0
    n = int(g["seg_count"][0])
    assert np.array_equal(st1.cpu().numpy(), g["seg_states"][0, :n])


@pytest.mark.parametrize("seed,B,T,S,Dm,gaussian", [
    (0, 2, 40, 4, 10, True), (1, 1, 100, 16, 20, False), (2, 1, 60, 64, 40, True), (3, 2, 1, 3, 4, True)])
def test_forward_vs_fp64(seed, B, T, S, Dm, gaussian):
    rng = np.random.default_rng(seed)
    q, cs, li, lT, du = random_tables(rng, B, T, S, Dm, gaussian)
    lp, la = ops.semimarkov_forward(t(q), None if cs is None else t(cs), t(li), t(lT), t(du), True)
    lp, la = lp.cpu().numpy(), la.cpu().numpy()
    for b in range(B):
        tot, ra = O.c_smk_forward64(q[b], cs, li, lT, du)
        assert abs(lp[b] - tot) <= 2e-6 * max(1.0, abs(tot)), (lp[b], tot)
        fin = np.isfinite(ra)
        assert np.array_equal(fin, np.isfinite(la[b]))
        np.testing.assert_allclose(la[b][fin], ra[fin], rtol=2e-6, atol=2e-4)


def test_module_forward_and_supervised():
    g = golden("smk_gamma")
    m = load_model(g).to(DEV)
    x = t(g["x"])
    r = m(x)
    assert r["log_probability"].shape == (x.shape[0],)
    assert r["forward_variables"].shape == (x.shape[0], x.shape[1], m.num_states, m.max_duration)
    # log P(o) >= the best segmentation's score
    assert bool(torch.all(r["log_probability"].cpu() >= torch.from_numpy(g["scores"]) - 1e-3))
    n = int(g["seg_count"][0])
    st = t(g["seg_states"][0, :n]).unsqueeze(0)
    du = t(g["seg_durs"][0, :n]).unsqueeze(0)
    with torch.no_grad():
        rs = m(x[:1], st, du)
    np.testing.assert_allclose(float(rs["log_probability"]), g["supervised"][0][0], rtol=2e-6, atol=2e-5)


def test_c5_shape_smoke():
    """S=64, Dmax=40 (BASELINE config 5 shape), T=2000: segments tile the sequence and the
    decoded score equals the supervised score of the decoded segmentation plus the initial
    state's log-probability (the reference's supervised forward omits it, :280-306)."""
    torch.manual_seed(0)
    m = SemiMarkovHMM(64, 80, max_duration=40).to(DEV)
    x = torch.randn(2, 2000, 80, device=DEV)
    res = m.viterbi_decode_batch(x)
    for b, (st, du, sc) in enumerate(res):
        assert int(du.sum()) == 2000
        assert bool(torch.all(st[1:] != st[:-1]))
        with torch.no_grad():
            sup = m(x[b:b + 1], st.unsqueeze(0), du.unsqueeze(0))["log_probability"]
        li = float(m._log_initial()[int(st[0])])
        assert abs(float(sup) + li - float(sc)) <= 2e-6 * abs(float(sc)), (float(sup), li, float(sc))


# ------------------------------------------------------------------ the general form (S > 64 / Dmax > 63)
@pytest.mark.parametrize("seed,B,T,S,Dm,gaussian,ties", [
    (20, 2, 60, 70, 10, True, False),     # S > 64
    (21, 1, 200, 5, 80, True, False),     # Dmax > 63
    (22, 2, 150, 3, 100, False, True),    # Dmax > 63, tie-heavy
    (23, 1, 40, 130, 6, True, True),      # S > 128, tie-heavy
    (24, 2, 1, 90, 70, True, False),      # T = 1
    (25, 1, 70, 66, 64, False, False),    # both just past the register form
])
def test_wide_viterbi_bitexact_vs_literal(seed, B, T, S, Dm, gaussian, ties):
    """SemiMarkovHMM.viterbi_decode (semi_markov.py:455-570) beyond the register form's S <= 64,
    Dmax <= 63: csrc/semimarkov.hip smk_wide_kernel, bit-exact (segments and score) against
    the literal loop."""
    rng = np.random.default_rng(seed)
    q, cs, li, lT, du = random_tables(rng, B, T, S, Dm, gaussian, ties)
    got = gpu_viterbi(q, cs, li, lT, du)
    for b in range(B):
        ss, sd, sc = O.c_smk_viterbi(q[b], cs, li, lT, du)
        gs, gd, gsc = got[b]
        assert np.array_equal(gs, ss) and np.array_equal(gd, sd), (b, gs, ss, gd, sd)
        assert np.float32(gsc) == np.float32(sc) or (np.isinf(gsc) and np.isinf(sc)), (gsc, sc)


def test_wide_forced_equals_register_form():
    """HMM355_FORM_GENERAL forces the general form on a size the register form holds: the same
    segments and scores bit for bit, the forward within float64 tolerance of both."""
    rng = np.random.default_rng(30)
    for gaussian, ties in ((True, False), (False, True)):
        q, cs, li, lT, du = random_tables(rng, 3, 300, 20, 30, gaussian, ties)
        a = gpu_viterbi(q, cs, li, lT, du)
        fa = ops.semimarkov_forward(t(q), None if cs is None else t(cs), t(li), t(lT), t(du), True)
        b = gpu_viterbi(q, cs, li, lT, du, ops.FORM_GENERAL)
        fb = ops.semimarkov_forward(t(q), None if cs is None else t(cs), t(li), t(lT), t(du), True, ops.FORM_GENERAL)
        for (s1, d1, c1), (s2, d2, c2) in zip(a, b):
            assert np.array_equal(s1, s2) and np.array_equal(d1, d2) and np.float32(c1) == np.float32(c2)
        np.testing.assert_allclose(fb[0].cpu().numpy(), fa[0].cpu().numpy(), rtol=2e-6)
        la, lb = fa[1].cpu().numpy(), fb[1].cpu().numpy()
        assert np.array_equal(np.isfinite(la), np.isfinite(lb))
        np.testing.assert_allclose(lb[np.isfinite(lb)], la[np.isfinite(la)], rtol=2e-6, atol=2e-4)


@pytest.mark.parametrize("seed,B,T,S,Dm,gaussian", [(40, 1, 50, 72, 8, True), (41, 2, 120, 4, 90, False)])
def test_wide_forward_vs_fp64(seed, B, T, S, Dm, gaussian):
    rng = np.random.default_rng(seed)
    q, cs, li, lT, du = random_tables(rng, B, T, S, Dm, gaussian)
    lp, la = ops.semimarkov_forward(t(q), None if cs is None else t(cs), t(li), t(lT), t(du), True)
    lp, la = lp.cpu().numpy(), la.cpu().numpy()
    for b in range(B):
        tot, ra = O.c_smk_forward64(q[b], cs, li, lT, du)
        assert abs(lp[b] - tot) <= 2e-6 * max(1.0, abs(tot)), (lp[b], tot)
        fin = np.isfinite(ra)
        assert np.array_equal(fin, np.isfinite(la[b]))
        np.testing.assert_allclose(la[b][fin], ra[fin], rtol=2e-6, atol=2e-4)


def test_wide_module_large_model():
    """SemiMarkovHMM(68 states, max_duration 66) end to end through the module: the quad table
    for S > 64 and the general-form decode, checked against the literal loop on the module's
    own tables."""
    torch.manual_seed(3)
    m = SemiMarkovHMM(68, 12, max_duration=66).to(DEV)
    x = torch.randn(1, 90, 12, device=DEV)
    (st, du, sc), = m.viterbi_decode_batch(x)
    with torch.no_grad():
        q, cs, li, lT, dtab = (v.cpu().numpy() if v is not None else None for v in m._tables(x))
    ss, sd, sref = O.c_smk_viterbi(q[0], cs, li, lT, dtab)
    assert np.array_equal(st.cpu().numpy(), ss) and np.array_equal(du.cpu().numpy(), sd)
    assert np.float32(float(sc)) == np.float32(sref)
