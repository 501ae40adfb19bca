"""CPU: the semi-Markov oracle and the host-side tables against the reference's own outputs
(tests/golden/smk_*.npz, written by tests/golden/make_golden.py from SemiMarkovHMM).

What is pinned here:
- the per-candidate duration table and the segment constant the kernels consume are the
  reference's bits (exact);
- the C restatement of semi_markov.py:455-570 (oracle/hmm_oracle.c: smk_viterbi_literal)
  reproduces the reference's segmentations exactly and its score to ~1 ulp of the segment
  sums (the reference's torch-CPU reduction order over features / frames is ISA-dependent);
- the fp64 segment forward equals brute-force enumeration of all segmentations.  The
  reference's own forward raises TypeError (semi_markov.py:353), so its VALUE is parity
  unpinned against the reference and pinned by enumeration instead.
"""

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hmm_oracle as O
from pytorch_hmm_amd.semi_markov import DurationModel, SemiMarkovHMM

SMK = ["smk_gamma", "smk_poisson", "smk_gaussian", "smk_neuraldur", "smk_neuralobs", "smk_short", "smk_s8"]


def load_model(g):
    S, D, Dmax, T, nseq, min_d = (int(v) for v in g["config"])
    m = SemiMarkovHMM(S, D, max_duration=Dmax, duration_distribution=str(g["dist"]),
                      observation_model=str(g["obs_model"]), min_duration=min_d)
    sd = {k[len("param__"):].replace("__", "."): torch.from_numpy(v) for k, v in g.items() if k.startswith("param__")}
    m.load_state_dict(sd)
    return m.eval()


def host_tables(m, x):
    """The kernel's inputs, formed on CPU: quad from the C oracle (kernel order)."""
    if m.observation_model_type == "gaussian":
        cs, var = m._gaussian_tables()
        q = O.c_smk_quad(x, m.observation_means.detach().numpy(), var.numpy())
        cs = cs.numpy()
    else:
        with torch.no_grad():
            q = m.neural_obs_model(torch.from_numpy(x).unsqueeze(0))[0].numpy()
        cs = None
    with torch.no_grad():
        return q, cs, m._log_initial().numpy(), m._log_transitions().numpy(), m.duration_model.candidate_table().numpy()


@pytest.mark.parametrize("name", SMK)
def test_duration_tables_bitexact(name):
    g = golden(name)
    m = load_model(g)
    with torch.no_grad():
        tab = m.duration_model.candidate_table().numpy()
        dist = m.duration_model(torch.arange(m.num_states)).numpy()
    assert np.array_equal(tab, g["dur_candidates"]), np.abs(tab - g["dur_candidates"]).max()
    assert np.array_equal(dist, g["dur_distribution"])
    if m.observation_model_type == "gaussian":
        assert np.array_equal(m._gaussian_tables()[0].numpy(), g["seg_const"])


@pytest.mark.parametrize("name", SMK)
def test_oracle_viterbi_matches_reference(name):
    g = golden(name)
    m = load_model(g)
    x = g["x"]
    for b in range(x.shape[0]):
        q, cs, li, lT, du = host_tables(m, x[b])
        ss, sd, sc = O.c_smk_viterbi(q, cs, li, lT, du)
        n = int(g["seg_count"][b])
        assert np.array_equal(ss, g["seg_states"][b, :n]), (ss, g["seg_states"][b, :n])
        assert np.array_equal(sd, g["seg_durs"][b, :n])
        ref = float(g["scores"][b])
        assert abs(float(sc) - ref) <= 2e-6 * max(1.0, abs(ref)), (sc, ref)


@pytest.mark.parametrize("name", ["smk_gamma", "smk_poisson", "smk_neuralobs"])
def test_supervised_forward_matches_reference(name):
    g = golden(name)
    m = load_model(g)
    x = torch.from_numpy(g["x"])
    for b in range(x.shape[0]):
        n = int(g["seg_count"][b])
        st = torch.from_numpy(g["seg_states"][b, :n]).unsqueeze(0)
        du = torch.from_numpy(g["seg_durs"][b, :n]).unsqueeze(0)
        with torch.no_grad():
            r = m(x[b:b + 1], st, du)
        got = [float(r[k]) for k in ("log_probability", "log_observation", "log_duration", "log_transition")]
        np.testing.assert_allclose(got, g["supervised"][b], rtol=2e-6, atol=2e-5)


def _all_segmentations(T, S, Dm):
    """Every (states, durations) segmentation of T frames with no self-transitions."""
    out = []

    def rec(t, segs):
        if t == T:
            out.append(list(segs))
            return
        for d in range(1, min(Dm, T - t) + 1):
            for s in range(S):
                if segs and segs[-1][0] == s:
                    continue
                rec(t + d, segs + [(s, d)])
    rec(0, [])
    return out


def _seg_score(q, cs, li, lT, du, segs):
    t, tot, prev = 0, 0.0, None
    for s, d in segs:
        Q = float(np.sum(q[t:t + d, s], dtype=np.float64))
        o = (float(cs[s]) - 0.5 * Q) if cs is not None else Q
        tot += (float(li[s]) if prev is None else float(lT[prev, s])) + o + float(du[s, d - 1])
        prev, t = s, t + d
    return tot


@pytest.mark.parametrize("seed,T,S,Dm", [(0, 4, 3, 10), (1, 6, 3, 3), (2, 7, 2, 4), (3, 5, 4, 2)])
def test_forward64_equals_enumeration(seed, T, S, Dm):
    rng = np.random.default_rng(seed)
    q = rng.random((T, S), dtype=np.float32) * 4
    cs = rng.standard_normal(S).astype(np.float32)
    li = np.log(rng.dirichlet(np.ones(S))).astype(np.float32)
    lT = np.log(rng.dirichlet(np.ones(S), size=S)).astype(np.float32)
    du = np.log(rng.dirichlet(np.ones(Dm), size=S)).astype(np.float32)
    segs = _all_segmentations(T, S, Dm)
    scores = np.array([_seg_score(q, cs, li, lT, du, sg) for sg in segs])
    ref = float(np.log(np.sum(np.exp(scores - scores.max()))) + scores.max())
    tot, _ = O.c_smk_forward64(q, cs, li, lT, du)
    assert abs(tot - ref) < 1e-9 * max(1, abs(ref)), (tot, ref)
    # the Viterbi oracle finds the best segmentation of the same enumeration
    ss, sd, sc = O.c_smk_viterbi(q, cs, li, lT, du)
    best = segs[int(np.argmax(scores))]
    assert abs(float(sc) - scores.max()) < 1e-4
    assert _seg_score(q, cs, li, lT, du, list(zip(ss.tolist(), sd.tolist()))) == pytest.approx(scores.max(), abs=1e-4)
    assert len(best) >= 1


def test_duration_model_api_shapes():
    """tests/test_integration.py:151-209 of the reference: shapes and sample bounds."""
    torch.manual_seed(0)
    for kind in ["gamma", "poisson", "gaussian", "neural"]:
        dm = DurationModel(num_states=5, max_duration=20, distribution_type=kind)
        idx = torch.randint(0, 5, (3,))
        assert dm(idx).shape == (3, 20)
        smp = dm.sample(idx)
        assert len(smp) == 3 and bool(torch.all(smp >= 1))
    with pytest.raises(ValueError):
        DurationModel(3, distribution_type="weibull")
    m = SemiMarkovHMM(4, 6, max_duration=10)
    st, du, obs = m.sample(num_states=5, max_length=50)
    assert len(st) == len(du) and obs.shape[1] == 6
    assert sum(int(d) for d in du.tolist()) == obs.shape[0] <= 50  # frames per segment = int(duration)


def test_param_table_cache_rebuilds_on_new_parameter():
    """A replaced parameter must invalidate the device tables even if its storage address and
    version coincide with the old one (ADVICE: address + version keys alone can alias)."""
    torch.manual_seed(0)
    m = SemiMarkovHMM(3, 4, max_duration=6)
    t0 = m._param_tables(torch.device("cpu"))
    assert m._param_tables(torch.device("cpu")) is t0  # unchanged parameters: cache hit
    m.transition_logits = torch.nn.Parameter(torch.randn(3, 3))
    t1 = m._param_tables(torch.device("cpu"))
    assert t1 is not t0
    assert not torch.equal(t1[3], t0[3])
    with torch.no_grad():
        m.initial_logits.add_(1.0)  # in-place update bumps the version
    assert m._param_tables(torch.device("cpu")) is not t1
