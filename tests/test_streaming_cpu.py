"""CPU: the streaming-decoder oracle (oracle/hmm_oracle.c: stream_greedy_f32 /
stream_beam_f32) against the reference's own StreamingHMMProcessor outputs
(tests/golden/stream_*.npz, written by tests/golden/make_golden.py): greedy states and
confidences, beam hypotheses (scores, last states, path lengths) after every chunk, and the
returned best-path states — all exact, given the reference's emission log-probabilities."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hmm_oracle as O

NAMES = ["stream_n5", "stream_n12", "stream_n3k16"]


def beam_chain(g):
    """Run the oracle over the fixture's chunks; yields per chunk (hs, hl, plen, states, path0)."""
    N, D, K = (int(v) for v in g["config"][:3])
    nchunks = int(g["config"][6])
    hs = np.full(min(K, N), -float(torch.log(torch.tensor(N, dtype=torch.float))), np.float32)
    hl = np.arange(min(K, N))
    paths = [[] for _ in range(len(hs))]
    first = True
    for i in range(nchunks):
        e = g[f"emis{i}"]
        T = e.shape[0]
        hs, hl, par, hst = O.c_stream_beam(e, g["log_T"], K, hs, hl, first)
        first = False
        new = []
        for r in range(len(hs)):
            tail, rr = [], r
            for t in range(T - 1, -1, -1):
                tail.append(int(hst[t, rr]))
                rr = int(par[t, rr])
            new.append(paths[rr] + tail[::-1])
        paths = new
        yield hs, hl, np.array([len(p) for p in paths]), np.array(paths[0][-T:]), np.array(paths[0])


@pytest.mark.parametrize("name", NAMES)
def test_greedy_oracle_matches_reference(name):
    g = golden(name)
    N = int(g["config"][0])
    log_n = float(torch.log(torch.tensor(N)))
    prev = -1
    for i in range(int(g["config"][6])):
        st, sc = O.c_stream_greedy(g[f"emis{i}"], g["log_T"], prev, log_n)
        assert np.array_equal(st, g[f"greedy_states{i}"])
        # the score is the oracle's; confidence = exp(score) goes through torch-CPU's exp, whose
        # vector path differs by an ulp between host ISAs (AVX2 here vs AVX-512 on the GPU box)
        np.testing.assert_allclose(torch.exp(torch.from_numpy(sc)).numpy(), g[f"greedy_conf{i}"],
                                   rtol=2.5e-7, atol=0)
        prev = int(st[-1])


@pytest.mark.parametrize("name", NAMES)
def test_beam_oracle_matches_reference(name):
    g = golden(name)
    for i, (hs, hl, plen, states, path0) in enumerate(beam_chain(g)):
        assert np.array_equal(hs, g[f"beam_hs{i}"]), (i, hs, g[f"beam_hs{i}"])
        assert np.array_equal(hl, g[f"beam_hl{i}"])
        assert np.array_equal(plen, g[f"beam_plen{i}"])
        assert np.array_equal(path0, g[f"beam_path0_{i}"])
        assert np.array_equal(states, g[f"beam_states{i}"])
        conf = torch.exp(torch.tensor(hs[0]) / int(plen[0]))
        assert float(conf) == float(g[f"beam_conf{i}"][0])


def test_async_worker_queue_semantics():
    """start/add/get/stop of the async path (reference streaming.py:123-181), with the chunk
    decode replaced by a host stub so no GPU is needed: results come back in order, a
    failing chunk warns and the worker keeps serving, stop() joins promptly."""
    import time as _t
    import warnings as _w
    from pytorch_hmm_amd.streaming import StreamingHMMProcessor
    p = StreamingHMMProcessor(num_states=4, feature_dim=3, chunk_size=4)
    calls = []

    def fake(chunk):
        if chunk.numel() == 0:
            raise RuntimeError("empty")
        calls.append(int(chunk[0, 0]))
        return int(chunk[0, 0])
    p.process_chunk = fake
    p.start_async_processing()
    p.start_async_processing()  # idempotent
    with _w.catch_warnings(record=True) as rec:
        _w.simplefilter("always")
        assert p.add_audio_chunk_async(torch.zeros(0, 3))
        for i in range(3):
            assert p.add_audio_chunk_async(torch.full((2, 3), float(i)))
        got, t_end = [], _t.time() + 10
        while len(got) < 3 and _t.time() < t_end:
            r = p.get_result_async()
            if r is None:
                _t.sleep(0.01)
            else:
                got.append(r)
    assert got == [0, 1, 2] and calls == [0, 1, 2]
    assert any("Error in async processing" in str(x.message) for x in rec)
    t0 = _t.time()
    p.stop_async_processing()
    assert _t.time() - t0 < 2 and p.processing_thread is None and not p.is_processing
    assert p.get_result_async() is None


def test_log_transition_table_cached_per_parameter_version():
    """The per-chunk log(softmax + 1e-8) table is built once per parameter version (no host
    round trip per chunk), and rebuilt when the logits change in place or are replaced."""
    from pytorch_hmm_amd.streaming import StreamingHMMProcessor
    torch.manual_seed(0)
    p = StreamingHMMProcessor(6, 4, chunk_size=16, overlap_size=4).eval()
    a = p._log_transitions()
    assert p._log_transitions() is a
    ref = torch.log(torch.softmax(p.transition_logits.detach(), -1) + 1e-8)
    assert torch.equal(a, ref)
    with torch.no_grad():
        p.transition_logits.add_(0.5 * torch.randn_like(p.transition_logits))
    b = p._log_transitions()
    assert b is not a and torch.equal(b, torch.log(torch.softmax(p.transition_logits.detach(), -1) + 1e-8))
    p.transition_logits = torch.nn.Parameter(torch.zeros(6, 6))
    c = p._log_transitions()
    assert c is not b and torch.allclose(c, torch.full((6, 6), float(np.log(1 / 6 + 1e-8))))


def test_log_transition_cache_sees_data_writes_state_dicts_and_training():
    """writes through .data do not bump the version counter.  Training mode re-forms
    the table every chunk (as the reference does); in eval mode load_state_dict, train()/eval()
    and refresh_transitions() invalidate it."""
    from pytorch_hmm_amd.streaming import StreamingHMMProcessor
    torch.manual_seed(1)
    p = StreamingHMMProcessor(5, 4, chunk_size=16, overlap_size=4)
    want = lambda: torch.log(torch.softmax(p.transition_logits.detach(), -1) + 1e-8)
    assert p.training
    a = p._log_transitions()
    p.transition_logits.data -= 0.3 * torch.randn(5, 5)      # an optimiser writing .data
    assert torch.equal(p._log_transitions(), want()) and not torch.equal(a, want())
    p.eval()
    b = p._log_transitions()
    assert p._log_transitions() is b
    sd = {k: v.clone() for k, v in p.state_dict().items()}
    sd["transition_logits"] = torch.randn(5, 5)
    p.load_state_dict(sd)
    assert torch.equal(p._log_transitions(), want())
    p.transition_logits.data.copy_(torch.randn(5, 5))        # bypasses the version counter...
    p.refresh_transitions()                                  # ...so the documented hook
    assert torch.equal(p._log_transitions(), want())
    p.transition_logits.data.mul_(2.0)
    p.train(); p.eval()
    assert torch.equal(p._log_transitions(), want())


def test_optimize_for_latency_steps():
    """optimize_for_latency (reference streaming.py:444-483): one adjustment per call, from the
    mean chunk time: above the target narrow the beam (not below 2), then greedy, then chunks
    x0.8 (not below 80); below half the target beam search back on at width 4, then +1 up to 8;
    in between nothing; without timing data a warning and nothing."""
    import warnings as _w
    from pytorch_hmm_amd.streaming import StreamingHMMProcessor
    p = StreamingHMMProcessor(4, 3, chunk_size=160, beam_width=3)
    with _w.catch_warnings(record=True) as rec:
        _w.simplefilter("always")
        p.optimize_for_latency(10.0)
    assert any("No performance data" in str(x.message) for x in rec) and p.beam_width == 3
    p.processing_times.extend([40.0, 60.0])         # mean 50 ms
    seen = []
    for _ in range(6):
        p.optimize_for_latency(25.0)
        seen.append((p.use_beam_search, p.beam_width, p.chunk_size))
    assert seen == [(True, 2, 160), (False, 2, 160), (False, 2, 128), (False, 2, 102), (False, 2, 81),
                    (False, 2, 80)]
    p.optimize_for_latency(60.0)                    # 50 in [30, 60]: unchanged
    assert (p.use_beam_search, p.beam_width, p.chunk_size) == (False, 2, 80)
    for want in [(True, 4), (True, 5), (True, 6), (True, 7), (True, 8), (True, 8)]:
        p.optimize_for_latency(200.0)
        assert (p.use_beam_search, p.beam_width) == want


def test_latency_breakdown_reports_measured_phases():
    """get_latency_breakdown (reference streaming.py:485-503): {} before any chunk; then the
    reference's keys, each the mean of the host-timed phase, and 'total' the mean chunk time."""
    from pytorch_hmm_amd.streaming import StreamingHMMProcessor, _PHASES
    p = StreamingHMMProcessor(4, 3, chunk_size=8)
    assert p.get_latency_breakdown() == {}
    for k, vals in zip(_PHASES, ([1.0, 3.0], [2.0, 2.0], [0.5, 0.5], [4.0, 6.0], [0.25, 0.75])):
        p.phase_times[k].extend(vals)
    p.processing_times.extend([8.0, 12.0])
    got = p.get_latency_breakdown()
    assert list(got) == ["feature_extraction", "emission_computation", "transition_computation",
                         "viterbi_decoding", "bookkeeping", "total"]
    assert got == {"feature_extraction": 2.0, "emission_computation": 2.0, "transition_computation": 0.5,
                   "viterbi_decoding": 5.0, "bookkeeping": 0.5, "total": 10.0}


def test_phase_clock_charges_marks():
    """The per-chunk clock charges the time between marks to the named phase."""
    import time as _t
    from pytorch_hmm_amd.streaming import StreamingHMMProcessor
    p = StreamingHMMProcessor(4, 3)
    p._mark("viterbi_decoding")                      # no chunk in flight: ignored
    p._clock = {"_last": _t.perf_counter()}
    _t.sleep(0.02)
    p._mark("viterbi_decoding")
    p._mark("bookkeeping")
    assert p._clock["viterbi_decoding"] >= 15.0 and p._clock["bookkeeping"] < 15.0


def test_adaptive_latency_controller_rules(monkeypatch):
    """AdaptiveLatencyController.update (reference streaming.py:506-592): nothing before ten
    observations or within a second of the last recommendation; then from the last 20
    latencies: overloaded (mean > 1.2 target) -> chunk x0.9 (adopted), beam width 3, beam search
    iff mean <= 2 target; headroom (mean < 0.6 target, variance < 10) -> chunk x1.1 only with
    > 100 frames buffered, width 6, beam on; jittery (variance > 25) -> greedy, chunk x0.9 (not
    adopted)."""
    import pytorch_hmm_amd as ph
    from pytorch_hmm_amd import streaming as S
    clock = [1000.0]
    monkeypatch.setattr(S.time, "time", lambda: clock[0])
    c = ph.AdaptiveLatencyController(initial_chunk_size=160, min_chunk_size=80, max_chunk_size=320,
                                     target_latency_ms=30.0)
    assert (c.chunk_size, c.min_chunk_size, c.max_chunk_size, c.target_latency_ms) == (160, 80, 320, 30.0)
    for _ in range(9):
        assert c.update(50.0, 100) == {}
    assert c.update(50.0, 100) == {"chunk_size": 144, "beam_width": 3, "use_beam_search": True}
    assert c.chunk_size == 144
    clock[0] += 0.5
    assert c.update(50.0, 100) == {}                 # cooldown
    clock[0] += 1.0
    for _ in range(20):
        c.latency_history.append(70.0)
    assert c.update(70.0, 100) == {"chunk_size": 129, "beam_width": 3, "use_beam_search": False}
    # headroom: needs a full window of low, steady latencies
    c2 = ph.AdaptiveLatencyController(target_latency_ms=30.0)
    for _ in range(10):
        r = c2.update(10.0, 50)
    assert r == {"beam_width": 6, "use_beam_search": True} and c2.chunk_size == 160
    assert c2.update(10.0, 50) == {}                # cooldown after a recommendation
    clock[0] += 2.0
    assert c2.update(10.0, 150) == {"chunk_size": 176, "beam_width": 6, "use_beam_search": True}
    # jittery: mean inside the band, variance large
    c3 = ph.AdaptiveLatencyController(target_latency_ms=30.0)
    for v in [20.0, 40.0] * 5:
        r = c3.update(v, 0)
    assert r == {"use_beam_search": False, "chunk_size": 144} and c3.chunk_size == 160
