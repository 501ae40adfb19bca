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
