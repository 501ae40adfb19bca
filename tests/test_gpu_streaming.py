"""GPU: the streaming decoders (csrc/stream.hip) through the C ABI and the drop-in
StreamingHMMProcessor.

- kernels vs the C oracle (itself pinned to the reference, tests/test_streaming_cpu.py):
  exact states, step scores, hypotheses and back-pointers, given the same fp32 inputs —
  the reference's own emission log-probs from the fixtures, and random / tie-heavy inputs up
  to N = 256, K = 32 (K = 16 above N = 128) over several 64-frame tiles;
- the processor (emission net on the GPU) against the reference's process_chunk and direct
  decode outputs: states exact; confidences within 1e-5 relative (GEMM rounding in the
  emission net).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hmm_oracle as O
from pytorch_hmm_amd import ops
from pytorch_hmm_amd.streaming import StreamingHMMProcessor
from test_streaming_cpu import NAMES, beam_chain

pytestmark = pytest.mark.gpu
DEV = "cuda"


def t(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV)


def gpu_beam(emis, log_T, K, hs, hl, first):
    """emis (B,T,N); hs/hl lists per stream -> per stream (hs, hl, parent, hstate, states)."""
    B = emis.shape[0]
    S = ops.STREAM_SLOTS
    hs_t = torch.full((B, S), float("-inf"))
    hl_t = torch.zeros((B, S), dtype=torch.int32)
    for b in range(B):
        hs_t[b, :len(hs[b])] = torch.from_numpy(np.asarray(hs[b], np.float32))
        hl_t[b, :len(hl[b])] = torch.from_numpy(np.asarray(hl[b], np.int32))
    hs_t, hl_t = hs_t.to(DEV), hl_t.to(DEV)
    cnt = torch.tensor([len(x) for x in hs], dtype=torch.int32, device=DEV)
    fr = torch.tensor([int(f) for f in first], dtype=torch.int32, device=DEV)
    live = max(len(x) for x in hs)
    states, par, hst = ops.stream_beam(t(emis), t(log_T), K, hs_t, hl_t, cnt, fr, live_max=live)
    out = []
    for b in range(B):
        k = int(cnt[b])
        out.append((hs_t[b, :k].cpu().numpy(), hl_t[b, :k].cpu().numpy(), par[b].cpu().numpy(),
                    hst[b].cpu().numpy(), states[b].cpu().numpy()))
    return out


@pytest.mark.parametrize("name", NAMES)
def test_kernels_on_reference_emissions(name):
    g = golden(name)
    N, D, K = (int(v) for v in g["config"][:3])
    log_n = float(torch.log(torch.tensor(N)))
    prev = -1
    for i in range(int(g["config"][6])):
        st, sc = ops.stream_greedy(t(g[f"emis{i}"][None]), t(g["log_T"]), torch.tensor([prev], dtype=torch.int32,
                                   device=DEV), log_n)
        ost, osc = O.c_stream_greedy(g[f"emis{i}"], g["log_T"], prev, log_n)
        assert np.array_equal(st[0].cpu().numpy(), ost) and np.array_equal(sc[0].cpu().numpy(), osc)
        assert np.array_equal(st[0].cpu().numpy(), g[f"greedy_states{i}"])
        prev = int(ost[-1])
    hs = [np.full(min(K, N), -float(torch.log(torch.tensor(N, dtype=torch.float))), np.float32)]
    hl = [np.arange(min(K, N))]
    first = [True]
    for i, (rhs, rhl, plen, rstates, _) in enumerate(beam_chain(g)):
        (ghs, ghl, par, hst, gst), = gpu_beam(g[f"emis{i}"][None], g["log_T"], K, hs, hl, first)
        assert np.array_equal(ghs, rhs) and np.array_equal(ghl, rhl)
        assert np.array_equal(ghs, g[f"beam_hs{i}"])
        assert np.array_equal(gst, g[f"beam_states{i}"])
        hs, hl, first = [ghs], [ghl], [False]


@pytest.mark.parametrize("seed,B,T,N,K,ties,k0", [
    (0, 3, 300, 128, 16, False, None), (1, 2, 129, 64, 8, False, None), (2, 4, 70, 7, 5, True, None),
    (3, 2, 65, 100, 3, True, None), (4, 1, 1, 9, 1, False, None),
    (5, 2, 80, 20, 4, False, 12),     # beam lowered: 12 live hypotheses, K = 4
    (6, 2, 90, 100, 8, True, 8),
    # round 5: N <= 256 (log T read from global memory above 128) and beams up to 32
    (7, 2, 150, 256, 16, False, None), (8, 2, 100, 200, 12, True, None), (9, 2, 130, 129, 9, False, None),
    (10, 2, 130, 128, 32, False, None), (11, 2, 70, 64, 32, True, None), (12, 2, 90, 50, 24, False, 30)])
def test_kernels_vs_oracle_random(seed, B, T, N, K, ties, k0):
    rng = np.random.default_rng(seed)
    if ties:
        emis = -rng.integers(0, 3, (B, T, N)).astype(np.float32)
        log_T = -rng.integers(0, 2, (N, N)).astype(np.float32)
    else:
        emis = np.log(rng.dirichlet(np.ones(N), size=(B, T))).astype(np.float32)
        log_T = np.log(rng.dirichlet(np.ones(N), size=N) + 1e-8).astype(np.float32)
    prev = rng.integers(-1, N, B).astype(np.int32)
    st, sc = ops.stream_greedy(t(emis), t(log_T), t(prev), 1.5)
    for b in range(B):
        ost, osc = O.c_stream_greedy(emis[b], log_T, int(prev[b]), 1.5)
        assert np.array_equal(st[b].cpu().numpy(), ost) and np.array_equal(sc[b].cpu().numpy(), osc)
    k0 = [min(K, N) if k0 is None else k0] * B
    hs = [np.sort(rng.standard_normal(k).astype(np.float32))[::-1].copy() for k in k0]
    hl = [rng.integers(0, N, k) for k in k0]
    first = [b % 2 == 0 for b in range(B)]
    res = gpu_beam(emis, log_T, K, hs, hl, first)
    for b in range(B):
        ohs, ohl, opar, ohst = O.c_stream_beam(emis[b], log_T, K, hs[b], hl[b], first[b])
        ghs, ghl, gpar, ghst, gst = res[b]
        assert np.array_equal(ghs, ohs) and np.array_equal(ghl, ohl)
        k = len(ohs)
        assert np.array_equal(gpar[:, :k], opar[:, :k]) and np.array_equal(ghst[:, :k], ohst[:, :k])


def load_proc(g, beam):
    N, D, K, cs, md, la = (int(v) for v in g["config"][:6])
    p = StreamingHMMProcessor(N, D, chunk_size=cs, lookahead_frames=la, max_delay_frames=md,
                              use_beam_search=beam, beam_width=K)
    sd = {k[len("param__"):].replace("__", "."): torch.from_numpy(v) for k, v in g.items() if k.startswith("param__")}
    p.load_state_dict(sd)
    return p.to(DEV).eval()


@pytest.mark.parametrize("name", NAMES)
def test_processor_vs_reference(name):
    g = golden(name)
    n = int(g["config"][6])
    for beam in (False, True):
        p = load_proc(g, beam)
        tag = "beam" if beam else "greedy"
        for i in range(n):
            f = t(g[f"feat{i}"])
            st, conf = p._beam_search_decode(f) if beam else p._greedy_decode(f)
            assert np.array_equal(st.cpu().numpy(), g[f"{tag}_states{i}"]), (tag, i)
            np.testing.assert_allclose(conf.cpu().numpy(), g[f"{tag}_conf{i}"], rtol=1e-5)
        # process_chunk on a fresh stream
        p.reset_streaming_state()
        ptag = "pb" if beam else "pg"
        for i in range(int(g["config"][7])):
            r = p.process_chunk(t(g[f"chunk{i}"]))
            assert r.status == str(g[f"{ptag}_status{i}"]), (ptag, i, r.status)
            if r.decoded_states is not None:
                assert np.array_equal(r.decoded_states.cpu().numpy(), g[f"{ptag}_states{i}"])
                assert r.confidence == pytest.approx(float(g[f"{ptag}_conf{i}"]), rel=1e-5)
        stats = p.get_performance_stats()
        assert "avg_processing_time_ms" in stats or "message" in stats
        assert p.flush_buffer().status == "flushed"


def test_beam_limits():
    """K <= 32, and K <= 16 above N = 128 (the lane's candidate mask): larger asks raise."""
    rng = np.random.default_rng(0)
    for N, K in ((200, 17), (64, 33)):
        emis = np.log(rng.dirichlet(np.ones(N), size=(1, 8))).astype(np.float32)
        log_T = np.log(rng.dirichlet(np.ones(N), size=N) + 1e-8).astype(np.float32)
        with pytest.raises((ValueError, RuntimeError)):
            gpu_beam(emis, log_T, K, [np.zeros(1, np.float32)], [np.zeros(1, np.int64)], [True])
