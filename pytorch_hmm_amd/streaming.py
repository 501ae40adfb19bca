"""Real-time streaming decoder — drop-in for the reference's streaming.py (§8(f) row 4).

``StreamingHMMProcessor`` (streaming.py:35-503) keeps the reference's constructor,
parameter names (``transition_logits``, ``emission_net``) and chunk/buffer behaviour.  Its two
per-frame Python loops run as gfx950 kernels (csrc/stream.hip): ``_greedy_decode``
(streaming.py:267-320) as one wave-argmax chain per chunk and ``_beam_search_decode``
(streaming.py:322-377) as K rounds of wave argmax per frame over the hypotheses'
expansions, with the reference's stable tie order.  The emission network stays a torch
module (two GEMMs on hipBLASLt); the chunk buffering and bookkeeping are host logic, as in
the reference.

The latency-control helpers are host policy with the reference's public behaviour
(``optimize_for_latency`` streaming.py:444-483, ``get_latency_breakdown`` :485-503,
``AdaptiveLatencyController`` :506-592), written here as explicit rule tables
(``_LATENCY_STEPS``, ``AdaptiveLatencyController._RULES``).  One difference by design: the
reference's breakdown is a fixed 10/30/10/40/10 % split of the mean chunk time; here each
phase of a decoded chunk is timed on the host (``_PHASES``) and the breakdown reports those
means under the reference's keys.
"""
import queue
import threading
import time
import warnings
from collections import deque
from dataclasses import dataclass
from typing import Any, Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


@dataclass
class StreamingResult:
    """Result of one processed chunk (streaming.py:23-32)."""
    decoded_states: Optional[torch.Tensor]
    confidence: float
    processing_time_ms: float
    buffer_size: int
    chunk_id: int
    status: str
    metadata: Dict[str, Any]


class StreamingHMMProcessor(nn.Module):
    def __init__(self, num_states: int, feature_dim: int, chunk_size: int = 160, overlap_size: int = 80,
                 lookahead_frames: int = 5, max_delay_frames: int = 50, use_beam_search: bool = True,
                 beam_width: int = 8, buffer_size: int = 1000):
        super().__init__()
        self.num_states = num_states
        self.feature_dim = feature_dim
        self.chunk_size = chunk_size
        self.overlap_size = overlap_size
        self.lookahead_frames = lookahead_frames
        self.max_delay_frames = max_delay_frames
        self.use_beam_search = use_beam_search
        self.beam_width = beam_width
        self.buffer_size = buffer_size
        self.transition_logits = nn.Parameter(torch.randn(num_states, num_states) * 0.1)
        self.emission_net = nn.Sequential(
            nn.Linear(feature_dim, 128), nn.ReLU(), nn.Dropout(0.1), nn.Linear(128, num_states),
            nn.LogSoftmax(dim=-1))
        self.reset_streaming_state()
        self.processing_times = deque(maxlen=1000)
        # host wall time of each phase of the decoded chunks (get_latency_breakdown)
        self.phase_times = {k: deque(maxlen=1000) for k in _PHASES}
        self.chunk_counter = 0
        self.total_frames_processed = 0
        self.processing_queue = queue.Queue(maxsize=self.buffer_size)
        self.result_queue = queue.Queue(maxsize=self.buffer_size)
        self.is_processing = False
        self.processing_thread = None

    # -- stream state (streaming.py:102-117) ------------------------------------------------
    def reset_streaming_state(self):
        self.feature_buffer = deque(maxlen=self.max_delay_frames + self.lookahead_frames)
        self.viterbi_states = []
        self.viterbi_scores = []
        self.beam_hypotheses = []
        self.last_output_frame = -1
        self.chunk_counter = 0
        self.total_frames_processed = 0
        if self.use_beam_search:
            init = -torch.log(torch.tensor(self.num_states, dtype=torch.float))
            self.beam_hypotheses = [(init, [], s) for s in range(min(self.beam_width, self.num_states))]

    def get_transition_matrix(self) -> torch.Tensor:
        return F.softmax(self.transition_logits, dim=-1)

    def refresh_transitions(self):
        """Drop the cached log-transition table: the next chunk re-forms it.  Needed only after
        writing the logits through ``.data`` (``p.data.copy_(...)``, ``p.data -= ...``) in eval
        mode: such writes do not bump the parameter's version counter, so the cache cannot see
        them.  (In-place ops on the parameter itself, ``load_state_dict``, ``train()``/``eval()``
        and replacing the parameter are all seen; in training mode the table is re-formed on
        every chunk, as the reference does.)"""
        self._log_t_cache = None

    def train(self, mode: bool = True):
        self._log_t_cache = None
        return super().train(mode)

    def _load_from_state_dict(self, *args, **kwargs):
        self._log_t_cache = None
        return super()._load_from_state_dict(*args, **kwargs)

    def _log_transitions(self):
        """log(softmax + 1e-8) (streaming.py:289-290), formed on a CPU copy — the reference's
        path is torch-CPU — so the kernels see its bits.  In eval mode it is cached on the
        parameter's identity, storage and version: a chunk makes no device -> host -> device
        round trip (and no host sync) unless the transition logits changed since the last chunk
        (see refresh_transitions for ``.data`` writes).  In training mode, where an optimiser
        may write the logits in any way between chunks, it is re-formed every chunk."""
        p = self.transition_logits
        key = (p.data_ptr(), p._version, str(p.device))
        c = getattr(self, "_log_t_cache", None)
        if c is None or c[0] != key or c[1] is not p or (self.training and p.requires_grad):
            lt = torch.log(F.softmax(p.detach().cpu(), dim=-1) + 1e-8).to(p.device)
            self._log_t_cache = (key, p, lt)
            c = self._log_t_cache
        return c[2]

    # -- async helpers (streaming.py:123-181) -----------------------------------------------
    # Same public calls and drop semantics as the reference (a full input queue refuses the
    # chunk, a full result queue drops the result, a failing chunk warns and the worker keeps
    # serving). The worker blocks on the queue instead of polling it, and stop() wakes it with
    # a sentinel, so an idle stream costs no CPU and stop() returns as soon as the current
    # chunk is done.
    _STOP = object()

    def start_async_processing(self):
        if self.is_processing:
            return
        self.is_processing = True
        self.processing_thread = threading.Thread(target=self._async_processing_loop, daemon=True)
        self.processing_thread.start()

    def stop_async_processing(self):
        if not self.is_processing:
            return
        self.is_processing = False
        th, self.processing_thread = self.processing_thread, None
        if th is not None:
            while th.is_alive():
                try:  # the sentinel needs one free slot; retry while the worker drains
                    self.processing_queue.put(self._STOP, timeout=0.05)
                    break
                except queue.Full:
                    continue
            th.join()

    def _async_processing_loop(self):
        q = self.processing_queue
        while True:
            chunk = q.get()
            try:
                if chunk is self._STOP:
                    return
                if not self.is_processing:
                    continue  # chunks queued behind a stop are discarded, as the reference does
                try:
                    result = self.process_chunk(chunk)
                except Exception as e:  # noqa: BLE001 — the reference warns and keeps serving
                    warnings.warn(f"Error in async processing: {e}")
                    continue
                try:
                    self.result_queue.put_nowait(result)
                except queue.Full:
                    pass
            finally:
                q.task_done()

    def add_audio_chunk_async(self, audio_chunk: torch.Tensor) -> bool:
        try:
            self.processing_queue.put_nowait(audio_chunk)
            return True
        except queue.Full:
            return False

    def get_result_async(self) -> Optional[StreamingResult]:
        try:
            return self.result_queue.get_nowait()
        except queue.Empty:
            return None

    # -- chunk processing (streaming.py:183-265) --------------------------------------------
    def _mark(self, phase: str):
        """Charge the host time since the previous mark of this chunk to `phase`."""
        c = getattr(self, "_clock", None)
        if c is not None:
            now = time.perf_counter()
            c[phase] = c.get(phase, 0.0) + (now - c["_last"]) * 1e3
            c["_last"] = now

    def process_chunk(self, audio_chunk: torch.Tensor) -> StreamingResult:
        t0 = time.time()
        self._clock = {"_last": time.perf_counter()}
        for frame in audio_chunk:
            self.feature_buffer.append(frame)
        available = len(self.feature_buffer)
        required = self.chunk_size + self.lookahead_frames
        if available < required:
            self._clock = None
            return StreamingResult(None, 0.0, (time.time() - t0) * 1000, available, self.chunk_counter,
                                   "buffering", {"frames_needed": required - available})
        start = max(0, self.last_output_frame + 1)
        end = available - self.lookahead_frames
        if end <= start:
            self._clock = None
            return StreamingResult(None, 0.0, (time.time() - t0) * 1000, available, self.chunk_counter,
                                   "waiting_for_lookahead", {})
        features = torch.stack(list(self.feature_buffer)[start:end])
        self._mark("feature_extraction")
        states, conf = self._decode(features)
        self.last_output_frame = end - 1
        self.total_frames_processed += len(features)
        dt = (time.time() - t0) * 1000
        self.processing_times.append(dt)
        self._mark("bookkeeping")
        clock, self._clock = self._clock, None
        for k in _PHASES:
            self.phase_times[k].append(clock.get(k, 0.0))
        self.chunk_counter += 1
        rtf = (len(features) * 1000 / 100) / dt if dt > 0 else float("inf")
        return StreamingResult(states, conf.mean().item() if conf is not None else 0.0, dt, available,
                               self.chunk_counter, "decoded",
                               {"frames_processed": len(features), "real_time_factor": rtf,
                                "buffer_utilization": available / self.feature_buffer.maxlen})

    def _decode(self, features):
        return self._beam_search_decode(features) if self.use_beam_search else self._greedy_decode(features)

    def flush_buffer(self) -> Optional[StreamingResult]:
        if len(self.feature_buffer) == 0:
            return None
        states, conf = self._decode(torch.stack(list(self.feature_buffer)))
        self.chunk_counter += 1
        return StreamingResult(states, conf.mean().item() if conf is not None else 0.0, 0.0, 0, self.chunk_counter,
                               "flushed", {"final_chunk": True})

    # -- decoders (streaming.py:267-377) on the GPU -----------------------------------------
    def _greedy_decode(self, features: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """One greedy chain over the chunk; continues from the stream's last state."""
        with torch.no_grad():
            emis = self.emission_net(features)
            self._mark("emission_computation")
            prev = self.viterbi_states[-1] if self.viterbi_states else -1
            prev_t = torch.tensor([prev], dtype=torch.int32, device=emis.device)
            log_n = float(torch.log(torch.tensor(self.num_states)))
            log_t = self._log_transitions()
            self._mark("transition_computation")
            states, scores = ops.stream_greedy(emis.unsqueeze(0), log_t, prev_t, log_n)
            states, scores = states[0], scores[0]
            st_list, sc_list = states.tolist(), scores.tolist()   # (waits for the decode)
            self._mark("viterbi_decoding")
            self.viterbi_states.extend(st_list)
            self.viterbi_scores.extend(sc_list)
            if len(self.viterbi_states) > self.max_delay_frames:
                excess = len(self.viterbi_states) - self.max_delay_frames
                self.viterbi_states = self.viterbi_states[excess:]
                self.viterbi_scores = self.viterbi_scores[excess:]
        return states, torch.exp(scores)

    def _beam_search_decode(self, features: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Beam search over the chunk; the hypotheses (score, path, last state) carry over."""
        T = features.shape[0]
        with torch.no_grad():
            emis = self.emission_net(features)
            self._mark("emission_computation")
            dev = emis.device
            K = self.beam_width
            hyps = self.beam_hypotheses
            kc = len(hyps)
            kmax = ops.STREAM_SLOTS if self.num_states <= 128 else 16  # (stream.hip: the lane's candidate mask)
            if not 1 <= K <= kmax or kc > kmax:
                raise ValueError(f"beam_width must be in [1, {kmax}] on this path for {self.num_states} states, got {K}")
            hs = torch.full((1, ops.STREAM_SLOTS), float("-inf"), device=dev)
            hl = torch.zeros((1, ops.STREAM_SLOTS), dtype=torch.int32, device=dev)
            if kc:
                hs[0, :kc] = torch.stack([torch.as_tensor(h[0], dtype=torch.float32) for h in hyps]).to(dev)
                hl[0, :kc] = torch.tensor([h[2] for h in hyps], dtype=torch.int32, device=dev)
            cnt = torch.tensor([kc], dtype=torch.int32, device=dev)
            first = torch.tensor([int(kc > 0 and all(len(h[1]) == 0 for h in hyps))], dtype=torch.int32, device=dev)
            log_t = self._log_transitions()
            self._mark("transition_computation")
            states, parent, hstate = ops.stream_beam(emis.unsqueeze(0), log_t, K, hs, hl, cnt, first,
                                                     live_max=max(kc, 1))
            # rebuild the hypotheses' paths: new hypothesis r descends from old hypothesis h0
            kn = int(cnt.item())
            par, hst = parent[0].cpu().tolist(), hstate[0].cpu().tolist()
            self._mark("viterbi_decoding")
            new = []
            for r in range(kn):
                tail, rr = [], r
                for t in range(T - 1, -1, -1):
                    tail.append(hst[t][rr])
                    rr = par[t][rr]
                tail.reverse()
                new.append((hs[0, r], hyps[rr][1] + tail, hl[0, r].item()))
            self.beam_hypotheses = new
            best_score, best_path, _ = new[0]
            st = states[0] if len(best_path) >= T else torch.tensor(best_path, dtype=torch.long, device=dev)
            conf = torch.full((T,), float(torch.exp(best_score.cpu() / len(best_path))), device=dev)
        return st, conf

    # -- monitoring (streaming.py:409-503) ---------------------------------------------------
    def get_performance_stats(self) -> Dict[str, float]:
        if not self.processing_times:
            return {"message": "No processing data available"}
        times = list(self.processing_times)
        avg = sum(times) / len(times)
        frame_ms = self.chunk_size * 1000 / 100
        return {
            "total_chunks_processed": self.chunk_counter,
            "total_frames_processed": self.total_frames_processed,
            "avg_processing_time_ms": avg, "max_processing_time_ms": max(times),
            "min_processing_time_ms": min(times),
            "std_processing_time_ms": torch.tensor(times).std().item(),
            "real_time_factor": frame_ms / avg if avg > 0 else float("inf"),
            "throughput_fps": self.total_frames_processed / (sum(times) / 1000) if times else 0,
            "buffer_utilization": len(self.feature_buffer) / self.feature_buffer.maxlen,
            "chunk_size": self.chunk_size, "lookahead_frames": self.lookahead_frames,
            "beam_width": self.beam_width if self.use_beam_search else 1,
            "processing_mode": "beam_search" if self.use_beam_search else "greedy",
        }

    # -- latency control (streaming.py:444-503) --------------------------------------------
    def optimize_for_latency(self, target_latency_ms: float = 50.0):
        """One adjustment step toward `target_latency_ms` from the mean chunk time so far:
        above the target the first applicable entry of ``_LATENCY_STEPS["slower"]`` is taken
        (narrow the beam, then greedy decoding, then shorter chunks); below half the target
        the first of ``["faster"]`` (beam search back on at width 4, then a wider beam).
        Without timing data it warns and changes nothing (streaming.py:444-483)."""
        stats = self.get_performance_stats()
        if "avg_processing_time_ms" not in stats:
            warnings.warn("No performance data available for optimization")
            return
        lat = stats["avg_processing_time_ms"]
        if lat > target_latency_ms:
            table = _LATENCY_STEPS["slower"]
        elif lat < 0.5 * target_latency_ms:
            table = _LATENCY_STEPS["faster"]
        else:
            return
        for applies, apply in table:
            if applies(self):
                print(apply(self))
                return

    def get_latency_breakdown(self) -> Dict[str, float]:
        """Mean host time (ms) per phase of the decoded chunks, under the reference's keys
        (streaming.py:485-503), plus 'total' = the mean chunk time; {} before any chunk was
        decoded.  The phases are measured (``_mark``), not a fixed split: feature_extraction
        (buffering and stacking the frames), emission_computation (the emission network),
        transition_computation (the log-transition table), viterbi_decoding (the decode kernel
        and reading its result back), bookkeeping (path and state updates)."""
        stats = self.get_performance_stats()
        if "avg_processing_time_ms" not in stats:
            return {}
        out = {k: (sum(v) / len(v) if v else 0.0) for k, v in self.phase_times.items()}
        out["total"] = stats["avg_processing_time_ms"]
        return out


# phases timed per decoded chunk (get_latency_breakdown), in the reference's key order
_PHASES = ("feature_extraction", "emission_computation", "transition_computation", "viterbi_decoding",
           "bookkeeping")


def _set(p, **kw):
    for k, v in kw.items():
        setattr(p, k, v)


# optimize_for_latency's steps: (applies(processor), apply(processor) -> message), first match wins
_LATENCY_STEPS = {
    "slower": (
        (lambda p: p.use_beam_search and p.beam_width > 2,
         lambda p: (_set(p, beam_width=max(2, p.beam_width - 1)), f"Reduced beam width to {p.beam_width}")[1]),
        (lambda p: p.use_beam_search,
         lambda p: (_set(p, use_beam_search=False), "Switched to greedy decoding for lower latency")[1]),
        (lambda p: p.chunk_size > 80,
         lambda p: (_set(p, chunk_size=max(80, int(p.chunk_size * 0.8))), f"Reduced chunk size to {p.chunk_size}")[1]),
    ),
    "faster": (
        (lambda p: not p.use_beam_search,
         lambda p: (_set(p, use_beam_search=True, beam_width=4), "Enabled beam search for better accuracy")[1]),
        (lambda p: p.beam_width < 8,
         lambda p: (_set(p, beam_width=p.beam_width + 1), f"Increased beam width to {p.beam_width}")[1]),
    ),
}


class AdaptiveLatencyController:
    """Recommends streaming parameters from a window of observed chunk latencies
    (streaming.py:506-592).  ``update`` records one chunk's latency and, at most once per
    ``cooldown_s`` and only after ``min_history`` observations, classifies the mean and
    variance of the last ``window`` latencies into one regime of ``_RULES`` (first match):

      overloaded  mean > 1.2 x target: shrink the chunk by ``adaptation_rate`` (not below
                  min_chunk_size), beam width 3, beam search only while mean <= 2 x target
      headroom    mean < 0.6 x target and variance < 10: grow the chunk (not above
                  max_chunk_size) when the buffer holds > 100 frames, beam width 6, beam on
      jittery     variance > 25: greedy decoding, chunk 0.9x (recommended, not adopted)

    and returns the recommendations (an empty dict when none applies or it is too early)."""

    window = 20
    min_history = 10
    cooldown_s = 1.0

    def __init__(self, initial_chunk_size: int = 160, min_chunk_size: int = 80, max_chunk_size: int = 320,
                 target_latency_ms: float = 50.0, adaptation_rate: float = 0.1):
        self.chunk_size = initial_chunk_size
        self.min_chunk_size = min_chunk_size
        self.max_chunk_size = max_chunk_size
        self.target_latency_ms = target_latency_ms
        self.adaptation_rate = adaptation_rate
        self.latency_history = deque(maxlen=100)
        self.adjustment_cooldown = 0
        self.last_adjustment_time = 0

    def _overloaded(self, mean, var, buffer_size):
        rec = {}
        if self.chunk_size > self.min_chunk_size:
            self.chunk_size = rec["chunk_size"] = max(self.min_chunk_size,
                                                      int(self.chunk_size * (1 - self.adaptation_rate)))
        rec["beam_width"] = 3
        rec["use_beam_search"] = not mean > 2 * self.target_latency_ms
        return rec

    def _headroom(self, mean, var, buffer_size):
        rec = {}
        if self.chunk_size < self.max_chunk_size and buffer_size > 100:
            self.chunk_size = rec["chunk_size"] = min(self.max_chunk_size,
                                                      int(self.chunk_size * (1 + self.adaptation_rate)))
        rec["beam_width"] = 6
        rec["use_beam_search"] = True
        return rec

    def _jittery(self, mean, var, buffer_size):
        return {"use_beam_search": False, "chunk_size": max(self.min_chunk_size, int(self.chunk_size * 0.9))}

    _RULES = (
        (lambda c, m, v: m > 1.2 * c.target_latency_ms, _overloaded),
        (lambda c, m, v: m < 0.6 * c.target_latency_ms and v < 10.0, _headroom),
        (lambda c, m, v: v > 25.0, _jittery),
    )

    def update(self, processing_time_ms: float, buffer_size: int) -> Dict[str, Any]:
        self.latency_history.append(processing_time_ms)
        now = time.time()
        if now - self.last_adjustment_time < self.cooldown_s or len(self.latency_history) < self.min_history:
            return {}
        recent = torch.tensor(list(self.latency_history)[-self.window:])
        mean, var = float(recent.mean()), float(recent.var())
        rec = {}
        for matches, rule in self._RULES:
            if matches(self, mean, var):
                rec = rule(self, mean, var, buffer_size)
                break
        if rec:
            self.last_adjustment_time = now
        return rec
