"""Explicit-duration HMM — drop-ins for the reference's semi_markov.py (§8(f) row 3).

``DurationModel`` (semi_markov.py:9-192), ``SemiMarkovHMM`` (:195-633) and
``AdaptiveDurationHSMM`` (:636-680) keep the reference's parameter names, shapes and
initialisation order (``state_dict`` compatible, same draws under the same seed).

The hot path is the segment recursion: ``viterbi_decode`` (semi_markov.py:455-570) and the
unsupervised segment forward (:308-383).  The reference walks (t, s, d, s', d') in Python
and rescoring every candidate segment from the raw frames; here one gfx950 kernel scores
all frames against all states (``ops.semimarkov_quad``) and one workgroup per sequence runs
the recursion (``ops.semimarkov_viterbi`` / ``ops.semimarkov_forward``, csrc/semimarkov.hip).
The small parameter tables — log initial / transition probabilities, the per-state segment
constant and variances, and the duration log-probabilities — are formed on the host with the
reference's own torch expressions, so the kernels see the reference's table bits.
"""
import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Gamma, Normal, Poisson

from . import ops

class DurationModel(nn.Module):
    """Per-state duration distribution over d = 1..max_duration (semi_markov.py:9-192)."""

    def __init__(self, num_states: int, max_duration: int = 50, distribution_type: str = "gamma",
                 min_duration: int = 1, hidden_dim: int = 128):
        super().__init__()
        self.num_states = num_states
        self.max_duration = max_duration
        self.distribution_type = distribution_type
        self.min_duration = min_duration
        self.hidden_dim = hidden_dim
        if distribution_type == "gamma":
            self.alpha_params = nn.Parameter(torch.ones(num_states))
            self.beta_params = nn.Parameter(torch.ones(num_states))
        elif distribution_type == "poisson":
            self.lambda_params = nn.Parameter(torch.ones(num_states) * 5)
        elif distribution_type == "gaussian":
            self.mean_params = nn.Parameter(torch.ones(num_states) * 10)
            self.std_params = nn.Parameter(torch.ones(num_states))
        elif distribution_type == "neural":
            self.duration_net = nn.Sequential(
                nn.Embedding(num_states, hidden_dim), nn.Linear(hidden_dim, hidden_dim), nn.ReLU(),
                nn.Linear(hidden_dim, max_duration), nn.LogSoftmax(dim=-1))
        else:
            raise ValueError(f"Unknown distribution_type: {distribution_type}")
        self._d_cache = {}

    # -- the reference's per-state parametric density (semi_markov.py:122-153) --------------
    def _state_scalars(self, s: int, P=None):
        P = P if P is not None else dict(self.named_parameters())
        k = self.distribution_type
        if k == "gamma":
            return F.softplus(P["alpha_params"][s]) + 1e-6, F.softplus(P["beta_params"][s]) + 1e-6
        if k == "poisson":
            return (F.softplus(P["lambda_params"][s]) + 1e-6,)
        return F.softplus(P["mean_params"][s]) + self.min_duration, F.softplus(P["std_params"][s]) + 1e-6

    def _parametric(self, s: int, durations: torch.Tensor, log_d=None, lgamma_d1=None, P=None) -> torch.Tensor:
        """Density of state s at `durations` (float).  log_d / lgamma_d1 may carry
        log(durations + 1e-8) / lgamma(durations + 1) formed elsewhere (see _elementwise);
        P optionally maps parameter names to the tensors to use (CPU copies)."""
        k = self.distribution_type
        if k == "gamma":
            a, b = self._state_scalars(s, P)
            ld = torch.log(durations + 1e-8) if log_d is None else log_d
            lp = (a - 1) * ld - b * durations
            lp = lp - (torch.lgamma(a) - a * torch.log(b))
        elif k == "poisson":
            (lam,) = self._state_scalars(s, P)
            lg = torch.lgamma(durations + 1) if lgamma_d1 is None else lgamma_d1
            lp = durations * torch.log(lam + 1e-8) - lam
            lp = lp - lg
        else:
            mean, std = self._state_scalars(s, P)
            lp = -0.5 * torch.log(2 * math.pi * std ** 2)
            lp = lp - 0.5 * ((durations - mean) / std) ** 2
        return torch.where(durations >= self.min_duration, lp, torch.full_like(lp, float("-inf")))

    def _elementwise(self, n: int):
        """log(d + 1e-8) and lgamma(d + 1) for d = 1..n, each formed on a ONE-element tensor.

        The reference evaluates a candidate's duration on a one-element tensor
        (semi_markov.py:109-118), where ATen takes the scalar libm path; over a whole arange the
        vectorised path may differ in the last bit.  Only these two transcendentals see the
        duration vector (the rest is IEEE + - * /), so caching them per d reproduces the
        reference's per-candidate bits with vector arithmetic."""
        if n not in self._d_cache:
            ld, lg = [], []
            for d in range(1, n + 1):
                t = torch.tensor([float(d)])
                ld.append(torch.log(t + 1e-8))
                lg.append(torch.lgamma(t + 1))
            self._d_cache[n] = (torch.cat(ld), torch.cat(lg))
        return self._d_cache[n]

    def candidate_table(self) -> torch.Tensor:
        """(S, max_duration) log-probabilities exactly as the reference's decoders read them:
        duration_model(tensor([s]), tensor([d]))[0] for every (s, d) (semi_markov.py:502-505).

        Formed on CPU copies of the parameters — the reference's decoding path is torch-CPU
         — then moved to the parameters' device."""
        S, Dm = self.num_states, self.max_duration
        dev = self._device()
        with torch.no_grad():
            P = {n: p.detach().cpu() for n, p in self.named_parameters()}
            if self.distribution_type == "neural":
                # one batch-1 evaluation per state, as the reference's calls make it
                net = {k[len("duration_net."):]: v for k, v in P.items()}
                rows = [torch.func.functional_call(self.duration_net, net, (torch.tensor([s]),))[0]
                        for s in range(S)]
                return torch.stack(rows).to(dev)
            log_d, lg_d1 = self._elementwise(Dm)
            d = torch.arange(1, Dm + 1).float()
            return torch.stack([self._parametric(s, d, log_d, lg_d1, P) for s in range(S)]).to(dev)

    def _device(self):
        return next(self.parameters()).device

    # -- reference API ---------------------------------------------------------------------
    def forward(self, state_indices: torch.Tensor, durations: Optional[torch.Tensor] = None) -> torch.Tensor:
        if durations is None:
            return self._distribution(state_indices)
        return self._probability(state_indices, durations)

    def _distribution(self, state_indices):
        """(n,) states -> (n, max_duration) (semi_markov.py:81-98)."""
        if self.distribution_type == "neural":
            return self.duration_net(state_indices)
        d = torch.arange(1, self.max_duration + 1, device=state_indices.device).float()
        out = torch.zeros(state_indices.shape[0], self.max_duration, device=state_indices.device)
        for i, s in enumerate(state_indices.tolist()):
            out[i] = self._parametric(int(s), d)
        return out

    def _probability(self, state_indices, durations):
        """Log-probability of durations[i] in state_indices[i] (semi_markov.py:100-120)."""
        dev = state_indices.device
        if self.distribution_type == "neural":
            full = self.duration_net(state_indices)
            di = torch.clamp(durations - 1, 0, self.max_duration - 1)
            return full[torch.arange(state_indices.shape[0], device=dev), di]
        out = torch.zeros_like(durations, dtype=torch.float, device=dev)
        for i, (s, d) in enumerate(zip(state_indices.tolist(), durations)):
            out[i] = self._parametric(int(s), d.float().unsqueeze(0)).squeeze()
        return out

    def sample(self, state_indices: torch.Tensor, num_samples: int = 1) -> torch.Tensor:
        """Duration draws per state (semi_markov.py:155-192; same draw order)."""
        dev = state_indices.device
        if self.distribution_type == "neural":
            probs = torch.exp(self.duration_net(state_indices))
            out = torch.multinomial(probs, num_samples, replacement=True) + 1
            return out.squeeze(-1) if num_samples == 1 else out
        out = torch.zeros(len(state_indices), num_samples, device=dev)
        for i, s in enumerate(state_indices):
            k = self.distribution_type
            if k == "gamma":
                a = F.softplus(self.alpha_params[s]) + 1e-6
                b = F.softplus(self.beta_params[s]) + 1e-6
                out[i] = Gamma(a, b).sample((num_samples,))
            elif k == "poisson":
                out[i] = Poisson(F.softplus(self.lambda_params[s]) + 1e-6).sample((num_samples,))
            else:
                mean = F.softplus(self.mean_params[s]) + self.min_duration
                std = F.softplus(self.std_params[s]) + 1e-6
                out[i] = torch.clamp(Normal(mean, std).sample((num_samples,)),
                                     min=self.min_duration, max=self.max_duration)
        out = torch.clamp(out, min=self.min_duration)
        return out.squeeze(-1) if num_samples == 1 else out


class SemiMarkovHMM(nn.Module):
    """Hidden semi-Markov model with explicit durations (semi_markov.py:195-633)."""

    def __init__(self, num_states: int, observation_dim: int, max_duration: int = 50,
                 duration_distribution: str = "gamma", observation_model: str = "gaussian",
                 min_duration: int = 1):
        super().__init__()
        self.num_states = num_states
        self.observation_dim = observation_dim
        self.max_duration = max_duration
        self.min_duration = min_duration
        self.duration_model = DurationModel(num_states=num_states, max_duration=max_duration,
                                            distribution_type=duration_distribution, min_duration=min_duration)
        self.transition_logits = nn.Parameter(torch.randn(num_states, num_states))
        self.initial_logits = nn.Parameter(torch.zeros(num_states))
        if observation_model == "gaussian":
            self.observation_means = nn.Parameter(torch.randn(num_states, observation_dim))
            self.observation_logvars = nn.Parameter(torch.zeros(num_states, observation_dim))
        elif observation_model == "neural":
            from .neural import NeuralObservationModel
            self.neural_obs_model = NeuralObservationModel(num_states=num_states, observation_dim=observation_dim,
                                                           model_type="gaussian")
        self.observation_model_type = observation_model

    # -- parameter tables (the reference's torch expressions, on CPU copies) -----------------
    def _cpu(self, name):
        return getattr(self, name).detach().cpu()

    def _log_initial(self):
        return torch.log(F.softmax(self._cpu("initial_logits"), dim=0) + 1e-8)          # :491-492

    def _log_transitions(self):
        return torch.log(F.softmax(self._cpu("transition_logits"), dim=1) + 1e-8)       # :510-511

    def _gaussian_tables(self):
        """(seg_const (S,), var (S,D)) — per state, as _compute_segment_observation_logprob
        forms them on the (D,) parameter rows (semi_markov.py:416-421)."""
        S, D = self.num_states, self.observation_dim
        lvs = self._cpu("observation_logvars")
        cs, var = [], []
        for s in range(S):
            lv = lvs[s]
            var.append(torch.exp(lv))
            cs.append(-0.5 * torch.sum(lv) - 0.5 * D * math.log(2 * math.pi))
        return torch.stack(cs), torch.stack(var)

    def _param_tables(self, dev):
        """Device copies of the parameter tables, rebuilt only when a parameter changes
        (storage or in-place version), so repeated decodes pay one host pass per update."""
        params = tuple(self.parameters())
        key = (str(dev),) + tuple((p.data_ptr(), p._version) for p in params)
        cached = getattr(self, "_tab_cache", None)
        # identity as well as (address, version): a freed parameter's storage can be reused
        # by a new tensor at version 0, which must not hit the old tables
        if (cached is None or cached[0] != key or len(cached[2]) != len(params)
                or any(a is not b for a, b in zip(cached[2], params))):
            with torch.no_grad():
                if self.observation_model_type == "gaussian":
                    cs, var = self._gaussian_tables()
                    cs, var_t = cs.to(dev), var.t().contiguous().to(dev)
                else:
                    cs = var_t = None
                tabs = (cs, var_t, self._log_initial().to(dev), self._log_transitions().to(dev),
                        self.duration_model.candidate_table().to(dev))
            self._tab_cache = cached = (key, tabs, params)
        return cached[1]

    def _tables(self, observations):
        cs, var_t, li, lT, du = self._param_tables(observations.device)
        if self.observation_model_type == "gaussian":
            quad = ops.semimarkov_quad(observations, self.observation_means.detach().t().contiguous(), var_t)
        elif self.observation_model_type == "neural":
            # per-frame log-densities of every state; a segment's score is their sum (:426-433)
            quad = self.neural_obs_model(observations).float().contiguous()
        else:
            raise ValueError(f"Unknown observation_model: {self.observation_model_type}")
        return quad, cs, li, lT, du

    # -- decoding (semi_markov.py:455-570) ---------------------------------------------------
    def viterbi_decode(self, observations: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(T, D) -> (segment states, segment durations, best path log-probability (0-d))."""
        if observations.dim() != 2:
            raise ValueError(f"viterbi_decode expects (seq_len, obs_dim), got {tuple(observations.shape)}")
        (res,) = self.viterbi_decode_batch(observations.unsqueeze(0))
        return res

    def viterbi_decode_batch(self, observations: torch.Tensor) -> List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        """(B, T, D) -> one (states, durations, score) per sequence (one kernel launch)."""
        with torch.no_grad():
            seg_s, seg_d, cnt, scores = ops.semimarkov_viterbi(*self._tables(observations))
        T = observations.shape[1]
        out = []
        for b, n in enumerate(cnt.tolist()):
            out.append((seg_s[b, T - n:], seg_d[b, T - n:], scores[b]))
        return out

    # -- likelihoods (semi_markov.py:258-383) ------------------------------------------------
    def forward(self, observations: torch.Tensor, state_sequence: Optional[torch.Tensor] = None,
                duration_sequence: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        if state_sequence is not None and duration_sequence is not None:
            return self._supervised_forward(observations, state_sequence, duration_sequence)
        return self._unsupervised_forward(observations)

    def _unsupervised_forward(self, observations: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Segment forward: log P(o) marginalised over all segmentations.

        The reference (semi_markov.py:308-383) means logaddexp over the same candidate set
        as its Viterbi, but calls torch.logaddexp with a Python float and raises TypeError;
        this computes that recursion for every sequence of the batch (the reference would
        read only observations[0]).  Returns log_probability (B,) and forward_variables
        (B, T, S, max_duration) (log alpha[t][s][d-1], -inf where impossible)."""
        with torch.no_grad():
            lp, alpha = ops.semimarkov_forward(*self._tables(observations), True)
        return {"log_probability": lp, "forward_variables": alpha}

    def _supervised_forward(self, observations, state_sequence, duration_sequence):
        """Log-probability of a given segmentation (semi_markov.py:280-306)."""
        B, T, _ = observations.shape
        log_obs = self._segmentation_obs(observations, state_sequence, duration_sequence)
        log_dur = self.duration_model(state_sequence.flatten(), duration_sequence.flatten())
        log_dur = log_dur.view(B, -1).sum(dim=1)
        log_tr = self._compute_transition_logprobs(state_sequence)
        return {"log_probability": log_obs + log_dur + log_tr, "log_observation": log_obs,
                "log_duration": log_dur, "log_transition": log_tr}

    def _segmentation_obs(self, observations, state_sequence, duration_sequence):
        """Sum of the scores of the segments that fit in the sequence (:385-409).  Each frame
        is scored against its segment's state (differentiable torch glue: this is the
        supervised loss, not the decoding hot path)."""
        B, T, _ = observations.shape
        dur = duration_sequence.long()
        st = state_sequence.long()
        K = st.shape[1]
        ends = torch.cumsum(dur, dim=1)
        fits = ends <= T  # durations are positive, so the fitting segments are a prefix
        t = torch.arange(T, device=observations.device).expand(B, T).contiguous()
        seg_of_t = torch.searchsorted(ends, t, right=True)          # segment holding frame t
        covered = seg_of_t < K
        k = seg_of_t.clamp(max=K - 1)
        covered = covered & fits.gather(1, k)
        fs = st.gather(1, k)                                        # frame -> state
        if self.observation_model_type == "gaussian":
            mu = self.observation_means[fs]
            var = torch.exp(self.observation_logvars)[fs]
            per_frame = torch.sum((observations - mu) ** 2 / var, dim=-1)
            cs = -0.5 * torch.sum(self.observation_logvars, dim=1) - 0.5 * self.observation_dim * math.log(2 * math.pi)
        else:
            per_frame = self.neural_obs_model(observations).gather(2, fs.unsqueeze(-1)).squeeze(-1)
            cs = None
        Q = torch.zeros(B, K, dtype=per_frame.dtype, device=per_frame.device)
        Q = Q.scatter_add(1, k, torch.where(covered, per_frame, torch.zeros_like(per_frame)))
        seg = cs[st] - 0.5 * Q if cs is not None else Q
        return torch.where(fits, seg, torch.zeros_like(seg)).sum(dim=1)

    def _compute_transition_logprobs(self, state_sequence: torch.Tensor) -> torch.Tensor:
        """Sum of log transition probabilities along each segment sequence (:437-453)."""
        lt = torch.log(F.softmax(self.transition_logits, dim=1) + 1e-8)
        if state_sequence.shape[1] < 2:
            return torch.zeros(state_sequence.shape[0], device=lt.device)
        return lt[state_sequence[:, :-1], state_sequence[:, 1:]].sum(dim=1)

    def sample(self, num_states: int, max_length: int = 100) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Draw a segment sequence and its frames (semi_markov.py:572-633; same draw order)."""
        dev = next(self.parameters()).device
        state = torch.multinomial(F.softmax(self.initial_logits, dim=0), 1).item()
        trans = F.softmax(self.transition_logits, dim=1)
        states, durs, frames, total = [], [], [], 0
        for _ in range(num_states):
            if total >= max_length:
                break
            dur = self.duration_model.sample(torch.tensor([state], device=dev)).item()
            dur = min(dur, max_length - total)
            states.append(state)
            durs.append(dur)
            if self.observation_model_type == "gaussian":
                mean = self.observation_means[state]
                std = torch.exp(0.5 * self.observation_logvars[state])
                frames.append(torch.normal(mean.unsqueeze(0).expand(int(dur), -1),
                                           std.unsqueeze(0).expand(int(dur), -1)))
            total += dur
            if total < max_length:
                state = torch.multinomial(trans[state], 1).item()
        obs = torch.cat(frames, dim=0) if frames else torch.zeros(0, self.observation_dim, device=dev)
        return torch.tensor(states, device=dev), torch.tensor(durs, device=dev), obs


class AdaptiveDurationHSMM(SemiMarkovHMM):
    """SemiMarkovHMM with a context-conditioned duration network (semi_markov.py:636-680)."""

    def __init__(self, num_states: int, observation_dim: int, context_dim: int, **kwargs):
        super().__init__(num_states, observation_dim, **kwargs)
        self.context_dim = context_dim
        self.context_duration_net = nn.Sequential(
            nn.Linear(context_dim + num_states, 128), nn.ReLU(), nn.Linear(128, 128), nn.ReLU(),
            nn.Linear(128, self.max_duration), nn.LogSoftmax(dim=-1))
        self.state_embedding = nn.Embedding(num_states, num_states)

    def compute_contextual_duration_probs(self, state_indices: torch.Tensor, context: torch.Tensor) -> torch.Tensor:
        return self.context_duration_net(torch.cat([context, self.state_embedding(state_indices)], dim=-1))
