"""MixtureGaussianHMMLayer — drop-in for the reference's GMM-HMM layer
(mixture_gaussian.py:20-384).

Parameters keep the reference's names, shapes and initialisation (``transition_logits`` or
the ``transition_matrix`` buffer, ``mixture_weights_logits``, ``means``, ``log_vars``;
mixture_gaussian.py:59-105) so state_dicts load unchanged.  The emission
(get_observation_log_probs, :157-214 with the mixture log-sum-exp :141-155) runs in the
gfx950 GMM scorer without the reference's (B,T,S,C,D) temporary; Viterbi (:290-338) runs
in the recursion kernels with the reference's uniform start lp_0 - log(S) and returns
max delta_{T-1} as the sequence score.  Covariance 'diag', 'tied' and 'spherical' map
onto per-dimension log-variances; 'full' (Cholesky, :216-240) whitens with W = L^-1 through
chunked hipBLASLt GEMMs (_full_log_probs) and shares the Viterbi kernel.
"""
import math
import warnings
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .autograd import GmmLogProb, ViterbiScore, needs_grad


class MixtureGaussianHMMLayer(nn.Module):
    def __init__(self, num_states: int, feature_dim: int, num_components: int = 3,
                 covariance_type: str = "diag", learnable_transitions: bool = True,
                 max_sequence_length: int = 10000):
        super().__init__()
        self.num_states = num_states
        self.feature_dim = feature_dim
        self.num_components = num_components
        self.covariance_type = covariance_type
        self.learnable_transitions = learnable_transitions
        self.max_sequence_length = max_sequence_length
        self.eps = 1e-8
        self.log_eps = math.log(self.eps)
        self._init_parameters()

    def _init_parameters(self):
        """Same draws, in the same order, as mixture_gaussian.py:59-105."""
        S, C, D = self.num_states, self.num_components, self.feature_dim
        if self.learnable_transitions:
            self.transition_logits = nn.Parameter(torch.randn(S, S) * 0.1)
        else:
            self.register_buffer("transition_matrix", self._create_left_to_right_matrix())
        self.mixture_weights_logits = nn.Parameter(torch.randn(S, C) * 0.1)
        gain = math.sqrt(2.0 / D)
        self.means = nn.Parameter(torch.randn(S, C, D) * gain)
        if self.covariance_type == "diag":
            self.log_vars = nn.Parameter(torch.zeros(S, C, D))
        elif self.covariance_type == "full":
            tril = D * (D + 1) // 2
            self.cholesky_params = nn.Parameter(torch.zeros(S, C, tril))
            with torch.no_grad():
                diag = [i * (i + 1) // 2 + i for i in range(D)]
                self.cholesky_params.data[:, :, diag] = 0.1
        elif self.covariance_type == "tied":
            self.log_vars = nn.Parameter(torch.zeros(D))
        elif self.covariance_type == "spherical":
            self.log_vars = nn.Parameter(torch.zeros(S, C))
        else:
            raise ValueError(f"Unknown covariance_type: {self.covariance_type}")

    def _create_left_to_right_matrix(self) -> torch.Tensor:
        """0.8 self-loop / 0.2 forward, final state absorbing (mixture_gaussian.py:119-128)."""
        S = self.num_states
        P = torch.zeros(S, S)
        idx = torch.arange(S - 1)
        P[idx, idx] = 0.8
        P[idx, idx + 1] = 0.2
        P[S - 1, S - 1] = 1.0
        return P

    def get_transition_matrix(self) -> torch.Tensor:
        if self.learnable_transitions:
            return F.softmax(self.transition_logits, dim=-1)
        return self.transition_matrix

    def _safe_log(self, x: torch.Tensor) -> torch.Tensor:
        return torch.log(torch.clamp(x, min=self.eps))

    def _component_log_vars(self) -> torch.Tensor:
        """(S,C,D) per-dimension log-variances for the scorer."""
        S, C, D = self.num_states, self.num_components, self.feature_dim
        if self.covariance_type == "diag":
            return self.log_vars
        if self.covariance_type == "tied":
            return self.log_vars.view(1, 1, D).expand(S, C, D)
        if self.covariance_type == "spherical":
            return self.log_vars.unsqueeze(-1).expand(S, C, D)
        raise ValueError("covariance_type='full' has no per-dimension variances (see _full_log_probs)")

    def _get_cholesky_factors(self) -> torch.Tensor:
        """(S,C,D,D) lower-triangular factors, exp on the diagonal (mixture_gaussian.py:271-289)."""
        S, C, D = self.num_states, self.num_components, self.feature_dim
        L = torch.zeros(S * C, D, D, device=self.cholesky_params.device, dtype=self.cholesky_params.dtype)
        ti = torch.tril_indices(D, D, device=L.device)
        L[:, ti[0], ti[1]] = self.cholesky_params.view(-1, self.cholesky_params.size(-1))
        di = torch.arange(D, device=L.device)
        L[:, di, di] = torch.exp(L[:, di, di])
        return L.view(S, C, D, D)

    # frames per whitening GEMM: keeps the (frames, S*C*D) product near 256 MiB
    _FULL_CHUNK_BYTES = 256 << 20

    def _full_log_probs(self, observations: torch.Tensor, log_w: torch.Tensor) -> torch.Tensor:
        """covariance_type='full' (mixture_gaussian.py:216-240, LSE :141-155).  The reference
        solves L z = x - mu per (frame, state, component) (a (B,T,S,C,D) temporary: 10.5 GB at
        config 3).  Here W = L^-1 and b = W mu are formed once per call (S*C triangular solves
        of D x D), and ||W x - b||^2 for every frame is one GEMM over a chunk of frames
        (hipBLASLt): (frames, D) x (D, S*C*D), squared and summed per (state, component).
        Same math as the reference's triangular solve; fp32 rounding differs (tests: 1e-4)."""
        B, T, D = observations.shape
        S, C = self.num_states, self.num_components
        L = self._get_cholesky_factors()
        eye = torch.eye(D, device=L.device, dtype=L.dtype).expand(S, C, D, D)
        W = torch.linalg.solve_triangular(L, eye, upper=False)                  # (S,C,D,D)
        bias = (W @ self.means.unsqueeze(-1)).squeeze(-1)                       # (S,C,D)
        log_det = 2 * torch.sum(torch.log(torch.diagonal(L, dim1=-2, dim2=-1) + self.eps), dim=-1)  # (S,C)
        Wt = W.reshape(S * C * D, D).t()                                        # (D, S*C*D)
        bflat = bias.reshape(S * C * D)
        const = log_det + D * math.log(2 * math.pi)                             # (S,C)
        x = observations.reshape(B * T, D)
        rows = max(1, self._FULL_CHUNK_BYTES // (4 * S * C * D))
        out = []
        for r0 in range(0, B * T, rows):
            z = torch.addmm(-bflat, x[r0:r0 + rows], Wt)                        # W x - W mu
            mahal = z.square().view(-1, S, C, D).sum(-1)                         # (n,S,C)
            lpc = -0.5 * (mahal + const) + log_w                                 # (n,S,C)
            m = lpc.max(dim=-1, keepdim=True)[0]
            m = torch.where(torch.isinf(m), torch.zeros_like(m), m)
            out.append(self._safe_log(torch.exp(lpc - m).sum(-1)) + m.squeeze(-1))
        return torch.cat(out, 0).view(B, T, S)

    def get_observation_log_probs(self, observations: torch.Tensor) -> torch.Tensor:
        """(B,T,D) -> (B,T,S): log sum_c w_sc N(x; mu_sc, diag exp(log_vars_sc))
        (mixture_gaussian.py:157-214)."""
        B, T, _ = observations.shape
        if T > self.max_sequence_length:
            warnings.warn(f"Sequence length {T} exceeds recommended maximum "
                          f"{self.max_sequence_length}. Consider chunked processing.")
        if self.covariance_type == "full":
            # torch ops on the device (differentiable by autograd), then the Viterbi kernel
            return self._full_log_probs(observations, self._safe_log(F.softmax(self.mixture_weights_logits, dim=-1)))
        if needs_grad(observations, *self.parameters()):
            log_w = self._safe_log(F.softmax(self.mixture_weights_logits, dim=-1))
            return GmmLogProb.apply(observations, self.means, self._component_log_vars(), log_w, 1)
        with torch.no_grad():
            log_w = self._safe_log(F.softmax(self.mixture_weights_logits, dim=-1))
            return ops.gmm_diag_logprob(observations, self.means, self._component_log_vars(), log_w, 1)

    def _transition_plan(self, log_transitions: torch.Tensor):
        """The banded-structure plan of log T (ops.make_plan), cached while the transition
        parameter is unchanged (same tensor, same version, same device): a fixed or learned
        matrix is measured once, not on every forward."""
        src = self.transition_logits if self.learnable_transitions else self.transition_matrix
        c = self.__dict__.get("_plan_cache")
        if (c is not None and c[0] is src and c[1] == (src._version, src.data_ptr()) and c[2] == log_transitions.device
                and c[3] == tuple(log_transitions.shape)):
            return c[4]
        # (a trainable matrix under autograd changes every step: skip the plan's host read, so
        # a training forward makes no synchronous device -> host copy; ops.make_plan)
        plan = ops.make_plan(log_transitions.detach(),
                             read_banded=not (torch.is_grad_enabled() and src.requires_grad))
        self.__dict__["_plan_cache"] = (src, (src._version, src.data_ptr()), log_transitions.device,
                                        tuple(log_transitions.shape), plan)
        return plan

    def _viterbi_decode(self, obs_log_probs: torch.Tensor,
                        log_transitions: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(states (B,T), max_j delta_{T-1}[j] (B,)) with delta_0 = lp_0 - log S
        (mixture_gaussian.py:290-338)."""
        S = obs_log_probs.shape[-1]
        init = -(torch.zeros(S, device=obs_log_probs.device) + math.log(S))
        plan = self._transition_plan(log_transitions)
        if needs_grad(obs_log_probs, log_transitions):
            # the score's gradient follows the decoded path (the reference's max-plus autograd)
            return ViterbiScore.apply(obs_log_probs, log_transitions, init, plan)
        states, _, final = ops.viterbi(obs_log_probs, log_transitions, init, ops.OBS_LOG, plan)
        return states, final

    def _inference_tables(self, device):
        """(log T, log w, the uniform start vector, the transition plan) for inference, formed with
        the reference's expressions (mixture_gaussian.py:130-135, :141-155, :305) and cached while
        the parameters they come from are unchanged (same tensors, same versions): a decode of a
        fixed model launches no per-call softmax / log / clamp kernels (~10 small launches,
        ~80 us of serial latency before the scorer at config 3, profiles/r5m_c3).  Writes through
        ``.data`` (``p.data.copy_(...)``, ``p.data -= ...``) bump no version counter: call
        refresh_tables() after them (load_state_dict, train()/eval(), in-place ops on the
        parameters and replacing them are all seen)."""
        src = self.transition_logits if self.learnable_transitions else self.transition_matrix
        wl = self.mixture_weights_logits
        key = (id(src), src._version, src.data_ptr(), id(wl), wl._version, wl.data_ptr(), str(device))
        c = self.__dict__.get("_inf_cache")
        if c is not None and c[0] == key and c[1] is src and c[2] is wl:
            return c[3]
        log_T = self._safe_log(self.get_transition_matrix())
        log_w = self._safe_log(F.softmax(wl, dim=-1))
        S = self.num_states
        init = -(torch.zeros(S, device=device) + math.log(S))
        tabs = (log_T, log_w, init, self._transition_plan(log_T))
        self.__dict__["_inf_cache"] = (key, src, wl, tabs)
        return tabs

    def refresh_tables(self):
        """Drop the cached inference tables and transition plans (after writes through ``.data``,
        which the cache cannot see); the next forward re-forms them."""
        self.__dict__.pop("_inf_cache", None)
        self.__dict__.pop("_plan_cache", None)

    def train(self, mode: bool = True):
        self.refresh_tables()
        return super().train(mode)

    def _load_from_state_dict(self, *args, **kwargs):
        self.refresh_tables()
        return super()._load_from_state_dict(*args, **kwargs)

    def forward(self, observations: torch.Tensor,
                return_log_probs: bool = False) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        if self.covariance_type != "full" and not needs_grad(observations, *self.parameters()):
            # inference: the cached tables (_inference_tables), the GMM scorer, then the decode;
            # the same bits as get_observation_log_probs followed by _viterbi_decode
            B, T, _ = observations.shape
            if T > self.max_sequence_length:
                warnings.warn(f"Sequence length {T} exceeds recommended maximum "
                              f"{self.max_sequence_length}. Consider chunked processing.")
            with torch.no_grad():
                log_T, log_w, init, plan = self._inference_tables(observations.device)
                lp = ops.gmm_diag_logprob(observations, self.means, self._component_log_vars(), log_w, 1)
                states, _, scores = ops.viterbi(lp, log_T, init, ops.OBS_LOG, plan)
            return (states, scores) if return_log_probs else (states, None)
        log_transitions = self._safe_log(self.get_transition_matrix())
        obs_log_probs = self.get_observation_log_probs(observations)
        states, scores = self._viterbi_decode(obs_log_probs, log_transitions)
        return (states, scores) if return_log_probs else (states, None)

    def get_model_info(self) -> dict:
        total = sum(p.numel() for p in self.parameters())
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        return {"num_states": self.num_states, "feature_dim": self.feature_dim,
                "num_components": self.num_components, "covariance_type": self.covariance_type,
                "learnable_transitions": self.learnable_transitions, "total_parameters": total,
                "trainable_parameters": trainable, "memory_efficient": True,
                "max_sequence_length": self.max_sequence_length}
