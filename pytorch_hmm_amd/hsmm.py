"""HSMMLayer — drop-in for the reference's explicit-duration HMM layer (hsmm.py:20-470).

Parameters keep the reference's names, shapes and initialisation (``transition_logits``,
``observation_means``, ``observation_log_vars``, ``duration_shape``/``duration_rate``
(gamma), ``duration_lambda`` (poisson), ``duration_scale``/``duration_concentration``
(weibull), ``duration_means`` and ``duration_range`` buffers; hsmm.py:61-106).  The duration
and transition tables are the reference's torch expressions (tiny, S x Dmax); the
observation scores run in the gfx950 GMM scorer (one component) and the segment Viterbi
(hsmm.py:208-354) in the HSMM kernels (csrc/hsmm.hip, csrc/hsmm_wide.hip), bit-exact given the
same tables at every supported size: the segment sums follow torch.sum's CPU cascade order
(csrc/tsum.h), pinned to torch.sum for every length 1..1024 and to a reference fixture with
83- and 82-frame segments (tests/golden/hsmm_d96.npz).
"""
import math
import warnings
from typing import Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .autograd import GmmLogProb, needs_grad


class HSMMLayer(nn.Module):
    def __init__(self, num_states: int, feature_dim: int, duration_distribution: str = "gamma",
                 max_duration: int = 50, learnable_duration_params: bool = True, min_duration: int = 1):
        super().__init__()
        # the segment-Viterbi kernels (csrc/hsmm.hip): S <= 64 with Dmax <= 71, or S <= 128 with
        # Dmax <= 63, keep every open segment in registers; larger layers, up to S <= 1024 and
        # Dmax <= 1024, take the general form of csrc/hsmm_wide.hip (M history and segment sums
        # in HBM).  The reference has no limit; beyond these sizes the layer is rejected here, at
        # construction, rather than at the first forward (BASELINE config 5 is S = 64, Dmax = 40).
        # The general form costs time and memory: at S = 64, T = 2000, B = 32 the decode takes
        # 4.8 ms with 36 MiB of workspace at Dmax = 71 and 23 ms with 1.58 GiB at Dmax = 100
        # (B*T*S*(Dmax+1) fp32; ops.hsmm_viterbi decodes the batch in slices that fit the free
        # memory; INTEGRATION.md "Supported sizes", profiles/r5u_hsmm_wide_edge.log).
        if not 1 <= num_states <= 1024:
            raise ValueError(f"HSMMLayer on gfx950 supports 1 <= num_states <= 1024, got {num_states}")
        if not 1 <= max_duration <= 1024:
            raise ValueError(f"HSMMLayer on gfx950 supports 1 <= max_duration <= 1024, got {max_duration}")
        self.num_states = num_states
        self.feature_dim = feature_dim
        self.duration_distribution = duration_distribution
        self.max_duration = max_duration
        self.min_duration = min_duration
        self.learnable_duration_params = learnable_duration_params
        self.eps = 1e-8
        self._init_parameters()
        self.register_buffer("duration_range",
                             torch.arange(self.min_duration, self.max_duration + 1, dtype=torch.float))

    def _init_parameters(self):
        S, D = self.num_states, self.feature_dim
        self.transition_logits = nn.Parameter(torch.randn(S, S) * 0.1)
        self.observation_means = nn.Parameter(torch.randn(S, D) * 0.1)
        self.observation_log_vars = nn.Parameter(torch.zeros(S, D))
        if self.learnable_duration_params:
            if self.duration_distribution == "gamma":
                self.duration_shape = nn.Parameter(torch.ones(S) * 2.0)
                self.duration_rate = nn.Parameter(torch.ones(S) * 0.2)
            elif self.duration_distribution == "poisson":
                self.duration_lambda = nn.Parameter(torch.ones(S) * 10.0)
            elif self.duration_distribution == "weibull":
                self.duration_scale = nn.Parameter(torch.ones(S) * 10.0)
                self.duration_concentration = nn.Parameter(torch.ones(S) * 2.0)
            else:
                raise ValueError(f"Unknown duration distribution: {self.duration_distribution}")
        else:
            self.register_buffer("duration_means", torch.ones(S) * 10.0)

    # -- parameter tables (reference expressions, hsmm.py:108-179) ----------------------
    def get_transition_matrix(self) -> torch.Tensor:
        logits = self.transition_logits.clone()
        logits.fill_diagonal_(float("-inf"))
        return F.softmax(logits, dim=-1)

    def get_duration_probabilities(self) -> torch.Tensor:
        d = self.duration_range.unsqueeze(0)
        if self.duration_distribution == "gamma":
            shape = F.softplus(self.duration_shape).unsqueeze(1)
            rate = F.softplus(self.duration_rate).unsqueeze(1)
            lp = ((shape - 1) * torch.log(d + self.eps) - rate * d - torch.lgamma(shape)
                  + shape * torch.log(rate + self.eps))
        elif self.duration_distribution == "poisson":
            lam = F.softplus(self.duration_lambda).unsqueeze(1)
            lp = d * torch.log(lam + self.eps) - lam - torch.lgamma(d + 1)
        elif self.duration_distribution == "weibull":
            scale = F.softplus(self.duration_scale).unsqueeze(1)
            conc = F.softplus(self.duration_concentration).unsqueeze(1)
            lp = (torch.log(conc + self.eps) - conc * torch.log(scale + self.eps)
                  + (conc - 1) * torch.log(d + self.eps) - (d / scale) ** conc)
        else:
            return None
        lp = torch.where(d >= self.min_duration, lp, torch.full_like(lp, float("-inf")))
        return torch.exp(lp)

    def get_observation_log_probs(self, observations: torch.Tensor) -> torch.Tensor:
        """(B,T,D) -> (B,T,S) diagonal-Gaussian log-densities (hsmm.py:181-206)."""
        S = self.num_states
        zeros = torch.zeros(S, 1, device=observations.device)
        if needs_grad(observations, self.observation_means, self.observation_log_vars):
            return GmmLogProb.apply(observations, self.observation_means.unsqueeze(1),
                                    self.observation_log_vars.unsqueeze(1), zeros, 0)
        with torch.no_grad():
            return ops.gmm_diag_logprob(observations, self.observation_means.unsqueeze(1),
                                        self.observation_log_vars.unsqueeze(1), zeros, 0)

    # -- decoding (hsmm.py:208-354) -------------------------------------------------------
    def viterbi_decode_hsmm(self, observations: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(states (B,T) int64, best segmentation score (B,))."""
        B, T, _ = observations.shape
        if T > 1000:
            warnings.warn(f"Long sequence ({T} frames) may cause memory issues in HSMM decoding.")
        with torch.no_grad():  # the segment Viterbi is not differentiated (as in the reference)
            obs_log_probs = self.get_observation_log_probs(observations)
            dur_lp = torch.log(self.get_duration_probabilities() + self.eps)
            log_T = torch.log(self.get_transition_matrix() + self.eps)
        if dur_lp.shape[1] < self.max_duration:
            # the reference indexes duration_log_probs[s, d-1] for d up to max_duration
            raise IndexError(f"index {dur_lp.shape[1]} is out of bounds for dimension 1 with size {dur_lp.shape[1]}")
        return ops.hsmm_viterbi(obs_log_probs, dur_lp[:, :self.max_duration], log_T)

    def forward(self, observations: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.viterbi_decode_hsmm(observations)

    def get_expected_durations(self) -> torch.Tensor:
        if self.duration_distribution == "gamma":
            return F.softplus(self.duration_shape) / F.softplus(self.duration_rate)
        if self.duration_distribution == "poisson":
            return F.softplus(self.duration_lambda)
        if self.duration_distribution == "weibull":
            scale = F.softplus(self.duration_scale)
            conc = F.softplus(self.duration_concentration)
            return scale * torch.exp(torch.lgamma(1 + 1 / conc))
        return self.duration_means

    def get_model_info(self) -> dict:
        total = sum(p.numel() for p in self.parameters())
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        return {"num_states": self.num_states, "feature_dim": self.feature_dim,
                "duration_distribution": self.duration_distribution, "max_duration": self.max_duration,
                "min_duration": self.min_duration, "expected_durations": self.get_expected_durations().tolist(),
                "total_parameters": total, "trainable_parameters": trainable}
