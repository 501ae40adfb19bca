"""HMMLayer / GaussianHMMLayer — nn.Module drop-ins for the reference's layers
(hmm_layer.py:11-217 and :220-363).

Same constructor arguments, parameter names and shapes (state_dict compatible:
``log_transition_logits`` / ``transition_matrix``, ``log_initial_logits``, ``means``,
``log_scales``), same train/eval dispatch, same first-call quirk of ``_get_hmm`` (call 1
builds an HMMPyTorch, which renormalises P; later calls assign log(P + 1e-8) directly,
hmm_layer.py:75-89).  The recursions run in the HIP kernels (ops.py); the Gaussian
emission of GaussianHMMLayer runs in the gfx950 GMM scorer (single component).
"""
from typing import Optional, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .autograd import GmmLogProb, needs_grad
from .hmm import HMMPyTorch
from .utils import create_left_to_right_matrix, create_transition_matrix


class HMMLayer(nn.Module):
    """HMM as a layer over per-frame state scores x (B,T,K) (reference hmm_layer.py:11-217)."""

    def __init__(self, num_states: int, learnable_transitions: bool = True,
                 transition_type: str = "left_to_right", self_loop_prob: float = 0.7,
                 viterbi_inference: bool = True, apply_sigmoid: bool = True):
        super().__init__()
        self.num_states = num_states
        self.viterbi_inference = viterbi_inference
        self.apply_sigmoid = apply_sigmoid
        if transition_type == "left_to_right":
            P_init = create_left_to_right_matrix(num_states, self_loop_prob)
        else:
            P_init = create_transition_matrix(num_states, transition_type, self_loop_prob)
        if learnable_transitions:
            self.log_transition_logits = nn.Parameter(torch.log(P_init + 1e-8))   # :48
        else:
            self.register_buffer("transition_matrix", P_init)                      # :51
            self.log_transition_logits = None
        p0_init = torch.ones(num_states) / num_states
        self.log_initial_logits = nn.Parameter(torch.log(p0_init + 1e-8))        # :55-56
        self._hmm = None

    # -- parameters (hmm_layer.py:61-89) ---------------------------------------------
    def _get_transition_matrix(self) -> torch.Tensor:
        if self.log_transition_logits is not None:
            return F.softmax(self.log_transition_logits, dim=1)
        return self.transition_matrix

    def _get_initial_probabilities(self) -> torch.Tensor:
        return F.softmax(self.log_initial_logits, dim=0)

    def _param_key(self):
        """Identity + version of the tensors P and p0 derive from (and whether autograd is
        recording through them)."""
        src = self.log_transition_logits if self.log_transition_logits is not None else self.transition_matrix
        init = self.log_initial_logits
        grad = torch.is_grad_enabled() and (src.requires_grad or init.requires_grad)
        return (src, src._version, src.device, init, init._version, grad)

    def _get_hmm(self) -> HMMPyTorch:
        if self._hmm is not None:
            # later calls assign log(P + 1e-8) (hmm_layer.py:83-86).  With the parameters
            # unchanged since the previous later call and no autograd, the assigned tensors
            # would be bit-identical: keep them, so HMMPyTorch's device copies and transition
            # plan stay cached (no per-call softmax/log/plan launches).
            key = self._param_key()
            old = self.__dict__.get("_hmm_key")
            if (old is not None and not key[5] and old[0] is key[0] and old[3] is key[3]
                    and old[1:3] == key[1:3] and old[4:] == key[4:]):
                return self._hmm
        P = self._get_transition_matrix()
        p0 = self._get_initial_probabilities()
        device = P.device
        if self._hmm is None:
            self._hmm = HMMPyTorch(P, p0, device=str(device))
            self.__dict__["_hmm_key"] = None   # call 2 must re-derive (first-call quirk)
        else:
            self._hmm.P = P
            self._hmm.log_P = torch.log(P + 1e-8)
            self._hmm.p0 = p0
            self._hmm.log_p0 = torch.log(p0 + 1e-8)
            self._hmm.device = str(device)
            self.__dict__["_hmm_key"] = self._param_key()
        return self._hmm

    # -- forward (hmm_layer.py:91-142) -------------------------------------------------
    def forward(self, x: torch.Tensor,
                return_alignment: bool = False) -> Union[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]]:
        if self.apply_sigmoid:
            x = torch.sigmoid(x)
        if x.dim() == 2:
            x = x.unsqueeze(0)
        B, T, K = x.shape
        if K != self.num_states:
            raise ValueError(f"Input feature dim {K} must match num_states {self.num_states}")
        hmm = self._get_hmm()
        if self.training:
            posteriors = hmm.posteriors(x)
        elif self.viterbi_inference:
            states, _ = hmm.viterbi_decode(x)
            posteriors = F.one_hot(states, num_classes=self.num_states).float()
        else:
            posteriors = hmm.posteriors(x)
        if return_alignment and not self.training:
            alignment = states if self.viterbi_inference else torch.argmax(posteriors, dim=-1)
            return posteriors, alignment
        return posteriors

    def compute_loss(self, observations: torch.Tensor,
                     target_alignment: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Cross-entropy on posteriors when a target alignment is given, else -mean of
        compute_likelihood (hmm_layer.py:144-173)."""
        hmm = self._get_hmm()
        if target_alignment is not None:
            posteriors = self.forward(observations)
            return F.cross_entropy(posteriors.view(-1, self.num_states), target_alignment.view(-1))
        if self.apply_sigmoid:
            observations = torch.sigmoid(observations)
        return -hmm.compute_likelihood(observations).mean()

    def align(self, observations: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(states, log_delta) by Viterbi (hmm_layer.py:175-191)."""
        hmm = self._get_hmm()
        if self.apply_sigmoid:
            observations = torch.sigmoid(observations)
        return hmm.viterbi_decode(observations)

    def sample(self, seq_length: int, batch_size: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
        return self._get_hmm().sample(seq_length, batch_size)

    def get_transition_matrix(self) -> torch.Tensor:
        return self._get_transition_matrix()

    def get_initial_probabilities(self) -> torch.Tensor:
        return self._get_initial_probabilities()

    def extra_repr(self) -> str:
        return f"num_states={self.num_states}, viterbi_inference={self.viterbi_inference}"


def _gaussian_component_params(log_scales: torch.Tensor, covariance_type: str, D: int):
    """(K,1,D) log-variances for the GMM scorer from GaussianHMMLayer.log_scales
    (hmm_layer.py:286-319: log_var = 2*log_scales; 'full' uses the diagonal; 'spherical'
    one value per state)."""
    if covariance_type == "full":
        lv = 2 * torch.diagonal(log_scales, dim1=-2, dim2=-1)
    elif covariance_type == "spherical":
        lv = (2 * log_scales).expand(-1, D)
    else:
        lv = 2 * log_scales
    return lv.unsqueeze(1)


class GaussianHMMLayer(nn.Module):
    """Gaussian emissions + HMMLayer(apply_sigmoid=False) (reference hmm_layer.py:220-363)."""

    def __init__(self, num_states: int, feature_dim: int, covariance_type: str = "diag",
                 learnable_transitions: bool = True, transition_type: str = "left_to_right"):
        super().__init__()
        self.num_states = num_states
        self.feature_dim = feature_dim
        self.covariance_type = covariance_type
        self.hmm_layer = HMMLayer(num_states=num_states, learnable_transitions=learnable_transitions,
                                  transition_type=transition_type, apply_sigmoid=False)
        self.means = nn.Parameter(torch.randn(num_states, feature_dim))
        if covariance_type == "full":
            self.log_scales = nn.Parameter(torch.zeros(num_states, feature_dim, feature_dim))
        elif covariance_type == "diag":
            self.log_scales = nn.Parameter(torch.zeros(num_states, feature_dim))
        elif covariance_type == "spherical":
            self.log_scales = nn.Parameter(torch.zeros(num_states, 1))
        else:
            raise ValueError(f"Unknown covariance_type: {covariance_type}")

    def _compute_gaussian_log_probs(self, observations: torch.Tensor) -> torch.Tensor:
        """(B,T,D) -> (B,T,K) Gaussian log-densities on the gfx950 scorer
        (hmm_layer.py:270-323)."""
        B, T, D = observations.shape
        log_w = torch.zeros(self.num_states, 1, device=self.means.device)
        if needs_grad(observations, self.means, self.log_scales):
            lv = _gaussian_component_params(self.log_scales, self.covariance_type, D)
            return GmmLogProb.apply(observations, self.means.unsqueeze(1), lv, log_w, 0)
        lv = _gaussian_component_params(self.log_scales.detach(), self.covariance_type, D)
        return ops.gmm_diag_logprob(observations.detach(), self.means.detach().unsqueeze(1), lv, log_w, 0)

    def forward(self, observations: torch.Tensor) -> torch.Tensor:
        observation_probs = torch.exp(self._compute_gaussian_log_probs(observations))
        return self.hmm_layer(observation_probs)

    def compute_loss(self, observations: torch.Tensor) -> torch.Tensor:
        observation_probs = torch.exp(self._compute_gaussian_log_probs(observations))
        hmm = self.hmm_layer._get_hmm()
        return -hmm.compute_likelihood(observation_probs).mean()

    def extra_repr(self) -> str:
        return (f"num_states={self.num_states}, feature_dim={self.feature_dim}, "
                f"covariance_type={self.covariance_type}")
