"""HMM / HMMPyTorch — drop-in for the reference's core recursions (hmm.py:7-254).

Parameter preparation is the reference's own arithmetic (renormalise P, log(P + 1e-8),
uniform or renormalised p0, hmm.py:20-55), done once on the device the parameters are
given on, so the kernels see the reference's log_P / log_p0 bits.  The per-time-step
loops are replaced by the gfx950 kernels behind torch.ops.hmm355 (see ops.py,
pytorch_hmm_amd/csrc/*.hip); observations must live on a ROCm GPU.
"""
from typing import Optional, Tuple, Union

import numpy as np
import torch

from . import ops
from .autograd import SequenceLogLik, forward_backward_with_grad, needs_grad


class HMM:
    """Base class: transition matrix P (K,K) and initial distribution p0 (K)
    (reference hmm.py:7-55; same validation and the same ValueError messages)."""

    def __init__(self, P: Union[np.ndarray, torch.Tensor], p0: Optional[Union[np.ndarray, torch.Tensor]] = None,
                 device: str = "cpu"):
        if isinstance(P, np.ndarray):
            P = torch.from_numpy(P).float()
        P = P.to(device)
        self.K = P.shape[0]
        self.device = device
        if len(P.shape) != 2:
            raise ValueError(f"P shape should have length 2. found {len(P.shape)}")
        if P.shape[0] != P.shape[1]:
            raise ValueError(f"P should be square, found {P.shape}")
        P = P / P.sum(dim=1, keepdim=True)
        self.P = P
        self.log_P = torch.log(P + 1e-8)
        if p0 is None:
            self.p0 = torch.ones(self.K, device=device) / self.K
        else:
            if isinstance(p0, np.ndarray):
                p0 = torch.from_numpy(p0).float()
            p0 = p0.to(device)
            if len(p0) != self.K:
                raise ValueError(f"dimensions of p0 {p0.shape} must match P[0] {P.shape[0]}")
            self.p0 = p0 / p0.sum()
        self.log_p0 = torch.log(self.p0 + 1e-8)


class HMMPyTorch(HMM):
    """Forward-backward, Viterbi and likelihood on MI355X (reference hmm.py:58-254)."""

    # -- helpers -------------------------------------------------------------------
    def _device_params(self, dev):
        """(log_P, log_p0, plan) on device `dev`.  Device copies and the transition plan
        (ops.make_plan: the banded structure of log_P, measured once) are cached while log_P /
        log_p0 are unchanged."""
        lp, l0 = self.log_P, self.log_p0
        # The entry holds the source tensors themselves: a hit needs the SAME objects at the
        # same version (a freed host buffer's address can be reused by a new tensor).
        cache = self.__dict__.setdefault("_dev_cache", {})
        hit = cache.get(str(dev))
        if (hit is None or hit[0] is not lp or hit[1] is not l0 or hit[2] != (lp._version, l0._version)
                or lp.requires_grad or l0.requires_grad):
            lpd = lp if lp.device == dev else lp.to(dev)
            l0d = l0 if l0.device == dev else l0.to(dev)
            # A plan re-formed every call (log_P requires grad: a training step changes it)
            # skips the host read of its structure, so a training forward never waits on the
            # device (ops.make_plan read_banded=False).
            grad = lp.requires_grad or l0.requires_grad
            plan = ops.make_plan(lpd.detach(), read_banded=not grad) if dev.type == "cuda" else None
            hit = (lp, l0, (lp._version, l0._version), lpd, l0d, plan)
            if not grad:
                cache[str(dev)] = hit
        return hit[3], hit[4], hit[5]

    @staticmethod
    def _as_batch(observations):
        if observations.dim() == 2:
            return observations.unsqueeze(0), True
        return observations, False

    # -- reference API -------------------------------------------------------------
    def forward_backward(self, observations: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(posterior, forward, backward), each (B,T,K) — 2-D input is NOT squeezed, as in
        the reference (hmm.py:66-130).  forward/backward are exp(log alpha)/exp(log beta) and
        underflow to 0 for long sequences exactly as the reference's do."""
        obs, _ = self._as_batch(observations)
        B, T, K = obs.shape
        assert K == self.K, f"Observation dim {K} must match model states {self.K}"
        log_P, log_p0, plan = self._device_params(obs.device)
        mask = ops.FB_POSTERIOR | ops.FB_FORWARD | ops.FB_BACKWARD
        if needs_grad(obs, log_P, log_p0):
            # differentiable through all three outputs (autograd.ForwardBackwardFn)
            return forward_backward_with_grad(obs, log_P, log_p0, ops.OBS_PROB, mask, plan)
        post, fwd, bwd, _, _ = ops.forward_backward(obs.detach(), log_P.detach(), log_p0.detach(), ops.OBS_PROB,
                                                    mask, plan)
        return post, fwd, bwd

    def posteriors(self, observations: torch.Tensor) -> torch.Tensor:
        """Posterior only (what HMMLayer needs); skips the forward/backward outputs."""
        obs, _ = self._as_batch(observations)
        assert obs.shape[-1] == self.K, f"Observation dim {obs.shape[-1]} must match model states {self.K}"
        log_P, log_p0, plan = self._device_params(obs.device)
        if needs_grad(obs, log_P, log_p0):
            return forward_backward_with_grad(obs, log_P, log_p0, ops.OBS_PROB, ops.FB_POSTERIOR, plan)[0]
        return ops.forward_backward(obs.detach(), log_P.detach(), log_p0.detach(), ops.OBS_PROB,
                                    ops.FB_POSTERIOR, plan)[0]

    def viterbi_decode(self, observations: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(states (B,T) int64, log_delta (B,T,K)); 2-D input squeezed (hmm.py:132-184)."""
        obs, squeeze = self._as_batch(observations)
        B, T, K = obs.shape
        assert K == self.K, f"Observation dim {K} must match model states {self.K}"
        log_P, log_p0, plan = self._device_params(obs.device)
        states, delta, _ = ops.viterbi(obs.detach(), log_P.detach(), log_p0.detach(), ops.OBS_PROB, plan)
        if squeeze:
            return states.squeeze(0), delta.squeeze(0)
        return states, delta

    def compute_likelihood(self, observations: torch.Tensor) -> torch.Tensor:
        """The reference's value logsumexp(log(forward[:, -1] + 1e-8)) (hmm.py:186-211),
        including its saturation at log(K*1e-8) once exp(log alpha) underflows."""
        obs, squeeze = self._as_batch(observations)
        B, T, K = obs.shape
        assert K == self.K, f"Observation dim {K} must match model states {self.K}"
        log_P, log_p0, plan = self._device_params(obs.device)
        if needs_grad(obs, log_P, log_p0):
            ll = SequenceLogLik.apply(obs, log_P, log_p0, ops.OBS_PROB, "ref")
        else:
            ll = ops.forward_backward(obs, log_P, log_p0, ops.OBS_PROB, 0, plan)[4]
        return ll.squeeze(0) if squeeze else ll

    def log_likelihood(self, observations: torch.Tensor) -> torch.Tensor:
        """Extension: the well-defined sequence log-likelihood log sum_j alpha_{T-1}[j]
        (what compute_likelihood would return without exp() underflow)."""
        obs, squeeze = self._as_batch(observations)
        assert obs.shape[-1] == self.K, f"Observation dim {obs.shape[-1]} must match model states {self.K}"
        log_P, log_p0, plan = self._device_params(obs.device)
        if needs_grad(obs, log_P, log_p0):
            ll = SequenceLogLik.apply(obs, log_P, log_p0, ops.OBS_PROB, "exact")
        else:
            ll = ops.forward_backward(obs, log_P, log_p0, ops.OBS_PROB, 0, plan)[3]
        return ll.squeeze(0) if squeeze else ll

    def sample(self, seq_length: int, batch_size: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
        """Sample (states, one-hot observations) — reference hmm.py:213-245 (not on the hot
        path; plain torch sampling on the parameters' device)."""
        dev = self.P.device
        states = torch.zeros(batch_size, seq_length, dtype=torch.long, device=dev)
        observations = torch.zeros(batch_size, seq_length, self.K, device=dev)
        states[:, 0] = torch.distributions.Categorical(self.p0).sample((batch_size,))
        for t in range(seq_length):
            if t > 0:
                states[:, t] = torch.distributions.Categorical(self.P[states[:, t - 1]]).sample()
            observations[torch.arange(batch_size, device=dev), t, states[:, t]] = 1.0
        return states, observations

    def to(self, device: str):
        """Move parameters (reference hmm.py:247-254)."""
        self.device = device
        self.P = self.P.to(device)
        self.log_P = self.log_P.to(device)
        self.p0 = self.p0.to(device)
        self.log_p0 = self.log_p0.to(device)
        return self
