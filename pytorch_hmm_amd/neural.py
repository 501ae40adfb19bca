"""NeuralHMM / ContextualNeuralHMM — drop-ins for the reference's neural HMMs
(neural.py:10-588).

The transition and observation networks are ordinary torch modules with the reference's
constructor arguments, submodule names and initialisation (state_dict compatible:
``transition_model.network.*`` / ``rnn`` / ``transformer`` / ``output_layer``,
``observation_model.{feature_net,state_embedding,mean_net,logvar_net,weight_net,ar_net,
output_net}``, ``transition_matrix``, ``initial_logits``).  The hot path — the recursions over a
(B,T,N,N) tensor of per-step log transition matrices (neural.py:403-511) — runs in the
time-varying HIP kernels (csrc/tv.hip) via ops.tv_forward_backward / ops.tv_viterbi; a static
matrix (no context network, neural.py:383-385) is passed with zero strides instead of being
expanded into HBM.
"""
import math
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .autograd import needs_grad, TvSequenceLogLik, tv_forward_backward_with_grad


class NeuralTransitionModel(nn.Module):
    """Context -> per-step transition matrices (B,T,N,N) (reference neural.py:10-120)."""

    def __init__(self, num_states: int, context_dim: int, hidden_dim: int = 256, model_type: str = "mlp",
                 dropout: float = 0.1):
        super().__init__()
        self.num_states = num_states
        self.context_dim = context_dim
        self.hidden_dim = hidden_dim
        self.model_type = model_type
        K2 = num_states * num_states
        if model_type == "mlp":
            self.network = nn.Sequential(
                nn.Linear(context_dim + num_states, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
                nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
                nn.Linear(hidden_dim, K2))
        elif model_type == "rnn":
            self.rnn = nn.LSTM(context_dim, hidden_dim, batch_first=True, dropout=dropout)
            self.output_layer = nn.Linear(hidden_dim + num_states, K2)
        elif model_type == "transformer":
            layer = nn.TransformerEncoderLayer(d_model=context_dim, nhead=8, dim_feedforward=hidden_dim,
                                               dropout=dropout, batch_first=True)
            self.transformer = nn.TransformerEncoder(layer, num_layers=3)
            self.output_layer = nn.Linear(context_dim + num_states, K2)
        else:
            raise ValueError(f"Unknown model_type: {model_type}")

    def forward(self, context: torch.Tensor, current_state: Optional[torch.Tensor] = None) -> torch.Tensor:
        B = context.shape[0]
        single = context.dim() == 2
        if single:
            context = context.unsqueeze(1)
        T = context.shape[1]
        if current_state is None:   # uniform state belief (neural.py:87-89)
            current_state = torch.ones(B, T, self.num_states, device=context.device) / self.num_states
        elif current_state.dim() == 2:
            current_state = current_state.unsqueeze(1)
        if self.model_type == "mlp":
            logits = self.network(torch.cat([context, current_state], dim=-1))
        elif self.model_type == "rnn":
            h, _ = self.rnn(context)
            logits = self.output_layer(torch.cat([h, current_state], dim=-1))
        else:
            h = self.transformer(context)
            logits = self.output_layer(torch.cat([h, current_state], dim=-1))
        probs = F.softmax(logits.view(B, T, self.num_states, self.num_states), dim=-1)
        return probs.squeeze(1) if single else probs


class NeuralObservationModel(nn.Module):
    """Per-state observation log-densities (B,T,N) (reference neural.py:123-293).

    The reference scores one state at a time, re-running feature_net per state
    (neural.py:195-200).  In eval mode the features are identical for every state, so they
    are computed once and broadcast over the state embeddings; in train mode the per-state
    loop is kept so every state draws its own dropout masks, as in the reference."""

    def __init__(self, num_states: int, observation_dim: int, hidden_dim: int = 256, model_type: str = "gaussian",
                 num_components: int = 3, dropout: float = 0.1):
        super().__init__()
        self.num_states = num_states
        self.observation_dim = observation_dim
        self.hidden_dim = hidden_dim
        self.model_type = model_type
        self.num_components = num_components
        if model_type == "gaussian":
            self.mean_net = nn.Linear(hidden_dim, observation_dim)
            self.logvar_net = nn.Linear(hidden_dim, observation_dim)
        elif model_type == "mixture":
            self.weight_net = nn.Linear(hidden_dim, num_components)
            self.mean_net = nn.Linear(hidden_dim, num_components * observation_dim)
            self.logvar_net = nn.Linear(hidden_dim, num_components * observation_dim)
        elif model_type == "autoregressive":
            self.ar_net = nn.LSTM(observation_dim, hidden_dim, batch_first=True)
            self.output_net = nn.Linear(hidden_dim, observation_dim)
        self.state_embedding = nn.Embedding(num_states, hidden_dim)
        self.feature_net = nn.Sequential(
            nn.Linear(observation_dim, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
            nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.Dropout(dropout))

    def forward(self, observations: torch.Tensor, state_indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        if state_indices is not None:
            return self._score(observations, self.state_embedding(state_indices), self.feature_net(observations))
        B, T, _ = observations.shape
        if self.training and any(isinstance(m, nn.Dropout) and m.p > 0 for m in self.feature_net):
            cols = []
            for s in range(self.num_states):
                idx = torch.full((B, T), s, device=observations.device, dtype=torch.long)
                cols.append(self._score(observations, self.state_embedding(idx), self.feature_net(observations)))
            return torch.stack(cols, dim=-1)
        feats = self.feature_net(observations).unsqueeze(2)                   # (B,T,1,H)
        emb = self.state_embedding.weight.view(1, 1, self.num_states, -1)    # (1,1,N,H)
        return self._score(observations.unsqueeze(2), emb, feats)

    def _score(self, x, state_emb, feats):
        combined = state_emb + feats
        if self.model_type == "gaussian":
            return self._gaussian_log_prob(x, self.mean_net(combined), self.logvar_net(combined))
        if self.model_type == "mixture":
            C, D = self.num_components, self.observation_dim
            w = F.softmax(self.weight_net(combined), dim=-1)
            means = self.mean_net(combined).view(*combined.shape[:-1], C, D)
            log_vars = self.logvar_net(combined).view(*combined.shape[:-1], C, D)
            comp = self._gaussian_log_prob(x.unsqueeze(-2), means, log_vars)
            return torch.logsumexp(torch.log(w + 1e-8) + comp, dim=-1)
        if self.model_type == "autoregressive":
            xs = x.squeeze(2) if x.dim() == 4 else x
            h, _ = self.ar_net(xs)
            mse = F.mse_loss(self.output_net(h), xs, reduction="none").mean(dim=-1)
            lp = -mse
            return lp.unsqueeze(-1).expand(*combined.shape[:-1]) if combined.dim() == 4 else lp
        raise ValueError(f"Unknown model_type: {self.model_type}")

    def _gaussian_log_prob(self, x, mean, log_var):
        """neural.py:259-270."""
        var = torch.exp(log_var)
        log_norm = -0.5 * (self.observation_dim * math.log(2 * math.pi) + torch.sum(log_var, dim=-1))
        return log_norm - 0.5 * torch.sum((x - mean) ** 2 / var, dim=-1)

    def sample(self, state_indices: torch.Tensor, num_samples: int = 1) -> torch.Tensor:
        B, T = state_indices.shape
        emb = self.state_embedding(state_indices)
        if self.model_type == "gaussian":
            means, log_vars = self.mean_net(emb), self.logvar_net(emb)
            return means + torch.exp(0.5 * log_vars) * torch.randn_like(means)
        return torch.zeros(B, T, self.observation_dim, device=state_indices.device)


class NeuralHMM(nn.Module):
    """HMM with network-parameterised transitions and emissions (reference neural.py:296-519)."""

    def __init__(self, num_states: int, observation_dim: int, context_dim: int = 0, hidden_dim: int = 256,
                 transition_type: str = "mlp", observation_type: str = "gaussian", dropout: float = 0.1):
        super().__init__()
        self.num_states = num_states
        self.observation_dim = observation_dim
        self.context_dim = context_dim
        if context_dim > 0:
            self.transition_model = NeuralTransitionModel(num_states, context_dim, hidden_dim, transition_type,
                                                          dropout)
        else:
            self.transition_matrix = nn.Parameter(torch.randn(num_states, num_states))
            self.transition_model = None
        self.observation_model = NeuralObservationModel(num_states, observation_dim, hidden_dim, observation_type,
                                                        dropout=dropout)
        self.initial_logits = nn.Parameter(torch.zeros(num_states))

    # -- the recursion inputs (neural.py:374-389) -------------------------------------------
    def _log_transitions(self, B: int, T: int, context: Optional[torch.Tensor]) -> torch.Tensor:
        if self.transition_model is not None and context is not None:
            return torch.log(self.transition_model(context) + 1e-8)                 # (B,T',N,N)
        # no context network: ONE (N,N) matrix for every (b,t) (neural.py:383-385 expands it;
        # the kernels take it with zero strides)
        return torch.log(F.softmax(self.transition_matrix, dim=1) + 1e-8)

    def _log_initial(self) -> torch.Tensor:
        return torch.log(F.softmax(self.initial_logits, dim=0) + 1e-8)

    def forward(self, observations: torch.Tensor,
                context: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(posteriors, forward, backward), each (B,T,N) (neural.py:355-401)."""
        B, T, _ = observations.shape
        log_obs = self.observation_model(observations)
        log_A = self._log_transitions(B, T, context)
        log_init = self._log_initial()
        mask = ops.FB_POSTERIOR | ops.FB_FORWARD | ops.FB_BACKWARD
        if needs_grad(log_obs, log_A, log_init):
            # differentiable outputs: the analytic adjoint on csrc/tv.hip (autograd.TvForwardBackwardFn)
            return tv_forward_backward_with_grad(log_obs, log_A, log_init, mask)
        post, fwd, bwd, _, _ = ops.tv_forward_backward(log_obs, log_A, log_init, mask)
        return post, fwd, bwd

    def viterbi_decode(self, observations: torch.Tensor,
                       context: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """(states (B,T) int64, log_delta (B,T,N)) (neural.py:463-511)."""
        B, T, _ = observations.shape
        with torch.no_grad():
            log_obs = self.observation_model(observations)
            log_A = self._log_transitions(B, T, context)
            return ops.tv_viterbi(log_obs, log_A, self._log_initial())

    def compute_likelihood(self, observations: torch.Tensor,
                           context: Optional[torch.Tensor] = None) -> torch.Tensor:
        """LSE(log(forward[:, -1] + 1e-8)) per sequence (neural.py:513-519), differentiable."""
        B, T, _ = observations.shape
        log_obs = self.observation_model(observations)
        log_A = self._log_transitions(B, T, context)
        log_init = self._log_initial()
        if needs_grad(log_obs, log_A, log_init):
            return TvSequenceLogLik.apply(log_obs, log_A, log_init, "ref")
        return ops.tv_forward_backward(log_obs, log_A, log_init, 0)[4]


class ContextualNeuralHMM(NeuralHMM):
    """NeuralHMM over phoneme-embedding + prosody context (reference neural.py:522-588)."""

    def __init__(self, num_states: int, observation_dim: int, phoneme_vocab_size: int,
                 linguistic_context_dim: int = 64, prosody_dim: int = 16, **kwargs):
        self.phoneme_vocab_size = phoneme_vocab_size
        self.linguistic_context_dim = linguistic_context_dim
        self.prosody_dim = prosody_dim
        super().__init__(num_states=num_states, observation_dim=observation_dim,
                         context_dim=linguistic_context_dim + prosody_dim, **kwargs)
        self.phoneme_embedding = nn.Embedding(phoneme_vocab_size, linguistic_context_dim)
        self.prosody_encoder = nn.Linear(prosody_dim, prosody_dim)

    def encode_context(self, phoneme_sequence: torch.Tensor, prosody_features: torch.Tensor) -> torch.Tensor:
        return torch.cat([self.phoneme_embedding(phoneme_sequence), self.prosody_encoder(prosody_features)], dim=-1)

    def forward_with_context(self, observations: torch.Tensor, phoneme_sequence: torch.Tensor,
                             prosody_features: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        return self.forward(observations, self.encode_context(phoneme_sequence, prosody_features))
