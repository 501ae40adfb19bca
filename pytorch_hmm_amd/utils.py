"""Transition-matrix factories used to build the hot path's inputs.

Same names, arguments and results as the reference's factories (utils.py:9-103) so that
`HMMPyTorch(create_left_to_right_matrix(128, 0.7))` builds bit-identical parameters.
"""
import torch


def create_transition_matrix(num_states: int, transition_type: str = "ergodic",
                             self_loop_prob: float = 0.5, forward_prob: float = 0.4,
                             skip_prob: float = 0.1, device: str = "cpu") -> torch.Tensor:
    """Row-stochastic (K, K) matrix of type 'ergodic' | 'left_to_right' |
    'left_to_right_skip' | 'circular' (reference utils.py:9-77)."""
    K = num_states
    if transition_type == "ergodic":
        P = torch.ones(K, K, device=device) + torch.eye(K, device=device) * self_loop_prob * K
    elif transition_type in ("left_to_right", "left_to_right_skip", "circular"):
        P = torch.zeros(K, K, device=device)
        idx = torch.arange(K, device=device)
        if transition_type == "circular":
            P[idx, idx] = self_loop_prob
            P[idx, (idx + 1) % K] = forward_prob
        else:
            last = 1 if transition_type == "left_to_right" else 2
            body = idx[: max(K - last, 0)]
            P[body, body] = self_loop_prob
            P[body, body + 1] = forward_prob
            if transition_type == "left_to_right_skip":
                P[body, body + 2] = skip_prob
                if K >= 2:
                    P[K - 2, K - 2] = self_loop_prob
                    P[K - 2, K - 1] = forward_prob
            P[K - 1, K - 1] = 1.0
    else:
        raise ValueError(f"Unknown transition_type: {transition_type}")
    return P / P.sum(dim=1, keepdim=True)


def create_left_to_right_matrix(num_states: int, self_loop_prob: float = 0.7,
                                device: str = "cpu") -> torch.Tensor:
    """Bakis left-to-right matrix (reference utils.py:80-103)."""
    return create_transition_matrix(num_states, "left_to_right", self_loop_prob,
                                    1.0 - self_loop_prob, device=device)
