"""pytorch_hmm_amd — MI355X (gfx950) native HMM inference core.

Drop-in for the hot path of crlotwhite/pytorch_hmm: HMMPyTorch.forward_backward /
viterbi_decode / compute_likelihood, HMMLayer, GaussianHMMLayer,
MixtureGaussianHMMLayer and HSMMLayer, and the next rows of that path (NeuralHMM,
SemiMarkovHMM, StreamingHMMProcessor), with the per-time-step loops replaced by
hand-written HIP kernels (csrc/) behind the C ABI in include/hmm355.h and the
torch.library ops in ops.py.  Tensors must be on a ROCm GPU; there is no CPU path.
"""
from .hmm import HMM, HMMPyTorch
from .utils import create_left_to_right_matrix, create_transition_matrix
from . import ops

__all__ = ["HMM", "HMMPyTorch", "create_left_to_right_matrix", "create_transition_matrix", "ops"]

from .hmm_layer import HMMLayer, GaussianHMMLayer
from .mixture_gaussian import MixtureGaussianHMMLayer
from .hsmm import HSMMLayer
from .neural import NeuralHMM, ContextualNeuralHMM
from .semi_markov import DurationModel, SemiMarkovHMM, AdaptiveDurationHSMM
from .streaming import AdaptiveLatencyController, StreamingHMMProcessor, StreamingResult

__all__ += ["HMMLayer", "GaussianHMMLayer", "MixtureGaussianHMMLayer", "HSMMLayer", "NeuralHMM",
            "ContextualNeuralHMM", "DurationModel", "SemiMarkovHMM", "AdaptiveDurationHSMM",
            "StreamingHMMProcessor", "StreamingResult", "AdaptiveLatencyController"]
