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

try:  # layers are optional at import time only while they are being brought up
    from .hmm_layer import HMMLayer, GaussianHMMLayer  # noqa: F401
    __all__ += ["HMMLayer", "GaussianHMMLayer"]
except ImportError:  # pragma: no cover
    pass
try:
    from .mixture_gaussian import MixtureGaussianHMMLayer  # noqa: F401
    __all__ += ["MixtureGaussianHMMLayer"]
except ImportError:  # pragma: no cover
    pass
try:
    from .hsmm import HSMMLayer  # noqa: F401
    __all__ += ["HSMMLayer"]
except ImportError:  # pragma: no cover
    pass
try:
    from .neural import NeuralHMM, ContextualNeuralHMM  # noqa: F401
    from .semi_markov import DurationModel, SemiMarkovHMM, AdaptiveDurationHSMM  # noqa: F401
    from .streaming import StreamingHMMProcessor, StreamingResult, AdaptiveLatencyController  # noqa: F401
    __all__ += ["NeuralHMM", "ContextualNeuralHMM", "DurationModel", "SemiMarkovHMM", "AdaptiveDurationHSMM",
                "StreamingHMMProcessor", "StreamingResult", "AdaptiveLatencyController"]
except ImportError:  # pragma: no cover
    pass
