"""ctypes binding of libhmm355.so — the C ABI declared in include/hmm355.h.

The product path has exactly one implementation: the HIP kernels behind this library.
If the library is missing or a call fails, this module raises; there is no CPU fallback.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HMM355_LIB", os.path.join(_HERE, "lib", "libhmm355.so"))

OBS_PROB = 0
OBS_LOG = 1
FB_POSTERIOR = 1
FB_PAIR = 0x100
FB_PLAN_BANDED = 0x200  # HMM355_FB_PLAN_BANDED
VIT_PLAN_BANDED = 0x1  # HMM355_VIT_PLAN_BANDED
VIT_PLAN_DENSE = 0x2  # HMM355_VIT_PLAN_DENSE
PLAN_DENSE = 0x1  # HMM355_PLAN_DENSE
FORM_GENERAL = 0x1  # HMM355_FORM_GENERAL
FORM_SERIAL_WALK = 0x2  # HMM355_FORM_SERIAL_WALK
FB_FORWARD = 2
FB_BACKWARD = 4

# every symbol include/hmm355.h declares (checked by tests/test_native_abi.py)
EXPORTS = (
    "hmm355_strerror", "hmm355_version",
    "hmm355_fb_workspace_bytes", "hmm355_fb_workspace_layout", "hmm355_forward_backward_f32",
    "hmm355_forward_backward_ex_f32",
    "hmm355_viterbi_workspace_bytes", "hmm355_viterbi_workspace_bytes_ex", "hmm355_viterbi_f32",
    "hmm355_gmm_workspace_bytes", "hmm355_gmm_diag_logprob_f32",
    "hmm355_hsmm_workspace_bytes", "hmm355_hsmm_viterbi_f32", "hmm355_hsmm_workspace_bytes_ex",
    "hmm355_hsmm_viterbi_ex_f32",
    "hmm355_tv_fb_workspace_bytes", "hmm355_tv_forward_backward_f32", "hmm355_tv_forward_backward_ex_f32",
    "hmm355_tv_viterbi_workspace_bytes", "hmm355_tv_viterbi_f32",
    "hmm355_semimarkov_workspace_bytes", "hmm355_semimarkov_quad_f32",
    "hmm355_semimarkov_viterbi_f32", "hmm355_semimarkov_forward_f32", "hmm355_semimarkov_workspace_bytes_ex",
    "hmm355_semimarkov_viterbi_ex_f32", "hmm355_semimarkov_forward_ex_f32",
    "hmm355_stream_greedy_f32", "hmm355_stream_beam_f32",
    "hmm355_plan_bytes", "hmm355_plan_f32", "hmm355_plan_ex_f32", "hmm355_plan_banded",
    "hmm355_forward_backward_plan_f32", "hmm355_viterbi_plan_f32", "hmm355_viterbi_plan_ex_f32",
    "hmm355_fb_adjoint_f32", "hmm355_tv_fb_adjoint_f32",
)

_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load libhmm355.so (raises NativeError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"libhmm355.so not found at {LIB_PATH}; build it with "
            "`python -m pytorch_hmm_amd.build_native` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    P, I, U, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_size_t
    L.hmm355_strerror.argtypes, L.hmm355_strerror.restype = [I], ctypes.c_char_p
    L.hmm355_version.argtypes, L.hmm355_version.restype = [], I
    L.hmm355_fb_workspace_bytes.argtypes, L.hmm355_fb_workspace_bytes.restype = [I, I, I], S
    L.hmm355_fb_workspace_layout.argtypes, L.hmm355_fb_workspace_layout.restype = [I, I, I, P], I
    L.hmm355_forward_backward_f32.argtypes = [P, I, P, P, I, I, I, U, P, P, P, P, P, P, S, P]
    L.hmm355_forward_backward_f32.restype = I
    L.hmm355_forward_backward_ex_f32.argtypes = [P, I, P, P, P, I, I, I, U, P, P, P, P, P, P, S, P]
    L.hmm355_forward_backward_ex_f32.restype = I
    L.hmm355_viterbi_workspace_bytes.argtypes, L.hmm355_viterbi_workspace_bytes.restype = [I, I, I], S
    L.hmm355_viterbi_workspace_bytes_ex.argtypes, L.hmm355_viterbi_workspace_bytes_ex.restype = [I, I, I, I], S
    L.hmm355_viterbi_f32.argtypes = [P, I, P, P, I, I, I, P, P, P, P, S, P]
    L.hmm355_viterbi_f32.restype = I
    L.hmm355_gmm_workspace_bytes.argtypes, L.hmm355_gmm_workspace_bytes.restype = [I, I, I, I, I], S
    L.hmm355_gmm_diag_logprob_f32.argtypes = [P, P, P, P, I, I, I, I, I, I, P, P, S, P]
    L.hmm355_gmm_diag_logprob_f32.restype = I
    L.hmm355_hsmm_workspace_bytes.argtypes, L.hmm355_hsmm_workspace_bytes.restype = [I, I, I, I], S
    L.hmm355_hsmm_viterbi_f32.argtypes = [P, P, P, I, I, I, I, P, P, P, S, P]
    L.hmm355_hsmm_viterbi_f32.restype = I
    L.hmm355_hsmm_workspace_bytes_ex.argtypes, L.hmm355_hsmm_workspace_bytes_ex.restype = [I, I, I, I, U], S
    L.hmm355_hsmm_viterbi_ex_f32.argtypes = [P, P, P, I, I, I, I, U, P, P, P, S, P]
    L.hmm355_hsmm_viterbi_ex_f32.restype = I
    LL = ctypes.c_longlong
    L.hmm355_tv_fb_workspace_bytes.argtypes, L.hmm355_tv_fb_workspace_bytes.restype = [I, I, I], S
    L.hmm355_tv_forward_backward_f32.argtypes = [P, P, LL, LL, P, I, I, I, U, P, P, P, P, P, P, S, P]
    L.hmm355_tv_forward_backward_f32.restype = I
    L.hmm355_tv_forward_backward_ex_f32.argtypes = [P, P, LL, LL, P, P, I, I, I, U, P, P, P, P, P, P, S, P]
    L.hmm355_tv_forward_backward_ex_f32.restype = I
    L.hmm355_tv_viterbi_workspace_bytes.argtypes, L.hmm355_tv_viterbi_workspace_bytes.restype = [I, I, I], S
    L.hmm355_tv_viterbi_f32.argtypes = [P, P, LL, LL, P, I, I, I, P, P, P, S, P]
    L.hmm355_tv_viterbi_f32.restype = I
    L.hmm355_semimarkov_workspace_bytes.argtypes = [I, I, I, I]
    L.hmm355_semimarkov_workspace_bytes.restype = S
    L.hmm355_semimarkov_quad_f32.argtypes, L.hmm355_semimarkov_quad_f32.restype = [P, P, P, I, I, I, I, P, P], I
    L.hmm355_semimarkov_viterbi_f32.argtypes = [P, P, P, P, P, I, I, I, I, P, P, P, P, P, S, P]
    L.hmm355_semimarkov_viterbi_f32.restype = I
    L.hmm355_semimarkov_forward_f32.argtypes = [P, P, P, P, P, I, I, I, I, P, P, P, S, P]
    L.hmm355_semimarkov_forward_f32.restype = I
    L.hmm355_semimarkov_workspace_bytes_ex.argtypes = [I, I, I, I, U]
    L.hmm355_semimarkov_workspace_bytes_ex.restype = S
    L.hmm355_semimarkov_viterbi_ex_f32.argtypes = [P, P, P, P, P, I, I, I, I, U, P, P, P, P, P, S, P]
    L.hmm355_semimarkov_viterbi_ex_f32.restype = I
    L.hmm355_semimarkov_forward_ex_f32.argtypes = [P, P, P, P, P, I, I, I, I, U, P, P, P, S, P]
    L.hmm355_semimarkov_forward_ex_f32.restype = I
    F = ctypes.c_float
    L.hmm355_plan_bytes.argtypes, L.hmm355_plan_bytes.restype = [I], S
    L.hmm355_plan_f32.argtypes, L.hmm355_plan_f32.restype = [P, I, P, P], I
    L.hmm355_plan_ex_f32.argtypes, L.hmm355_plan_ex_f32.restype = [P, I, U, P, P], I
    L.hmm355_plan_banded.argtypes, L.hmm355_plan_banded.restype = [P, P], I
    L.hmm355_forward_backward_plan_f32.argtypes = [P, I, P, P, P, P, I, I, I, U, P, P, P, P, P, P, S, P]
    L.hmm355_forward_backward_plan_f32.restype = I
    L.hmm355_viterbi_plan_f32.argtypes = [P, I, P, P, P, I, I, I, P, P, P, P, S, P]
    L.hmm355_viterbi_plan_f32.restype = I
    L.hmm355_viterbi_plan_ex_f32.argtypes = [P, I, P, P, P, U, I, I, I, P, P, P, P, S, P]
    L.hmm355_viterbi_plan_ex_f32.restype = I
    L.hmm355_stream_greedy_f32.argtypes, L.hmm355_stream_greedy_f32.restype = [P, P, P, F, I, I, I, P, P, P], I
    L.hmm355_stream_beam_f32.argtypes = [P, P, I, I, I, I, I, P, P, P, P, P, P, P, P]
    L.hmm355_stream_beam_f32.restype = I
    L.hmm355_fb_adjoint_f32.argtypes, L.hmm355_fb_adjoint_f32.restype = [P, P, P, P, P, P, I, I, I, P, P, P], I
    LL = ctypes.c_longlong
    L.hmm355_tv_fb_adjoint_f32.argtypes = [P, P, LL, LL, P, P, P, P, I, I, I, P, P, P]
    L.hmm355_tv_fb_adjoint_f32.restype = I
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().hmm355_strerror(rc).decode()
        raise NativeError(f"hmm355 call failed ({rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(device):
    """The current HIP stream on `device` as a raw handle."""
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_gpu(*tensors):
    for t in tensors:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError(
                "pytorch_hmm_amd runs its hot path on ROCm GPUs only (MI355X/gfx950); got a "
                f"tensor on '{t.device}'. Move the inputs to 'cuda' (there is no CPU fallback).")
