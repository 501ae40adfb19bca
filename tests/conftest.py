import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); runs the HIP kernels")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    """Load a committed fixture (data only; written by tests/golden/make_golden.py)."""
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


@pytest.fixture
def gold():
    return golden


def force_dense_plans(monkeypatch):
    """Every transition plan made from here on selects the dense chains (HMM355_PLAN_DENSE):
    the layers and HMMPyTorch build their plans through ops.make_plan."""
    from pytorch_hmm_amd import ops
    orig = ops.make_plan
    monkeypatch.setattr(ops, "make_plan", lambda log_P, read_banded=True, dense=False: orig(log_P, read_banded, True))


# -- host numerics fingerprint ------------------------------------------------------------
# The fixtures under tests/golden/ were produced by the reference on torch-CPU in the build
# container. torch-CPU's vector exp/log/softmax and its GEMMs pick kernels by host ISA, so the
# torch-CPU parts of the oracle reproduce the fixtures bit for bit only on a host whose
# fingerprint below matches (the GPU box's host, e.g., differs in the last bit of exp). On such
# a host the oracle-vs-fixture bit-exactness tests are reported as xfail with the reason; the
# GPU parity tests, which compare the HIP path with the fixtures directly, are unaffected.
HOST_BITEXACT_TESTS = {
    "test_hsmm_layer_tables_match_reference", "test_hmmpytorch_oracle_bitexact",
    "test_ties_and_wiki", "test_hmmlayer_first_call_renormalises", "test_mixture_oracle",
    "test_mixture_chunked_emission_identical", "test_hsmm_oracle",
    "test_neural_oracle_bitexact", "test_duration_tables_bitexact", "test_mixture_cov_oracle",
    "test_gaussian_cov_log_probs",
}
FINGERPRINT_FILE = os.path.join(GOLDEN, "host_numerics.txt")


def host_numerics_fingerprint():
    import hashlib

    import torch
    g = torch.Generator().manual_seed(1234)
    x = torch.randn(4096, generator=g)
    a = torch.randn(128, 128, generator=g)
    parts = [torch.exp(x), torch.log(x.abs() + 1e-3), torch.softmax(a, dim=-1),
             torch.logsumexp(a, dim=-1), a @ a, torch.log_softmax(a, dim=0)]
    h = hashlib.sha256()
    for p in parts:
        h.update(p.contiguous().numpy().tobytes())
    return h.hexdigest()


def pytest_collection_modifyitems(config, items):
    try:
        with open(FINGERPRINT_FILE) as f:
            want = f.read().strip()
    except OSError:
        return
    if host_numerics_fingerprint() == want:
        return
    mark = pytest.mark.xfail(reason="torch-CPU numerics of this host differ from the host that "
                             "made tests/golden (fingerprint mismatch); oracle bit-exactness "
                             "vs fixtures is checked on the fixture host", strict=False)
    for it in items:
        if getattr(it, "originalname", it.name) in HOST_BITEXACT_TESTS:
            it.add_marker(mark)
