"""Diagnostic: time the GMM emission scorer (ops.gmm_diag_logprob) on the BASELINE layer shapes
for each scorer configuration (HMM355_GMM_CFG: 0 = first scorer, 1.. = v2 shapes, csrc/gmm.hip),
and check every configuration's output bits against the first scorer's."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_hmm_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
shapes = {"c3": (32, 2000, 80, 128, 4), "c2": (32, 2000, 80, 64, 1), "c5": (16, 2000, 80, 64, 1)}
for name, (B, T, D, S, C) in shapes.items():
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(B, T, D, device=dev, generator=g)
    mu = torch.randn(S, C, D, device=dev, generator=g)
    lv = torch.randn(S, C, D, device=dev, generator=g) * 0.3
    lw = torch.log_softmax(torch.randn(S, C, device=dev, generator=g), -1)
    ref = None
    for cfg in ("0", "1", "2", "3", "4", "5"):
        os.environ["HMM355_GMM_CFG"] = cfg
        out = ops.gmm_diag_logprob(x, mu, lv, lw, 1 if C > 1 else 0)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        same = torch.equal(out.view(torch.int32), ref.view(torch.int32))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            ops.gmm_diag_logprob(x, mu, lv, lw, 1 if C > 1 else 0)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        fl = 2.0 * B * T * S * C * D * 2
        print(f"{name} cfg {cfg}: {ms * 1e3:7.1f} us/call  {fl / ms / 1e9:6.1f} TFLOP/s fp64  bits==cfg0: {same}", flush=True)
