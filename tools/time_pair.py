"""Diagnostic: time forward_backward through the pair kernel vs the two-kernel path."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import hmm_oracle as O
from pytorch_hmm_amd import ops as o
N = 128
lP, lp0 = O.hmm_params(O.left_to_right_matrix(N, 0.7))
lP, lp0 = lP.cuda(), lp0.cuda()
plan = o.make_plan(lP); plain = plan.clone()
for B, T in [(1, 2000), (32, 2000), (32, 200), (64, 2000)]:
    obs = torch.softmax(torch.randn(B, T, N, device="cuda"), -1)
    res = {}
    for nm, pl in (("pair", plan), ("plain", plain)):
        for _ in range(2): o.forward_backward(obs, lP, lp0, o.OBS_PROB, 7, pl)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5): o.forward_backward(obs, lP, lp0, o.OBS_PROB, 7, pl)
        e1.record(); torch.cuda.synchronize()
        res[nm] = e0.elapsed_time(e1) / 5
    print(B, T, {k: round(v, 4) for k, v in res.items()}, flush=True)
