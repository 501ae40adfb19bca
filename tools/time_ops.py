"""Diagnostic: the NS ops (forward_backward mask 7, viterbi) at B=32 T=2000 N=128, timed alone
and side by side on two streams (the bench's pattern), for one transition matrix
(argv[1]: l2r | random)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytorch_hmm_amd as ph  # noqa: E402
from pytorch_hmm_amd import ops  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "random"
dev = torch.device("cuda", 0)
B, T, N = 32, 2000, 128
if kind == "random":
    gp = torch.Generator().manual_seed(4321)
    hmm = ph.HMMPyTorch(torch.softmax(torch.randn(N, N, generator=gp), dim=-1))
else:
    hmm = ph.HMMPyTorch(ph.create_left_to_right_matrix(N, 0.7))
g = torch.Generator(device=dev).manual_seed(1234)
obs = torch.softmax(torch.randn(B, T, N, device=dev, generator=g), dim=-1)
lP, lp0, plan = hmm._device_params(dev)
fb = lambda: ops.forward_backward(obs, lP, lp0, ops.OBS_PROB, 7, plan)
vit = lambda: ops.viterbi(obs, lP, lp0, ops.OBS_PROB, plan)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def both():
    cur = torch.cuda.current_stream(dev)
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        fb()
    with torch.cuda.stream(s2):
        vit()
    cur.wait_stream(s1)
    cur.wait_stream(s2)


print(kind, ops.plan_info(plan))
print(f"fb alone   {timed(fb) * 1e3:8.1f} us")
print(f"vit alone  {timed(vit) * 1e3:8.1f} us")
print(f"both       {timed(both) * 1e3:8.1f} us")
