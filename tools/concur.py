"""Diagnostic: the forward-backward and Viterbi ops alone and side by side on two streams (the
bench step), with the psi followers on and off, through the product C ABI with a plan.
Run on the GPU box: python tools/concur.py  (MAT=random|l2r|trained-like, B/T/N from the env)."""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import torch
import pytorch_hmm_amd._native as nat
from pytorch_hmm_amd import ops
dev = torch.device("cuda", 0)
B, T, N = int(os.environ.get("B", 32)), int(os.environ.get("T", 2000)), int(os.environ.get("N", 128))
gp = torch.Generator().manual_seed(4321)
mat = os.environ.get("MAT", "random")
if mat == "random":
    P = torch.softmax(torch.randn(N, N, generator=gp), dim=-1)
else:
    P = torch.zeros(N, N); i = torch.arange(N - 1); P[i, i] = 0.7; P[i, i + 1] = 0.3; P[N - 1, N - 1] = 1.0
lP = torch.log(P / P.sum(1, keepdim=True) + 1e-8).to(dev)
lp0 = torch.full((N,), -4.85, device=dev)
g = torch.Generator(device=dev).manual_seed(1234)
obs = torch.softmax(torch.randn(B, T, N, device=dev, generator=g), -1)
plan = ops.make_plan(lP)
sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def fb():
    return ops.forward_backward(obs, lP, lp0, ops.OBS_PROB, 7, plan)


def vit():
    return ops.viterbi(obs, lP, lp0, ops.OBS_PROB, plan)


def timed(which, reps=5):
    """median over reps of the per-op HIP-event times when the listed ops run together"""
    res = {n: [] for n in which}
    for r in range(reps + 1):
        ev = {}
        for n in which:
            s_ = sA if n == "fb" else sB
            with torch.cuda.stream(s_):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s_)
                for _ in range(3):
                    (fb if n == "fb" else vit)()
                e1.record(s_)
                ev[n] = (e0, e1)
        torch.cuda.synchronize()
        if r:
            for n in which:
                res[n].append(ev[n][0].elapsed_time(ev[n][1]) / 3)
    return {n: sorted(v)[len(v) // 2] for n, v in res.items()}


for follow in ("0", "1"):
    os.environ["HMM355_VIT_FOLLOW"] = follow
    a = timed(["fb"]); b = timed(["vit"]); c = timed(["fb", "vit"])
    print(f"[{mat}] followers={follow}: fb alone {a['fb']*1e3:.1f} us, vit alone {b['vit']*1e3:.1f} us, "
          f"together fb {c['fb']*1e3:.1f} us vit {c['vit']*1e3:.1f} us", flush=True)
