"""Diagnostic: MixtureGaussianHMMLayer inference at BASELINE config 3 (B=32, T=2000, S=128,
C=4, D=80), the scorer and the decode in series vs ops.gmm_viterbi's overlap with several
slice schedules (one process, interleaved rounds, ms per call)."""
import sys
import torch
sys.path.insert(0, ".")
from pytorch_hmm_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
B, T, S, C, D = 32, 2000, 128, 4, 80
g = torch.Generator(device=dev).manual_seed(0)
means = torch.randn(S, C, D, device=dev, generator=g)
log_vars = 0.3 * torch.randn(S, C, D, device=dev, generator=g)
log_w = torch.log_softmax(torch.randn(S, C, device=dev, generator=g), -1)
lT = torch.log(torch.softmax(torch.randn(S, S, device=dev, generator=g), -1) + 1e-8)
init = torch.full((S,), -4.85, device=dev)
plan = ops.make_plan(lT)
x = torch.randn(B, T, D, device=dev, generator=g)
variants = {"series": dict(overlap=False)}
for ff, sf in ((64, 128), (128, 128), (128, 192), (128, 256), (192, 192), (256, 256)):
    variants[f"overlap {ff}/{sf}"] = dict(overlap=True, first_frames=ff, slice_frames=sf)


def timed(kw, n=10):
    for _ in range(2):
        ops.gmm_viterbi(x, means, log_vars, log_w, lT, init, plan, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        ops.gmm_viterbi(x, means, log_vars, log_w, lT, init, plan, **kw)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


res = {k: [] for k in variants}
for _ in range(3):
    for k, kw in variants.items():
        res[k].append(timed(kw))
for k, v in res.items():
    print(f"{k:22s} {min(v):.3f} ms", flush=True)
