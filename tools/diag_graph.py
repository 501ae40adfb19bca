"""Diagnostic: forward_backward with posterior followers captured into two HIP graphs (own
workspaces and outputs), replayed alternately with different inputs."""
import ctypes
import sys
sys.path.insert(0, ".")
import torch
import pytorch_hmm_amd as ph
from pytorch_hmm_amd import ops, _native as nat

dev = torch.device("cuda", 0)
B, T, N = 8, 600, 128
hmm = ph.HMMPyTorch(ph.create_left_to_right_matrix(N, 0.7))
lP, lp0, plan = hmm._device_params(dev)
L = nat.lib()
p = nat.ptr
g = torch.Generator(device=dev).manual_seed(3)
base = torch.softmax(torch.randn(B, T, N, device=dev, generator=g), -1)
obs = base.clone()
nb = L.hmm355_fb_workspace_bytes(B, T, N)
cnt_bytes = (2 * B * 128 + 255) // 256 * 256
ws = [torch.zeros(nb, dtype=torch.uint8, device=dev) for _ in range(2)]
post = [torch.zeros(B, T, N, device=dev) for _ in range(2)]
ll = [torch.zeros(B, device=dev) for _ in range(2)]
lr = [torch.zeros(B, device=dev) for _ in range(2)]
mask = ops.FB_POSTERIOR | nat.FB_PLAN_BANDED


def call(i):
    rc = L.hmm355_forward_backward_plan_f32(p(obs), ops.OBS_PROB, p(lP), p(lp0), p(plan), None, B, T, N, mask,
                                            p(post[i]), None, None, p(ll[i]), p(lr[i]), p(ws[i]), nb,
                                            nat.stream_of(dev))
    assert rc == 0, rc


def counts(i):
    c = ws[i][nb - cnt_bytes:].view(torch.int32)[: 2 * B * 32].view(2 * B, 32)[:, 0]
    return c.tolist()


s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(s):
    call(0)
    call(1)
torch.cuda.synchronize()
graphs = []
for i in range(2):
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        call(i)
    graphs.append(gr)
torch.cuda.synchronize()
for k in range(6):
    i = k % 2
    x = base.clone()
    x[:, :, k % N] += 0.5 + 0.1 * k
    obs.copy_(x)
    torch.cuda.synchronize()
    before = counts(i)
    post[i].fill_(-7.0)
    ll[i].fill_(-7.0)
    ws[i][nb - cnt_bytes:].fill_(0)
    torch.cuda.synchronize()
    graphs[i].replay()
    torch.cuda.synchronize()
    r = ops.forward_backward(obs, lP, lp0, ops.OBS_PROB, 1, plan, follow=False)
    ref = r[0]
    torch.cuda.synchronize()
    d = float((post[i] - ref).abs().max())
    untouched = int((post[i] == -7.0).all(-1).sum())
    print(f"step {k} slot {i}: maxdiff {d:.3g} untouched rows {untouched} loglik diff {float((ll[i] - r[3]).abs().max()):.3g}"
          f" counts before {before[:4]} after {counts(i)[:4]}", flush=True)
