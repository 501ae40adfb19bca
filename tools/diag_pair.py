"""Diagnostic: pair kernel (HMM355_FB_PAIR) vs the two-kernel path, per output and time step."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import hmm_oracle as O
from pytorch_hmm_amd import ops as o
B, T, N = 2, int(os.environ.get("T", 300)), 128
rng = np.random.default_rng(0)
lP, lp0 = O.hmm_params(O.left_to_right_matrix(N, 0.7))
obs = torch.softmax(torch.from_numpy(rng.standard_normal((B, T, N)).astype(np.float32)), -1).cuda()
lP, lp0 = lP.cuda(), lp0.cuda()
plan = o.make_plan(lP); plain = plan.clone()
a = o.forward_backward(obs, lP, lp0, o.OBS_PROB, 7, plan)
b = o.forward_backward(obs, lP, lp0, o.OBS_PROB, 7, plain)
for name, x, y in zip(["post", "fwd", "bwd", "ll", "lik"], a, b):
    x, y = x.cpu().numpy(), y.cpu().numpy()
    d = np.abs(x - y) > 1e-6 * np.abs(y) + 1e-30
    print(name, "bad", int(d.sum()), "of", d.size)
    if x.ndim == 3:
        bt = d.any(-1)
        for bb in range(B):
            ts = np.nonzero(bt[bb])[0]
            print("  b", bb, "bad t:", len(ts), ts[:8], ts[-8:] if len(ts) else "")
            if len(ts):
                t0 = ts[0]
                print("   t0", t0, "x", x[bb, t0, :6], "y", y[bb, t0, :6])
    else:
        print("  ", x, y)

# --- scratch rows: call the C ABI with our own workspaces
import ctypes
from pytorch_hmm_amd import _native as nat
L = nat.lib()
NP = 128
def call(mask, pl):
    ws = torch.zeros(L.hmm355_fb_workspace_bytes(B, T, N), dtype=torch.uint8, device="cuda")
    post = torch.zeros(B, T, N, device="cuda"); fw = torch.zeros_like(post); bw = torch.zeros_like(post)
    ll = torch.zeros(B, device="cuda"); lr = torch.zeros(B, device="cuda")
    rc = L.hmm355_forward_backward_plan_f32(nat.ptr(obs), 0, nat.ptr(lP), nat.ptr(lp0), nat.ptr(pl), None, B, T, N, mask,
        nat.ptr(post), nat.ptr(fw), nat.ptr(bw), nat.ptr(ll), nat.ptr(lr), nat.ptr(ws), ws.numel(), nat.stream_of(obs.device))
    torch.cuda.synchronize()
    fl = ws.view(torch.float32)
    U = fl[: B * T * NP].view(B, T, NP).cpu().numpy(); V = fl[B * T * NP: 2 * B * T * NP].view(B, T, NP).cpu().numpy()
    return rc, post.cpu().numpy(), U, V
rc1, p1, U1, V1 = call(7 | 0x100, plan)
rc2, p2, U2, V2 = call(7, plan)
print("rc", rc1, rc2)
nz = lambda A: np.nonzero(np.abs(A).sum(-1)[0])[0]
print("pair U rows written (b0):", len(nz(U1)), nz(U1)[:5], nz(U1)[-5:])
print("pair V rows written (b0):", len(nz(V1)), nz(V1)[:5], nz(V1)[-5:])
ru = nz(U1); rv = nz(V1)
print("U rows equal plain:", np.array_equal(U1[0, ru], U2[0, ru]), " V rows equal plain:", np.array_equal(V1[0, rv], V2[0, rv]))
# posterior from plain rows
def postf(u, v):
    p = (u / u.max(-1, keepdims=True)) * (v / v.max(-1, keepdims=True)); return p / p.sum(-1, keepdims=True)
pp = postf(U2[0], V2[0])[:, :N]
for t in [0, 1, 5, 100, 150, 200, 298, 299]:
    e = np.abs(p1[0, t] - pp[t]).max()
    # which V / U row would explain it
    cands = [(np.abs(p1[0, t] - postf(U2[0, t], V2[0, s])[:N]).max(), s) for s in range(T)]
    candu = [(np.abs(p1[0, t] - postf(U2[0, s], V2[0, t])[:N]).max(), s) for s in range(T)]
    print("t", t, "err", e, "best V row", min(cands), "best U row", min(candu))
