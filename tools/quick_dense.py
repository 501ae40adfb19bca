import os, sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
os.environ["HMM355_DENSE"] = "1"
from pytorch_hmm_amd import ops
from oracle import hmm_oracle as O
dev = torch.device("cuda", 0)
for N, T in ((128, 100), (64, 37), (100, 2000)):
    rng = np.random.default_rng(N + T)
    P = torch.from_numpy(rng.random((N, N), dtype=np.float32))
    lP, lp0 = O.hmm_params(P)
    lo = np.log(rng.random((3, T, N), dtype=np.float32) + np.float32(1e-3)).astype(np.float32)
    s, d, f = ops.viterbi(torch.from_numpy(lo).to(dev), lP.to(dev), lp0.to(dev), ops.OBS_LOG, None)
    torch.cuda.synchronize()
    cs, cd, _ = O.c_viterbi(lo, lP.numpy(), lp0.numpy())
    print("vit", N, T, np.array_equal(s.cpu().numpy(), cs), np.array_equal(d.cpu().numpy(), cd), flush=True)
    out = ops.forward_backward(torch.from_numpy(lo).to(dev), lP.to(dev), lp0.to(dev), ops.OBS_LOG, 7, None)
    torch.cuda.synchronize()
    la, lb, post, ll = O.c_fb64(lo, lP.numpy(), lp0.numpy())
    print("fb", N, T, float(np.abs(out[0].cpu().numpy() - post).max()), flush=True)
