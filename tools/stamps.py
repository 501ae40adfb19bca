"""Diagnostic: per-segment cycles of one recursion step (HMM355_STAMP=1 build).
Build here:  python tools/stamps.py build      Run on the GPU box: python tools/stamps.py
Segments per step and wave: gather (barrier -> partials in VGPRs), compute (-> step result),
write (ds_write issued + retired), barrier (+ loop overhead + the per-16-step staging)."""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "ablate_libs", "libhmm355_stamp.so")
if sys.argv[1:] == ["build"]:
    sys.path.insert(0, os.path.dirname(HERE))
    from pytorch_hmm_amd import build_native as bn
    print(bn.build(force=True, defines=["HMM355_STAMP=1"], out=LIB))
    sys.exit(0)
import numpy as np
import torch
L = ctypes.CDLL(LIB)
P_, I, U, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_size_t
L.hmm355_fb_workspace_bytes.argtypes, L.hmm355_fb_workspace_bytes.restype = [I, I, I], S
L.hmm355_forward_backward_f32.argtypes = [P_, I, P_, P_, I, I, I, U, P_, P_, P_, P_, P_, P_, S, P_]
L.hmm355_viterbi_workspace_bytes.argtypes, L.hmm355_viterbi_workspace_bytes.restype = [I, I, I], S
L.hmm355_viterbi_f32.argtypes = [P_, I, P_, P_, I, I, I, P_, P_, P_, P_, S, P_]
dev = torch.device("cuda", 0)
B, T, N = int(os.environ.get("B", 32)), int(os.environ.get("T", 2000)), int(os.environ.get("N", 128))
NW = {64: 4, 128: 8, 256: 16}[128 if N > 64 and N <= 128 else (64 if N <= 64 else 256)]
obs = torch.softmax(torch.randn(B, T, N, device=dev), -1)
if os.environ.get("HMM355_DENSE") == "1":
    P = torch.rand(N, N, device=dev)
else:  # left-to-right 0.7 (the bench matrix): banded chains
    P = torch.zeros(N, N, device=dev); i = torch.arange(N - 1, device=dev)
    P[i, i] = 0.7; P[i, i + 1] = 0.3; P[N - 1, N - 1] = 1.0
lP = torch.log(P / P.sum(1, keepdim=True) + 1e-8); lp0 = torch.full((N,), -4.85, device=dev)
p = lambda t: ctypes.c_void_p(t.data_ptr())
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
post = torch.empty(B, T, N, device=dev); ll = torch.empty(B, device=dev); lr = torch.empty(B, device=dev)
ws = torch.empty(L.hmm355_fb_workspace_bytes(B, T, N), dtype=torch.uint8, device=dev)
states = torch.empty(B, T, dtype=torch.int64, device=dev); delta = torch.empty(B, T, N, device=dev); fin = torch.empty(B, device=dev)
wsv = torch.empty(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=dev)
names = ["gather", "compute", "write", "barrier"] if os.environ.get("HMM355_DENSE") == "1" else ["issue+reduce", "window+update", "block-end", "block-barrier"]


def report(tag, fn, nblocks):
    sym = getattr(L, f"hmm355_debug_stamps_{tag}")
    sym.argtypes = [P_, I]
    for _ in range(3):
        assert fn() == 0
    torch.cuda.synchronize()
    n = 512 * 16 * 8
    buf = (ctypes.c_ulonglong * n)()
    assert sym(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[: nblocks * NW].astype(np.float64)
    if os.environ.get("HMM355_DENSE") != "1":  # banded: the chain is wave 0 of each block
        a = a.reshape(nblocks, NW, 8)[:, :1].repeat(NW, axis=1).reshape(-1, 8)
    steps = np.maximum(a[:, 4], 1)
    seg = a[:, :4] / steps[:, None]
    clk = a[:, 6] / np.maximum(a[:, 7], 1) * 100.0
    print(f"[{tag}] cycles/step by segment (mean over waves):",
          {k: round(float(seg[:, i].mean()), 1) for i, k in enumerate(names)},
          "total/step", round(float((a[:, 5] / steps).mean()), 1), "clock MHz", round(float(np.median(clk)), 0))
    per_wave = seg.reshape(nblocks, NW, 4).mean(0)
    for w in range(NW):
        print(f"   wave {w}:", [round(float(x)) for x in per_wave[w]])


report("fb", lambda: L.hmm355_forward_backward_f32(p(obs), 0, p(lP), p(lp0), B, T, N, 1, p(post), None, None,
                                                     p(ll), p(lr), p(ws), ws.numel(), st), 2 * B)
report("vit", lambda: L.hmm355_viterbi_f32(p(obs), 0, p(lP), p(lp0), B, T, N, p(states), p(delta), p(fin),
                                             p(wsv), wsv.numel(), st), B)
