"""Diagnostic: time the recursion kernels of ablation builds (HMM355_ABL bits) in ONE
process, interleaved rounds (cdna guide §5.4 rule 24).  Build: python tools/ablate.py build
Run on the GPU box: python tools/ablate.py run"""
import ctypes, os, sys, json
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
VARIANTS = [int(v) for v in os.environ.get("ABL_VARIANTS", "0,1,2,31").split(",")]
LIBD = os.path.join(ROOT, "gpurun_out", "..", "tools", "ablate_libs")

def libpath(v):
    return os.path.join(HERE, "ablate_libs", f"libhmm355_abl{v}.so")

if sys.argv[1] == "build":
    from pytorch_hmm_amd import build_native as bn
    only = [int(a) for a in sys.argv[2:]] or VARIANTS
    for v in only:
        print(bn.build(force=True, defines=[f"HMM355_ABL={v}"], out=libpath(v)))
    sys.exit(0)

import torch
import pytorch_hmm_amd._native as nat
dev = torch.device("cuda", 0)
B, T, N = int(os.environ.get("B", 32)), int(os.environ.get("T", 2000)), int(os.environ.get("N", 128))
obs = torch.softmax(torch.randn(B, T, N, device=dev), -1)
if os.environ.get("MAT") == "l2r":   # the BASELINE matrix (banded chains)
    from pytorch_hmm_amd.utils import create_left_to_right_matrix
    P = create_left_to_right_matrix(N, 0.7).to(dev)
else:
    P = torch.rand(N, N, device=dev)
lP = torch.log(P / P.sum(1, keepdim=True) + 1e-8); lp0 = torch.full((N,), -4.85, device=dev)
libs = {}
for v in VARIANTS:
    L = ctypes.CDLL(libpath(v))
    nat_L = nat.lib  # reuse argtypes by copying
    P_, I, U, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_size_t
    L.hmm355_fb_workspace_bytes.argtypes, L.hmm355_fb_workspace_bytes.restype = [I, I, I], S
    L.hmm355_forward_backward_f32.argtypes = [P_, I, P_, P_, I, I, I, U, P_, P_, P_, P_, P_, P_, S, P_]
    L.hmm355_viterbi_workspace_bytes.argtypes, L.hmm355_viterbi_workspace_bytes.restype = [I, I, I], S
    L.hmm355_viterbi_f32.argtypes = [P_, I, P_, P_, I, I, I, P_, P_, P_, P_, S, P_]
    libs[v] = L
post = torch.empty(B, T, N, device=dev); fwd = torch.empty_like(post); bwd = torch.empty_like(post)
ll = torch.empty(B, device=dev); lr = torch.empty(B, device=dev)
ws = torch.empty(max(L.hmm355_fb_workspace_bytes(B, T, N) for L in libs.values()), dtype=torch.uint8, device=dev)
states = torch.empty(B, T, dtype=torch.int64, device=dev); delta = torch.empty(B, T, N, device=dev); fin = torch.empty(B, device=dev)
wsv = torch.empty(max(L.hmm355_viterbi_workspace_bytes(B, T, N) for L in libs.values()), dtype=torch.uint8, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
p = lambda t: ctypes.c_void_p(t.data_ptr())
def fb(L):
    return L.hmm355_forward_backward_f32(p(obs), 0, p(lP), p(lp0), B, T, N, 7, p(post), p(fwd), p(bwd), p(ll), p(lr), p(ws), ws.numel(), st)
def vit(L):
    return L.hmm355_viterbi_f32(p(obs), 0, p(lP), p(lp0), B, T, N, p(states), p(delta), p(fin), p(wsv), wsv.numel(), st)
res = {v: {"fb": [], "vit": []} for v in VARIANTS}
for rnd in range(5):
    for v in VARIANTS:
        for name, fn in (("fb", fb), ("vit", vit)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn(libs[v]); e0.record(); 
            for _ in range(3): assert fn(libs[v]) == 0
            e1.record(); torch.cuda.synchronize()
            res[v][name].append(e0.elapsed_time(e1) / 3)
for v in VARIANTS:
    fbm = sorted(res[v]["fb"])[2]; vm = sorted(res[v]["vit"])[2]
    print(f"ABL={v:3d}  fb {fbm*1e3:8.1f} us ({fbm*1e6/T:6.1f} ns/step)   vit {vm*1e3:8.1f} us ({vm*1e6/T:6.1f} ns/step)")
