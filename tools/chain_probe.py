"""Diagnostic: one FB and one Viterbi call on the l2r (banded) matrix per library, B=32 T=2000
N=128 (run under rocprofv3 --kernel-trace).  usage: python tools/chain_probe.py LIB [LIB...]"""
import ctypes, sys, torch
dev = torch.device("cuda", 0)
B, T, N = 32, 2000, 128
obs = torch.softmax(torch.randn(B, T, N, device=dev), -1)
P = torch.zeros(N, N, device=dev); i = torch.arange(N - 1, device=dev)
P[i, i] = 0.7; P[i, i + 1] = 0.3; P[N - 1, N - 1] = 1.0
lP = torch.log(P + 1e-8); lp0 = torch.full((N,), -4.85, device=dev)
states = torch.empty(B, T, dtype=torch.int64, device=dev); delta = torch.empty(B, T, N, device=dev); fin = torch.empty(B, device=dev)
post = torch.empty(B, T, N, device=dev); ll = torch.empty(B, device=dev); lr = torch.empty(B, device=dev)
p = lambda t: ctypes.c_void_p(t.data_ptr())
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P_, I, U, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_size_t
for lib in sys.argv[1:]:
    L = ctypes.CDLL(lib)
    L.hmm355_viterbi_workspace_bytes.argtypes, L.hmm355_viterbi_workspace_bytes.restype = [I, I, I], S
    L.hmm355_viterbi_f32.argtypes = [P_, I, P_, P_, I, I, I, P_, P_, P_, P_, S, P_]
    L.hmm355_fb_workspace_bytes.argtypes, L.hmm355_fb_workspace_bytes.restype = [I, I, I], S
    L.hmm355_forward_backward_f32.argtypes = [P_, I, P_, P_, I, I, I, U, P_, P_, P_, P_, P_, P_, S, P_]
    wsv = torch.zeros(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=dev)
    wsf = torch.zeros(L.hmm355_fb_workspace_bytes(B, T, N), dtype=torch.uint8, device=dev)
    for _ in range(5):
        L.hmm355_viterbi_f32(p(obs), 0, p(lP), p(lp0), B, T, N, p(states), p(delta), p(fin), p(wsv), wsv.numel(), st)
        L.hmm355_forward_backward_f32(p(obs), 0, p(lP), p(lp0), B, T, N, 1, p(post), None, None, p(ll), p(lr), p(wsf), wsf.numel(), st)
    torch.cuda.synchronize()
    print("done", lib)
