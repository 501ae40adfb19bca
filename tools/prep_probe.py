"""Diagnostic: per-kernel durations of one Viterbi call on the l2r matrix for ablation libs
(run under rocprofv3 --kernel-trace).  usage: python tools/prep_probe.py LIB [LIB...]"""
import ctypes, sys, torch
dev = torch.device("cuda", 0)
B, T, N = 32, 2000, 128
obs = torch.softmax(torch.randn(B, T, N, device=dev), -1)
P = torch.zeros(N, N, device=dev); i = torch.arange(N - 1, device=dev)
P[i, i] = 0.7; P[i, i + 1] = 0.3; P[N - 1, N - 1] = 1.0
lP = torch.log(P + 1e-8); lp0 = torch.full((N,), -4.85, device=dev)
states = torch.empty(B, T, dtype=torch.int64, device=dev); delta = torch.empty(B, T, N, device=dev); fin = torch.empty(B, device=dev)
p = lambda t: ctypes.c_void_p(t.data_ptr())
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for lib in sys.argv[1:]:
    L = ctypes.CDLL(lib)
    P_, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.hmm355_viterbi_workspace_bytes.argtypes, L.hmm355_viterbi_workspace_bytes.restype = [I, I, I], S
    L.hmm355_viterbi_f32.argtypes = [P_, I, P_, P_, I, I, I, P_, P_, P_, P_, S, P_]
    ws = torch.zeros(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=dev)  # zero desc = dense if prep is ablated
    for _ in range(5):
        L.hmm355_viterbi_f32(p(obs), 0, p(lP), p(lp0), B, T, N, p(states), p(delta), p(fin), p(ws), ws.numel(), st)
    torch.cuda.synchronize()
    print("done", lib)
