"""Diagnostic A/B of recursion-kernel variants (compile-time defines) in ONE process, interleaved
rounds.  Build here:   AB="m0:HMM355_FBSCALE=0 m3:HMM355_FBSCALE=3" python tools/ab.py build
Run on the GPU box:    AB="m0 m3" python tools/ab.py run
Each variant is a library with the forward-backward / Viterbi sources only
(build_native.RECURSION_SOURCES) under tools/ablate_libs/.  Times per op (HIP events, median of 5
rounds of 3 calls) on a random dense matrix, a few-steps-trained-like dense matrix and the
north-star left-to-right matrix; B, T, N from the environment (32, 2000, 128)."""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
SPEC = os.environ.get("AB", "").split()


def libpath(name):
    return os.path.join(HERE, "ablate_libs", f"libhmm355_ab_{name}.so")


if sys.argv[1] == "build":
    from pytorch_hmm_amd import build_native as bn
    for item in SPEC:
        name, _, defs = item.partition(":")
        print(bn.build(force=False, defines=[d for d in defs.split(",") if d], out=libpath(name),
                       sources=bn.RECURSION_SOURCES), flush=True)
    sys.exit(0)

import torch
names = [s.partition(":")[0] for s in SPEC]
dev = torch.device("cuda", 0)
B, T, N = int(os.environ.get("B", 32)), int(os.environ.get("T", 2000)), int(os.environ.get("N", 128))
g = torch.Generator(device=dev).manual_seed(0)
obs = torch.softmax(torch.randn(B, T, N, device=dev, generator=g), -1)
mats = {"random": torch.rand(N, N, device=dev, generator=g)}
i = torch.arange(N - 1, device=dev)
l2r = torch.zeros(N, N, device=dev); l2r[i, i] = 0.7; l2r[i, i + 1] = 0.3; l2r[N - 1, N - 1] = 1.0
mats["l2r"] = l2r
P_, I, U, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_size_t
libs = {}
for n in names:
    L = ctypes.CDLL(libpath(n))
    L.hmm355_fb_workspace_bytes.argtypes, L.hmm355_fb_workspace_bytes.restype = [I, I, I], S
    L.hmm355_forward_backward_f32.argtypes = [P_, I, P_, P_, I, I, I, U, P_, P_, P_, P_, P_, P_, S, P_]
    L.hmm355_viterbi_workspace_bytes.argtypes, L.hmm355_viterbi_workspace_bytes.restype = [I, I, I], S
    L.hmm355_viterbi_f32.argtypes = [P_, I, P_, P_, I, I, I, P_, P_, P_, P_, S, P_]
    libs[n] = L
post = torch.empty(B, T, N, device=dev); fwd = torch.empty_like(post); bwd = torch.empty_like(post)
ll = torch.empty(B, device=dev); lr = torch.empty(B, device=dev)
ws = torch.empty(max(L.hmm355_fb_workspace_bytes(B, T, N) for L in libs.values()), dtype=torch.uint8, device=dev)
states = torch.empty(B, T, dtype=torch.int64, device=dev); delta = torch.empty(B, T, N, device=dev)
fin = torch.empty(B, device=dev)
wsv = torch.empty(max(L.hmm355_viterbi_workspace_bytes(B, T, N) for L in libs.values()), dtype=torch.uint8, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
p = lambda t: ctypes.c_void_p(t.data_ptr())
lp0 = torch.full((N,), -4.85, device=dev)
for mname, P in mats.items():
    lP = torch.log(P / P.sum(1, keepdim=True) + 1e-8)
    fb = lambda L: L.hmm355_forward_backward_f32(p(obs), 0, p(lP), p(lp0), B, T, N, int(os.environ.get("FBMASK", 7)), p(post), p(fwd), p(bwd),
                                                 p(ll), p(lr), p(ws), ws.numel(), st)
    vit = lambda L: L.hmm355_viterbi_f32(p(obs), 0, p(lP), p(lp0), B, T, N, p(states), p(delta), p(fin), p(wsv),
                                         wsv.numel(), st)
    res = {n: {"fb": [], "vit": []} for n in names}
    outs = {}
    for rnd in range(5):
        for n in names:
            for op, fn in (("fb", fb), ("vit", vit)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                assert fn(libs[n]) == 0
                e0.record()
                for _ in range(3):
                    assert fn(libs[n]) == 0
                e1.record()
                torch.cuda.synchronize()
                res[n][op].append(e0.elapsed_time(e1) / 3)
            if rnd == 0:
                outs[n] = (post.clone(), ll.clone(), states.clone())
    ref = outs[names[0]]
    for n in names:
        f = sorted(res[n]["fb"])[2]
        v = sorted(res[n]["vit"])[2]
        d = (outs[n][0] - ref[0]).abs().max().item()
        dl = ((outs[n][1] - ref[1]).abs() / ref[1].abs()).max().item()
        same = torch.equal(outs[n][2], ref[2])
        print(f"[{mname}] {n:10s} fb {f * 1e3:8.1f} us ({f * 1e6 / T:6.1f} ns/step)  vit {v * 1e3:8.1f} us  "
              f"| post max|d| {d:.2e} loglik rel {dl:.2e} states {'=' if same else 'DIFF'}", flush=True)
