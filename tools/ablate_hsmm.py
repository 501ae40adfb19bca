"""Diagnostic: time the HSMM segment-Viterbi kernels of ablation builds (HMM355_ABL bits,
csrc/hsmm.hip: 1 no per-step barrier, 1<<20 no predecessor phase, 1<<21 no slot work) in ONE
process, interleaved rounds.  Results are wrong by construction except ABL=0: timing only.
Build here: python tools/ablate_hsmm.py build   Run on the GPU box: python tools/ablate_hsmm.py run"""
import ctypes, os, subprocess, sys
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
VARIANTS = [int(v) for v in os.environ.get("ABL_VARIANTS", "0,1,1048576,2097152,3145729").split(",")]
OUT = os.path.join(HERE, "abl_hsmm")

def libpath(v):
    return os.path.join(OUT, f"libhsmm_abl{v}.so")

if sys.argv[1] == "build":
    os.makedirs(OUT, exist_ok=True)
    for v in VARIANTS:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
               "-fno-slp-vectorize", "-fno-honor-nans", "-Wno-unused-result", f"-DHMM355_ABL={v}",
               "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "pytorch_hmm_amd", "csrc", "hsmm.hip"),
               "-o", libpath(v)]
        subprocess.check_call(cmd)
        print(libpath(v))
    sys.exit(0)

import torch
dev = torch.device("cuda", 0)
B, T, S, Dm = (int(os.environ.get(k, d)) for k, d in (("B", 16), ("T", 2000), ("S", 64), ("DM", 40)))
g = torch.Generator(device="cpu").manual_seed(0)
if os.environ.get("C5"):  # config 5's tables: HSMMLayer(64,80,40) random init, randn features
    sys.path.insert(0, ROOT)
    import pytorch_hmm_amd as ph
    torch.manual_seed(0)
    layer = ph.HSMMLayer(S, 80, max_duration=Dm).to(dev)
    with torch.no_grad():
        lp = layer.get_observation_log_probs(torch.randn(B, T, 80, generator=g).to(dev)).contiguous()
        dur = torch.log(layer.get_duration_probabilities() + layer.eps)[:, :Dm].contiguous()
        logT = torch.log(layer.get_transition_matrix() + layer.eps).contiguous()
else:
    lp = (-(torch.rand(B, T, S, generator=g) * 40 + 80)).to(dev)
    dur = torch.log(torch.rand(S, Dm, generator=g) + 1e-8).to(dev)
    logT = torch.log(torch.rand(S, S, generator=g) + 1e-8).to(dev)
P_, I, Sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
p = lambda t: ctypes.c_void_p(t.data_ptr())
libs = {}
for v in VARIANTS:
    L = ctypes.CDLL(libpath(v))
    L.hmm355_hsmm_workspace_bytes.argtypes, L.hmm355_hsmm_workspace_bytes.restype = [I, I, I, I], Sz
    L.hmm355_hsmm_viterbi_f32.argtypes = [P_, P_, P_, I, I, I, I, P_, P_, P_, Sz, P_]
    libs[v] = L
ws = torch.empty(libs[VARIANTS[0]].hmm355_hsmm_workspace_bytes(B, T, S, Dm), dtype=torch.uint8, device=dev)
states = torch.empty(B, T, dtype=torch.int64, device=dev)
scores = torch.empty(B, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
res = {v: [] for v in VARIANTS}
for rnd in range(5):
    for v in VARIANTS:
        L = libs[v]
        call = lambda: L.hmm355_hsmm_viterbi_f32(p(lp), p(dur), p(logT), B, T, S, Dm, p(states), p(scores), p(ws), ws.numel(), st)
        assert call() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            call()
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 3)
for v in VARIANTS:
    m = sorted(res[v])[2]
    print(f"ABL={v:8d}  fwd+backtrace {m*1e3:8.1f} us ({m*1e6/T:6.1f} ns/step)")
if os.environ.get("SEGSTATS"):
    # serial segments walked by the stitch (chunked backtrace diagnostics), the last call's
    L = libs[VARIANTS[0]]
    assert L.hmm355_hsmm_viterbi_f32(p(lp), p(dur), p(logT), B, T, S, Dm, p(states), p(scores), p(ws), ws.numel(), st) == 0
    torch.cuda.synchronize()
    C = (T + 63) // 64
    al = lambda x: (x + 255) // 256 * 256
    n = B * T * S
    off = 2 * al(n * 4) + al(B * 8) + al(B * C * (64 + 256 + 2) * 16)
    cnt = ws[off:off + (B * C + 3 * B) * 4].view(torch.int32).cpu()
    segs = [int((states[i, 1:] != states[i, :-1]).sum()) + 1 for i in range(B)]
    print("segments per sequence", segs[:4], "stitch serial steps", cnt[B * C:B * C + B].tolist()[:8], "record counts", cnt[:C].tolist())
    print("stitch setup us", [x / 100 for x in cnt[B * C + B:B * C + 2 * B].tolist()[:8]], "loop us", [x / 100 for x in cnt[B * C + 2 * B:].tolist()[:8]])
