"""Diagnostic: HSMM decode time of the register-slot kernels vs the general form
(csrc/hsmm_wide.hip, HMM355_HSMM_WIDE=1 forces it) on the GPU.  python tools/time_hsmm_wide.py"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_hmm_amd import ops
dev = torch.device("cuda", 0)
CASES = [(16, 2000, 64, 40, "0"), (16, 2000, 64, 40, "1"), (16, 2000, 200, 50, "0"),
         (16, 2000, 512, 64, "0"), (4, 2000, 64, 400, "0")]
if os.environ.get("EDGE") == "1":   # the register form's edge (Dmax 71) and the general form above it
    CASES = [(16, 2000, 64, 71, "0"), (16, 2000, 64, 72, "0"), (16, 2000, 64, 100, "0"), (16, 2000, 64, 127, "0"),
             (32, 2000, 64, 71, "0"), (32, 2000, 64, 100, "0")]
for B, T, S, Dm, force in CASES:
    os.environ["HMM355_HSMM_WIDE"] = force
    g = torch.Generator(device=dev).manual_seed(0)
    lp = -(torch.rand(B, T, S, device=dev, generator=g) * 40 + 80)
    dur = torch.log(torch.rand(S, Dm, device=dev, generator=g) + 1e-8)
    logT = torch.log(torch.rand(S, S, device=dev, generator=g) + 1e-8)
    ops.hsmm_viterbi(lp, dur, logT)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        ops.hsmm_viterbi(lp, dur, logT)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    wsb = ops.nat.lib().hmm355_hsmm_workspace_bytes(B, T, S, Dm)
    print(f"B={B} T={T} S={S} Dmax={Dm} wide={'forced' if force == '1' else 'auto'}: {ms:.2f} ms/decode, "
          f"{B * T / ms / 1e3:.3f} M frames/s, workspace {wsb / 2**20:.1f} MiB", flush=True)
