"""Diagnostic: HSMM walker phase cycles at the config-5 shape (build with HMM355_HSMM_STAMP:
  python -c "from pytorch_hmm_amd import build_native as bn; bn.build(defines=['HMM355_HSMM_STAMP'], out='tools/ablate_libs/libhmm355_hstamp.so')"
run on the GPU box: HMM355_LIB=tools/ablate_libs/libhmm355_hstamp.so python tools/hsmm_stamp.py)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pytorch_hmm_amd as ph
from pytorch_hmm_amd import _native

dev = torch.device("cuda", 0)
B, T, S, Dm, D = 16, 2000, 64, 40, 80
from pytorch_hmm_amd.hsmm import HSMMLayer
torch.manual_seed(0)
layer = HSMMLayer(S, D, max_duration=Dm).to(dev)
x = torch.randn(B, T, D, device=dev)
L = ctypes.CDLL(_native.LIB_PATH)
buf = (ctypes.c_ulonglong * 8)()
with torch.no_grad():
    for _ in range(2):
        layer.viterbi_decode_hsmm(x) if hasattr(layer, "viterbi_decode_hsmm") else layer(x)
    torch.cuda.synchronize()
    L.hmm355_diag_hsmm_stamp(buf)
    n = 5
    for _ in range(n):
        layer.viterbi_decode_hsmm(x) if hasattr(layer, "viterbi_decode_hsmm") else layer(x)
    torch.cuda.synchronize()
    L.hmm355_diag_hsmm_stamp(buf)
v = [x / n for x in buf]
segs = v[6]
names = ["emit/loop", "RT1 + state search", "RT2 (column, pcol)", "obs sums + d' search", "xb / tie / barrier"]
print(f"walk segments per call {segs:.0f} (per sequence {segs / B:.1f})")
for i, nm in enumerate(names):
    print(f"{nm:28s} {v[i] / max(segs, 1):8.0f} cycles per segment")
print(f"stitch: prologue {v[7] / B:8.0f} cycles per sequence, whole {v[5] / B:8.0f}")
