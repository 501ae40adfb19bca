"""Diagnostic: the north-star ops through the raw C ABI of one or more library builds, timed
alone and side by side on two streams (the bench's pattern), interleaved in one process.

    python tools/time_follow.py LIB[:FLAGS] ...      FLAGS: f = followers (FB_PLAN_BANDED /
                                                     VIT_PLAN_BANDED), p = FB pair kernel
e.g. python tools/time_follow.py pytorch_hmm_amd/lib/libhmm355.so:f pytorch_hmm_amd/lib/libhmm355.so
     tools/ablate_libs/libhmm355_r5.so
B=32, T=2000, N=128, left_to_right(0.7), softmax emissions (OBS_PROB), FB mask 7."""
import ctypes
import os
import sys

import torch

B, T, N = int(os.environ.get("B", 32)), int(os.environ.get("T", 2000)), int(os.environ.get("N", 128))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1234)
obs = torch.softmax(torch.randn(B, T, N, device=dev, generator=g), -1)
i = torch.arange(N - 1, device=dev)
P = torch.zeros(N, N, device=dev)
P[i, i] = 0.7
P[i, i + 1] = 0.3
P[N - 1, N - 1] = 1.0
lP = torch.log(P / P.sum(1, keepdim=True) + 1e-8)
lp0 = torch.log(torch.full((N,), 1.0 / N, device=dev) + 1e-8)
Pv, I, U, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_size_t
p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
s_fb, s_vit = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def make(spec):
    path, _, fl = spec.partition(":")
    L = ctypes.CDLL(path)
    L.hmm355_fb_workspace_bytes.argtypes, L.hmm355_fb_workspace_bytes.restype = [I, I, I], S
    L.hmm355_viterbi_workspace_bytes.argtypes, L.hmm355_viterbi_workspace_bytes.restype = [I, I, I], S
    L.hmm355_plan_bytes.argtypes, L.hmm355_plan_bytes.restype = [I], S
    L.hmm355_plan_f32.argtypes, L.hmm355_plan_f32.restype = [Pv, I, Pv, Pv], I
    L.hmm355_forward_backward_plan_f32.argtypes = [Pv, I, Pv, Pv, Pv, Pv, I, I, I, U, Pv, Pv, Pv, Pv, Pv, Pv, S, Pv]
    L.hmm355_viterbi_plan_ex_f32.argtypes = [Pv, I, Pv, Pv, Pv, U, I, I, I, Pv, Pv, Pv, Pv, S, Pv]
    plan = torch.empty(L.hmm355_plan_bytes(N), dtype=torch.uint8, device=dev)
    assert L.hmm355_plan_f32(p(lP), N, p(plan), None) == 0
    torch.cuda.synchronize()
    ws_f = torch.empty(L.hmm355_fb_workspace_bytes(B, T, N), dtype=torch.uint8, device=dev)
    ws_v = torch.empty(L.hmm355_viterbi_workspace_bytes(B, T, N), dtype=torch.uint8, device=dev)
    post, fwd, bwd = (torch.empty(B, T, N, device=dev) for _ in range(3))
    ll, lr, fin = (torch.empty(B, device=dev) for _ in range(3))
    states = torch.empty(B, T, dtype=torch.int64, device=dev)
    delta = torch.empty(B, T, N, device=dev)
    mask = 7 | (0x200 if "f" in fl else 0) | (0x100 if "p" in fl else 0)
    vflags = 0x1 if "f" in fl else 0

    def fb(stream):
        st = ctypes.c_void_p(stream.cuda_stream)
        rc = L.hmm355_forward_backward_plan_f32(p(obs), 0, p(lP), p(lp0), p(plan), None, B, T, N, mask, p(post), p(fwd),
                                                p(bwd), p(ll), p(lr), p(ws_f), ws_f.numel(), st)
        assert rc == 0, rc

    def vit(stream):
        st = ctypes.c_void_p(stream.cuda_stream)
        rc = L.hmm355_viterbi_plan_ex_f32(p(obs), 0, p(lP), p(lp0), p(plan), vflags, B, T, N, p(states), p(delta),
                                          p(fin), p(ws_v), ws_v.numel(), st)
        assert rc == 0, rc
    return fb, vit


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def both(fb, vit):
    cur = torch.cuda.current_stream(dev)
    s_fb.wait_stream(cur)
    s_vit.wait_stream(cur)
    fb(s_fb)
    vit(s_vit)
    cur.wait_stream(s_fb)
    cur.wait_stream(s_vit)


if __name__ == "__main__":
    specs = sys.argv[1:]
    runs = {s: make(s) for s in specs}
    res = {s: {"fb": [], "vit": [], "both": []} for s in specs}
    for rnd in range(3):
        for s, (fb, vit) in runs.items():
            cur = torch.cuda.current_stream(dev)
            res[s]["fb"].append(timed(lambda: fb(cur)))
            res[s]["vit"].append(timed(lambda: vit(cur)))
            res[s]["both"].append(timed(lambda: both(fb, vit)))
    for s in specs:
        r = res[s]
        print(f"{s:60s} fb {min(r['fb']):7.1f}  vit {min(r['vit']):7.1f}  both {min(r['both']):7.1f} us", flush=True)
