"""Diagnostic: cycles and shader clock of the banded chain waves (HMM355_STAMP=1 build,
recur.h band_chain), each op alone and both ops side by side on two streams.
Build here:  python tools/band_stamps.py build        Run on the GPU box: python tools/band_stamps.py [f]
(f: the work beside the chains on).  Per chain: cycles per step, cycles per step at the block
barriers (waiting for the helpers), and the clock (s_memtime cycles / s_memrealtime at 100 MHz)."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("STAMP_LIB", os.path.join(HERE, "ablate_libs", "libhmm355_stamp.so"))
if sys.argv[1:] == ["build"]:
    sys.path.insert(0, os.path.dirname(HERE))
    from pytorch_hmm_amd import build_native as bn
    print(bn.build(force=True, defines=["HMM355_STAMP=1"], out=LIB, sources=bn.RECURSION_SOURCES))
    sys.exit(0)
import numpy as np
import torch

FOLLOW = len(sys.argv) > 1 and "f" in sys.argv[1]
sys.argv = [sys.argv[0]] + [LIB + ":" + (sys.argv[1] if len(sys.argv) > 1 else "")]
sys.path.insert(0, HERE)
import time_follow as tf  # noqa: E402  (builds the inputs and the two op closures)

L = ctypes.CDLL(LIB)
fb, vit = tf.make(sys.argv[1])
NW = 16  # stamp slots per workgroup (recur.h band_chain / rec_band, follow.h)


def raw(tag, nblk):
    sym = getattr(L, f"hmm355_debug_stamps_{tag}")
    sym.argtypes = [ctypes.c_void_p, ctypes.c_int]
    n = 512 * 16 * 8
    buf = (ctypes.c_ulonglong * n)()
    assert sym(buf, n) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(-1, NW, 8)[:nblk, 0].astype(np.float64)


def timeline(name, chains, fol, nstamp):
    """real-time (us) of each chain's end, its final publish, and its follower's stamps,
    from the earliest chain start; medians over the sequences"""
    t0 = chains[:, 0].min()
    med = lambda x: float(np.median(x))
    msg = (f"  {name:10s} chain start {med(chains[:, 0] - t0) / 100:6.1f} end {med(chains[:, 1] - t0) / 100:6.1f}"
           f" (max {(chains[:, 1] - t0).max() / 100:6.1f}) publish {med(chains[:, 2] - t0) / 100:6.1f}")
    if fol is not None:
        msg += "  follower " + " ".join(f"{med(fol[:, k] - t0) / 100:6.1f}" for k in range(nstamp))
        msg += f" (last exit {(fol[:, nstamp - 1] - t0).max() / 100:6.1f})"
    print(msg, flush=True)


def helpers(name, tag, nblk, waves):
    """cycles per block of the staging helpers' work and their wait at the block barrier"""
    sym = getattr(L, f"hmm355_debug_stamps_{tag}")
    sym.argtypes = [ctypes.c_void_p, ctypes.c_int]
    n = 512 * 16 * 8
    buf = (ctypes.c_ulonglong * n)()
    assert sym(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, NW, 8)[:nblk].astype(np.float64)
    for w in waves:
        nb = np.maximum(a[:, w, 4], 1)
        print(f"  {name:10s} helper wave {w:2d}: work/block {np.mean(a[:, w, 0] / nb):7.0f}  wait/block {np.mean(a[:, w, 1] / nb):7.0f}")


def read(tag, nblk):
    sym = getattr(L, f"hmm355_debug_stamps_{tag}")
    sym.argtypes = [ctypes.c_void_p, ctypes.c_int]
    n = 512 * 16 * 8
    buf = (ctypes.c_ulonglong * n)()
    assert sym(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[: nblk * NW].reshape(nblk, NW, 8)[:, 0].astype(np.float64)
    return a


def show(name, a):
    steps = np.maximum(a[:, 4], 1)
    tot = a[:, 5] / steps
    bar = a[:, 3] / steps
    clk = a[:, 6] / np.maximum(a[:, 7], 1) * 100.0
    print(f"  {name:10s} cycles/step {tot.mean():7.1f} (max {tot.max():7.1f})  barrier/step {bar.mean():6.1f}"
          f"  clock MHz {np.median(clk):6.0f} (min {clk.min():6.0f})  chain us {np.median(a[:, 7]) / 100:7.1f}", flush=True)


B = tf.B
cur = torch.cuda.current_stream(tf.dev)
for mode in ("fb", "vit", "both"):
    for _ in range(3):
        if mode == "fb":
            fb(cur)
        elif mode == "vit":
            vit(cur)
        else:
            tf.both(fb, vit)
    torch.cuda.synchronize()
    print(mode, flush=True)
    fl = FOLLOW
    if mode in ("fb", "both"):
        a = read("fb", 2 * B)
        show("alpha", a[0::2])
        show("beta", a[1::2])
        helpers("fb", "fb", 2 * B, (1, 2, 3))
        r = raw("fb", 4 * B)
        ch = r[:2 * B].reshape(B, 2, 8)
        late = np.where(ch[:, 0, 1:2] >= ch[:, 1, 1:2], ch[:, 0], ch[:, 1])  # the later chain of each pair
        timeline("fb", late, r[2 * B:3 * B] if fl else None, 3)
        if fl:
            timeline("fb f1", late, r[3 * B:], 3)
    if mode in ("vit", "both"):
        show("viterbi", read("vit", B))
        helpers("vit", "vit", B, (1, 2, 3, 9, 10, 11))
        r = raw("vit", 2 * B)
        timeline("vit", r[:B], r[B:] if fl else None, 4)
