"""Build libhmm355.so (the gfx950 HIP kernels + C ABI) in-tree with hipcc.

    python -m pytorch_hmm_amd.build_native      (or __graft_entry__.build())

The shared library lands in pytorch_hmm_amd/lib/ so it travels with the repository
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libhmm355.so")
SOURCES = ["capi.hip", "fb.hip", "fb_np64.hip", "fb_np128.hip", "fb_np256.hip", "viterbi.hip", "vit_np64.hip",
           "vit_np128.hip", "vit_np256.hip", "gmm.hip", "hsmm.hip", "hsmm_wide.hip", "tv.hip", "semimarkov.hip", "stream.hip", "adjoint.hip"]
ARCH = os.environ.get("HMM355_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fno-slp-vectorize", "-fno-honor-nans",
         "-Wno-unused-result", "-I" + os.path.join(HERE, "..", "include")]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


# the sources of the forward-backward / Viterbi entry points alone (diagnostic A/B builds, tools/ab.py)
RECURSION_SOURCES = ["capi.hip", "fb.hip", "fb_np64.hip", "fb_np128.hip", "fb_np256.hip", "viterbi.hip",
                     "vit_np64.hip", "vit_np128.hip", "vit_np256.hip"]


def build(force=False, verbose=False, defines=(), out=None, sources=None):
    """Compile csrc/*.hip into `out` (default pytorch_hmm_amd/lib/libhmm355.so).
    `defines` (e.g. ["HMM355_ABL=2"]) and `sources` (a subset of SOURCES) are for diagnostic
    builds only."""
    lib = out or LIB
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    srcs = [s for s in (sources or SOURCES) if os.path.exists(os.path.join(CSRC, s))]
    # every header the sources include (csrc/*.h and the public header) is a dependency
    deps = ([os.path.join(CSRC, s) for s in srcs] + sorted(glob.glob(os.path.join(CSRC, "*.h"))) +
            [os.path.join(HERE, "..", "include", "hmm355.h"), os.path.abspath(__file__)])
    if not force and os.path.exists(lib):
        lt = os.path.getmtime(lib)
        if all(os.path.getmtime(d) <= lt for d in deps if os.path.exists(d)):
            return LIB
    hipcc = _hipcc()
    # objects are reused only under the same flags, defines and target (a hash in the dir name)
    import hashlib
    fh = hashlib.sha256("\0".join([*FLAGS, *defines, ARCH]).encode()).hexdigest()[:12]
    tag = os.path.splitext(os.path.basename(lib))[0] + "-" + fh
    objdir = os.path.join(os.path.dirname(lib), "obj", tag)
    os.makedirs(objdir, exist_ok=True)

    def includes(path, seen):
        """the quoted #includes of `path`, transitively (csrc headers and the public header)"""
        with open(path) as f:
            for line in f:
                t = line.strip()
                if t.startswith("#include \""):
                    inc = os.path.normpath(os.path.join(os.path.dirname(path), t.split('"')[1]))
                    if inc not in seen and os.path.exists(inc):
                        seen.add(inc)
                        includes(inc, seen)
        return seen

    this = os.path.abspath(__file__)

    def compile_one(s):
        obj = os.path.join(objdir, s.replace(".hip", ".o"))
        src = os.path.join(CSRC, s)
        # an object newer than its source, the headers it includes and this script is reused
        newest = max(os.path.getmtime(d) for d in includes(src, {src, this}))
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest:
            return obj
        cmd = [hipcc, *FLAGS, *["-D" + d for d in defines], "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = lib + ".tmp"
    subprocess.run([hipcc, "-shared", f"--offload-arch={ARCH}", "-o", tmp, *objs], check=True)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
