"""CPU: the C ABI library (pytorch_hmm_amd/lib/libhmm355.so, cross-compiled for gfx950) loads
without a GPU, exports exactly what include/hmm355.h declares, and rejects bad arguments
with the documented status codes before launching anything (no compute calls here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hmm355.h")


@pytest.fixture(scope="module")
def L():
    from pytorch_hmm_amd import _native as nat
    if not os.path.exists(nat.LIB_PATH):
        from pytorch_hmm_amd import build_native
        build_native.build()
    return nat.lib()


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hmm355_[a-z0-9_]+)\s*\(", src)))


def header_defines():
    return dict((m.group(1), int(m.group(2).rstrip("u"), 0))
                for m in re.finditer(r"#define\s+(HMM355_[A-Z0-9_]+)\s+\(?(-?(?:0x[0-9a-fA-F]+|\d+)u?)\)?",
                                     open(HEADER).read()))


def test_exports_match_header(L):
    from pytorch_hmm_amd import _native as nat
    declared = header_functions()
    assert declared == sorted(nat.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", nat.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = sorted(set(re.findall(r"\b(hmm355_[a-z0-9_]+)\b", out)) - {"hmm355_debug_stamps_fb", "hmm355_debug_stamps_vit"})
    assert exported == declared
    for name in declared:
        assert hasattr(L, name)


def test_constants_match_header():
    from pytorch_hmm_amd import _native as nat
    d = header_defines()
    assert d["HMM355_OBS_PROB"] == nat.OBS_PROB and d["HMM355_OBS_LOG"] == nat.OBS_LOG
    assert (d["HMM355_FB_POSTERIOR"], d["HMM355_FB_FORWARD"], d["HMM355_FB_BACKWARD"]) == \
        (nat.FB_POSTERIOR, nat.FB_FORWARD, nat.FB_BACKWARD)
    assert d["HMM355_FB_PAIR"] == nat.FB_PAIR == 0x100
    assert d["HMM355_FB_PLAN_BANDED"] == nat.FB_PLAN_BANDED
    assert (d["HMM355_VIT_PLAN_BANDED"], d["HMM355_VIT_PLAN_DENSE"]) == (nat.VIT_PLAN_BANDED, nat.VIT_PLAN_DENSE)
    assert d["HMM355_PLAN_DENSE"] == nat.PLAN_DENSE
    assert (d["HMM355_FORM_GENERAL"], d["HMM355_FORM_SERIAL_WALK"]) == (nat.FORM_GENERAL, nat.FORM_SERIAL_WALK)
    assert d["HMM355_OK"] == 0


def test_version_and_strerror(L):
    assert L.hmm355_version() > 0
    d = header_defines()
    for code in ("HMM355_E_ARG", "HMM355_E_STATES", "HMM355_E_SHAPE", "HMM355_E_WORKSPACE", "HMM355_E_DURATION"):
        assert L.hmm355_strerror(d[code]).decode()
    assert L.hmm355_strerror(0).decode()


def test_workspace_sizes(L):
    B, T, N = 32, 2000, 128
    fb = L.hmm355_fb_workspace_bytes(B, T, N)
    assert fb >= 2 * B * T * 128 * 4 + 2 * B * T * 4  # scaled alpha/beta rows + log-scales
    vit = L.hmm355_viterbi_workspace_bytes(B, T, N)
    assert vit >= B * T * 128                          # uint8 backpointers
    # OBS_LOG decodes take no log-emission buffer; the default size is OBS_PROB's
    assert L.hmm355_viterbi_workspace_bytes_ex(B, T, N, 0) == vit
    assert L.hmm355_viterbi_workspace_bytes_ex(B, T, N, 1) == vit - B * T * N * 4
    assert L.hmm355_viterbi_workspace_bytes_ex(B, T, N, 2) == 0
    assert L.hmm355_gmm_workspace_bytes(32, 2000, 80, 128, 4) > 0
    assert L.hmm355_hsmm_workspace_bytes(16, 2000, 64, 40) > 0


def test_fb_workspace_layout_matches_header(L):
    """include/hmm355.h's forward-backward workspace layout (U | V | LA | LB | BandDesc | (B,NP) |
    (B) | (B,T) | CA | CB | the followers' counts, 256-B aligned) is what hmm355_fb_workspace_bytes
    sizes and what hmm355_fb_workspace_layout reports -- the offsets the adjoint reads U / V / LA /
    LB / CA / CB at (autograd.fb_layout), for every padded state count (N 200: NP 256)."""
    from pytorch_hmm_amd.autograd import FB_PIECES, fb_layout
    al = lambda n: ((n + 255) // 256) * 256
    for B, T, N in ((32, 2000, 128), (3, 17, 5), (2, 1, 200), (7, 129, 64), (4, 300, 200)):
        NP = 64 if N <= 64 else (128 if N <= 128 else 256)
        rows = B * T
        sizes = [rows * NP * 4, rows * NP * 4, rows * 4, rows * 4, L.hmm355_plan_bytes(N), B * NP * 4, B * 4,
                 rows * 4, rows * 4, rows * 4]
        off = fb_layout(B, T, N)
        # U | V and LA | LB and CA | CB are contiguous pairs, each pair 256-B aligned
        want, pos, pair = {}, 0, 0
        for name, nbytes in zip(FB_PIECES, sizes):
            want[name] = pos + pair
            if name in ("U", "LA", "CA"):
                pair = nbytes
            else:
                pos, pair = pos + al(pair + nbytes), 0
        assert off == want, (B, T, N, off, want)
        assert L.hmm355_fb_workspace_bytes(B, T, N) == pos + al(2 * B * 128), (B, T, N)


def test_release_build_reads_no_environment():
    """the library's behaviour does not depend on the process environment --
    a release build imports no getenv (the diagnostic switches exist only in HMM355_DIAG builds)."""
    from pytorch_hmm_amd import _native as nat
    out = subprocess.run(["nm", "-D", "--undefined-only", nat.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert not re.search(r"\b(secure_)?getenv\b", out), "libhmm355.so imports getenv"


def test_argument_rejection_before_launch(L):
    """Invalid arguments return the documented code; nothing touches the (absent) GPU."""
    d = header_defines()
    fake = ctypes.c_void_p(0x1000)  # never dereferenced: validation fails first
    # N out of range
    rc = L.hmm355_viterbi_f32(fake, 0, fake, fake, 1, 10, 300, fake, fake, fake, fake, 1 << 30, None)
    assert rc == d["HMM355_E_STATES"]
    rc = L.hmm355_forward_backward_f32(fake, 0, fake, fake, 1, 10, 0, 1, fake, None, None, None, None, fake, 1 << 30, None)
    assert rc == d["HMM355_E_STATES"]
    # T < 1
    rc = L.hmm355_viterbi_f32(fake, 0, fake, fake, 1, 0, 8, fake, fake, fake, fake, 1 << 30, None)
    assert rc == d["HMM355_E_SHAPE"]
    # null input
    rc = L.hmm355_viterbi_f32(None, 0, fake, fake, 1, 10, 8, fake, fake, fake, fake, 1 << 30, None)
    assert rc == d["HMM355_E_ARG"]
    # workspace too small
    rc = L.hmm355_forward_backward_f32(fake, 0, fake, fake, 2, 10, 8, 1, fake, None, None, None, None, fake, 16, None)
    assert rc == d["HMM355_E_WORKSPACE"]
    # bad obs_mode
    rc = L.hmm355_viterbi_f32(fake, 7, fake, fake, 1, 10, 8, fake, fake, fake, fake, 1 << 30, None)
    assert rc == d["HMM355_E_ARG"]
    # HSMM: duration table out of range
    rc = L.hmm355_hsmm_viterbi_f32(fake, fake, fake, 1, 10, 4, 0, fake, fake, fake, 1 << 30, None)
    assert rc == d["HMM355_E_DURATION"]
    rc = L.hmm355_hsmm_viterbi_f32(fake, fake, fake, 1, 10, 4, 1025, fake, fake, fake, 1 << 30, None)
    assert rc == d["HMM355_E_DURATION"]
    rc = L.hmm355_hsmm_viterbi_f32(fake, fake, fake, 1, 10, 1025, 8, fake, fake, fake, 1 << 30, None)
    assert rc == d["HMM355_E_STATES"]
    # the register-slot geometries and the general form (csrc/hsmm_wide.hip: S * (Dmax + 1)
    # floats per frame) both report a workspace; beyond S, Dmax <= 1024 nothing does
    assert L.hmm355_hsmm_workspace_bytes(2, 100, 64, 127) > 0 and L.hmm355_hsmm_workspace_bytes(2, 100, 128, 63) > 0
    assert L.hmm355_hsmm_workspace_bytes(2, 100, 129, 8) >= 2 * 100 * 129 * 9 * 4
    assert L.hmm355_hsmm_workspace_bytes(2, 100, 65, 64) >= 2 * 100 * 65 * 65 * 4
    assert L.hmm355_hsmm_workspace_bytes(2, 100, 1025, 8) == 0 and L.hmm355_hsmm_workspace_bytes(2, 100, 8, 1025) == 0
    # a workspace one byte short of the general form's
    need = L.hmm355_hsmm_workspace_bytes(1, 10, 200, 8)
    rc = L.hmm355_hsmm_viterbi_f32(fake, fake, fake, 1, 10, 200, 8, fake, fake, fake, need - 1, None)
    assert rc == d["HMM355_E_WORKSPACE"]
    # B == 0 is a no-op success
    assert L.hmm355_viterbi_f32(None, 0, None, None, 0, 10, 8, None, None, None, None, 0, None) == 0
