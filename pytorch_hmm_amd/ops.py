"""PyTorch-ROCm custom ops over the hmm355 C ABI (namespace ``hmm355``).

Each op allocates its outputs (and the C ABI's workspace) through the torch caching
allocator on the input's device and launches on the current HIP stream.  The ops are
registered with torch.library so they are visible to torch.compile / export and have
shape-only fake implementations; their only real implementation is the HIP library.

  torch.ops.hmm355.forward_backward(obs, log_P, log_p0, obs_mode, out_mask)
      -> (posterior, forward, backward, loglik, lik_ref)
  torch.ops.hmm355.viterbi(obs, log_P, init, obs_mode) -> (states, log_delta, final_score)
  torch.ops.hmm355.gmm_diag_logprob(x, means, log_vars, log_w, mix_lse) -> log_probs
  torch.ops.hmm355.hsmm_viterbi(lp, dur_lp, log_T) -> (states, scores)
  torch.ops.hmm355.tv_forward_backward(log_obs, log_A, log_p0, out_mask)
      -> (posterior, forward, backward, loglik, lik_ref)
  torch.ops.hmm355.tv_viterbi(log_obs, log_A, init) -> (states, log_delta)
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _native as nat

OBS_PROB = nat.OBS_PROB
OBS_LOG = nat.OBS_LOG
FB_POSTERIOR = nat.FB_POSTERIOR
FB_PAIR = nat.FB_PAIR
FB_PLAN_BANDED = nat.FB_PLAN_BANDED
VIT_PLAN_BANDED = nat.VIT_PLAN_BANDED
VIT_PLAN_DENSE = nat.VIT_PLAN_DENSE
FORM_GENERAL = nat.FORM_GENERAL
FORM_SERIAL_WALK = nat.FORM_SERIAL_WALK
FB_FORWARD = nat.FB_FORWARD
FB_BACKWARD = nat.FB_BACKWARD

_EMPTY = (0,)


def _f32c(t):
    return t.to(torch.float32).contiguous()


def _workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


# ------------------------------------------------------------------ forward-backward
def make_plan(log_P: Tensor, read_banded: bool = True, dense: bool = False) -> Tensor:
    """Measure log_P's banded structure once (hmm355_plan_ex_f32) into a device byte tensor that
    forward_backward / viterbi accept as `plan` (valid while log_P is unchanged).  dense=True
    (HMM355_PLAN_DENSE) makes a plan that selects the dense chains whatever the structure (the
    parity tests run both chain families on one matrix).

    The kernels read the structure from the plan on the device; the host only needs it to
    choose between launch shapes (the pair kernel, the psi followers), and reading it back is
    one synchronous device -> host copy.  With read_banded=False (a plan re-formed on every
    training step, where log_P changes each call) that read is skipped and the plan's host
    word stays unknown (None): forward_backward takes the two-kernel path, whose chains branch
    on the device-side structure, and viterbi asks for psi followers, which return at once on
    a banded plan (vit_kern.h vit_psi_follow) -- so the call stays asynchronous."""
    nat.require_gpu(log_P)
    log_P = _f32c(log_P)
    N = log_P.shape[0]
    L = nat.lib()
    plan = torch.empty(L.hmm355_plan_bytes(N), dtype=torch.uint8, device=log_P.device)
    with torch.cuda.device(log_P.device):
        nat.check(L.hmm355_plan_ex_f32(nat.ptr(log_P), N, nat.PLAN_DENSE if dense else 0, nat.ptr(plan),
                                       nat.stream_of(log_P.device)))
        if not read_banded:
            plan._hmm355_banded = None
            return plan
        # banded in both directions: forward_backward then runs both chains of a sequence in
        # one workgroup (HMM355_FB_PAIR, csrc/fbpair.h).  One synchronous read per plan.
        banded = L.hmm355_plan_banded(nat.ptr(plan), nat.stream_of(log_P.device))
    if banded < 0:
        nat.check(banded)
    plan._hmm355_banded = banded == 1
    return plan


def plan_info(plan: Optional[Tensor]) -> dict:
    """Which chains a plan selects (band.h BandDesc: wc/wr window widths, Toeplitz windows).
    Reads a few ints back to the host."""
    if plan is None:
        return {"forward": "detected per call", "backward": "detected per call", "viterbi": "detected per call"}
    h = plan[: 4 * 7177].cpu().view(torch.int32).tolist()
    wc, wr = h[0], h[1]
    tcd0, tcw, trd0, trw = h[7172:7176]
    band_max = 8   # band.h kBandMax

    def name(w, tw, td0):
        if w > band_max:
            return "dense"
        return f"banded(W={w}, toeplitz {td0}..{td0 + tw - 1})" if tw > 0 else f"banded(W={w})"
    col = name(wc, tcw, tcd0)
    return {"forward": col, "viterbi": col, "backward": name(wr, trw, trd0)}


_CUS = {}


# forward_backward's posterior beside the chains (follow=None): measured per round on MI355X
# (DESIGN.md §5); a caller's True / False wins
FB_FOLLOW_DEFAULT = True


def fb_follow_default(follow: Optional[bool]) -> bool:
    return FB_FOLLOW_DEFAULT if follow is None else bool(follow)


def _use_pair(B: int, dev) -> bool:
    """Both chains of a sequence in one workgroup (csrc/fbpair.h, HMM355_FB_PAIR) when the
    batch is larger than half the CUs: the two-kernel path then needs more CU-owning
    workgroups (2B) than the chip has and runs in two rounds, while the pair kernel needs B.
    Measured: B=32 two-kernel 0.24 ms vs pair 0.38 ms; B=256 FB op 0.90 vs 0.51
    ms.  (forward_backward's `pair` argument overrides it.)"""
    key = str(dev)
    if key not in _CUS:
        _CUS[key] = torch.cuda.get_device_properties(dev).multi_processor_count
    return B > _CUS[key] // 2


@torch.library.custom_op("hmm355::forward_backward", mutates_args=())
def forward_backward(obs: Tensor, log_P: Tensor, log_p0: Tensor, obs_mode: int,
                     out_mask: int, plan: Optional[Tensor] = None, pair: Optional[bool] = None,
                     follow: Optional[bool] = None) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """pair / follow (None = chosen from the batch and the plan): with a host-known banded plan,
    `pair` runs both chains of a sequence in one workgroup (HMM355_FB_PAIR, large batches) and
    otherwise `follow` forms the posterior inside the chains' launch (HMM355_FB_PLAN_BANDED)."""
    nat.require_gpu(obs, log_P, log_p0)
    obs, log_P, log_p0 = _f32c(obs), _f32c(log_P), _f32c(log_p0)
    B, T, N = obs.shape
    dev = obs.device
    L = nat.lib()
    post = torch.empty((B, T, N) if out_mask & FB_POSTERIOR else _EMPTY, device=dev)
    fwd = torch.empty((B, T, N) if out_mask & FB_FORWARD else _EMPTY, device=dev)
    bwd = torch.empty((B, T, N) if out_mask & FB_BACKWARD else _EMPTY, device=dev)
    loglik = torch.empty(B, device=dev)
    lik_ref = torch.empty(B, device=dev)
    if B == 0:
        return post, fwd, bwd, loglik, lik_ref
    nbytes = L.hmm355_fb_workspace_bytes(B, T, N)
    ws = _workspace(nbytes, dev)
    banded = plan is not None and getattr(plan, "_hmm355_banded", False) is True
    use_pair = banded and (_use_pair(B, dev) if pair is None else pair)
    if use_pair:
        out_mask |= FB_PAIR
    elif banded and (out_mask & FB_POSTERIOR) and fb_follow_default(follow):
        out_mask |= FB_PLAN_BANDED
    with torch.cuda.device(dev):
        nat.check(L.hmm355_forward_backward_plan_f32(
            nat.ptr(obs), obs_mode, nat.ptr(log_P), nat.ptr(log_p0), nat.ptr(plan), None, B, T, N, out_mask,
            nat.ptr(post) if out_mask & FB_POSTERIOR else None,
            nat.ptr(fwd) if out_mask & FB_FORWARD else None,
            nat.ptr(bwd) if out_mask & FB_BACKWARD else None,
            nat.ptr(loglik), nat.ptr(lik_ref), nat.ptr(ws), ws.numel(), nat.stream_of(dev)))
    return post, fwd, bwd, loglik, lik_ref


@forward_backward.register_fake
def _(obs, log_P, log_p0, obs_mode, out_mask, plan=None, pair=None, follow=None):
    B, T, N = obs.shape
    mk = lambda bit: obs.new_empty((B, T, N) if out_mask & bit else _EMPTY)
    return mk(FB_POSTERIOR), mk(FB_FORWARD), mk(FB_BACKWARD), obs.new_empty(B), obs.new_empty(B)


# ---------------------------------------------------------------------------- Viterbi
@torch.library.custom_op("hmm355::viterbi", mutates_args=())
def viterbi(obs: Tensor, log_P: Tensor, init: Tensor, obs_mode: int,
            plan: Optional[Tensor] = None, follow: Optional[bool] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """follow (None = on): with a plan, the work beside the chain inside its launch -- for a
    host-known banded plan the log leaders and the decode follower (HMM355_VIT_PLAN_BANDED), for a
    dense one the psi followers (HMM355_VIT_PLAN_DENSE)."""
    nat.require_gpu(obs, log_P, init)
    obs, log_P, init = _f32c(obs), _f32c(log_P), _f32c(init)
    B, T, N = obs.shape
    dev = obs.device
    L = nat.lib()
    states = torch.empty((B, T), dtype=torch.int64, device=dev)
    delta = torch.empty((B, T, N), device=dev)
    final = torch.empty(B, device=dev)
    if B == 0:
        return states, delta, final
    ws = _workspace(L.hmm355_viterbi_workspace_bytes_ex(B, T, N, obs_mode), dev)
    flags = 0
    if plan is not None and follow is not False:
        if getattr(plan, "_hmm355_banded", False) is True:
            flags = VIT_PLAN_BANDED   # the decode beside the banded chain (csrc/follow.h)
        else:
            # a dense plan: the argmax pointers computed beside the chain, on the CUs it leaves
            # (a plan whose structure the host never read,
            # make_plan(read_banded=False), asks for them too: on a banded matrix they return at once)
            flags = VIT_PLAN_DENSE
    with torch.cuda.device(dev):
        nat.check(L.hmm355_viterbi_plan_ex_f32(
            nat.ptr(obs), obs_mode, nat.ptr(log_P), nat.ptr(init), nat.ptr(plan), flags, B, T, N,
            nat.ptr(states), nat.ptr(delta), nat.ptr(final), nat.ptr(ws), ws.numel(), nat.stream_of(dev)))
    return states, delta, final


@viterbi.register_fake
def _(obs, log_P, init, obs_mode, plan=None, follow=None):
    B, T, N = obs.shape
    return (obs.new_empty((B, T), dtype=torch.int64), obs.new_empty((B, T, N)), obs.new_empty(B))


# ------------------------------------------------------------------- GMM emission
@torch.library.custom_op("hmm355::gmm_diag_logprob", mutates_args=())
def gmm_diag_logprob(x: Tensor, means: Tensor, log_vars: Tensor, log_w: Tensor, mix_lse: int) -> Tensor:
    nat.require_gpu(x, means, log_vars, log_w)
    x, means, log_vars, log_w = _f32c(x), _f32c(means), _f32c(log_vars), _f32c(log_w)
    B, T, D = x.shape
    S, C, D2 = means.shape
    if D2 != D:
        raise ValueError(f"feature dim mismatch: x has {D}, means have {D2}")
    out = torch.empty((B, T, S), device=x.device)
    if B * T == 0:
        return out
    L = nat.lib()
    ws = _workspace(L.hmm355_gmm_workspace_bytes(B, T, D, S, C), x.device)
    with torch.cuda.device(x.device):
        nat.check(L.hmm355_gmm_diag_logprob_f32(
            nat.ptr(x), nat.ptr(means), nat.ptr(log_vars), nat.ptr(log_w), B, T, D, S, C, mix_lse,
            nat.ptr(out), nat.ptr(ws), ws.numel(), nat.stream_of(x.device)))
    return out


@gmm_diag_logprob.register_fake
def _(x, means, log_vars, log_w, mix_lse):
    return x.new_empty((x.shape[0], x.shape[1], means.shape[0]))


# ------------------------------------------------------------------------------- HSMM
@torch.library.custom_op("hmm355::hsmm_viterbi", mutates_args=())
def hsmm_viterbi(lp: Tensor, dur_lp: Tensor, log_T: Tensor, flags: int = 0) -> Tuple[Tensor, Tensor]:
    """flags: kernel-form flags (FORM_GENERAL, FORM_SERIAL_WALK; identical results)."""
    nat.require_gpu(lp, dur_lp, log_T)
    lp, dur_lp, log_T = _f32c(lp), _f32c(dur_lp), _f32c(log_T)
    B, T, S = lp.shape
    Dm = dur_lp.shape[1]
    dev = lp.device
    states = torch.empty((B, T), dtype=torch.int64, device=dev)
    scores = torch.empty(B, device=dev)
    if B == 0:
        return states, scores
    L = nat.lib()
    # The general form (S or Dmax beyond the register-slot kernels) keeps a (B,T,S,Dmax+1) fp32
    # table: checked against the device's free memory up front, and decoded in batch slices
    # that fit when the whole batch does not (sequences are independent).
    wsb = lambda b_, t_, s_, d_: L.hmm355_hsmm_workspace_bytes_ex(b_, t_, s_, d_, flags)
    Bc = _ws_batch(wsb, B, T, S, Dm, dev, "HSMM decode")
    ws = _workspace(wsb(Bc, T, S, Dm), dev)
    with torch.cuda.device(dev):
        for b0 in range(0, B, Bc):
            nb = min(Bc, B - b0)
            nat.check(L.hmm355_hsmm_viterbi_ex_f32(
                nat.ptr(lp[b0:b0 + nb]), nat.ptr(dur_lp), nat.ptr(log_T), nb, T, S, Dm, flags,
                nat.ptr(states[b0:b0 + nb]), nat.ptr(scores[b0:b0 + nb]), nat.ptr(ws), ws.numel(),
                nat.stream_of(dev)))
    return states, scores


_HSMM_WS_CHECK_BYTES = 1 << 30  # workspaces above this are checked against free device memory


def _ws_batch(ws_bytes, B, T, S, Dm, dev, what):
    """The batch slice whose workspace fits the device (general-form segment recursions keep a
    (B,T,S,Dmax) fp32 table): B when the whole batch's workspace is small or fits, else the
    largest slice that fits; OutOfMemoryError when not even one sequence does."""
    need = ws_bytes(B, T, S, Dm)
    if need <= _HSMM_WS_CHECK_BYTES:
        return B
    per_seq = ws_bytes(1, T, S, Dm)
    free, _ = torch.cuda.mem_get_info(dev)
    avail = free + torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    if per_seq > 0.9 * avail:
        raise torch.cuda.OutOfMemoryError(
            f"{what} of one sequence (T={T}, S={S}, max_duration={Dm}) needs {per_seq / 2**30:.1f} GiB "
            f"of workspace (about T*S*max_duration*4 bytes), {avail / 2**30:.1f} GiB are available on {dev}")
    return max(1, min(B, int(0.9 * avail) // per_seq))


@hsmm_viterbi.register_fake
def _(lp, dur_lp, log_T, flags=0):
    B, T, S = lp.shape
    return lp.new_empty((B, T), dtype=torch.int64), lp.new_empty(B)


# ------------------------------------------------- time-varying transitions (NeuralHMM)
def _tv_matrix(log_A: Tensor, B: int, T: int, N: int):
    """(tensor, batch stride, step stride) for the C ABI.  log_A is (N,N) (one matrix for all
    steps) or (B,T,N,N) with contiguous rows — an expand()ed static matrix keeps its zero
    strides, so it is never materialised (neural.py:385 expands one (N,N) over (B,T))."""
    if log_A.dtype != torch.float32:
        log_A = log_A.float()
    if log_A.dim() == 2:
        if tuple(log_A.shape) != (N, N):
            raise ValueError(f"transition matrix shape {tuple(log_A.shape)} != ({N}, {N})")
        return log_A.contiguous(), 0, 0
    if log_A.dim() != 4 or log_A.shape[0] != B or tuple(log_A.shape[2:]) != (N, N):
        raise ValueError(f"log transition tensor shape {tuple(log_A.shape)} != ({B}, {T}, {N}, {N})")
    if log_A.shape[1] < T - 1:  # steps 0..T-2 are read (neural.py:419-458)
        raise IndexError(f"log transition tensor has {log_A.shape[1]} steps, the recursion needs {T - 1}")
    if log_A.stride(3) != 1 or log_A.stride(2) != N or min(log_A.stride(0), log_A.stride(1)) < 0:
        log_A = log_A.contiguous()
    if log_A.stride(0) == 0 and log_A.stride(1) == 0:
        return log_A, 0, 0
    if log_A.stride(1) == 0 or log_A.stride(0) == 0:
        log_A = log_A.contiguous()
    return log_A, log_A.stride(0), log_A.stride(1)


@torch.library.custom_op("hmm355::tv_forward_backward", mutates_args=())
def tv_forward_backward(log_obs: Tensor, log_A: Tensor, log_p0: Tensor,
                        out_mask: int) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    nat.require_gpu(log_obs, log_A, log_p0)
    log_obs, log_p0 = _f32c(log_obs), _f32c(log_p0)
    B, T, N = log_obs.shape
    dev = log_obs.device
    L = nat.lib()
    post = torch.empty((B, T, N) if out_mask & FB_POSTERIOR else _EMPTY, device=dev)
    fwd = torch.empty((B, T, N) if out_mask & FB_FORWARD else _EMPTY, device=dev)
    bwd = torch.empty((B, T, N) if out_mask & FB_BACKWARD else _EMPTY, device=dev)
    loglik = torch.empty(B, device=dev)
    lik_ref = torch.empty(B, device=dev)
    if B == 0:
        return post, fwd, bwd, loglik, lik_ref
    A, sb, st = _tv_matrix(log_A, B, T, N)
    ws = _workspace(L.hmm355_tv_fb_workspace_bytes(B, T, N), dev)
    with torch.cuda.device(dev):
        nat.check(L.hmm355_tv_forward_backward_f32(
            nat.ptr(log_obs), nat.ptr(A), sb, st, nat.ptr(log_p0), B, T, N, out_mask,
            nat.ptr(post) if out_mask & FB_POSTERIOR else None,
            nat.ptr(fwd) if out_mask & FB_FORWARD else None,
            nat.ptr(bwd) if out_mask & FB_BACKWARD else None,
            nat.ptr(loglik), nat.ptr(lik_ref), nat.ptr(ws), ws.numel(), nat.stream_of(dev)))
    return post, fwd, bwd, loglik, lik_ref


@tv_forward_backward.register_fake
def _(log_obs, log_A, log_p0, out_mask):
    B, T, N = log_obs.shape
    mk = lambda bit: log_obs.new_empty((B, T, N) if out_mask & bit else _EMPTY)
    return mk(FB_POSTERIOR), mk(FB_FORWARD), mk(FB_BACKWARD), log_obs.new_empty(B), log_obs.new_empty(B)


@torch.library.custom_op("hmm355::tv_viterbi", mutates_args=())
def tv_viterbi(log_obs: Tensor, log_A: Tensor, init: Tensor) -> Tuple[Tensor, Tensor]:
    nat.require_gpu(log_obs, log_A, init)
    log_obs, init = _f32c(log_obs), _f32c(init)
    B, T, N = log_obs.shape
    dev = log_obs.device
    states = torch.empty((B, T), dtype=torch.int64, device=dev)
    delta = torch.empty((B, T, N), device=dev)
    if B == 0:
        return states, delta
    A, sb, st = _tv_matrix(log_A, B, T, N)
    L = nat.lib()
    ws = _workspace(L.hmm355_tv_viterbi_workspace_bytes(B, T, N), dev)
    with torch.cuda.device(dev):
        nat.check(L.hmm355_tv_viterbi_f32(
            nat.ptr(log_obs), nat.ptr(A), sb, st, nat.ptr(init), B, T, N, nat.ptr(states), nat.ptr(delta),
            nat.ptr(ws), ws.numel(), nat.stream_of(dev)))
    return states, delta


@tv_viterbi.register_fake
def _(log_obs, log_A, init):
    B, T, N = log_obs.shape
    return log_obs.new_empty((B, T), dtype=torch.int64), log_obs.new_empty((B, T, N))


# ------------------------------------------------------- explicit-duration (semi-Markov)
@torch.library.custom_op("hmm355::semimarkov_quad", mutates_args=())
def semimarkov_quad(x: Tensor, means_t: Tensor, vars_t: Tensor) -> Tensor:
    """(B,T,Df) frames, (Df,S) means / variances -> (B,T,S) sum_k (x-mu)^2/var (k ascending)."""
    nat.require_gpu(x, means_t, vars_t)
    x, means_t, vars_t = _f32c(x), _f32c(means_t), _f32c(vars_t)
    B, T, Df = x.shape
    S = means_t.shape[1]
    if means_t.shape[0] != Df or tuple(vars_t.shape) != tuple(means_t.shape):
        raise ValueError(f"feature dim mismatch: x has {Df}, means {tuple(means_t.shape)}, "
                         f"variances {tuple(vars_t.shape)} (expected ({Df}, S))")
    q = torch.empty((B, T, S), device=x.device)
    with torch.cuda.device(x.device):
        nat.check(nat.lib().hmm355_semimarkov_quad_f32(
            nat.ptr(x), nat.ptr(means_t), nat.ptr(vars_t), B, T, Df, S, nat.ptr(q),
            nat.stream_of(x.device)))
    return q


@semimarkov_quad.register_fake
def _(x, means_t, vars_t):
    return x.new_empty((x.shape[0], x.shape[1], means_t.shape[1]))


def _smk_args(quad, seg_const, log_init, log_T, dur_lp):
    nat.require_gpu(quad, seg_const, log_init, log_T, dur_lp)
    quad, log_init, log_T, dur_lp = _f32c(quad), _f32c(log_init), _f32c(log_T), _f32c(dur_lp)
    seg_const = None if seg_const is None else _f32c(seg_const)
    B, T, S = quad.shape
    if tuple(log_T.shape) != (S, S) or log_init.shape != (S,) or dur_lp.shape[0] != S:
        raise ValueError(f"parameter shapes {tuple(log_init.shape)}, {tuple(log_T.shape)}, "
                         f"{tuple(dur_lp.shape)} do not match {S} states")
    if seg_const is not None and seg_const.shape != (S,):
        raise ValueError(f"segment constant shape {tuple(seg_const.shape)} != ({S},)")
    return quad, seg_const, log_init, log_T, dur_lp, B, T, S, dur_lp.shape[1]


@torch.library.custom_op("hmm355::semimarkov_viterbi", mutates_args=())
def semimarkov_viterbi(quad: Tensor, seg_const: Optional[Tensor], log_init: Tensor, log_T: Tensor,
                       dur_lp: Tensor, flags: int = 0) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """-> seg_states (B,T) int64, seg_durs (B,T) int64 (right-aligned), seg_count (B) int32,
    scores (B).  flags: FORM_GENERAL forces the general form (identical results)."""
    quad, seg_const, log_init, log_T, dur_lp, B, T, S, Dm = _smk_args(quad, seg_const, log_init, log_T, dur_lp)
    dev = quad.device
    seg_s = torch.empty((B, T), dtype=torch.int64, device=dev)
    seg_d = torch.empty((B, T), dtype=torch.int64, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    scores = torch.empty(B, device=dev)
    if B == 0:
        return seg_s, seg_d, cnt, scores
    L = nat.lib()
    wsb = lambda b_, t_, s_, d_: L.hmm355_semimarkov_workspace_bytes_ex(b_, t_, s_, d_, flags)
    Bc = _ws_batch(wsb, B, T, S, Dm, dev, "semi-Markov decode")
    ws = _workspace(wsb(Bc, T, S, Dm), dev)
    with torch.cuda.device(dev):
        for b0 in range(0, B, Bc):
            nb = min(Bc, B - b0)
            nat.check(L.hmm355_semimarkov_viterbi_ex_f32(
                nat.ptr(quad[b0:b0 + nb]), nat.ptr(seg_const), nat.ptr(log_init), nat.ptr(log_T), nat.ptr(dur_lp),
                nb, T, S, Dm, flags, nat.ptr(seg_s[b0:b0 + nb]), nat.ptr(seg_d[b0:b0 + nb]), nat.ptr(cnt[b0:b0 + nb]),
                nat.ptr(scores[b0:b0 + nb]), nat.ptr(ws), ws.numel(), nat.stream_of(dev)))
    return seg_s, seg_d, cnt, scores


@semimarkov_viterbi.register_fake
def _(quad, seg_const, log_init, log_T, dur_lp, flags=0):
    B, T, _ = quad.shape
    return (quad.new_empty((B, T), dtype=torch.int64), quad.new_empty((B, T), dtype=torch.int64),
            quad.new_empty(B, dtype=torch.int32), quad.new_empty(B))


@torch.library.custom_op("hmm355::semimarkov_forward", mutates_args=())
def semimarkov_forward(quad: Tensor, seg_const: Optional[Tensor], log_init: Tensor, log_T: Tensor,
                       dur_lp: Tensor, want_alpha: bool, flags: int = 0) -> Tuple[Tensor, Tensor]:
    """-> log_prob (B), log_alpha (B,T,S,Dmax) (empty (0,) unless want_alpha)."""
    quad, seg_const, log_init, log_T, dur_lp, B, T, S, Dm = _smk_args(quad, seg_const, log_init, log_T, dur_lp)
    dev = quad.device
    lp = torch.empty(B, device=dev)
    alpha = torch.empty((B, T, S, Dm) if want_alpha else (0,), device=dev)
    if B == 0:
        return lp, alpha
    L = nat.lib()
    wsb = lambda b_, t_, s_, d_: L.hmm355_semimarkov_workspace_bytes_ex(b_, t_, s_, d_, flags)
    Bc = _ws_batch(wsb, B, T, S, Dm, dev, "semi-Markov forward")
    ws = _workspace(wsb(Bc, T, S, Dm), dev)
    with torch.cuda.device(dev):
        for b0 in range(0, B, Bc):
            nb = min(Bc, B - b0)
            nat.check(L.hmm355_semimarkov_forward_ex_f32(
                nat.ptr(quad[b0:b0 + nb]), nat.ptr(seg_const), nat.ptr(log_init), nat.ptr(log_T), nat.ptr(dur_lp),
                nb, T, S, Dm, flags, nat.ptr(alpha[b0:b0 + nb]) if want_alpha else None, nat.ptr(lp[b0:b0 + nb]),
                nat.ptr(ws), ws.numel(), nat.stream_of(dev)))
    return lp, alpha


@semimarkov_forward.register_fake
def _(quad, seg_const, log_init, log_T, dur_lp, want_alpha, flags=0):
    B, T, S = quad.shape
    return quad.new_empty(B), quad.new_empty((B, T, S, dur_lp.shape[1]) if want_alpha else (0,))


# ------------------------------------------------------------------ streaming decoders
STREAM_SLOTS = 32   # hypothesis slots per stream (max beam width; 16 when N > 128)

@torch.library.custom_op("hmm355::stream_greedy", mutates_args=())
def stream_greedy(emis: Tensor, log_T: Tensor, prev_state: Tensor, log_n: float) -> Tuple[Tensor, Tensor]:
    """(B,T,N) emission log-probs -> greedy chain states (B,T) int64 and step scores (B,T).
    prev_state (B) int32: the stream's last decoded state, or -1 for its first chunk."""
    nat.require_gpu(emis, log_T, prev_state)
    emis, log_T = _f32c(emis), _f32c(log_T)
    prev_state = prev_state.to(torch.int32).contiguous()
    B, T, N = emis.shape
    states = torch.empty((B, T), dtype=torch.int64, device=emis.device)
    scores = torch.empty((B, T), device=emis.device)
    with torch.cuda.device(emis.device):
        nat.check(nat.lib().hmm355_stream_greedy_f32(
            nat.ptr(emis), nat.ptr(log_T), nat.ptr(prev_state), float(log_n), B, T, N,
            nat.ptr(states), nat.ptr(scores), nat.stream_of(emis.device)))
    return states, scores


@stream_greedy.register_fake
def _(emis, log_T, prev_state, log_n):
    B, T, _ = emis.shape
    return emis.new_empty((B, T), dtype=torch.int64), emis.new_empty((B, T))


def stream_beam(emis: Tensor, log_T: Tensor, beam_width: int, hyp_score: Tensor, hyp_last: Tensor,
                hyp_count: Tensor, first: Tensor, live_max: int = STREAM_SLOTS):
    """One chunk of beam search for B streams.  hyp_score (B,32) fp32, hyp_last (B,32) int32
    and hyp_count (B) int32 are the streams' hypotheses (rank order, STREAM_SLOTS slots),
    updated IN PLACE; K = beam_width <= 32 (<= 16 when N > 128), N <= 256;
    first (B) int32 marks streams whose paths are still empty; live_max bounds hyp_count.  Returns (best-path states
    (B,T) int64, parent (B,T,K) int16, state (B,T,K) int16): new hypothesis r at step t came
    from hypothesis parent[t, r] of step t-1 and entered state[t, r]."""
    nat.require_gpu(emis, log_T, hyp_score, hyp_last, hyp_count, first)
    emis, log_T = _f32c(emis), _f32c(log_T)
    B, T, N = emis.shape
    K = int(beam_width)
    for name, ten, dt in (("hyp_score", hyp_score, torch.float32), ("hyp_last", hyp_last, torch.int32),
                          ("hyp_count", hyp_count, torch.int32), ("first", first, torch.int32)):
        if ten.dtype != dt or not ten.is_contiguous():
            raise ValueError(f"{name} must be a contiguous {dt} tensor")
    if tuple(hyp_score.shape) != (B, STREAM_SLOTS) or tuple(hyp_last.shape) != (B, STREAM_SLOTS):
        raise ValueError(f"hypothesis tensors must be ({B}, {STREAM_SLOTS})")
    dev = emis.device
    states = torch.empty((B, T), dtype=torch.int64, device=dev)
    parent = torch.empty((B, T, K), dtype=torch.int16, device=dev)
    hstate = torch.empty((B, T, K), dtype=torch.int16, device=dev)
    with torch.cuda.device(dev):
        nat.check(nat.lib().hmm355_stream_beam_f32(
            nat.ptr(emis), nat.ptr(log_T), B, T, N, K, int(live_max), nat.ptr(hyp_score), nat.ptr(hyp_last),
            nat.ptr(hyp_count), nat.ptr(first), nat.ptr(parent), nat.ptr(hstate), nat.ptr(states),
            nat.stream_of(dev)))
    return states, parent, hstate
