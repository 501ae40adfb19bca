"""Autograd for the forward-backward path (HMMLayer.compute_loss / training).

The reference differentiates through its Python loops with plain autograd
(hmm.py:89-101 via hmm_layer.py:144-173; test_hmm.py:189-208 trains HMMLayer through
compute_loss).  Here the gradient is the analytic adjoint of the forward recursion, run by
the same HIP kernels:

For a loss L(log alpha_{T-1}) with g = dL/d log alpha_{T-1} and G = sum_j g_j, the adjoint
lambda_t = dL/d log alpha_t satisfies lambda_t = alpha_t * mu_t where mu is the BACKWARD
recursion started from mu_{T-1} = g / alpha_{T-1} (hmm355_forward_backward_ex_f32 with
log_beta_T = log mu_{T-1}); sum_j lambda_t(j) = G at every t, so
    dL/d log_obs_t = G * posterior'_t          (posterior' = u v / sum(u v) of that pass)
    dL/d log_p0    = sum_b G_b posterior'_{b,0}
    dL/d log_P     = exp(log_P) * sum_{b,t} G_b X_t (x) Y_t,
        X_t = u_{t-1} / (c_{t-1} * sum_k u_t v_t),  Y_t = e_t * v_t,  c_{t-1} = sum u_{t-1}
(u, v: the scaled rows the chains store; every factor is O(1), no exp of log-scales).  The
last contraction is a plain batched GEMM (torch.einsum -> hipBLASLt).

Losses: 'ref'   = the reference's compute_likelihood value LSE_j log(exp(log alpha_{T-1,j}) + 1e-8)
                  (its gradient underflows to 0 exactly where the reference's does);
        'exact' = log sum_j alpha_{T-1,j}  (HMMPyTorch.log_likelihood).
Back-propagating THROUGH the posteriors / forward / backward outputs (HMMLayer training,
the supervised cross-entropy of compute_loss) is ForwardBackwardFn: the adjoint of both
recursions with per-step sources, on hmm355_fb_adjoint_f32 (csrc/adjoint.hip); with one
transition matrix per step (NeuralHMM) TvForwardBackwardFn on hmm355_tv_fb_adjoint_f32
(csrc/tv.hip).
"""
import math

import torch

from . import _native as nat


def needs_grad(*tensors) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


def _pad(N):
    return 64 if N <= 64 else (128 if N <= 128 else 256)


FB_PIECES = ("U", "V", "LA", "LB", "band", "binit", "bscale", "rmax", "CA", "CB")


def fb_layout(B, T, N):
    """{piece: byte offset} of the forward-backward workspace (hmm355_fb_workspace_layout)."""
    import ctypes
    out = (ctypes.c_size_t * len(FB_PIECES))()
    nat.check(nat.lib().hmm355_fb_workspace_layout(B, T, N, out))
    return dict(zip(FB_PIECES, out))


def _run_fb(obs, log_P, log_p0, obs_mode, log_beta_T=None, posterior=False, out_mask=None, plan=None):
    """One hmm355_forward_backward_plan_f32 call; returns (posterior|None, loglik, lik_ref, U, V,
    LA, LB), or with `out_mask` ((posterior, forward, backward) per the mask, loglik, lik_ref, U,
    V, LA, LB)."""
    B, T, N = obs.shape
    NP = _pad(N)
    dev = obs.device
    L = nat.lib()
    ws = torch.empty(L.hmm355_fb_workspace_bytes(B, T, N), dtype=torch.uint8, device=dev)
    mask = out_mask if out_mask is not None else (nat.FB_POSTERIOR if posterior else 0)
    mk = lambda bit: torch.empty(B, T, N, device=dev) if mask & bit else None
    post, fwd, bwd = mk(nat.FB_POSTERIOR), mk(nat.FB_FORWARD), mk(nat.FB_BACKWARD)
    loglik = torch.empty(B, device=dev)
    lik_ref = torch.empty(B, device=dev)
    with torch.cuda.device(dev):
        nat.check(L.hmm355_forward_backward_plan_f32(
            nat.ptr(obs), obs_mode, nat.ptr(log_P), nat.ptr(log_p0), nat.ptr(plan), nat.ptr(log_beta_T), B, T, N,
            mask, nat.ptr(post), nat.ptr(fwd), nat.ptr(bwd), nat.ptr(loglik), nat.ptr(lik_ref),
            nat.ptr(ws), ws.numel(), nat.stream_of(dev)))
    rows = B * T
    # the workspace pieces, at the offsets the library reports (hmm355_fb_workspace_layout)
    o = fb_layout(B, T, N)
    fl = ws.view(torch.float32)
    piece = lambda name, n: fl[o[name] // 4: o[name] // 4 + n]
    U = piece("U", rows * NP).view(B, T, NP)[..., :N]
    V = piece("V", rows * NP).view(B, T, NP)[..., :N]
    LA = piece("LA", rows).view(B, T)
    LB = piece("LB", rows).view(B, T)
    CA = piece("CA", rows).view(B, T)
    CB = piece("CB", rows).view(B, T)
    if out_mask is not None:
        return (post, fwd, bwd), loglik, lik_ref, U, V, LA, LB, CA, CB
    return post, loglik, lik_ref, U, V, LA, LB, CA, CB


def _staged_emissions(obs, obs_mode):
    """The emissions the chains multiply by: obs + 1e-8 (OBS_PROB, hmm.py:86) or exp(obs - M_t)
    with M_t the row maximum (OBS_LOG; 0 for a row without a finite maximum, hmm355.h)."""
    if obs_mode == nat.OBS_PROB:
        return obs + 1e-8
    m = obs.amax(-1, keepdim=True)
    m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
    return torch.exp(obs - m)


class SequenceLogLik(torch.autograd.Function):
    """(B,) log-likelihood of each sequence ('ref' or 'exact'), differentiable in obs,
    log_P and log_p0."""

    @staticmethod
    def forward(ctx, obs, log_P, log_p0, obs_mode, kind, plan=None):
        nat.require_gpu(obs, log_P, log_p0)
        obs_c, lP, l0 = (t.detach().to(torch.float32).contiguous() for t in (obs, log_P, log_p0))
        _, loglik, lik_ref, *_ = _run_fb(obs_c, lP, l0, obs_mode, plan=plan)
        ctx.save_for_backward(obs_c, lP, l0)
        ctx.obs_mode, ctx.kind, ctx.plan = obs_mode, kind, plan
        return lik_ref if kind == "ref" else loglik

    @staticmethod
    def backward(ctx, gout):
        obs, lP, l0 = ctx.saved_tensors
        B, T, N = obs.shape
        _, _, _, U, _, LA, _, _, _ = _run_fb(obs, lP, l0, ctx.obs_mode, plan=ctx.plan)
        a_last = torch.log(U[:, -1]) + LA[:, -1:]                 # log alpha_{T-1}  (B,N)
        if ctx.kind == "ref":
            f = torch.exp(a_last)                                 # the reference's forward[:, -1]
            z = torch.log(f + 1e-8)
            w = torch.softmax(z, dim=-1)
            g = w * f / (f + 1e-8)                                # dL/d log alpha_{T-1}
            log_mu = torch.log(w) - z                             # log(g / alpha_{T-1})
        else:
            g = torch.softmax(a_last, dim=-1)
            log_mu = torch.zeros_like(a_last)
        G = g.sum(-1) * gout                                      # (B,)
        post, _, _, U, V, _, _, CA, _ = _run_fb(obs, lP, l0, ctx.obs_mode, log_beta_T=log_mu.contiguous(),
                                                posterior=True, plan=ctx.plan)
        grad_lo = G[:, None, None] * post
        if ctx.obs_mode == nat.OBS_PROB:
            grad_obs = grad_lo / (obs + 1e-8)
            e = obs + 1e-8
        else:
            grad_obs = grad_lo
            # the kernels' shifted emissions e_t = exp(lo_t - M_t) (hmm355.h, OBS_LOG): the
            # shift cancels in X_t (x) Y_t, and unshifted exp(lo) would underflow
            m = obs.amax(-1, keepdim=True)
            m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
            e = torch.exp(obs - m)
        grad_l0 = (G[:, None] * post[:, 0]).sum(0)
        grad_lP = None
        if T > 1 and ctx.needs_input_grad[1]:
            c = CA                                                # U_{t+1} = A^T U_t e_{t+1} / c_t
            S = (U * V).sum(-1)                                   # (B,T)
            X = U[:, :-1] / (c[:, :-1] * S[:, 1:]).unsqueeze(-1) * G[:, None, None]
            Y = e[:, 1:] * V[:, 1:]
            M = torch.einsum("bti,btj->ij", X, Y)
            grad_lP = torch.exp(lP) * M
        return grad_obs, grad_lP, grad_l0, None, None, None


def _run_tv_fb(log_obs, A, sb, st, log_p0, log_beta_T=None, posterior=False, out_mask=None):
    """One hmm355_tv_forward_backward_ex_f32 call; returns (posterior|None, loglik, lik_ref, U, V, E, LA),
    with `out_mask` the first item is the (posterior, forward, backward) tuple per the mask."""
    B, T, N = log_obs.shape
    NP = _pad(N)
    dev = log_obs.device
    L = nat.lib()
    ws = torch.empty(L.hmm355_tv_fb_workspace_bytes(B, T, N), dtype=torch.uint8, device=dev)
    mask = out_mask if out_mask is not None else (nat.FB_POSTERIOR if posterior else 0)
    mk = lambda bit: torch.empty(B, T, N, device=dev) if mask & bit else None
    post, fwd, bwd = mk(nat.FB_POSTERIOR), mk(nat.FB_FORWARD), mk(nat.FB_BACKWARD)
    loglik = torch.empty(B, device=dev)
    lik_ref = torch.empty(B, device=dev)
    with torch.cuda.device(dev):
        nat.check(L.hmm355_tv_forward_backward_ex_f32(
            nat.ptr(log_obs), nat.ptr(A), sb, st, nat.ptr(log_p0), nat.ptr(log_beta_T), B, T, N,
            mask, nat.ptr(post), nat.ptr(fwd), nat.ptr(bwd), nat.ptr(loglik), nat.ptr(lik_ref),
            nat.ptr(ws), ws.numel(), nat.stream_of(dev)))
    if out_mask is not None:
        post = (post, fwd, bwd)
    rows = B * T
    al = lambda n: ((n + 255) // 256) * 256
    fl = ws.view(torch.float32)
    U = fl[: rows * NP].view(B, T, NP)[..., :N]
    V = fl[rows * NP: 2 * rows * NP].view(B, T, NP)[..., :N]
    off = al(2 * rows * NP * 4) + al(2 * rows * 4)          # after U|V and LA|LB (hmm355.h)
    E = fl[off // 4: off // 4 + rows * NP].view(B, T, NP)[..., :N]
    offL = al(2 * rows * NP * 4) // 4
    LA = fl[offL: offL + rows].view(B, T)
    return post, loglik, lik_ref, U, V, E, LA


class TvSequenceLogLik(torch.autograd.Function):
    """(B,) log-likelihood of each sequence under per-step transition matrices
    (NeuralHMM.compute_likelihood, neural.py:513-519), differentiable in log_obs, log_A
    ((N,N) or (B,T,N,N)) and log_p0.  The adjoint of module docstring with the shifted
    emissions E_t = exp(log_obs_t - M_t) the tv kernels use: dL/d log_A_k = G exp(log_A_k)
    (X_{k+1} (x) Y_{k+1}) for the matrix k between steps k and k+1."""

    @staticmethod
    def forward(ctx, log_obs, log_A, log_p0, kind):
        from .ops import _tv_matrix
        nat.require_gpu(log_obs, log_A, log_p0)
        lo = log_obs.detach().to(torch.float32).contiguous()
        l0 = log_p0.detach().to(torch.float32).contiguous()
        B, T, N = lo.shape
        A, sb, st = _tv_matrix(log_A.detach(), B, T, N)
        _, loglik, lik_ref, _, _, _, _ = _run_tv_fb(lo, A, sb, st, l0)
        ctx.save_for_backward(lo, A, l0)
        ctx.sb, ctx.st, ctx.kind, ctx.static = sb, st, kind, log_A.dim() == 2
        return lik_ref if kind == "ref" else loglik

    @staticmethod
    def backward(ctx, gout):
        lo, A, l0 = ctx.saved_tensors
        B, T, N = lo.shape
        _, _, _, U, _, _, LA = _run_tv_fb(lo, A, ctx.sb, ctx.st, l0)
        a_last = torch.log(U[:, -1]) + LA[:, -1:]
        if ctx.kind == "ref":
            f = torch.exp(a_last)
            z = torch.log(f + 1e-8)
            w = torch.softmax(z, dim=-1)
            g = w * f / (f + 1e-8)
            log_mu = torch.log(w) - z
        else:
            g = torch.softmax(a_last, dim=-1)
            log_mu = torch.zeros_like(a_last)
        G = g.sum(-1) * gout
        post, _, _, U, V, E, _ = _run_tv_fb(lo, A, ctx.sb, ctx.st, l0, log_beta_T=log_mu.contiguous(), posterior=True)
        grad_lo = G[:, None, None] * post
        grad_l0 = (G[:, None] * post[:, 0]).sum(0)
        grad_A = None
        if ctx.needs_input_grad[1]:
            c = U.sum(-1)
            S = (U * V).sum(-1)
            X = U[:, :-1] / (c[:, :-1] * S[:, 1:]).unsqueeze(-1) * G[:, None, None]   # (B,T-1,N)
            Y = E[:, 1:] * V[:, 1:]                                                   # (B,T-1,N)
            if ctx.static:
                grad_A = torch.exp(A) * torch.einsum("bti,btj->ij", X, Y)
            else:
                Af = A if A.stride(1) != 0 else A.expand(B, T, N, N)
                grad_A = torch.zeros(B, T, N, N, device=lo.device)
                if T > 1:
                    grad_A[:, :-1] = torch.exp(Af[:, :-1]) * X.unsqueeze(-1) * Y.unsqueeze(-2)
        return grad_lo, grad_A, grad_l0, None


def _adjoint_sources(U, V, E, post, fwd, bwd, gp, gf, gb, CA=None, CB=None):
    """Per-step sources and scales of the two adjoint chains (ForwardBackwardFn's docstring):
    srcW = v (Gp - <gamma, Gp>) / sum(u v) + Gf exp(LA), srcZ = u (Gp - <gamma, Gp>) / sum(u v)
    + Gb exp(LB) (Gf exp(LA) = Gf forward / u), Fw_t = 1 / sum u_t, Fz_t = 1 / sum v_t E_t
    (t >= 1).  Formed in fp64 from the stored fp32 rows, returned as contiguous fp32.  The step
    factors are the chains' own normalisers CA / CB (hmm355.h; the dense chain's rows do not sum
    to 1, so they are not the row sums there)."""
    B, T, N = U.shape
    U64, V64 = U.double(), V.double()
    Suv = (U64 * V64).sum(-1, keepdim=True)
    srcW = torch.zeros(B, T, N, dtype=torch.float64, device=U.device)
    srcZ = torch.zeros_like(srcW)
    if gp is not None:
        g64 = gp.double()
        q = (g64 - (post.double() * g64).sum(-1, keepdim=True)) / torch.where(Suv > 0, Suv, torch.ones_like(Suv))
        q = torch.where(Suv > 0, q, torch.zeros_like(q))
        srcW += V64 * q
        srcZ += U64 * q
    if gf is not None:
        srcW += torch.where(U64 > 0, gf.double() * fwd.double() / torch.where(U64 > 0, U64, torch.ones_like(U64)),
                            torch.zeros_like(U64))
    if gb is not None:
        srcZ += torch.where(V64 > 0, gb.double() * bwd.double() / torch.where(V64 > 0, V64, torch.ones_like(V64)),
                            torch.zeros_like(V64))
    Fw = torch.zeros(B, T, device=U.device)                                    # 1/c_t (t <= T-2)
    Fz = torch.zeros(B, T, device=U.device)                                    # 1/c'_{t-1} (t >= 1)
    if T > 1:
        # (CA / CB None: chains that normalise every step exactly, c_t = sum u_t -- csrc/tv.hip)
        ca = CA[:, :-1].double() if CA is not None else U64[:, :-1].sum(-1)
        cb = CB[:, 1:].double() if CB is not None else (V64[:, 1:] * E[:, 1:].double()).sum(-1)
        Fw[:, :-1] = (1.0 / ca).float()
        Fz[:, 1:] = (1.0 / cb).float()
    return srcW.float().contiguous(), Fw, srcZ.float().contiguous(), Fz


class ForwardBackwardFn(torch.autograd.Function):
    """HMMPyTorch.forward_backward outputs (posterior, forward, backward) per `out_mask`,
    differentiable in obs, log_P and log_p0 — the reference back-propagates through its
    log-space loops (hmm.py:89-130; HMMLayer training mode hmm_layer.py:119-121, supervised
    compute_loss :159-165).  Forward: the gfx950 chains, keeping their scaled rows
    (alpha_t = U_t exp(LA_t), beta_t = V_t exp(LB_t)).  Backward: the analytic adjoint.

    With a = log alpha, b = log beta, gamma = exp(a + b - LSE(a + b)) and output gradients
    Gp, Gf, Gb, the direct adjoints are
        h_t = gamma_t (Gp_t - <gamma_t, Gp_t>) + Gf_t exp(a_t)     (of a_t)
        k_t = gamma_t (Gp_t - <gamma_t, Gp_t>) + Gb_t exp(b_t)     (of b_t).
    The total adjoint of a_t is alpha_t * W_t e^{-LA_t}, W the forward recursion's adjoint in
    alpha's scaling, and that of b_t is beta_t * Z_t e^{-LB_t}:
        W_{t-1} = h_{t-1} / u_{t-1} + (1/c_{t-1}) A (E_t W_t),          c_t = CA_t
        Z_{t+1} = k_{t+1} / v_{t+1} + (1/c'_t) E_{t+1} (A^T Z_t),       c'_t = CB_{t+1}
    with c, c' the chains' step normalisers (u_{t+1} = A^T u_t E_{t+1} / c_t, v_t = A E_{t+1}
    v_{t+1} / c'_t; hmm355.h workspace CA / CB)
    (hmm355_fb_adjoint_f32), where h/u = v (Gp - <.,.>) / sum(u v) + Gf exp(LA) and
    k/v = u (Gp - <.,.>) / sum(u v) + Gb exp(LB) are O(1) (no division by a vanishing u or v).
    Then, with P = Z - k/v the propagated part of Z,
        dL/d log_obs_t = u_t W_t + v_t P_t
        dL/d log_p0    = sum_b u_0 W_0
        dL/d log_P     = exp(log_P) * sum_{b,t} [ (u_{t-1}/c_{t-1}) (x) (E_t W_t)
                                                 + Z_t (x) (E_{t+1} v_{t+1} / c'_t) ]
    (two GEMMs over the frames, hipBLASLt through torch)."""

    @staticmethod
    def forward(ctx, obs, log_P, log_p0, obs_mode, out_mask, plan=None):
        nat.require_gpu(obs, log_P, log_p0)
        obs_c, lP, l0 = (t.detach().to(torch.float32).contiguous() for t in (obs, log_P, log_p0))
        outs, _, _, U, V, _, _, CA, CB = _run_fb(obs_c, lP, l0, obs_mode, out_mask=out_mask | nat.FB_POSTERIOR,
                                                 plan=plan)
        post, fwd, bwd = outs
        ctx.save_for_backward(obs_c, lP, l0, U, V, post, fwd, bwd, CA, CB)
        ctx.obs_mode, ctx.out_mask = obs_mode, out_mask
        ctx.set_materialize_grads(False)   # outputs the loss does not use arrive as None
        res = tuple(o for bit, o in ((nat.FB_POSTERIOR, post), (nat.FB_FORWARD, fwd), (nat.FB_BACKWARD, bwd))
                    if out_mask & bit)
        return res

    @staticmethod
    def backward(ctx, *grads):
        obs, lP, l0, U, V, post, fwd, bwd, CA, CB = ctx.saved_tensors
        B, T, N = obs.shape
        returned = [k for bit, k in ((nat.FB_POSTERIOR, "p"), (nat.FB_FORWARD, "f"), (nat.FB_BACKWARD, "b"))
                    if ctx.out_mask & bit]
        got = dict(zip(returned, grads))
        gp, gf, gb = got.get("p"), got.get("f"), got.get("b")
        E = _staged_emissions(obs, ctx.obs_mode).contiguous()
        srcW, Fw, srcZ, Fz = _adjoint_sources(U, V, E, post, fwd, bwd, gp, gf, gb, CA, CB)
        W = torch.empty(B, T, N, device=obs.device)
        P = torch.empty(B, T, N, device=obs.device)
        L = nat.lib()
        with torch.cuda.device(obs.device):
            nat.check(L.hmm355_fb_adjoint_f32(nat.ptr(E), nat.ptr(lP), nat.ptr(srcW), nat.ptr(Fw), nat.ptr(srcZ),
                                              nat.ptr(Fz), B, T, N, nat.ptr(W), nat.ptr(P),
                                              nat.stream_of(obs.device)))
        grad_lo = U * W + V * P
        grad_obs = grad_lo / (obs + 1e-8) if ctx.obs_mode == nat.OBS_PROB else grad_lo
        grad_l0 = (U[:, 0] * W[:, 0]).sum(0)
        grad_lP = None
        if ctx.needs_input_grad[1]:
            M = torch.zeros(N, N, device=obs.device)
            if T > 1:
                X1 = U[:, :-1] * Fw[:, :-1, None]
                Y1 = E[:, 1:] * W[:, 1:]
                Z = srcZ + P
                Y2 = E[:, 1:] * V[:, 1:] * Fz[:, 1:, None]
                M = torch.einsum("bti,btj->ij", X1, Y1) + torch.einsum("bti,btj->ij", Z[:, :-1], Y2)
            grad_lP = torch.exp(lP) * M
        return grad_obs, grad_lP, grad_l0, None, None, None


class TvForwardBackwardFn(torch.autograd.Function):
    """NeuralHMM.forward outputs (posterior, forward, backward) per `out_mask` under per-step
    transition matrices, differentiable in log_obs, log_A ((N,N) or (B,T,N,N)) and log_p0 —
    the reference back-propagates through its per-step logsumexp loops (neural.py:391-461).
    Forward: csrc/tv.hip's chains (log-emissions staged as E_t = exp(lo_t - M_t)).  Backward:
    ForwardBackwardFn's adjoint with the step's own matrix: hmm355_tv_fb_adjoint_f32 runs the
    W / Z chains streaming A_k = exp(log_A_k) as the forward does, then
        dL/d log_obs_t = u_t W_t + v_t P_t,   dL/d log_p0 = sum_b u_0 W_0,
        dL/d log_A_k   = exp(log_A_k) * [ (u_k / c_k) (x) (E_{k+1} W_{k+1})
                                          + Z_k (x) (E_{k+1} v_{k+1} / c'_k) ]   (k <= T-2; 0 at k = T-1)
    (summed over (b, k) for one static matrix)."""

    @staticmethod
    def forward(ctx, log_obs, log_A, log_p0, out_mask):
        from .ops import _tv_matrix
        nat.require_gpu(log_obs, log_A, log_p0)
        lo = log_obs.detach().to(torch.float32).contiguous()
        l0 = log_p0.detach().to(torch.float32).contiguous()
        B, T, N = lo.shape
        A, sb, st = _tv_matrix(log_A.detach(), B, T, N)
        outs, _, _, U, V, E, _ = _run_tv_fb(lo, A, sb, st, l0, out_mask=out_mask | nat.FB_POSTERIOR)
        post, fwd, bwd = outs
        ctx.save_for_backward(lo, A, l0, U, V, E, post, fwd, bwd)
        ctx.sb, ctx.st, ctx.static, ctx.out_mask = sb, st, log_A.dim() == 2, out_mask
        ctx.a_shape = tuple(log_A.shape)
        ctx.set_materialize_grads(False)
        return tuple(o for bit, o in ((nat.FB_POSTERIOR, post), (nat.FB_FORWARD, fwd), (nat.FB_BACKWARD, bwd))
                     if out_mask & bit)

    @staticmethod
    def backward(ctx, *grads):
        lo, A, l0, U, V, E, post, fwd, bwd = ctx.saved_tensors
        B, T, N = lo.shape
        returned = [k for bit, k in ((nat.FB_POSTERIOR, "p"), (nat.FB_FORWARD, "f"), (nat.FB_BACKWARD, "b"))
                    if ctx.out_mask & bit]
        got = dict(zip(returned, grads))
        E = E.contiguous()
        srcW, Fw, srcZ, Fz = _adjoint_sources(U, V, E, post, fwd, bwd, got.get("p"), got.get("f"), got.get("b"))
        W = torch.empty(B, T, N, device=lo.device)
        P = torch.empty(B, T, N, device=lo.device)
        L = nat.lib()
        with torch.cuda.device(lo.device):
            nat.check(L.hmm355_tv_fb_adjoint_f32(nat.ptr(E), nat.ptr(A), ctx.sb, ctx.st, nat.ptr(srcW), nat.ptr(Fw),
                                                 nat.ptr(srcZ), nat.ptr(Fz), B, T, N, nat.ptr(W), nat.ptr(P),
                                                 nat.stream_of(lo.device)))
        grad_lo = U * W + V * P
        grad_l0 = (U[:, 0] * W[:, 0]).sum(0)
        grad_A = None
        if ctx.needs_input_grad[1]:
            if ctx.static:
                M = torch.zeros(N, N, device=lo.device)
                if T > 1:
                    X1 = U[:, :-1] * Fw[:, :-1, None]
                    Y1 = E[:, 1:] * W[:, 1:]
                    Y2 = E[:, 1:] * V[:, 1:] * Fz[:, 1:, None]
                    M = torch.einsum("bti,btj->ij", X1, Y1) + torch.einsum("bti,btj->ij", (srcZ + P)[:, :-1], Y2)
                grad_A = torch.exp(A) * M
            else:
                # matrices k = 0 .. T-2 are used; any further ones (log_A may carry T or more
                # steps, neural.py:377-381) get a zero gradient
                grad_A = torch.zeros(ctx.a_shape, device=lo.device)
                if T > 1:
                    # both outer products of a step as one K = 2 batched GEMM, then * exp(log_A_k)
                    Lf = torch.stack([U[:, :-1] * Fw[:, :-1, None], (srcZ + P)[:, :-1]], -1)        # (B,T-1,N,2)
                    Rf = torch.stack([E[:, 1:] * W[:, 1:], E[:, 1:] * V[:, 1:] * Fz[:, 1:, None]], -2)  # (B,T-1,2,N)
                    g = torch.matmul(Lf, Rf)
                    g.mul_(torch.exp(A.expand(ctx.a_shape)[:, :T - 1]))
                    grad_A[:, :T - 1] = g
        return grad_lo, grad_A, grad_l0, None


def tv_forward_backward_with_grad(log_obs, log_A, log_p0, out_mask):
    """Differentiable NeuralHMM forward-backward outputs (tuple per out_mask)."""
    return TvForwardBackwardFn.apply(log_obs, log_A, log_p0, out_mask)


def forward_backward_with_grad(obs, log_P, log_p0, obs_mode, out_mask, plan=None):
    """Differentiable forward-backward outputs (tuple per out_mask: posterior, forward, backward)."""
    return ForwardBackwardFn.apply(obs, log_P, log_p0, obs_mode, out_mask, plan)


class GmmLogProb(torch.autograd.Function):
    """Diagonal-Gaussian (mixture) emission log-probabilities: forward by the gfx950 scorer
    (ops.gmm_diag_logprob), backward analytic.  With comp[b,t,s,c] the component log-density
    plus log_w and r = d lp / d comp (softmax over c of the reference's clamped LSE,
    mixture_gaussian.py:141-155; r = 1 when mix_lse == 0):
        d/d means   = r g (x - mu) / var          d/d log_vars = r g ((x - mu)^2 / var - 1) / 2
        d/d x       = -sum_{s,c} r g (x - mu) / var                d/d log_w = r g
    expanded into GEMMs over the frames (hipBLASLt through torch.matmul), T-chunked."""

    @staticmethod
    def forward(ctx, x, means, log_vars, log_w, mix_lse):
        from . import ops
        lp = ops.gmm_diag_logprob(x.detach(), means.detach(), log_vars.detach(), log_w.detach(), mix_lse)
        ctx.save_for_backward(x, means, log_vars, log_w, lp)
        ctx.mix_lse = mix_lse
        return lp

    @staticmethod
    def backward(ctx, g):
        x, means, log_vars, log_w, lp = ctx.saved_tensors
        B, T, D = x.shape
        S, C, _ = means.shape
        mu = means.detach().float().reshape(S * C, D)
        lv = log_vars.detach().float().reshape(S * C, D)
        iv = torch.exp(-lv)                                   # 1 / var
        cst = lv.sum(-1) + D * math.log(2 * math.pi)          # (SC)
        lw = log_w.detach().float().reshape(S * C)
        q2 = (mu * mu * iv).sum(-1)                           # sum mu^2 / var
        gm = torch.zeros_like(mu)      # sum gc (x - mu) / var  pieces
        gx2 = torch.zeros_like(mu)     # sum gc x^2
        gx1 = torch.zeros_like(mu)     # sum gc x
        gsum = torch.zeros(S * C, device=x.device)
        grad_x = torch.empty_like(x, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        step = max(1, (1 << 22) // max(1, B * S * C))       # frames-of-T per chunk (bounded temp)
        xf = x.detach().float()
        for t0 in range(0, T, step):
            xc = xf[:, t0:t0 + step].reshape(-1, D)           # (F, D)
            gl = g[:, t0:t0 + step].reshape(-1, S).float()    # (F, S)
            maha = (xc * xc) @ iv.t() - 2.0 * (xc @ (mu * iv).t()) + q2   # (F, SC)
            comp = -0.5 * (maha + cst) + lw
            if ctx.mix_lse:
                comp3 = comp.view(-1, S, C)
                m = comp3.max(-1, keepdim=True)[0]
                m = torch.where(torch.isinf(m), torch.zeros_like(m), m)
                ex = torch.exp(comp3 - m)
                se = ex.sum(-1, keepdim=True)
                r = torch.where(se > 1e-8, ex / se, torch.zeros_like(ex))   # clamp(min=1e-8) has 0 slope below
                gc = (r * gl.unsqueeze(-1)).reshape(-1, S * C)
            else:
                gc = gl.reshape(-1, S * C)
            gsum += gc.sum(0)
            gx1 += gc.t() @ xc
            gx2 += gc.t() @ (xc * xc)
            if grad_x is not None:
                gxx = -(xc * (gc @ iv) - gc @ (mu * iv))
                grad_x[:, t0:t0 + step] = gxx.view(B, -1, D)
        grad_means = (gx1 - mu * gsum[:, None]) * iv
        grad_lv = 0.5 * ((gx2 - 2 * mu * gx1 + mu * mu * gsum[:, None]) * iv - gsum[:, None])
        return (grad_x, grad_means.view(S, C, D).to(means.dtype), grad_lv.view(S, C, D).to(log_vars.dtype),
                gsum.view(S, C).to(log_w.dtype), None)


class ViterbiScore(torch.autograd.Function):
    """(states, max_j delta_{T-1}[j]) of the Viterbi recursion (ops.viterbi, OBS_LOG), with the
    gradient of the score: the reference's max-plus recursion (mixture_gaussian.py:290-338)
    routes it along the decoded path only — d/d lp[b,t,s_t] = g_b, d/d log_T[s_{t-1},s_t] += g_b."""

    @staticmethod
    def forward(ctx, lp, log_T, init, plan=None):
        from . import ops
        states, _, final = ops.viterbi(lp.detach(), log_T.detach(), init.detach(), ops.OBS_LOG, plan)
        ctx.save_for_backward(states)
        ctx.shapes = (lp.shape, log_T.shape)
        ctx.mark_non_differentiable(states)
        return states, final

    @staticmethod
    def backward(ctx, g_states, g):
        (states,) = ctx.saved_tensors
        (B, T, S), _ = ctx.shapes
        grad_lp = torch.zeros(B, T, S, device=g.device)
        grad_lp.scatter_(2, states.unsqueeze(-1), g.view(B, 1, 1).expand(B, T, 1).contiguous())
        grad_T = torch.zeros(S * S, device=g.device)
        if T > 1:
            idx = (states[:, :-1] * S + states[:, 1:]).reshape(-1)
            grad_T.index_add_(0, idx, g.view(B, 1).expand(B, T - 1).reshape(-1))
        grad_init = torch.zeros(S, device=g.device).index_add_(0, states[:, 0], g)
        return grad_lp, grad_T.view(S, S), grad_init, None
