"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference hot path (the parity oracle).

Every function below restates one reference routine in torch-CPU ops, in the reference's
op order, so that on the same machine its outputs are bit-identical to the reference's
(pinned by tests/golden/*.npz, produced by the reference itself via
tests/golden/make_golden.py).  Citations are file:line into crlotwhite/pytorch_hmm
(/root/reference/pytorch_hmm).  The product (pytorch_hmm_amd) never imports this module.
"""
import ctypes
import math
import os
import subprocess

import numpy as np
import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------- params
def transition_matrix(num_states, transition_type="ergodic", self_loop_prob=0.5,
                      forward_prob=0.4, skip_prob=0.1):
    """utils.py:9-77 (create_transition_matrix)."""
    K = num_states
    if transition_type == "ergodic":
        P = torch.ones(K, K) + torch.eye(K) * self_loop_prob * K
    else:
        P = torch.zeros(K, K)
        for i in range(K):
            if transition_type == "left_to_right":
                if i < K - 1:
                    P[i, i], P[i, i + 1] = self_loop_prob, forward_prob
                else:
                    P[i, i] = 1.0
            elif transition_type == "left_to_right_skip":
                if i < K - 2:
                    P[i, i], P[i, i + 1], P[i, i + 2] = self_loop_prob, forward_prob, skip_prob
                elif i < K - 1:
                    P[i, i], P[i, i + 1] = self_loop_prob, forward_prob
                else:
                    P[i, i] = 1.0
            elif transition_type == "circular":
                P[i, i] = self_loop_prob
                P[i, (i + 1) % K] = forward_prob
            else:
                raise ValueError(f"Unknown transition_type: {transition_type}")
    return P / P.sum(dim=1, keepdim=True)


def left_to_right_matrix(num_states, self_loop_prob=0.7):
    """utils.py:80-103."""
    return transition_matrix(num_states, "left_to_right", self_loop_prob, 1.0 - self_loop_prob)


def hmm_params(P, p0=None):
    """hmm.py:20-55: renormalise P, log(P+1e-8); p0 uniform or renormalised, log(p0+1e-8)."""
    if isinstance(P, np.ndarray):
        P = torch.from_numpy(P).float()
    K = P.shape[0]
    P = P / P.sum(dim=1, keepdim=True)
    log_P = torch.log(P + 1e-8)
    if p0 is None:
        p0 = torch.ones(K) / K
    else:
        if isinstance(p0, np.ndarray):
            p0 = torch.from_numpy(p0).float()
        p0 = p0 / p0.sum()
    return log_P, torch.log(p0 + 1e-8)


def hmmlayer_params(logits, init_logits, first_call):
    """hmm_layer.py:61-89: softmax params; call 1 goes through HMM.__init__ (renormalises),
    later calls assign log(P+1e-8) directly."""
    P = F.softmax(logits, dim=1)
    p0 = F.softmax(init_logits, dim=0)
    if first_call:
        return hmm_params(P, p0)
    return torch.log(P + 1e-8), torch.log(p0 + 1e-8)


# ------------------------------------------------------------------- forward-backward
def forward_backward(obs, log_P, log_p0):
    """hmm.py:66-130.  Returns posterior, forward, backward (each (B,T,K), probability
    domain, NOT squeezed) plus the internal log_alpha / log_beta."""
    if obs.dim() == 2:
        obs = obs.unsqueeze(0)
    B, T, K = obs.shape
    log_obs = torch.log(obs + 1e-8)
    la = torch.zeros(B, T, K)
    la[:, 0] = log_p0 + log_obs[:, 0]
    for t in range(1, T):
        la[:, t] = torch.logsumexp(la[:, t - 1, :, None] + log_P[None, :, :], dim=1) + log_obs[:, t]
    lb = torch.zeros(B, T, K)
    lb[:, -1] = 0.0
    for t in range(T - 2, -1, -1):
        lb[:, t] = torch.logsumexp(log_P[None, :, :] + log_obs[:, t + 1, None, :]
                                   + lb[:, t + 1, None, :], dim=2)
    lp = la + lb
    lp = lp - torch.logsumexp(lp, dim=-1, keepdim=True)
    return torch.exp(lp), torch.exp(la), torch.exp(lb), la, lb


def compute_likelihood(obs, log_P, log_p0):
    """hmm.py:186-211 (saturates once exp(log_alpha) underflows, as the reference does)."""
    squeeze = obs.dim() == 2
    _, fwd, _, _, _ = forward_backward(obs, log_P, log_p0)
    ll = torch.logsumexp(torch.log(fwd[:, -1] + 1e-8), dim=-1)
    return ll.squeeze(0) if squeeze else ll


# ---------------------------------------------------------------------------- Viterbi
def viterbi_decode(obs, log_P, log_p0):
    """hmm.py:132-184 (first-index ties; 2-D input squeezed)."""
    squeeze = obs.dim() == 2
    if squeeze:
        obs = obs.unsqueeze(0)
    return viterbi_from_log(torch.log(obs + 1e-8), log_P, log_p0, squeeze)


def viterbi_from_log(log_obs, log_P, init, squeeze=False):
    B, T, K = log_obs.shape
    delta = torch.zeros(B, T, K)
    psi = torch.zeros(B, T, K, dtype=torch.long)
    delta[:, 0] = init + log_obs[:, 0]
    for t in range(1, T):
        delta[:, t], psi[:, t] = torch.max(delta[:, t - 1, :, None] + log_P[None, :, :], dim=1)
        delta[:, t] += log_obs[:, t]
    states = torch.zeros(B, T, dtype=torch.long)
    states[:, -1] = torch.argmax(delta[:, -1], dim=1)
    for t in range(T - 2, -1, -1):
        states[:, t] = psi[torch.arange(B), t + 1, states[:, t + 1]]
    if squeeze:
        return states.squeeze(0), delta.squeeze(0)
    return states, delta


# ------------------------------------------------------ NeuralHMM (time-varying transitions)
def neural_forward_backward(log_obs, log_trans, log_init):
    """neural.py:391-461: forward step t uses log_trans[:, t-1] (:419-427), backward step t
    log_trans[:, t] (:449-458); log_trans (B,T,K,K).  Returns posterior, forward, backward and
    the internal log_forward / log_backward."""
    B, T, K = log_obs.shape
    if log_trans.dim() == 2:  # the static matrix expanded over (B,T), neural.py:385
        log_trans = log_trans.unsqueeze(0).unsqueeze(0).expand(B, T, -1, -1)
    lf = torch.full((B, T, K), float("-inf"))
    lf[:, 0] = log_init + log_obs[:, 0]
    for t in range(1, T):
        lf[:, t] = torch.logsumexp(lf[:, t - 1].unsqueeze(-1) + log_trans[:, t - 1], dim=1) + log_obs[:, t]
    lb = torch.full((B, T, K), float("-inf"))
    lb[:, -1] = 0.0
    for t in range(T - 2, -1, -1):
        comb = log_trans[:, t] + log_obs[:, t + 1].unsqueeze(1) + lb[:, t + 1].unsqueeze(1)
        lb[:, t] = torch.logsumexp(comb, dim=-1)
    lp = lf + lb
    lp = lp - torch.logsumexp(lp, dim=-1, keepdim=True)
    return torch.exp(lp), torch.exp(lf), torch.exp(lb), lf, lb


def neural_viterbi(log_obs, log_trans, log_init):
    """neural.py:463-511 (states (B,T), log_delta (B,T,K))."""
    B, T, K = log_obs.shape
    if log_trans.dim() == 2:
        log_trans = log_trans.unsqueeze(0).unsqueeze(0).expand(B, T, -1, -1)
    delta = torch.full((B, T, K), float("-inf"))
    psi = torch.zeros((B, T, K), dtype=torch.long)
    delta[:, 0] = log_init + log_obs[:, 0]
    for t in range(1, T):
        delta[:, t], psi[:, t] = torch.max(delta[:, t - 1].unsqueeze(-1) + log_trans[:, t - 1], dim=1)
        delta[:, t] += log_obs[:, t]
    states = torch.zeros((B, T), dtype=torch.long)
    states[:, -1] = torch.argmax(delta[:, -1], dim=1)
    for t in range(T - 2, -1, -1):
        states[:, t] = psi[torch.arange(B), t + 1, states[:, t + 1]]
    return states, delta


# --------------------------------------------------------------------- Gaussian layer
def gaussian_log_probs(x, means, log_scales, covariance_type="diag"):
    """hmm_layer.py:270-323."""
    B, T, D = x.shape
    diff = x.unsqueeze(-2) - means.unsqueeze(0).unsqueeze(0)
    if covariance_type == "spherical":
        log_var = 2 * log_scales
        var = torch.exp(log_var)
        mahal = torch.sum(diff ** 2, dim=-1) / var.squeeze(-1)
        log_norm = -0.5 * (D * np.log(2 * np.pi) + D * log_var.squeeze(-1))
    else:
        if covariance_type == "full":
            log_var = 2 * torch.diagonal(log_scales, dim1=-2, dim2=-1)
        else:
            log_var = 2 * log_scales
        var = torch.exp(log_var)
        mahal = torch.sum(diff ** 2 / var.unsqueeze(0).unsqueeze(0), dim=-1)
        log_norm = -0.5 * (D * np.log(2 * np.pi) + torch.sum(log_var, dim=-1))
    return log_norm.unsqueeze(0).unsqueeze(0) - 0.5 * mahal


# ---------------------------------------------------------------------- mixture layer
def _safe_log(x, eps=1e-8):
    return torch.log(torch.clamp(x, min=eps))                       # mixture_gaussian.py:137-139


def _mix_lse(x, dim):
    """mixture_gaussian.py:141-155."""
    m = torch.max(x, dim=dim, keepdim=True)[0]
    m = torch.where(torch.isinf(m), torch.zeros_like(m), m)
    s = torch.sum(torch.exp(x - m), dim=dim, keepdim=False)
    return _safe_log(s) + m.squeeze(dim)


def mixture_log_probs(x, mixture_weights_logits, means, log_vars, t_chunk=None, covariance_type="diag"):
    """mixture_gaussian.py:157-214 (diag :200-214, tied :242-253, spherical :255-269).  t_chunk
    evaluates the (B,T,S,C,D) broadcast in slices of T (identical per-element ops; bounds host
    memory at full size)."""
    B, T, D = x.shape
    log_w = _safe_log(F.softmax(mixture_weights_logits, dim=-1))
    var = torch.exp(log_vars)
    outs = []
    step = T if not t_chunk else t_chunk
    for t0 in range(0, T, step):
        xe = x[:, t0:t0 + step].unsqueeze(2).unsqueeze(3)
        diff = xe - means.unsqueeze(0).unsqueeze(0)
        if covariance_type == "diag":
            const = torch.sum(log_vars, dim=-1).unsqueeze(0).unsqueeze(0)
            comp = -0.5 * (torch.sum(diff ** 2 / var.unsqueeze(0).unsqueeze(0), dim=-1) + const
                           + D * math.log(2 * math.pi))
        elif covariance_type == "tied":
            comp = -0.5 * (torch.sum(diff ** 2 / var.unsqueeze(0).unsqueeze(0).unsqueeze(0).unsqueeze(0), dim=-1)
                           + torch.sum(log_vars) + D * math.log(2 * math.pi))
        elif covariance_type == "spherical":
            ve = var.unsqueeze(0).unsqueeze(0).unsqueeze(-1)
            comp = -0.5 * (torch.sum(diff ** 2, dim=-1) / ve.squeeze(-1)
                           + D * log_vars.unsqueeze(0).unsqueeze(0) + D * math.log(2 * math.pi))
        else:
            raise ValueError(covariance_type)
        outs.append(_mix_lse(comp + log_w.unsqueeze(0).unsqueeze(0), dim=-1))
    return torch.cat(outs, dim=1)


def mixture_log_transitions(transition_logits):
    """mixture_gaussian.py:130-135 + :357."""
    return _safe_log(F.softmax(transition_logits, dim=-1))


def mixture_viterbi(lp, log_T):
    """mixture_gaussian.py:290-338: delta_0 = lp_0 - log(S); returns (states, max delta_{T-1})."""
    B, T, S = lp.shape
    init = torch.zeros(S) - math.log(S)
    states, delta = viterbi_from_log(lp, log_T, init)
    final_scores = torch.max(delta[:, -1, :], dim=-1)[0]
    return states, final_scores


def mixture_init_vector(S):
    """The value the reference subtracts at t=0 (obs_log_probs[:,0,:] - math.log(S)) as the
    additive init vector the kernels take: lp + (-c) == lp - c exactly in IEEE fp32."""
    return -(torch.zeros(S) + math.log(S))


# ------------------------------------------------------------------------ HSMM layer
def hsmm_log_probs(x, means, log_vars):
    """hsmm.py:181-206."""
    D = x.shape[-1]
    diff = x.unsqueeze(2) - means.unsqueeze(0).unsqueeze(0)
    var = torch.exp(log_vars).unsqueeze(0).unsqueeze(0)
    return -0.5 * (torch.sum(diff ** 2 / var, dim=-1)
                   + torch.sum(log_vars, dim=-1).unsqueeze(0).unsqueeze(0) + D * math.log(2 * math.pi))


def hsmm_duration_log_probs(shape_p, rate_p, min_duration, max_duration, eps=1e-8):
    """hsmm.py:115-143 (gamma) then log(p + eps) (hsmm.py:226-227)."""
    d = torch.arange(min_duration, max_duration + 1, dtype=torch.float).unsqueeze(0)
    shape = F.softplus(shape_p).unsqueeze(1)
    rate = F.softplus(rate_p).unsqueeze(1)
    lp = ((shape - 1) * torch.log(d + eps) - rate * d - torch.lgamma(shape)
          + shape * torch.log(rate + eps))
    lp = torch.where(d >= min_duration, lp, torch.full_like(lp, float("-inf")))
    return torch.log(torch.exp(lp) + eps)


def hsmm_log_transitions(transition_logits, eps=1e-8):
    """hsmm.py:108-113 then log(p + eps) (hsmm.py:228-229)."""
    logits = transition_logits.clone()
    logits.fill_diagonal_(float("-inf"))
    return torch.log(F.softmax(logits, dim=-1) + eps)


# --------------------------------------------------------------- C oracle (ctypes)
_lib = None


def c_oracle():
    """Load (building if needed) oracle/lib/liboracle.so."""
    global _lib
    if _lib is not None:
        return _lib
    so = os.path.join(_HERE, "lib", "liboracle.so")
    src = os.path.join(_HERE, "hmm_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    lib = ctypes.CDLL(so)
    P = ctypes.c_void_p
    I = ctypes.c_int
    lib.viterbi_f32.argtypes = [P, P, P, I, I, I, P, P, P]
    lib.fb_f64.argtypes = [P, P, P, I, I, I, P, P, P, P]
    lib.gmm_diag_f64.argtypes = [P, P, P, P, I, I, I, I, I, P]
    L = ctypes.c_longlong
    lib.tv_viterbi_f32.argtypes = [P, P, L, L, P, I, I, I, P, P]
    lib.tv_fb_f64.argtypes = [P, P, L, L, P, I, I, I, P, P, P, P]
    lib.hsmm_viterbi_literal.argtypes = [P, P, P, I, I, I, P, P]
    lib.hsmm_viterbi_fast.argtypes = [P, P, P, I, I, I, P, P]
    lib.torch_sum_f32.argtypes = [P, ctypes.c_ssize_t, ctypes.c_longlong]
    lib.torch_sum_f32.restype = ctypes.c_float
    lib.smk_quad_f32.argtypes = [P, P, P, I, I, I, P]
    lib.smk_viterbi_literal.argtypes = [P, P, P, P, P, I, I, I, P, P, P]
    lib.smk_viterbi_literal.restype = I
    lib.smk_forward_f64.argtypes = [P, P, P, P, P, I, I, I, P]
    lib.smk_forward_f64.restype = ctypes.c_double
    lib.stream_greedy_f32.argtypes = [P, P, I, ctypes.c_float, I, I, P, P]
    lib.stream_beam_f32.argtypes = [P, P, I, I, I, P, P, P, I, P, P]
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def c_viterbi(log_obs, log_P, init):
    lo = _f32(log_obs)
    B, T, N = lo.shape
    lP, it = _f32(log_P), _f32(init)
    states = np.zeros((B, T), np.int64)
    delta = np.zeros((B, T, N), np.float32)
    psi = np.zeros((B, T, N), np.uint8)
    c_oracle().viterbi_f32(_p(lo), _p(lP), _p(it), B, T, N, _p(states), _p(delta), _p(psi))
    return states, delta, psi


def c_fb64(log_obs, log_P, log_p0):
    lo = _f32(log_obs)
    B, T, N = lo.shape
    la = np.zeros((B, T, N)); lb = np.zeros((B, T, N)); post = np.zeros((B, T, N))
    ll = np.zeros(B)
    c_oracle().fb_f64(_p(lo), _p(_f32(log_P)), _p(_f32(log_p0)), B, T, N, _p(la), _p(lb), _p(post), _p(ll))
    return la, lb, post, ll


def _tv_strides(log_A, B, T, N):
    """(contiguous array, batch stride, step stride) for log_A of shape (N,N) or (B,T,N,N)."""
    A = _f32(log_A)
    if A.ndim == 2:
        return A, 0, 0
    assert A.shape == (B, T, N, N), A.shape
    return A, T * N * N, N * N


def c_tv_viterbi(log_obs, log_A, init):
    lo = _f32(log_obs)
    B, T, N = lo.shape
    A, sb, st = _tv_strides(log_A, B, T, N)
    states = np.zeros((B, T), np.int64)
    delta = np.zeros((B, T, N), np.float32)
    c_oracle().tv_viterbi_f32(_p(lo), _p(A), sb, st, _p(_f32(init)), B, T, N, _p(states), _p(delta))
    return states, delta


def c_tv_fb64(log_obs, log_A, log_p0):
    lo = _f32(log_obs)
    B, T, N = lo.shape
    A, sb, st = _tv_strides(log_A, B, T, N)
    la = np.zeros((B, T, N)); lb = np.zeros((B, T, N)); post = np.zeros((B, T, N))
    ll = np.zeros(B)
    c_oracle().tv_fb_f64(_p(lo), _p(A), sb, st, _p(_f32(log_p0)), B, T, N, _p(la), _p(lb), _p(post), _p(ll))
    return la, lb, post, ll


def c_gmm64(x, means, log_vars, log_w):
    x = _f32(x)
    B, T, D = x.shape
    S, C, _ = means.shape
    out = np.zeros((B, T, S))
    c_oracle().gmm_diag_f64(_p(x), _p(_f32(means)), _p(_f32(log_vars)), _p(_f32(log_w)),
                            B, T, D, S, C, _p(out))
    return out


def c_hsmm(lp, dur_lp, log_T, literal=False, workers=1):
    """lp (B,T,S); returns states (B,T) int64 and scores (B,) float32.  `workers` > 1 runs the
    sequences on that many threads (ctypes releases the GIL)."""
    lp = _f32(lp)
    B, T, S = lp.shape
    Dm = dur_lp.shape[1]
    du, lT = _f32(dur_lp), _f32(log_T)
    states = np.zeros((B, T), np.int64)
    scores = np.zeros(B, np.float32)
    fn = c_oracle().hsmm_viterbi_literal if literal else c_oracle().hsmm_viterbi_fast

    def one(b):
        lpb = np.ascontiguousarray(lp[b])
        sb = np.zeros(T, np.int64)
        sc = np.zeros(1, np.float32)
        fn(_p(lpb), _p(du), _p(lT), T, S, Dm, _p(sb), _p(sc))
        states[b], scores[b] = sb, sc[0]

    if workers > 1 and B > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=min(workers, B)) as ex:
            list(ex.map(one, range(B)))
    else:
        for b in range(B):
            one(b)
    return states, scores


def c_torch_sum(col):
    """torch.sum of a 1-D float32 view (any stride), in torch-CPU's cascade order
    (oracle/hmm_oracle.c torch_sum_f32; reference hsmm.py:273,285)."""
    a = np.asarray(col)
    assert a.dtype == np.float32 and a.ndim == 1
    stride = a.strides[0] // 4 if a.size > 1 else 1
    return np.float32(c_oracle().torch_sum_f32(a.ctypes.data_as(ctypes.c_void_p), stride, a.size))


def c_smk_quad(x, means, var):
    """x (T,D), means/var (S,D) -> q (T,S) float32 (k ascending)."""
    x, mu, va = _f32(x), _f32(means), _f32(var)
    T, D = x.shape
    S = mu.shape[0]
    q = np.zeros((T, S), np.float32)
    c_oracle().smk_quad_f32(_p(x), _p(mu), _p(va), T, D, S, _p(q))
    return q


def c_smk_viterbi(q, seg_const, log_init, log_T, dur_lp):
    """One sequence: q (T,S) -> (segment states, segment durations, score) (semi_markov.py:455-570)."""
    q = _f32(q)
    T, S = q.shape
    Dm = dur_lp.shape[1]
    cs = None if seg_const is None else _f32(seg_const)
    ss = np.zeros(T, np.int64)
    sd = np.zeros(T, np.int64)
    sc = np.zeros(1, np.float32)
    n = c_oracle().smk_viterbi_literal(_p(q), None if cs is None else _p(cs), _p(_f32(log_init)),
                                       _p(_f32(log_T)), _p(_f32(dur_lp)), T, S, Dm, _p(ss), _p(sd), _p(sc))
    return ss[:n], sd[:n], sc[0]


def c_smk_forward64(q, seg_const, log_init, log_T, dur_lp):
    """One sequence: -> (log P(o), log alpha (T,S,Dmax) float64)."""
    q = _f32(q)
    T, S = q.shape
    Dm = dur_lp.shape[1]
    cs = None if seg_const is None else _f32(seg_const)
    la = np.zeros((T, S, Dm))
    tot = c_oracle().smk_forward_f64(_p(q), None if cs is None else _p(cs), _p(_f32(log_init)),
                                     _p(_f32(log_T)), _p(_f32(dur_lp)), T, S, Dm, _p(la))
    return tot, la


def c_stream_greedy(emis, log_T, prev, log_n):
    """emis (T,N) -> states (T,) int64, scores (T,) float32 (streaming.py:267-320)."""
    e = _f32(emis)
    T, N = e.shape
    st = np.zeros(T, np.int64)
    sc = np.zeros(T, np.float32)
    c_oracle().stream_greedy_f32(_p(e), _p(_f32(log_T)), int(prev), float(np.float32(log_n)), T, N, _p(st), _p(sc))
    return st, sc


def c_stream_beam(emis, log_T, K, hyp_scores, hyp_last, first):
    """One chunk of streaming.py:322-377.  Returns (new scores, new last states, parent (T,K),
    state (T,K)); hypothesis r at step t came from parent[t, r] and entered state[t, r]."""
    e = _f32(emis)
    T, N = e.shape
    kc = len(hyp_scores)
    hs = np.zeros(max(K, kc), np.float32); hs[:kc] = hyp_scores
    hl = np.zeros(max(K, kc), np.int32); hl[:kc] = hyp_last
    kio = np.array([kc], np.int32)
    par = np.zeros((T, K), np.int16)
    hst = np.zeros((T, K), np.int16)
    c_oracle().stream_beam_f32(_p(e), _p(_f32(log_T)), T, N, K, _p(hs), _p(hl), _p(kio), int(first), _p(par), _p(hst))
    k = int(kio[0])
    return hs[:k].copy(), hl[:k].copy(), par, hst


def uniform_obs(seed, shape, lo=0.0, hi=1.0):
    """Machine-independent inputs (PCG64 integers -> float32, no transcendentals); the same
    generator as tests/golden/make_golden.py."""
    rng = np.random.default_rng(seed)
    x = rng.random(shape, dtype=np.float32)
    return (x * np.float32(hi - lo) + np.float32(lo)).astype(np.float32)
