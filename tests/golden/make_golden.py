#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE here.

This script is the only place that imports crlotwhite/pytorch_hmm (read-only at
/root/reference).  It runs in the build container only; the reference never travels
to the GPU box.  What travels is the .npz files this script writes: inputs, the
parameters the reference derived from them, and the reference's outputs.

Run (from the repo root):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Each fixture records torch.__version__ and the sha256 of its inputs.  Reference call
sites are cited per fixture (file:line into /root/reference/pytorch_hmm).
"""
import hashlib
import math
import os
import sys
import time

import numpy as np
import torch

REF = os.environ.get("HMM_REFERENCE", "/root/reference")
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
import pytorch_hmm  # noqa: E402  (prints its auto_configure banner)
from pytorch_hmm.hmm import HMMPyTorch  # noqa: E402
from pytorch_hmm.hmm_layer import HMMLayer, GaussianHMMLayer  # noqa: E402
from pytorch_hmm.mixture_gaussian import MixtureGaussianHMMLayer  # noqa: E402
from pytorch_hmm.hsmm import HSMMLayer  # noqa: E402
from pytorch_hmm.semi_markov import SemiMarkovHMM  # noqa: E402
from pytorch_hmm.streaming import StreamingHMMProcessor  # noqa: E402
from pytorch_hmm.neural import NeuralHMM, ContextualNeuralHMM  # noqa: E402
from pytorch_hmm.utils import (  # noqa: E402
    create_left_to_right_matrix, create_transition_matrix)

OUT = os.path.dirname(os.path.abspath(__file__))
torch.set_num_threads(min(8, os.cpu_count() or 1))


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def npf(t):
    return t.detach().cpu().numpy()


def save(name, **arrays):
    meta = dict(torch_version=torch.__version__, generator="tests/golden/make_golden.py")
    arrays = {k: (np.asarray(v) if not isinstance(v, np.ndarray) else v) for k, v in arrays.items()}
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, __meta__=np.array(repr(meta)), **arrays)
    print(f"  wrote {name}.npz ({os.path.getsize(path)/1024:.1f} KiB)")


class CaptureExp:
    """Record the arguments of torch.exp while the reference's forward_backward runs:
    hmm.py:126-128 calls exp(log_posterior), exp(log_forward), exp(log_backward) in order."""

    def __enter__(self):
        self.args = []
        self._orig = torch.exp

        def rec(x, *a, **k):
            self.args.append(x.detach().clone())
            return self._orig(x, *a, **k)
        torch.exp = rec
        return self

    def __exit__(self, *exc):
        torch.exp = self._orig


def fb_with_internals(hmm, obs):
    with CaptureExp() as cap:
        post, fwd, bwd = hmm.forward_backward(obs)
    log_post, log_alpha, log_beta = cap.args[-3], cap.args[-2], cap.args[-1]
    loglik = torch.logsumexp(log_alpha[:, -1], dim=-1)   # meaningful LSE(alpha_{T-1})
    return post, fwd, bwd, log_alpha, log_beta, loglik


def uniform_obs(seed, shape, lo=0.0, hi=1.0):
    """Machine-independent inputs: integer PCG64 stream -> float32, no transcendentals."""
    rng = np.random.default_rng(seed)
    x = rng.random(shape, dtype=np.float32)
    return (x * np.float32(hi - lo) + np.float32(lo)).astype(np.float32)


# --------------------------------------------------------------------------------------
def fx_hmmpytorch(name, P, B, T, seed, p0=None):
    """HMMPyTorch forward_backward / viterbi_decode / compute_likelihood
    (hmm.py:66-130, 132-184, 186-211)."""
    torch.manual_seed(seed)
    N = P.shape[0]
    obs = torch.softmax(torch.randn(B, T, N), dim=-1)          # examples/benchmark.py:160-162
    hmm = HMMPyTorch(P, p0) if p0 is not None else HMMPyTorch(P)
    post, fwd, bwd, la, lb, ll = fb_with_internals(hmm, obs)
    states, delta = hmm.viterbi_decode(obs)
    lik = hmm.compute_likelihood(obs)
    save(name, P=npf(P), p0=(npf(p0) if p0 is not None else np.zeros(0, np.float32)),
         obs=npf(obs), log_obs=npf(torch.log(obs + 1e-8)), log_P=npf(hmm.log_P),
         log_p0=npf(hmm.log_p0), posterior=npf(post), forward=npf(fwd), backward=npf(bwd),
         log_alpha=npf(la), log_beta=npf(lb), loglik=npf(ll), states=npf(states),
         log_delta=npf(delta), compute_likelihood=npf(lik), input_sha256=sha(npf(obs)))


def fx_ties():
    """First-index tie semantics (torch.max, hmm.py:167; argmax :174)."""
    N, B, T = 8, 2, 50
    P = create_left_to_right_matrix(N, 0.5)
    obs = torch.full((B, T, N), 1.0 / N)
    hmm = HMMPyTorch(P)
    s1, d1 = hmm.viterbi_decode(obs)
    Pu = torch.ones(N, N)                                    # ergodic, all-equal rows
    hmm2 = HMMPyTorch(Pu)
    s2, d2 = hmm2.viterbi_decode(obs)
    save("ties", P=npf(P), Pu=npf(Pu), obs=npf(obs), log_obs=npf(torch.log(obs + 1e-8)),
         log_P=npf(hmm.log_P), log_p0=npf(hmm.log_p0), states=npf(s1), log_delta=npf(d1),
         log_Pu=npf(hmm2.log_P), log_p0u=npf(hmm2.log_p0), states_u=npf(s2), log_delta_u=npf(d2))


def fx_wiki():
    """tests/test_hmm.py:306-333 weather example (2-D input -> squeezed outputs)."""
    P = torch.tensor([[0.7, 0.3], [0.4, 0.6]])
    p0 = torch.tensor([0.6, 0.4])
    hmm = HMMPyTorch(P, p0)
    obs = torch.tensor([[0.1, 0.4, 0.5], [0.6, 0.3, 0.1]]).T.contiguous()
    states, delta = hmm.viterbi_decode(obs)
    post, fwd, bwd = hmm.forward_backward(obs)
    lik = hmm.compute_likelihood(obs)
    save("wiki", P=npf(P), p0=npf(p0), obs=npf(obs), log_P=npf(hmm.log_P), log_p0=npf(hmm.log_p0),
         states=npf(states), log_delta=npf(delta), posterior=npf(post), forward=npf(fwd),
         backward=npf(bwd), compute_likelihood=npf(lik))


def fx_hmmlayer_c1():
    """BASELINE config 1: HMMLayer(5), x ~ randn(2,100,5), seed 0 (hmm_layer.py:91-191).
    Call order matters: call 1 renormalises P (hmm.py:39), later calls do not (hmm_layer.py:83-86)."""
    torch.manual_seed(0)
    layer = HMMLayer(5)
    x = torch.randn(2, 100, 5)
    layer.train()
    with CaptureExp() as cap:
        post1 = layer(x)                                       # call 1 -> HMMPyTorch(P, p0)
    la1, lb1 = cap.args[-2], cap.args[-1]
    log_P1, log_p01 = layer._hmm.log_P.detach().clone(), layer._hmm.log_p0.detach().clone()
    layer.eval()
    onehot2, align2 = layer(x, return_alignment=True)          # call 2 -> log(P+1e-8)
    log_P2, log_p02 = layer._hmm.log_P.detach().clone(), layer._hmm.log_p0.detach().clone()
    states3, delta3 = layer.align(x)                           # call 3
    layer.train()
    loss4 = layer.compute_loss(x)                              # call 4 (unsupervised NLL)
    lik4 = layer._hmm.compute_likelihood(torch.sigmoid(x))
    save("hmmlayer_c1", x=npf(x), obs=npf(torch.sigmoid(x)),
         log_obs=npf(torch.log(torch.sigmoid(x) + 1e-8)),
         logits=npf(layer.log_transition_logits), init_logits=npf(layer.log_initial_logits),
         posterior1=npf(post1), log_alpha1=npf(la1), log_beta1=npf(lb1),
         log_P1=npf(log_P1), log_p01=npf(log_p01), log_P2=npf(log_P2), log_p02=npf(log_p02),
         onehot2=npf(onehot2), align2=npf(align2), states3=npf(states3), log_delta3=npf(delta3),
         loss4=npf(loss4), likelihood4=npf(lik4), input_sha256=sha(npf(x)))


def fx_gaussian(name, K, D, B, T, seed):
    """GaussianHMMLayer (hmm_layer.py:220-359): diag Gaussian log-probs -> exp -> HMMLayer."""
    torch.manual_seed(seed)
    layer = GaussianHMMLayer(K, D)
    x = torch.randn(B, T, D)
    lp = layer._compute_gaussian_log_probs(x)
    probs = torch.exp(lp)
    layer.train()
    post = layer(x)                                              # call 1 (FB)
    layer.eval()
    onehot, states = layer.hmm_layer(probs, return_alignment=True)   # call 2 (Viterbi)
    loss = layer.compute_loss(x)                                 # call 3
    save(name, x=npf(x), means=npf(layer.means), log_scales=npf(layer.log_scales),
         logits=npf(layer.hmm_layer.log_transition_logits),
         init_logits=npf(layer.hmm_layer.log_initial_logits), log_probs=npf(lp), probs=npf(probs),
         posterior=npf(post), onehot=npf(onehot), states=npf(states), loss=npf(loss),
         input_sha256=sha(npf(x)))


def fx_mixture(name, S, D, C, B, T, seed, x=None):
    """MixtureGaussianHMMLayer (mixture_gaussian.py:157-214, 290-365)."""
    torch.manual_seed(seed)
    m = MixtureGaussianHMMLayer(S, D, num_components=C)
    if x is None:
        x = torch.randn(B, T, D)
    with torch.no_grad():
        lp = m.get_observation_log_probs(x)
        log_T = m._safe_log(m.get_transition_matrix())
        log_w = m._safe_log(torch.softmax(m.mixture_weights_logits, dim=-1))
        states, scores = m(x, return_log_probs=True)
    save(name, x=npf(x), transition_logits=npf(m.transition_logits),
         mixture_weights_logits=npf(m.mixture_weights_logits), means=npf(m.means),
         log_vars=npf(m.log_vars), log_probs=npf(lp), log_T=npf(log_T), log_w=npf(log_w),
         states=npf(states), scores=npf(scores), input_sha256=sha(npf(x)))


def fx_mixture_full(name, S, D, C, B, T, seed):
    """MixtureGaussianHMMLayer(covariance_type='full') (mixture_gaussian.py:216-240, 271-289):
    Cholesky parameters perturbed off the diagonal so the triangular solve is exercised."""
    torch.manual_seed(seed)
    m = MixtureGaussianHMMLayer(S, D, num_components=C, covariance_type="full")
    with torch.no_grad():
        m.cholesky_params.add_(0.15 * torch.randn_like(m.cholesky_params))
    x = torch.randn(B, T, D)
    with torch.no_grad():
        lp = m.get_observation_log_probs(x)
        log_T = m._safe_log(m.get_transition_matrix())
        states, scores = m(x, return_log_probs=True)
    save(name, x=npf(x), transition_logits=npf(m.transition_logits),
         mixture_weights_logits=npf(m.mixture_weights_logits), means=npf(m.means),
         cholesky_params=npf(m.cholesky_params), log_probs=npf(lp), log_T=npf(log_T),
         states=npf(states), scores=npf(scores), input_sha256=sha(npf(x)))


def fx_mixture_cov(name, S, D, C, B, T, seed, cov):
    """MixtureGaussianHMMLayer(covariance_type='tied' | 'spherical') (mixture_gaussian.py:242-269,
    LSE :141-155, Viterbi :290-338).  The log-variances are drawn off their zero init so the
    variance terms of each branch's expression (sum diff^2/var + sum log_var for 'tied';
    sum diff^2 / var + D*log_var for 'spherical') take part."""
    torch.manual_seed(seed)
    m = MixtureGaussianHMMLayer(S, D, num_components=C, covariance_type=cov)
    with torch.no_grad():
        m.log_vars.copy_(0.4 * torch.randn_like(m.log_vars))
    x = torch.randn(B, T, D)
    with torch.no_grad():
        lp = m.get_observation_log_probs(x)
        log_T = m._safe_log(m.get_transition_matrix())
        states, scores = m(x, return_log_probs=True)
    save(name, x=npf(x), transition_logits=npf(m.transition_logits),
         mixture_weights_logits=npf(m.mixture_weights_logits), means=npf(m.means),
         log_vars=npf(m.log_vars), log_probs=npf(lp), log_T=npf(log_T), states=npf(states),
         scores=npf(scores), covariance_type=np.array(cov), input_sha256=sha(npf(x)))


def fx_gaussian_cov(name, K, D, B, T, seed, cov):
    """GaussianHMMLayer(covariance_type='spherical' | 'full') (hmm_layer.py:289-298 and :311-319,
    the 'full' branch using the diagonal of log_scales), then exp -> HMMLayer as fx_gaussian.
    Small D so exp(log_probs) does not underflow and the HMM sees real emissions; log_scales
    drawn off their zero init (for 'full' the whole (K,D,D) tensor, of which the reference
    reads only the diagonal)."""
    torch.manual_seed(seed)
    layer = GaussianHMMLayer(K, D, covariance_type=cov)
    with torch.no_grad():
        layer.log_scales.copy_(0.3 * torch.randn_like(layer.log_scales))
    x = torch.randn(B, T, D)
    lp = layer._compute_gaussian_log_probs(x)
    probs = torch.exp(lp)
    layer.train()
    post = layer(x)                                              # call 1 (FB)
    layer.eval()
    onehot, states = layer.hmm_layer(probs, return_alignment=True)   # call 2 (Viterbi)
    loss = layer.compute_loss(x)                                 # call 3
    save(name, x=npf(x), means=npf(layer.means), log_scales=npf(layer.log_scales),
         logits=npf(layer.hmm_layer.log_transition_logits),
         init_logits=npf(layer.hmm_layer.log_initial_logits), log_probs=npf(lp), probs=npf(probs),
         posterior=npf(post), onehot=npf(onehot), states=npf(states), loss=npf(loss),
         covariance_type=np.array(cov), input_sha256=sha(npf(x)))


def fx_hsmm(name, S, D, Dmax, B, T, seed, dur_params=None):
    """HSMMLayer segment Viterbi (hsmm.py:181-354); the literal 5-deep loop, small sizes only.
    dur_params = (shape, rate) raw parameter values (before softplus) to favour long segments."""
    torch.manual_seed(seed)
    h = HSMMLayer(S, D, max_duration=Dmax)
    if dur_params is not None:
        with torch.no_grad():
            h.duration_shape.fill_(dur_params[0])
            h.duration_rate.fill_(dur_params[1])
    x = torch.randn(B, T, D)
    with torch.no_grad():
        lp = h.get_observation_log_probs(x)
        dur_lp = torch.log(h.get_duration_probabilities() + h.eps)
        log_T = torch.log(h.get_transition_matrix() + h.eps)
        t0 = time.time()
        states, scores = h(x)
    print(f"    hsmm {name}: {time.time()-t0:.1f}s")
    save(name, x=npf(x), transition_logits=npf(h.transition_logits),
         observation_means=npf(h.observation_means), observation_log_vars=npf(h.observation_log_vars),
         duration_shape=npf(h.duration_shape), duration_rate=npf(h.duration_rate),
         log_probs=npf(lp), dur_log_probs=npf(dur_lp), log_T=npf(log_T),
         states=npf(states), scores=npf(scores), input_sha256=sha(npf(x)))


def fx_semimarkov(name, S, D, Dmax, T, nseq, seed, dist="gamma", min_duration=1, obs_model="gaussian"):
    """SemiMarkovHMM.viterbi_decode (semi_markov.py:455-570), its per-candidate duration
    log-probabilities (duration_model(tensor([s]), tensor([d]))[0], :502-505), the segment
    constant (:416-421), DurationModel.forward over all durations (:81-98) and the supervised
    forward of the decoded segmentation (:280-306).  Eval mode (the neural observation model
    has dropout)."""
    torch.manual_seed(seed)
    m = SemiMarkovHMM(S, D, max_duration=Dmax, duration_distribution=dist, observation_model=obs_model,
                      min_duration=min_duration)
    m.eval()
    x = torch.randn(nseq, T, D)
    with torch.no_grad():
        dur = torch.full((S, Dmax), float("nan"))
        for s_ in range(S):
            for d in range(1, Dmax + 1):
                dur[s_, d - 1] = m.duration_model(torch.tensor([s_]), torch.tensor([d]))[0]
        dist_all = m.duration_model(torch.arange(S))
        if obs_model == "gaussian":
            cs = torch.stack([-0.5 * torch.sum(m.observation_logvars[s_]) - 0.5 * D * math.log(2 * math.pi)
                              for s_ in range(S)])
        else:
            cs = torch.zeros(S)
        t0 = time.time()
        seg_states, seg_durs, scores, counts, sup = [], [], [], [], []
        for b in range(nseq):
            st, du, sc = m.viterbi_decode(x[b])
            seg_states.append(npf(st)); seg_durs.append(npf(du)); scores.append(float(sc))
            counts.append(len(st))
            r = m(x[b:b + 1], st.unsqueeze(0), du.unsqueeze(0))
            sup.append([float(r[k]) for k in ("log_probability", "log_observation", "log_duration", "log_transition")])
    print(f"    semimarkov {name}: {time.time()-t0:.1f}s")
    K = max(counts)
    pad = lambda a: np.concatenate([a, -np.ones(K - len(a), np.int64)])
    params = {"param__" + k.replace(".", "__"): npf(v) for k, v in m.state_dict().items()}
    save(name, x=npf(x), dur_candidates=npf(dur), dur_distribution=npf(dist_all), seg_const=npf(cs),
         seg_states=np.stack([pad(a) for a in seg_states]), seg_durs=np.stack([pad(a) for a in seg_durs]),
         seg_count=np.array(counts), scores=np.array(scores, np.float32), supervised=np.array(sup, np.float32),
         config=np.array([S, D, Dmax, T, nseq, min_duration]), dist=np.array(dist), obs_model=np.array(obs_model),
         input_sha256=sha(npf(x)), **params)


def fx_streaming(name, N, D, K, lens, seed, chunk_size=20, max_delay=50, lookahead=3, n_proc=6):
    """StreamingHMMProcessor (streaming.py:35-503), eval mode (the emission net has dropout):
    _greedy_decode and _beam_search_decode called directly on consecutive chunks (the
    emission log-probs, returned states / confidences and, for beam, the hypotheses after
    each chunk), then process_chunk on a fresh stream of n_proc chunks (statuses, states)."""
    torch.manual_seed(seed)
    g = StreamingHMMProcessor(N, D, chunk_size=chunk_size, lookahead_frames=lookahead, max_delay_frames=max_delay,
                              use_beam_search=False).eval()
    b = StreamingHMMProcessor(N, D, chunk_size=chunk_size, lookahead_frames=lookahead, max_delay_frames=max_delay,
                              use_beam_search=True, beam_width=K).eval()
    b.load_state_dict(g.state_dict())
    feats = [torch.randn(L, D) for L in lens]
    out = {}
    t0 = time.time()
    with torch.no_grad():
        for i, f in enumerate(feats):
            out[f"emis{i}"] = npf(g.emission_net(f))
            st, conf = g._greedy_decode(f)
            out[f"greedy_states{i}"], out[f"greedy_conf{i}"] = npf(st), npf(conf)
            st, conf = b._beam_search_decode(f)
            out[f"beam_states{i}"], out[f"beam_conf{i}"] = npf(st), npf(conf)
            out[f"beam_hs{i}"] = np.array([float(h[0]) for h in b.beam_hypotheses], np.float32)
            out[f"beam_hl{i}"] = np.array([h[2] for h in b.beam_hypotheses], np.int64)
            out[f"beam_plen{i}"] = np.array([len(h[1]) for h in b.beam_hypotheses], np.int64)
            out[f"beam_path0_{i}"] = np.array(b.beam_hypotheses[0][1], np.int64)
        out["log_T"] = npf(torch.log(g.get_transition_matrix() + 1e-8))
        # process_chunk on fresh streams (greedy and beam)
        chunks = [torch.randn(chunk_size // 2 + 3, D) for _ in range(n_proc)]
        for tag, proc in (("pg", g), ("pb", b)):
            proc.reset_streaming_state()
            for i, c in enumerate(chunks):
                r = proc.process_chunk(c)
                out[f"{tag}_status{i}"] = np.array(r.status)
                out[f"{tag}_states{i}"] = npf(r.decoded_states) if r.decoded_states is not None else np.zeros(0, np.int64)
                out[f"{tag}_conf{i}"] = np.array(r.confidence, np.float64)
        for i, c in enumerate(chunks):
            out[f"chunk{i}"] = npf(c)
    print(f"    streaming {name}: {time.time()-t0:.1f}s")
    params = {"param__" + k.replace(".", "__"): npf(v) for k, v in g.state_dict().items()}
    save(name, config=np.array([N, D, K, chunk_size, max_delay, lookahead, len(lens), n_proc]),
         **{f"feat{i}": npf(f) for i, f in enumerate(feats)}, **out, **params)


def _neural_capture(m, x, ctx, call_fb, call_vit):
    """Log-emissions, log-transitions, the FB outputs with log_forward / log_backward (the last
    two torch.exp arguments, neural.py:401), Viterbi and compute_likelihood of one NeuralHMM."""
    with torch.no_grad():
        lo = m.observation_model(x)
        if m.transition_model is not None and ctx is not None:
            lt = torch.log(m.transition_model(ctx) + 1e-8)                      # neural.py:379-380
        else:
            lt = torch.log(torch.softmax(m.transition_matrix, dim=1) + 1e-8)    # :383-384 (K,K)
        li = torch.log(torch.softmax(m.initial_logits, dim=0) + 1e-8)          # :388-389
        with CaptureExp() as cap:
            post, fwd, bwd = call_fb()
        lf, lb = cap.args[-2], cap.args[-1]
        states, delta = call_vit()
        lik = m.compute_likelihood(x, ctx)
    return dict(log_obs=npf(lo), log_trans=npf(lt), log_init=npf(li), posterior=npf(post),
                forward=npf(fwd), backward=npf(bwd), log_forward=npf(lf), log_backward=npf(lb),
                states=npf(states), log_delta=npf(delta), compute_likelihood=npf(lik))


def fx_neural(name, K, D, C, H, B, T, seed, ttype="mlp", otype="gaussian", keep_params=True):
    """NeuralHMM forward / viterbi_decode / compute_likelihood (neural.py:355-519) in eval mode
    (dropout off).  C = 0: the static transition_matrix expanded over (B,T) (neural.py:383-385)."""
    torch.manual_seed(seed)
    m = NeuralHMM(K, D, context_dim=C, hidden_dim=H, transition_type=ttype, observation_type=otype).eval()
    x = torch.randn(B, T, D)
    ctx = torch.randn(B, T, C) if C > 0 else None
    out = _neural_capture(m, x, ctx, lambda: m(x, ctx), lambda: m.viterbi_decode(x, ctx))
    sd = {"sd__" + k: npf(v) for k, v in m.state_dict().items()} if keep_params else {}
    save(name, x=npf(x), ctx=(npf(ctx) if ctx is not None else np.zeros(0, np.float32)),
         config=np.array([K, D, C, H]), ttype=np.array(ttype), otype=np.array(otype),
         input_sha256=sha(npf(x)), **out, **sd)


def fx_contextual(name, K, D, V, LD, PD, B, T, seed):
    """ContextualNeuralHMM.forward_with_context (neural.py:522-588), eval mode."""
    torch.manual_seed(seed)
    m = ContextualNeuralHMM(K, D, phoneme_vocab_size=V, linguistic_context_dim=LD, prosody_dim=PD).eval()
    x = torch.randn(B, T, D)
    ph = torch.randint(0, V, (B, T))
    pr = torch.randn(B, T, PD)
    with torch.no_grad():
        ctx = m.encode_context(ph, pr)
    out = _neural_capture(m, x, ctx, lambda: m.forward_with_context(x, ph, pr), lambda: m.viterbi_decode(x, ctx))
    sd = {"sd__" + k: npf(v) for k, v in m.state_dict().items()}
    save(name, x=npf(x), phonemes=npf(ph), prosody=npf(pr), ctx=npf(ctx), config=np.array([K, D, V, LD, PD]),
         input_sha256=sha(npf(x)), **out, **sd)


def fx_fullsize_ns():
    """North-star shape B=32, T=2000, N=128 (left-to-right 0.7): machine-independent uniform
    inputs (PCG64 -> float32) so the GPU box can regenerate them bit-for-bit.  Stores the
    reference's Viterbi states (uint8), per-sequence LSE(alpha_{T-1}), final delta row and
    a few posterior rows; the full tensors are checked on the box against the oracle."""
    B, T, N = 32, 2000, 128
    obs_np = uniform_obs(20251015, (B, T, N))
    obs = torch.from_numpy(obs_np)
    hmm = HMMPyTorch(create_left_to_right_matrix(N, 0.7))
    t0 = time.time()
    post, fwd, bwd, la, lb, ll = fb_with_internals(hmm, obs)
    t1 = time.time()
    states, delta = hmm.viterbi_decode(obs)
    t2 = time.time()
    print(f"    NS reference: FB {t1-t0:.3f}s  Viterbi {t2-t1:.3f}s")
    rows = np.array([0, 1, 999, 1998, 1999])
    save("fullsize_ns", seed=np.int64(20251015), shape=np.array([B, T, N]),
         log_P=npf(hmm.log_P), log_p0=npf(hmm.log_p0),
         states=npf(states).astype(np.uint8), loglik=npf(ll), delta_last=npf(delta[:, -1]),
         post_rows=rows, posterior_rows=npf(post[:, rows]), log_alpha_last=npf(la[:, -1]),
         log_beta_first=npf(lb[:, 0]), compute_likelihood=npf(hmm.compute_likelihood(obs)),
         log_obs_sha256=sha(npf(torch.log(obs + 1e-8))), input_sha256=sha(obs_np),
         ref_fb_seconds=np.float64(t1 - t0), ref_viterbi_seconds=np.float64(t2 - t1))


def fx_fullsize_mixture():
    """BASELINE config 3 shape (S=128, C=4, D=80, B=32, T=2000) with machine-independent x."""
    B, T, D, S, C = 32, 2000, 80, 128, 4
    x = torch.from_numpy(uniform_obs(7, (B, T, D), -2.0, 2.0))
    torch.manual_seed(0)
    m = MixtureGaussianHMMLayer(S, D, num_components=C)
    with torch.no_grad():
        t0 = time.time()
        lp = m.get_observation_log_probs(x)
        states, scores = m(x, return_log_probs=True)
        print(f"    C3 reference: {time.time()-t0:.2f}s")
    save("fullsize_mixture", shape=np.array([B, T, D, S, C]), x_seed=np.int64(7),
         transition_logits=npf(m.transition_logits),
         mixture_weights_logits=npf(m.mixture_weights_logits), means=npf(m.means),
         log_vars=npf(m.log_vars), states=npf(states).astype(np.uint8), scores=npf(scores),
         lp_rows=npf(lp[:, :4]), lp_sha256=sha(npf(lp)), input_sha256=sha(npf(x)))


def fx_fullsize_gaussian():
    """BASELINE config 2 at full size: GaussianHMMLayer(64, 80), seed-0 init, B=32, T=2000
    (hmm_layer.py:220-359), machine-independent x in [-2, 2).  At D = 80 every Gaussian
    density underflows in exp (hmm_layer.py:325-340), so the HMM sees constant emissions
    exp(lp) = 0 -> log(0 + 1e-8) everywhere: the Viterbi recursion is
    2000 steps of first-index ties (hmm.py:167, :174) on the 64-state chain.  Same call
    order as fx_gaussian: train FB (call 1), eval Viterbi (call 2), compute_loss (call 3)."""
    B, T, K, D = 32, 2000, 64, 80
    x = torch.from_numpy(uniform_obs(11, (B, T, D), -2.0, 2.0))
    torch.manual_seed(0)
    layer = GaussianHMMLayer(K, D)
    with torch.no_grad():
        t0 = time.time()
        lp = layer._compute_gaussian_log_probs(x)
        probs = torch.exp(lp)
        layer.train()
        post = layer(x)                                              # call 1 (FB)
        layer.eval()
        onehot, states = layer.hmm_layer(probs, return_alignment=True)   # call 2 (Viterbi)
        loss = layer.compute_loss(x)                                 # call 3
        print(f"    C2 reference: {time.time()-t0:.2f}s, max lp {float(lp.max()):.1f}, "
              f"nonzero probs {int((probs > 0).sum())}")
    rows = np.arange(0, T, 20)
    post_np, st_np = npf(post), npf(states)
    save("fullsize_gaussian", shape=np.array([B, T, K, D]), x_seed=np.int64(11),
         means=npf(layer.means), log_scales=npf(layer.log_scales),
         logits=npf(layer.hmm_layer.log_transition_logits),
         init_logits=npf(layer.hmm_layer.log_initial_logits),
         lp_rows=npf(lp[:, :4]), lp_max=np.float32(lp.max()), probs_nonzero=np.int64((probs > 0).sum()),
         states=st_np.astype(np.uint8), post_rows=rows, posterior_rows=post_np[:, rows],
         posterior_seq_equal=np.bool_(bool((post_np == post_np[:1]).all())),
         loss=npf(loss), input_sha256=sha(npf(x)))


def main():
    only = set(sys.argv[1:])
    jobs = [
        ("hmmpytorch_l2r", lambda: fx_hmmpytorch("hmmpytorch_l2r", create_left_to_right_matrix(128, 0.7), 2, 256, 1234)),
        ("hmmpytorch_ergodic", lambda: fx_hmmpytorch("hmmpytorch_ergodic", create_transition_matrix(128, "ergodic"), 2, 256, 1235)),
        ("hmmpytorch_small", lambda: fx_hmmpytorch("hmmpytorch_small", create_left_to_right_matrix(3, 0.7), 2, 10, 5,
                                                    p0=torch.tensor([0.5, 0.3, 0.2]))),
        ("hmmpytorch_n200", lambda: fx_hmmpytorch("hmmpytorch_n200", create_transition_matrix(200, "left_to_right_skip", 0.5, 0.4, 0.1), 2, 64, 77)),
        ("ties", fx_ties),
        ("wiki", fx_wiki),
        ("hmmlayer_c1", fx_hmmlayer_c1),
        ("gaussian_c2", lambda: fx_gaussian("gaussian_c2", 64, 80, 2, 128, 0)),
        ("gaussian_small", lambda: fx_gaussian("gaussian_small", 3, 5, 2, 12, 1)),
        ("mixture_s16", lambda: fx_mixture("mixture_s16", 16, 80, 4, 2, 256, 0)),
        ("mixture_s128", lambda: fx_mixture("mixture_s128", 128, 80, 4, 1, 64, 0)),
        ("mixture_single", lambda: fx_mixture("mixture_single", 1, 10, 1, 1, 20, 3)),
        ("mixture_full", lambda: fx_mixture_full("mixture_full", 6, 7, 3, 2, 40, 11)),
        ("mixture_tied", lambda: fx_mixture_cov("mixture_tied", 16, 20, 4, 2, 128, 21, "tied")),
        ("mixture_spherical", lambda: fx_mixture_cov("mixture_spherical", 16, 20, 4, 2, 128, 22, "spherical")),
        ("gaussian_spherical", lambda: fx_gaussian_cov("gaussian_spherical", 8, 6, 2, 64, 23, "spherical")),
        ("gaussian_full", lambda: fx_gaussian_cov("gaussian_full", 8, 6, 2, 64, 24, "full")),
        ("hsmm_s5", lambda: fx_hsmm("hsmm_s5", 5, 30, 20, 2, 30, 0)),
        ("hsmm_s2", lambda: fx_hsmm("hsmm_s2", 2, 3, 2, 1, 4, 1)),
        ("hsmm_s8", lambda: fx_hsmm("hsmm_s8", 8, 20, 10, 1, 40, 2)),
        # segments of 72+ frames (decoded: 83 + 82) whose sums take torch.sum's cascade order
        # (hsmm.py:273,285), not the plain 4-lane order: gamma mode ~85 frames
        ("hsmm_d96", lambda: fx_hsmm("hsmm_d96", 3, 6, 96, 1, 165, 1, dur_params=(30.0, -0.9))),
        ("smk_gamma", lambda: fx_semimarkov("smk_gamma", 4, 6, 10, 30, 2, 0)),
        ("smk_poisson", lambda: fx_semimarkov("smk_poisson", 5, 8, 8, 40, 1, 1, dist="poisson", min_duration=2)),
        ("smk_gaussian", lambda: fx_semimarkov("smk_gaussian", 6, 5, 12, 48, 1, 2, dist="gaussian")),
        ("smk_neuraldur", lambda: fx_semimarkov("smk_neuraldur", 4, 6, 6, 20, 2, 3, dist="neural")),
        ("smk_neuralobs", lambda: fx_semimarkov("smk_neuralobs", 3, 4, 5, 15, 1, 4, obs_model="neural")),
        ("stream_n5", lambda: fx_streaming("stream_n5", 5, 30, 4, [40, 25, 33], 0)),
        ("stream_n12", lambda: fx_streaming("stream_n12", 12, 16, 8, [64, 70, 9], 1, chunk_size=30)),
        ("stream_n3k16", lambda: fx_streaming("stream_n3k16", 3, 8, 16, [10, 12], 2)),
        ("smk_s8", lambda: fx_semimarkov("smk_s8", 8, 16, 16, 96, 1, 6)),
        ("smk_short", lambda: fx_semimarkov("smk_short", 3, 4, 10, 4, 2, 5)),
        ("neural_mlp_small", lambda: fx_neural("neural_mlp_small", 5, 8, 12, 64, 2, 20, 0)),
        ("neural_static", lambda: fx_neural("neural_static", 6, 10, 0, 32, 2, 25, 1)),
        ("neural_rnn", lambda: fx_neural("neural_rnn", 7, 6, 4, 16, 2, 15, 2, ttype="rnn")),
        ("neural_mixture", lambda: fx_neural("neural_mixture", 5, 6, 5, 16, 2, 12, 3, otype="mixture")),
        ("neural_k32", lambda: fx_neural("neural_k32", 32, 16, 8, 64, 2, 24, 4)),
        ("neural_k128", lambda: fx_neural("neural_k128", 128, 16, 8, 64, 1, 6, 5, keep_params=False)),
        ("contextual_small", lambda: fx_contextual("contextual_small", 6, 10, 50, 32, 8, 2, 15, 6)),
        ("fullsize_ns", fx_fullsize_ns),
        ("fullsize_mixture", fx_fullsize_mixture),
        ("fullsize_gaussian", fx_fullsize_gaussian),
    ]
    for name, fn in jobs:
        if only and name not in only:
            continue
        print(name)
        fn()


if __name__ == "__main__":
    main()
