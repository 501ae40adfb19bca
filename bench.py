#!/usr/bin/env python3
"""Benchmark: frames/s of forward-backward + Viterbi (BASELINE.json metric).

Workload (BASELINE configs[1] / the north-star shape): HMMPyTorch with a 128-state
left-to-right (0.7) transition matrix, B=32 sequences of T=2000 frames per GPU, emissions
softmax(randn(B,T,N)) (examples/benchmark.py:160-162), synthetic, resident in HBM.
One step = HMMPyTorch.forward_backward (posterior, forward, backward) + viterbi_decode
(states, trellis) over the batch; the two run on two HIP streams of the same GPU.
N GPUs = one process per GPU (torchrun), B=32 per rank (weak scaling; --strong splits a
global B=32 over the ranks instead); with world > 1 every step also gathers the posteriors
and states to rank 0 over RCCL (BASELINE config 4's gather; --no-gather leaves it out and
the JSON line says so), on a third stream, event-ordered and double-buffered (NsStep).

Prints ONE JSON line on rank 0.  Besides the contract fields it carries
  roofline     for the dominant kernel (HIP events on its stream, over the timed steps)
  cpu_baseline the oracle (torch-CPU restatement, bit-identical to the reference) timed on
               the host cores on a bounded sample (rank 0, N=1 only)
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--batch", type=int, default=32, help="sequences per GPU")
    p.add_argument("--T", type=int, default=2000)
    p.add_argument("--N", type=int, default=128)
    p.add_argument("--no-gather", action="store_true",
                   help="world > 1: leave out the RCCL gather of posteriors + states to rank 0 that every "
                        "multi-GPU step does by default (BASELINE config 4); the JSON line records it")
    p.add_argument("--gather", action="store_true", help=argparse.SUPPRESS)   # the default since round 3
    p.add_argument("--strong", action="store_true",
                   help="strong scaling: --batch is the GLOBAL batch, split over the ranks "
                        "(default: weak scaling, --batch sequences per rank)")
    p.add_argument("--serial", action="store_true", help="run FB and Viterbi on one stream")
    p.add_argument("--overlap-steps", action="store_true",
                   help="layer workloads c2/c3/c5: consecutive steps on two alternating streams (step "
                        "k+1's emission beside step k's recursion; two batches in flight)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline budget (0 = skip)")
    p.add_argument("--graph", action="store_true",
                   help="ns workload: replay each op from a captured HIP graph instead of launching it "
                        "eagerly (round 6: each op is one launch, eager is faster -- DESIGN.md §5)")
    p.add_argument("--no-graph", action="store_true", help=argparse.SUPPRESS)  # (the default since round 6)
    p.add_argument("--transition", default="left_to_right", choices=["left_to_right", "ergodic", "random", "trained"],
                   help="transition matrix of the workload (BASELINE: left_to_right 0.7; SURVEY §8(d) also "
                        "names create_transition_matrix(N,'ergodic'); 'random' = a dense learned-style "
                        "matrix softmax(randn), which takes the dense chains)")
    p.add_argument("--workload", default="ns", choices=["ns", "c1", "c2", "c3", "c5", "neural", "smk", "stream"],
                   help="ns: the BASELINE metric (default).  c1/c2/c3/c5: BASELINE configs 1, 2, 3, 5 "
                        "(HMMLayer, GaussianHMMLayer, MixtureGaussianHMMLayer, HSMMLayer) through the layers")
    p.add_argument("--tv-static", action="store_true",
                   help="neural workload, diagnostic: one (N,N) matrix for every step (L2-resident)")
    p.add_argument("--tv-only", choices=["fb", "vit"], default=None,
                   help="neural workload, diagnostic: run only the forward-backward or only the Viterbi call")
    p.add_argument("--no-kernel-profile", action="store_true",
                   help="layer workloads: skip the torch.profiler pass that finds the dominant kernel")
    p.add_argument("--no-follow", action="store_true",
                   help="ns workload, diagnostic: run the passes after the chains instead of the work "
                        "beside them in the chains' launches (csrc/follow.h); = --follow none")
    p.add_argument("--follow", choices=["default", "none", "fb", "vit", "all"], default="default",
                   help="ns workload, diagnostic: which op runs its work beside the chains (default: "
                        "the ops' own choice)")
    return p.parse_args()


def ns_follow(args):
    """(fb, vit) follow arguments of the ns step's two ops (None = the op's default)"""
    mode = "none" if args.no_follow else args.follow
    return {"default": (None, None), "none": (False, False), "fb": (True, False),
            "vit": (False, True), "all": (True, True)}[mode]


def spawn_ranks(args):
    """`bench.py --gpus N` outside a launcher: start N ranks through torch.distributed.run as
    child processes (this parent never touches the GPU) and exit with their status."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch N ranks with "
                 "torch.distributed.run, or run `bench.py --gpus N` without a launcher to spawn them)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return rank, world, local


def csrc_sha16():
    """sha256 (16 hex digits) of the kernel sources (pytorch_hmm_amd/csrc): a committed PMC
    summary records it (tools/prof_summary.py), so a bench line reports those bytes as the
    kernel's current traffic only when they were counted on these sources."""
    import glob
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(HERE, "pytorch_hmm_amd", "csrc", "*.h")) +
                    glob.glob(os.path.join(HERE, "pytorch_hmm_amd", "csrc", "*.hip"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def traffic_fields(v, src, fresh):
    """roofline fields for PMC bytes from a committed summary: `traffic` when they were counted
    on the current kernel sources; else `traffic` null and the stale bytes as
    `traffic_committed` (no stale counts beside live timings)."""
    if v is None:
        return {"traffic": None, "traffic_source": None}
    if fresh:
        return {"traffic": v, "traffic_source": src}
    return {"traffic": None, "traffic_committed": v,
            "traffic_source": f"{src} (counted on earlier kernel sources)"}


def profiled_traffic(op, B, T, N, transition):
    """HBM bytes per launch of `op` from the committed rocprofv3 PMC summary (FETCH_SIZE x 2 +
    WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction; tools/gpu_prof.sh -> profiles/),
    when it was taken on this exact configuration: (bytes, file, counted on these sources);
    else (None, None, False)."""
    import glob
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*_summary.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        cfg = d.get("bench_config") or {}
        if (cfg.get("batch_per_gpu"), cfg.get("seq_len"), cfg.get("num_states")) != (B, T, N):
            continue
        if transition not in str(cfg.get("transition", "")):
            continue
        v = d.get("ops", {}).get(op, {}).get("hbm_bytes_per_launch")
        if v:
            return float(v), os.path.relpath(f, HERE), d.get("csrc_sha16") == csrc_sha16()
    return None, None, False


def profiled_kernel_traffic(kernel, desc):
    """HBM bytes per launch of `kernel` (a torch.profiler kernel name) from the committed
    rocprofv3 PMC summary of the same layer workload (tools/gpu_prof.sh --workload ...;
    FETCH_SIZE x 2 + WRITE_SIZE): (bytes, file, counted on these sources) or (None, None, False)."""
    import glob
    import re
    m = re.search(r"hmm355::(\w+)(<[^>]*>)?", kernel or "")
    if not m:
        return None, None, False
    short = (m.group(1) + (m.group(2) or "")).replace(" ", "")
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*_summary.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        cfg = d.get("bench_config") or {}
        if any(cfg.get(k) != desc.get(k) for k in ("workload", "batch_per_gpu", "seq_len", "num_states")):
            continue
        v = (d.get("traffic") or {}).get(short, {}).get("hbm_bytes_per_launch")
        if v:
            return float(v), os.path.relpath(f, HERE), d.get("csrc_sha16") == csrc_sha16()
    return None, None, False


def cpu_baseline(B, T, N, budget, P):
    """Time the oracle (reference op sequence on torch-CPU) on the NS workload (transition
    matrix P), repeated until `budget` seconds of CPU work are spent (at least one FB+Viterbi
    pair)."""
    from oracle import hmm_oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    threads = max(1, min(threads, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(1234)
    obs = torch.softmax(torch.randn(B, T, N, generator=g), dim=-1)
    lP, lp0 = O.hmm_params(P.detach().cpu())
    frames, elapsed, reps = 0, 0.0, 0
    with torch.no_grad():
        while reps == 0 or (elapsed < budget and reps < 64):
            t0 = time.perf_counter()
            O.forward_backward(obs, lP, lp0)
            O.viterbi_decode(obs, lP, lp0)
            elapsed += time.perf_counter() - t0
            frames += B * T
            reps += 1
    return {"value": frames / elapsed, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x (forward_backward + viterbi_decode) at B={B} T={T} N={N} "
                      f"(oracle/hmm_oracle.py, the reference op sequence on torch-CPU, "
                      f"{threads} threads, {elapsed:.1f}s)"}


VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector peak (spec)
VALU64_PEAK_TFLOPS = 78.6  # FP64 vector peak (spec): the GMM scorer accumulates in fp64 (csrc/gmm.hip)


def kernel_profile(step, steps=3):
    """{kernel name: (launches, total device ms)} over `steps` extra steps, from torch.profiler
    (roctracer kernel records on ROCm).  Empty if the profiler yields no device events."""
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    out = {}
    for e in prof.key_averages():
        t_us = getattr(e, "self_device_time_total", None)
        if t_us is None:
            t_us = getattr(e, "self_cuda_time_total", 0.0)
        if t_us and t_us > 0 and e.count > 0:
            out[e.key] = (e.count / steps, t_us / 1e3 / steps)
    return out


def kernel_roofline(kprof, models, frames):
    """The roofline of the kernel that takes the most device time per step, from its OWN
    average launch duration and its algorithmic bytes / flops per frame (`models`: name
    substring -> ("hbm", bytes/frame) | ("valu", flops/frame)); None if it has no model."""
    if not kprof:
        return None
    name, (launches, ms) = max(kprof.items(), key=lambda kv: kv[1][1])
    for sub, (bound, per_frame) in models.items():
        if sub in name:
            avg_ms = ms / launches
            amount = per_frame * frames
            if bound in ("valu", "valu64"):
                ach = amount / (avg_ms * 1e-3) / 1e12
                peak = VALU64_PEAK_TFLOPS if bound == "valu64" else VALU_PEAK_TFLOPS
                return {"bound": bound, "kernel": name, "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                        "frac": ach / peak, "traffic": None, "flops_per_launch": amount,
                        "avg_launch_ms": avg_ms, "launches_per_step": launches, "share_of_step_device_time":
                        ms / sum(v[1] for v in kprof.values()), "source": "torch.profiler kernel records"}
            ach = amount / (avg_ms * 1e-3) / 1e9
            return {"bound": "hbm", "kernel": name, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": ach / HBM_PEAK_GBS, "traffic": None, "bytes_per_launch": amount, "avg_launch_ms": avg_ms,
                    "launches_per_step": launches, "share_of_step_device_time": ms / sum(v[1] for v in kprof.values()),
                    "source": "torch.profiler kernel records"}
    return {"kernel": name, "avg_launch_ms": ms / launches, "note": "dominant kernel has no algorithmic model"}


def layer_workload(args, rank, world, dev):
    """BASELINE configs 1/2/3/5 through the drop-in layers.
    One step = the config's reference call sequence on one synthetic batch (random-init layer
    of the named architecture, seed 0), inputs resident in HBM; each rank runs its own batch
    (weak scaling).  Prints one JSON line with the dominant kernel's roofline and a bounded
    CPU baseline (the oracle restatement, rank 0, N=1)."""
    import pytorch_hmm_amd as ph
    from oracle import hmm_oracle as O
    wl = args.workload
    torch.manual_seed(0)
    gx = torch.Generator(device=dev).manual_seed(1234 + rank)
    if wl == "c1":
        B, T, K = 2, 100, 5
        layer = ph.HMMLayer(K).to(dev)
        x = torch.randn(B, T, K, device=dev, generator=gx)

        def step():
            layer.train()
            post = layer(x)                 # forward-backward posteriors
            layer.eval()
            onehot, align = layer(x, return_alignment=True)   # Viterbi
            return post, align
        desc = {"workload": "HMMLayer(5) train forward-backward + eval Viterbi", "batch_per_gpu": B,
                "seq_len": T, "num_states": K}
        dom, flops, bytes_ = "hmm_layer_pair", None, (16 * K + 8 * K + 8) * B * T
        models = {"fb_recur": ("hbm", 16 * K), "vit_fwd": ("hbm", 8 * K), "fb_posterior": ("hbm", 20 * K)}
    elif wl == "c2":
        B, T, K, D = 32, 2000, 64, 80
        layer = ph.GaussianHMMLayer(K, D).to(dev)
        x = torch.randn(B, T, D, device=dev, generator=gx)

        def step():
            layer.train()
            post = layer(x)                 # Gaussian emission + forward-backward
            layer.eval()
            onehot = layer(x)               # Gaussian emission + Viterbi
            return post, onehot
        desc = {"workload": "GaussianHMMLayer(64,80) train forward-backward + eval Viterbi", "batch_per_gpu": B,
                "seq_len": T, "num_states": K, "feature_dim": D}
        dom, flops, bytes_ = "gaussian_pair", None, (2 * 4 * D + 8 * K + 12 * K) * B * T
        models = {"gmm_score": ("valu64", 4.0 * K * D), "fb_recur": ("hbm", 16 * K), "vit_fwd": ("hbm", 8 * K),
                  "fb_posterior": ("hbm", 20 * K)}
    elif wl == "c3":
        B, T, S, C, D = 32, 2000, 128, 4, 80
        layer = ph.MixtureGaussianHMMLayer(S, D, num_components=C).to(dev)
        x = torch.randn(B, T, D, device=dev, generator=gx)

        def step():
            return layer(x, return_log_probs=True)   # GMM emission + Viterbi
        desc = {"workload": "MixtureGaussianHMMLayer(128,80,num_components=4) forward (emission + Viterbi)",
                "batch_per_gpu": B, "seq_len": T, "num_states": S, "num_components": C, "feature_dim": D}
        dom, flops, bytes_ = "gmm_score_kernel", 4.0 * S * C * D * B * T, (4 * D + 4 * S) * B * T
        models = {"gmm_score": ("valu64", 4.0 * S * C * D), "vit_fwd": ("hbm", 8 * S)}
    elif wl == "neural":
        # NeuralHMM recursions (neural.py:391-511) at the north-star shape with a transition
        # matrix per (sequence, step): the network outputs log_obs (B,T,N) and
        # log_A = log(softmax + 1e-8) (B,T,N,N) (4.2 GB) are resident in HBM; one step =
        # forward_backward (posteriors, forward, backward) + viterbi_decode, on two streams.
        B, T, N = args.batch, args.T, args.N
        lo = torch.randn(B, T, N, device=dev, generator=gx) * 3 - 40
        if args.tv_static:   # diagnostic: one matrix for every step (L2-resident)
            lA = torch.log(torch.softmax(torch.randn(N, N, device=dev, generator=gx) * 2, dim=-1) + 1e-8)
        else:
            lA = torch.log(torch.softmax(torch.randn(B, T, N, N, device=dev, generator=gx) * 2, dim=-1) + 1e-8)
        only = args.tv_only or ""   # diagnostic: "fb" or "vit"
        init = torch.full((N,), -math.log(N), device=dev)
        layer = (lo, lA, init)
        s_fb, s_vit = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        mask = ph.ops.FB_POSTERIOR | ph.ops.FB_FORWARD | ph.ops.FB_BACKWARD

        # the two calls on two streams (one stream of log_A each)
        def step():
            cur = torch.cuda.current_stream(dev)
            s_fb.wait_stream(cur)
            s_vit.wait_stream(cur)
            r1 = r2 = None
            if only != "vit":
                with torch.cuda.stream(s_fb):
                    r1 = ph.ops.tv_forward_backward(lo, lA, init, mask)
            if only != "fb":
                with torch.cuda.stream(s_vit):
                    r2 = ph.ops.tv_viterbi(lo, lA, init)
            cur.wait_stream(s_fb)
            cur.wait_stream(s_vit)
            return r1, r2
        desc = {"workload": "NeuralHMM forward_backward + viterbi_decode, per-step transition matrices",
                "batch_per_gpu": B, "seq_len": T, "num_states": N}
        # algorithmic bytes per frame: FB reads its step's matrix and emissions, writes
        # posterior/forward/backward; Viterbi reads matrix + emissions, writes delta + state
        dom, flops, bytes_ = "tv_pair", None, (8 * N * N + 24 * N + 8) * B * T
        models = {"tv_fb": ("hbm", 2 * 4 * N * N + 4 * N), "tv_vit": ("hbm", 4 * N * N + 8 * N),
                  "tv_fbv": ("hbm", 2 * 4 * N * N + 12 * N)}
    elif wl == "smk":
        # SemiMarkovHMM.viterbi_decode (semi_markov.py:455-570) batched over the C5 shape
        # (the BASELINE C5 text names semi_markov.py): quad scorer + segment Viterbi + backtrace
        from pytorch_hmm_amd.semi_markov import SemiMarkovHMM
        B, T, S, D, Dm = 16, 2000, 64, 80, 40
        layer = SemiMarkovHMM(S, D, max_duration=Dm).to(dev)
        x = torch.randn(B, T, D, device=dev, generator=gx)

        def step():
            return layer.viterbi_decode_batch(x)
        desc = {"workload": "SemiMarkovHMM(64,80,max_duration=40) viterbi_decode (segment Viterbi)",
                "batch_per_gpu": B, "seq_len": T, "num_states": S, "max_duration": Dm, "feature_dim": D}
        dom, flops, bytes_ = "smk_fwd_kernel", 2.0 * (S * S * Dm + S * S) * B * T, (4 * D + 8) * B * T
        models = {"smk_fwd": ("valu", 2.0 * (S * S * Dm + S * S)), "smk_quad": ("valu", 3.0 * S * D)}
    elif wl == "stream":
        # StreamingHMMProcessor decode (streaming.py:267-377) for many concurrent streams: one
        # 160-frame chunk (the reference's default chunk_size) per stream, emission net
        # (Linear-ReLU-Linear-LogSoftmax) + greedy chain + beam search (K = 8), N = 64 states
        from pytorch_hmm_amd.streaming import StreamingHMMProcessor
        B, T, N, D, K = 256, 160, 64, 80, 8
        layer = StreamingHMMProcessor(N, D, beam_width=K).to(dev).eval()
        x = torch.randn(B, T, D, device=dev, generator=gx)
        log_T = layer._log_transitions()
        prev = torch.full((B,), -1, dtype=torch.int32, device=dev)
        hs0 = torch.full((B, ph.ops.STREAM_SLOTS), float("-inf"), device=dev)
        hs0[:, :K] = -math.log(N)
        hl0 = torch.zeros((B, ph.ops.STREAM_SLOTS), dtype=torch.int32, device=dev)
        hl0[:, :K] = torch.arange(K, dtype=torch.int32, device=dev)
        first = torch.ones(B, dtype=torch.int32, device=dev)

        def step():
            emis = layer.emission_net(x)
            g = ph.ops.stream_greedy(emis, log_T, prev, math.log(N))
            hs, hl = hs0.clone(), hl0.clone()
            cnt = torch.full((B,), K, dtype=torch.int32, device=dev)
            return g, ph.ops.stream_beam(emis, log_T, K, hs, hl, cnt, first, live_max=K)
        desc = {"workload": "StreamingHMMProcessor chunk decode (emission net + greedy + beam K=8), concurrent streams",
                "batch_per_gpu": B, "seq_len": T, "num_states": N, "feature_dim": D, "beam_width": K}
        dom, flops, bytes_ = "stream_beam_kernel", None, (4 * D + 8 * N + 16 + 4 * K) * B * T
        models = {"stream_beam": ("hbm", 4 * N + 8 + 4 * K), "stream_greedy": ("hbm", 4 * N + 8)}
    else:  # c5
        B, T, S, D, Dm = 16, 2000, 64, 80, 40
        layer = ph.HSMMLayer(S, D, max_duration=Dm).to(dev)
        x = torch.randn(B, T, D, device=dev, generator=gx)

        def step():
            return layer(x)                 # Gaussian emission + segment Viterbi
        desc = {"workload": "HSMMLayer(64,80,max_duration=40) forward (segment Viterbi)", "batch_per_gpu": B,
                "seq_len": T, "num_states": S, "max_duration": Dm, "feature_dim": D}
        # the reorganised recursion hsmm_fwd issues (csrc/hsmm.hip): per end time and state, each of
        # the Dmax open segments takes its obs-sum add, the two delta adds and the max into Dm (4
        # ops), and the predecessor maximum M adds and maxes S candidates: 4*S*Dmax + 2*S^2 per frame
        # (rounds 3-5 priced 2(S^2 Dmax + S^2), the literal loop's count, 17x this)
        hs_ops = 4.0 * S * Dm + 2.0 * S * S
        dom, flops, bytes_ = "hsmm_fwd_kernel", hs_ops * B * T, (4 * S + 8) * B * T
        models = {"hsmm_fwd": ("valu", hs_ops), "gmm_score": ("valu64", 4.0 * S * D)}

    # --overlap-steps: consecutive steps alternate between two HIP streams (each step's own
    # calls stay in order on its stream), so step k+1's full-chip emission scoring runs on the
    # CUs that step k's per-sequence recursion leaves idle -- the throughput of a stream of
    # batches, two in flight.  The serial step time (one stream) is measured too and reported
    # beside it.  Off by default: the default line is one batch at a time.
    overlap = args.overlap_steps and wl in ("c2", "c3", "c5")
    main_s = torch.cuda.current_stream(dev)
    side = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)] if overlap else None

    def run(k):
        if side is None:
            return step()
        with torch.cuda.stream(side[k & 1]):
            return step()
    serial_ms = None
    with torch.no_grad():
        for k in range(max(args.warmup, 1)):
            run(k)
        torch.cuda.synchronize(dev)
        if overlap:
            n_ser = min(args.steps, 5)
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(n_ser):
                step()
            s1.record()
            torch.cuda.synchronize(dev)
            serial_ms = s0.elapsed_time(s1) / n_ser
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        if side is not None:
            for s_ in side:
                s_.wait_stream(main_s)
        for k in range(args.steps):
            run(k)
        if side is not None:
            for s_ in side:
                main_s.wait_stream(s_)
        e1.record()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    step_ms = e0.elapsed_time(e1) / args.steps
    frames = desc["batch_per_gpu"] * desc["seq_len"]
    value = frames * world * args.steps / elapsed
    kroof = None
    if not args.no_kernel_profile:
        try:
            with torch.no_grad():
                kroof = kernel_roofline(kernel_profile(step), models, frames)
        except Exception as exc:  # the profiler is a measurement aid, not part of the step
            kroof = {"note": f"torch.profiler unavailable: {type(exc).__name__}"}
    if kroof is not None and "frac" in kroof:
        roof = kroof
        # the committed PMC bytes of the same kernel (for a VALU-bound kernel too: HBM bytes far
        # above its algorithmic bytes would still be the first thing to fix)
        roof.update(traffic_fields(*profiled_kernel_traffic(roof.get("kernel"), desc)))
    elif flops is not None:
        achieved = flops / (step_ms * 1e-3) / 1e12
        roof = {"bound": "valu", "kernel": dom, "achieved": achieved, "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / VALU_PEAK_TFLOPS, "traffic": None, "flops_per_launch": flops,
                "avg_launch_ms": step_ms, "note": "whole step time (HIP events) as the launch duration"}
    else:
        achieved = bytes_ / (step_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None, "bytes_per_launch": bytes_,
                "avg_launch_ms": step_ms, "note": "whole step time (HIP events) as the launch duration"}
    out = {"metric": f"frames/sec {desc['workload']}", "value": value, "unit": "frames/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic: randn features, random-init layer (seed 0)",
           "config": dict(desc, global_batch=desc["batch_per_gpu"] * world, parallelism=f"batch-sharded x{world}"),
           "roofline": roof}
    if overlap:
        out["step_overlap"] = ("consecutive steps on two alternating HIP streams (two batches in flight): "
                               "step k+1's emission scoring runs beside step k's recursion")
        out["ms_per_step_serial"] = serial_ms
    if kroof is not None and roof is not kroof:
        out["kernel_profile"] = kroof
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = layer_cpu_baseline(wl, layer, args.cpu_seconds)
        out["cpu_baseline"]["speedup_gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)


def layer_cpu_baseline(wl, layer, budget):
    """Bounded CPU baseline for a layer workload: the oracle restatement of the reference's op
    sequence (torch-CPU, or the C restatement for the HSMM recursion, whose literal reference
    loop takes ~55 h per sequence at this size), on a sample of the batch."""
    from oracle import hmm_oracle as O
    import numpy as np
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), os.cpu_count() or 1))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(7)
    frames, elapsed, reps = 0, 0.0, 0
    with torch.no_grad():
        sd = {k: v.detach().cpu() for k, v in layer.state_dict().items()} if wl != "neural" else None
        while reps == 0 or (elapsed < budget and reps < 64):
            t0 = time.perf_counter()
            if wl == "c1":
                x = torch.randn(2, 100, 5, generator=g)
                lP, lp0 = O.hmmlayer_params(sd["log_transition_logits"], sd["log_initial_logits"], True)
                O.forward_backward(torch.sigmoid(x), lP, lp0)
                O.viterbi_decode(torch.sigmoid(x), lP, lp0)
                n = 200
            elif wl == "c2":
                x = torch.randn(2, 2000, 80, generator=g)
                lP, lp0 = O.hmmlayer_params(sd["hmm_layer.log_transition_logits"], sd["hmm_layer.log_initial_logits"], True)
                pr = torch.exp(O.gaussian_log_probs(x, sd["means"], sd["log_scales"]))
                O.forward_backward(pr, lP, lp0)
                O.viterbi_decode(pr, lP, lp0)
                n = 4000
            elif wl == "c3":
                x = torch.randn(1, 2000, 80, generator=g)
                lp = O.mixture_log_probs(x, sd["mixture_weights_logits"], sd["means"], sd["log_vars"], t_chunk=250)
                O.mixture_viterbi(lp, O.mixture_log_transitions(sd["transition_logits"]))
                n = 2000
            elif wl == "neural":
                lo, lA, init = layer
                b, Tn = frames // 200 % lo.shape[0], 200
                lo_b, lA_b = lo[b:b + 1, :Tn].cpu().numpy(), lA[b:b + 1, :Tn].cpu().numpy()
                t0 = time.perf_counter()   # time the restatement only, not the device->host copy
                O.c_tv_fb64(lo_b, lA_b, init.cpu().numpy())
                O.c_tv_viterbi(lo_b, lA_b, init.cpu().numpy())
                n = Tn
            elif wl == "stream":
                # greedy + beam (K = 8) over one 160-frame chunk of one stream, C restatement of
                # streaming.py:267-377 (the reference's Python beam loop runs K*N tensor ops per frame)
                N, K = 64, 8
                x = torch.randn(160, 80, generator=g)
                emis = torch.func.functional_call(layer.emission_net, {k[len("emission_net."):]: v for k, v in sd.items()
                                                                       if k.startswith("emission_net.")}, (x,)).numpy()
                lT = torch.log(torch.softmax(sd["transition_logits"], dim=-1) + 1e-8).numpy()
                O.c_stream_greedy(emis, lT, -1, math.log(N))
                O.c_stream_beam(emis, lT, K, np.full(K, -math.log(N), np.float32), np.arange(K), True)
                n = 160
            elif wl == "smk":
                # the literal (t, s, d, s', d') recursion of semi_markov.py:455-570 in C; the
                # reference's Python loop runs ~15 us per candidate, i.e. hours
                Tn = 100
                x = torch.randn(Tn, 80, generator=g).numpy()
                cs, var = layer._gaussian_tables()
                q = O.c_smk_quad(x, sd["observation_means"].numpy(), var.numpy())
                O.c_smk_viterbi(q, cs.numpy(), layer._log_initial().numpy(), layer._log_transitions().numpy(),
                                layer.duration_model.candidate_table().cpu().numpy())
                n = Tn
            else:
                x = torch.randn(1, 2000, 80, generator=g)
                lp = O.hsmm_log_probs(x, sd["observation_means"], sd["observation_log_vars"])
                du = O.hsmm_duration_log_probs(sd["duration_shape"], sd["duration_rate"], 1, 40)
                O.c_hsmm(lp.numpy(), du.numpy(), O.hsmm_log_transitions(sd["transition_logits"]).numpy())
                n = 2000
            elapsed += time.perf_counter() - t0
            frames += n
            reps += 1
    kind_note = {"c1": "B=2 T=100", "c2": "B=2 of 32, T=2000", "c3": "B=1 of 32, T=2000",
                 "c5": "B=1 of 16, T=2000; HSMM recursion in the C restatement (1 thread)",
                 "stream": "one stream x 160 frames; emission net (torch-CPU) + greedy + beam K=8 in C (1 thread)",
                 "smk": "one sequence x 100 frames; the literal segment Viterbi in C (1 thread)",
                 "neural": "one sequence x 200 steps; the C restatement (fp64 FB + fp32 Viterbi, 1 thread)"}[wl]
    return {"value": frames / elapsed, "unit": "frames/s", "cores": threads if wl not in ("c5", "neural", "smk", "stream") else 1,
            "kind": "port",
            "sample": f"{reps} x ({kind_note}) oracle restatement of the reference op sequence, {elapsed:.1f}s"}


class NsStep:
    """One bench step of the NS workload: `ops["fb"]()` (forward-backward; posterior first in
    its outputs) and `ops["vit"]()` (Viterbi; states first), each on its own HIP stream and
    replayed from a captured HIP graph, then — with a `gatherer` (world > 1, BASELINE config 4)
    — the RCCL gather of posteriors + states to rank 0 on a third stream.

    Ordering is by events only: the gather stream waits for the two ops' end events of the same
    step; an op stream waits only for the gather that last read the output slot it is about to
    overwrite.  Outputs are double-buffered (two captured graphs per op, each with its own
    outputs), so step k's gather overlaps step k+1's compute and no step joins the streams.
    On a CPU device (the gloo tests) the same control flow runs without streams or graphs:
    each op is called and its outputs are gathered in program order."""

    def __init__(self, ops_, dev, gatherer=None, use_graph=True, serial=False):
        self.ops, self.dev, self.gatherer = ops_, dev, gatherer
        self.cuda = dev.type == "cuda"
        self.use_graph = use_graph and self.cuda
        self.nbuf = 2 if gatherer is not None else 1
        self.names = ("fb", "vit")
        self.out = [dict() for _ in range(self.nbuf)]
        self.graph = [dict() for _ in range(self.nbuf)]
        self.k = 0
        self.timing = None  # {op: [(start, end) events]} while set: each op bracketed on its stream
        if self.cuda:
            s_fb = torch.cuda.Stream(dev)
            self.stream = {"fb": s_fb, "vit": s_fb if serial else torch.cuda.Stream(dev)}
            self.s_comm = torch.cuda.Stream(dev) if gatherer is not None else None
            self.op_end = [{n: torch.cuda.Event() for n in self.names} for _ in range(self.nbuf)]
            self.read_done = [None] * self.nbuf   # event: the gather that read slot i finished
        if self.use_graph:
            self._capture()

    def _capture(self):
        main_s = torch.cuda.current_stream(self.dev)
        for n in self.names:   # warm the op (workspace allocation, plan) before capture
            s_ = self.stream[n]
            s_.wait_stream(main_s)
            with torch.cuda.stream(s_):
                for _ in range(2):
                    self.ops[n]()
        torch.cuda.synchronize(self.dev)
        for slot in range(self.nbuf):
            for n in self.names:
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=self.stream[n]):
                    self.out[slot][n] = self.ops[n]()
                self.graph[slot][n] = gr
        torch.cuda.synchronize(self.dev)

    def outputs(self, slot=None):
        """(posterior, states) of the most recent step (or of `slot`)."""
        o = self.out[(self.k - 1) % self.nbuf if slot is None else slot]
        return o["fb"][0], o["vit"][0]

    def __call__(self):
        slot = self.k % self.nbuf
        if not self.cuda:
            for n in self.names:
                self.out[slot][n] = self.ops[n]()
            if self.gatherer is not None:
                self.gatherer(*self.outputs(slot))
            self.k += 1
            return
        for n in self.names:
            s_ = self.stream[n]
            if self.read_done[slot] is not None:
                s_.wait_event(self.read_done[slot])
            with torch.cuda.stream(s_):
                if self.timing is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record(s_)
                if self.use_graph:
                    self.graph[slot][n].replay()
                else:
                    self.out[slot][n] = self.ops[n]()
                if self.timing is not None:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record(s_)
                    self.timing[n].append((e0, e1))
                if self.gatherer is not None:
                    self.op_end[slot][n].record(s_)
        if self.gatherer is not None:
            sc = self.s_comm
            for n in self.names:
                sc.wait_event(self.op_end[slot][n])
            post, states = self.outputs(slot)
            if not self.use_graph:   # eager outputs come from the op streams' allocator pools
                post.record_stream(sc)
                states.record_stream(sc)
            with torch.cuda.stream(sc):
                if self.timing is not None:
                    g0 = torch.cuda.Event(enable_timing=True)
                    g0.record(sc)
                self.gatherer(post, states)
                ev = torch.cuda.Event(enable_timing=self.timing is not None)
                ev.record(sc)
                if self.timing is not None:
                    self.timing["gather"].append((g0, ev))
            self.read_done[slot] = ev
        self.k += 1


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    rank, world, local = setup_dist(args)
    if args.workload != "ns":
        layer_workload(args, rank, world, torch.device("cuda", local))
        if world > 1:
            dist.destroy_process_group()
        return
    dev = torch.device("cuda", local)
    import pytorch_hmm_amd as ph
    from pytorch_hmm_amd import ops
    from pytorch_hmm_amd.distributed import BatchGather, batch_slice

    T, N = args.T, args.N
    if args.strong:
        # strong scaling: --batch is the global batch, each rank takes a contiguous slice of it
        if args.batch % world:
            sys.exit(f"bench.py --strong: global batch {args.batch} is not divisible by {world} ranks")
        s0, s1 = batch_slice(args.batch, rank, world)
        B = s1 - s0
    else:
        B = args.batch
    if args.transition == "ergodic":
        hmm = ph.HMMPyTorch(ph.create_transition_matrix(N, "ergodic"))
    elif args.transition == "random":
        gp = torch.Generator().manual_seed(4321)
        hmm = ph.HMMPyTorch(torch.softmax(torch.randn(N, N, generator=gp), dim=-1))
    elif args.transition == "trained":
        # a trained layer's tables (hmm_layer.py:61-89): HMMLayer(N) after three Adam steps
        # (lr 1e-3) on compute_loss over random scores at T = 8 (no saturation, so every
        # logit moves): no structural zeros are left and the dense chains run
        torch.manual_seed(0)
        layer = ph.HMMLayer(N).to(dev)
        opt = torch.optim.Adam(layer.parameters(), lr=1e-3)
        gt = torch.Generator(device=dev).manual_seed(0)
        layer.train()
        for _ in range(3):
            loss = layer.compute_loss(torch.randn(4, 8, N, device=dev, generator=gt))
            opt.zero_grad()
            loss.backward()
            opt.step()
        layer.eval()
        with torch.no_grad():
            layer(torch.randn(1, 2, N, device=dev, generator=gt))   # later-call tables
        hmm = layer._hmm
    else:
        hmm = ph.HMMPyTorch(ph.create_left_to_right_matrix(N, 0.7))
    if args.strong:
        g = torch.Generator(device=dev).manual_seed(1234)
        obs = torch.softmax(torch.randn(args.batch, T, N, device=dev, generator=g), dim=-1)[s0:s1].contiguous()
    else:
        g = torch.Generator(device=dev).manual_seed(1234 + rank)
        obs = torch.softmax(torch.randn(B, T, N, device=dev, generator=g), dim=-1)
    lP, lp0, plan = hmm._device_params(dev)   # what HMMPyTorch passes (log_P fixed at init)
    chains = ops.plan_info(plan)               # the chains that actually run (band.h)

    gather = world > 1 and not args.no_gather
    gatherer = None
    if gather:
        # BASELINE config 4: posteriors + states of every rank gathered to rank 0 each step,
        # into receive buffers allocated once (pytorch_hmm_amd.distributed.BatchGather; the
        # same NsStep + BatchGather run over gloo in tests/test_distributed.py)
        gatherer = BatchGather([torch.empty(B, T, N, device=dev), torch.empty(B, T, dtype=torch.int64, device=dev)])

    # A step is one forward_backward (posterior, forward, backward) and one viterbi_decode of
    # the batch (+ the gather when world > 1).  The two ops are independent, so each runs on
    # its own stream; consecutive steps pipeline across the streams (no per-step join: a
    # cross-stream join costs two cross-queue signal hops, ~35 us).  Each op is one launch
    # (the work beside the chains runs inside it), launched eagerly: a HIP graph replay put
    # ~19 us between consecutive replays on a stream, eager launches ~11 (--graph replays).
    fb_fl, vit_fl = ns_follow(args)
    step = NsStep({"fb": lambda: ops.forward_backward(obs, lP, lp0, ops.OBS_PROB, 7, plan, follow=fb_fl),
                   "vit": lambda: ops.viterbi(obs, lP, lp0, ops.OBS_PROB, plan, follow=vit_fl)},
                  dev, gatherer, use_graph=args.graph and not args.no_graph, serial=args.serial)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # per-op launch durations for the roofline: HIP events on each op's own stream around its
    # graph replay, over the timed steps (an event pair costs the step ~1-2 us of queue work;
    # the wall clock below is what `value` uses)
    step.timing = {n: [] for n in (*step.names, "gather")}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ev, step.timing = step.timing, None
    fb_ms = sum(a.elapsed_time(b) for a, b in ev["fb"]) / len(ev["fb"])
    vit_ms = sum(a.elapsed_time(b) for a, b in ev["vit"]) / len(ev["vit"])
    gather_info = None
    if ev["gather"]:
        # the gather's own time on the communication stream (events around the dist.gather
        # calls), and the bytes it moves into rank 0 per step: (world - 1) slices of posteriors
        # (B*T*N fp32) + states (B*T int64); DESIGN.md §6 models it against xGMI
        g_ms = [a.elapsed_time(b) for a, b in ev["gather"]]
        rx = (world - 1) * B * T * (4 * N + 8)
        gather_info = {"gather_ms": sum(g_ms) / len(g_ms), "gather_ms_max": max(g_ms),
                       "bytes_into_rank0_per_step": rx,
                       "rank0_rx_GBps": rx / (sum(g_ms) / len(g_ms) * 1e-3) / 1e9,
                       "model_ms_at_153GBps_per_link": B * T * (4 * N + 8) / 153e9 * 1e3}
    global_b = args.batch if args.strong else B * world
    value = global_b * T * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    tdesc = {"left_to_right": "left_to_right(0.7)", "ergodic": "ergodic",
             "random": "random dense softmax(randn(N,N))",
             "trained": "trained HMMLayer(N) tables (3 Adam steps)"}[args.transition]
    # roofline of the dominant op, algorithmic bytes per SURVEY.md §8(d)
    banded = plan is not None and getattr(plan, "_hmm355_banded", False)
    pair = banded and ops._use_pair(B, dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    # (the C ABI's conditions for the work beside the chains: fb.hip, viterbi.hip vit_follow_ok)
    fb_fl, vit_fl = ns_follow(args)
    fb_follow = banded and not pair and fb_fl is not False and ops.fb_follow_default(fb_fl) and 3 * B <= cus
    vit_follow = banded and vit_fl is not False and N > 64 and 4 * B <= cus
    if fb_ms >= vit_ms:
        dom, dur_ms, bytes_per_launch = "forward_backward", fb_ms, 16 * N * B * T
        kernels = ("fb_pair_kernel" if pair else
                   "fb_recur_kernel (chains + posterior followers)" if fb_follow else "fb_recur_kernel + fb_posterior_kernel")
    else:
        dom, dur_ms, bytes_per_launch = "viterbi", vit_ms, (8 * N + 8) * B * T
        kernels = ("vit_fwd_kernel (chains + log leaders + decode followers)" if vit_follow else
                   "vit_log_obs_kernel + vit_fwd_kernel + vit_psi_kernel + vit_backtrace_kernel")
    achieved = bytes_per_launch / (dur_ms * 1e-3) / 1e9
    dom_traffic = traffic_fields(*profiled_traffic(dom, B, T, N, args.transition))
    # both ops' fractions (north_star's target names forward-backward's)
    op_roofline = {}
    for name, ms, bpl in (("forward_backward", fb_ms, 16 * N * B * T), ("viterbi", vit_ms, (8 * N + 8) * B * T)):
        a_ = bpl / (ms * 1e-3) / 1e9
        op_roofline[name] = dict({"achieved": a_, "frac": a_ / HBM_PEAK_GBS, "bytes_per_launch": bpl,
                                  "avg_launch_ms": ms},
                                 **traffic_fields(*profiled_traffic(name, B, T, N, args.transition)))
    out = {
        "metric": "frames/sec forward-backward+Viterbi, B=32 T=2000 N=128, 1/2/4/8 GPU",
        "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "f32", "data": f"synthetic: softmax(randn(B,T,N)) emissions, {tdesc} transitions",
        "config": {"workload": "HMMPyTorch forward_backward + viterbi_decode", "batch_per_gpu": B,
                   "global_batch": global_b, "seq_len": T, "num_states": N,
                   "transition": tdesc, "chain": chains, "world_size_seen": world,
                   "parallelism": f"batch-sharded x{world}",
                   "streams": 1 if args.serial else 2,
                   "gather": ("RCCL gather of posteriors + states to rank 0 every step (double-buffered, "
                              "event-ordered)") if gather else (False if world == 1 else "skipped (--no-gather)"),
                   "hip_graph": step.use_graph, "step_pipelining": "per-op streams, no per-step join",
                   "transition_plan": plan is not None,
                   "fb_kernel": ("pair (both chains + outputs in one workgroup)" if pair else
                                 "chains + posterior followers in one launch" if fb_follow else "two-kernel"),
                   "viterbi_kernel": ("chains + log leaders + decode followers in one launch" if vit_follow else
                                      "log pass + chain + psi pass + backtrace")},
        "op_ms": {"forward_backward": fb_ms, "viterbi": vit_ms},
        "roofline": {"bound": "hbm", "kernel": dom, "kernels": kernels, "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     **dom_traffic,
                     "bytes_per_launch": bytes_per_launch, "avg_launch_ms": dur_ms},
        "roofline_ops": op_roofline,
    }
    if gather_info is not None:
        out["gather"] = gather_info
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(B, T, N, args.cpu_seconds, hmm.P)
        out["cpu_baseline"]["speedup_gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
