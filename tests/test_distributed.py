"""CPU, world_size 2 over gloo: the multi-GPU data path (batch sharding + gather to rank 0,
pytorch_hmm_amd/distributed.py — the same helpers bench.py uses) reassembles exactly what an
unsharded run produces.  The per-shard compute here is the oracle (CPU); on the GPU box the
same path runs the HIP kernels over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pytorch_hmm_amd.distributed import batch_slice, gather_batch, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import hmm_oracle as O
        g = torch.Generator().manual_seed(99)
        obs = torch.softmax(torch.randn(B, 40, 6, generator=g), -1)          # same on every rank
        lP, lp0 = O.hmm_params(O.left_to_right_matrix(6, 0.7))
        states, delta = O.viterbi_decode(shard(obs, rank, world), lP, lp0)
        post = O.forward_backward(shard(obs, rank, world), lP, lp0)[0]
        full_s = gather_batch(states, B)
        full_d = gather_batch(delta, B)
        full_p = gather_batch(post, B)
        if rank == 0:
            s_ref, d_ref = O.viterbi_decode(obs, lP, lp0)
            p_ref = O.forward_backward(obs, lP, lp0)[0]
            q.put((torch.equal(full_s, s_ref), torch.equal(full_d, d_ref), torch.equal(full_p, p_ref)))
        else:
            q.put(None if full_s is None else "non-dst got data")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [5, 8])
def test_sharded_gather_equals_unsharded(B):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    results = [q.get(timeout=10) for _ in range(world)]
    assert (True, True, True) in results
    assert None in results


def test_batch_slice_balanced():
    for B in range(0, 40):
        for W in (1, 2, 3, 8):
            sl = [batch_slice(B, r, W) for r in range(W)]
            assert sl[0][0] == 0 and sl[-1][1] == B
            assert all(sl[i][1] == sl[i + 1][0] for i in range(W - 1))
            sizes = [e - s for s, e in sl]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        batch_slice(4, 2, 2)


def _bench_gather_worker(rank, world, port, q):
    """bench.py's own step object (bench.NsStep) with stub ops on the CPU: each step, each
    rank's "forward-backward" and "Viterbi" stubs produce a fresh (B,T,N) posterior and (B,T)
    states batch, and the step's gather (pytorch_hmm_amd.distributed.BatchGather, receive
    buffers allocated once) moves them to rank 0; the output slots alternate (double
    buffering), and repeated steps reuse the same receive buffers."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from pytorch_hmm_amd.distributed import BatchGather
        B, T, N = 3, 30, 5
        calls = {"fb": 0, "vit": 0}

        def stub(kind, r, k):
            g = torch.Generator().manual_seed(1000 * k + 10 * r + (kind == "vit"))
            if kind == "fb":
                return (torch.softmax(torch.randn(B, T, N, generator=g), -1), None)
            return (torch.randint(0, N, (B, T), generator=g), None)

        def op(kind):
            def f():
                calls[kind] += 1
                return stub(kind, rank, calls[kind])
            return f
        gatherer = BatchGather([torch.empty(B, T, N), torch.empty(B, T, dtype=torch.int64)])
        step = bench.NsStep({"fb": op("fb"), "vit": op("vit")}, torch.device("cpu"), gatherer)
        ok = step.nbuf == 2 and not step.use_graph
        bufs = [id(b) for b in gatherer.bufs[0]] if rank == 0 else None
        for k in range(1, 4):
            step()
            post, states = step.outputs()
            ok &= torch.equal(post, stub("fb", rank, k)[0]) and torch.equal(states, stub("vit", rank, k)[0])
            if rank == 0:
                ok &= [id(b) for b in gatherer.bufs[0]] == bufs
                for r in range(world):
                    ok &= torch.equal(gatherer.full(0)[r * B:(r + 1) * B], stub("fb", r, k)[0])
                    ok &= torch.equal(gatherer.full(1)[r * B:(r + 1) * B], stub("vit", r, k)[0])
        q.put(bool(ok) if rank == 0 else (bool(ok) and gatherer.full(0) is None))
    finally:
        dist.destroy_process_group()


def test_bench_gather_path():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert all(q.get(timeout=10) for _ in range(world))


def test_bench_flags():
    """Multi-GPU defaults: the gather is on unless --no-gather; --strong splits the batch."""
    import sys
    import bench
    argv = sys.argv
    try:
        sys.argv = ["bench.py", "--gpus", "2"]
        a = bench.parse()
        assert not a.no_gather and not a.strong
        sys.argv = ["bench.py", "--gpus", "4", "--strong", "--no-gather"]
        a = bench.parse()
        assert a.no_gather and a.strong
    finally:
        sys.argv = argv
