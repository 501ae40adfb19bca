"""Diagnostic: tests/test_gpu_bench_step.py's gather-ordering case with the rows that differ
reported (FB followers on / off)."""
import sys
import torch
sys.path.insert(0, ".")
import bench  # noqa: E402
import pytorch_hmm_amd as ph  # noqa: E402
from pytorch_hmm_amd import ops  # noqa: E402
sys.path.insert(0, "tests")
from test_gpu_bench_step import CopyGather  # noqa: E402

DEV = "cuda"
for use_graph in (True, False):
    for follow in (None, False):
        B, T, N, steps = 8, 600, 128, 6
        dev = torch.device(DEV, 0)
        hmm = ph.HMMPyTorch(ph.create_left_to_right_matrix(N, 0.7))
        lP, lp0, plan = hmm._device_params(dev)
        g = torch.Generator(device=dev).manual_seed(3)
        base = torch.softmax(torch.randn(B, T, N, device=dev, generator=g), -1)
        obs = base.clone()
        gat = CopyGather(B, T, N, steps)
        step = bench.NsStep({"fb": lambda: ops.forward_backward(obs, lP, lp0, ops.OBS_PROB, 7, plan, follow=follow),
                             "vit": lambda: ops.viterbi(obs, lP, lp0, ops.OBS_PROB, plan)}, dev, gat, use_graph=use_graph)
        inputs = []
        for k in range(steps):
            torch.cuda.synchronize(dev)
            x = base.clone()
            x[:, :, k % N] += 0.5 + 0.1 * k
            obs.copy_(x)
            inputs.append(x)
            torch.cuda.synchronize(dev)
            step()
        torch.cuda.synchronize(dev)
        for k in range(steps):
            p_ref = ops.forward_backward(inputs[k], lP, lp0, ops.OBS_PROB, 1, plan, follow=False)[0]
            d = (gat.post[k] - p_ref).abs().amax(-1)  # (B, T)
            bad = (d > 1e-6).nonzero()
            print(f"graph={use_graph} follow={follow} step {k}: bad rows {bad.shape[0]}", end="")
            if bad.shape[0]:
                bs = sorted(set(bad[:, 0].tolist()))
                print(f" seqs {bs} t range {bad[:, 1].min().item()}..{bad[:, 1].max().item()}"
                      f" nan {bool(torch.isnan(gat.post[k]).any())}", end="")
                # is the bad row equal to a previous step's posterior?
                for j in range(k):
                    pj = ops.forward_backward(inputs[j], lP, lp0, ops.OBS_PROB, 1, plan, follow=False)[0]
                    b0, t0 = bad[0].tolist()
                    if float((gat.post[k][b0, t0] - pj[b0, t0]).abs().max()) < 1e-6:
                        print(f" (row equals step {j}'s)", end="")
            print(flush=True)
