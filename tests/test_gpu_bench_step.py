"""GPU: bench.py's step object (bench.NsStep) on real HIP streams and graphs, with a gather.

The multi-GPU step replays each op's captured HIP graph on its own stream and gathers the
posteriors + states on a third stream, ordered by events only, with two output slots so one
step's gather overlaps the next step's compute (BASELINE config 4).  A one-GPU box cannot run
RCCL across ranks, so the gatherer here is a device-to-device copy into receive buffers on the
gather stream — the same position in the step.  Each step gets different emissions (written
while the device is idle, before the step), so if the gather stream did not wait for the same
step's op streams it would copy the slot's previous contents (the step before last) and fail.
What this does not reach: overlap of one step's gather with the next step's compute (the
host synchronises between steps here to change the inputs)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


class CopyGather:
    def __init__(self, B, T, N, steps):
        self.post = [torch.empty(B, T, N, device=DEV) for _ in range(steps)]
        self.states = [torch.empty(B, T, dtype=torch.int64, device=DEV) for _ in range(steps)]
        self.k = 0

    def __call__(self, post, states):
        self.post[self.k].copy_(post)
        self.states[self.k].copy_(states)
        self.k += 1


@pytest.mark.parametrize("use_graph", [True, False], ids=["graph", "eager"])
@torch.no_grad()
def test_ns_step_gather_ordering(use_graph):
    import bench
    import pytorch_hmm_amd as ph
    from pytorch_hmm_amd import ops
    B, T, N, steps = 8, 600, 128, 5
    dev = torch.device(DEV, 0)
    hmm = ph.HMMPyTorch(ph.create_left_to_right_matrix(N, 0.7))
    lP, lp0, plan = hmm._device_params(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    base = torch.softmax(torch.randn(B, T, N, device=dev, generator=g), -1)
    obs = base.clone()
    gat = CopyGather(B, T, N, steps)
    step = bench.NsStep({"fb": lambda: ops.forward_backward(obs, lP, lp0, ops.OBS_PROB, 7, plan),
                         "vit": lambda: ops.viterbi(obs, lP, lp0, ops.OBS_PROB, plan)},
                        dev, gat, use_graph=use_graph)
    assert step.nbuf == 2 and step.use_graph == use_graph
    inputs = []
    for k in range(steps):
        # a different input per step, written where both op streams see it before their replay
        torch.cuda.synchronize(dev)
        x = base.clone()
        x[:, :, k % N] += 0.5 + 0.1 * k
        obs.copy_(x)
        inputs.append(x)
        torch.cuda.synchronize(dev)
        step()
    torch.cuda.synchronize(dev)
    assert gat.k == steps
    for k in range(steps):
        p_ref, _, _, _, _ = ops.forward_backward(inputs[k], lP, lp0, ops.OBS_PROB, 1, plan)
        s_ref = ops.viterbi(inputs[k], lP, lp0, ops.OBS_PROB, plan)[0]
        assert torch.equal(gat.states[k], s_ref), f"step {k}: gathered states are not this step's"
        assert float((gat.post[k] - p_ref).abs().max()) < 1e-6, f"step {k}: gathered posterior differs"
    # the steps really differed (a stale slot could not pass)
    assert not torch.equal(gat.states[0], gat.states[1]) or not torch.equal(gat.post[0], gat.post[1])
