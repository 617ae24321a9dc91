"""DLPack zero-copy interop on the caller side: a
learner's device action buffer from any DLPack producer drives step() and
rollout() without a copy, and the engine's outputs export back the same way."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class Foreign:
    """A non-torch DLPack producer over a torch tensor's memory."""

    def __init__(self, t):
        self.t = t

    def __dlpack__(self, stream=None, **kw):
        return self.t.__dlpack__() if stream is None else self.t.__dlpack__(stream=stream)

    def __dlpack_device__(self):
        return self.t.__dlpack_device__()


def test_dlpack_actions_zero_copy_and_equal():
    import gym_simpletetris_amd as G
    n, T = 3000, 40
    a = G.TetrisBatch(n, seeds=range(n), autoreset="same_step")
    b = G.TetrisBatch(n, seeds=range(n), autoreset="same_step")
    a.reset()
    b.reset()
    acts = torch.empty((T, n), dtype=torch.uint8, device=a.device)
    for t in range(T):
        a.gen_actions(t, 0x99, out=acts[t])
    assert b._actions(Foreign(acts[0])).data_ptr() == acts[0].data_ptr()  # no copy
    for t in range(T // 2):
        oa, ra, da = a.step(acts[t])
        ob, rb, db = b.step(Foreign(acts[t]))
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db), t
    oa, ra, da = a.rollout(acts[T // 2:])
    ob, rb, db = b.rollout(Foreign(acts[T // 2:]))
    assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db)
    # consumer side: the outputs export over DLPack without a copy
    assert torch.from_dlpack(Foreign(ob)).data_ptr() == ob.data_ptr()
    a.close()
    b.close()
