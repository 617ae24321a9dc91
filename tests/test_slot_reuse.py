"""TetrisVecEnv copy=True output-slot reuse: _Slot.idle() must report a slot
busy while the caller holds ANY of its outputs -- a returned tensor, a view of
one, an info-row or final-obs view -- and idle once all are dropped (host
logic only: the slot's tensors on the CPU here; the GPU test
test_gpu_vec_env.py::test_vec_env_copy_reuses_only_dropped_slots runs the
env itself)."""
import sys

import pytest
import torch

from gym_simpletetris_amd.envs.tetris_env import _Slot, _SlotLayout


@pytest.mark.parametrize("f32,final", [(False, True), (True, True), (False, False), (True, False)])
def test_slot_idle_tracks_every_reference(f32, final):
    lay = _SlotLayout(1001, 9, 15, f32, final)
    z = _Slot(lay, torch.device("cpu"))
    assert z.idle()
    none_refs = [None] * 100  # None's own count moving must not matter
    assert z.idle()
    del none_refs

    held = [lambda: z.obs, lambda: z.obs[2], lambda: z.reward, lambda: z.reward[5:9], lambda: z.done,
            lambda: z.done.view(torch.uint8), lambda: z.info_rows(), lambda: z.info_rows()[3],
            lambda: z.obs.detach(), lambda: torch.utils.dlpack.to_dlpack(z.obs)]
    if f32:
        held += [lambda: z.obs_f32, lambda: z.obs_f32.unsqueeze(-1), lambda: z.obs_f32[7]]
    if final:
        held += [lambda: z.final_obs(), lambda: z.final_obs()[0]]
    for i, make in enumerate(held):
        h = make()
        assert not z.idle(), i
        del h
        assert z.idle(), i
    # a container holding a tensor counts too
    box = {"o": z.obs}
    assert not z.idle()
    box.clear()
    assert z.idle()


def test_slot_idle_baseline_is_per_slot():
    lay = _SlotLayout(64, 10, 20, False, True)
    a = _Slot(lay, torch.device("cpu"))
    b = _Slot(lay, torch.device("cpu"))
    keep = a.obs
    assert not a.idle() and b.idle()
    del keep
    assert a.idle() and b.idle()
    assert sys.getrefcount(a.obs) == sys.getrefcount(b.obs)
