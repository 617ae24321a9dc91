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


@pytest.mark.parametrize("f32,final", [(False, True), (True, False)])
def test_slot_idle_under_inference_mode(f32, final):
    """The same under torch.inference_mode(), where views do not keep their
    base tensor alive: a fresh slot is idle, and a held obs /
    reward view or an info-row view keeps it busy, whether the slot was
    built inside the mode or outside it and checked inside."""
    lay = _SlotLayout(1001, 10, 20, f32, final)
    with torch.inference_mode():
        z = _Slot(lay, torch.device("cpu"))
        assert z.idle()
        for make in (lambda: z.reward.view(7, 143), lambda: z.obs[3], lambda: z.info_rows(),
                     lambda: z.info_rows()[2], lambda: z.done[:10]):
            h = make()
            assert not z.idle()
            del h
            assert z.idle()
    y = _Slot(lay, torch.device("cpu"))
    with torch.inference_mode():
        assert y.idle()
        h = y.reward.view(7, 143)
        assert not y.idle()
        del h
        assert y.idle()


class _FakeSlot:
    def __init__(self, held, i):
        self.held, self.i = held, i

    def idle(self):
        return self.i not in self.held


def _drive(T, hold):
    """Run the copy=True pool policy for T steps; hold(t, i, held) returns the
    ids of the slots the caller holds after step t used slot i."""
    from gym_simpletetris_amd.envs.tetris_env import _SlotPool
    pool = _SlotPool(64)
    held, made, reused = set(), [0], 0
    for t in range(T):
        def new():
            made[0] += 1
            return _FakeSlot(held, made[0])
        slot, r = pool.take(new)
        reused += r
        held = hold(t, slot.i, held)
        for z in pool.q:
            z.held = held
    return reused, made[0], len(pool)


def _fifo(d):
    import collections
    q = collections.deque()

    def f(t, i, held):
        q.append(i)
        while len(q) > d:
            q.popleft()
        return set(q)
    return f


@pytest.mark.parametrize("d", [0, 1, 8, 20])
def test_pool_settles_at_holding_depth(d):
    """A loop keeping the last d steps' outputs: d + 1 slots, then no
    allocation at all (one idle() test per step)."""
    reused, made, size = _drive(200, _fifo(d))
    assert made == d + 1 and reused == 200 - (d + 1) and size == d + 1


def test_pool_forgets_slots_kept_for_good():
    """Every 10th step's outputs kept forever beside a depth-3 window: the
    kept slots leave the pool instead of blocking the reuse behind them."""
    f3 = _fifo(3)
    keep = set()

    def hold(t, i, held):
        if t % 10 == 0:
            keep.add(i)
        return f3(t, i, held) | keep
    reused, made, size = _drive(200, hold)
    assert made <= 20 + 4 + 4 and size <= 8, (reused, made, size)
