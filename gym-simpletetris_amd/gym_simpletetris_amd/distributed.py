"""Multi-GPU sharding of the env batch: one process per GPU.

Envs are independent state machines (the reference's only shared state is the
global `random`, tetris_env.py:187, which the engine replaces by per-env
MT19937 streams), so the batch shards by contiguous global index with NO
collective in the step.  Seeds and synthetic actions are keyed by the global
env index, so results are identical at any GPU count.

The one exchange the north star names -- delivering every shard's packed
obs / reward / done to rank 0 -- is `gather_outputs`: one torch.distributed
gather (RCCL over xGMI with the 'nccl' backend; gloo on CPU in the tests) of a
single contiguous int32 buffer per rank, laid out [W + 2][n_local]:
rows 0..W-1 packed obs words, row W reward, row W+1 done bytes.  Collective
gathers need one size on every rank, so when n_global % world != 0 the short
ranks pad their buffer to the longest shard (`shard_cap`) for the transfer and
`assemble` drops the padding columns again.

With `wire=True` (ShardedTetris) each rank steps with st_step_wire straight
into a [wire_words][n_local] int32 buffer -- per env one bit stream of the
obs columns, the reward's 32 bits and done: 8 words (32 B) per 10x20 env
instead of W + 2 (48 B), so the per-step gather moves 1.5x fewer bytes into
rank 0 -- and rank 0 turns the gathered rows back into (obs, reward, done)
with st_unwire_shards straight from the receive buffer (`unwire_recv`; or
`assemble_wire` from a list of per-rank buffers), bit-exact.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n_global: int, world: int, rank: int) -> Tuple[int, int]:
    """(offset, count) of rank's contiguous block; the first n_global % world
    ranks get one extra env."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base, rem = divmod(n_global, world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def shard_cap(n_global: int, world: int) -> int:
    """Columns of the largest shard (rank 0's): the gather's common width."""
    return -(-n_global // world)


def output_buffer(width: int, n_local: int, device) -> torch.Tensor:
    """The per-rank packed output buffer [W + 2][n_local] int32."""
    return torch.zeros((width + 2, n_local), dtype=torch.int32, device=device)


def buffer_views(buf: torch.Tensor, width: int):
    """(obs [W][n] int32, reward [n] int32, done [n] uint8) views into buf."""
    n = buf.shape[1]
    done = buf[width + 1].view(torch.uint8)[:n]
    return buf[:width], buf[width], done


def gather_outputs(buf: torch.Tensor, group=None, dst: int = 0,
                   n_cap: Optional[int] = None) -> Optional[List[torch.Tensor]]:
    """Gather every rank's packed buffer to `dst`.  `n_cap` (default: this
    buffer's width) is the common column count; a shorter buffer is sent
    zero-padded to it, so ragged shards (shard_range with n_global % world
    != 0) gather correctly.  Returns the [W + 2][n_cap] buffers on `dst`."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    rows, n = buf.shape
    n_cap = n if n_cap is None else n_cap
    if n > n_cap:
        raise ValueError(f"shard of {n} envs exceeds the gather width {n_cap}")
    send = buf
    if n < n_cap:
        send = buf.new_zeros((rows, n_cap))
        send[:, :n] = buf
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, gather_list=bufs, dst=dst, group=group)
    return bufs


def assemble(bufs: List[torch.Tensor], width: int, counts: Optional[List[int]] = None):
    """Rank-0 side: concatenate gathered buffers into global (obs [W][N],
    reward [N], done bool [N]) in global env order; `counts[r]` = rank r's
    real envs (shard_range), default every column of every buffer.  done is
    torch.bool, as from the wire format's assemble_wire / unwire_recv."""
    counts = [b.shape[1] for b in bufs] if counts is None else counts
    if len(counts) != len(bufs):
        raise ValueError(f"{len(counts)} counts for {len(bufs)} buffers")
    obs = torch.cat([b[:width, :c] for b, c in zip(bufs, counts)], dim=1)
    reward = torch.cat([b[width, :c] for b, c in zip(bufs, counts)])
    done = torch.cat([buffer_views(b, width)[2][:c] for b, c in zip(bufs, counts)])
    return obs, reward, done.view(torch.bool)


def assemble_wire(bufs: List[torch.Tensor], width: int, height: int,
                  counts: Optional[List[int]] = None):
    """Rank-0 side of the wire format: gathered [words][n_cap] int32 buffers
    (any device; unpacked on the GPU by st_unwire, on `device` or the
    buffers' own) -> global (obs [W][N], reward [N], done [N]) in global env
    order, on the GPU."""
    from .engine import unwire
    counts = [b.shape[1] for b in bufs] if counts is None else counts
    if len(counts) != len(bufs):
        raise ValueError(f"{len(counts)} counts for {len(bufs)} buffers")
    dev = next((b.device for b in bufs if b.device.type == "cuda"), None)
    if dev is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    wire = torch.cat([b[:, :c].to(dev) for b, c in zip(bufs, counts)], dim=1).contiguous()
    return unwire(wire, width, height)


def unwire_recv(recv: torch.Tensor, width: int, height: int, n_global: int, out=None):
    """Rank-0 side of the wire format, straight from one contiguous receive
    buffer int32 [world, words, n_cap] on the GPU (gather into its views
    recv[r]) -> global (obs [W][N], reward [N], done bool [N]) in global env
    order, by st_unwire_shards (no concatenation)."""
    from .engine import unwire_shards
    return unwire_shards(recv, width, height, n_global, out=out)


class ShardedTetris:
    """This rank's shard of a global batch of `n_global` envs."""

    def __init__(self, n_global: int, seed: int = 0, rank: Optional[int] = None,
                 world: Optional[int] = None, device=None, wire: bool = False, **engine_kwargs):
        from .engine import TetrisBatch
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        self.offset, self.n = shard_range(n_global, self.world, self.rank)
        self.n_cap = shard_cap(n_global, self.world)
        self.counts = [shard_range(n_global, self.world, r)[1] for r in range(self.world)]
        # the public step stays asynchronous: actions are range-checked by the
        # step kernel (validate_actions='async'), not by a per-step sync
        engine_kwargs.setdefault("validate_actions", "async")
        self.engine = TetrisBatch(self.n, device=device,
                                  seeds=[seed + self.offset + e for e in range(self.n)],
                                  **engine_kwargs)
        self.wire = bool(wire)
        if self.wire:  # st_step_wire's rows (see the module docstring)
            self.buf = torch.zeros((self.engine.wire_words, self.n), dtype=torch.int32,
                                   device=self.engine.device)
        else:
            self.buf = output_buffer(self.engine.width, self.n, self.engine.device)
            self._obs, self._rew, self._done = buffer_views(self.buf, self.engine.width)

    def reset(self):
        self.engine.reset()

    def step(self, actions: torch.Tensor):
        """Step the shard, writing straight into the gather buffer (the
        engine's own action checks apply: shape, dtype, device, and 0..6 --
        by default in the step kernel, so a KeyError for an out-of-range
        device action comes at the next step or engine.check_actions()).
        Returns (obs, reward, done) views of the buffer, or with wire=True the
        buffer itself (the wire rows)."""
        if self.wire:
            return self.engine.step_wire(actions, out=self.buf)
        return self.engine.step(actions, obs="packed", out=(self._obs, self._rew, self._done))

    def gather(self, dst: int = 0, cpu: bool = False):
        """RCCL gather of the packed outputs to `dst` (cpu=True: via host
        memory, for the gloo backend in tests); padded to `n_cap` columns,
        pass the result to `assemble` for the global (obs, reward, done)."""
        return gather_outputs(self.buf.cpu() if cpu else self.buf, dst=dst, n_cap=self.n_cap)

    def assemble(self, bufs: List[torch.Tensor]):
        """Global (obs [W][N], reward [N], done [N]) from gather()'s result."""
        if self.wire:
            return assemble_wire(bufs, self.engine.width, self.engine.height, self.counts)
        return assemble(bufs, self.engine.width, self.counts)
