"""Multi-GPU host logic: which rank evaluates which segment, and the host transport for the exchange step.

Reference: the query-api sends every segment to the worker pod ``Math.floorMod(key.hashCode, podCount)``
(core/src/main/scala/com/cardinal/discovery/WorkerManager.scala:150-156) and merges the pods' partial
aggregates (core/src/main/scala/com/cardinal/eval/TimeGroupedSketchAggregator.scala:57-114).  Here a node's
GPUs are the pods: ``lk_eval_pushdown_dist`` scans the segments with ``shard[i] == rank`` and merges the
partial tables on rank 0.  The assignment only moves work, never results (partial tables merge exactly), so
the bench uses the byte-balanced assignment and a deployment may keep the reference's hash rule.

The exchange runs over RCCL by default (``Engine.comm_init``); ``gloo_allgather`` adapts a
torch.distributed process group (gloo) to the library's host all-gather callback (``lk_comm_init_host``),
which lets several ranks share one GPU and gives the CPU tests a transport to exercise.
"""
from typing import Callable, List, Optional, Sequence

import numpy as np


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode: s[0]*31^(n-1) + ... over UTF-16 code units, in 32-bit two's complement."""
    h = 0
    data = s.encode("utf-16-be")
    for i in range(0, len(data), 2):
        h = (31 * h + ((data[i] << 8) | data[i + 1])) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def hash_shards(keys: Sequence[str], world: int) -> List[int]:
    """The reference's pod rule, Math.floorMod(key.hashCode, n) (WorkerManager.scala:150-156)."""
    return [java_string_hash(k) % world for k in keys]   # Python % is floorMod for a positive divisor


def modulo_shards(n: int, world: int) -> List[int]:
    """Segment i -> rank i % world (the library's default when no shard array is passed)."""
    return [i % world for i in range(n)]


def block_shards(n: int, world: int) -> List[int]:
    """Contiguous blocks: rank r gets segments [r*n/world, (r+1)*n/world)."""
    return [min(world - 1, i * world // n) for i in range(n)] if n else []


def balanced_shards(sizes: Sequence[int], world: int) -> List[int]:
    """Byte-balanced assignment (longest-processing-time first): the largest remaining segment goes to the
    least-loaded rank; ties go to the lower rank.  Deterministic for given sizes."""
    load = [0] * world
    out = [0] * len(sizes)
    for i in sorted(range(len(sizes)), key=lambda i: (-sizes[i], i)):
        r = min(range(world), key=lambda r: (load[r], r))
        out[i] = r
        load[r] += sizes[i]
    return out


def gloo_allgather(group=None) -> Callable[[bytes], List[bytes]]:
    """Fixed-size all-gather of byte strings over a torch.distributed group (every rank passes the same size)."""
    import torch
    import torch.distributed as dist

    def allgather(data: bytes) -> List[bytes]:
        world = dist.get_world_size(group)
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8) if data else torch.zeros(0, dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t, group=group)
        return [bytes(o.numpy().tobytes()) for o in out]

    return allgather


def make_callback(allgather: Callable[[bytes], List[bytes]]):
    """Wrap a byte all-gather as the C callback lk_allgather_fn(user, send, bytes, recv) -> 0 / -1."""
    import ctypes

    from . import _lib

    def fn(user, send, nbytes, recv):
        try:
            data = ctypes.string_at(send, nbytes) if nbytes else b""
            parts = allgather(data)
            blob = b"".join(parts)
            if len(blob) != nbytes * len(parts):
                return -1
            if blob:
                ctypes.memmove(recv, blob, len(blob))
            return 0
        except Exception:   # never unwind through the C frame
            import traceback
            traceback.print_exc()
            return -1

    return _lib.ALLGATHER_FN(fn)


__all__ = ["java_string_hash", "hash_shards", "modulo_shards", "block_shards", "balanced_shards",
           "gloo_allgather", "make_callback"]
