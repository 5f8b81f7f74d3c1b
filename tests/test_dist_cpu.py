"""The N>1 path on CPU: world_size-2 gloo runs of the sharded protocol (no GPU).

What lk_eval_pushdown_dist does across ranks (lakeside_amd/csrc/comm.cpp, eval.cpp):
  1. every rank scans only the segments with shard[i] == rank;
  2. the glob column unions are agreed over ranks (all-gather, element-wise max);
  3. every rank produces a partial table of per-glob SQL-group cells in a shared key space;
  4. rank 0 gathers the partial tables, folds them cell by cell (rows/counts add, min/max, sums), then
     finalizes per glob and merges globs exactly as the single-GPU path.
Here the same decomposition runs with the oracle as the per-rank scanner and gloo as the transport, over
the committed golden cases and several shard assignments, and must reproduce the golden rows — so any
assignment of segments to GPUs yields the single-GPU answer.  The host-transport bridge (the C callback
lk_comm_init_host calls) is exercised over the same gloo group.
"""
import ctypes
import json
import os
import socket

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _allgather_var(ag, data: bytes):
    """Variable-length all-gather over a fixed-size one: sizes first, then blobs padded to the largest
    (the protocol of HostComm::allgather_bytes, comm.cpp)."""
    import struct
    sizes = [struct.unpack("<Q", b)[0] for b in ag(struct.pack("<Q", len(data)))]
    mx = max(1, max(sizes))
    blobs = ag(data + b"\0" * (mx - len(data)))
    return [b[:n] for b, n in zip(blobs, sizes)]


def _shards(rule, paths, world):
    from lakeside_amd import dist as D
    if rule == "modulo":
        return D.modulo_shards(len(paths), world)
    if rule == "hash":
        return D.hash_shards([os.path.basename(p) for p in paths], world)
    if rule == "balanced":
        return D.balanced_shards([os.path.getsize(p) for p in paths], world)
    if rule == "all_on_last":
        return [world - 1] * len(paths)
    raise ValueError(rule)


def _worker(rank, world, port, rules):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import numpy as np
    import pyarrow.parquet as pq
    import torch.distributed as dist

    from lakeside_amd import dist as D
    from oracle import dataexpr as dx
    from tests.parity import assert_rows_equal, from_jsonable

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ag = D.gloo_allgather()
        # ---- the C callback the library calls (lk_allgather_fn), over gloo ----
        cb = D.make_callback(ag)
        send = (ctypes.c_uint8 * 16)(*[(rank * 16 + i) & 0xFF for i in range(16)])
        recv = (ctypes.c_uint8 * (16 * world))()
        assert cb(None, ctypes.addressof(send), 16, ctypes.addressof(recv)) == 0
        assert bytes(recv) == bytes(bytearray((r * 16 + i) & 0xFF for r in range(world) for i in range(16)))
        assert _allgather_var(ag, b"x" * (rank + 3)) == [b"x" * (r + 3) for r in range(world)]

        with open(os.path.join(GOLDEN, "cases.json")) as f:
            cases = json.load(f)
        for rule in rules:
            for case in cases:
                pr = dx.parse_pushdown(json.dumps(case["request"]))
                paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
                shard = _shards(rule, paths, world)
                agg = case["request"]["baseExpr"]["chart"]["aggregation"]
                glob_parts = []
                for g in dx.globs_of(pr, case["glob_size"]):
                    mine = [j for j, i in enumerate(g) if shard[i] == rank]
                    local = set()
                    for j in mine:
                        local |= set(pq.ParquetFile(paths[g[j]]).schema_arrow.names)
                    agreed = set()
                    for blob in _allgather_var(ag, json.dumps(sorted(local)).encode()):
                        agreed |= set(json.loads(blob.decode()))
                    cells = dx.evaluate_glob(pr, g, [paths[i] for i in g], only=mine, union=sorted(agreed))
                    parts = [None] * world
                    dist.all_gather_object(parts, cells)
                    glob_parts.append(parts)
                if rank != 0:
                    continue
                label = f"{rule}/{case['name']}"
                glob_cells = [dx.merge_partial_cells(parts) for parts in glob_parts]
                for gi, (cells, want) in enumerate(zip(glob_cells, case["expected_per_glob"])):
                    got = [(c.ts, c.agg_value(agg), c.tags) for c in cells]
                    assert_rows_equal(got, from_jsonable(want), agg, f"{label} glob {gi}")
                if case["expected_merged"] is not None:
                    got = dx.merge_glob_cells(pr, glob_cells)
                    assert_rows_equal(got, from_jsonable(case["expected_merged"]), agg, label)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sharding_rules():
    from lakeside_amd import dist as D
    # java.lang.String.hashCode known answers
    assert D.java_string_hash("") == 0
    assert D.java_string_hash("hello") == 99162322
    assert D.java_string_hash("polygenelubricants") == -2147483648
    assert D.hash_shards(["polygenelubricants"], 3) == [(-2147483648) % 3]
    assert D.modulo_shards(5, 2) == [0, 1, 0, 1, 0]
    assert D.block_shards(4, 2) == [0, 0, 1, 1]
    assert D.balanced_shards([10, 1, 1, 8], 2) == [0, 1, 1, 1]
    assert sorted(D.balanced_shards([5] * 8, 8)) == list(range(8))


@pytest.mark.timeout(600)
def test_sharded_protocol_world2_gloo():
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(WORLD, _free_port(), ["modulo", "hash", "balanced", "all_on_last"]), nprocs=WORLD,
             join=True)
