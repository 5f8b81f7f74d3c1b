"""The sharded path on the GPU (lk_eval_pushdown_dist): golden parity at world 2 and world 1.

The box has one GPU and RCCL refuses two ranks on one device, so the world-2 run uses the library's host
transport (lk_comm_init_host over gloo): both ranks scan their shard on cuda:0, exchange dictionaries and
glob unions, and rank 0 gathers and folds the partial tables with the same merge kernel RCCL feeds.  The
world-1 run goes through an RCCL communicator.  Expected rows: the committed golden merged rows.
"""
import json
import os
import socket

import pytest

from tests.parity import assert_rows_equal, from_jsonable

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

pytestmark = pytest.mark.gpu


def _cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return [c for c in json.load(f) if c["expected_merged"] is not None]


def _tag_cases():
    with open(os.path.join(GOLDEN, "tag_cases.json")) as f:
        return json.load(f)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(rule, n, world):
    from lakeside_amd import dist as D
    return {"modulo": D.modulo_shards(n, world), "block": D.block_shards(n, world),
            "all_on_last": [world - 1] * n}[rule]


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from lakeside_amd.evaluator import Engine
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(0)
    try:
        eng.comm_init_host(world, rank)
        for rule in ("modulo", "block", "all_on_last"):
            for case in _cases():
                paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
                res = eng.eval_pushdown_dist(json.dumps(case["request"]), paths, _shard(rule, len(paths), world),
                                             case["glob_size"])
                if rank == 0:
                    agg = case["request"]["baseExpr"]["chart"]["aggregation"]
                    assert_rows_equal(res.rows(), from_jsonable(case["expected_merged"]), agg,
                                      f"world {world} {rule} {case['name']}")
                else:
                    assert len(res) == 0
            for case in _tag_cases():   # tag queries: counts per tag value, merged over the shards
                paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
                res = eng.eval_pushdown_dist(json.dumps(case["request"]), paths, _shard(rule, len(paths), world),
                                             case["glob_size"])
                if rank == 0:
                    key = lambda t: sorted(t.items())   # noqa: E731
                    assert sorted(res.tags, key=key) == sorted(case["expected_merged"], key=key), \
                        f"world {world} {rule} tag {case['name']}"
                else:
                    assert len(res) == 0
            print(f"rank {rank}: {rule} ok", flush=True)
        # Every rank loads every segment: identical dictionaries -> the dim space is agreed by fingerprint (no
        # dictionary exchange); above, the ranks' value sets differed and the dictionaries were exchanged.
        for case in _cases():
            for p in case["segments"]:
                eng.load_segment(os.path.join(GOLDEN, p))
        for case in _cases():
            paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
            res = eng.eval_pushdown_dist(json.dumps(case["request"]), paths, _shard("modulo", len(paths), world),
                                         case["glob_size"])
            if rank == 0:
                agg = case["request"]["baseExpr"]["chart"]["aggregation"]
                assert_rows_equal(res.rows(), from_jsonable(case["expected_merged"]), agg,
                                  f"world {world} same dictionaries {case['name']}")
        dist.barrier()
    finally:
        eng.close()
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dist_world2_host_transport_golden():
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port()), nprocs=2, join=True)


@pytest.mark.timeout(120)
def test_dist_world1_rccl_golden():
    from lakeside_amd.evaluator import Engine
    eng = Engine(0)
    try:
        eng.comm_init(Engine.unique_id(), 1, 0)
        for case in _cases():
            paths = [os.path.join(GOLDEN, p) for p in case["segments"]]
            res = eng.eval_pushdown_dist(json.dumps(case["request"]), paths, None, case["glob_size"])
            agg = case["request"]["baseExpr"]["chart"]["aggregation"]
            assert_rows_equal(res.rows(), from_jsonable(case["expected_merged"]), agg, f"rccl world 1 {case['name']}")
    finally:
        eng.close()
