"""Parquet page decompression (lakeside_amd/csrc/codec.cpp, used by the segment loader) on the CPU: every page of
a table written with each codec, decompressed by our code, must equal the pages of the same table written
uncompressed (page boundaries follow the uncompressed sizes, so the plain payloads match byte for byte).
Covers v1 and v2 data pages, dictionary pages, NULLs, an all-NULL column (empty dictionary page) and PLAIN
int64/double columns."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "lakeside_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = str(tmp_path_factory.mktemp("codec") / "page_codec_check")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", SRC, "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
                    os.path.join(ROOT, "tools", "page_codec_check.cpp"), os.path.join(SRC, "codec.cpp"),
                    os.path.join(SRC, "parquet.cpp"), "-o", out, "-lz", "-l:libzstd.so.1", "-l:liblz4.so.1",
                    "-l:libbrotlidec.so.1"],
                   check=True)
    return out


def _table():
    import pyarrow as pa
    rng = np.random.default_rng(7)
    n = 50000
    return pa.table({
        "_cardinalhq.timestamp": pa.array(np.sort(rng.integers(0, 3_600_000, n)), pa.int64()),
        "_cardinalhq.value": pa.array(rng.lognormal(0, 2, n), pa.float64(), mask=rng.random(n) < 0.05),
        "_cardinalhq.name": pa.array([f"metric_{i:02d}" for i in rng.integers(0, 16, n)], pa.string()),
        "resource.service.name": pa.array([f"svc-{i:03d}" for i in rng.integers(0, 100, n)], pa.string(),
                                          mask=rng.random(n) < 0.05),
        "empty": pa.nulls(n, pa.string()),
    })


@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("codec", ["snappy", "gzip", "zstd", "lz4", "brotli"])
def test_pages_decompress_to_the_uncompressed_pages(checker, tmp_path, codec, version):
    import pyarrow.parquet as pq
    t = _table()
    strings = ["_cardinalhq.name", "resource.service.name", "empty"]
    kw = dict(use_dictionary=strings, data_page_version=version, row_group_size=20000, data_page_size=8192,
              column_encoding={"_cardinalhq.timestamp": "PLAIN", "_cardinalhq.value": "PLAIN"})
    plain, comp = str(tmp_path / "plain.parquet"), str(tmp_path / f"{codec}.parquet")
    pq.write_table(t, plain, compression="NONE", **kw)
    pq.write_table(t, comp, compression=codec, **kw)
    want = subprocess.run([checker, plain], check=True, capture_output=True, text=True).stdout
    got = subprocess.run([checker, comp], check=True, capture_output=True, text=True).stdout
    assert got == want and len(want.split()) == 5


def test_corrupt_page_is_an_error(checker, tmp_path):
    import pyarrow.parquet as pq
    path = str(tmp_path / "z.parquet")
    pq.write_table(_table(), path, compression="zstd", use_dictionary=["_cardinalhq.name"])
    data = bytearray(open(path, "rb").read())
    at = data.index(b"\x28\xb5\x2f\xfd")          # the first page's zstd frame magic
    data[at:at + 4] = bytes(4)
    open(path, "wb").write(bytes(data))
    r = subprocess.run([checker, path], capture_output=True, text=True)
    assert r.returncode == 1 and "error" in r.stderr
