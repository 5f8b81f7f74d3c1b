"""bench.py's launcher contract, on the CPU (no GPU here): `--gpus N` without an external launcher starts N rank
processes itself, and refuses -- loudly, with a non-zero status -- when the GPUs it needs are not visible, instead of
degrading to one process."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=600, env=env, cwd=ROOT)


def test_gpus_8_without_8_gpus_fails_loudly():
    r = _run(["--gpus", "8", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 8 visible GPUs" in r.stderr, r.stderr[-2000:]
    assert r.stdout.strip() == ""   # no bench line


def test_host_rehearsal_without_any_gpu_fails_loudly():
    r = _run(["--gpus", "2", "--comm", "host", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "no GPU visible" in r.stderr, r.stderr[-2000:]


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=2" in r.stderr
