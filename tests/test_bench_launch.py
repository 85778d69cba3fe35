"""bench.py --gpus N: N ranks, or a refusal -- never a one-GPU number under an
N-GPU request (round-5 review item 2).  CPU only: the spawn path runs with
the ENET_BENCH_STUB coder (host memcpy, gloo); the refusal with no GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "ENET_BENCH_STUB"):
        e.pop(k, None)
    e.update(kw)
    return e


def test_gpus_n_spawns_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1"],
                       env=_env(ENET_BENCH_STUB="1"), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3


def test_gpus_one_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--steps", "2", "--warmup", "1"],
                       env=_env(ENET_BENCH_STUB="1"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") not in (None, "") or
                    os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPUs may be visible")
def test_gpus_n_refused_without_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "--gpus 2 requested" in r.stderr
    assert not r.stdout.strip()


def test_world_size_mismatch_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
