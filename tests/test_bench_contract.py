"""The driver's bench.py contract on CPU (gloo): ``python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N --steps K --warmup W`` prints exactly ONE JSON line (rank 0) with the whole-job value,
the step accounting and the config -- for a single process and for 2 ranks (data-parallel and
tensor-parallel stages), on a tiny model so it runs in seconds.  The 8-GPU node runs the same code
path with RCCL."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world: int, *extra: str, self_launch: bool = False):
    args = ["--gpus", str(world), "--steps", "2", "--warmup", "1", "--model", "tiny-gqa4", "--hours", "0.2",
            "--max-new-tokens", "6", "--chunk-tokens", "400", "--no-graphs", *extra]
    if world == 1 or self_launch:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), *args]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only, one line
    return json.loads(lines[0])


@pytest.mark.parametrize("world,extra", [(1, ()), (2, ("--parallel", "dp")), (2, ("--parallel", "tp"))])
def test_bench_prints_one_json_line(world, extra):
    out = _run(world, *extra)
    assert KEYS <= set(out)
    assert out["n_gpus"] == world and out["steps"] == 2 and out["warmup"] == 1
    assert out["unit"] == "chunks/s" and out["higher_is_better"] is True and out["dtype"] == "bf16"
    cfg = out["config"]
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(cfg)
    # value = whole-job chunks per second of one timed step (MAX over ranks of the timed region)
    assert out["value"] == pytest.approx(cfg["global_batch"] / (out["ms_per_step"] / 1000.0), rel=1e-3)
    assert out["engine_rank0"]["dp"] * out["engine_rank0"]["tp"] == world or extra == ("--parallel", "tp")
    if extra == ("--parallel", "tp"):
        assert "tp2" in cfg["parallelism"]
    assert out["ranks_seen"] == world
    assert out["backend"] == ("gloo" if world > 1 else "none")
    # the timed work is the pinned work: every generation produced exactly max_new tokens
    tw = out["timed_work"]
    assert tw["pinned_ok"] and tw["errors"] == 0 and tw["requests"] > 0
    assert tw["completion_tokens"] == tw["requested_tokens"] > 0


def test_bench_self_launches_ranks():
    """``python bench.py --gpus 2`` with no torchrun environment runs 2 ranks (not one process) and
    produces the same summary as the torchrun launch."""
    own = _run(2, "--parallel", "dp", self_launch=True)
    ref = _run(2, "--parallel", "dp")
    assert own["n_gpus"] == 2 and own["ranks_seen"] == 2 and own["backend"] == "gloo"
    assert own["summary_sha16"] == ref["summary_sha16"]
    assert own["config"]["global_batch"] == ref["config"]["global_batch"]
