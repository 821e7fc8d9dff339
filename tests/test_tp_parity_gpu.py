"""Tensor-parallel paths against the textbook fp32 forward on ONE GPU: 2 and 4 ranks share the device
(gloo + the custom all-reduce's IPC buffers), so the sequence-parallel prefill, the TP-push decode, the
vocab-parallel sampler and the context-parallel prefill + KV hand-off run their real kernels and
collectives; rank 0 checks the gathered logits with the TP=1 parity bounds (tests/_tp_parity_worker.py).
VERDICT r3 item 6."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_tp_paths_match_fp32(world):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(world), "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "_tp_parity_worker.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert r.stdout.count("tp parity ok") == world, r.stdout[-2000:]
    print([ln for ln in r.stdout.splitlines() if "parity:" in ln])
