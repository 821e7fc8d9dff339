"""tools/diagnose_bench.py reads a multi-GPU bench line and flags what the first N = 8 run needs looked at
(CPU only)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(d):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "diagnose_bench.py"), "-"], input=json.dumps(d),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout.splitlines()


def test_flags_slow_stage_failed_path_and_high_latency():
    d = {"metric": "chunks/sec", "value": 4.0, "unit": "chunks/s", "n_gpus": 8, "ranks_seen": 8, "backend": "nccl",
         "config": {"parallelism": "auto"},
         "timed_work": {"requests": 100, "errors": 0, "completion_tokens": 100000, "requested_tokens": 100000,
                        "pinned_ok": True},
         "p2p_selftest": {"tp4": {"one_shot": "ok", "push_stream": "ok", "push_skinny": "n/a", "shapes": "hidden 4096"},
                          "tp8": {"one_shot": "ok", "push_stream": "failed", "why": {"push_stream": "mismatch"},
                                  "shapes": "hidden 4096"}},
         "ar_recoveries": 0,
         "stages": {"map": {"tp": 4, "predicted_s": 3.0, "measured_s": 3.1},
                    "reduce_l1": {"tp": 8, "predicted_s": 2.0, "measured_s": 3.4}},
         "p2p_latency_us": {"tp4": {"push_us": 8.0, "push_us_per_row": 0.1, "fused_us": 9.0},
                            "tp8": {"push_us": 35.0, "push_us_per_row": 0.3, "fused_us": 40.0}}}
    out = _run(d)
    text = "\n".join(out)
    assert out[0].startswith("# chunks/sec: 4.0")
    assert "ok: ranks seen 8 of 8" in text
    assert "ok: P2P self-test tp4 every exercised path ok" in text  # "n/a" and "shapes" are not failures
    assert "CHECK: P2P self-test tp8 failed: push_stream (mismatch)" in text
    assert "ok: stage map at tp 4" in text and "CHECK: stage reduce_l1 at tp 8" in text
    assert "CHECK: tp8 decode all-reduce cross-GPU cost 35.0 us" in text and "--ar-lat-us 35.0" in text
    assert "ok: tp4 decode all-reduce" in text


def test_one_gpu_line_and_missing_line():
    out = _run({"metric": "m", "value": 2.17, "unit": "chunks/s", "n_gpus": 1, "ranks_seen": 1, "backend": "none",
                "p2p_selftest": None, "stages": {"map": {"tp": 1, "predicted_s": 8.9, "measured_s": 8.9}},
                "p2p_latency_us": None, "ar_recoveries": 0})
    assert not any(l.startswith("CHECK") for l in out), out
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "diagnose_bench.py"), "-"], input="nothing here",
                       capture_output=True, text=True, timeout=60)
    assert "no bench.py JSON line" in r.stdout
