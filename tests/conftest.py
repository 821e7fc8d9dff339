import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE_EXAMPLE = "/root/reference/transcript-example.json"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels / engine on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def example_transcript():
    """The reference's bundled example (read-only mount); synthetic stand-in elsewhere."""
    import json
    if os.path.isfile(REFERENCE_EXAMPLE):
        with open(REFERENCE_EXAMPLE, encoding="utf-8") as f:
            return json.load(f)
    pytest.skip("reference example transcript not available on this machine")


@pytest.fixture(scope="session")
def synth10h():
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript
    return synthetic_transcript(10.0, seed=0)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU on this host")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
