"""HF safetensors checkpoint round trip (engine/weights.py) on the CPU reference ops."""

import json
import os

import torch

from llm_map_reduce_summarizer_amd.engine.config import get_model_config
from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
from llm_map_reduce_summarizer_amd.engine.model import LlamaModel
from llm_map_reduce_summarizer_amd.engine.weights import config_from_hf, save_hf


def test_roundtrip_same_tokens(tmp_path):
    cfg = get_model_config("tiny-gqa4", init_std=0.05)
    a = LLMEngine(cfg, device="cpu", max_model_len=256, max_num_seqs=4, kv_pages=32, seed=3)
    save_hf(a.model, str(tmp_path))
    meta = json.load(open(os.path.join(tmp_path, "config.json")))
    assert meta["num_key_value_heads"] == 2 and meta["intermediate_size"] == 1024
    c2 = config_from_hf(str(tmp_path), "ckpt")
    assert (c2.hidden, c2.n_layers, c2.n_heads, c2.n_kv_heads, c2.ffn) == (512, 2, 8, 2, 1024)
    b = LLMEngine(c2, device="cpu", max_model_len=256, max_num_seqs=4, kv_pages=32, seed=99,
                  weights_path=str(tmp_path))
    for la, lb in zip(a.model.layers, b.model.layers):
        for n in ("ln1", "wqkv", "wo", "ln2", "wgu", "wdown"):
            assert torch.equal(getattr(la, n), getattr(lb, n)), n
    p = [[128000] + list(range(40, 90)), [128000] + list(range(7, 30))]
    ps = [SamplingParams(5, 0.0, 0), SamplingParams(5, 0.7, 1)]
    assert [o.token_ids for o in a.generate(p, ps)] == [o.token_ids for o in b.generate(p, ps)]


def test_tp_shard_and_tied_head(tmp_path):
    from safetensors.torch import load_file, save_file
    cfg = get_model_config("tiny-gqa4", init_std=0.05)
    full = LlamaModel(cfg, torch.device("cpu"), seed=5)
    save_hf(full, str(tmp_path))
    f = os.path.join(tmp_path, "model.safetensors")
    t = load_file(f)
    t["model.embed_tokens.weight"] = t.pop("lm_head.weight")  # tied embedding / head checkpoint
    save_file(t, f)
    halves = [LlamaModel(cfg, torch.device("cpu"), tp_rank=r, tp_size=2, weights_path=str(tmp_path))
              for r in range(2)]
    assert torch.equal(torch.cat([h.lm_head for h in halves]), halves[0].embed)
    assert torch.equal(torch.cat([h.layers[1].wdown for h in halves], 1), full.layers[1].wdown)
    hd, hq = cfg.head_dim, cfg.n_heads // 2
    assert torch.equal(halves[1].layers[0].wqkv[:hq * hd], full.layers[0].wqkv[hq * hd:2 * hq * hd])


def test_fp8_load(tmp_path):
    cfg = get_model_config("tiny", init_std=0.05)
    save_hf(LlamaModel(cfg, torch.device("cpu"), seed=1), str(tmp_path))
    m = LlamaModel(cfg, torch.device("cpu"), weight_dtype="fp8", weights_path=str(tmp_path))
    assert m.layers[0].wgu.q.dtype == torch.float8_e4m3fn
